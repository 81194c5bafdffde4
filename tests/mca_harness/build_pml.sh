#!/bin/bash
# TEST HARNESS ONLY: compile ompi_amd/mca/pml/rocm against the stand-in
# headers in tests/mca_harness/pml_include + coll_include (+ include/ for
# the shared ones) and link libompi_amd.
set -e
H=$(cd "$(dirname "$0")" && pwd)
R=$(cd "$H/../.." && pwd)
OUT=${1:-$H/pml_harness}
gcc -std=gnu11 -O1 -Wall -Wextra -Wno-unused-parameter -Wno-missing-field-initializers -DHARNESS_COLL \
    -I"$H/pml_include" -I"$H/coll_include" -I"$H/include" -I"$R/include" -I"$R/ompi_amd/mca/pml/rocm" \
    -I/opt/rocm/include \
    "$R/ompi_amd/mca/pml/rocm/pml_rocm.c" "$H/pml_harness.c" "$H/pml_saved.c" "$H/dev_helpers.c" "$H/progress_stub.c" \
    -L"$R/ompi_amd" -lompi_amd -L/opt/rocm/lib -lamdhip64 \
    -Wl,-rpath,"$R/ompi_amd" -Wl,-rpath,/opt/rocm/lib -lrt -o "$OUT"
