#!/bin/bash
# TEST HARNESS ONLY: compile ompi_amd/mca/coll/rocm against the stand-in
# headers in tests/mca_harness/coll_include (+ include/ for the shared ones)
# and link libompi_amd + the oracle.
set -e
H=$(cd "$(dirname "$0")" && pwd)
R=$(cd "$H/../.." && pwd)
OUT=${1:-$H/coll_harness}
gcc -std=gnu11 -O1 -DHARNESS_COLL -Wall -Wextra -Wno-unused-parameter -Wno-missing-field-initializers \
    -I"$H/coll_include" -I"$H/include" -I"$R/include" -I"$R/ompi_amd/mca/coll/rocm" \
    -I/opt/rocm/include \
    "$R/ompi_amd/mca/coll/rocm/coll_rocm_module.c" "$H/coll_harness.c" "$H/coll_saved.c" "$H/dev_helpers.c" "$H/progress_stub.c" \
    -L"$R/ompi_amd" -lompi_amd -L"$R/oracle" -loracle -L/opt/rocm/lib -lamdhip64 \
    -Wl,-rpath,"$R/ompi_amd" -Wl,-rpath,"$R/oracle" -Wl,-rpath,/opt/rocm/lib -lrt -o "$OUT"
