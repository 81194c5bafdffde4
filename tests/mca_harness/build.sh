#!/bin/bash
# TEST HARNESS ONLY: compile ompi_amd/mca/op/rocm against the stand-in
# headers in tests/mca_harness/include and link libompi_amd + the oracle.
set -e
H=$(cd "$(dirname "$0")" && pwd)
R=$(cd "$H/../.." && pwd)
OUT=${1:-$H/op_select_harness}
gcc -std=gnu11 -O1 -Wall -Wextra -Wno-unused-parameter -Wno-missing-field-initializers \
    -I"$H/include" -I"$R/include" -I/opt/rocm/include \
    "$R/ompi_amd/mca/op/rocm/op_rocm_component.c" "$H/op_select_harness.c" "$H/dev_helpers.c" \
    -L"$R/ompi_amd" -lompi_amd -L"$R/oracle" -loracle -L/opt/rocm/lib -lamdhip64 \
    -Wl,-rpath,"$R/ompi_amd" -Wl,-rpath,"$R/oracle" -Wl,-rpath,/opt/rocm/lib -o "$OUT"
