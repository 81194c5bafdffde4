#!/bin/bash
# TEST HARNESS ONLY: compile ompi_amd/mca/common/rocm (the convertor seam)
# against the stand-in opal datatype headers in tests/mca_harness/ddt_include
# and link libompi_amd + the oracle.
set -e
H=$(cd "$(dirname "$0")" && pwd)
R=$(cd "$H/../.." && pwd)
OUT=${1:-$H/ddt_harness}
# CUDA=1: the layout and hooks of an OPAL_CUDA_SUPPORT build (function table,
# convertor->stream); CUDA=0: a ROCm-only build (neither exists)
CUDA=${2:-1}
gcc -std=gnu11 -DOPAL_CUDA_SUPPORT=$CUDA -O1 -Wall -Wextra -Wno-unused-parameter -Wno-missing-field-initializers \
    -I"$H/ddt_include" -I"$H/include" -I"$R/include" -I"$R/ompi_amd/mca/common/rocm" \
    -I/opt/rocm/include \
    "$R/ompi_amd/mca/common/rocm/opal_datatype_rocm.c" "$H/ddt_harness.c" "$H/dev_helpers.c" \
    -L"$R/ompi_amd" -lompi_amd -L"$R/oracle" -loracle -L/opt/rocm/lib -lamdhip64 -lpthread \
    -Wl,-rpath,"$R/ompi_amd" -Wl,-rpath,"$R/oracle" -Wl,-rpath,/opt/rocm/lib -o "$OUT"
