#!/bin/bash
# TEST HARNESS ONLY: compile ompi_amd/mca/osc/rocm against the stand-in
# headers in tests/mca_harness/osc_include (+ coll_include / include for the
# shared ones) and link libompi_amd + the oracle; the communicator's own
# collectives (rocm_query's agreement) are coll_saved.c's host stand-ins.
set -e
H=$(cd "$(dirname "$0")" && pwd)
R=$(cd "$H/../.." && pwd)
OUT=${1:-$H/osc_harness}
gcc -std=gnu11 -O1 -DHARNESS_OSC -Wall -Wextra -Wno-unused-parameter -Wno-missing-field-initializers \
    -I"$H/osc_include" -I"$H/coll_include" -I"$H/include" -I"$R/include" \
    -I"$R/ompi_amd/mca/osc/rocm" -I/opt/rocm/include \
    "$R/ompi_amd/mca/osc/rocm/osc_rocm_component.c" "$H/osc_harness.c" "$H/coll_saved.c" "$H/dev_helpers.c" "$H/progress_stub.c" \
    -L"$R/ompi_amd" -lompi_amd -L"$R/oracle" -loracle -L/opt/rocm/lib -lamdhip64 \
    -Wl,-rpath,"$R/ompi_amd" -Wl,-rpath,"$R/oracle" -Wl,-rpath,/opt/rocm/lib -lrt -o "$OUT"
