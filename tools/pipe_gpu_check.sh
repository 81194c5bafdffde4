#!/bin/bash
# Round-4 GPU checks of the new paths: the pipelined allreduce schemes
# (coll_worker cases) and osc derived-datatype accumulates (p2p_osc worker
# case, osc/rocm harness), each step under its own time limit.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
P2P_OSC_ONLY=osc_accumulate_derived timeout -k 10 400 python -u -m pytest -x -v --timeout 300 \
    --timeout-method thread tests/test_p2p_osc_gpu.py > gpurun_out/osc_ddt_parity.log 2>&1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_mca_glue.py -k "osc_component_device_path" > gpurun_out/osc_harness.log 2>&1
COLL_CASES=pipelined_schemes,alg4_ar_sum_f32_big,alg5_ar_sum_f32_big_inplace,alg6_ar_sum_f32_big_odd,alg4_pipelined_nonblocking,alg5_iallreduce_mixed,alg4_persistent_big,alg6_free_realloc,alg5_persistent_big_inplace,alg6_ar_maxloc_double_int,autotune_large_allreduce \
    timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
    tests/test_coll_gpu.py -k "parity" > gpurun_out/pipe_parity.log 2>&1
