set -e
export COLL_CASES=pipelined_schemes,alg4_ar_sum_f32_big,alg5_ar_sum_f32_big_inplace,alg6_ar_sum_f32_big_odd,alg4_pipelined_nonblocking,alg5_iallreduce_mixed,alg4_persistent_big,alg6_free_realloc,alg5_persistent_big_inplace,alg6_ar_maxloc_double_int,autotune_large_allreduce
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_coll_gpu.py -k "parity" > gpurun_out/pipe_parity.log 2>&1
