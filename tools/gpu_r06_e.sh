cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_mca_glue.py tests/test_p2p_osc_gpu.py tests/test_osc_ddt_fuzz_gpu.py > gpurun_out/e.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/e.log | tail -40
exit $rc
