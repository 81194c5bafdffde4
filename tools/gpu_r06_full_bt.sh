cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export OMPI_AMD_BACKTRACE=1
timeout -k 10 1100 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/full_bt.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/full_bt.log | cut -c1-600 | tail -12
exit $rc
