cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1150 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/full.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/full.log | cut -c1-600 | tail -12
exit $rc
