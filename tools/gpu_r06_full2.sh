# the GPU suite twice on one box (flakiness check before round end)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 560 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/full_$i.log 2>&1; rc=$?
  grep -E "FAILED|passed|failed" gpurun_out/full_$i.log | cut -c1-400 | tail -4
  [ $rc -ne 0 ] && exit $rc
done
exit 0
