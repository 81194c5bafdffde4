cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for own in 0 1; do
  ROWS_OWN_STREAM=$own timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rows_own$own -o run -- python3 tools/p2p_osc_rows.py 8 > gpurun_out/prof_rows_own$own.log 2>&1; rc=$?
  echo "own=$own rc=$rc"; tail -1 gpurun_out/prof_rows_own$own.log | cut -c1-300
  if [ $rc -ne 0 ]; then echo STOP; exit $rc; fi
done
find gpurun_out/prof_rows_own0 gpurun_out/prof_rows_own1 -name "*kernel_stats.csv" | head -20
