cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
o=gpurun_out/r06_p2p_osc_rows.jsonl
rm -f $o
for spec in "8 4 0" "8 1 0" "8 4 1" "4 4 0"; do
  set -- $spec
  GPU_MAX_HW_QUEUES=$2 ROWS_OWN_STREAM=$3 timeout -k 10 240 python -u tools/p2p_osc_rows.py $1 $o > /dev/null 2>&1; rc=$?
  echo "n=$1 q=$2 own=$3 rc=$rc"; tail -1 $o | cut -c1-700
  if [ $rc -ne 0 ]; then echo STOP; exit $rc; fi
done
