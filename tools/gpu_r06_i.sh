# the cross-communicator cases at N=4, three times back to back, then after a
# 3-rank run (a failure at N=4 showed only after earlier runs on the box)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
C=cross_comm_order_own_stream,cross_comm_grow_own_stream,cross_comm_random_own_stream,cross_comm_random_own_stream_b
for n in 4 4 4 3 4 4; do
  timeout -k 10 120 python -u tools/run_worker.py coll $n COLL_CASES=$C TIMEOUT=100 TAG=cci_n > gpurun_out/cci.log 2>&1; rc=$?
  echo "n=$n rc=$rc $(tail -1 gpurun_out/cci.log | cut -c1-40)"; ps -eo pid,stat,etime,cmd | grep -c "[c]oll_worker" || true
  [ $rc -ne 0 ] && exit 1
done
exit 0
