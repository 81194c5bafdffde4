cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for n in 2 3 4 8; do
  timeout -k 10 250 python -u tools/run_worker.py coll $n COLL_CASES=cross_comm_order_own_stream,cross_comm_grow_own_stream,cross_comm_random_own_stream,cross_comm_random_own_stream_b TAG=ccr_n > gpurun_out/ccr_$n.log 2>&1; rc=$?
  cut -c1-700 gpurun_out/ccr_$n.log | tail -5; if [ $rc -ne 0 ]; then echo STOP $rc; exit $rc; fi
done
