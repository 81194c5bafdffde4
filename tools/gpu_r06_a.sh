cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for n in 2 3 8; do
  timeout -k 10 250 python -u tools/run_worker.py coll $n COLL_CASES=cross_comm_order_own_stream TAG=ccown_n > gpurun_out/ccown_$n.log 2>&1; rc=$?
  tail -1 gpurun_out/ccown_$n.log; if [ $rc -gt 1 ]; then echo STOP $rc; exit $rc; fi
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_mca_glue.py > gpurun_out/glue.log 2>&1; rc=$?
tail -5 gpurun_out/glue.log; if [ $rc -gt 1 ]; then echo STOP $rc; exit $rc; fi
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_p2p_osc_gpu.py > gpurun_out/p2posc.log 2>&1; rc=$?
tail -5 gpurun_out/p2posc.log
