# cross-layer progress case (coll / p2p / osc on three communicators) at N = 2, 3, 4, 8
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for n in 2 3 4 8; do
  timeout -k 10 200 python -u tools/run_worker.py p2p_osc $n P2P_OSC_CASES=cross_layer_progress TIMEOUT=180 TAG=xl_n > gpurun_out/xl_$n.log 2>&1; rc=$?
  cut -c1-900 gpurun_out/xl_$n.log | tail -4; if [ $rc -ne 0 ]; then echo STOP $rc; exit $rc; fi
done
