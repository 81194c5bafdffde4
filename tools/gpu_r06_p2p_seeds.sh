# the p2p / osc worker's randomized cases under more seeds (STRESS_SEED)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
C=p2p_random_channels,p2p_random_channels_b,p2p_random_channels_any_source,osc_random_epochs_after_p2p_s3000,osc_random_epochs_after_p2p_s5000,osc_random_epochs,osc_random_epochs_b,osc_random_epochs_separate,cross_layer_progress
for n in 4 8 3; do
  for seed in 1000 2000; do
    timeout -k 10 170 python -u tools/run_worker.py p2p_osc $n P2P_OSC_CASES=$C STRESS_SEED=$seed TIMEOUT=150 TAG=pos_n > gpurun_out/pos.log 2>&1; rc=$?
    echo "n=$n seed=$seed rc=$rc $(tail -1 gpurun_out/pos.log | cut -c1-30)"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/pos.log | cut -c1-600; exit 1; fi
  done
done
exit 0
