# the randomized cross-communicator cases under more seeds (STRESS_SEED)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
C=cross_comm_random_own_stream,cross_comm_random_own_stream_b
for n in 4 8 3; do
  for seed in ${SEEDS:-1000 2000 3000}; do
    timeout -k 10 120 python -u tools/run_worker.py coll $n COLL_CASES=$C STRESS_SEED=$seed TIMEOUT=100 TAG=ccs_n > gpurun_out/ccs.log 2>&1; rc=$?
    echo "n=$n seed=$seed rc=$rc $(tail -1 gpurun_out/ccs.log | cut -c1-30)"
    if [ $rc -ne 0 ]; then exit 1; fi
  done
done
exit 0
