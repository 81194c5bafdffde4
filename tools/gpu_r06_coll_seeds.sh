# the coll worker's randomized sequences under more seeds (STRESS_SEED)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
C=random_sequence,random_sequence_user_ipc
for n in 4 8 3 2; do
  for seed in 1000 2000; do
    timeout -k 10 170 python -u tools/run_worker.py coll $n COLL_CASES=$C STRESS_SEED=$seed TIMEOUT=150 TAG=crs_n > gpurun_out/crs.log 2>&1; rc=$?
    echo "n=$n seed=$seed rc=$rc $(tail -1 gpurun_out/crs.log | cut -c1-30)"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/crs.log | cut -c1-600; exit 1; fi
  done
done
exit 0
