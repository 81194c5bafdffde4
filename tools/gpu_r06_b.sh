cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for os_ in 0 1; do
  HARNESS_OWN_STREAM=$os_ timeout -k 10 320 bash tools/coll_harness_bench.sh 2 gpurun_out/seam_n2_own$os_.jsonl; rc=$?
  if [ $rc -ne 0 ]; then echo STOP $rc; exit $rc; fi
  head -4 gpurun_out/seam_n2_own$os_.jsonl
done
