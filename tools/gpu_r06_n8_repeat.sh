# Repeat the N=8 p2p/osc suite with stack dumps armed; stop at the first failure
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export OMPI_AMD_BACKTRACE=1
for i in 1 2 3; do
  timeout -k 10 380 python -u -m pytest -x -q --timeout 360 --timeout-method thread -m gpu tests/test_p2p_osc_gpu.py -k "parity" > gpurun_out/n8rep_$i.log 2>&1 || { echo "run $i failed"; mkdir -p gpurun_out/n8fail; cp gpurun_out/coll_logs/raw_p2p_osc_n*_rank*.txt gpurun_out/n8fail/; exit 1; }
  tail -1 gpurun_out/n8rep_$i.log
done
