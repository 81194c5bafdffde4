# N=1 bench, then shared-GPU rehearsals at N=2 and N=8 (every rank on cuda:0)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || { tail -5 gpurun_out/bench_n1.err; exit 1; }
cut -c1-300 gpurun_out/bench_n1.json
for n in 2 8; do
  timeout -k 10 400 python -u bench.py --gpus $n --steps 10 --warmup 3 > gpurun_out/bench_n$n.json 2> gpurun_out/bench_n$n.err || { tail -5 gpurun_out/bench_n$n.err; exit 1; }
  cut -c1-300 gpurun_out/bench_n$n.json
done
