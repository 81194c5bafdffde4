#!/bin/bash
# MPI_Allreduce / MPI_Iallreduce / MPI_Allreduce_init through coll/rocm's
# installed function table (tests/mca_harness/coll_harness.c,
# HARNESS_COLL_BENCH=1), N ranks sharing this node's GPU 0, 8 B - 256 MiB.
# build: tests/mca_harness/build_coll.sh tools/coll_harness_bin
# usage: tools/coll_harness_bench.sh N OUT.jsonl   (OMPI_AMD_HOST_MARKS=0: waits on events only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
n=${1:-2}
out=${2:-gpurun_out/coll_harness_bench_n$n.jsonl}
export HARNESS_GPU=1 HARNESS_COLL_BENCH=1 OMPI_AMD_COLL_TIMEOUT_MS=20000
name=$(python3 -c "import secrets;print(secrets.token_hex(3))")
pids=()
for ((r = 1; r < n; ++r)); do
    timeout -k 5 300 tools/coll_harness_bin $name $r $n > /dev/null 2> gpurun_out/coll_bench_r$r.err &
    pids+=($!)
done
timeout -k 5 300 tools/coll_harness_bin $name 0 $n > "$out" 2> gpurun_out/coll_bench_r0.err
rc=$?
for p in "${pids[@]}"; do wait $p || rc=$?; done
echo "rc=$rc"
exit $rc
