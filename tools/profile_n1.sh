#!/bin/bash
# One round's N=1 evidence on the GPU box: the bench line, a rocprofv3
# kernel-trace --stats pass of the same command, and the two PMC passes
# (FETCH_SIZE, WRITE_SIZE; separate runs, MI355X_MICROARCH.md §HBM).
# usage: tools/profile_n1.sh <tag>    -> gpurun_out/<tag>_*
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-rXX}
out=gpurun_out/prof_$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py > "gpurun_out/${tag}_bench_n1.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/ktrace" -o run \
    -- python3 -u bench.py --no-cpu-baseline > "gpurun_out/${tag}_bench_n1_under_rocprof.json"
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d "$out/pmc_$c" -o run \
        -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > /dev/null
done
find "$out" -name "*kernel_stats.csv" -o -name "*counter_collection.csv" | sort
