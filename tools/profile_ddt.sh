#!/bin/bash
# The convertor's final kernels on the GPU box: the fragment bench line, a
# rocprofv3 kernel-trace --stats pass of the same command, and the two PMC
# passes (FETCH_SIZE, WRITE_SIZE; separate runs, MI355X_MICROARCH.md §HBM).
# usage: tools/profile_ddt.sh <tag>    -> gpurun_out/<tag>_ddt_*
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-rXX}
out=gpurun_out/prof_ddt_$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/ddt_frag_bench.py > "gpurun_out/${tag}_ddt_frag_bench.jsonl"
export FRAG_MODES=iov_batch  # one launch per fAdvance train: the kernels, not the host loop
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/ktrace" -o run \
    -- python3 -u tools/ddt_frag_bench.py > "gpurun_out/${tag}_ddt_frag_bench_under_rocprof.jsonl"
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$out/pmc_$c" -o run \
        -- python3 -u tools/ddt_frag_bench.py > /dev/null
done
find "$out" -name "*kernel_stats.csv" -o -name "*counter_collection.csv" | sort
