#!/bin/bash
# osc derived-target accumulate (ddt_acc_kernel) at the bench's shape:
# the event-timed line, a rocprofv3 kernel-trace --stats pass, and the two
# PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs, MI355X_MICROARCH.md §HBM).
# usage: tools/profile_ddt_acc.sh <tag>  -> gpurun_out/<tag>_ddt_acc*
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-rXX}
out=gpurun_out/prof_ddt_acc_$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 120 python3 -u tools/osc_ddt_acc_once.py > "gpurun_out/${tag}_ddt_acc.jsonl"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/ktrace" -o run \
    -- python3 -u tools/osc_ddt_acc_once.py >> "gpurun_out/${tag}_ddt_acc.jsonl"
for c in FETCH_SIZE WRITE_SIZE; do
    ACC_ITERS=3 timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$out/pmc_$c" -o run \
        -- python3 -u tools/osc_ddt_acc_once.py > /dev/null
done
find "$out" -name "*kernel_stats.csv" -o -name "*counter_collection.csv" | sort
