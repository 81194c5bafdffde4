#!/bin/bash
# blacs-indexed (and struct{int,double}) pack / unpack through one convertor
# call over a 256 MiB packed stream (BASELINE configs[2], tools/ddt_sweep.py):
# the line per tile-size setting, then a rocprofv3 kernel-trace --stats pass
# and the two PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs,
# MI355X_MICROARCH.md §HBM) of the default setting.
# usage: tools/profile_blacs.sh <tag> [tile-size settings...]  -> gpurun_out/<tag>_blacs_*
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-rXX}
shift || true
out=gpurun_out/prof_blacs_$tag
mkdir -p "$out"
export TMPDIR=/tmp SWEEP_TYPES=blacs_indexed,struct_int_double SWEEP_SIZES=268435456 SWEEP_WHOLE=1
for v in default "$@"; do
    if [ "$v" = default ]; then
        timeout -k 10 120 python3 -u tools/ddt_sweep.py | sed "s/^{/{\"setting\": \"default\", /"
    else
        env "$v" timeout -k 10 120 python3 -u tools/ddt_sweep.py | sed "s/^{/{\"setting\": \"$v\", /"
    fi
done > "gpurun_out/${tag}_blacs_sweep.jsonl"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/ktrace" -o run \
    -- python3 -u tools/ddt_sweep.py > "gpurun_out/${tag}_blacs_under_rocprof.jsonl"
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$out/pmc_$c" -o run \
        -- python3 -u tools/ddt_sweep.py > /dev/null
done
find "$out" -name "*kernel_stats.csv" -o -name "*counter_collection.csv" | sort
