#!/bin/bash
# Kernel trace of the coll/rocm latency bench (tools/coll_harness_bench.sh):
# rank 0 under rocprofv3 --kernel-trace --stats, rank 1 plain, 2 ranks on GPU 0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export HARNESS_GPU=1 HARNESS_COLL_BENCH=1 OMPI_AMD_COLL_TIMEOUT_MS=20000
name=$(python3 -c "import secrets;print(secrets.token_hex(3))")
timeout -k 5 300 tools/coll_harness_bin $name 1 2 > /dev/null 2> gpurun_out/seamprof_r1.err &
p1=$!
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/seamprof -o seam -- \
    tools/coll_harness_bin $name 0 2 > gpurun_out/seamprof_r0.jsonl 2> gpurun_out/seamprof_r0.err
rc=$?
wait $p1 || rc=$?
echo "rc=$rc"
exit $rc
