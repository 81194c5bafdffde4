#!/bin/bash
# host-buffer ping-pong through pml/rocm, host_path 0 vs 1
# (tests/mca_harness/pml_harness.c, HARNESS_PML_BENCH=1; build:
# tests/mca_harness/build_pml.sh tools/pml_harness_bin)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HARNESS_GPU=1 HARNESS_PML_BENCH=1 OMPI_AMD_COLL_TIMEOUT_MS=20000
name=$(python3 -c "import secrets;print(secrets.token_hex(3))")
timeout -k 5 300 tools/pml_harness_bin $name 1 2 > /dev/null 2> gpurun_out/pml_ab_r1.err &
p1=$!
timeout -k 5 300 tools/pml_harness_bin $name 0 2 > gpurun_out/r04_pml_host_path_ab.jsonl 2> gpurun_out/pml_ab_r0.err
r0=$?
wait $p1
echo "rc0=$r0 rc1=$?"
