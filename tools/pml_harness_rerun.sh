#!/bin/bash
# pml harness (tests/mca_harness/pml_harness.c) run directly, N ranks, up to
# K times, stopping at the first failure with every rank's stderr kept
# (gpurun_out/pml_n<N>_r<rank>_<k>.err; IPC trace on).
# build: tests/mca_harness/build_pml.sh tools/pml_harness_bin
# usage: tools/pml_harness_rerun.sh N K
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
n=${1:-3}
runs=${2:-3}
export HARNESS_GPU=1 OMPI_AMD_COLL_TIMEOUT_MS=20000 OMPI_AMD_IPC_TRACE=${OMPI_AMD_IPC_TRACE:-0}
for ((k = 1; k <= runs; ++k)); do
    name=$(python3 -c "import secrets;print(secrets.token_hex(3))")
    pids=()
    for ((r = 1; r < n; ++r)); do
        timeout -k 5 150 tools/pml_harness_bin $name $r $n > gpurun_out/pml_n${n}_r${r}_$k.out \
            2> gpurun_out/pml_n${n}_r${r}_$k.err &
        pids+=($!)
    done
    timeout -k 5 150 tools/pml_harness_bin $name 0 $n > gpurun_out/pml_n${n}_r0_$k.out \
        2> gpurun_out/pml_n${n}_r0_$k.err
    rc=$?
    for p in "${pids[@]}"; do wait $p || rc=$?; done
    echo "run $k: rc=$rc"
    [ $rc -eq 0 ] || exit $rc
done
