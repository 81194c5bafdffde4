#!/bin/bash
# Any MCA harness (coll / pml / osc) run directly, N ranks, up to K times,
# stopping at the first failure with every rank's stderr kept
# (gpurun_out/<name>_n<N>_r<rank>_<k>.err).
# build: tests/mca_harness/build_{coll,pml,osc}.sh tools/<name>_harness_bin
# usage: tools/harness_rerun.sh coll|pml|osc N K
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
h=${1:-pml}
n=${2:-3}
runs=${3:-3}
bin=tools/${h}_harness_bin
export HARNESS_GPU=1 OMPI_AMD_COLL_TIMEOUT_MS=20000
for ((k = 1; k <= runs; ++k)); do
    name=$(python3 -c "import secrets;print(secrets.token_hex(3))")
    pids=()
    for ((r = 1; r < n; ++r)); do
        timeout -k 5 150 $bin $name $r $n > gpurun_out/${h}_n${n}_r${r}_$k.out 2> gpurun_out/${h}_n${n}_r${r}_$k.err &
        pids+=($!)
    done
    timeout -k 5 150 $bin $name 0 $n > gpurun_out/${h}_n${n}_r0_$k.out 2> gpurun_out/${h}_n${n}_r0_$k.err
    rc=$?
    for p in "${pids[@]}"; do wait $p || rc=$?; done
    echo "$h n=$n run $k: rc=$rc"
    [ $rc -eq 0 ] || exit $rc
done
