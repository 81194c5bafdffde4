set -e
PIPE_AB_PASSES=1,2,4 timeout -k 10 500 python3 -u tools/pipe_ab.py 2 16777216,268435456 256,1024 > gpurun_out/r04_pipe_passes_n2.jsonl 2> gpurun_out/r04_pipe_passes_n2.err
PIPE_AB_PASSES=1,2 timeout -k 10 500 python3 -u tools/pipe_ab.py 4 16777216,268435456 256 > gpurun_out/r04_pipe_passes_n4.jsonl 2> gpurun_out/r04_pipe_passes_n4.err
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
PIPE_AB_SCHEMES=pull,pull_pipe,push,push_pipe timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pipe_n2 -o run -- python3 -u tools/pipe_ab.py 2 268435456 256 > gpurun_out/r04_pipe_ab_n2_rocprof.jsonl 2>&1
