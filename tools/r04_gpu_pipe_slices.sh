set -e
PIPE_AB_SLICES=16384,65536,262144,1048576,4194304 PIPE_AB_SCHEMES=push,push_pipe,pull,pull_pipe \
  timeout -k 10 400 python3 -u tools/pipe_ab.py 2 268435456 256 > gpurun_out/r04_pipe_slices_n2.jsonl 2> gpurun_out/r04_pipe_slices_n2.err
PIPE_AB_SLICES=65536,262144,1048576,4194304 PIPE_AB_SCHEMES=push,push_pipe \
  timeout -k 10 400 python3 -u tools/pipe_ab.py 4 268435456 256 > gpurun_out/r04_pipe_slices_n4.jsonl 2> gpurun_out/r04_pipe_slices_n4.err
