set -e
tools/profile_blacs.sh r04nt OMPI_AMD_DDT_TILE_BYTES=8192 OMPI_AMD_DDT_TILE_BYTES=32768 OMPI_AMD_DDT_TILE_BYTES=49152 OMPI_AMD_DDT_UNPACK_NT=0 > gpurun_out/prof_blacs_r04nt.txt 2>&1
timeout -k 10 300 python3 -u tools/pipe_ab.py 2 67108864,268435456 256,512 > gpurun_out/r04_pipe_ab_n2.jsonl 2> gpurun_out/r04_pipe_ab_n2.err
timeout -k 10 300 python3 -u tools/pipe_ab.py 4 67108864,268435456 256 > gpurun_out/r04_pipe_ab_n4.jsonl 2> gpurun_out/r04_pipe_ab_n4.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pipe_n2 -o run -- python3 -u tools/pipe_ab.py 2 268435456 256 > gpurun_out/r04_pipe_ab_n2_rocprof.jsonl 2>&1
