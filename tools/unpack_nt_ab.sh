set -e
export SWEEP_TYPES=blacs_indexed,struct_int_double,vector_bl1,vector_bl2,vector_bl8,vector_bl64 SWEEP_SIZES=268435456 SWEEP_WHOLE=1 SWEEP_TOP=268435456
for t in 0 1 0 1; do
  OMPI_AMD_DDT_UNPACK_NT=$t timeout -k 10 120 python3 -u tools/ddt_sweep.py | grep '"unpack"' | grep "\"calls\": 1," | sed "s/^{/{\"nt\": $t, /"
done > gpurun_out/r04_unpack_nt_ab.jsonl
# the fragment path (one fAdvance over 4096 x 64 KiB iovecs: ddt_iov_tile_kernel)
for t in 0 1; do
  FRAG_MODES=iov_batch OMPI_AMD_DDT_UNPACK_NT=$t timeout -k 10 200 python3 -u tools/ddt_frag_bench.py | grep '"unpack"' | sed "s/^{/{\"nt\": $t, /"
done > gpurun_out/r04_unpack_nt_frag_ab.jsonl
