set -e
export SWEEP_TYPES=blacs_indexed,struct_int_double,vector_bl1,vector_bl2 SWEEP_SIZES=268435456 SWEEP_WHOLE=1 SWEEP_TOP=268435456
for t in 0 32 64 128 0; do
  OMPI_AMD_DDT_UNPACK_TOUCH=$t timeout -k 10 120 python3 -u tools/ddt_sweep.py | grep '"unpack"' | grep "\"calls\": 1," | sed "s/^{/{\"touch\": $t, /"
done > gpurun_out/r04_unpack_touch_ab.jsonl
