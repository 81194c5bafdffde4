#!/bin/bash
# Unpack tile size (typed bytes a tile spans) x tile order (0 strided by the
# grid, 1 a contiguous run per workgroup) x type, one convertor call over
# 256 MiB packed (tools/ddt_sweep.py), default nt policy.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export SWEEP_TYPES=${SWEEP_TYPES:-blacs_indexed,struct_int_double,vector_bl1,vector_bl2,vector_bl8,vector_bl64} SWEEP_SIZES=268435456 SWEEP_WHOLE=1 SWEEP_TOP=268435456
for order in ${ORDERS:-0 2}; do
for tb in ${TILES:-4096 8192 12288 16384 24576}; do
  OMPI_AMD_DDT_TILE_ORDER=$order OMPI_AMD_DDT_UNPACK_TILE_BYTES=$tb timeout -k 10 120 python3 -u tools/ddt_sweep.py | grep '"unpack"' | grep "\"calls\": 1," | grep '"packed_bytes": 2684' | sed "s/^{/{\"order\": $order, \"unpack_tile_bytes\": $tb, /"
done
done > gpurun_out/r04_unpack_tile_sweep.jsonl
