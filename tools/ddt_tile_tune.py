#!/usr/bin/env python3
"""A/B of the staged tile pack (ddt_pack_tile_kernel): LDS tile size and
tile vs the per-granule kernels, on the layouts it takes (256 MiB packed,
whole-stream window).  Each setting runs in its own process (the knobs are
read once per process).  One JSON line per point."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, os, statistics, sys
sys.path.insert(0, %r)
import torch
from ompi_amd import datatype as dd
i32, f64 = dd.predefined("MPI_INT"), dd.predefined("MPI_DOUBLE")
lens = [13, 13, 13, 13, 13, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1]
disps = [286, 308, 330, 352, 374, 396, 419, 442, 465, 488, 511, 534, 557, 580, 603, 626, 649, 672]
P = 256 << 20
cases = [("struct_int_double", dd.type_struct([1, 1], [0, 8], [i32, f64]), None),
         ("blacs_indexed", dd.type_indexed(lens, disps, i32), None),
         ("vector_bl1", dd.type_vector(P // 8, 1, 2, f64), 1),
         ("vector_bl2", dd.type_vector(P // 16, 2, 4, f64), 1),
         ("vector_bl8", dd.type_vector(P // 64, 8, 16, f64), 1)]
for name, dt, cnt in cases:
    count = cnt or P // dt.size
    total = dt.size * count
    src = torch.empty((count - 1) * dt.extent + dt.true_span, dtype=torch.uint8, device="cuda").random_()
    out = torch.empty(total, dtype=torch.uint8, device="cuda")
    def run():
        cv = dd.Convertor(); cv.prepare_for_send(dt, count, src); cv.pack(out, total)
    run(); torch.cuda.synchronize()
    vals = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            run()
        e1.record(); torch.cuda.synchronize()
        vals.append(e0.elapsed_time(e1) / 5)
    ms = statistics.median(vals)
    print(json.dumps({"type": name, "packed_bytes": total, "ms": round(ms, 4),
                      "GBps": round(2 * total / (ms * 1e-3) / 1e9, 1),
                      "tile": os.environ.get("OMPI_AMD_DDT_TILE", "1"),
                      "tile_bytes": os.environ.get("OMPI_AMD_DDT_TILE_BYTES", "default"),
                      "wide": os.environ.get("OMPI_AMD_DDT_TILE_WIDE", "0")}), flush=True)
''' % ROOT

settings = ([{"OMPI_AMD_DDT_TILE": "0"}] +
            [{"OMPI_AMD_DDT_TILE_BYTES": str(b)} for b in (8192, 12288, 16384, 24576, 32768)] +
            [{"OMPI_AMD_DDT_TILE_WIDE": "1", "OMPI_AMD_DDT_TILE_BYTES": str(b)}
             for b in (8192, 16384)])
if len(sys.argv) > 1 and sys.argv[1] == "wide":
    settings = [{}, {"OMPI_AMD_DDT_TILE_WIDE": "1"}, {"OMPI_AMD_DDT_TILE_WIDE": "1", "OMPI_AMD_DDT_TILE_BYTES": "8192"}]
for st in settings:
    env = {**os.environ, **st}
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True,
                       timeout=300)
    sys.stdout.write(r.stdout)
    if r.returncode != 0:
        sys.stderr.write(r.stderr[-2000:])
        sys.exit(r.returncode)
