#!/usr/bin/env python3
"""One staged tile pack and one staged tile unpack (struct {int, double},
256 MiB packed) x 20 each, for rocprofv3 --kernel-trace --stats: the
per-launch durations of ddt_pack_tile_kernel / ddt_unpack_tile_kernel
against their algorithmic bytes (2 x packed)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ompi_amd import datatype as dd  # noqa: E402

i32, f64 = dd.predefined("MPI_INT"), dd.predefined("MPI_DOUBLE")
dt = dd.type_struct([1, 1], [0, 8], [i32, f64])
count = (256 << 20) // dt.size
src = torch.empty((count - 1) * dt.extent + dt.true_span, dtype=torch.uint8, device="cuda").random_()
out = torch.empty(dt.size * count, dtype=torch.uint8, device="cuda")
for _ in range(20):
    cv = dd.Convertor()
    cv.prepare_for_send(dt, count, src)
    cv.pack(out, dt.size * count)
for _ in range(20):
    cv = dd.Convertor()
    cv.prepare_for_recv(dt, count, src)
    cv.unpack(out, dt.size * count)
torch.cuda.synchronize()
print("packed and unpacked", dt.size * count, "bytes x 20")
