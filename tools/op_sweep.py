#!/usr/bin/env python3
"""BASELINE configs[1]: single-GPU MPI_Op 3-buffer sweep — SUM / MAX / BAND
over int32 / fp32 / fp64 (BAND: int32 only, as op/base defines it), 4 KiB to
1 GiB per buffer, plus the 2-buffer form and MAXLOC DOUBLE_INT at the top
size.  One JSON line per point: kernel time from HIP events on the launch
stream (median of 5 batches), algorithmic GB/s = 3 * bytes / t, fraction of
the 8 TB/s HBM peak.  Sizes below ~64 MiB are launch/latency bound and run
out of the 256 MiB Infinity Cache: report, don't read them as HBM rates."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from ompi_amd import op as mop  # noqa: E402

PEAK = 8000.0


def time_op(fn, iters):
    s = torch.cuda.current_stream()
    for _ in range(3):
        fn(s)
    vals = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(iters):
            fn(s)
        e1.record(s)
        torch.cuda.synchronize()
        vals.append(e0.elapsed_time(e1) / iters)
    return statistics.median(vals)


def main():
    top = int(os.environ.get("SWEEP_TOP", 1 << 30))
    sizes = []
    b = 4096
    while b <= top:
        sizes.append(b)
        b *= 4 if b < (1 << 26) else 2
    cases = [(mop.MPI_SUM, mop.MPI_INT32_T), (mop.MPI_SUM, mop.MPI_FLOAT), (mop.MPI_SUM, mop.MPI_DOUBLE),
             (mop.MPI_MAX, mop.MPI_INT32_T), (mop.MPI_MAX, mop.MPI_FLOAT), (mop.MPI_MAX, mop.MPI_DOUBLE),
             (mop.MPI_BAND, mop.MPI_INT32_T)]
    a = torch.empty(top, dtype=torch.uint8, device="cuda").random_()
    bb = torch.empty(top, dtype=torch.uint8, device="cuda").random_()
    o = torch.empty(top, dtype=torch.uint8, device="cuda")
    for op, dt in cases:
        for nbytes in sizes:
            n = nbytes // dt.extent
            iters = max(3, min(200, (1 << 30) // nbytes))
            ms = time_op(lambda s: mop.reduce_local_3buff_async(a, bb, o, n, dt, op, stream=s), iters)
            gbs = 3 * n * dt.extent / (ms * 1e-3) / 1e9
            print(json.dumps({"form": "3buff", "op": op.name, "type": dt.name, "bytes": nbytes,
                              "ms": round(ms, 5), "GBps": round(gbs, 1),
                              "frac_hbm": round(gbs / PEAK, 4)}), flush=True)
    for op, dt in [(mop.MPI_SUM, mop.MPI_FLOAT), (mop.MPI_MAX, mop.MPI_DOUBLE),
                   (mop.MPI_MAXLOC, mop.MPI_DOUBLE_INT)]:
        n = top // dt.extent
        for form in ("2buff", "3buff"):
            if form == "2buff":
                ms = time_op(lambda s: mop.reduce_local_async(a, bb, n, dt, op, stream=s), 5)
            else:
                ms = time_op(lambda s: mop.reduce_local_3buff_async(a, bb, o, n, dt, op, stream=s), 5)
            gbs = 3 * n * dt.extent / (ms * 1e-3) / 1e9
            print(json.dumps({"form": form, "op": op.name, "type": dt.name, "bytes": top,
                              "ms": round(ms, 5), "GBps": round(gbs, 1),
                              "frac_hbm": round(gbs / PEAK, 4)}), flush=True)


if __name__ == "__main__":
    main()
