#!/usr/bin/env python3
"""BASELINE configs[2]: device-buffer pack/unpack through the convertor on
one GPU.  vector(count, blocklen in {1,2,8,64} doubles, stride 2*blocklen),
packed 4 KiB .. 1 GiB; blacs-like indexed (descending block lengths, tiled);
struct {int, double}.  Chunk sizes: whole stream and 64 KiB (one launch per
convertor call, as the PML would drive it).  Algorithmic bytes = 2 x packed
bytes (strided read + dense write).  One JSON line per point."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from ompi_amd import datatype as dd  # noqa: E402

PEAK = 8000.0


def span(dt, count):
    return (count - 1) * dt.extent + dt.true_span


def bench_type(name, dt, count, chunks, top_iters=20):
    total = dt.size * count
    src = torch.empty(span(dt, count), dtype=torch.uint8, device="cuda").random_()
    packed = torch.empty(total, dtype=torch.uint8, device="cuda")
    for chunk in chunks:
        c = min(chunk, total)
        ncalls = (total + c - 1) // c
        if ncalls > 20000:
            continue

        def run(kind):
            cv = dd.Convertor()
            if kind == "pack":
                cv.prepare_for_send(dt, count, src)
                fn = cv.pack
            else:
                cv.prepare_for_recv(dt, count, src)
                fn = cv.unpack
            pos = 0
            while pos < total:
                _, n = fn(packed.data_ptr() + pos, c)
                pos += n

        for kind in ("pack", "unpack"):
            iters = max(10, min(top_iters, (1 << 28) // max(total, 1)))
            run(kind)
            torch.cuda.synchronize()
            vals = []
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(iters):
                    run(kind)
                e1.record()
                torch.cuda.synchronize()
                vals.append(e0.elapsed_time(e1) / iters)
            ms = statistics.median(vals)
            gbs = 2 * total / (ms * 1e-3) / 1e9
            print(json.dumps({"type": name, "kind": kind, "packed_bytes": total, "chunk": c,
                              "calls": ncalls, "ms": round(ms, 5), "GBps": round(gbs, 1),
                              "frac_hbm": round(gbs / PEAK, 4), "nelems": dt.nelems}), flush=True)


def main():
    top = int(os.environ.get("SWEEP_TOP", 1 << 30))
    only = os.environ.get("SWEEP_TYPES")  # comma-separated type names (default: all)
    want = (lambda n: True) if not only else (lambda n: n in only.split(","))
    d = dd.predefined("MPI_DOUBLE")
    sizes = [4096, 1 << 20, 64 << 20, 256 << 20, top]
    for bl in (1, 2, 8, 64):
        if not want(f"vector_bl{bl}"):
            continue
        for packed in sizes:
            count = packed // (8 * bl)
            dt = dd.type_vector(count, bl, 2 * bl, d)
            bench_type(f"vector_bl{bl}", dt, 1, [packed, 65536])
            dt.free()
    # blacs-style indexed (ddt_lib.c:273-300 lengths), tiled: count elements
    i32 = dd.predefined("MPI_INT")
    lens = [13, 13, 13, 13, 13, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1]
    disps = [286, 308, 330, 352, 374, 396, 419, 442, 465, 488, 511, 534, 557, 580, 603, 626, 649, 672]
    blacs = dd.type_indexed(lens, disps, i32)
    big = [int(x) for x in os.environ.get("SWEEP_SIZES", "1048576,67108864,268435456").split(",")]
    chunks = lambda p: [p] if os.environ.get("SWEEP_WHOLE") == "1" else [p, 65536]
    for packed in big if want("blacs_indexed") else ():
        bench_type("blacs_indexed", blacs, packed // blacs.size, chunks(packed))
    st = dd.type_struct([1, 1], [0, 8], [i32, d])
    for packed in big if want("struct_int_double") else ():
        bench_type("struct_int_double", st, packed // st.size, chunks(packed))


if __name__ == "__main__":
    main()
