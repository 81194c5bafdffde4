#!/usr/bin/env python3
"""BASELINE configs[2] at the PML's fragment size: a 256 MiB packed stream
moved through the convertor's fAdvance in 64 KiB fragments.

Three ways of driving it (one JSON line each, per datatype and direction):
  per_call   one fAdvance call per fragment (out_size = 1) and the
             synchronisation the blocking convertor does after each call —
             what a PML that converts one fragment at a time costs;
  per_call_async  the same calls with no per-call synchronisation
             (CONVERTOR_CUDA_ASYNC: the PML waits on the stream later);
  iov_batch  ONE fAdvance call over all 4096 fragments as an iovec array
             (one kernel launch; ompi_amd_ddt_pack_iov).
Algorithmic bytes = 2 x packed bytes (typed read + packed write), against
the 8 TB/s HBM peak.  Times are HIP events on the convertor's stream.
"""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from ompi_amd import _lib  # noqa: E402
from ompi_amd import datatype as dd  # noqa: E402

PEAK = 8000.0
TOTAL = int(os.environ.get("FRAG_TOTAL", 256 << 20))
FRAG = int(os.environ.get("FRAG_BYTES", 64 << 10))


def types():
    d = dd.predefined("MPI_DOUBLE")
    i = dd.predefined("MPI_INT")
    out = []
    for bl in (1, 8, 64):
        count = TOTAL // (8 * bl)
        out.append((f"vector_bl{bl}", dd.type_vector(count, bl, 2 * bl, d), 1))
    st = dd.type_struct([1, 1], [0, 8], [i, d])
    out.append(("struct_int_double", st, TOTAL // st.size))
    return out


def main():
    torch.cuda.init()
    stream = torch.cuda.Stream()
    lib = _lib.load()
    nfrag = TOTAL // FRAG
    for name, dt, count in types():
        total = dt.size * count
        span = (count - 1) * dt.extent + dt.true_span
        typed = torch.empty(span, dtype=torch.uint8, device="cuda").random_()
        packed = torch.empty(total, dtype=torch.uint8, device="cuda")
        base = packed.data_ptr()
        iovs = (_lib.Iovec * nfrag)(*[_lib.Iovec(base + k * FRAG, FRAG) for k in range(nfrag)])
        for kind in ("pack", "unpack"):
            modes = os.environ.get("FRAG_MODES", "per_call,per_call_async,iov_batch").split(",")
            for mode in modes:
                def run():
                    cv = dd.Convertor()
                    (cv.prepare_for_send if kind == "pack" else cv.prepare_for_recv)(
                        dt, count, typed, stream)
                    fn = cv.pack_iov if kind == "pack" else cv.unpack_iov
                    if mode == "iov_batch":  # prebuilt iovec array: the call is all that is timed
                        out = ctypes.c_uint32(nfrag)
                        moved = ctypes.c_size_t(0)
                        abi = lib.ompi_amd_ddt_pack_iov if kind == "pack" else lib.ompi_amd_ddt_unpack_iov
                        rc = abi(dt._handle, count, typed.data_ptr(), 0, iovs, ctypes.byref(out),
                                 ctypes.byref(moved), stream.cuda_stream)
                        assert rc == 1 and moved.value == total, (rc, moved.value)
                        return
                    pos = 0
                    while pos < total:
                        rc, _, _, moved = fn([(base + pos, FRAG)])
                        pos += moved
                        if mode == "per_call":
                            lib.ompi_amd_stream_synchronize(stream.cuda_stream)
                    assert pos == total
                run()
                torch.cuda.synchronize()
                vals = []
                for _ in range(5):
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    run()
                    e1.record(stream)
                    torch.cuda.synchronize()
                    vals.append(e0.elapsed_time(e1))
                ms = statistics.median(vals)
                gbs = 2 * total / (ms * 1e-3) / 1e9
                print(json.dumps({"type": name, "kind": kind, "mode": mode, "packed_bytes": total,
                                  "fragment": FRAG, "fragments": nfrag, "ms": round(ms, 4),
                                  "GBps": round(gbs, 1), "frac_hbm": round(gbs / PEAK, 4)}),
                      flush=True)
        dt.free()


if __name__ == "__main__":
    main()
