"""Single-process probe of the one-sided and point-to-point data kernels on
one MI355X (communicator of size 1, the target is this rank's own window,
so the kernels are HBM-bound exactly as the op kernel is):

  accumulate  lock + acc_kernel + unlock: reads target and origin, writes
              target (3 bytes of HBM traffic per window byte)
  put         copy kernel origin -> window (2 bytes per byte)
  self send   sendrecv to self: the receiver's copy kernel (2 bytes per byte)

Prints one JSON line per case (event-timed on a dedicated stream).
usage: python tools/osc_probe.py [MiB]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from ompi_amd import coll, osc, pml  # noqa: E402
from ompi_amd import op as mop  # noqa: E402


def timed(fn, stream, iters=20, warm=3):
    for _ in range(warm):
        fn()
    stream.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for _ in range(iters):
        fn()
    b.record(stream)
    b.synchronize()
    return a.elapsed_time(b) / iters / 1e3


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    S = mib << 20
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    comm = coll.Communicator(f"probe_{os.getpid()}", 0, 1, 0)
    win = osc.Window.allocate(comm, S, disp_unit=4)
    x = torch.ones(S // 4, device="cuda")
    r = torch.empty_like(x)
    torch.cuda.synchronize()
    out = []
    for op, dt in ((mop.MPI_SUM, mop.MPI_FLOAT), (mop.MPI_MAX, mop.MPI_DOUBLE),
                   (mop.MPI_MAXLOC, mop.MPI_DOUBLE_INT)):
        cnt = S // dt.extent
        t = timed(lambda: win.accumulate(x, cnt, dt, 0, 0, op, stream=s), s)
        out.append({"case": f"accumulate_{op.name}_{dt.name}", "bytes": S, "ms": round(t * 1e3, 4),
                    "hbm_gbs": round(3 * S / t / 1e9, 1)})
    t = timed(lambda: win.get_accumulate(x, r, S // 4, mop.MPI_FLOAT, 0, 0, mop.MPI_SUM, stream=s), s)
    out.append({"case": "get_accumulate_SUM_MPI_FLOAT", "bytes": S, "ms": round(t * 1e3, 4),
                "hbm_gbs": round(5 * S / t / 1e9, 1)})
    t = timed(lambda: win.put(x, 0, 0, S, stream=s), s)
    out.append({"case": "put", "bytes": S, "ms": round(t * 1e3, 4), "hbm_gbs": round(2 * S / t / 1e9, 1)})
    t = timed(lambda: pml.sendrecv(comm, x, 0, 5, r, 0, 5, stream=s), s, iters=10)
    out.append({"case": "sendrecv_self", "bytes": S, "ms": round(t * 1e3, 4),
                "hbm_gbs": round(2 * S / t / 1e9, 1)})
    t = timed(lambda: mop.reduce_local_async(x, r, S // 4, mop.MPI_FLOAT, mop.MPI_SUM, stream=s), s)
    out.append({"case": "op_2buff_SUM_MPI_FLOAT (reference point)", "bytes": S,
                "ms": round(t * 1e3, 4), "hbm_gbs": round(3 * S / t / 1e9, 1)})
    for o in out:
        print(json.dumps(o), flush=True)
    win.free()
    comm.free()


if __name__ == "__main__":
    main()
