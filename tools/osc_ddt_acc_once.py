#!/usr/bin/env python3
"""The bench's derived-target accumulate row alone (bench.py next_rows_n1
accumulate_ddt_vector_bl1_f64): a size-1 communicator, a 256 MiB window, a
128 MiB packed f64 origin SUMmed into every other double (MPI_Type_vector
of single doubles at stride 2).  Prints one JSON line (event-timed); run
under rocprofv3 --kernel-trace / --pmc by tools/profile_ddt_acc.sh.
Algorithmic bytes per call 1.5 x S (origin read, target slots read and
written)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from ompi_amd import coll, osc  # noqa: E402
from ompi_amd import datatype as ddt  # noqa: E402
from ompi_amd import op as mop  # noqa: E402

S = int(os.environ.get("ACC_MIB", "256")) << 20
iters = int(os.environ.get("ACC_ITERS", "10"))
# ACC_WIN=allocate (the bench row: MPI_Win_allocate, the shadow arena) or
# create (MPI_Win_create over a torch allocation)
how = os.environ.get("ACC_WIN", "allocate")
s = torch.cuda.Stream()
comm = coll.Communicator(f"ddtacc_{os.getpid()}", 0, 1, torch.cuda.current_device())
if how == "create":
    wmem = torch.zeros(S // 4, device="cuda")
    win = osc.Window.create(comm, wmem, S, disp_unit=4)
else:
    win = osc.Window.allocate(comm, S, disp_unit=4)
x = torch.ones(S // 4, device="cuda")
tvec = ddt.type_vector(S // 16, 1, 2, ddt.predefined("MPI_DOUBLE")).commit()
torch.cuda.synchronize()


def fn():
    win.accumulate_ddt(x, S // 16, None, 0, 0, 1, tvec, mop.MPI_DOUBLE, mop.MPI_SUM, stream=s)


try:
    for _ in range(2):
        fn()
    s.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(iters):
        fn()
    b.record(s)
    b.synchronize()
    t = a.elapsed_time(b) / iters / 1e3
    print(json.dumps({"row": "accumulate_ddt_vector_bl1_f64", "window": how, "bytes": S, "ms": round(t * 1e3, 4),
                      "algorithmic_bytes": int(1.5 * S), "hbm_gbs": round(1.5 * S / t / 1e9, 1),
                      "frac_of_8TBs": round(1.5 * S / t / 8e12, 4)}), flush=True)
finally:
    win.free()
    comm.free()
