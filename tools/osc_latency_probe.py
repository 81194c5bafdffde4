#!/usr/bin/env python3
"""Small one-sided operations under MPI_Win_lock_all, N ranks sharing one
GPU: per-call time of MPI_Fetch_and_op (int64 SUM, +1) on a counter every
rank hits (rank 0's) and on the next rank's, MPI_Compare_and_swap, and
MPI_Accumulate (fp32 SUM) of 8 B .. 64 KiB into the next rank — each call
followed by MPI_Win_flush (the result is usable), and pipelined (k calls,
one flush).  One JSON line per row from rank 0: max over ranks of the
per-call mean.  Env OMPI_AMD_OSC_SMALL_BYTES=0 runs the accumulate-lock
operations as separate lock / copy / op / unlock launches (the A/B).

usage: python tools/osc_latency_probe.py N
"""
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker():
    import torch
    import torch.distributed as dist
    from ompi_amd import coll, osc
    from ompi_amd import op as mop
    rank, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=n)
    comm = coll.Communicator.from_torch_distributed(device=0)
    steps = int(os.environ.get("OLP_STEPS", "40"))
    stream = torch.cuda.Stream()
    I64, I32, F, SUM = mop.MPI_INT64_T, mop.MPI_INT32_T, mop.MPI_FLOAT, mop.MPI_SUM
    nxt = (rank + 1) % n
    S = 1 << 20
    win = osc.Window.allocate(comm, S, disp_unit=1)

    def worst(t):
        out = [0.0] * n
        dist.all_gather_object(out, t)
        return round(max(out) * 1e6, 2)

    def timed(fn, k=1):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        return worst((time.perf_counter() - t0) / (steps * k))

    one = torch.ones(1, dtype=torch.int64, device="cuda")
    res = torch.empty(1, dtype=torch.int64, device="cuda")
    cmp_ = torch.zeros(1, dtype=torch.int32, device="cuda")
    org = torch.full((1,), rank + 1, dtype=torch.int32, device="cuda")
    res32 = torch.empty(1, dtype=torch.int32, device="cuda")
    x = torch.ones((64 << 10) // 4, device="cuda")
    rows = []
    try:
        win.lock_all(stream=stream)

        def fop(t, disp=0):
            win.fetch_and_op(one, res, I64, t, disp, SUM, stream=stream)
            win.flush(t, stream=stream)
        rows.append({"op": "fetch_and_op_flush", "target": "rank0 (all ranks)", "us": timed(lambda: fop(0))})
        rows.append({"op": "fetch_and_op_flush", "target": "next rank", "us": timed(lambda: fop(nxt, 16))})
        k = 16

        def fop_k():
            for _ in range(k):
                win.fetch_and_op(one, res, I64, nxt, 8, SUM, stream=stream)
            win.flush(nxt, stream=stream)
        rows.append({"op": "fetch_and_op_x16_one_flush", "target": "next rank", "us": timed(fop_k, k)})

        def cas():
            win.compare_and_swap(org, cmp_, res32, I32, nxt, 64, stream=stream)
            win.flush(nxt, stream=stream)
        rows.append({"op": "compare_and_swap_flush", "target": "next rank", "us": timed(cas)})
        for nbytes in (8, 1024, 16 << 10, 64 << 10):
            cnt = nbytes // 4

            def acc():
                win.accumulate(x, cnt, F, nxt, 4096, SUM, stream=stream)
                win.flush(nxt, stream=stream)
            rows.append({"op": "accumulate_sum_f32_flush", "bytes": nbytes, "target": "next rank",
                         "us": timed(acc)})
        win.unlock_all(stream=stream)
        # rank 0's counter took 3 + steps fetch_and_op from every rank
        got = torch.empty(1, dtype=torch.int64, device="cuda")
        win.lock(0, osc.LOCK_SHARED, stream=stream)
        win.get(got, 0, 0, 8, stream=stream)
        win.unlock(0, stream=stream)
        stream.synchronize()
        exact = int(got.item()) == n * (3 + steps)
    finally:
        win.free()
    if rank == 0:
        small = os.environ.get("OMPI_AMD_OSC_SMALL_BYTES", "default (16384)")
        for r in rows:
            print(json.dumps(dict(r, ranks=n, small_bytes=small, counter_exact=exact)), flush=True)
    comm.free()
    dist.barrier()


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), OLP_WORKER="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)], env=env))
    rc = 0
    for p in procs:
        rc |= p.wait(timeout=600)
    sys.exit(rc)


if __name__ == "__main__":
    if os.environ.get("OLP_WORKER"):
        worker()
    else:
        main()
