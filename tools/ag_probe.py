#!/usr/bin/env python3
"""Allgather / bcast per-call time, N ranks sharing one GPU (the bench's
config5 shape: 64 MiB total), default path and landing path; one JSON line
per point from rank 0.  usage: python tools/ag_probe.py N [total_bytes]
(AG_PROF_DIR=dir: rank 0 runs under rocprofv3 --kernel-trace)."""
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
    from ompi_amd import coll
    rank, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=n)
    comm = coll.Communicator.from_torch_distributed(device=0)
    total = int(os.environ["AG_TOTAL"])
    blk = total // n
    x = torch.full((blk,), rank, dtype=torch.uint8, device="cuda")
    y = torch.empty(total, dtype=torch.uint8, device="cuda")
    steps = 10
    for land in (0, 1):
        comm.set_param("land_blocking", land)
        for name, fn in (("allgather", lambda: comm.allgather(x, y, blk)),
                         ("bcast", lambda: comm.bcast(y, total, 0))):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(steps):
                fn()
            torch.cuda.synchronize()
            t = (time.perf_counter() - t0) / steps
            worst = [0.0] * n
            dist.all_gather_object(worst, t)
            if rank == 0:
                print(json.dumps({"ranks": n, "coll": name, "land_blocking": land, "total": total,
                                  "us": round(max(worst) * 1e6, 1)}), flush=True)
    comm.free()
    dist.barrier()


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    total = sys.argv[2] if len(sys.argv) > 2 else str(64 << 20)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), AG_TOTAL=total, AG_WORKER="1")
        cmd = [sys.executable, os.path.abspath(__file__)]
        if r == 0 and os.environ.get("AG_PROF_DIR"):  # rank 0's kernels traced
            cmd = ["rocprofv3", "--kernel-trace", "-d", os.environ["AG_PROF_DIR"], "-o", "ag",
                   "--"] + cmd
        procs.append(subprocess.Popen(cmd, env=env))
    rc = 0
    for p in procs:
        rc |= p.wait(timeout=600)
    sys.exit(rc)


if __name__ == "__main__":
    if os.environ.get("AG_WORKER"):
        worker()
    else:
        main()
