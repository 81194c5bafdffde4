#!/usr/bin/env python3
"""Small-call latency breakdown, N ranks sharing one GPU: blocking allreduce
vs MPI_Iallreduce (post, wait, free timed separately) vs a persistent start,
and device-buffer sendrecv at small sizes.  One JSON line per point from
rank 0 (max over ranks of the per-call mean).

usage: python tools/nb_latency_probe.py N [sizes_bytes,...]
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
    from ompi_amd import coll, pml
    from ompi_amd import op as mop
    rank, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=n)
    comm = coll.Communicator.from_torch_distributed(device=0)
    sizes = [int(v) for v in os.environ["NBP_SIZES"].split(",")]
    steps = int(os.environ.get("NBP_STEPS", "50"))
    F, SUM = mop.MPI_FLOAT, mop.MPI_SUM

    def worst(t):
        out = [0.0] * n
        dist.all_gather_object(out, t)
        return round(max(out) * 1e6, 2)

    def timed(fn):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        return worst((time.perf_counter() - t0) / steps)

    for nbytes in sizes:
        count = max(nbytes // 4, 1)
        x = torch.ones(count, device="cuda")
        y = torch.empty_like(x)
        row = {"ranks": n, "bytes": nbytes}
        row["allreduce_us"] = timed(lambda: comm.allreduce(x, y, count, F, SUM))
        plan = comm.allreduce_init(x, y, count, F, SUM)
        row["persistent_start_wait_us"] = timed(lambda: (plan.start(), plan.wait()))
        plan.free()
        parts = {"post": 0.0, "wait": 0.0, "free": 0.0}

        def nb():
            t0 = time.perf_counter()
            r = comm.iallreduce(x, y, count, F, SUM)
            t1 = time.perf_counter()
            r.wait()
            t2 = time.perf_counter()
            r.free()
            t3 = time.perf_counter()
            parts["post"] += t1 - t0
            parts["wait"] += t2 - t1
            parts["free"] += t3 - t2
        row["iallreduce_post_wait_free_us"] = timed(nb)
        tot = steps + 5
        row["iallreduce_parts_us_rank0"] = {k: round(v / tot * 1e6, 2) for k, v in parts.items()}
        row["exact"] = bool(torch.all(y == float(n)).item())
        # device sendrecv ring
        src, dst = (rank + 1) % n, (rank - 1) % n
        for kind in ("device",):  # host buffers: tools/pml_host_path_ab.sh
            dev = "cuda" if kind == "device" else "cpu"
            a = torch.full((count,), float(rank), device=dev)
            b = torch.empty_like(a)
            row[f"sendrecv_{kind}_us"] = timed(
                lambda: pml.sendrecv(comm, a, src, 7, b, dst, 7, nbytes, nbytes))
            row[f"sendrecv_{kind}_exact"] = bool(torch.all(b == float(dst)).item())
        if rank == 0:
            print(json.dumps(row), flush=True)
        del x, y
    comm.free()
    dist.barrier()


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    sizes = sys.argv[2] if len(sys.argv) > 2 else "8,65536,1048576"
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), NBP_SIZES=sizes, NBP_WORKER="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)], env=env))
    rc = 0
    for p in procs:
        rc |= p.wait(timeout=600)
    sys.exit(rc)


if __name__ == "__main__":
    if os.environ.get("NBP_WORKER"):
        worker()
    else:
        main()
