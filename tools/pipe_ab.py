#!/usr/bin/env python3
"""Phased vs pipelined staged allreduce schemes, N ranks sharing one GPU
(VERDICT r3 item 5 rehearsal; HBM-bound — not an xGMI figure).

For each size and scheme pair (staged pull 0 / pull_pipe 6, push-gather 2 /
push_pipe 4, push-land 3 / land_pipe 5) x grid: per-call time (max over
ranks of the mean of K calls between barriers; PIPE_AB_PASSES: the
pipelined schemes' passes per workgroup, PIPE_AB_SCHEMES: a subset), and for the phased schemes
the per-phase kernel times the library's profile mode records (fold,
gather, scatter).  One JSON line per point from rank 0.

usage: python tools/pipe_ab.py N [sizes_bytes,...] [grids,...]
(launches N child processes; run it under rocprofv3 --kernel-trace to see
the copy / barrier / fold kernels of the phased schemes beside the single
pipelined launch)
"""
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PAIRS = ((0, "pull"), (6, "pull_pipe"), (2, "push"), (4, "push_pipe"), (3, "push_land"),
         (5, "land_pipe"))


def worker():
    import torch
    import torch.distributed as dist
    from ompi_amd import coll
    from ompi_amd import op as mop
    rank, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=n)
    comm = coll.Communicator.from_torch_distributed(device=0)
    sizes = [int(v) for v in os.environ["PIPE_AB_SIZES"].split(",")]
    grids = [int(v) for v in os.environ["PIPE_AB_GRIDS"].split(",")]
    steps = int(os.environ.get("PIPE_AB_STEPS", "10"))
    passes = [int(v) for v in os.environ.get("PIPE_AB_PASSES", "1").split(",")]
    only = os.environ.get("PIPE_AB_SCHEMES")  # comma-separated scheme names
    stream = torch.cuda.current_stream()
    for nbytes in sizes:
        count = nbytes // 4
        x = torch.ones(count, device="cuda")
        y = torch.empty_like(x)
        for alg, name in PAIRS:
          if only and name not in only.split(","):
              continue
          for sl in (passes if alg in (4, 5, 6) else passes[:1]):
            comm.set_param("algorithm", alg)
            comm.set_param("pipe_passes", sl)
            for g in grids:
                comm.set_param("blocks", g)

                def call():
                    comm.allreduce(x, y, count, mop.MPI_FLOAT, mop.MPI_SUM, stream=stream)

                for _ in range(3):
                    call()
                torch.cuda.synchronize()
                dist.barrier()
                t0 = time.perf_counter()
                for _ in range(steps):
                    call()
                torch.cuda.synchronize()
                t = (time.perf_counter() - t0) / steps
                worst = [0.0] * n
                dist.all_gather_object(worst, t)
                comm.set_param("profile", 1)
                for _ in range(steps):
                    call()
                torch.cuda.synchronize()
                comm.set_param("profile", 0)
                phases = {}
                for k, ph in enumerate(("fold", "gather", "scatter")):
                    ms, calls = comm.phase_ms(k)
                    if calls:
                        phases[ph] = round(ms / calls * 1e3, 1)
                ok = bool(torch.all(y == float(n)).item())
                if rank == 0:
                    print(json.dumps({"ranks": n, "bytes": nbytes, "scheme": name, "algorithm": alg,
                                      "blocks": g, "pipe_passes": sl if alg in (4, 5, 6) else None,
                                      "us_per_call": round(max(worst) * 1e6, 1),
                                      "phase_kernel_us": phases, "exact": ok,
                                      "pipe_calls": comm.get_param("pipe_calls")}), flush=True)
                dist.barrier()
        del x, y
    comm.free()
    dist.barrier()


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    sizes = sys.argv[2] if len(sys.argv) > 2 else str(256 << 20)
    grids = sys.argv[3] if len(sys.argv) > 3 else "256,512"
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), PIPE_AB_SIZES=sizes, PIPE_AB_GRIDS=grids,
                   PIPE_AB_WORKER="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)], env=env))
    rc = 0
    for p in procs:
        rc |= p.wait(timeout=900)
    sys.exit(rc)


if __name__ == "__main__":
    if os.environ.get("PIPE_AB_WORKER"):
        worker()
    else:
        main()
