#!/usr/bin/env python3
"""Headline benchmark for the MI355X reduction-collective hot path.

BASELINE.json metric: "Allreduce busBW GB/s @256MiB fp32 SUM at 2/4/8 GPUs;
MPI_Op HBM GB/s".

* N = 1 (configs[1]): the MPI_Op 3-buffer kernel, fp32 SUM, 1 GiB per buffer
  (the top of the 4 KiB-1 GiB sweep; 3 GiB of HBM traffic per step, well past
  the 256 MiB Infinity Cache).  value = algorithmic HBM GB/s = 3*n*4 B / t.
* N > 1 (configs[3] headline point): MPI_Allreduce fp32 SUM of 256 MiB per
  rank through the xGMI IPC collective.  value = busBW = S/t * 2(N-1)/N.

A step is one pass of the hot path over one batch of synthetic input that is
already resident in HBM.  Timing: W untimed warmup steps, barrier +
synchronize, K timed steps, barrier + synchronize, max over ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Deployment requirement: the peers' IPC mappings need
# the HSA runtime's dmabuf IPC mode.  Set before torch or the library touch
# the GPU, unless the environment already chose (the library's load-time
# constructor applies the same default to an mpirun job).
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
XGMI_LINK_GBS = 153.0          # per-link, R(N) = (N-1) x 153
METRIC = "Allreduce busBW GB/s @256MiB fp32 SUM at 2/4/8 GPUs; MPI_Op HBM GB/s"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--op-bytes", type=int, default=1 << 30, help="bytes per op buffer (N=1)")
    p.add_argument("--ar-bytes", type=int, default=256 << 20, help="allreduce bytes (N>1)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-extras", action="store_true",
                   help="N>1: skip the exactness check, size sweep and configs[4] collectives; "
                        "N=1: skip the one-sided / point-to-point rows")
    return p.parse_args()


def host_cpu() -> dict:
    """The host the CPU baseline ran on (BASELINE.md §5 asks for nproc and
    the CPU model beside the core count used)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        allowed = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        allowed = None
    return {"nproc": os.cpu_count(), "cpus_allowed": allowed, "cpu_model": model}


def cpu_baseline_op(seconds: float) -> dict:
    """The oracle's op/base restatement (scalar C loop, 1 thread) on a
    bounded sample of the same workload: 3-buffer fp32 SUM, 64 MiB/buffer."""
    import numpy as np

    from oracle import oracle as orc

    n = (64 << 20) // 4
    rng = np.random.default_rng(20261015)
    a = rng.standard_normal(n, dtype=np.float32)
    b = rng.standard_normal(n, dtype=np.float32)
    out = np.empty_like(a)
    orc.time_op_3buff(3, 15, a, b, out, n, 1)  # warm
    iters, total = 0, 0.0
    while total < seconds:
        total += orc.time_op_3buff(3, 15, a, b, out, n, 4)
        iters += 4
    gbs = 3.0 * n * 4 * iters / total / 1e9
    return {"value": round(gbs, 3), "unit": "GB/s", "cores": 1, "kind": "port", **host_cpu(),
            "sample": f"oracle op/base restatement, 3-buffer fp32 SUM, 64 MiB/buffer, "
                      f"{iters} iterations in {total:.1f} s, 1 thread"}


def bench_op(args):
    import torch

    from ompi_amd import op as mop

    n = args.op_bytes // 4
    g = torch.Generator(device="cuda").manual_seed(20261015)
    a = torch.randn(n, device="cuda", generator=g)
    b = torch.randn(n, device="cuda", generator=g)
    out = torch.empty_like(a)
    stream = torch.cuda.current_stream()
    for _ in range(args.warmup):
        mop.reduce_local_3buff_async(a, b, out, n, mop.MPI_FLOAT, mop.MPI_SUM, stream=stream)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        mop.reduce_local_3buff_async(a, b, out, n, mop.MPI_FLOAT, mop.MPI_SUM, stream=stream)
    ev1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps  # events on the launch stream
    algo_bytes = 3.0 * n * 4
    achieved = algo_bytes / (kernel_ms * 1e-3) / 1e9
    res = {
        "metric": METRIC,
        "value": round(algo_bytes * args.steps / wall / 1e9, 2),
        "unit": "GB/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (torch.randn, seed 20261015), resident in HBM",
        "config": {"workload": "MPI_Op 3-buffer SUM fp32, 1 GiB per buffer (BASELINE configs[1])",
                   "count": n, "bytes_per_buffer": args.op_bytes, "op": "MPI_SUM",
                   "datatype": "MPI_FLOAT", "kernel": "op_vec_kernel<float,SUM,3buff>"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": load_traffic("op_sum_f32_3buff_1GiB"),
                     "kernel_ms": round(kernel_ms, 4),
                     "algorithmic_bytes_per_launch": int(algo_bytes)},
    }
    return res


def load_traffic(key: str):
    """HBM bytes per launch from the committed PMC pass (profiles/pmc.json,
    FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM + WRITE_SIZE)."""
    path = os.path.join(ROOT, "profiles", "pmc.json")
    try:
        with open(path) as f:
            return json.load(f).get(key)
    except (OSError, ValueError):
        return None


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` started without a launcher: run the same command
    as N ranks under torch.distributed.run (one process per GPU, rendezvous
    on 127.0.0.1) and return its exit status.  Called before anything here
    touches the GPU; the ranks are children, so nothing is exec'd."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + sys.argv[1:]
    print(f"[bench] no WORLD_SIZE: launching {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.run(cmd).returncode


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 or args.gpus > 1:
        from ompi_amd import coll_bench
        try:
            res = coll_bench.bench_allreduce(args, METRIC, XGMI_LINK_GBS)
        except Exception as e:
            # say what failed on the one line the driver reads, then fail
            if int(os.environ.get("RANK", "0")) == 0:
                print(json.dumps({"metric": METRIC, "value": 0.0, "unit": "GB/s",
                                  "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                                  "higher_is_better": True, "scaling": "weak",
                                  "vs_baseline": None, "dtype": "f32", "data": "synthetic",
                                  "config": {"workload": "MPI_Allreduce fp32 SUM 256 MiB"},
                                  "error": f"{type(e).__name__}: {e}"}), flush=True)
            raise
        if res is None:
            return
    else:
        res = bench_op(args)
        if not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline_op(args.cpu_seconds)
            try:  # BASELINE configs[0]: the host-only allreduce row (never breaks the line)
                from ompi_amd import coll_bench
                row = coll_bench.cpu_baseline_ring(8, 64 << 20, 2.0 * 7 / 8, warmup=5, iters=20)
                row["config"] = ("BASELINE configs[0]: MPI_Allreduce MPI_SUM MPI_FLOAT 64 MiB, 8 host "
                                 "processes, coll/tuned ring_segmented (1 MiB segments) + op/base")
                res["cpu_allreduce_configs0"] = row
            except Exception as e:  # noqa: BLE001
                res["cpu_allreduce_configs0_error"] = f"{type(e).__name__}: {e}"
        if not args.no_extras:
            try:  # SURVEY §8f rows 1 / 4 on one GPU; never breaks the headline
                from ompi_amd import coll_bench
                res["next_rows_n1"] = coll_bench.single_gpu_rows()
            except Exception as e:  # noqa: BLE001
                res["next_rows_n1_error"] = f"{type(e).__name__}: {e}"
            try:  # BASELINE configs[1] / [2] at their top sizes; never breaks the headline
                from ompi_amd import coll_bench
                res["config_rows_n1"] = coll_bench.config_rows()
            except Exception as e:  # noqa: BLE001
                res["config_rows_n1_error"] = f"{type(e).__name__}: {e}"
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
