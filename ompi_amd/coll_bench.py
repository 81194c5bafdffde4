"""Multi-GPU leg of bench.py: MPI_Allreduce fp32 SUM over the xGMI IPC
collective, one process per GPU (torch.distributed.run), with RCCL's
allreduce of the same buffer timed beside it as the comparator.

busBW = S / t * 2(N-1)/N; roofline R(N) = (N-1) x 153 GB/s.
Before the timed region the data-movement scheme (pull, pull+push, push)
and the transfer grid are chosen by measurement among the variants that
are bit-exact on dataset E (a dynamic-rules file in coll/tuned terms); all
candidates are reported in config.schemes.  The dominant kernel is the
fused ring-order reduction (phase 0); its achieved rate is the xGMI bytes
arriving at this GPU during the launch over its event-timed duration.
"""
from __future__ import annotations

import os
import sys
import time


_PHASE = {"what": None, "t0": 0.0, "pending": None}
# An extras phase (after the headline was measured) that runs longer than
# this is taken as stuck: every rank's watchdog ends its process with exit
# status 3, and rank 0 first prints the headline line it already holds, so a
# hang in a side row never costs the driver the headline and never passes
# for a clean run.
EXTRAS_PHASE_LIMIT_S = float(os.environ.get("OMPI_AMD_BENCH_EXTRAS_LIMIT_S", "240"))


def _progress(rank, what):
    """One stderr line per bench phase on rank 0 (a long multi-rank run shows
    where it is; the GPU box's watchdog takes a silent run for a hung one)."""
    _PHASE["what"], _PHASE["t0"] = what, time.time()
    if rank == 0:
        import sys
        print(f"[bench] {time.strftime('%H:%M:%S')} {what}", file=sys.stderr, flush=True)


def _watchdog(comm, rank, world):
    """Every rank: a phase running over 30 s prints the communicator's epoch
    and (OMPI_AMD_DEBUG_PROGRESS=1) its barrier progress record; an extras
    phase past EXTRAS_PHASE_LIMIT_S ends the process (rank 0 prints the
    headline line first)."""
    import json
    import sys
    import threading

    def run():
        while True:
            time.sleep(15)
            what, t0 = _PHASE["what"], _PHASE["t0"]
            if what is None or time.time() - t0 < 30:
                continue
            vals = {}
            for k in ["epoch", "dbg_entered", "dbg_left"] + [f"dbg_seen{p}" for p in range(world)]:
                try:
                    vals[k] = comm.get_param(k)
                except Exception:  # noqa: BLE001 (debug record off)
                    pass
            print(f"[bench watchdog rank {rank}] {what} running {time.time() - t0:.0f} s: {vals}",
                  file=sys.stderr, flush=True)
            pending = _PHASE["pending"]
            if pending is not None and time.time() - t0 > EXTRAS_PHASE_LIMIT_S:
                if rank == 0:
                    pending["extras_error"] = (f"watchdog: '{what}' still running after "
                                               f"{time.time() - t0:.0f} s; extras abandoned")
                    print(json.dumps(dict(pending)), flush=True)
                sys.stderr.flush()
                os._exit(3)  # the headline line is out; the run still failed

    threading.Thread(target=run, daemon=True).start()


def _timed(fn, steps, warmup, dist, torch, dev="cuda"):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _settle(comm, fn, torch, limit=96):
    """Run a blocking allreduce until the library's autotune of its size
    bucket has decided (autotune_state 2), or it does not tune this size
    (state stays 0 or a settled bucket's 2): the first kTuneCalls = 72
    calls of a new large size try every candidate, slow grids included, and
    must not land inside a timed region (coll_ipc.hip, ompi_amd_allreduce).
    Every rank makes the same calls, so every rank stops at the same one."""
    for _ in range(limit):
        fn()
        torch.cuda.synchronize()
        if comm.get_param("autotune_state") != 1:
            return


def bench_allreduce(args, metric: str, link_gbs: float):
    import torch
    import torch.distributed as dist

    from . import coll
    from . import op as mop

    local = int(os.environ.get("LOCAL_RANK", "0"))
    # OMPI_AMD_BENCH_SHARE_GPU=1: rehearsal with every rank on cuda:0 (a
    # one-GPU box); RCCL refuses two ranks per GPU, so gloo carries the
    # timing barrier and the comparator is skipped.
    shared = os.environ.get("OMPI_AMD_BENCH_SHARE_GPU") == "1"
    nlocal = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
    if not shared and torch.cuda.device_count() < nlocal:
        # fewer GPUs than local ranks: a labelled rehearsal rather than a
        # crash in set_device (the line carries "shared_gpu_rehearsal": true)
        print(f"[bench] {torch.cuda.device_count()} GPU(s) for {nlocal} local ranks: "
              "every rank on cuda:0 (shared-GPU rehearsal)", file=sys.stderr, flush=True)
        shared = True
    if shared:
        local = 0
    torch.cuda.set_device(local)
    if shared:
        dist.init_process_group("gloo")
    else:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    tdev = "cpu" if shared else "cuda"
    rank, world = dist.get_rank(), dist.get_world_size()
    comm = coll.Communicator.from_torch_distributed(device=local)
    _watchdog(comm, dist.get_rank(), dist.get_world_size())

    n = args.ar_bytes // 4
    g = torch.Generator(device="cuda").manual_seed(20261015 + rank)
    x = torch.rand(n, device="cuda", generator=g) * 2 - 1
    y = torch.empty_like(x)
    stream = torch.cuda.current_stream()

    def ours():
        comm.allreduce(x, y, n, mop.MPI_FLOAT, mop.MPI_SUM, stream=stream)

    # The headline runs what coll/rocm ships (coll_rocm_module.c): staged
    # (coll_rocm_user_ipc 0) with coll_rocm_autotune 1 — the library itself
    # measures its staged schemes x grids on the first calls of a size and
    # keeps the fastest (ompi_amd_allreduce); the bench
    # never picks.  Every scheme, user-IPC ones included, is measured after
    # the headline, among the extras (each first checked bit-exact on
    # dataset E at this size), and reported under config.schemes only.
    S = n * 4
    factor = 2.0 * (world - 1) / world
    default = {"algorithm": comm.get_param("algorithm"), "user_ipc": comm.get_param("user_ipc"),
               "blocks": comm.get_param("blocks")}
    default_name = (f"{dict(ALGORITHMS)[default['algorithm']]}/"
                    f"{'user' if default['user_ipc'] else 'staged'}/{default['blocks']}")
    best = {"algorithm": default["algorithm"]}
    best_name = default_name
    # coll/rocm ships coll_rocm_autotune = 1 (a communicator built outside
    # the MCA glue starts with it off): the first calls of this size try
    # the candidates, every rank then runs the one whose slowest rank was
    # fastest (each candidate's best of two rounds) — what an MPI job gets
    # from its first allreduces of this size
    autotune = None
    if not os.environ.get("OMPI_AMD_BENCH_NO_AUTOTUNE"):
        comm.set_param("autotune", 1)
        _progress(rank, "autotune: one call per candidate")
        calls = 0
        while calls < 96:  # 36 candidates (18 with copy_nt fixed) x 2 rounds decide at the 72nd
            ours()
            torch.cuda.synchronize()
            calls += 1
            if comm.get_param("autotune_state") == 2:
                break
        if comm.get_param("autotune_state") == 2:
            a_c, b_c = comm.get_param("autotune_algorithm"), comm.get_param("autotune_blocks")
            nt_c = comm.get_param("autotune_copy_nt")
            best = {"algorithm": a_c}
            best_name = f"{dict(ALGORITHMS)[a_c]}/staged/{b_c}/{'nt' if nt_c else 'plain'}"
            autotune = {"choice": best_name, "calls": calls,
                        "worst_rank_us": {
                            f"{dict(ALGORITHMS)[comm.get_param(f'autotune_alg{k}')]}/staged/"
                            f"{comm.get_param(f'autotune_grid{k}')}/"
                            f"{'nt' if comm.get_param(f'autotune_nt{k}') else 'plain'}":
                            comm.get_param(f"autotune_us{k}")
                            for k in range(comm.get_param("autotune_ncand"))}}

    _progress(rank, f"headline: {best_name}")
    t = _timed(ours, args.steps, args.warmup, dist, torch, tdev)
    err = comm.error()
    # per-phase kernel time over one more profiled pass of K steps
    comm.set_param("profile", 1)
    for _ in range(args.steps):
        ours()
    torch.cuda.synchronize()
    comm.set_param("profile", 0)
    phases = [comm.phase_ms(k) for k in range(3)]  # fold, gather, scatter: (ms total, calls)
    default_exact = _exact_ok(comm, dist, torch, mop, n, rank, shared)

    t_rccl = None
    if not shared:
        rccl_buf = x.clone()

        def rccl():
            dist.all_reduce(rccl_buf)

        t_rccl = _timed(rccl, args.steps, args.warmup, dist, torch)

    busbw = S / (t / args.steps) * factor / 1e9
    busbw_rccl = S / (t_rccl / args.steps) * factor / 1e9 if t_rccl else None
    roof = (world - 1) * link_gbs
    # xGMI bytes arriving at this GPU during one launch of each phase kernel
    # (per rank, (N-1)/N x S moves over the links per direction and phase):
    #   fold    pull: peers' blocks pulled; pull+push: that plus the peers'
    #           finished blocks pushed in; push (user_ipc): finished blocks
    #           pushed in; push-gather (staged push, the default): none — it
    #           folds its landing slots locally (HBM)
    #   gather  the other owners' finished blocks pulled
    #   scatter the peers' input blocks pushed into this rank's landing slots
    alg, user = best["algorithm"], bool(comm.get_param("user_ipc"))
    part = (world - 1) / world * S
    # push-land (3): the fold stores its result into every peer's landing
    # buffer (part out), the second phase is a local copy; with user_ipc it
    # is the push scheme
    # the pipelined schemes (4-6) time one launch per call as "fold": both
    # transfer phases' bytes arrive during it (scatter or pull, then gather)
    fold_bytes = {0: part, 1: 2 * part, 2: part if user else 0.0, 3: part,
                  4: 2 * part, 5: 2 * part, 6: 2 * part}[alg]
    xgmi = {"fold": fold_bytes,
            "gather": part if alg in (0, 2) and not (alg == 2 and user) else 0.0,
            "scatter": part if alg in (2, 3) else 0.0}
    ph = {}
    for k, name in enumerate(("fold", "gather", "scatter")):
        ms, calls = phases[k]
        if calls:
            avg = ms / calls
            ph[name] = {"kernel_ms": round(avg, 4), "xgmi_bytes": int(xgmi[name]),
                        "gbs": round(xgmi[name] / (avg * 1e-3) / 1e9, 1) if xgmi[name] else None}
    xg = {k: v for k, v in ph.items() if v["gbs"]}
    dom = max(xg, key=lambda k: xg[k]["kernel_ms"]) if xg else None
    red_gbs = xg[dom]["gbs"] if dom else None
    roof = (world - 1) * link_gbs
    # the kernel behind each phase timer: the pipelined schemes (4-6) run
    # one pipe_allreduce_kernel per call, timed as "fold"
    kernel = ({"fold": "pipe_allreduce_kernel<float,SUM>"} if alg in PIPE_ALGS and not user else
              {"fold": "reduce_kernel<float,SUM,8>", "gather": "copy_kernel",
               "scatter": "copy_kernel"}).get(dom)
    # HBM + fabric bytes per launch of that phase's kernel from the committed
    # PMC passes (profiles/pmc.json, tools/profile_allreduce_pmc.sh): L2-to-
    # fabric requests of the launching GPU, local and peer memory alike
    traffic = _phase_traffic(world, alg, user, dom)
    res = {
        "metric": metric,
        "value": round(busbw, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(t * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic U(-1,1) per rank (seed 20261015+rank), resident in HBM",
        "config": {"workload": "MPI_Allreduce fp32 SUM 256 MiB per rank, xGMI IPC ring-order "
                               "fused reduce (BASELINE configs[3] headline point)",
                   "count": n, "bytes": S, "op": "MPI_SUM", "datatype": "MPI_FLOAT",
                   "parallelism": (f"{world} ranks sharing cuda:0" if shared
                                   else f"{world} ranks, 1 GPU each"), "busbw_factor": factor,
                   "algorithm": best_name, "algorithm_is_library_default": True,
                   "library_default_scheme": default_name, "autotune": autotune,
                   "bit_exact_dataset_E": default_exact,
                   "ipc_mode_legacy": comm.get_param("ipc_mode_legacy"),
                   "schemes": {}},
        # in the shared-GPU rehearsal no byte crosses xGMI (every "peer" is
        # this GPU's HBM): a fraction of R(N) would be meaningless, so none
        "roofline": {"bound": "xgmi", "achieved": red_gbs,
                     "peak": roof, "unit": "GB/s",
                     "frac": round(red_gbs / roof, 4) if red_gbs and not shared else None,
                     "traffic": traffic,
                     # why None: every MI355X pass so far shared one GPU
                     # between the ranks, where the device-wide TCC counters
                     # of a rank-0 dispatch also count the peers' concurrent
                     # kernels (they meet at device barriers), so no per-
                     # launch figure of one rank exists to commit
                     "traffic_source": ("profiles/pmc.json" if traffic is not None else
                                        "none: no dedicated-GPU PMC pass (shared-GPU counters "
                                        "mix the ranks' concurrent kernels)"),
                     "kernel": kernel,
                     "phase": dom, "kernel_ms": xg[dom]["kernel_ms"] if dom else None,
                     "phases": ph,
                     "busbw_frac_of_R": None if shared else round(busbw / roof, 4)},
        "rccl_comparator": ({"busbw": round(busbw_rccl, 2), "unit": "GB/s",
                             "ms_per_step": round(t_rccl * 1e3 / args.steps, 4)}
                            if t_rccl else None),
        "shared_gpu_rehearsal": shared,
        "device_error": err,
    }
    if not getattr(args, "no_cpu_baseline", False):
        # every rank waits while rank 0 runs the CPU ring on `world` cores
        dist.barrier()
        if rank == 0:
            _progress(rank, "cpu baseline (CPU ring restatement)")
            res["cpu_baseline"] = cpu_baseline_ring(world, S, factor)
        dist.barrier()
    if not args.no_extras:
        # the extras allocate buffers per size: the library default (staged)
        _PHASE["pending"] = res
        try:
            if os.environ.get("OMPI_AMD_BENCH_TEST_HANG"):  # the watchdog's own test
                _progress(rank, "extras: forced hang")
                time.sleep(1e9)
            if not os.environ.get("OMPI_AMD_BENCH_NO_SCHEMES"):
                res["config"]["schemes"] = _schemes(comm, dist, torch, mop, n, rank, shared,
                                                    tdev, ours, default)
            comm.set_param("user_ipc", 0)
            # the scheme sweep set explicit schemes (which turns autotune
            # off); the rows below measure what the library ships: autotune
            # on, each new size settled (_settle) before its timed region
            # (the headline bucket keeps its choice)
            comm.set_param("autotune", 0 if os.environ.get("OMPI_AMD_BENCH_NO_AUTOTUNE") else 1)
            _progress(rank, "extras: check")
            res["check"] = _check_exact(comm, dist, torch, mop, n, rank, shared)
            _progress(rank, "extras: sweep")
            res["sweep"] = _sweep(comm, dist, torch, mop, world, shared, tdev)
            _progress(rank, "extras: config5")
            res["config5"] = _config5(comm, dist, torch, mop, world, rank, tdev)
            _progress(rank, "extras: variants")
            res["variants"] = _variants(comm, dist, torch, mop, world, tdev)
            _progress(rank, "extras: copy_nt")
            res["copy_nt"] = _copy_nt(comm, dist, torch, mop, world, tdev, args.ar_bytes)
            _progress(rank, "extras: next_rows")
            res["next_rows"] = _next_rows(comm, dist, torch, mop, world, rank, tdev)
            _progress(rank, "extras: p2p_osc")
            res["p2p_osc"] = _p2p_osc_rows(comm, dist, torch, mop, world, rank, tdev)
        except Exception as e:  # extras never break the headline line
            res["extras_error"] = f"{type(e).__name__}: {e}"
        _PHASE["pending"] = None
    comm.free()
    dist.barrier()
    dist.destroy_process_group()
    return res if rank == 0 else None


def _phase_traffic(world: int, alg: int, user: bool, phase):
    """Bytes per launch of `phase`'s kernel under scheme `alg` at `world`
    ranks from profiles/pmc.json (FETCH_SIZE x 2 + WRITE_SIZE, separate
    rocprofv3 --pmc passes of tools/allreduce_pmc_probe.py: the ranks share
    one MI355X there, so peer accesses are counted as the same L2-to-fabric
    requests a dedicated GPU sends over xGMI), or None when no pass exists
    for this (N, scheme, phase)."""
    import json as _json

    if phase is None or user:
        return None
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    try:
        with open(os.path.join(root, "profiles", "pmc.json")) as f:
            entry = _json.load(f).get(f"allreduce_256MiB_n{world}_{dict(ALGORITHMS)[alg]}")
    except (OSError, ValueError):
        return None
    if not entry or phase not in entry.get("phases", {}):
        return None
    return entry["phases"][phase]["traffic"]


def _schemes(comm, dist, torch, mop, n, rank, shared, tdev, ours, default):
    """Every data-movement scheme x transfer grid, measured after the
    headline (config.schemes only; the headline is the library default).
    ipc "staged": peers read library-owned memory (shadow arena / landing
    buffers; the default, user_ipc = 0); "user": peers map the caller's
    x / y directly (user_ipc = 1; these buffers live for the whole run, so
    no mapping goes stale).  Each scheme is first checked bit-exact on
    dataset E at this size."""
    S = n * 4
    world = dist.get_world_size()
    factor = 2.0 * (world - 1) / world
    schemes = {}
    for ipc in ("staged", "user"):
        comm.set_param("user_ipc", 1 if ipc == "user" else 0)
        for a, name in ALGORITHMS:
            if ipc == "user" and a in PIPE_ALGS:
                continue  # with user_ipc they run the phased push / pull
            comm.set_param("algorithm", a)
            comm.set_param("blocks", default["blocks"])
            _progress(rank, f"extras: scheme {name}/{ipc}: exactness check")
            exact = _exact_ok(comm, dist, torch, mop, n, rank, shared)
            _progress(rank, f"extras: scheme {name}/{ipc}: bit_exact={exact}, "
                            f"timing {len(BLOCKS)} grids")
            for blocks in BLOCKS:
                comm.set_param("blocks", blocks)
                ta = _timed(ours, 5, 2, dist, torch, tdev) / 5
                schemes[f"{name}/{ipc}/{blocks}"] = {
                    "algorithm": a, "ipc": ipc, "blocks": blocks, "bit_exact": exact,
                    "us": round(ta * 1e6, 2), "busbw": round(S / ta * factor / 1e9, 2)}
    comm.set_param("user_ipc", default["user_ipc"])
    comm.set_param("algorithm", default["algorithm"])
    comm.set_param("blocks", default["blocks"])
    return schemes


def cpu_baseline_ring(world: int, nbytes: int, factor: float, seconds: float = 10.0,
                      warmup: int = 2, iters: int | None = None) -> dict:
    """The reference's CPU path for this metric, restated: coll/tuned's
    ring_segmented allreduce (coll_base_allreduce.c:618-856) with op/base's
    loop as the reduction, `world` host processes over POSIX shared memory
    (tools/cpu_ring_baseline.c, linked against the oracle; bit-exact with the
    oracle's ring_segmented on dataset R, tests/test_coll_cpu.py), on the
    same message size.  A bounded sample of about `seconds` of ring time,
    or exactly `iters` timed iterations after `warmup`."""
    import json as _json
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "tools", "cpu_ring_baseline")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.join(root, "tools"), "cpu_ring_baseline"],
                       check=True, capture_output=True)
    if iters is None:
        est = nbytes / 1.5e9  # seconds per iteration at the ~1.7 GB/s algbw seen in round 1
        iters = max(5, min(200, int(seconds / max(est, 1e-6))))
    out = subprocess.run([exe, str(world), str(nbytes), str(warmup), str(iters)], check=True,
                         capture_output=True, text=True, timeout=600)
    line = _json.loads(out.stdout.strip().splitlines()[-1])
    import bench as _bench  # host_cpu(): nproc and CPU model beside the cores used
    return {"value": line["busbw_GBps"], "unit": "GB/s", "cores": world, "kind": "port",
            **_bench.host_cpu(),
            "sample": f"ring_segmented restatement (tools/cpu_ring_baseline.c, oracle op/base "
                      f"loop), {world} processes x 1 core over POSIX shm, {nbytes} B per rank, "
                      f"{iters} timed iterations after {warmup} warm-ups (median "
                      f"{line['median_s']:.4f} s, algbw {line['algbw_GBps']} GB/s); value is "
                      f"busBW = S/t x {factor:.3f}"}


ALGORITHMS = ((0, "pull"), (1, "pull_push"), (2, "push"), (3, "push_land"), (4, "push_pipe"),
              (5, "land_pipe"), (6, "pull_pipe"))
PIPE_ALGS = (4, 5, 6)  # one pipelined launch per call (staged only; user_ipc runs them phased)
BLOCKS = (256, 512, 1024, 2048)  # grid cap of the transfer kernels


def _exact_ok(comm, dist, torch, mop, n, rank, shared):
    """Dataset E bit-exactness of the current scheme on all ranks (None in
    the shared-GPU rehearsal, where RCCL is unavailable: tests cover it)."""
    if shared:
        return None
    res = _check_exact(comm, dist, torch, mop, n, rank, shared)
    return bool(res["bit_exact_all_ranks"])


def _check_exact(comm, dist, torch, mop, n, rank, shared):
    """Dataset E (k * 2^-8, |k| <= 1024): every summation order is exact,
    so our result must equal RCCL's (and the integer sum) bit for bit."""
    g = torch.Generator(device="cuda").manual_seed(777 + rank)
    k = torch.randint(-1024, 1025, (n,), device="cuda", generator=g, dtype=torch.int32)
    x = k.to(torch.float32) * (2.0 ** -8)
    y = torch.empty_like(x)
    comm.allreduce(x, y, n, mop.MPI_FLOAT, mop.MPI_SUM, blocking=True)
    if shared:
        return {"dataset": "E", "note": "shared-GPU rehearsal: exactness checked by tests"}
    ksum = k.clone()
    dist.all_reduce(ksum)
    exact = ksum.to(torch.float32) * (2.0 ** -8)
    ok = bool(torch.equal(y, exact))
    flag = torch.tensor([1 if ok else 0], device="cuda")
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return {"dataset": "E", "bytes": n * 4, "bit_exact_all_ranks": bool(flag.item())}


def _sweep(comm, dist, torch, mop, world, shared, tdev):
    """BASELINE configs[3]: fp32 SUM allreduce busBW, 8 B .. 1 GiB, ours
    and RCCL side by side."""
    out = []
    factor = 2.0 * (world - 1) / world
    sizes = (8, 1024, 65536, 1 << 20, 16 << 20, 64 << 20, 256 << 20, 1 << 30)
    if os.environ.get("OMPI_AMD_BENCH_SWEEP"):  # e.g. "1073741824": a subset (rehearsals)
        sizes = tuple(int(v) for v in os.environ["OMPI_AMD_BENCH_SWEEP"].split(","))
    for nbytes in sizes:
        _progress(dist.get_rank(), f"sweep {nbytes} B")
        n = max(1, nbytes // 4)
        x = torch.ones(n, device="cuda")
        y = torch.empty_like(x)
        steps = 20 if nbytes <= (64 << 20) else 5
        _settle(comm, lambda: comm.allreduce(x, y, n, mop.MPI_FLOAT, mop.MPI_SUM), torch)
        t = _timed(lambda: comm.allreduce(x, y, n, mop.MPI_FLOAT, mop.MPI_SUM), steps, 3,
                   dist, torch, tdev) / steps
        row = {"bytes": n * 4, "us": round(t * 1e6, 2),
               "busbw": round(n * 4 / t * factor / 1e9, 3)}
        if not shared:
            tr = _timed(lambda: dist.all_reduce(x), steps, 3, dist, torch) / steps
            row["rccl_us"] = round(tr * 1e6, 2)
            row["rccl_busbw"] = round(n * 4 / tr * factor / 1e9, 3)
        out.append(row)
        del x, y
    return out


def _config5(comm, dist, torch, mop, world, rank, tdev):
    """BASELINE configs[4]: reduce_scatter_block (MPI_DOUBLE_INT MAXLOC),
    allgather and bcast, 64 MiB per rank; busBW per nccl-tests convention."""
    res = {}
    rcount = (64 << 20) // 16 // world
    buf = torch.zeros(rcount * world * 16, dtype=torch.uint8, device="cuda")
    out = torch.zeros(rcount * 16, dtype=torch.uint8, device="cuda")
    S = rcount * world * 16
    t = _timed(lambda: comm.reduce_scatter_block(buf, out, rcount, mop.MPI_DOUBLE_INT,
                                                 mop.MPI_MAXLOC), 10, 3, dist, torch, tdev) / 10
    res["reduce_scatter_block_maxloc_double_int"] = {
        "bytes_total": S, "us": round(t * 1e6, 2),
        "busbw": round(S / t * (world - 1) / world / 1e9, 3)}
    per = (64 << 20) // world
    src = torch.zeros(per, dtype=torch.uint8, device="cuda")
    dst = torch.zeros(per * world, dtype=torch.uint8, device="cuda")
    t = _timed(lambda: comm.allgather(src, dst, per), 10, 3, dist, torch, tdev) / 10
    res["allgather"] = {"bytes_total": per * world, "us": round(t * 1e6, 2),
                        "busbw": round(per * world / t * (world - 1) / world / 1e9, 3)}
    b = torch.zeros(64 << 20, dtype=torch.uint8, device="cuda")
    t = _timed(lambda: comm.bcast(b, b.numel(), 0), 10, 3, dist, torch, tdev) / 10
    res["bcast"] = {"bytes": b.numel(), "us": round(t * 1e6, 2),
                    "busbw": round(b.numel() / t / 1e9, 3)}
    # A/B: the same two calls through the landing
    # buffers (stores, no per-call descriptor swap, one more local copy) —
    # what the nonblocking / persistent forms always take
    comm.set_param("land_blocking", 1)
    try:
        t = _timed(lambda: comm.allgather(src, dst, per), 10, 3, dist, torch, tdev) / 10
        res["allgather_landing"] = {"bytes_total": per * world, "us": round(t * 1e6, 2),
                                    "busbw": round(per * world / t * (world - 1) / world / 1e9, 3)}
        t = _timed(lambda: comm.bcast(b, b.numel(), 0), 10, 3, dist, torch, tdev) / 10
        res["bcast_landing"] = {"bytes": b.numel(), "us": round(t * 1e6, 2),
                                "busbw": round(b.numel() / t / 1e9, 3)}
    finally:
        comm.set_param("land_blocking", 0)
    # MPI_Reduce fp32 SUM 64 MiB to root 0 (tuned pipeline order); every
    # rank reduces 1/N of the vector and stores it into the root's rbuf
    nf = (64 << 20) // 4
    xr = torch.ones(nf, device="cuda")
    yr = torch.zeros(nf, device="cuda") if rank == 0 else None
    t = _timed(lambda: comm.reduce(xr, yr, nf, mop.MPI_FLOAT, mop.MPI_SUM, 0), 10, 3,
               dist, torch, tdev) / 10
    res["reduce_sum_f32_root0"] = {"bytes": nf * 4, "us": round(t * 1e6, 2),
                                   "algbw": round(nf * 4 / t / 1e9, 3)}
    return res


def _variants(comm, dist, torch, mop, world, tdev):
    """Design A/B points measured in the same run (the multi-GPU node is only
    reachable through this bench): the small/medium-message paths around
    the fused_bytes / small_bytes switches — one fused launch (every rank
    folds all blocks), staged two-shot (scratch, no host rendezvous) and
    zero-copy (per-call IPC handle swap) — at the headline's scheme."""
    out = {"small_path": []}
    paths = (("fused", 4 << 20, 4 << 20), ("staged_two_shot", 0, 4 << 20), ("zero_copy", 0, 0))
    for nbytes in (16 << 10, 64 << 10, 256 << 10, 1 << 20, 2 << 20):
        n = nbytes // 4
        x = torch.ones(n, device="cuda")
        y = torch.empty_like(x)
        row = {"bytes": nbytes}
        for name, fused, small in paths:
            comm.set_param("fused_bytes", fused)
            comm.set_param("small_bytes", small)
            _settle(comm, lambda: comm.allreduce(x, y, n, mop.MPI_FLOAT, mop.MPI_SUM), torch)
            t = _timed(lambda: comm.allreduce(x, y, n, mop.MPI_FLOAT, mop.MPI_SUM), 20, 3,
                       dist, torch, tdev) / 20
            row[name + "_us"] = round(t * 1e6, 2)
        out["small_path"].append(row)
        del x, y
    comm.set_param("fused_bytes", 64 << 10)
    comm.set_param("small_bytes", 1 << 20)
    return out


def _copy_nt(comm, dist, torch, mop, world, tdev, nbytes):
    """A/B of the copy kernels' stores (param copy_nt: plain vs
    non-temporal) on the headline allreduce as the library runs it
    (autotuned scheme), with the per-phase kernel time of each."""
    n = nbytes // 4
    x = torch.ones(n, device="cuda")
    y = torch.empty_like(x)
    res = {}
    saved = comm.get_param("copy_nt") if comm.get_param("copy_nt_fixed") else -1
    try:
        for nt in (0, 1):
            comm.set_param("copy_nt", nt)
            fn = lambda: comm.allreduce(x, y, n, mop.MPI_FLOAT, mop.MPI_SUM)  # noqa: E731
            _settle(comm, fn, torch)
            t = _timed(fn, 10, 3, dist, torch, tdev) / 10
            comm.set_param("profile", 1)
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            comm.set_param("profile", 0)
            ph = {}
            for k, name in enumerate(("fold", "gather", "scatter")):
                tot, calls = comm.phase_ms(k)  # read once: it resets the phase's record
                if calls:
                    ph[name] = round(tot / calls, 4)
            res["nt" if nt else "plain"] = {"us": round(t * 1e6, 2),
                                           "busbw": round(nbytes / t * 2 * (world - 1) / world / 1e9, 3),
                                           "phase_kernel_ms": ph}
    finally:
        comm.set_param("copy_nt", saved)
    return res


def _next_rows(comm, dist, torch, mop, world, rank, tdev):
    """SURVEY §8f rows 2-3 measured beside the headline: reduce_scatter
    (uneven counts), scan / exscan, and allreduce as a plain call, a
    persistent plan start (MPI_Allreduce_init: no handle swap per start)
    and a nonblocking post + wait (MPI_Iallreduce), per size."""
    F, SUM = mop.MPI_FLOAT, mop.MPI_SUM
    res = {}
    # reduce_scatter, 64 MiB total, rank r gets (1 + r/N) shares
    weights = [world + r for r in range(world)]
    total = (64 << 20) // 4
    rcounts = [total * w // sum(weights) for w in weights]
    x = torch.ones(sum(rcounts), device="cuda")
    y = torch.empty(max(rcounts), device="cuda")
    t = _timed(lambda: comm.reduce_scatter(x, y, rcounts, F, SUM), 10, 3, dist, torch, tdev) / 10
    S = sum(rcounts) * 4
    res["reduce_scatter_f32_uneven"] = {"bytes_total": S, "us": round(t * 1e6, 2),
                                        "busbw": round(S / t * (world - 1) / world / 1e9, 3)}
    del x, y
    for name, fn in (("scan", comm.scan), ("exscan", comm.exscan)):
        n = (16 << 20) // 4
        x = torch.ones(n, device="cuda")
        y = torch.empty_like(x)
        t = _timed(lambda: fn(x, y, n, F, SUM), 10, 3, dist, torch, tdev) / 10
        res[f"{name}_f32_16MiB"] = {"bytes": n * 4, "us": round(t * 1e6, 2),
                                    "algbw": round(n * 4 / t / 1e9, 3)}
        del x, y
    rows = []
    for nbytes in (64 << 10, 1 << 20, 16 << 20, 256 << 20):
        n = nbytes // 4
        x = torch.ones(n, device="cuda")
        y = torch.empty_like(x)
        steps = 20 if nbytes <= (16 << 20) else 5
        row = {"bytes": nbytes}
        _settle(comm, lambda: comm.allreduce(x, y, n, F, SUM), torch)
        t = _timed(lambda: comm.allreduce(x, y, n, F, SUM), steps, 3, dist, torch, tdev) / steps
        row["allreduce_us"] = round(t * 1e6, 2)
        plan = comm.allreduce_init(x, y, n, F, SUM)
        t = _timed(lambda: plan.start(), steps, 3, dist, torch, tdev) / steps
        plan.free()
        row["persistent_start_us"] = round(t * 1e6, 2)

        def post_wait():
            r = comm.iallreduce(x, y, n, F, SUM)
            r.wait()
            r.free()
        t = _timed(post_wait, steps, 3, dist, torch, tdev) / steps
        row["iallreduce_post_wait_us"] = round(t * 1e6, 2)
        rows.append(row)
        del x, y
    res["allreduce_call_kinds"] = rows
    return res


def _p2p_osc_rows(comm, dist, torch, mop, world, rank, tdev):
    """SURVEY §8f rows 1 and 4 beside the headline: device-buffer
    MPI_Sendrecv around the ring (receiver pulls the sender's buffer over
    xGMI), and one-sided MPI_Put / MPI_Accumulate(SUM fp32) into the next
    rank's window per fence epoch, MPI_Fetch_and_op on one shared counter.
    Rates are bytes per rank over the max-over-ranks time; an accumulate
    moves 2 bytes over xGMI per window byte (target read + write)."""
    from ompi_amd import osc, pml
    res = {}
    nxt, prv = (rank + 1) % world, (rank - 1) % world
    # a peer lock that never comes must not stall the bench: short bound,
    # and the rows stop at the first device error
    comm.set_param("timeout_ms", 5000)

    def check(what):  # collective: every rank stops together
        e = torch.tensor([abs(comm.error())], dtype=torch.int64, device=tdev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        if int(e.item()):
            raise RuntimeError(f"device error on some rank after {what}")
    rows = []
    for nbytes in (8, 64 << 10, 16 << 20, 256 << 20):
        s = torch.ones(max(nbytes, 16), dtype=torch.uint8, device="cuda")
        r = torch.empty_like(s)
        steps = 20 if nbytes <= (16 << 20) else 5
        t = _timed(lambda: pml.sendrecv(comm, s, nxt, 1, r, prv, 1, sbytes=nbytes,
                                        rbytes=nbytes), steps, 3, dist, torch, tdev) / steps
        rows.append({"bytes": nbytes, "us": round(t * 1e6, 2),
                     "gbs_per_rank": round(nbytes / t / 1e9, 3)})
        del s, r
    res["sendrecv_ring"] = rows
    check("sendrecv")
    S = 64 << 20
    win = osc.Window.allocate(comm, S, disp_unit=4)
    try:
        x = torch.ones(S // 4, device="cuda")
        steps = 10

        def put_epoch():
            win.put(x, nxt, 0, S)
            win.fence()
        t = _timed(put_epoch, steps, 2, dist, torch, tdev) / steps
        check("put")
        res["put_64MiB_fence"] = {"bytes": S, "us": round(t * 1e6, 2),
                                  "gbs_per_rank": round(S / t / 1e9, 3)}

        def acc_epoch():
            win.accumulate(x, S // 4, mop.MPI_FLOAT, nxt, 0, mop.MPI_SUM)
            win.fence()
        t = _timed(acc_epoch, steps, 2, dist, torch, tdev) / steps
        check("accumulate")
        res["accumulate_sum_f32_64MiB_fence"] = {
            "bytes": S, "us": round(t * 1e6, 2), "gbs_per_rank": round(S / t / 1e9, 3),
            "xgmi_gbs_per_rank": round(2 * S / t / 1e9, 3)}
        one = torch.ones(1, dtype=torch.int64, device="cuda")
        out = torch.empty(1, dtype=torch.int64, device="cuda")
        k = 50

        def fops():
            for _ in range(k):
                win.fetch_and_op(one, out, mop.MPI_INT64_T, 0, 0, mop.MPI_SUM)
            win.fence()
        t = _timed(fops, 3, 1, dist, torch, tdev) / 3
        check("fetch_and_op")
        res["fetch_and_op_shared_counter"] = {"ops_per_rank": k, "us_per_op": round(t * 1e6 / k, 2),
                                              "contenders": world}
    finally:
        win.free()
    return res


def single_gpu_rows(mib: int = 256):
    """N=1 leg of SURVEY §8f rows 1 and 4 (bench.py, beside the headline): a
    communicator of size 1, so the target window and the p2p peer are this
    GPU and every kernel is HBM-bound exactly like the op kernel.  Event-
    timed on a dedicated stream; algorithmic HBM bytes per call: accumulate
    3 x S (read target, read origin, write target), get_accumulate 5 x S
    (+ fetch copy), put and the p2p receive copy 2 x S, the derived-target
    accumulate 1.5 x S (S/2 packed origin bytes into every other double:
    origin read, target slots read and written).  Plus two latency rows in
    microseconds (host clock): fetch_and_op and an 8-byte accumulate, each
    followed by MPI_Win_flush, under lock_all."""
    import torch

    from . import coll, osc, pml
    from . import op as mop

    S = mib << 20
    s = torch.cuda.Stream()
    comm = coll.Communicator(f"n1rows_{os.getpid()}", 0, 1, torch.cuda.current_device())
    win = osc.Window.allocate(comm, S, disp_unit=4)
    x = torch.ones(S // 4, device="cuda")
    r = torch.empty_like(x)
    torch.cuda.synchronize()

    def timed(fn, iters=10):
        for _ in range(2):
            fn()
        s.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(iters):
            fn()
        b.record(s)
        b.synchronize()
        return a.elapsed_time(b) / iters / 1e3

    from . import datatype as ddt
    tvec = ddt.type_vector(S // 16, 1, 2, ddt.predefined("MPI_DOUBLE")).commit()
    rows = {}
    try:
        for name, fn, factor in (
            ("accumulate_sum_f32", lambda: win.accumulate(x, S // 4, mop.MPI_FLOAT, 0, 0,
                                                          mop.MPI_SUM, stream=s), 3),
            ("get_accumulate_sum_f32", lambda: win.get_accumulate(x, r, S // 4, mop.MPI_FLOAT, 0,
                                                                  0, mop.MPI_SUM, stream=s), 5),
            ("put", lambda: win.put(x, 0, 0, S, stream=s), 2),
            # derived target (MPI_Type_vector of single doubles at stride 2,
            # spanning the window): the origin's S/2 packed bytes folded into
            # every other double — read origin, read + write target slots
            ("accumulate_ddt_vector_bl1_f64", lambda: win.accumulate_ddt(
                x, S // 16, None, 0, 0, 1, tvec, mop.MPI_DOUBLE, mop.MPI_SUM, stream=s), 1.5),
            ("sendrecv_self", lambda: pml.sendrecv(comm, x, 0, 1, r, 0, 1, stream=s), 2),
        ):
            t = timed(fn)
            gbs = factor * S / t / 1e9
            rows[name] = {"bytes": S, "ms": round(t * 1e3, 4), "hbm_gbs": round(gbs, 1),
                          "frac_of_8TBs": round(gbs / 8000.0, 4)}
        # small one-sided latency under lock_all (host clock, each call
        # completed by MPI_Win_flush): the single-launch accumulate-lock path
        import time as _time
        one = torch.ones(1, dtype=torch.int64, device="cuda")
        res1 = torch.empty(1, dtype=torch.int64, device="cuda")
        win.lock_all(stream=s)
        try:
            for name, fn in (
                ("fetch_and_op_i64_flush_us",
                 lambda: win.fetch_and_op(one, res1, mop.MPI_INT64_T, 0, 0, mop.MPI_SUM, stream=s)),
                ("accumulate_8B_f32_flush_us",
                 lambda: win.accumulate(x, 2, mop.MPI_FLOAT, 0, 64, mop.MPI_SUM, stream=s)),
            ):
                for _ in range(5):
                    fn()
                    win.flush(0, stream=s)
                t0 = _time.perf_counter()
                for _ in range(50):
                    fn()
                    win.flush(0, stream=s)
                rows[name] = round((_time.perf_counter() - t0) / 50 * 1e6, 2)
        finally:
            win.unlock_all(stream=s)
    finally:
        win.free()
        comm.free()
    return rows


def config_rows():
    """BASELINE configs[1] and configs[2] beside the N = 1 headline (bench.py
    extras; the full sweeps are tools/op_sweep.py and tools/ddt_sweep.py).
    Op: 3-buffer SUM / MAX / BAND over int32 / fp32 / fp64 at 64 MiB and
    1 GiB per buffer, MAXLOC DOUBLE_INT at 1 GiB; algorithmic bytes 3 x n x
    extent.  Convertor: one pack and one unpack call over 256 MiB packed for
    vector bl 1 / 2 / 8 / 64 doubles (stride 2 x bl), blacs-style indexed
    and struct {int, double}; algorithmic bytes 2 x packed.  Event-timed on
    a dedicated stream, median of three batches."""
    import statistics

    import torch

    from . import datatype as dd
    from . import op as mop

    s = torch.cuda.Stream()

    def timed(fn, iters):
        for _ in range(2):
            fn()
        s.synchronize()
        vals = []
        for _ in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for _ in range(iters):
                fn()
            b.record(s)
            b.synchronize()
            vals.append(a.elapsed_time(b) / iters)
        return statistics.median(vals)

    top = 1 << 30
    a = torch.empty(top, dtype=torch.uint8, device="cuda").random_()
    bb = torch.empty(top, dtype=torch.uint8, device="cuda").random_()
    o = torch.empty(top, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    op_rows = []
    cases = [(mop.MPI_SUM, mop.MPI_INT32_T), (mop.MPI_SUM, mop.MPI_FLOAT), (mop.MPI_SUM, mop.MPI_DOUBLE),
             (mop.MPI_MAX, mop.MPI_INT32_T), (mop.MPI_MAX, mop.MPI_FLOAT), (mop.MPI_MAX, mop.MPI_DOUBLE),
             (mop.MPI_BAND, mop.MPI_INT32_T), (mop.MPI_MAXLOC, mop.MPI_DOUBLE_INT)]
    for op, dt in cases:
        for nbytes in ((top,) if op is mop.MPI_MAXLOC else (64 << 20, top)):
            n = nbytes // dt.extent
            ms = timed(lambda: mop.reduce_local_3buff_async(a, bb, o, n, dt, op, stream=s),
                       10 if nbytes == top else 40)
            gbs = 3 * n * dt.extent / (ms * 1e-3) / 1e9
            op_rows.append({"op": op.name, "type": dt.name, "bytes": nbytes, "ms": round(ms, 4),
                            "hbm_gbs": round(gbs, 1), "frac_of_8TBs": round(gbs / 8000.0, 4)})
    del a, bb, o
    torch.cuda.empty_cache()

    S = 256 << 20
    d = dd.predefined("MPI_DOUBLE")
    i32 = dd.predefined("MPI_INT")
    lens = [13, 13, 13, 13, 13, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1]
    disps = [286, 308, 330, 352, 374, 396, 419, 442, 465, 488, 511, 534, 557, 580, 603, 626, 649, 672]
    types = [(f"vector_bl{bl}", dd.type_vector(S // (8 * bl), bl, 2 * bl, d), 1) for bl in (1, 2, 8, 64)]
    blacs = dd.type_indexed(lens, disps, i32)
    types.append(("blacs_indexed", blacs, S // blacs.size))
    st = dd.type_struct([1, 1], [0, 8], [i32, d])
    types.append(("struct_int_double", st, S // st.size))
    ddt_rows = []
    packed = torch.empty(S, dtype=torch.uint8, device="cuda")
    for name, dt, count in types:
        total = dt.size * count
        typed = torch.empty((count - 1) * dt.extent + dt.true_span, dtype=torch.uint8,
                            device="cuda").random_()
        torch.cuda.synchronize()
        for kind in ("pack", "unpack"):
            def one():
                cv = dd.Convertor()
                if kind == "pack":
                    cv.prepare_for_send(dt, count, typed, stream=s)
                    cv.pack(packed.data_ptr(), total)
                else:
                    cv.prepare_for_recv(dt, count, typed, stream=s)
                    cv.unpack(packed.data_ptr(), total)
            # 20 calls a batch: the first call's host work (convertor set-up,
            # ~50 us, while the stream idles) sits inside the event pair
            ms = timed(one, 20)
            gbs = 2 * total / (ms * 1e-3) / 1e9
            ddt_rows.append({"type": name, "kind": kind, "packed_bytes": total, "ms": round(ms, 4),
                             "hbm_gbs": round(gbs, 1), "frac_of_8TBs": round(gbs / 8000.0, 4)})
        del typed
        dt.free()
    return {"configs1_op_3buff": op_rows, "configs2_convertor_256MiB": ddt_rows}
