#!/usr/bin/env python3
"""IPC open storm probe (one GPU box, N processes sharing cuda:0).

The library's intermittent failure: hipIpcOpenMemHandle refuses a live peer
allocation with "invalid device pointer" (DESIGN.md §4.6), at collective
setup points where every rank opens every peer's fresh allocation at once
(window creation, landing growth).  This probe reproduces that pattern
without the library and varies one thing at a time:

  order  "same":    every rank opens peers 0, 1, ..., N-1 (each exporter
                    answers N-1 importers at once)
         "stagger": rank r opens peers r+1, r+2, ... (one importer per
                    exporter at a time)
         "busy_sync": half the ranks keep the GPU busy (large device copies
                    + hipDeviceSynchronize, ~tens of ms) while the other half
                    open their handles — an exporter blocked in the runtime
         "busy_sleep": the same with the busy half asleep on the host (no
                    HIP call) — the control for busy_sync
         "churn":   every exporter frees its previous round's buffer BEFORE
                    the importers close their mappings of it (the registry's
                    retire order), and the importers open the new handles
                    while still holding the old mappings
  and records, per round: every open's result, the exporter-side fd and
  thread counts (does exporting start a server thread / open sockets?).

Rounds allocate fresh buffers of varying size, export them, exchange the
64-byte handles through shared memory, open all peers, close, free.
Output: one JSON line per (order) with failure counts, plus one line of
process resources after the first export.  ctypes on libamdhip64 only.
"""
import ctypes
import json
import multiprocessing as mp
import os
import sys
import time

HIP = "/opt/rocm/lib/libamdhip64.so"
BIG = 1 << 30


class Handle(ctypes.Structure):  # hipIpcMemHandle_t: passed BY VALUE to the open
    _fields_ = [("reserved", ctypes.c_char * 64)]


def fd_summary():
    kinds = {}
    for fd in os.listdir("/proc/self/fd"):
        try:
            t = os.readlink(f"/proc/self/fd/{fd}")
        except OSError:
            continue
        k = t.split(":")[0] if ":" in t else ("dmabuf" if "dmabuf" in t else
                                              ("kfd" if "kfd" in t else ("dri" if "dri" in t else "file")))
        kinds[k] = kinds.get(k, 0) + 1
    return kinds


def worker(rank, n, rounds, handles, results, barrier, order):
    hip = ctypes.CDLL(HIP)
    hip.hipSetDevice(0)
    hip.hipGetErrorString.restype = ctypes.c_char_p
    before = (fd_summary(), len(os.listdir("/proc/self/task")))
    big_a, big_b = ctypes.c_void_p(), ctypes.c_void_p()
    if order.startswith("busy"):
        assert hip.hipMalloc(ctypes.byref(big_a), ctypes.c_size_t(BIG)) == 0
        assert hip.hipMalloc(ctypes.byref(big_b), ctypes.c_size_t(BIG)) == 0
    fails, opens, first_err = 0, 0, None
    prev, held = None, []
    for r in range(rounds):
        size = (1 + (r * 7 + rank * 3) % 40) * (1 << 20) + (r % 5) * 4096 + 64
        p = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(size)) == 0
        h = Handle()
        assert hip.hipIpcGetMemHandle(ctypes.byref(h), p) == 0
        handles[rank * 64:(rank + 1) * 64] = bytes(h)
        if r == 0 and rank == 0:
            results.put(("res", {"fds_before": before[0], "threads_before": before[1],
                                 "fds_after_export": fd_summary(),
                                 "threads_after_export": len(os.listdir("/proc/self/task"))}))
        barrier.wait()
        peers = [(rank + k) % n for k in range(1, n)] if order == "stagger" else \
            [q for q in range(n) if q != rank]
        busy = order.startswith("busy") and (rank + r) % 2 == 1
        if order.startswith("busy"):
            # the busy half exports and stays busy; the other half opens them
            peers = [] if busy else [q for q in peers if (q + r) % 2 == 1]
        if busy:
            if order == "busy_sync":
                t_end = time.time() + 0.05
                while time.time() < t_end:
                    hip.hipMemcpy(big_b, big_a, ctypes.c_size_t(BIG), 3)  # device to device
                    hip.hipDeviceSynchronize()
            else:
                time.sleep(0.05)
        if order == "churn" and prev is not None:
            hip.hipFree(prev)  # freed while the peers still map it
            prev = None
        mapped = []
        for q in peers:
            hq = Handle.from_buffer_copy(bytes(handles[q * 64:(q + 1) * 64]))
            m = ctypes.c_void_p()
            e = hip.hipIpcOpenMemHandle(ctypes.byref(m), hq, ctypes.c_uint(1))
            opens += 1
            if e != 0:
                fails += 1
                if first_err is None:
                    first_err = f"round {r} peer {q}: {hip.hipGetErrorString(e).decode()}"
                hip.hipGetLastError()
            else:
                mapped.append(m)
        barrier.wait()
        if order == "churn":
            for m in held:  # last round's mappings, after their exporters freed them
                hip.hipIpcCloseMemHandle(m)
            held = mapped
            prev = p
            barrier.wait()
            continue
        for m in mapped:
            hip.hipIpcCloseMemHandle(m)
        barrier.wait()
        hip.hipFree(p)
        barrier.wait()
    results.put(("rank", {"rank": rank, "opens": opens, "fails": fails, "first_err": first_err,
                          "fds_end": fd_summary(), "threads_end": len(os.listdir("/proc/self/task"))}))


def run(n, rounds, order):
    ctx = mp.get_context("spawn")
    handles = ctx.Array(ctypes.c_char, 64 * n, lock=False)
    results = ctx.Queue()
    barrier = ctx.Barrier(n)
    procs = [ctx.Process(target=worker, args=(r, n, rounds, handles, results, barrier, order))
             for r in range(n)]
    t0 = time.time()
    for p in procs:
        p.start()
    out = {"res": None, "ranks": []}
    for _ in range(n + 1):
        kind, v = results.get(timeout=300)
        if kind == "res":
            out["res"] = v
        else:
            out["ranks"].append(v)
    for p in procs:
        p.join(timeout=60)
    fails = sum(v["fails"] for v in out["ranks"])
    opens = sum(v["opens"] for v in out["ranks"])
    errs = [v["first_err"] for v in out["ranks"] if v["first_err"]]
    print(json.dumps({"n": n, "order": order, "rounds": rounds, "opens": opens, "fails": fails,
                      "seconds": round(time.time() - t0, 1), "first_errors": errs[:4],
                      "resources_rank0": out["res"],
                      "end_rank0": next(v for v in out["ranks"] if v["rank"] == 0)}), flush=True)


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    for order in sys.argv[3].split(",") if len(sys.argv) > 3 else ("same", "stagger"):
        run(n, rounds, order)
