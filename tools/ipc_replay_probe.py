#!/usr/bin/env python3
"""Replay of the library's refused-open sequence.

Both refusals recorded in round 3 opened a peer buffer
that its exporter had just allocated in place of one it freed while the
importers still mapped it: the importer's registry retired (closed) the
stale mapping and opened the new handle right after.  The round-3 storm
probe (tools/ipc_storm_probe.py) never reused a freed exported address
while an importer still held it, so it did not replay that sequence.  This
probe does, with hipMalloc/hipFree directly (no library), N processes on
one GPU, one exporter per round (the others import):

  recycle_close_open   exporter frees X (importers still map it), allocates
                       X' of the same size (same address when the runtime
                       reuses it) and exports it; each importer closes its
                       mapping of X and opens X' at once — the registry's
                       order (ipc_registry.cpp: retire, then open)
  recycle_gap          the same with 20 ms between the close and the open
  closed_first         importers close X before the exporter frees it,
                       then X' is allocated, exported and opened
  fresh_address        X' is allocated while X is alive (a different
                       address) and exported, then X is freed; importers
                       close X and open X'
  fresh_free_after     the same, but X is freed only after every importer
                       opened X' (and closed X)
  fresh_keep           X' allocated, exported and opened while X stays
                       allocated until the end of the run (never freed
                       between exports)

Output: one JSON line per order: opens, refusals, how many rounds reused
the freed address, the first errors.  ctypes on libamdhip64 only.
"""
import ctypes
import json
import multiprocessing as mp
import sys
import time

HIP = "/opt/rocm/lib/libamdhip64.so"


class Handle(ctypes.Structure):  # hipIpcMemHandle_t: passed BY VALUE to the open
    _fields_ = [("reserved", ctypes.c_char * 64)]


def worker(rank, n, rounds, size, handles, addr, results, barrier, order):
    hip = ctypes.CDLL(HIP)
    hip.hipSetDevice(0)
    hip.hipGetErrorString.restype = ctypes.c_char_p
    opens = fails = reused = 0
    errs = []
    held = {}  # exporter -> this rank's mapping of its current buffer
    mine = None
    kept = []  # fresh_keep / fresh_free_after: earlier buffers still allocated

    def export(p):
        h = Handle()
        assert hip.hipIpcGetMemHandle(ctypes.byref(h), p) == 0
        handles[rank * 64:(rank + 1) * 64] = bytes(h)
        addr[rank] = p.value

    def open_peer(q, r):
        nonlocal opens, fails
        h = Handle.from_buffer_copy(bytes(handles[q * 64:(q + 1) * 64]))
        m = ctypes.c_void_p()
        e = hip.hipIpcOpenMemHandle(ctypes.byref(m), h, ctypes.c_uint(1))
        opens += 1
        if e != 0:
            fails += 1
            if len(errs) < 3:
                errs.append(f"round {r} exporter {q}: {hip.hipGetErrorString(e).decode()}")
            hip.hipGetLastError()
            return None
        return m

    # round 0: every rank exports a buffer, every rank maps every peer's
    mine = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(mine), ctypes.c_size_t(size)) == 0
    export(mine)
    barrier.wait()
    for q in range(n):
        if q != rank:
            held[q] = open_peer(q, 0)
    barrier.wait()
    for r in range(1, rounds):
        ex = r % n  # this round's exporter
        if order == "closed_first" and rank != ex:
            if held.get(ex):
                hip.hipIpcCloseMemHandle(held[ex])
            held[ex] = None
        barrier.wait()
        if rank == ex:
            old = mine.value
            nxt = ctypes.c_void_p()
            if order.startswith("fresh"):
                assert hip.hipMalloc(ctypes.byref(nxt), ctypes.c_size_t(size)) == 0
                export(nxt)
                if order == "fresh_address":
                    hip.hipFree(mine)
                else:
                    kept.append(mine)
            else:
                hip.hipFree(mine)  # the importers may still map it
                assert hip.hipMalloc(ctypes.byref(nxt), ctypes.c_size_t(size)) == 0
                export(nxt)
            reused += int(nxt.value == old)
            mine = nxt
        barrier.wait()
        if rank != ex:
            if order != "closed_first" and held.get(ex):
                hip.hipIpcCloseMemHandle(held[ex])  # retire the stale mapping
                if order == "recycle_gap":
                    time.sleep(0.02)
            held[ex] = open_peer(ex, r)
        barrier.wait()
        if order == "fresh_free_after" and rank == ex:
            for k in kept:
                hip.hipFree(k)
            kept.clear()
    for m in held.values():
        if m:
            hip.hipIpcCloseMemHandle(m)
    barrier.wait()
    hip.hipFree(mine)
    for k in kept:
        hip.hipFree(k)
    results.put({"rank": rank, "opens": opens, "fails": fails, "reused": reused, "errs": errs})


def run(n, rounds, size, order):
    ctx = mp.get_context("spawn")
    handles = ctx.Array(ctypes.c_char, 64 * n, lock=False)
    addr = ctx.Array(ctypes.c_uint64, n, lock=False)
    results = ctx.Queue()
    barrier = ctx.Barrier(n)
    procs = [ctx.Process(target=worker, args=(r, n, rounds, size, handles, addr, results, barrier, order))
             for r in range(n)]
    t0 = time.time()
    for p in procs:
        p.start()
    outs = [results.get(timeout=240) for _ in range(n)]
    for p in procs:
        p.join(timeout=60)
    print(json.dumps({"order": order, "n": n, "rounds": rounds, "size": size,
                      "opens": sum(o["opens"] for o in outs), "refusals": sum(o["fails"] for o in outs),
                      "address_reused": sum(o["reused"] for o in outs),
                      "first_errors": [e for o in outs for e in o["errs"]][:4],
                      "seconds": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    size = sys.argv[3] if len(sys.argv) > 3 else str(20 << 20)  # comma-separated sizes
    orders = sys.argv[4].split(",") if len(sys.argv) > 4 else \
        ("recycle_close_open", "recycle_gap", "closed_first", "fresh_address", "fresh_free_after",
         "fresh_keep")
    for sz in str(size).split(","):
        for o in orders:
            run(n, rounds, int(sz), o)
