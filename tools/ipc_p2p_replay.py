#!/usr/bin/env python3
"""Replay of pml harness section 9 with bare HIP calls.

Round 4's intermittent refused EXPORT (hipIpcGetMemHandle "invalid
argument" on a fresh 8 MiB allocation; pml harness section 9 with
p2p_user_ipc = 1, about once in 20-40 runs, always on the odd rank) happened
in this order, per iteration, at N = 2:
  both   allocate ds, dr (8 MiB) and fill ds
  even   export ds; wait for the odd rank's handle; import it (closing its
         mapping of the odd rank's previous, freed ds first: the registry's
         retire-then-open); copy through the mapping into dr
  odd    import the even rank's ds (same retire-then-open), copy it into dr,
         then export its own ds   <- refused here
  both   free ds and dr (peers still map them until their next import)
This probe runs that order for many iterations without the library, the
copy through the mapping by hipMemcpyAsync + stream sync, and counts export
and open refusals.  Variants (argv[2], comma-separated):
  plain        the order above
  no_copy      no copy through the new mapping (is device work involved?)
  keep_stale   close the stale mapping only AFTER the export (is the close
               right before the export involved?)
  gap          2 ms between the import and the export
Output: one JSON line per variant.  ctypes on libamdhip64 only.
"""
import ctypes
import json
import multiprocessing as mp
import sys
import time

HIP = "/opt/rocm/lib/libamdhip64.so"
N_BYTES = 8 << 20


class Handle(ctypes.Structure):
    _fields_ = [("reserved", ctypes.c_char * 64)]


def worker(rank, iters, variant, handles, ok, results, barrier):
    hip = ctypes.CDLL(HIP)
    assert hip.hipSetDevice(0) == 0
    hip.hipGetErrorString.restype = ctypes.c_char_p
    peer = 1 - rank
    st = {"exports": 0, "export_refusals": 0, "opens": 0, "open_refusals": 0, "addr_reuse": 0}
    errs = []
    mapped = None  # this rank's mapping of the peer's current buffer
    stream = ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(stream)) == 0
    host = (ctypes.c_ubyte * N_BYTES)()
    last_ds = None

    def export(ds, it):
        h = Handle()
        e = hip.hipIpcGetMemHandle(ctypes.byref(h), ds)
        st["exports"] += 1
        if e != 0:
            st["export_refusals"] += 1
            if len(errs) < 4:
                errs.append(f"iter {it} rank {rank} export {ds.value:#x}: {hip.hipGetErrorString(e).decode()}")
            hip.hipGetLastError()
            ok[rank] = 0
        else:
            handles[rank * 64:(rank + 1) * 64] = bytes(h)
            ok[rank] = 1

    def import_peer(it, dr, close_first):
        nonlocal mapped
        stale = mapped
        if stale is not None and close_first:
            hip.hipIpcCloseMemHandle(stale)
            stale = None
        m = ctypes.c_void_p()
        if not ok[peer]:
            mapped = None
            return stale
        e = hip.hipIpcOpenMemHandle(ctypes.byref(m), Handle.from_buffer_copy(bytes(handles[peer * 64:peer * 64 + 64])),
                                    ctypes.c_uint(1))
        st["opens"] += 1
        if e != 0:
            st["open_refusals"] += 1
            if len(errs) < 4:
                errs.append(f"iter {it} rank {rank} open: {hip.hipGetErrorString(e).decode()}")
            hip.hipGetLastError()
            mapped = None
            return stale
        mapped = m
        if variant != "no_copy":
            assert hip.hipMemcpyAsync(dr, m, ctypes.c_size_t(N_BYTES), 3, stream) == 0
            assert hip.hipStreamSynchronize(stream) == 0
        return stale

    for it in range(iters):
        ds, dr = ctypes.c_void_p(), ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(ds), ctypes.c_size_t(N_BYTES)) == 0
        assert hip.hipMalloc(ctypes.byref(dr), ctypes.c_size_t(N_BYTES)) == 0
        st["addr_reuse"] += int(ds.value == last_ds)
        last_ds = ds.value
        assert hip.hipMemcpy(ds, host, ctypes.c_size_t(N_BYTES), 1) == 0
        close_first = variant != "keep_stale"
        if rank == 0:
            export(ds, it)
            barrier.wait()  # even's handle published
            barrier.wait()  # odd's handle published
            stale = import_peer(it, dr, close_first)
        else:
            barrier.wait()
            stale = import_peer(it, dr, close_first)
            if variant == "gap":
                time.sleep(0.002)
            export(ds, it)
            barrier.wait()
        if stale is not None:
            hip.hipIpcCloseMemHandle(stale)
        barrier.wait()
        hip.hipFree(ds)
        hip.hipFree(dr)
        barrier.wait()
    if mapped is not None:
        hip.hipIpcCloseMemHandle(mapped)
    results.put({"rank": rank, "st": st, "errs": errs})


def run(iters, variant):
    ctx = mp.get_context("spawn")
    handles = ctx.Array(ctypes.c_char, 128, lock=False)
    ok = ctx.Array(ctypes.c_int, 2, lock=False)
    results = ctx.Queue()
    barrier = ctx.Barrier(2)
    procs = [ctx.Process(target=worker, args=(r, iters, variant, handles, ok, results, barrier)) for r in range(2)]
    t0 = time.time()
    for p in procs:
        p.start()
    outs = [results.get(timeout=600) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    by_rank = {o["rank"]: o["st"] for o in outs}
    print(json.dumps({"variant": variant, "iters": iters, "by_rank": by_rank,
                      "first_errors": [e for o in outs for e in o["errs"]][:4],
                      "seconds": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    variants = sys.argv[2].split(",") if len(sys.argv) > 2 else ("plain", "no_copy", "keep_stale", "gap")
    for v in variants:
        run(iters, v)
