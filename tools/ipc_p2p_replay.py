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
  realloc      after the import the odd rank frees its send buffer and
               allocates it again before exporting (an allocation made after
               the close)
  exporter_keeps  the even rank frees its previous send buffer only after
               the odd rank closed its mapping of it (the close releases no
               freed memory)
  close_sync   hipDeviceSynchronize between the import and the export
  retry        a refused export is tried again at once (does it stick?)
  dummy_export after the import, one export of a long-lived 4 MiB allocation
               first (does one export absorb the failure?)
  predict      the library's rule: after each close the odd rank notes the
               buffer id of a fresh allocation (a watermark); an allocation
               with a lower id (it predates the close) is not exported but
               counted as staged
keep_stale also records whether the open of the recycled address returned
the still-open stale mapping (the runtime's answer for an address it maps),
and every variant checks the bytes copied through the mapping (each
iteration's send buffer holds its iteration number).
Round 5 result (profiles/r05_ipc_p2p_replay.jsonl): plain refuses ~22-31 %
of the odd rank's exports, keep_stale none.
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
    st = {"exports": 0, "export_refusals": 0, "opens": 0, "open_refusals": 0, "addr_reuse": 0,
          "retry_ok": 0, "dummy_refusals": 0, "open_returned_stale": 0, "wrong_bytes": 0,
          "predicted_stage": 0, "ids_not_increasing": 0}
    errs = []
    mapped = None  # this rank's mapping of the peer's current buffer
    stream = ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(stream)) == 0
    host = (ctypes.c_ubyte * N_BYTES)()
    last_ds = None
    last_id = [0]
    keep = None

    dummy = ctypes.c_void_p()
    if variant == "dummy_export":
        assert hip.hipMalloc(ctypes.byref(dummy), ctypes.c_size_t(4 << 20)) == 0

    watermark = [0]

    def buffer_id(p):
        v = ctypes.c_ulonglong()
        # HIP_POINTER_ATTRIBUTE_BUFFER_ID = 7 (hip/driver_types.h)
        if hip.hipPointerGetAttribute(ctypes.byref(v), ctypes.c_int(7), p) != 0:
            hip.hipGetLastError()
            return 0
        return v.value

    def note_close():
        if variant != "predict":
            return
        t = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(t), ctypes.c_size_t(4096)) == 0
        watermark[0] = max(watermark[0], buffer_id(t))
        hip.hipFree(t)

    def export(ds, it):
        if variant == "predict" and buffer_id(ds) < watermark[0]:
            st["predicted_stage"] += 1
            ok[rank] = 0
            return
        h = Handle()
        e = hip.hipIpcGetMemHandle(ctypes.byref(h), ds)
        st["exports"] += 1
        if e != 0 and variant == "retry":
            hip.hipGetLastError()
            e = hip.hipIpcGetMemHandle(ctypes.byref(h), ds)
            st["retry_ok"] += int(e == 0)
            st["export_refusals"] += 1
            if e == 0:
                handles[rank * 64:(rank + 1) * 64] = bytes(h)
                ok[rank] = 1
                return
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
            note_close()
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
        if stale is not None and m.value == stale.value:
            st["open_returned_stale"] += 1
        mapped = m
        if variant != "no_copy":
            assert hip.hipMemcpyAsync(dr, m, ctypes.c_size_t(N_BYTES), 3, stream) == 0
            assert hip.hipStreamSynchronize(stream) == 0
            probe = (ctypes.c_ubyte * 64)()
            assert hip.hipMemcpy(probe, ctypes.c_void_p(dr.value + N_BYTES - 64), ctypes.c_size_t(64), 2) == 0
            st["wrong_bytes"] += int(any(b != (it & 0xFF) for b in probe))
        return stale

    for it in range(iters):
        ds, dr = ctypes.c_void_p(), ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(ds), ctypes.c_size_t(N_BYTES)) == 0
        assert hip.hipMalloc(ctypes.byref(dr), ctypes.c_size_t(N_BYTES)) == 0
        st["addr_reuse"] += int(ds.value == last_ds)
        last_ds = ds.value
        bid = buffer_id(ds)
        st["ids_not_increasing"] += int(bid <= last_id[0])
        last_id[0] = bid
        ctypes.memset(host, it & 0xFF, N_BYTES)
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
            elif variant == "close_sync":
                assert hip.hipDeviceSynchronize() == 0
            elif variant == "realloc":
                hip.hipFree(ds)
                assert hip.hipMalloc(ctypes.byref(ds), ctypes.c_size_t(N_BYTES)) == 0
                ctypes.memset(host, it & 0xFF, N_BYTES)
                assert hip.hipMemcpy(ds, host, ctypes.c_size_t(N_BYTES), 1) == 0
            elif variant == "dummy_export":
                h = Handle()
                if hip.hipIpcGetMemHandle(ctypes.byref(h), dummy) != 0:
                    st["dummy_refusals"] += 1
                    hip.hipGetLastError()
            export(ds, it)
            barrier.wait()
        if stale is not None:
            hip.hipIpcCloseMemHandle(stale)
        barrier.wait()
        if variant == "exporter_keeps" and rank == 0:
            # freed one round later: the odd rank's close of its mapping of
            # this buffer (next round) does not release freed memory
            if keep is not None:
                hip.hipFree(keep)
            keep = ds
        else:
            hip.hipFree(ds)
        hip.hipFree(dr)
        barrier.wait()
    if keep is not None:
        hip.hipFree(keep)
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
    variants = sys.argv[2].split(",") if len(sys.argv) > 2 else \
        ("plain", "no_copy", "keep_stale", "gap", "realloc", "exporter_keeps", "close_sync", "retry",
         "dummy_export", "predict")
    for v in variants:
        run(iters, v)
