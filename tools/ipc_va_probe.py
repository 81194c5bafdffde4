#!/usr/bin/env python3
"""Does a just-closed IPC import range poison the next allocation there?
(VERDICT r4 "next" item 1.)

The two runtime refusals round 4 still worked around share one lead: the
range involved had just been unmapped IN THE SAME PROCESS.
  - p2p: hipIpcGetMemHandle refused ("invalid argument") a fresh 8 MiB
    application allocation, right after this process received a peer's
    buffer through an IPC mapping (pml harness section 9);
  - registry: a re-import of a peer's recycled 20 MiB range was refused right
    after this process closed its stale mapping of that range.
Hypothesis: once an import mapping at V is closed, a NEW local allocation
that the runtime places over V is not exportable (the export fails, or the
peers' opens of its handle fail), because the runtime's bookkeeping still
associates V with the import.

Orders (2 processes on one GPU, E = rank 0 exports, I = rank 1 imports;
one JSON line per (order, size)):
  over_closed_import  I opens E's X at V, touches it, closes V, then
                      allocates Y until Y overlaps V (up to 8 tries; the
                      misses stay allocated until the round ends), exports Y;
                      E opens Y's handle
  natural             the same with ONE allocation after the close (records
                      how often the runtime places it over V by itself)
  control_open        I allocates Y while V is still mapped (Y cannot
                      overlap V), then closes V, exports Y; E opens it
  import_over_freed   I allocates Y, frees it, then opens E's X (which may
                      land over the freed Y): the import side
  exporter_freed      as over_closed_import, but E frees X before I closes V
                      (the library's order: a peer's buffer is retired after
                      its owner freed it)
Each line: rounds, how many overlapped, export refusals and open refusals
split by overlap, the first errors.  ctypes on libamdhip64 only (no library).
"""
import ctypes
import json
import multiprocessing as mp
import sys
import time

HIP = "/opt/rocm/lib/libamdhip64.so"


class Handle(ctypes.Structure):  # hipIpcMemHandle_t, passed by value to the open
    _fields_ = [("reserved", ctypes.c_char * 64)]


def overlap(a, b, size):
    return a is not None and b is not None and a < b + size and b < a + size


def worker(rank, rounds, size, order, shared, results, barrier):
    hip = ctypes.CDLL(HIP)
    assert hip.hipSetDevice(0) == 0
    hip.hipGetErrorString.restype = ctypes.c_char_p
    st = {"over": 0, "export_fail_over": 0, "export_fail_clear": 0, "open_fail_over": 0,
          "open_fail_clear": 0, "import_over_freed": 0, "import_fail_over": 0, "import_fail_clear": 0}
    errs = []

    def err(e):
        return hip.hipGetErrorString(e).decode()

    def malloc():
        p = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(size)) == 0
        return p

    for r in range(rounds):
        # --- E exports a fresh X
        x = None
        if rank == 0:
            x = malloc()
            assert hip.hipMemset(x, 1, ctypes.c_size_t(size)) == 0
            assert hip.hipDeviceSynchronize() == 0
            h = Handle()
            assert hip.hipIpcGetMemHandle(ctypes.byref(h), x) == 0
            shared["hx"][:] = bytes(h)
        barrier.wait()
        y = None
        extras = []
        if rank == 1:
            if order == "import_over_freed":
                yf = malloc()
                yv = yf.value
                hip.hipFree(yf)
            if order == "control_open":
                y = malloc()
            v = ctypes.c_void_p()
            e = hip.hipIpcOpenMemHandle(ctypes.byref(v), Handle.from_buffer_copy(bytes(shared["hx"][:])),
                                        ctypes.c_uint(1))
            if order == "import_over_freed":
                ov = e == 0 and overlap(v.value, yv, size)
                st["import_over_freed"] += int(ov)
                if e != 0:
                    st["import_fail_over" if ov else "import_fail_clear"] += 1
                    if len(errs) < 4:
                        errs.append(f"round {r} import ({'over' if ov else 'clear'}): {err(e)}")
                    hip.hipGetLastError()
            else:
                assert e == 0, f"open of X refused: {err(e)}"
            if e == 0:
                assert hip.hipMemset(v, 2, ctypes.c_size_t(size)) == 0  # touch through the mapping
                assert hip.hipDeviceSynchronize() == 0
        barrier.wait()
        if order == "exporter_freed" and rank == 0:
            hip.hipFree(x)
            x = None
        barrier.wait()
        ok_export = 0
        if rank == 1:
            vv = v.value if v.value else None
            if v.value:
                assert hip.hipIpcCloseMemHandle(v) == 0
            if order in ("over_closed_import", "natural", "exporter_freed"):
                tries = 8 if order != "natural" else 1
                for _ in range(tries):
                    cand = malloc()
                    if overlap(cand.value, vv, size):
                        y = cand
                        break
                    extras.append(cand)
                if y is None:
                    y = extras.pop()
            if order != "import_over_freed":
                ov = overlap(y.value, vv, size)
                st["over"] += int(ov)
                h = Handle()
                e = hip.hipIpcGetMemHandle(ctypes.byref(h), y)
                if e != 0:
                    st["export_fail_over" if ov else "export_fail_clear"] += 1
                    if len(errs) < 4:
                        errs.append(f"round {r} export ({'over' if ov else 'clear'}) y={y.value:#x} "
                                    f"v={vv:#x}: {err(e)}")
                    hip.hipGetLastError()
                else:
                    ok_export = 1
                    shared["hy"][:] = bytes(h)
                shared["flag"][0] = ok_export
                shared["flag"][1] = int(ov)
        barrier.wait()
        if rank == 0 and order != "import_over_freed" and shared["flag"][0]:
            w = ctypes.c_void_p()
            e = hip.hipIpcOpenMemHandle(ctypes.byref(w), Handle.from_buffer_copy(bytes(shared["hy"][:])),
                                        ctypes.c_uint(1))
            ov = bool(shared["flag"][1])
            if e != 0:
                st["open_fail_over" if ov else "open_fail_clear"] += 1
                if len(errs) < 4:
                    errs.append(f"round {r} open of Y ({'over' if ov else 'clear'}): {err(e)}")
                hip.hipGetLastError()
            else:
                hip.hipIpcCloseMemHandle(w)
        barrier.wait()
        if y is not None:
            hip.hipFree(y)
        for p in extras:
            hip.hipFree(p)
        if x is not None:
            hip.hipFree(x)
        barrier.wait()
    results.put({"rank": rank, "st": st, "errs": errs})


def run(rounds, size, order):
    ctx = mp.get_context("spawn")
    shared = {"hx": ctx.Array(ctypes.c_char, 64, lock=False), "hy": ctx.Array(ctypes.c_char, 64, lock=False),
              "flag": ctx.Array(ctypes.c_int, 2, lock=False)}
    results = ctx.Queue()
    barrier = ctx.Barrier(2)
    procs = [ctx.Process(target=worker, args=(r, rounds, size, order, shared, results, barrier))
             for r in range(2)]
    t0 = time.time()
    for p in procs:
        p.start()
    outs = [results.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    tot = {}
    for o in outs:
        for k, v in o["st"].items():
            tot[k] = tot.get(k, 0) + v
    print(json.dumps({"order": order, "size": size, "rounds": rounds, **tot,
                      "first_errors": [e for o in outs for e in o["errs"]][:4],
                      "seconds": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    sizes = sys.argv[2] if len(sys.argv) > 2 else f"{8 << 20},{20 << 20}"
    orders = sys.argv[3].split(",") if len(sys.argv) > 3 else \
        ("over_closed_import", "natural", "control_open", "import_over_freed", "exporter_freed")
    for sz in sizes.split(","):
        for o in orders:
            run(rounds, int(sz), o)
