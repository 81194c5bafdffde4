"""One rank of the process-wide IPC mapping test (tests/test_ipc_registry_gpu.py).

Two library communicators over the same ranks both map every peer's device
buffer X: communicator A through an osc window created over X, communicator
B through zero-copy allreduces with X as the send buffer (user_ipc = 1).  The
IPC registry (ompi_amd/csrc/ipc_registry.h) must hand both the same mapping
(ipc_shared grows) and keep it open while either still holds it:

  1. allreduce on B, window put/get on A: both bit-exact;
  2. the window is freed: B's next allreduces stay bit-exact (A's close of
     its references must not unmap B's);
  3. a new window on A over X, then B is destroyed: the window's put / get
     stay byte-exact;
  4. a freed + reallocated buffer at the address it had: the exporter does
     not export it again (reused_exports; ROCm 7.2 may refuse the peers'
     re-import right after they retire the old mapping) and
     the call runs through the shadow, exact;
  5. A's nonblocking allreduce launched on rank 0 only, while B's blocking
     allreduce retires stale mappings there (B exports reused addresses:
     param reuse_shadow = 0, to drive the registry's retire path): B
     completes at once (only the stale mappings' holders are quiesced) and
     both results are exact.

Prints one JSON line per step; exits 0 only if all passed.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from ompi_amd import coll, osc  # noqa: E402
from ompi_amd import op as mop  # noqa: E402
from oracle import oracle as orc  # noqa: E402

SEED = 20261017


def data(rank, count, salt):
    rng = np.random.default_rng(SEED + 100 * salt + rank)
    return rng.uniform(-1, 1, count).astype(np.float32)


def main():
    rank, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    device = int(os.environ.get("OMPI_AMD_DEVICE", "0"))
    torch.cuda.set_device(device)
    dist.init_process_group("gloo", rank=rank, world_size=n)
    A = coll.Communicator.from_torch_distributed(device=device)
    B = coll.Communicator.from_torch_distributed(device=device)
    for c in (A, B):
        c.set_param("timeout_ms", 20000)
    B.set_param("user_ipc", 1)
    B.set_param("algorithm", 0)  # pull: peers map X (the send buffer) directly
    count = (6 << 20) // 4 + 3   # zero-copy size on every N
    F, SUM = mop.MPI_FLOAT, mop.MPI_SUM
    ok_all = True

    def report(step, ok, msg="", **kw):
        nonlocal ok_all
        ok_all &= bool(ok)
        print(json.dumps({"rank": rank, "case": step, "ok": bool(ok), "msg": msg, **kw}), flush=True)

    def allreduce_check(X, salt):
        xs = [data(r, count, salt) for r in range(n)]
        exp, _ = orc.allreduce([x.copy() for x in xs], count, SUM.index, F.code)
        X[:count].copy_(torch.from_numpy(xs[rank]))
        y = torch.zeros(count, device="cuda")
        B.allreduce(X, y, count, F, SUM, blocking=True)
        got = y.cpu().numpy()
        ok = np.array_equal(got.view(np.uint32), exp[rank].view(np.uint32))
        return ok, "" if ok else f"{int((got != exp[rank]).sum())} of {count} differ"

    def window_check(win, X, salt):
        """put my pattern into the next rank's X, fence, get the previous
        rank's X back: byte-exact."""
        nxt, prv = (rank + 1) % n, (rank - 1) % n
        mine = torch.from_numpy(data(rank, 4096, salt)).cuda()
        win.fence(blocking=True)
        win.put(mine, nxt, 0, 4096 * 4)
        win.fence(blocking=True)
        got_local = X[:4096].cpu().numpy()          # written by prv
        back = torch.empty(4096, device="cuda")
        win.get(back, nxt, 0, 4096 * 4)             # what I wrote into nxt
        win.fence(blocking=True)
        ok = (np.array_equal(got_local.view(np.uint32), data(prv, 4096, salt).view(np.uint32)) and
              np.array_equal(back.cpu().numpy().view(np.uint32), mine.cpu().numpy().view(np.uint32)))
        return ok, "" if ok else "window bytes differ"

    X = torch.zeros(count + 64, device="cuda")
    try:
        shared0 = A.get_param("ipc_shared")
        win = osc.Window.create(A, X, disp_unit=4)
        ok, msg = allreduce_check(X, 1)
        shared = A.get_param("ipc_shared") - shared0
        report("shared_mapping_allreduce", ok and shared >= n - 1,
               msg or ("" if shared >= n - 1 else f"ipc_shared grew by {shared}, expected >= {n - 1}"),
               ipc_shared=shared, ipc_live=A.get_param("ipc_live"))
        ok, msg = window_check(win, X, 2)
        report("shared_mapping_window", ok, msg)
        win.free()  # A drops its references: B's mappings of X must stay
        msgs = []
        for k in range(3):
            ok, msg = allreduce_check(X, 3 + k)
            if not ok:
                msgs.append(f"allreduce {k}: {msg}")
        report("window_freed_allreduce_on", not msgs, "; ".join(msgs),
               ipc_live=A.get_param("ipc_live"), ipc_refs=A.get_param("ipc_refs"))
        win = osc.Window.create(A, X, disp_unit=4)
        ok, msg = allreduce_check(X, 7)  # B maps X again (shared with the window)
        torch.cuda.synchronize()
        B.free()  # B's references go: the window's must stay
        B = None
        msgs = []
        for k in range(3):
            ok2, msg2 = window_check(win, X, 8 + k)
            if not ok2:
                msgs.append(f"window {k}: {msg2}")
        report("comm_destroyed_window_on", ok and not msgs, "; ".join([msg] + msgs).strip("; "))
        win.free()
        # a freed and reallocated peer buffer: the registry retires the old
        # mapping (once, for every holder) and maps the new allocation
        B = coll.Communicator.from_torch_distributed(device=device)
        B.set_param("timeout_ms", 20000)
        B.set_param("user_ipc", 1)
        B.set_param("algorithm", 0)
        win = osc.Window.create(A, X, disp_unit=4)
        ok, msg = allreduce_check(X, 11)
        win.free()
        torch.cuda.synchronize()
        retired0 = B.get_param("ipc_retired")
        reused0 = B.get_param("reused_exports")
        old_ptr = X.data_ptr()
        del X
        torch.cuda.empty_cache()
        dist.barrier()
        X = torch.zeros(count + 64, device="cuda")
        same = X.data_ptr() == old_ptr
        ok2, msg2 = allreduce_check(X, 12)
        retired = B.get_param("ipc_retired") - retired0
        reused = B.get_param("reused_exports") - reused0
        report("realloc_same_address_shadowed", ok and ok2 and (reused >= 1 or not same),
               "; ".join(m for m in (msg, msg2, "" if reused >= 1 or not same else
                                     "a reused address was exported again") if m),
               same_address=same, reused_exports=reused, ipc_retired=retired)
        # 5. a deferred call of A launched on rank 0 but not yet on its peers
        # while B's blocking call on rank 0 retires a stale mapping (ADVICE
        # r3): the registry quiesces only the stale mapping's holders (B),
        # and only up to B's own last kernels on each stream; the runtime's
        # close of the retired mapping still waits for every kernel of the
        # device (A's, spinning on its peers), so the peers' waits in B must
        # launch A meanwhile (progress_others, MPI's progress rule).  B's send
        # buffer is a raw hipMalloc freed and allocated again (same size:
        # normally the same address), so the peers' mappings of it go stale.
        import ctypes
        import time
        # the HIP runtime this process already runs (torch's): dlopen of
        # its exact path returns that handle, not a second runtime
        with open("/proc/self/maps") as f_:
            hip_path = next(ln.split()[-1] for ln in f_ if "libamdhip64.so" in ln)
        hip = ctypes.CDLL(hip_path)
        nbytes = 22 << 20  # a whole number of 2 MiB pages (exportable as is)

        def raw(vals):
            p_ = ctypes.c_void_p()
            assert hip.hipMalloc(ctypes.byref(p_), ctypes.c_size_t(nbytes)) == 0
            h = np.zeros(nbytes // 4, np.float32)
            h[:count] = vals
            assert hip.hipMemcpy(p_, h.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(nbytes), 1) == 0
            return p_

        A.set_param("user_ipc", 1)
        A.set_param("algorithm", 0)
        B.set_param("reuse_shadow", 0)
        y = torch.zeros(count, device="cuda")
        xs = [data(r, count, 15) for r in range(n)]
        p1 = raw(xs[rank])
        torch.cuda.synchronize()
        B.allreduce(p1.value, y, count, F, SUM, blocking=True)  # peers map p1
        torch.cuda.synchronize()
        dist.barrier()
        assert hip.hipFree(p1) == 0
        xs = [data(r, count, 13) for r in range(n)]
        xexp, _ = orc.allreduce([x.copy() for x in xs], count, SUM.index, F.code)
        p2 = raw(xs[rank])
        zs_h = [data(r, count, 14) for r in range(n)]
        zexp, _ = orc.allreduce([z.copy() for z in zs_h], count, SUM.index, F.code)
        zs = torch.from_numpy(zs_h[rank]).cuda()
        zo = torch.zeros(count, device="cuda")
        sB = torch.cuda.Stream()
        torch.cuda.synchronize()  # nothing of A is on the device yet
        retired0 = B.get_param("ipc_retired")
        reused = [None] * n
        dist.all_gather_object(reused, p2.value == p1.value)
        dist.barrier()
        if rank != 0:
            req = A.iallreduce(zs, zo, count, F, SUM)   # posted, not launched here yet
        dist.barrier()
        if rank == 0:
            req = A.iallreduce(zs, zo, count, F, SUM)   # every peer posted: launched on rank 0
        t0 = time.time()
        # B on a stream of its own, and no device-wide synchronisation until
        # A completes: device work of communicators sharing one stream is
        # serialised by the stream itself (A's launched call would hold B's
        # kernels back whatever the registry does)
        # (waits as coll/rocm's blocking call does: ompi_amd_comm_sync, which
        # launches A's deferred call on a rank whose peers already posted it)
        B.allreduce(p2.value, y, count, F, SUM, stream=sB)
        B.sync(sB)
        dt = time.time() - t0
        req.wait()
        req.free()
        torch.cuda.synchronize()
        ok = np.array_equal(y.cpu().numpy().view(np.uint32), xexp[rank].view(np.uint32))
        okz = np.array_equal(zo.cpu().numpy().view(np.uint32), zexp[rank].view(np.uint32))
        retired = B.get_param("ipc_retired") - retired0
        # a peer's reallocation at the same address must have been retired here
        need = any(reused[q] for q in range(n) if q != rank)
        report("deferred_on_A_while_B_retires", ok and okz and dt < 10.0 and (retired > 0 or not need),
               "; ".join(m for m in ("" if ok else "B's allreduce differs",
                                     "" if okz else "A's iallreduce differs",
                                     "" if dt < 10.0 else f"B's call took {dt:.1f} s",
                                     "" if retired > 0 or not need else "no stale mapping retired") if m),
               b_call_s=round(dt, 3), ipc_retired=retired, peers_reused_address=need)
        assert hip.hipFree(p2) == 0
    except Exception as e:  # noqa: BLE001
        report("exception", False, f"{type(e).__name__}: {e}")
    torch.cuda.synchronize()
    if B is not None:
        B.free()
    A.free()
    dist.destroy_process_group()
    sys.exit(0 if ok_all else 1)


if __name__ == "__main__":
    main()
