"""One rank of the multi-process collective parity test (tests/test_coll_gpu.py).

Launched N times with RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT and
OMPI_AMD_DEVICE.  Bootstraps a gloo group (only to broadcast the segment
name), creates an ompi_amd Communicator, runs every case on device buffers
and checks the result against the CPU oracle, which each rank evaluates for
all ranks from the deterministic per-rank inputs.  Prints one JSON line per
case and exits 0 only if all passed.
"""
import functools
import json
import os
import sys
import time
import signal
import traceback

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from ompi_amd import coll  # noqa: E402
from ompi_amd import op as mop  # noqa: E402
from oracle import oracle as orc  # noqa: E402

SEED = 20261015


def inputs(dt: mop.Datatype, count: int, rank: int, salt: int, kind: str = "R") -> np.ndarray:
    rng = np.random.default_rng(SEED + 1000 * salt + rank)
    nd = dt.np_dtype
    if nd.names:  # MAXLOC pairs: quantised values force ties (BASELINE config 5)
        a = np.zeros(count, dtype=nd)
        a["v"] = np.round(rng.random(count) * 1024) / 1024
        a["k"] = rank * count + np.arange(count)
        return a
    if nd.kind == "f":
        if kind == "E":  # exact: k * 2^-8, all orders agree
            return (rng.integers(-1024, 1025, count) * 2.0 ** -8).astype(nd)
        a = rng.uniform(-1, 1, count).astype(nd)
        if kind == "S":  # specials for MAX/MIN
            sp = np.array([np.nan, 0.0, -0.0, np.inf, -np.inf], dtype=nd)
            idx = rng.integers(0, count, max(1, count // 8))
            a[idx] = rng.choice(sp, len(idx))
        return a
    info = np.iinfo(nd)
    lo, hi = (-(1 << 20), 1 << 20) if nd.itemsize >= 4 else (info.min, info.max)
    if info.min == 0:
        lo = 0
    return rng.integers(lo, hi, count, dtype=nd, endpoint=True)


def to_dev(a: np.ndarray, extra: int = 0):
    raw = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
    t = torch.zeros(raw.nbytes + extra, dtype=torch.uint8, device="cuda")
    t[:raw.nbytes].copy_(torch.from_numpy(raw.copy()))
    return t


def mismatch(got: np.ndarray, exp: np.ndarray) -> str:
    """Where got and exp differ (for the failure report)."""
    if got.dtype.names:
        got, exp = got["v"], exp["v"]
    g = np.ascontiguousarray(got).view(np.uint8).reshape(got.size, -1)
    e = np.ascontiguousarray(exp).view(np.uint8).reshape(exp.size, -1)
    bad = np.flatnonzero((g != e).any(axis=1))
    if got.dtype.kind == "f":
        bad = bad[~(np.isnan(got[bad]) & np.isnan(exp[bad]))]
    if bad.size == 0:
        return ""
    zeros = int(np.count_nonzero(g[bad] == 0) // g.shape[1])
    return (f"{bad.size}/{got.size} differ, first {bad[:3].tolist()} last {int(bad[-1])}: "
            f"got {got[bad[:3]].tolist()} exp {exp[bad[:3]].tolist()}, {zeros} all-zero")


def checked(got: np.ndarray, exp: np.ndarray) -> tuple[bool, str]:
    ok = fields_equal(got, exp)
    return ok, "" if ok else mismatch(got, exp)


def fields_equal(got: np.ndarray, exp: np.ndarray) -> bool:
    if got.dtype.names:
        return all(np.array_equal(np.ascontiguousarray(got[f]).view(np.uint8),
                                  np.ascontiguousarray(exp[f]).view(np.uint8)) for f in ("v", "k"))
    g, e = got.view(np.uint8), exp.view(np.uint8)
    if np.array_equal(g, e):
        return True
    if got.dtype.kind == "f":
        nan = np.isnan(got) & np.isnan(exp)
        return np.array_equal(got[~nan].view(np.uint8), exp[~nan].view(np.uint8))
    return False


def case_allreduce(comm, rank, n, dt, op, count, salt, kind="R", inplace=False, repeat=1):
    for it in range(repeat):
        xs = [inputs(dt, count, r, salt + it, kind) for r in range(n)]
        exp, _ = orc.allreduce([x.copy() for x in xs], count, op.index, dt.code)
        s = to_dev(xs[rank])
        if inplace:
            comm.allreduce(coll.IN_PLACE, s, count, dt, op, blocking=True)
            out = s
        else:
            out = torch.zeros_like(s)
            comm.allreduce(s, out, count, dt, op, blocking=True)
        got = out.cpu().numpy()[:count * dt.extent].view(dt.np_dtype)
        if not fields_equal(got, exp[rank]):
            return False, f"iter {it}: {mismatch(got, exp[rank])}"
    return True, ""


def case_allreduce_wait(comm, rank, n, salt, repeat=40):
    """ompi_amd_allreduce_wait (coll/rocm's blocking MPI_Allreduce): at fused
    sizes the kernel's last workgroup stores the host-observed completion
    itself (a finished-workgroup counter reset by that workgroup), so many
    calls back to back, recursive-doubling and ring orders, one and many
    workgroups, in place, must each be exact before the next starts; a
    staged size takes the ordinary wait."""
    F = mop.MPI_FLOAT
    for it in range(repeat):
        count = (1, 2499, 2500, 16383, 100003)[it % 5]
        xs = [inputs(F, count, r, salt + it) for r in range(n)]
        exp, _ = orc.allreduce([x.copy() for x in xs], count, mop.MPI_SUM.index, F.code)
        s = to_dev(xs[rank])
        out = s if it % 3 == 2 else torch.zeros_like(s)
        torch.cuda.synchronize()  # inputs in place before the library's stream reads them
        if it % 3 == 2:
            comm.allreduce_wait(coll.IN_PLACE, s, count, F, mop.MPI_SUM)
        else:
            comm.allreduce_wait(s, out, count, F, mop.MPI_SUM)
        # no stream sync here: the wait itself is the completion
        got = out.cpu().numpy()[:count * 4].view(np.float32)
        if not fields_equal(got, exp[rank]):
            return False, f"iter {it} count {count}: {mismatch(got, exp[rank])}"
    return True, ""


def case_ring_segmented_R(comm, rank, n, count, salt, algorithm=None):
    """coll/tuned's ring_segmented decision (bytes > N x 1 MiB,
    coll_tuned_decision_fixed.c:72-86) on order-sensitive data (dataset R):
    the device result must be the oracle's ring_segmented bits.  Sized past
    N x 1 MiB at every N (at N = 8 the general cases' COLL_BIG is below it)."""
    assert count * 4 > n * (1 << 20), "not in the ring_segmented range"
    xs = [inputs(mop.MPI_FLOAT, count, r, salt, "R") for r in range(n)]
    exp, alg = orc.allreduce([x.copy() for x in xs], count, mop.MPI_SUM.index, mop.MPI_FLOAT.code)
    if alg != orc.ALG_RING_SEGMENTED:
        return False, f"oracle decision {alg}, expected ring_segmented"
    s = to_dev(xs[rank])
    out = torch.zeros_like(s)
    if algorithm is not None:
        comm.set_param("algorithm", algorithm)
    try:
        comm.allreduce(s, out, count, mop.MPI_FLOAT, mop.MPI_SUM, blocking=True)
    finally:
        if algorithm is not None:
            comm.set_param("algorithm", DEFAULT_ALG[0])
    got = out.cpu().numpy()[:count * 4].view(np.float32)
    ok = fields_equal(got, exp[rank])
    return ok, "" if ok else mismatch(got, exp[rank])


def case_forced(comm, rank, n, alg, dt, op, count, salt, inplace=False, how="blocking"):
    """MPI_Allreduce with coll_tuned_allreduce_algorithm forced to `alg`
    (coll_tuned_allreduce_decision.c:37-147): the device result must be the
    forced algorithm's bits (oracle.allreduce_forced), through the blocking,
    nonblocking or persistent entry point."""
    xs = [inputs(dt, count, r, salt) for r in range(n)]
    exp, _ = orc.allreduce_forced([x.copy() for x in xs], count, op.index, dt.code, alg,
                                  root0_inplace=inplace)
    s = to_dev(xs[rank])
    out = s if inplace else torch.zeros_like(s)
    src = coll.IN_PLACE if inplace else s
    comm.set_param("tuned_allreduce_algorithm", alg)
    try:
        if how == "blocking":
            comm.allreduce(src, out, count, dt, op, blocking=True)
        elif how == "nonblocking":
            req = comm.iallreduce(src, out, count, dt, op)
            req.wait()
            req.free()
            torch.cuda.synchronize()
        else:
            plan = comm.allreduce_init(src, out, count, dt, op)
            try:
                plan.start()
                plan.wait()
            finally:
                plan.free()
            torch.cuda.synchronize()
    finally:
        comm.set_param("tuned_allreduce_algorithm", 0)
    got = out.cpu().numpy()[:count * dt.extent].view(dt.np_dtype)
    return checked(got, exp[rank])


def case_rsb_kind(comm, rank, n, dt, op, rcount, salt, kind):
    return case_rsb(comm, rank, n, dt, op, rcount, salt, kind=kind)


def case_rsb(comm, rank, n, dt, op, rcount, salt, inplace=False, kind="R"):
    xs = [inputs(dt, rcount * n, r, salt, kind) for r in range(n)]
    exp = orc.reduce_scatter_block([x.copy() for x in xs], rcount, op.index, dt.code)
    s = to_dev(xs[rank])
    if inplace:
        comm.reduce_scatter_block(coll.IN_PLACE, s, rcount, dt, op, blocking=True)
        out = s
    else:
        out = torch.zeros(rcount * dt.extent, dtype=torch.uint8, device="cuda")
        comm.reduce_scatter_block(s, out, rcount, dt, op, blocking=True)
    got = out.cpu().numpy()[:rcount * dt.extent].view(dt.np_dtype)
    return checked(got, exp[rank].view(dt.np_dtype))


def case_reduce(comm, rank, n, dt, op, count, root, salt, inplace=False, kind="R"):
    root = root % n
    xs = [inputs(dt, count, r, salt, kind) for r in range(n)]
    exp, _ = orc.reduce([x.copy() for x in xs], count, op.index, dt.code, root, inplace)
    s = to_dev(xs[rank])
    out = None
    if rank == root:
        if inplace:
            comm.reduce(coll.IN_PLACE, s, count, dt, op, root, blocking=True)
            out = s
        else:
            out = torch.zeros_like(s)
            comm.reduce(s, out, count, dt, op, root, blocking=True)
    else:
        comm.reduce(s, None, count, dt, op, root, blocking=True)
    if rank != root:
        return True, ""
    got = out.cpu().numpy()[:count * dt.extent].view(dt.np_dtype)
    return checked(got, exp.view(dt.np_dtype))


def case_scan(comm, rank, n, dt, op, count, salt, exclusive=False, inplace=False):
    xs = [inputs(dt, count, r, salt) for r in range(n)]
    exp = orc.scan([x.copy() for x in xs], count, op.index, dt.code, exclusive)
    s = to_dev(xs[rank])
    fn = comm.exscan if exclusive else comm.scan
    if inplace:
        fn(coll.IN_PLACE, s, count, dt, op, blocking=True)
        out = s
    else:
        out = torch.zeros_like(s)
        fn(s, out, count, dt, op, blocking=True)
    if exclusive and rank == 0:
        return True, ""
    got = out.cpu().numpy()[:count * dt.extent].view(dt.np_dtype)
    return checked(got, exp[rank].view(dt.np_dtype))


def case_rs(comm, rank, n, dt, op, rcounts, salt, inplace=False, kind="R"):
    total = sum(rcounts)
    xs = [inputs(dt, total, r, salt, kind) for r in range(n)]
    exp, _ = orc.reduce_scatter([x.copy() for x in xs], rcounts, op.index, dt.code)
    s = to_dev(xs[rank], extra=16)
    if inplace:
        comm.reduce_scatter(coll.IN_PLACE, s, rcounts, dt, op, blocking=True)
        out = s
    else:
        out = torch.zeros((rcounts[rank] + 1) * dt.extent, dtype=torch.uint8, device="cuda")
        comm.reduce_scatter(s, out, rcounts, dt, op, blocking=True)
    got = out.cpu().numpy()[:rcounts[rank] * dt.extent].view(dt.np_dtype)
    return checked(got, exp[rank].view(dt.np_dtype))


def case_nb_reduce_scan_rs(comm, rank, n, salt, big):
    """MPI_Ireduce / MPI_Iscan / MPI_Iexscan / MPI_Ireduce_scatter (coll.h:
    276-300): eight calls outstanding at once — staged and landing sizes,
    the root in place, uneven reduce_scatter counts with an empty block and
    in place — with a blocking allreduce posted in between and rank 0
    posting while its peers sleep; every result bit-exact against the
    oracle's order of the blocking call."""
    import time
    F, D, I32 = mop.MPI_FLOAT, mop.MPI_DOUBLE, mop.MPI_INT32_T
    SUM, MAX = mop.MPI_SUM, mop.MPI_MAX
    checks, reqs = [], []
    if rank != 0:
        time.sleep(0.3)  # rank 0 posts everything before its peers arrive

    def ireduce(dt, op, count, root, inplace, sl):
        root %= n
        xs = [inputs(dt, count, r, sl) for r in range(n)]
        exp, _ = orc.reduce([x.copy() for x in xs], count, op.index, dt.code, root, inplace)
        s = to_dev(xs[rank])
        out = None
        if rank == root:
            out = s if inplace else torch.zeros_like(s)
            reqs.append(comm.ireduce(coll.IN_PLACE if inplace else s, out, count, dt, op, root))
            checks.append((f"ireduce {count} root {root}", out, count, dt, exp))
        else:
            reqs.append(comm.ireduce(s, None, count, dt, op, root))
        checks.append(("keep", s, 0, dt, None))

    def iscan(dt, op, count, exclusive, inplace, sl):
        xs = [inputs(dt, count, r, sl) for r in range(n)]
        exp = orc.scan([x.copy() for x in xs], count, op.index, dt.code, exclusive)
        s = to_dev(xs[rank])
        out = s if inplace else torch.zeros_like(s)
        reqs.append(comm.iscan(coll.IN_PLACE if inplace else s, out, count, dt, op,
                               exclusive=exclusive))
        if not (exclusive and rank == 0):
            checks.append((f"{'iexscan' if exclusive else 'iscan'} {count}", out, count, dt, exp[rank]))
        checks.append(("keep", s, 0, dt, None))

    def irs(dt, op, rcounts, inplace, sl):
        total = sum(rcounts)
        xs = [inputs(dt, total, r, sl) for r in range(n)]
        exp, _ = orc.reduce_scatter([x.copy() for x in xs], rcounts, op.index, dt.code)
        s = to_dev(xs[rank], extra=16)
        out = s if inplace else torch.zeros((rcounts[rank] + 1) * dt.extent, dtype=torch.uint8,
                                            device="cuda")
        reqs.append(comm.ireduce_scatter(coll.IN_PLACE if inplace else s, out, rcounts, dt, op))
        checks.append((f"ireduce_scatter {total}", out, rcounts[rank], dt, exp[rank]))
        checks.append(("keep", s, 0, dt, None))

    ireduce(F, SUM, 3001, n - 1, False, salt)
    ireduce(D, SUM, big // 2 + 3, 1, True, salt + 1)
    iscan(F, SUM, big + 7, False, False, salt + 2)
    iscan(I32, MAX, 5000, True, True, salt + 3)
    irs(F, SUM, [big // n + 5 * r if r != 1 else 0 for r in range(n)], False, salt + 4)
    # a blocking collective between the posts (it launches the deferred ones first)
    ok_b, msg_b = case_allreduce(comm, rank, n, F, SUM, 12345, salt + 5)
    irs(D, SUM, [big // (2 * n) + r for r in range(n)], True, salt + 6)
    ireduce(F, MAX, big + 11, 0, False, salt + 7)
    iscan(D, SUM, 999, True, False, salt + 8)
    for r in reqs:
        r.wait()
        r.free()
    torch.cuda.synchronize()
    msgs = [] if ok_b else [f"allreduce in between: {msg_b}"]
    for name, out, count, dt, exp in checks:
        if exp is None:
            continue
        got = out.cpu().numpy()[:count * dt.extent].view(dt.np_dtype)
        ok, msg = checked(got, np.asarray(exp).view(dt.np_dtype)[:count])
        if not ok:
            msgs.append(f"{name}: {msg}")
    return not msgs, "; ".join(msgs)


def case_persistent_rsb_ag_bcast(comm, rank, n, salt, big):
    """MPI_Reduce_scatter_block_init / MPI_Allgather_init / MPI_Bcast_init
    (coll.h:545-566): three starts each with fresh data in the same buffers,
    staged and zero-copy sizes, in place, every result checked against the
    oracle / the expected bytes; the three plans started back to back before
    any wait."""
    DI, F = mop.MPI_DOUBLE_INT, mop.MPI_FLOAT
    msgs = []
    for size_tag, rc_di, ag_bytes, bc_bytes in (("staged", 1000, 5000, 4097),
                                                ("zero_copy", big // 8 + 3, (big * 4) // n + 20,
                                                 big * 4 + 13)):
        sb = torch.zeros(rc_di * n * DI.extent, dtype=torch.uint8, device="cuda")
        rb = torch.zeros(rc_di * DI.extent, dtype=torch.uint8, device="cuda")
        agin = torch.zeros(ag_bytes, dtype=torch.uint8, device="cuda")
        agout = torch.zeros(ag_bytes * n, dtype=torch.uint8, device="cuda")
        bc = torch.zeros(bc_bytes, dtype=torch.uint8, device="cuda")
        root = (salt + len(size_tag)) % n
        p_rsb = comm.reduce_scatter_block_init(sb, rb, rc_di, DI, mop.MPI_MAXLOC)
        p_ag = comm.allgather_init(agin, agout, ag_bytes)
        p_bc = comm.bcast_init(bc, bc_bytes, root)
        try:
            for it in range(3):
                xs = [inputs(DI, rc_di * n, r, salt + it) for r in range(n)]
                exp = orc.reduce_scatter_block([x.copy() for x in xs], rc_di, mop.MPI_MAXLOC.index, DI.code)
                sb.copy_(torch.from_numpy(xs[rank].view(np.uint8).copy()).cuda())
                pays = [np.random.default_rng(SEED + 77 * it + r).integers(0, 256, ag_bytes, dtype=np.uint8)
                        for r in range(n)]
                agin.copy_(torch.from_numpy(pays[rank]).cuda())
                bpay = np.random.default_rng(SEED + 99 * it).integers(0, 256, bc_bytes, dtype=np.uint8)
                bc.copy_(torch.from_numpy(bpay if rank == root else np.zeros(bc_bytes, np.uint8)).cuda())
                torch.cuda.synchronize()
                p_rsb.start()
                p_ag.start()
                p_bc.start()
                for p in (p_rsb, p_ag, p_bc):
                    p.wait()
                torch.cuda.synchronize()
                got = rb.cpu().numpy().view(DI.np_dtype)
                ok, msg = checked(got, exp[rank].view(DI.np_dtype))
                if not ok:
                    msgs.append(f"{size_tag} start {it} rsb: {msg}")
                if not np.array_equal(agout.cpu().numpy(), np.concatenate(pays)):
                    msgs.append(f"{size_tag} start {it} allgather differs")
                if not np.array_equal(bc.cpu().numpy(), bpay):
                    msgs.append(f"{size_tag} start {it} bcast differs")
        finally:
            for p in (p_rsb, p_ag, p_bc):
                p.free()
    return not msgs, "; ".join(msgs)


def case_persistent_reduce_scan_rs(comm, rank, n, salt, big):
    """MPI_Reduce_init / MPI_Scan_init / MPI_Exscan_init /
    MPI_Reduce_scatter_init (coll.h:561-567 coll_reduce_init,
    coll_scan_init, coll_exscan_init, coll_reduce_scatter_init): three starts
    each with fresh data in the same buffers, staged and landing sizes, the
    reduce root in place, uneven reduce_scatter counts with an empty block,
    the four plans started back to back before any wait; every result
    bit-exact against the oracle's order of the blocking call."""
    F, D, I32 = mop.MPI_FLOAT, mop.MPI_DOUBLE, mop.MPI_INT32_T
    SUM, MAX = mop.MPI_SUM, mop.MPI_MAX
    msgs = []
    for tag, count, dt, op in (("staged", 3001, F, SUM), ("landing", big + 7, D, SUM),
                               ("landing_max", big // 2 + 5, I32, MAX)):
        root = (salt + count) % n
        root_inplace = tag == "landing"
        rcounts = [count // n + 3 * r if r != 1 else 0 for r in range(n)]
        ext = dt.extent
        sb = torch.zeros(count * ext, dtype=torch.uint8, device="cuda")
        rd = torch.zeros(count * ext, dtype=torch.uint8, device="cuda")
        sc = torch.zeros(count * ext, dtype=torch.uint8, device="cuda")
        ex = torch.zeros(count * ext, dtype=torch.uint8, device="cuda")
        rs = torch.zeros((rcounts[rank] + 1) * ext, dtype=torch.uint8, device="cuda")
        rsin = torch.zeros(sum(rcounts) * ext, dtype=torch.uint8, device="cuda")
        if rank == root:
            p_red = comm.reduce_init(coll.IN_PLACE if root_inplace else sb, rd, count, dt, op, root)
        else:
            p_red = comm.reduce_init(sb, None, count, dt, op, root)
        p_scan = comm.scan_init(sb, sc, count, dt, op)
        p_ex = comm.scan_init(sb, ex, count, dt, op, exclusive=True)
        p_rs = comm.reduce_scatter_init(rsin, rs, rcounts, dt, op)
        plans = (p_red, p_scan, p_ex, p_rs)
        try:
            for it in range(3):
                xs = [inputs(dt, count, r, salt + 10 * it) for r in range(n)]
                ys = [inputs(dt, sum(rcounts), r, salt + 10 * it + 5) for r in range(n)]
                red, _ = orc.reduce([x.copy() for x in xs], count, op.index, dt.code, root,
                                    root_inplace)
                scan = orc.scan([x.copy() for x in xs], count, op.index, dt.code, False)
                exs = orc.scan([x.copy() for x in xs], count, op.index, dt.code, True)
                rse, _ = orc.reduce_scatter([y.copy() for y in ys], rcounts, op.index, dt.code)
                mine = torch.from_numpy(xs[rank].view(np.uint8).copy()).cuda()
                sb.copy_(mine)
                if rank == root and root_inplace:
                    rd.copy_(mine)
                rsin.copy_(torch.from_numpy(ys[rank].view(np.uint8).copy()).cuda())
                torch.cuda.synchronize()
                for p in plans:
                    p.start()
                for p in plans:
                    p.wait()
                torch.cuda.synchronize()
                want = [("scan", sc, count, scan[rank]), ("reduce_scatter", rs, rcounts[rank], rse[rank])]
                if rank == root:
                    want.append(("reduce", rd, count, red))
                if rank > 0:
                    want.append(("exscan", ex, count, exs[rank]))
                for name, buf, c, e in want:
                    got = buf.cpu().numpy()[:c * ext].view(dt.np_dtype)
                    ok, msg = checked(got, np.asarray(e).view(dt.np_dtype)[:c])
                    if not ok:
                        msgs.append(f"{tag} start {it} {name}: {msg}")
        finally:
            for p in plans:
                p.free()
    return not msgs, "; ".join(msgs)


def case_zero_counts(comm, rank, n, salt):
    """Zero elements / bytes in every entry point — blocking, nonblocking and
    persistent — (MPI filters count 0 above coll only for some calls,
    allreduce.c:104): every call succeeds on every rank, nothing is written
    (sentinel bytes stay), and the communicator's epochs stay paired (a
    normal allreduce right after is bit-exact)."""
    F, SUM = mop.MPI_FLOAT, mop.MPI_SUM
    sent = np.full(64, 0xA5, np.uint8)
    a, b = to_dev(sent), to_dev(sent)
    comm.allreduce(a, b, 0, F, SUM)
    comm.reduce(a, b, 0, F, SUM, n - 1)
    comm.scan(a, b, 0, F, SUM)
    comm.exscan(a, b, 0, F, SUM)
    comm.reduce_scatter_block(a, b, 0, F, SUM)
    comm.reduce_scatter(a, b, [0] * n, F, SUM)
    comm.allgather(a, b, 0)
    comm.bcast(b, 0, 0)
    reqs = [comm.iallreduce(a, b, 0, F, SUM), comm.ireduce(a, b, 0, F, SUM, 0),
            comm.iscan(a, b, 0, F, SUM), comm.iscan(a, b, 0, F, SUM, exclusive=True),
            comm.ireduce_scatter_block(a, b, 0, F, SUM), comm.ireduce_scatter(a, b, [0] * n, F, SUM),
            comm.iallgather(a, b, 0), comm.ibcast(b, 0, n - 1)]
    for r in reqs:
        r.wait()
        r.free()
    plans = [comm.allreduce_init(a, b, 0, F, SUM), comm.reduce_scatter_block_init(a, b, 0, F, SUM),
             comm.allgather_init(a, b, 0), comm.bcast_init(b, 0, 0)]
    for _ in range(2):
        for p in plans:
            p.start()
        for p in plans:
            p.wait()
    for p in plans:
        p.free()
    torch.cuda.synchronize()
    for t, what in ((a, "sbuf"), (b, "rbuf")):
        if not np.array_equal(t.cpu().numpy(), sent):
            return False, f"a zero-count call wrote into {what}"
    return case_allreduce(comm, rank, n, F, SUM, 4099, salt)


def case_pipe(comm, rank, n, salt, big):
    """The pipelined schemes (param "algorithm" 4 push-gather, 5 push-land,
    6 staged pull: send, fold and gather of one call in one launch with
    per-slice flags, pipe_allreduce_kernel): bit-exact against the oracle on
    dataset R at the default (one pass per workgroup) and at 8 passes of
    slices down to 256 B, ragged counts, in place, fp64 and MAXLOC, and on buffers 4 B
    off 16-B alignment (the kernel's scalar paths); every call must have run
    the pipelined launch (param pipe_calls)."""
    F, D, DI = mop.MPI_FLOAT, mop.MPI_DOUBLE, mop.MPI_DOUBLE_INT
    SUM = mop.MPI_SUM
    try:
        for a in (4, 5, 6):
            comm.set_param("algorithm", a)
            for sl, passes in ((64 << 10, 1), (256, 8)):
                comm.set_param("pipe_slice", sl)
                comm.set_param("pipe_passes", passes)
                runs = [(F, SUM, big + 5, False), (F, SUM, big, True), (D, SUM, big // 2 + 3, False),
                        (DI, mop.MPI_MAXLOC, 262147, False)]
                for k, (dt, op, count, inplace) in enumerate(runs):
                    c0 = comm.get_param("pipe_calls")
                    ok, msg = case_allreduce(comm, rank, n, dt, op, count, salt + 10 * a + k,
                                             inplace=inplace)
                    if not ok:
                        return False, f"alg {a} slice {sl} {dt.name} {op.name} {count}: {msg}"
                    if n <= 8 and comm.get_param("pipe_calls") != c0 + 1:
                        return False, f"alg {a} slice {sl}: the call did not run pipelined"
            # misaligned: the send buffer 4 B past, the receive buffer 8 B past
            # a 16-B boundary (each rank alike)
            count = big + 3
            xs = [inputs(F, count, r, salt + 77) for r in range(n)]
            exp, _ = orc.allreduce([x.copy() for x in xs], count, SUM.index, F.code)
            raw = np.ascontiguousarray(xs[rank]).view(np.uint8)
            sb = torch.zeros(raw.nbytes + 16, dtype=torch.uint8, device="cuda")
            sb[4:4 + raw.nbytes].copy_(torch.from_numpy(raw.copy()))
            ob = torch.zeros(raw.nbytes + 16, dtype=torch.uint8, device="cuda")
            comm.allreduce(sb[4:], ob[8:], count, F, SUM, blocking=True)
            got = ob[8:8 + raw.nbytes].cpu().numpy().view(np.float32)
            if not np.array_equal(got.view(np.uint32), exp[rank].view(np.uint32)):
                return False, f"alg {a} misaligned: {mismatch(got, exp[rank])}"
        return True, f"{comm.get_param('pipe_calls')} pipelined calls, colocated {comm.get_param('colocated')}"
    finally:
        comm.set_param("pipe_slice", 64 << 10)
        comm.set_param("pipe_passes", 1)
        comm.set_param("algorithm", DEFAULT_ALG[0])


def case_autotune(comm, rank, n, salt, big):
    """param "autotune" (coll/rocm's default): the first 72 large blocking
    allreduces of a size bucket run the 36 candidates twice each
    (push-gather, push-land, staged pull and their pipelined launches x
    1024 / 512 / 256 blocks x non-temporal / plain stores while copy_nt is
    not fixed; a candidate counts its best round), the 72nd decides — on every
    rank alike — and later calls run the choice; every result bit-exact
    against the oracle on dataset R (the fold order is the same whatever
    the scheme), in place too, and a nonblocking allreduce of the same size
    posted meanwhile keeps the default scheme; once decided, a nonblocking
    and a persistent allreduce of that size take the fastest candidate that
    swaps no handles (push-gather / push-land, pipelined or not) with its grid."""
    F, SUM = mop.MPI_FLOAT, mop.MPI_SUM
    count = big + 11
    comm.set_param("autotune", 1)
    try:
        ncalls = 72
        for i in range(ncalls + 3):
            if i == 3:  # a nonblocking call in the middle of the tuning
                xs = [inputs(F, count, r, salt + 50) for r in range(n)]
                exp, _ = orc.allreduce([x.copy() for x in xs], count, SUM.index, F.code)
                sb = to_dev(xs[rank])
                ob = torch.zeros_like(sb)
                req = comm.iallreduce(sb, ob, count, F, SUM)
                req.wait()
                req.free()
                got = ob.cpu().numpy().view(np.float32)
                if not np.array_equal(got.view(np.uint32), exp[rank].view(np.uint32)):
                    return False, "iallreduce during the tuning differs"
            ok, msg = case_allreduce(comm, rank, n, F, SUM, count, salt + i, inplace=(i % 3 == 2))
            if not ok:
                return False, f"call {i}: {msg}"
            state = comm.get_param("autotune_state")
            if state != (1 if i < ncalls - 1 else 2):
                return False, f"call {i}: autotune_state {state}"
        choice = (comm.get_param("autotune_algorithm"), comm.get_param("autotune_blocks"),
                  comm.get_param("autotune_copy_nt"))
        nc = comm.get_param("autotune_ncand")
        if nc != 36:
            return False, f"{nc} candidates with copy_nt not fixed"
        times = [comm.get_param(f"autotune_us{k}") for k in range(nc)]
        # decided: a nonblocking and a persistent allreduce of this size take
        # the fastest push-type candidate (no handle swap) with its grid
        algs = [comm.get_param(f"autotune_alg{k}") for k in range(nc)]
        grids = [comm.get_param(f"autotune_grid{k}") for k in range(nc)]
        nts = [comm.get_param(f"autotune_nt{k}") for k in range(nc)]
        push = [k for k in range(nc) if algs[k] in (2, 3, 4, 5)]
        # (times are whole microseconds: a tie may hide a sub-microsecond order)
        fastest = min(times[k] for k in push)
        wanted = {(algs[k], grids[k], nts[k]) for k in push if times[k] == fastest}
        xs = [inputs(F, count, r, salt + 60) for r in range(n)]
        exp, _ = orc.allreduce([x.copy() for x in xs], count, SUM.index, F.code)
        sb = to_dev(xs[rank])
        ob = torch.zeros_like(sb)
        req = comm.iallreduce(sb, ob, count, F, SUM)
        req.wait()
        req.free()
        took_nb = (comm.get_param("nb_tuned_algorithm"), comm.get_param("nb_tuned_blocks"),
                   comm.get_param("nb_tuned_copy_nt"))
        if not np.array_equal(ob.cpu().numpy().view(np.uint32), exp[rank].view(np.uint32)):
            return False, f"iallreduce after the tuning ({took_nb}) differs"
        ob.zero_()
        plan = comm.allreduce_init(sb, ob, count, F, SUM)
        for _ in range(2):
            plan.start()
            plan.wait()
        plan.free()
        took_plan = (comm.get_param("nb_tuned_algorithm"), comm.get_param("nb_tuned_blocks"),
                     comm.get_param("nb_tuned_copy_nt"))
        if not np.array_equal(ob.cpu().numpy().view(np.uint32), exp[rank].view(np.uint32)):
            return False, f"persistent allreduce after the tuning ({took_plan}) differs"
        if took_nb not in wanted or took_plan != took_nb:
            return False, (f"deferred calls took {took_nb} / {took_plan}, expected the fastest "
                           f"push-type candidate {wanted}")
        everyone = [None] * n
        dist.all_gather_object(everyone, (choice, times, took_nb))
        if any(e != everyone[0] for e in everyone):
            return False, f"ranks chose differently: {everyone}"
        return True, (f"choice {choice}, deferred calls {took_nb}, worst-rank us per "
                      f"candidate {times}")
    finally:
        comm.set_param("autotune", 0)


def case_regrow(comm, rank, n, salt):
    """Landing-buffer growth several times in a row (large scans of rising
    size, an in-place reduce_scatter in between), every result checked."""
    F = mop.MPI_FLOAT
    fails = []  # every rank makes every call, whatever it finds
    for i, count in enumerate((300001, 1100003, 2500007, 9000011)):
        ok, msg = case_scan(comm, rank, n, F, mop.MPI_SUM, count, salt + i)
        if not ok:
            fails.append(f"scan {count}: {msg}")
        ok, msg = case_rs(comm, rank, n, F, mop.MPI_SUM, [count // n + r for r in range(n)],
                          salt + 10 + i, inplace=True)
        if not ok:
            fails.append(f"rs {count}: {msg}")
    return not fails, "; ".join(fails)


def case_free_realloc(comm, rank, n, count, salt):
    """Zero-copy allreduce, then every rank frees its buffers (the caching
    allocator returns the segments: hipFree) and allocates new ones of the
    same size — normally at the freed addresses — and the allreduce runs
    again on new data; three rounds, every result checked.  A peer mapping
    cached from the freed allocation must never serve the new one
    (common_cuda.c:1008-1150 is the reference's handle
    contract)."""
    F = mop.MPI_FLOAT
    msgs = []
    for it in range(3):
        xs = [inputs(F, count, r, salt + it) for r in range(n)]
        exp, _ = orc.allreduce([x.copy() for x in xs], count, mop.MPI_SUM.index, F.code)
        s = to_dev(xs[rank])
        out = torch.zeros_like(s)
        comm.allreduce(s, out, count, F, mop.MPI_SUM, blocking=True)
        got = out.cpu().numpy()[:count * F.extent].view(F.np_dtype)
        if not fields_equal(got, exp[rank]):
            msgs.append(f"round {it}: {mismatch(got, exp[rank])}")
        del s, out
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        dist.barrier()  # every rank freed before anyone allocates again
    msgs.append(f"mappings retired so far (exporter freed them): {comm.get_param('ipc_retired')}, "
                f"recycled handles shadowed: {comm.get_param('recycled_exports')}")
    return len(msgs) == 1, "; ".join(msgs)


def case_persistent(comm, rank, n, dt, op, count, salt, inplace=False, starts=3, expect_kind=None):
    """MPI_Allreduce_init + repeated starts, new data between starts (same
    buffers), other collectives interleaved, no sync between them.
    expect_kind: the path the plan must have taken (Plan.kind)."""
    s = torch.zeros(count * dt.extent, dtype=torch.uint8, device="cuda")
    out = s if inplace else torch.zeros_like(s)
    plan = comm.allreduce_init(coll.IN_PLACE if inplace else s, out, count, dt, op)
    try:
        if expect_kind is not None and plan.kind != expect_kind:
            return False, f"plan kind {plan.kind}, expected {expect_kind}"
        for it in range(starts):
            xs = [inputs(dt, count, r, salt + it) for r in range(n)]
            exp, _ = orc.allreduce([x.copy() for x in xs], count, op.index, dt.code)
            s.copy_(torch.from_numpy(xs[rank].view(np.uint8).copy()).cuda())
            plan.start()
            other = torch.zeros(4096, dtype=torch.uint8, device="cuda")
            comm.bcast(other, 4096, it % n)  # an unrelated collective in between
            plan.wait()
            while not plan.test():
                pass
            torch.cuda.synchronize()
            got = out.cpu().numpy()[:count * dt.extent].view(dt.np_dtype)
            if not fields_equal(got, exp[rank]):
                blocks = []
                for b in range(n):  # which ring blocks are wrong, and from whom
                    off, cnt = coll.block_partition(count, n, b)
                    if not fields_equal(got[off:off + cnt], exp[rank][off:off + cnt]):
                        blocks.append(b)
                return False, f"start {it} mismatch in blocks {blocks}: {mismatch(got, exp[rank])}"
        return True, ""
    finally:
        plan.free()


def case_iallreduce(comm, rank, n, salt, check_nonblocking=True):
    """MPI_Iallreduce: the calls return without waiting for any peer (rank 0
    posts while the others still sleep), five are outstanding at once
    (fused, staged and zero-copy sizes, one in place), a blocking collective
    runs in between, completion by test polling and wait; every result
    checked against the oracle."""
    import time
    F, D, I32 = mop.MPI_FLOAT, mop.MPI_DOUBLE, mop.MPI_INT32_T
    calls = [(F, mop.MPI_SUM, 3001, False), (F, mop.MPI_SUM, 600001, False),
             (I32, mop.MPI_MAX, 20000, False), (D, mop.MPI_SUM, 300003, True),
             (F, mop.MPI_SUM, (1 << 20) + 3, False)]
    prepared = []
    for i, (dt, op, cnt, ip) in enumerate(calls):
        xs = [inputs(dt, cnt, r, salt + i) for r in range(n)]
        exp, _ = orc.allreduce([x.copy() for x in xs], cnt, op.index, dt.code)
        s = to_dev(xs[rank])
        out = s if ip else torch.zeros_like(s)
        prepared.append((dt, op, cnt, ip, s, out, exp[rank]))
    torch.cuda.synchronize()
    dist.barrier()
    if rank != 0:
        time.sleep(0.5)
    t0 = time.perf_counter()
    reqs = [comm.iallreduce(coll.IN_PLACE if ip else s, out, cnt, dt, op)
            for dt, op, cnt, ip, s, out, _ in prepared]
    posted = time.perf_counter() - t0
    msgs = []
    if rank == 0 and check_nonblocking:
        t1 = time.perf_counter()
        early = reqs[1].test()
        tested = time.perf_counter() - t1
        if posted > 0.3 or tested > 0.1 or early:
            msgs.append(f"blocked: post {posted:.3f}s test {tested:.3f}s done-early {early}")
    other = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    comm.bcast(other, 4096, 0)  # a blocking collective with requests outstanding
    while not reqs[0].test():
        pass
    for r in reqs[1:]:
        r.wait()
    torch.cuda.synchronize()
    for r in reqs:
        r.free()
    for i, (dt, op, cnt, ip, s, out, exp) in enumerate(prepared):
        got = out.cpu().numpy()[:cnt * dt.extent].view(dt.np_dtype)
        ok, msg = checked(got, exp)
        if not ok:
            msgs.append(f"call {i}: {msg}")
    return not msgs, "; ".join(msgs)


def case_iallreduce_many(comm, rank, n, salt, calls=12):
    """More zero-copy MPI_Iallreduce calls outstanding than the handle-swap
    ring holds (ShmBoot::kRing = 8) while the peers still sleep: the posts
    launch their oldest deferred calls instead of waiting on their own
    unconsumed tickets, and every result is right."""
    import time
    F = mop.MPI_FLOAT
    cnt = 300007  # 1.2 MB: above small_bytes, so every call swaps handles
    prepared = []
    for i in range(calls):
        xs = [inputs(F, cnt, r, salt + i) for r in range(n)]
        exp, _ = orc.allreduce([x.copy() for x in xs], cnt, mop.MPI_SUM.index, F.code)
        s = to_dev(xs[rank])
        prepared.append((s, torch.zeros_like(s), exp[rank]))
    torch.cuda.synchronize()
    dist.barrier()
    if rank != 0:
        time.sleep(0.5)
    reqs = [comm.iallreduce(s, out, cnt, F, mop.MPI_SUM) for s, out, _ in prepared]
    for r in reqs:
        r.wait()
    torch.cuda.synchronize()
    for r in reqs:
        r.free()
    msgs = []
    for i, (s, out, exp) in enumerate(prepared):
        ok, msg = checked(out.cpu().numpy()[:cnt * 4].view(np.float32), exp)
        if not ok:
            msgs.append(f"call {i}: {msg}")
    return not msgs, "; ".join(msgs)


def case_cross_comm_order(comm, rank, n, salt, stream_per_comm=False, own=False):
    """Two communicators over the same ranks, nonblocking allreduces posted
    in OPPOSITE orders on even and odd ranks (MPI orders collectives per
    communicator only: rank 0 posts A then B while rank 1 posts B then A,
    then every rank waits for both) — at the fused, staged and large sizes,
    on one stream per rank (what coll/rocm's per-thread stream gives) or one
    per communicator; then persistent plans (made in one order) started in
    opposite orders.  A library that launched each call's kernels in post
    order on the shared stream would deadlock here (A's kernel behind B's on
    one rank, B's behind A's on the other)."""
    F = mop.MPI_FLOAT
    comm2 = coll.Communicator.from_torch_distributed(device=comm.device)
    comm2.set_param("timeout_ms", 20000)
    if own:  # what coll/rocm sets (coll_rocm_own_stream): each communicator on a queue of its own
        comm.set_param("own_stream", 1)
        comm2.set_param("own_stream", 1)
    s1 = torch.cuda.Stream()
    s2 = torch.cuda.Stream() if stream_per_comm else s1
    msgs = []
    try:
        for count in (7, 70001, (3 << 20) + 5):
            xs1 = [inputs(F, count, r, salt) for r in range(n)]
            xs2 = [inputs(F, count, r, salt + 1) for r in range(n)]
            e1, _ = orc.allreduce([x.copy() for x in xs1], count, mop.MPI_SUM.index, F.code)
            e2, _ = orc.allreduce([x.copy() for x in xs2], count, mop.MPI_SUM.index, F.code)
            x1, x2 = to_dev(xs1[rank]), to_dev(xs2[rank])
            o1, o2 = torch.zeros_like(x1), torch.zeros_like(x2)
            torch.cuda.synchronize()
            if rank % 2 == 0:
                r1 = comm.iallreduce(x1, o1, count, F, mop.MPI_SUM, stream=s1)
                r2 = comm2.iallreduce(x2, o2, count, F, mop.MPI_SUM, stream=s2)
            else:
                r2 = comm2.iallreduce(x2, o2, count, F, mop.MPI_SUM, stream=s2)
                r1 = comm.iallreduce(x1, o1, count, F, mop.MPI_SUM, stream=s1)
            for r_ in ((r1, r2) if rank % 2 == 0 else (r2, r1)):
                r_.wait()
            torch.cuda.synchronize()
            r1.free()
            r2.free()
            for o, e, what in ((o1, e1, "A"), (o2, e2, "B")):
                ok, msg = checked(o.cpu().numpy()[:count * 4].view(np.float32), e[rank])
                if not ok:
                    msgs.append(f"{count} floats on {what}: {msg}")
            if comm.error() or comm2.error():
                msgs.append(f"{count} floats: device error {comm.error()} / {comm2.error()}")
                break
            # persistent: plans made in the same order everywhere (their init
            # is collective), started in opposite orders, three times
            p1 = comm.allreduce_init(x1, o1, count, F, mop.MPI_SUM)
            p2 = comm2.allreduce_init(x2, o2, count, F, mop.MPI_SUM)
            try:
                for _ in range(3):
                    if rank % 2 == 0:
                        p1.start(stream=s1)
                        p2.start(stream=s2)
                    else:
                        p2.start(stream=s2)
                        p1.start(stream=s1)
                    p1.wait()
                    p2.wait()
                torch.cuda.synchronize()
            finally:
                p1.free()
                p2.free()
            for o, e, what in ((o1, e1, "A (persistent)"), (o2, e2, "B (persistent)")):
                ok, msg = checked(o.cpu().numpy()[:count * 4].view(np.float32), e[rank])
                if not ok:
                    msgs.append(f"{count} floats on {what}: {msg}")
            if comm.error() or comm2.error():
                msgs.append(f"{count} floats (persistent): device error {comm.error()} / {comm2.error()}")
                break
    finally:
        comm2.free()
        if own:
            comm.set_param("own_stream", 0)
    return not msgs, "; ".join(msgs[:3])


def case_cross_comm_grow(comm, rank, n, salt, nring=12):
    """Two fresh communicators (coll/rocm's own_stream), even ranks posting
    A's calls before B's and odd ranks B's before A's, then waiting in the
    opposite order: (1) nonblocking calls whose landing buffer must grow —
    ireduce_scatter_block, iscan, ireduce, iallgather, ibcast past the
    staged size — each growth queued at post and completed from progress
    (a growth at post time is a rendezvous, and two posted
    in opposite orders wait for each other); (2) `nring` ireduces per
    communicator, more tickets than the rendezvous ring holds (a full ring
    queues the rest for progress instead of waiting at the post)."""
    F, I32 = mop.MPI_FLOAT, mop.MPI_INT32_T
    SUM, MAX = mop.MPI_SUM, mop.MPI_MAX
    comms = []
    for _ in range(2):
        cc = coll.Communicator.from_torch_distributed(device=comm.device)
        cc.set_param("timeout_ms", 20000)
        cc.set_param("own_stream", 1)
        comms.append(cc)
    msgs = []

    def prep(ci, kind, count, dt, op, root, sl):
        # inputs, expected results and buffers made before anything is
        # posted: the posts then follow each other at once (a rank busy on
        # the host between posts leaves a peer's launched kernels waiting)
        cc = comms[ci]
        xs = [inputs(dt, count * (n if kind == "rsb" else 1), r, sl) for r in range(n)]
        s = to_dev(xs[rank])
        what = f"comm {ci} {kind} {count} {dt.name}"
        if kind == "rsb":
            exp = orc.reduce_scatter_block([x.copy() for x in xs], count, op.index, dt.code)
            o = torch.zeros(count * dt.extent, dtype=torch.uint8, device="cuda")
            return (lambda: cc.ireduce_scatter_block(s, o, count, dt, op)), o, exp[rank].view(xs[0].dtype), s, what
        if kind == "scan":
            exp = orc.scan([x.copy() for x in xs], count, op.index, dt.code, False)
            o = torch.zeros_like(s)
            return (lambda: cc.iscan(s, o, count, dt, op)), o, exp[rank], s, what
        if kind == "red":
            exp, _ = orc.reduce([x.copy() for x in xs], count, op.index, dt.code, root, False)
            o = torch.zeros_like(s) if rank == root else None
            return (lambda: cc.ireduce(s, o, count, dt, op, root)), o, (exp if rank == root else None), s, what
        if kind == "ag":
            o = torch.zeros(n * count * dt.extent, dtype=torch.uint8, device="cuda")
            return (lambda: cc.iallgather(s, o, count * dt.extent)), o, np.concatenate(xs), s, what
        o = s if rank == root else torch.zeros_like(s)
        return (lambda: cc.ibcast(o, count * dt.extent, root)), o, xs[root], s, what

    def post(prepared):
        torch.cuda.synchronize()  # MPI semantics: the buffers are ready at the call
        return [(go(), o, want, s_, what) for go, o, want, s_, what in prepared]

    def finish(posted, tag):
        for p in reversed(posted):
            p[0].wait()
        torch.cuda.synchronize()
        for r_, o, want, _, what in posted:
            r_.free()
            if want is None:
                continue
            got = o.cpu().numpy().view(np.uint8)[:want.nbytes].view(want.dtype)
            ok, msg = checked(got, want)
            if not ok:
                msgs.append(f"{tag} {what}: {msg}")

    try:
        plan = [("rsb", 300001, F, SUM, 0), ("scan", 400001, I32, MAX, 0),
                ("red", 700001, F, SUM, n - 1), ("ag", 500001, I32, MAX, 0),
                ("bc", 900001, F, SUM, n // 2)]
        order = [(ci, j) for ci in ((0, 1) if rank % 2 == 0 else (1, 0)) for j in range(len(plan))]
        posted = post([prep(ci, *plan[j], salt + 10 * ci + j) for ci, j in order])
        finish(posted, "growth")
        grows = [cc.get_param("landing_deferred_growths") for cc in comms]
        if n > 1 and min(grows) < 1:
            msgs.append(f"no deferred landing growth taken: {grows}")
        order = [(ci, j) for ci in ((0, 1) if rank % 2 == 0 else (1, 0)) for j in range(nring)]
        posted = post([prep(ci, "red", 777 + j, F, SUM, j % n, salt + 100 + 10 * ci + j)
                       for ci, j in order])
        finish(posted, "ring")
        for cc in comms:
            if cc.error():
                msgs.append(f"device error {cc.error()}")
    except Exception:  # reported now: the frees below may wait for peers
        traceback.print_exc()
        sys.stderr.flush()
        raise
    finally:
        for cc in comms:
            cc.free()
    return not msgs, "; ".join(msgs[:3])


def case_cross_comm_random(comm, rank, n, salt, ncomm=3, per_comm=6):
    """Randomized MPI-path ordering (coll/rocm's own_stream): three
    communicators over the same ranks, each with a sequence of nonblocking
    collectives drawn from one seed (the same on every rank: MPI orders a
    communicator's collectives) — iallreduce (up to past the zero-copy
    threshold), ireduce_scatter_block, iallgather, ibcast, ireduce, iscan
    below it — and every rank interleaving the three sequences in its OWN
    random order (legal: MPI orders nothing across communicators), then
    waiting for the requests in its own random order. Every result checked
    against the oracle; a device wait of one communicator queued in front
    of another's kernels would time out here."""
    F, I32 = mop.MPI_FLOAT, mop.MPI_INT32_T
    SUM, MAX = mop.MPI_SUM, mop.MPI_MAX
    plan_rng = np.random.default_rng(SEED + salt)
    comms = []
    for _ in range(ncomm):
        cc = coll.Communicator.from_torch_distributed(device=comm.device)
        cc.set_param("timeout_ms", 20000)
        cc.set_param("own_stream", 1)
        comms.append(cc)
    seqs = []
    for ci in range(ncomm):
        seq = []
        for j in range(per_comm):
            kind = ["ar", "ar", "rsb", "ag", "bc", "red", "scan"][int(plan_rng.integers(7))]
            count = int(plan_rng.choice([1, 777, 20000, 200001, 700001 if kind == "ar" else 60001]))
            dt, op = (F, SUM) if plan_rng.integers(2) else (I32, MAX)
            root = int(plan_rng.integers(n))
            seq.append((kind, count, dt, op, root, salt + 10 * ci + j))
        seqs.append(seq)
    mine = np.random.default_rng(SEED + salt + 1000 * (rank + 1))
    order = [ci for ci in range(ncomm) for _ in range(per_comm)]
    mine.shuffle(order)  # this rank's interleaving of the communicators' sequences
    nxt = [0] * ncomm
    prepared, posted, msgs = [], [], []
    try:
        # inputs, expected results and buffers first: the posts then follow
        # each other at once (a rank busy on the host between posts leaves a
        # peer's launched kernels waiting for it, up to the device timeout)
        for ci in order:
            kind, count, dt, op, root, sl = seqs[ci][nxt[ci]]
            nxt[ci] += 1
            cc = comms[ci]
            xs = [inputs(dt, count * (n if kind == "rsb" else 1), r, sl) for r in range(n)]
            s = to_dev(xs[rank])
            if kind == "ar":
                exp, _ = orc.allreduce([x.copy() for x in xs], count, op.index, dt.code)
                o = torch.zeros_like(s)
                go = functools.partial(cc.iallreduce, s, o, count, dt, op)
                want = exp[rank]
            elif kind == "rsb":
                exp = orc.reduce_scatter_block([x.copy() for x in xs], count, op.index, dt.code)
                o = torch.zeros(count * dt.extent, dtype=torch.uint8, device="cuda")
                go = functools.partial(cc.ireduce_scatter_block, s, o, count, dt, op)
                want = exp[rank].view(xs[0].dtype)
            elif kind == "ag":
                o = torch.zeros(n * count * dt.extent, dtype=torch.uint8, device="cuda")
                go = functools.partial(cc.iallgather, s, o, count * dt.extent)
                want = np.concatenate(xs)
            elif kind == "bc":
                o = s if rank == root else torch.zeros_like(s)
                go = functools.partial(cc.ibcast, o, count * dt.extent, root)
                want = xs[root]
            elif kind == "red":
                exp, _ = orc.reduce([x.copy() for x in xs], count, op.index, dt.code, root, False)
                o = torch.zeros_like(s) if rank == root else None
                go = functools.partial(cc.ireduce, s, o, count, dt, op, root)
                want = exp if rank == root else None
            else:
                exp = orc.scan([x.copy() for x in xs], count, op.index, dt.code, False)
                o = torch.zeros_like(s)
                go = functools.partial(cc.iscan, s, o, count, dt, op)
                want = exp[rank]
            prepared.append((go, o, want, s, f"comm {ci} {kind} {count} {dt.name}"))
        torch.cuda.synchronize()  # MPI semantics: the buffers are ready at the call
        timing = os.environ.get("CROSS_TIMING") == "1"
        for go, o, want, s, what in prepared:
            t0 = time.perf_counter()
            posted.append((go(), o, want, what))
            if timing:
                print(f"[post] {what} {1e3 * (time.perf_counter() - t0):.2f} ms", file=sys.stderr, flush=True)
        wait_order = list(range(len(posted)))
        mine.shuffle(wait_order)
        for i in wait_order:
            t0 = time.perf_counter()
            posted[i][0].wait()
            if timing:
                print(f"[wait] {posted[i][3]} {1e3 * (time.perf_counter() - t0):.2f} ms", file=sys.stderr,
                      flush=True)
        torch.cuda.synchronize()
        for r_, o, want, what in posted:
            r_.free()
            if want is None:
                continue
            got = o.cpu().numpy().view(np.uint8)[:want.nbytes].view(want.dtype)
            ok, msg = checked(got, want)
            if not ok:
                msgs.append(f"{what}: {msg}")
        for cc in comms:
            if cc.error():
                msgs.append(f"device error {cc.error()}")
    except Exception:  # reported now: the frees below may wait for peers
        traceback.print_exc()
        sys.stderr.flush()
        raise
    finally:
        for cc in comms:
            cc.free()
    return not msgs, "; ".join(msgs[:3])


def case_small_marks_two_streams(comm, rank, n, salt, rounds=6):
    """Small allreduces whose fused kernels store their own completion marks
    (blocking, nonblocking and persistent: one flag-page counter slot per
    call in flight): per round, eight MPI_Iallreduce calls
    alternating between two streams, two persistent plans started on
    either stream, and a blocking call, all outstanding together; waited
    in reverse order (requests by test polling for half of them); every
    result bit-exact against the oracle, and the plans' counter slots
    reused round after round."""
    F, I32 = mop.MPI_FLOAT, mop.MPI_INT32_T
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    sizes = [1, 7, 1000, 4099, 16384, 3, 65537 // 4, 2]
    pa_x = [inputs(F, 777, r, salt + 100) for r in range(n)]
    pb_x = [inputs(I32, 5000, r, salt + 101) for r in range(n)]
    pa_s, pb_s = to_dev(pa_x[rank]), to_dev(pb_x[rank])
    pa_o, pb_o = torch.zeros_like(pa_s), torch.zeros_like(pb_s)
    pa_exp, _ = orc.allreduce([x.copy() for x in pa_x], 777, mop.MPI_SUM.index, F.code)
    pb_exp, _ = orc.allreduce([x.copy() for x in pb_x], 5000, mop.MPI_MAX.index, I32.code)
    pa = comm.allreduce_init(pa_s, pa_o, 777, F, mop.MPI_SUM)
    pb = comm.allreduce_init(pb_s, pb_o, 5000, I32, mop.MPI_MAX)
    msgs = []
    try:
        for rd in range(rounds):
            prepared = []
            for i, cnt in enumerate(sizes):
                xs = [inputs(F, cnt, r, salt + 10 * rd + i) for r in range(n)]
                exp, _ = orc.allreduce([x.copy() for x in xs], cnt, mop.MPI_SUM.index, F.code)
                x = to_dev(xs[rank])
                prepared.append((cnt, x, torch.zeros_like(x), exp[rank]))
            bx = [inputs(F, 33, r, salt + 10 * rd + 9) for r in range(n)]
            bexp, _ = orc.allreduce([x.copy() for x in bx], 33, mop.MPI_SUM.index, F.code)
            b_s = to_dev(bx[rank])
            b_o = torch.zeros_like(b_s)
            torch.cuda.synchronize()
            reqs = [comm.iallreduce(x, o, cnt, F, mop.MPI_SUM, stream=(s1 if i % 2 == 0 else s2))
                    for i, (cnt, x, o, _) in enumerate(prepared)]
            pa.start(stream=s1 if rd % 2 == 0 else s2)
            pb.start(stream=s2 if rd % 2 == 0 else s1)
            comm.allreduce(b_s, b_o, 33, F, mop.MPI_SUM, blocking=True)
            pb.wait()
            pa.wait()
            for i in reversed(range(len(reqs))):
                if i % 2:
                    while not reqs[i].test():
                        pass
                else:
                    reqs[i].wait()
            torch.cuda.synchronize()
            for r in reqs:
                r.free()
            for i, (cnt, x, o, exp) in enumerate(prepared):
                ok, msg = checked(o.cpu().numpy()[:cnt * 4].view(np.float32), exp)
                if not ok:
                    msgs.append(f"round {rd} call {i}: {msg}")
            for what, got, exp in (("blocking", b_o.cpu().numpy()[:33 * 4].view(np.float32), bexp[rank]),
                                   ("plan SUM", pa_o.cpu().numpy()[:777 * 4].view(np.float32), pa_exp[rank]),
                                   ("plan MAX", pb_o.cpu().numpy()[:5000 * 4].view(np.int32), pb_exp[rank])):
                ok, msg = checked(got, exp)
                if not ok:
                    msgs.append(f"round {rd} {what}: {msg}")
            if msgs:
                break
    finally:
        pa.free()
        pb.free()
    return not msgs, "; ".join(msgs[:3])


# STRESS_SEED (env): shifts the seeds of the randomized cases (more plans
# than the committed ones, same checks)
STRESS_SEED = int(os.environ.get("STRESS_SEED", "0"))


def case_random_sequence(comm, rank, n, salt, calls=48):
    """A seeded random sequence (the same on every rank) of blocking-form
    collectives enqueued without any wait between them — allreduce, reduce
    (random root, sometimes in place), scan, exscan, reduce_scatter_block,
    reduce_scatter (uneven counts), allgather, bcast (random root) — plus
    MPI_Iallreduce requests waited only at the end; sizes from one element
    to past the zero-copy threshold, fp32 SUM / int32 MAX / fp64 SUM.  Every
    call's per-call resources (scratch halves, landing slots, barrier rows,
    shadows) are reused by the next ones while earlier calls may still run;
    every result is checked against the oracle after one synchronisation."""
    F, D, I32 = mop.MPI_FLOAT, mop.MPI_DOUBLE, mop.MPI_INT32_T
    rng = np.random.default_rng(4242 + salt)
    kinds = ["allreduce", "iallreduce", "reduce", "scan", "exscan", "rsb", "rs", "allgather", "bcast"]
    sizes = [1, 7, 2500, 70001, 300007, (1 << 20) // 4 + 3]
    types = [(F, mop.MPI_SUM), (I32, mop.MPI_MAX), (D, mop.MPI_SUM)]
    checks, reqs, keep = [], [], []
    for c in range(calls):
        kind = kinds[rng.integers(len(kinds))]
        cnt = int(sizes[rng.integers(len(sizes))])
        dt, op = types[rng.integers(len(types))]
        root = int(rng.integers(n))
        inplace = bool(rng.integers(2))
        sl = salt + 100 * c
        if kind in ("allreduce", "iallreduce"):
            xs = [inputs(dt, cnt, r, sl) for r in range(n)]
            exp, _ = orc.allreduce([x.copy() for x in xs], cnt, op.index, dt.code)
            x = to_dev(xs[rank])
            o = torch.zeros_like(x)
            if kind == "allreduce":
                comm.allreduce(x, o, cnt, dt, op)
            else:
                reqs.append(comm.iallreduce(x, o, cnt, dt, op))
            checks.append((c, kind, o, cnt, dt, exp[rank]))
            keep.append(x)
        elif kind == "reduce":
            xs = [inputs(dt, cnt, r, sl) for r in range(n)]
            exp, _ = orc.reduce([x.copy() for x in xs], cnt, op.index, dt.code, root, inplace)
            x = to_dev(xs[rank])
            if rank == root:
                o = x if inplace else torch.zeros_like(x)
                comm.reduce(coll.IN_PLACE if inplace else x, o, cnt, dt, op, root)
                checks.append((c, kind, o, cnt, dt, exp))
            else:
                comm.reduce(x, None, cnt, dt, op, root)
            keep.append(x)
        elif kind in ("scan", "exscan"):
            xs = [inputs(dt, cnt, r, sl) for r in range(n)]
            exp = orc.scan([x.copy() for x in xs], cnt, op.index, dt.code, kind == "exscan")
            x = to_dev(xs[rank])
            o = torch.zeros_like(x)
            (comm.exscan if kind == "exscan" else comm.scan)(x, o, cnt, dt, op)
            if not (kind == "exscan" and rank == 0):
                checks.append((c, kind, o, cnt, dt, exp[rank]))
            keep.append(x)
        elif kind == "rsb":
            rc = max(1, cnt // n)
            xs = [inputs(dt, rc * n, r, sl) for r in range(n)]
            exp = orc.reduce_scatter_block([x.copy() for x in xs], rc, op.index, dt.code)
            x = to_dev(xs[rank])
            o = torch.zeros(rc * dt.extent, dtype=torch.uint8, device="cuda")
            comm.reduce_scatter_block(x, o, rc, dt, op)
            checks.append((c, kind, o, rc, dt, exp[rank]))
            keep.append(x)
        elif kind == "rs":
            rcounts = [max(0, cnt // n + (r * 7 % 5) - 2) for r in range(n)]
            xs = [inputs(dt, sum(rcounts), r, sl) for r in range(n)]
            exp, _ = orc.reduce_scatter([x.copy() for x in xs], rcounts, op.index, dt.code)
            x = to_dev(xs[rank], extra=16)
            o = torch.zeros((rcounts[rank] + 1) * dt.extent, dtype=torch.uint8, device="cuda")
            comm.reduce_scatter(x, o, rcounts, dt, op)
            checks.append((c, kind, o, rcounts[rank], dt, exp[rank]))
            keep.append(x)
        elif kind == "allgather":
            nb = cnt * 4
            xs = [inputs(F, cnt, r, sl) for r in range(n)]
            x = to_dev(xs[rank])
            o = torch.zeros(nb * n, dtype=torch.uint8, device="cuda")
            comm.allgather(x, o, nb)
            checks.append((c, kind, o, cnt * n, F, np.concatenate(xs)))
            keep.append(x)
        else:  # bcast
            nb = cnt * 4
            xs = inputs(F, cnt, root, sl)
            b = to_dev(xs) if rank == root else torch.zeros(nb, dtype=torch.uint8, device="cuda")
            comm.bcast(b, nb, root)
            checks.append((c, kind, b, cnt, F, xs))
    for r_ in reqs:
        r_.wait()
    torch.cuda.synchronize()
    for r_ in reqs:
        r_.free()
    msgs = []
    for c, kind, o, cnt, dt, exp in checks:
        got = o.cpu().numpy()[:cnt * dt.extent].view(dt.np_dtype)
        ok, msg = checked(got, np.asarray(exp).view(dt.np_dtype))
        if not ok:
            msgs.append(f"call {c} {kind} ({cnt} x {dt.name}): {msg}")
    return not msgs, "; ".join(msgs[:3])


def headline_input(rank: int, count: int, salt: int) -> np.ndarray:
    """Dataset E at full size without materialising every rank's vector:
    x_r[i] = (((i * 2654435761 + r * 40503 + salt) mod 2049) - 1024) * 2^-8,
    so sums over any order are exact in fp32 and the expected sum is
    computed rank by rank in int32."""
    i = np.arange(count, dtype=np.int64)
    return ((i * 2654435761 + rank * 40503 + salt) % 2049 - 1024).astype(np.int32)


def case_headline(comm, rank, n, count, salt, algorithm):
    """BASELINE's headline point (256 MiB fp32 SUM allreduce) at full size,
    every element checked exactly (dataset E: exact in any order; the ring
    operand order itself is checked bit-exact on dataset R at the other
    sizes)."""
    F = mop.MPI_FLOAT
    s = torch.from_numpy(headline_input(rank, count, salt).astype(np.float32) * np.float32(2 ** -8)).cuda()
    out = torch.empty_like(s)
    comm.set_param("algorithm", algorithm)
    try:
        comm.allreduce(s, out, count, F, mop.MPI_SUM, blocking=True)
    finally:
        comm.set_param("algorithm", DEFAULT_ALG[0])
    exp = np.zeros(count, dtype=np.int32)
    for r in range(n):
        exp += headline_input(r, count, salt)
    got = out.cpu().numpy()
    ok = np.array_equal(got, exp.astype(np.float32) * np.float32(2 ** -8))
    return ok, "" if ok else mismatch(got, exp.astype(np.float32) * np.float32(2 ** -8))


def case_allgather(comm, rank, n, nbytes, salt, inplace=False):
    xs = [np.random.default_rng(SEED + salt + r).integers(0, 256, nbytes, dtype=np.uint8)
          for r in range(n)]
    exp = np.concatenate(xs)
    out = torch.zeros(nbytes * n, dtype=torch.uint8, device="cuda")
    if inplace:
        out[rank * nbytes:(rank + 1) * nbytes].copy_(torch.from_numpy(xs[rank]))
        comm.allgather(coll.IN_PLACE, out, nbytes, blocking=True)
    else:
        s = to_dev(xs[rank])
        comm.allgather(s, out, nbytes, blocking=True)
    return bool(np.array_equal(out.cpu().numpy(), exp)), ""


def case_bcast(comm, rank, n, nbytes, root, salt, expect_split=None):
    data = np.random.default_rng(SEED + salt).integers(0, 256, nbytes, dtype=np.uint8)
    buf = to_dev(data) if rank == root else torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
    before = comm.get_param("bcast_split")
    comm.bcast(buf, nbytes, root, blocking=True)
    ok = bool(np.array_equal(buf.cpu().numpy()[:nbytes], data))
    split = comm.get_param("bcast_split") - before
    if expect_split is not None and ok and split != expect_split:
        return False, f"scatter+allgather used {split} times, expected {expect_split}"
    return ok, ""


def case_bcast_paths(comm, rank, n, salt):
    """Large bcast as scatter + allgather vs the root pull, sizes around the
    split threshold and the 256-B block rounding, every root."""
    msgs = []
    before = comm.get_param("bcast_split")
    cases = (((4 << 20) - 1, 0), ((4 << 20), None), ((4 << 20) + 257, None),
             ((16 << 20) + 13, None), (n * 256 * 3 + 1 + (4 << 20), None))
    for i, (nbytes, split) in enumerate(cases):
        # above the threshold a refused export (recycled handle) may send a
        # call to the root pull: only the data and "never below" are exact
        for root in range(n):
            ok, msg = case_bcast(comm, rank, n, nbytes, root, salt + 7 * i + root, expect_split=split)
            if not ok:
                msgs.append(f"{nbytes} B root {root}: {msg or 'data differ'}")
    if comm.get_param("bcast_split") == before:
        msgs.append("no bcast ran as scatter + allgather")
    comm.set_param("bcast_split_bytes", 0)
    try:
        ok, msg = case_bcast(comm, rank, n, (16 << 20) + 13, n - 1, salt + 99, expect_split=0)
        if not ok:
            msgs.append(f"root pull, split off: {msg or 'data differ'}")
    finally:
        comm.set_param("bcast_split_bytes", 4 << 20)
    return not msgs, "; ".join(msgs)


def case_copy_nt(comm, rank, n, salt, big):
    """param copy_nt flipped from its default (non-temporal vs plain stores
    in the copy and fold kernels, the 8-GPU bench's A/B): a zero-copy
    allreduce on dataset R bit-exact against the oracle, in place too, and a
    byte-exact allgather and bcast."""
    F, SUM = mop.MPI_FLOAT, mop.MPI_SUM
    msgs = []
    saved = comm.get_param("copy_nt") if comm.get_param("copy_nt_fixed") else -1
    comm.set_param("copy_nt", 1 - comm.get_param("copy_nt"))  # the kind the other cases do not run
    try:
        for i, inplace in enumerate((False, True)):
            ok, msg = case_allreduce(comm, rank, n, F, SUM, big + 13, salt + i, inplace=inplace)
            if not ok:
                msgs.append(f"allreduce{' in place' if inplace else ''}: {msg}")
        ok, msg = case_allgather(comm, rank, n, (big * 4) // n + 9, salt + 5)
        if not ok:
            msgs.append(f"allgather: {msg or 'data differ'}")
        ok, msg = case_bcast(comm, rank, n, big * 4 + 7, n - 1, salt + 6)
        if not ok:
            msgs.append(f"bcast: {msg or 'data differ'}")
    finally:
        comm.set_param("copy_nt", saved)
    return not msgs, "; ".join(msgs)


def case_land_blocking(comm, rank, n, salt, big):
    """param land_blocking = 1 (the 8-GPU bench's A/B): blocking allgather
    and bcast of zero-copy sizes through the landing buffers (stores into the
    peers' landing slots, no descriptor swap) — unaligned block sizes, in
    place, every root — byte-exact, and every such call counted."""
    msgs = []
    small = comm.get_param("small_bytes")
    before = comm.get_param("landing_ag_bcast")
    want = 0
    comm.set_param("land_blocking", 1)
    try:
        for i, (nbytes, inplace) in enumerate((((big * 4) // n + 12, False), ((big * 4) // n + 5, True),
                                               (small + 16 * n + 3, False))):
            ok, msg = case_allgather(comm, rank, n, nbytes, salt + i, inplace)
            want += 1 if nbytes > small else 0
            if not ok:
                msgs.append(f"allgather {nbytes} B{' in place' if inplace else ''}: {msg or 'data differ'}")
        for root in range(n):
            for j, nbytes in enumerate((big * 4 + 3, small + 1, n * 256 * 3 + 1 + small)):
                ok, msg = case_bcast(comm, rank, n, nbytes, root, salt + 10 + 3 * root + j)
                want += 1 if nbytes > small else 0
                if not ok:
                    msgs.append(f"bcast {nbytes} B root {root}: {msg or 'data differ'}")
    finally:
        comm.set_param("land_blocking", 0)
    landed = comm.get_param("landing_ag_bcast") - before
    if comm.get_param("user_ipc") or comm.get_param("force_shadow"):
        want = 0
    if landed != want:
        msgs.append(f"{landed} calls took the landing path, expected {want}")
    return not msgs, "; ".join(msgs)


def case_nonblocking_mix(comm, rank, n, salt, big):
    """MPI_Ireduce_scatter_block / MPI_Iallgather / MPI_Ibcast (and one
    MPI_Iallreduce) posted back to back, staged and zero-copy sizes, in place
    and not, rank 0 posting while the others sleep; every result checked
    against the oracle / the inputs after all are waited on."""
    import time
    F, D = mop.MPI_FLOAT, mop.MPI_DOUBLE
    if rank != 0:
        time.sleep(0.05 * rank)
    todo, keep = [], []
    landed0 = comm.get_param("landing_ag_bcast")
    specs = [("rsb", F, 1001, False), ("rsb", F, big // n + 7, False), ("rsb", D, big // (2 * n) + 3, True),
             ("ag", None, 4099, False), ("ag", None, big * 4 // n + 5, True), ("bc", None, 70001, 0),
             ("bc", None, big * 4 + 3, 1), ("ar", F, big + 1, False), ("rsb", F, 5, True)]
    for i, (kind, dt, cnt, extra) in enumerate(specs):
        if kind == "rsb":
            xs = [inputs(dt, cnt * n, r, salt + i) for r in range(n)]
            exp = orc.reduce_scatter_block([x.copy() for x in xs], cnt, mop.MPI_SUM.index, dt.code)
            s = to_dev(xs[rank])
            if extra:  # in place
                req = comm.ireduce_scatter_block(coll.IN_PLACE, s, cnt, dt, mop.MPI_SUM)
                out = s
            else:
                out = torch.zeros(cnt * dt.extent, dtype=torch.uint8, device="cuda")
                req = comm.ireduce_scatter_block(s, out, cnt, dt, mop.MPI_SUM)
            todo.append((f"rsb{i}", req, out, cnt * dt.extent, exp[rank].view(np.uint8)))
            keep.append(s)
        elif kind == "ag":
            xs = [np.random.default_rng(SEED + salt + i + r).integers(0, 256, cnt, dtype=np.uint8)
                  for r in range(n)]
            out = torch.zeros(cnt * n, dtype=torch.uint8, device="cuda")
            if extra:
                out[rank * cnt:(rank + 1) * cnt].copy_(torch.from_numpy(xs[rank]))
                req = comm.iallgather(coll.IN_PLACE, out, cnt)
            else:
                s = to_dev(xs[rank])
                keep.append(s)
                req = comm.iallgather(s, out, cnt)
            todo.append((f"ag{i}", req, out, cnt * n, np.concatenate(xs)))
        elif kind == "bc":
            root = extra % n
            data = np.random.default_rng(SEED + salt + i).integers(0, 256, cnt, dtype=np.uint8)
            buf = to_dev(data) if rank == root else torch.zeros(cnt, dtype=torch.uint8, device="cuda")
            req = comm.ibcast(buf, cnt, root)
            todo.append((f"bc{i}", req, buf, cnt, data))
        else:
            xs = [inputs(dt, cnt, r, salt + i) for r in range(n)]
            exp, _ = orc.allreduce([x.copy() for x in xs], cnt, mop.MPI_SUM.index, dt.code)
            s = to_dev(xs[rank])
            out = torch.zeros_like(s)
            keep.append(s)
            req = comm.iallreduce(s, out, cnt, dt, mop.MPI_SUM)
            todo.append((f"ar{i}", req, out, cnt * dt.extent, exp[rank].view(np.uint8)))
    bad = []
    for name, req, out, nb, exp in reversed(todo):  # completion order is free
        req.wait()
    torch.cuda.synchronize()
    # the zero-copy-size iallgather and ibcast stored into the landing
    # buffers (no descriptor posted, no host rendezvous) in the staged mode
    landed = comm.get_param("landing_ag_bcast") - landed0
    small = comm.get_param("small_bytes")
    want = sum(1 for kind, _, cnt, _ in specs if kind in ("ag", "bc") and cnt > small)
    if comm.get_param("user_ipc") or comm.get_param("force_shadow"):
        want = 0  # the descriptor-posting path (peers read this rank's buffer or shadow)
    if landed != want:
        bad.append(f"{landed} deferred allgather / bcast calls took the landing path, expected {want}")
    for name, req, out, nb, exp in todo:
        req.free()
        got = out.cpu().numpy()[:nb]
        if not np.array_equal(got, exp[:nb]):
            bad.append(f"{name}: {int(np.count_nonzero(got != exp[:nb]))}/{nb} bytes differ")
    return not bad, "; ".join(bad)


def case_pipelined(comm, rank, n, salt):
    """Back-to-back NON-blocking collectives on one stream (staged scratch
    halves reused every other call, zero-copy mixed in), one sync at the
    end, host-side skew between ranks; every result checked afterwards."""
    import time
    F, I32 = mop.MPI_FLOAT, mop.MPI_INT32_T
    plan = [("ar", F, mop.MPI_SUM, 3001), ("ar", I32, mop.MPI_MAX, 20000),
            ("ag", None, None, 4099), ("ar", F, mop.MPI_SUM, 100003),
            ("bc", None, None, 70001), ("ar", I32, mop.MPI_SUM, 5),
            ("ar", F, mop.MPI_SUM, 600000), ("ar", I32, mop.MPI_BOR, 77),
            ("ag", None, None, 100), ("ar", F, mop.MPI_SUM, 20001)]
    pending = []
    for i, (kind, dt, op, cnt) in enumerate(plan):
        if (i + rank) % 3 == 0:
            time.sleep(0.002 * (rank + 1))
        if kind == "ar":
            xs = [inputs(dt, cnt, r, salt + i) for r in range(n)]
            exp, _ = orc.allreduce([x.copy() for x in xs], cnt, op.index, dt.code)
            s = to_dev(xs[rank])
            out = torch.zeros_like(s)
            comm.allreduce(s, out, cnt, dt, op)
            pending.append((i, out, exp[rank], dt, cnt * dt.extent, s))
        elif kind == "ag":
            xs = [np.random.default_rng(SEED + salt + i + r).integers(0, 256, cnt, dtype=np.uint8)
                  for r in range(n)]
            s = to_dev(xs[rank])
            out = torch.zeros(cnt * n, dtype=torch.uint8, device="cuda")
            comm.allgather(s, out, cnt)
            pending.append((i, out, np.concatenate(xs), None, cnt * n, s))
        else:
            data = np.random.default_rng(SEED + salt + i).integers(0, 256, cnt, dtype=np.uint8)
            root = i % n
            buf = to_dev(data) if rank == root else torch.zeros(cnt, dtype=torch.uint8, device="cuda")
            comm.bcast(buf, cnt, root)
            pending.append((i, buf, data, None, cnt, None))
    torch.cuda.synchronize()
    if comm.error() != 0:
        return False, f"device error {comm.error()}"
    for i, out, exp, dt, nb, _ in pending:
        got = out.cpu().numpy()[:nb]
        if dt is not None:
            ok = fields_equal(got.view(dt.np_dtype), exp)
        else:
            ok = np.array_equal(got, exp)
        if not ok:
            return False, f"step {i} ({plan[i][0]}) mismatch"
    return True, ""


DEFAULT_ALG = [0]  # the communicator's "algorithm" at creation (set in main)


def report(rank, n, obj):
    """One JSON line per case on stdout (read by the test) and, when
    COLL_LOG_DIR is set, appended to a per-rank file there (progress that a
    watchdog on the GPU box can see while the test still runs)."""
    try:  # process resources after the case (diagnostics for IPC open failures)
        obj.setdefault("fds", len(os.listdir("/proc/self/fd")))
    except OSError:
        pass
    line = json.dumps(obj)
    print(line, flush=True)
    d = os.environ.get("COLL_LOG_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, f"coll_n{n}_rank{rank}.jsonl"), "a") as f:
            f.write(line + "\n")


def main():
    rank, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    import faulthandler
    # a hung rank's Python stack, on the launcher's SIGUSR1 (test_coll_gpu.run_ranks)
    faulthandler.register(signal.SIGUSR1, all_threads=True)
    # a rank stuck for a minute prints every thread's stack (then again each
    # minute): a hang names the call it sits in
    faulthandler.dump_traceback_later(60, repeat=True, file=sys.stderr)
    device = int(os.environ.get("OMPI_AMD_DEVICE", "0"))
    torch.cuda.set_device(device)
    dist.init_process_group("gloo", rank=rank, world_size=n)
    comm = coll.Communicator.from_torch_distributed(device=device)
    comm.set_param("timeout_ms", 20000)
    DEFAULT_ALG[0] = comm.get_param("algorithm")
    if os.environ.get("OMPI_AMD_TEST_FORCE_SHADOW") == "1":  # every zero-copy call through shadows
        comm.set_param("force_shadow", 1)
    big = int(os.environ.get("COLL_BIG", 1 << 22))
    # the HSA IPC mode this rank runs under (not forced by the test: the
    # environment's, else the library's load-time default)
    report(rank, n, {"rank": rank, "case": "ipc_mode", "ok": True, "msg": "",
                     "env_at_load": comm.get_param("ipc_mode_legacy_env"),
                     "legacy": comm.get_param("ipc_mode_legacy")})
    F, D, I32, I64, I8, DI = (mop.MPI_FLOAT, mop.MPI_DOUBLE, mop.MPI_INT32_T, mop.MPI_INT64_T,
                              mop.MPI_INT8_T, mop.MPI_DOUBLE_INT)
    H = mop.MPIX_C_FLOAT16
    def user_ipc(fn, alg=0):  # zero-copy on the caller's own buffers (param "user_ipc")
        def run():
            comm.set_param("user_ipc", 1)
            comm.set_param("algorithm", alg)
            try:
                return fn()
            finally:
                comm.set_param("user_ipc", 0)
                comm.set_param("algorithm", DEFAULT_ALG[0])
        return run
    cases = [
        # user_ipc first, before any allocation churn
        ("user_ipc_ar_pull", user_ipc(lambda: case_allreduce(comm, rank, n, F, mop.MPI_SUM, big + 5, 160,
                                                             repeat=2))),
        ("user_ipc_ar_pullpush_inplace", user_ipc(lambda: case_allreduce(
            comm, rank, n, F, mop.MPI_SUM, big, 161, inplace=True), 1)),
        ("user_ipc_ar_push", user_ipc(lambda: case_allreduce(comm, rank, n, D, mop.MPI_SUM, big // 2 + 3,
                                                             162), 2)),
        ("user_ipc_rsb_allgather", user_ipc(lambda: (lambda a, b: (a[0] and b[0], a[1] + b[1]))(
            case_rsb(comm, rank, n, DI, mop.MPI_MAXLOC, big // 8, 163),
            case_allgather(comm, rank, n, (big * 4) // n + 12, 164)))),
        # VERDICT r1 item 1 under user_ipc: every rank frees its buffers
        # (hipFree through empty_cache) and reallocates them between calls
        ("user_ipc_free_realloc", user_ipc(lambda: case_free_realloc(comm, rank, n, big + 11, 165))),
        ("user_ipc_free_realloc_push", user_ipc(lambda: case_free_realloc(comm, rank, n, big + 13, 166),
                                                2)),
        ("ar_sum_f32_1", lambda: case_allreduce(comm, rank, n, F, mop.MPI_SUM, 1, 1)),
        ("allreduce_wait_fused_mark", lambda: case_allreduce_wait(comm, rank, n, 170)),
        ("ar_sum_f32_7", lambda: case_allreduce(comm, rank, n, F, mop.MPI_SUM, 7, 2)),
        ("ar_sum_f32_2499_tree", lambda: case_allreduce(comm, rank, n, F, mop.MPI_SUM, 2499, 3)),
        ("ar_sum_f32_2500_ring", lambda: case_allreduce(comm, rank, n, F, mop.MPI_SUM, 2500, 4)),
        ("ar_sum_f32_12345_staged", lambda: case_allreduce(comm, rank, n, F, mop.MPI_SUM, 12345, 5)),
        ("ar_sum_f32_big_odd", lambda: case_allreduce(comm, rank, n, F, mop.MPI_SUM, big + 5, 6)),
        # ring_segmented on dataset R at every N, past N x 1 MiB (12 MiB + 20 B
        # at N <= 8), under the default scheme and the two others
        ("ar_ring_segmented_R", lambda: case_ring_segmented_R(comm, rank, n,
                                                              max(3 << 20, n << 18) + 5, 170)),
        ("ar_ring_segmented_R_pull", lambda: case_ring_segmented_R(comm, rank, n,
                                                                   max(3 << 20, n << 18) + 9, 171, 0)),
        ("ar_ring_segmented_R_pullpush", lambda: case_ring_segmented_R(
            comm, rank, n, max(3 << 20, n << 18) + 13, 172, 1)),
        ("ar_ring_segmented_R_pushland", lambda: case_ring_segmented_R(
            comm, rank, n, max(3 << 20, n << 18) + 17, 173, 3)),
        ("ar_sum_f32_big", lambda: case_allreduce(comm, rank, n, F, mop.MPI_SUM, big, 7, repeat=3)),
        ("ar_sum_f32_big_inplace",
         lambda: case_allreduce(comm, rank, n, F, mop.MPI_SUM, big, 8, inplace=True)),
        ("ar_sum_f32_small_inplace",
         lambda: case_allreduce(comm, rank, n, F, mop.MPI_SUM, 5000, 9, inplace=True)),
        ("ar_sum_f32_200003_two_shot",
         lambda: case_allreduce(comm, rank, n, F, mop.MPI_SUM, 200003, 67, repeat=2)),
        ("ar_sum_f64_two_shot_inplace",
         lambda: case_allreduce(comm, rank, n, D, mop.MPI_SUM, 60001, 68, inplace=True)),
        ("ar_maxloc_double_int_fused",
         lambda: case_allreduce(comm, rank, n, DI, mop.MPI_MAXLOC, 3001, 69)),
        ("ar_max_f32_specials", lambda: case_allreduce(comm, rank, n, F, mop.MPI_MAX, 300001, 10, "S")),
        ("ar_min_f32_specials_tree", lambda: case_allreduce(comm, rank, n, F, mop.MPI_MIN, 999, 11, "S")),
        ("ar_sum_f64_big", lambda: case_allreduce(comm, rank, n, D, mop.MPI_SUM, big // 2 + 3, 12)),
        ("ar_sum_i32", lambda: case_allreduce(comm, rank, n, I32, mop.MPI_SUM, 1000003, 13)),
        # MPIX_C_FLOAT16 (opal_short_float_t): ring order at the zero-copy size,
        # the fused path, MAX on specials
        ("ar_sum_f16_big", lambda: case_allreduce(comm, rank, n, H, mop.MPI_SUM, 2 * big + 3, 180)),
        ("ar_sum_f16_fused", lambda: case_allreduce(comm, rank, n, H, mop.MPI_SUM, 3001, 181)),
        ("ar_max_f16_specials", lambda: case_allreduce(comm, rank, n, H, mop.MPI_MAX, 70001, 182, "S")),
        ("reduce_sum_f16_big_root1",
         lambda: case_reduce(comm, rank, n, H, mop.MPI_SUM, big + 1, 1 % n, 183)),
        ("ar_band_i64", lambda: case_allreduce(comm, rank, n, I64, mop.MPI_BAND, 77777, 14)),
        ("ar_prod_i8", lambda: case_allreduce(comm, rank, n, I8, mop.MPI_PROD, 50001, 15)),
        ("ar_maxloc_double_int", lambda: case_allreduce(comm, rank, n, DI, mop.MPI_MAXLOC, 262147, 16)),
        ("rsb_maxloc_double_int_small", lambda: case_rsb(comm, rank, n, DI, mop.MPI_MAXLOC, 1000, 17)),
        ("rsb_maxloc_double_int_big", lambda: case_rsb(comm, rank, n, DI, mop.MPI_MAXLOC, big // 8, 18)),
        ("rsb_sum_f32_big", lambda: case_rsb(comm, rank, n, F, mop.MPI_SUM, big // 4 + 1, 19)),
        ("rsb_sum_f32_inplace", lambda: case_rsb(comm, rank, n, F, mop.MPI_SUM, 4097, 20, True)),
        ("allgather_small", lambda: case_allgather(comm, rank, n, 1000, 21)),
        ("allgather_big", lambda: case_allgather(comm, rank, n, (big * 4) // n + 12, 22)),
        ("allgather_inplace", lambda: case_allgather(comm, rank, n, 65536, 23, True)),
        ("bcast_small_root0", lambda: case_bcast(comm, rank, n, 777, 0, 24)),
        ("bcast_big_rootlast", lambda: case_bcast(comm, rank, n, big * 4 + 3, n - 1, 25)),
        ("bcast_scatter_allgather", lambda: case_bcast_paths(comm, rank, n, 26)),
        ("allgather_bcast_land_blocking", lambda: case_land_blocking(comm, rank, n, 27, big)),
        ("copy_nt_stores", lambda: case_copy_nt(comm, rank, n, 28, big)),
        ("pipelined_nonblocking", lambda: case_pipelined(comm, rank, n, 26)),
        # reduce: staged (linear / binomial / binary by size) and zero-copy
        ("reduce_sum_f32_100_rootlast",
         lambda: case_reduce(comm, rank, n, F, mop.MPI_SUM, 100, n - 1, 40)),
        ("reduce_sum_f32_3000_root1",
         lambda: case_reduce(comm, rank, n, F, mop.MPI_SUM, 3000, 1, 41)),
        ("reduce_sum_f32_6000_root1_inplace",
         lambda: case_reduce(comm, rank, n, F, mop.MPI_SUM, 6000, 1, 42, inplace=True)),
        ("reduce_max_f32_specials_3000_inplace",
         lambda: case_reduce(comm, rank, n, F, mop.MPI_MAX, 3000, 0, 43, True, "S")),
        ("reduce_sum_f32_big_root2",
         lambda: case_reduce(comm, rank, n, F, mop.MPI_SUM, big + 3, 2, 44)),
        ("reduce_sum_f64_big_root0_inplace",
         lambda: case_reduce(comm, rank, n, D, mop.MPI_SUM, big // 2 + 1, 0, 45, inplace=True)),
        ("reduce_maxloc_double_int_big",
         lambda: case_reduce(comm, rank, n, DI, mop.MPI_MAXLOC, big // 8 + 7, n - 1, 46)),
        # rsb in the binomial / binary range of the tuned reduce decision
        ("rsb_sum_f32_mid", lambda: case_rsb(comm, rank, n, F, mop.MPI_SUM, 1500, 47)),
        ("rsb_sum_f32_small", lambda: case_rsb(comm, rank, n, F, mop.MPI_SUM, 300, 48)),
        ("rsb_max_f32_mid_specials",
         lambda: case_rsb_kind(comm, rank, n, F, mop.MPI_MAX, 1000, 49, "S")),
        # reduce_scatter: recursive halving (small / pof2 <= 256 KiB) and ring,
        # uneven counts with an empty block, staged and zero-copy, in place
        ("rs_sum_f32_small", lambda: case_rs(comm, rank, n, F, mop.MPI_SUM,
                                             [300 + 7 * r if r != 1 else 0 for r in range(n)], 56)),
        ("rs_sum_f32_mid", lambda: case_rs(comm, rank, n, F, mop.MPI_SUM,
                                           [9000 + 13 * r for r in range(n)], 57)),
        ("rs_max_f32_specials", lambda: case_rs(comm, rank, n, F, mop.MPI_MAX,
                                                [5000 + r for r in range(n)], 58, kind="S")),
        ("rs_sum_f32_big", lambda: case_rs(comm, rank, n, F, mop.MPI_SUM,
                                           [big // n + 11 * r for r in range(n)], 59)),
        ("rs_sum_f64_big_inplace", lambda: case_rs(comm, rank, n, D, mop.MPI_SUM,
                                                   [big // (2 * n) + r for r in range(n)], 70,
                                                   inplace=True)),
        ("rsb_sum_f32_big_inplace",
         lambda: case_rsb(comm, rank, n, F, mop.MPI_SUM, big // 4 + 3, 71, True)),
        # scan / exscan: staged and landing paths, in place
        ("scan_sum_f32_small", lambda: case_scan(comm, rank, n, F, mop.MPI_SUM, 5000, 50)),
        ("scan_sum_f32_big", lambda: case_scan(comm, rank, n, F, mop.MPI_SUM, big + 1, 51)),
        ("scan_sum_f32_big_inplace",
         lambda: case_scan(comm, rank, n, F, mop.MPI_SUM, big, 52, inplace=True)),
        ("exscan_sum_f64_small", lambda: case_scan(comm, rank, n, D, mop.MPI_SUM, 999, 53, True)),
        ("exscan_max_i32_big", lambda: case_scan(comm, rank, n, I32, mop.MPI_MAX, big, 54, True)),
        ("landing_regrow", lambda: case_regrow(comm, rank, n, 90)),
        ("zero_copy_free_realloc", lambda: case_free_realloc(comm, rank, n, big + 7, 92)),
        ("exscan_prod_i8_inplace",
         lambda: case_scan(comm, rank, n, I8, mop.MPI_PROD, 70001, 55, True, True)),
    ]
    cases += [
        ("zero_counts_every_entry_point", lambda: case_zero_counts(comm, rank, n, 96)),
        ("autotune_large_allreduce", lambda: case_autotune(comm, rank, n, 97, big)),
        ("pipelined_schemes", lambda: case_pipe(comm, rank, n, 120, big)),
        ("iallreduce_mixed", lambda: case_iallreduce(comm, rank, n, 90)),
        ("iallreduce_many_outstanding", lambda: case_iallreduce_many(comm, rank, n, 94)),
        ("small_marks_two_streams", lambda: case_small_marks_two_streams(comm, rank, n, 700)),
        ("random_sequence", lambda: case_random_sequence(comm, rank, n, 800 + STRESS_SEED)),
        ("random_sequence_user_ipc", user_ipc(lambda: case_random_sequence(comm, rank, n, 900 + STRESS_SEED))),
        ("persistent_small", lambda: case_persistent(comm, rank, n, F, mop.MPI_SUM, 3001, 80)),
        ("persistent_mid_inplace",
         lambda: case_persistent(comm, rank, n, D, mop.MPI_SUM, 70001, 81, inplace=True)),
        ("persistent_big", lambda: case_persistent(comm, rank, n, F, mop.MPI_SUM, big + 3, 82,
                                                   expect_kind=0 if DEFAULT_ALG[0] == 2 else None)),
        ("user_ipc_persistent_push_kind", user_ipc(lambda: case_persistent(
            comm, rank, n, F, mop.MPI_SUM, big + 3, 86, expect_kind=3), 2)),
        ("persistent_big_inplace",
         lambda: case_persistent(comm, rank, n, F, mop.MPI_MAX, big, 83, inplace=True)),
    ]
    # zero-copy allreduce under the two push schemes (param "algorithm")
    # the schemes other than the library default (which every unscoped case runs)
    for alg in [a for a in (0, 1, 2, 3, 4, 5, 6) if a != DEFAULT_ALG[0]]:
        def with_alg(fn, a=alg):
            def run():
                comm.set_param("algorithm", a)
                try:
                    return fn()
                finally:
                    comm.set_param("algorithm", DEFAULT_ALG[0])
            return run
        cases += [
            (f"alg{alg}_ar_sum_f32_big",
             with_alg(lambda: case_allreduce(comm, rank, n, F, mop.MPI_SUM, big, 60, repeat=2))),
            (f"alg{alg}_ar_sum_f32_big_odd",
             with_alg(lambda: case_allreduce(comm, rank, n, F, mop.MPI_SUM, big + 5, 61))),
            (f"alg{alg}_ar_sum_f32_big_inplace",
             with_alg(lambda: case_allreduce(comm, rank, n, F, mop.MPI_SUM, big, 62, inplace=True))),
            (f"alg{alg}_ar_sum_f64_big",
             with_alg(lambda: case_allreduce(comm, rank, n, D, mop.MPI_SUM, big // 2 + 3, 63))),
            (f"alg{alg}_ar_maxloc_double_int",
             with_alg(lambda: case_allreduce(comm, rank, n, DI, mop.MPI_MAXLOC, 262147, 64))),
            (f"alg{alg}_ar_max_f32_specials",
             with_alg(lambda: case_allreduce(comm, rank, n, F, mop.MPI_MAX, 300001, 65, "S"))),
            (f"alg{alg}_pipelined_nonblocking", with_alg(lambda: case_pipelined(comm, rank, n, 66))),
            (f"alg{alg}_iallreduce_mixed",
             with_alg(lambda: case_iallreduce(comm, rank, n, 91, check_nonblocking=False))),
            (f"alg{alg}_persistent_big",
             with_alg(lambda: case_persistent(comm, rank, n, F, mop.MPI_SUM, big + 1, 84))),
            (f"alg{alg}_free_realloc",
             with_alg(lambda: case_free_realloc(comm, rank, n, big + 9, 93))),
            (f"alg{alg}_persistent_big_inplace",
             with_alg(lambda: case_persistent(comm, rank, n, D, mop.MPI_SUM, big // 2, 85,
                                              inplace=True))),
        ]
    if os.environ.get("COLL_HEADLINE"):  # full-size headline only (tests/test_coll_gpu.py)
        hc = int(os.environ["COLL_HEADLINE"])
        cases = [(f"headline_alg{a}", lambda a=a: case_headline(comm, rank, n, hc, 95 + a, a))
                 for a in (0, 1, 2, 3, 4, 5, 6)]
    def shadowed_nb(fn):  # the export fallback for the nonblocking forms
        def run():
            comm.set_param("force_shadow", 1)
            try:
                return fn()
            finally:
                comm.set_param("force_shadow", 0)
        return run
    # coll/tuned's forced allreduce algorithms (1 basic_linear, 2 nonoverlapping,
    # 3 recursive doubling, 4 ring, 5 segmented ring, 6 Rabenseifner), every path
    if not os.environ.get("COLL_HEADLINE"):
        for alg in range(1, 7):
            for sz, tag in ((5003, "staged"), (200003, "two_shot"), (big + 3, "zero_copy")):
                cases.append((f"forced{alg}_sum_f32_{tag}",
                              lambda a=alg, c=sz: case_forced(comm, rank, n, a, F, mop.MPI_SUM, c, 120 + a)))
            cases.append((f"forced{alg}_sum_f64_big_inplace",
                          lambda a=alg: case_forced(comm, rank, n, a, D, mop.MPI_SUM, big // 2 + 1, 130 + a,
                                                    inplace=True)))
        cases += [
            ("forced6_maxloc_pairs", lambda: case_forced(comm, rank, n, 6, DI, mop.MPI_MAXLOC, 70001, 140)),
            ("forced6_max_specials_tiny", lambda: case_forced(comm, rank, n, 6, F, mop.MPI_MAX, 3, 141)),
            ("forced6_nonblocking", lambda: case_forced(comm, rank, n, 6, F, mop.MPI_SUM, big + 1, 142,
                                                        how="nonblocking")),
            ("forced6_persistent", lambda: case_forced(comm, rank, n, 6, F, mop.MPI_SUM, big + 1, 143,
                                                       how="persistent")),
            ("forced2_persistent_inplace", lambda: case_forced(comm, rank, n, 2, F, mop.MPI_SUM, 300001, 144,
                                                               inplace=True, how="persistent")),
            ("forced2_nonblocking", lambda: case_forced(comm, rank, n, 2, F, mop.MPI_SUM, big + 1, 145,
                                                        how="nonblocking")),
            ("forced2_blocking_inplace_f32", lambda: case_forced(comm, rank, n, 2, F, mop.MPI_SUM, 300001,
                                                                 144, inplace=True)),
            ("forced4_persistent_inplace", lambda: case_forced(comm, rank, n, 4, F, mop.MPI_SUM, 300001, 144,
                                                               inplace=True, how="persistent")),
            ("persistent_inplace_sum_f32", lambda: case_persistent(comm, rank, n, F, mop.MPI_SUM, 300001, 146,
                                                                   inplace=True)),
            ("nonblocking_rsb_ag_bcast", lambda: case_nonblocking_mix(comm, rank, n, 150, big)),
            ("nonblocking_reduce_scan_rs", lambda: case_nb_reduce_scan_rs(comm, rank, n, 180, big)),
            ("persistent_rsb_allgather_bcast", lambda: case_persistent_rsb_ag_bcast(comm, rank, n, 190, big)),
            ("persistent_reduce_scan_rs", lambda: case_persistent_reduce_scan_rs(comm, rank, n, 200, big)),
            ("nonblocking_rsb_ag_bcast_shadow",
             shadowed_nb(lambda: case_nonblocking_mix(comm, rank, n, 160, big))),
        ]
    # the export fallback (hipIpcGetMemHandle refused): every zero-copy path
    # through the communicator's shadow buffers ("force_shadow")
    def shadowed(fn):
        def run():
            comm.set_param("force_shadow", 1)
            try:
                ok, msg = fn()
            finally:
                comm.set_param("force_shadow", 0)
            return ok, msg
        return run
    if not os.environ.get("COLL_HEADLINE"):
        cases += [
            ("shadow_ar_pull", shadowed(lambda: case_allreduce(comm, rank, n, F, mop.MPI_SUM, big + 5, 100))),
            ("shadow_ar_pull_inplace",
             shadowed(lambda: case_allreduce(comm, rank, n, D, mop.MPI_SUM, big // 2 + 1, 101, inplace=True))),
            ("shadow_ar_pullpush", shadowed(with_alg(lambda: case_allreduce(comm, rank, n, F, mop.MPI_SUM,
                                                                            big + 3, 102), 1))),
            ("shadow_ar_push_inplace", shadowed(with_alg(lambda: case_allreduce(
                comm, rank, n, F, mop.MPI_SUM, big, 103, inplace=True), 2))),
            ("shadow_reduce_root_inplace",
             shadowed(lambda: case_reduce(comm, rank, n, F, mop.MPI_SUM, big + 3, 1, 104, inplace=True))),
            ("shadow_reduce_root_last",
             shadowed(lambda: case_reduce(comm, rank, n, DI, mop.MPI_MAXLOC, big // 8 + 7, n - 1, 105))),
            ("shadow_rsb", shadowed(lambda: case_rsb(comm, rank, n, F, mop.MPI_SUM, big // 4 + 1, 106))),
            ("shadow_rs_inplace", shadowed(lambda: case_rs(comm, rank, n, D, mop.MPI_SUM,
                                                           [big // (2 * n) + r for r in range(n)], 107,
                                                           inplace=True))),
            ("shadow_allgather_inplace", shadowed(lambda: case_allgather(comm, rank, n, (big * 4) // n + 12,
                                                                         108, True))),
            ("shadow_bcast", shadowed(lambda: case_bcast(comm, rank, n, big * 4 + 3, n - 1, 109))),
            ("shadow_iallreduce", shadowed(lambda: case_iallreduce(comm, rank, n, 110,
                                                                   check_nonblocking=False))),
            ("shadow_persistent", shadowed(lambda: case_persistent(comm, rank, n, F, mop.MPI_SUM, big + 1, 111))),
            ("shadow_persistent_push_inplace", shadowed(with_alg(lambda: case_persistent(
                comm, rank, n, D, mop.MPI_SUM, big // 2, 112, inplace=True), 2))),
        ]
    only = os.environ.get("COLL_CASES")
    # the MPI path (coll/rocm's own_stream): opposite-order nonblocking and
    # persistent calls on two communicators complete
    if not os.environ.get("COLL_HEADLINE"):
        cases += [("cross_comm_order_own_stream", lambda: case_cross_comm_order(comm, rank, n, 192, own=True)),
                  ("cross_comm_grow_own_stream", lambda: case_cross_comm_grow(comm, rank, n, 195)),
                  ("cross_comm_random_own_stream", lambda: case_cross_comm_random(comm, rank, n, 193 + STRESS_SEED)),
                  ("cross_comm_random_own_stream_b",
                   lambda: case_cross_comm_random(comm, rank, n, 194 + STRESS_SEED))]
    if only and "cross_comm" in only:
        # opt-in: the known limitation of DESIGN.md §8 item 9 (device-side
        # waits across communicators posted in opposite orders time out)
        cases += [("cross_comm_order_one_stream", lambda: case_cross_comm_order(comm, rank, n, 190)),
                  ("cross_comm_order_two_streams",
                   lambda: case_cross_comm_order(comm, rank, n, 191, True))]
    # COLL_FROM / COLL_UNTIL: a contiguous slice of the list (history-dependent failures)
    first, last = os.environ.get("COLL_FROM"), os.environ.get("COLL_UNTIL")
    if first or last:
        names = [c[0] for c in cases]
        lo = names.index(first) if first else 0
        hi = names.index(last) + 1 if last else len(names)
        cases = cases[lo:hi]
        only = None
    import threading
    cur = {"name": None, "t0": 0.0}

    def watchdog():  # a case running long prints the barrier progress record
        import time
        while True:
            time.sleep(20)
            name, t0 = cur["name"], cur["t0"]
            if name is None or time.time() - t0 < 40:
                continue
            try:
                keys = ["epoch", "dbg_entered", "dbg_left"] + [f"dbg_seen{p}" for p in range(n)]
                vals = {k: comm.get_param(k) for k in keys}
            except Exception as e:  # noqa: BLE001 (debug record off)
                vals = {"error": str(e)}
            print(f"[watchdog] case {name} running {time.time() - t0:.0f} s: {vals}",
                  file=sys.stderr, flush=True)

    threading.Thread(target=watchdog, daemon=True).start()
    ok_all = True
    for name, fn in cases:
        if only and name not in only.split(","):
            continue
        print(f"[case {name}] epoch {comm.get_param('epoch')}", file=sys.stderr, flush=True)
        import time as _t
        cur["name"], cur["t0"] = name, _t.time()
        try:
            ok, msg = fn()
        except Exception as e:  # report and stop: later cases would hang
            ok, msg = False, (f"[epoch {comm.get_param('epoch')}] {type(e).__name__}: {e} "
                              f"{traceback.format_exc()[-400:]}")
            report(rank, n, {"rank": rank, "case": name, "ok": ok, "msg": msg})
            ok_all = False
            break
        # barrier epochs diverge when ranks launched different device work
        report(rank, n, {"rank": rank, "case": name, "ok": bool(ok), "msg": msg,
                         "state": {k: comm.get_param(k) for k in (
                             "epoch", "shadowed", "recycled_exports", "exports_new", "imports_new",
                             "imports", "landing_bytes", "boot_calls", "memcpy_token_mismatch",
                             "ipc_opens", "ipc_closes", "ipc_shared", "ipc_retired", "ipc_live", "ipc_close_watermark",
                             "ipc_refusals")}})
        ok_all &= bool(ok)
    # zero-copy disabled: everything staged through the scratch
    if ok_all and not only and not os.environ.get("COLL_HEADLINE"):
        comm.set_param("zero_copy", 0)
        ok, msg = case_allreduce(comm, rank, n, F, mop.MPI_SUM, 1 << 20, 30)
        report(rank, n, {"rank": rank, "case": "ar_staged_only", "ok": bool(ok), "msg": msg})
        ok_all &= bool(ok)
    torch.cuda.synchronize()
    comm.free()
    dist.destroy_process_group()
    sys.exit(0 if ok_all else 1)


if __name__ == "__main__":
    main()
