"""One rank of the multi-process point-to-point and one-sided tests
(tests/test_p2p_osc_gpu.py).

Launched N times with RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT and
OMPI_AMD_DEVICE.  A gloo group broadcasts the communicator name and
separates the cases; all data moves through libompi_amd.so on device
buffers.  Expected results come from the deterministic per-rank inputs and,
for accumulates, from the CPU oracle's op/base restatement applied in the
target's order.  One JSON line per case; exit 0 only if all passed.
"""
import faulthandler
import ctypes
import functools
import json
import os
import sys
import signal
import time
import traceback

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from ompi_amd import _lib, coll, osc, pml  # noqa: E402
from ompi_amd import op as mop  # noqa: E402
from oracle import oracle as orc  # noqa: E402

SEED = 20261015
STREAM = None  # a dedicated stream (a NULL stream argument means hipStreamPerThread)


def payload(rank: int, salt: int, nbytes: int) -> np.ndarray:
    return np.random.default_rng(SEED + 7919 * salt + rank).integers(0, 256, nbytes, dtype=np.uint8)


def dev(a: np.ndarray, extra: int = 0) -> torch.Tensor:
    raw = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
    t = zeros(raw.nbytes + extra)
    with torch.cuda.stream(STREAM):
        t[:raw.nbytes].copy_(torch.from_numpy(raw.copy()))
    STREAM.synchronize()
    return t


def zeros(nbytes: int) -> torch.Tensor:
    """A zeroed device buffer, filled before any stream uses it (torch fills
    on its current stream, which does not order against STREAM)."""
    t = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    return t


def host(t: torch.Tensor) -> np.ndarray:
    STREAM.synchronize()
    return t.cpu().numpy()


def eq(got: np.ndarray, exp: np.ndarray, what: str):
    g = np.ascontiguousarray(got).view(np.uint8).reshape(-1)
    e = np.ascontiguousarray(exp).view(np.uint8).reshape(-1)
    if g.shape == e.shape and np.array_equal(g, e):
        return True, ""
    if g.shape != e.shape:
        return False, f"{what}: {g.shape} vs {e.shape} bytes"
    bad = np.flatnonzero(g != e)
    return False, f"{what}: {bad.size} bytes differ, first at {bad[:4].tolist()}"


# ----------------------------------------------------------------- p2p cases
def case_ring(comm, rank, n, nbytes, salt, soff=0, roff=0):
    """sendrecv around the ring (MPI_Sendrecv to rank+1 from rank-1), with
    byte offsets into both buffers."""
    nxt, prv = (rank + 1) % n, (rank - 1) % n
    s = dev(payload(rank, salt, nbytes), extra=soff + 8)
    if soff:
        s = dev(np.concatenate([np.zeros(soff, np.uint8), payload(rank, salt, nbytes)]), extra=8)
    r = zeros(nbytes + roff + 8)
    st = pml.sendrecv(comm, s[soff:soff + nbytes] if nbytes else s, nxt, 100 + salt,
                      r[roff:roff + nbytes] if nbytes else r, prv, 100 + salt,
                      sbytes=nbytes, rbytes=nbytes, stream=STREAM)
    if (st.source, st.tag, st.bytes) != (prv, 100 + salt, nbytes):
        return False, f"status {st}"
    got = host(r)
    ok, msg = eq(got[roff:roff + nbytes], payload(prv, salt, nbytes), "payload")
    if ok and (got[:roff].any() or got[roff + nbytes:].any()):
        return False, "bytes outside the receive window were written"
    return ok, msg


def case_aged_buffer_staged(comm, rank, n, salt, nbytes=(8 << 20) + 12):
    """p2p_user_ipc = 1 with the send buffer older than an IPC close of this
    process (the test hook p2p_age_all makes every buffer so; pml harness
    section 9 makes it happen for real): ROCm 7.2 may refuse to export such
    an allocation, so it is never offered for export — the
    message goes through a library stage, byte-exact, counted in
    p2p_unsafe_sends and p2p_staged_sends."""
    comm.set_param("p2p_user_ipc", 1)
    comm.set_param("p2p_age_all", 1)
    try:
        u0, s0 = comm.get_param("p2p_unsafe_sends"), comm.get_param("p2p_staged_sends")
        ok, msg = case_ring(comm, rank, n, nbytes, salt, soff=4, roff=8)
        u1, s1 = comm.get_param("p2p_unsafe_sends"), comm.get_param("p2p_staged_sends")
    finally:
        comm.set_param("p2p_age_all", 0)
        comm.set_param("p2p_user_ipc", 0)
    if ok and (u1 - u0 != 1 or s1 - s0 != 1):
        return False, f"aged sends {u1 - u0}, staged sends {s1 - s0} (want 1, 1)"
    return ok, msg


def case_stage_cap_aged(comm, rank, n, salt, nbytes=(4 << 20) + 8, k=8):
    """Staged sends (p2p_user_ipc = 0) with the send-stage pool at its cap
    (p2p_stage_mib 8, k outstanding sends of 4 MiB + 8 each way) and every
    buffer older than an IPC close (test hook p2p_age_all): a send that finds
    no free stage must not go out from the buffer itself (it may not be
    exportable) nor wait for the receiver — it takes a stage past the cap;
    every message byte-exact, p2p_unsafe_sends counts the ones past the cap.
    (the fallback to exporting the user buffer.)"""
    nxt, prv = (rank + 1) % n, (rank - 1) % n
    cap0 = comm.get_param("p2p_stage_mib")
    comm.set_param("p2p_stage_mib", 8)
    comm.set_param("p2p_age_all", 1)
    try:
        u0, d0 = comm.get_param("p2p_unsafe_sends"), comm.get_param("p2p_direct_sends")
        srcs = [dev(payload(rank, salt + j, nbytes)) for j in range(k)]
        sreqs = [pml.isend(comm, srcs[j], nxt, 40 + j, stream=STREAM) for j in range(k)]
        rbufs = [zeros(nbytes) for _ in range(k)]
        rreqs = [pml.irecv(comm, rbufs[j], prv, 40 + j, stream=STREAM) for j in range(k)]
        for j in range(k):
            rreqs[j].wait()
            ok, msg = eq(host(rbufs[j]), payload(prv, salt + j, nbytes), f"message {j}")
            if not ok:
                return ok, msg
            rreqs[j].free()
        for rq in sreqs:
            rq.wait()
            rq.free()
        u1, d1 = comm.get_param("p2p_unsafe_sends"), comm.get_param("p2p_direct_sends")
    finally:
        comm.set_param("p2p_age_all", 0)
        comm.set_param("p2p_stage_mib", cap0)
    if d1 != d0 or u1 - u0 < 1:
        return False, f"direct sends {d1 - d0} (want 0), past-the-cap sends {u1 - u0} (want >= 1)"
    return True, ""


def case_tags_out_of_order(comm, rank, n, salt):
    """Three sends with tags 5, 6, 7; receives posted as 7, 5, 6."""
    nxt, prv = (rank + 1) % n, (rank - 1) % n
    sizes = {5: 1000, 6: 70001, 7: 3}
    sends = {t: dev(payload(rank, salt + t, b)) for t, b in sizes.items()}
    reqs = [pml.isend(comm, sends[t], nxt, t, stream=STREAM) for t in (5, 6, 7)]
    rbufs = {t: zeros(sizes[t]) for t in sizes}
    rreqs = {t: pml.irecv(comm, rbufs[t], prv, t, stream=STREAM) for t in (7, 5, 6)}
    for t, rq in rreqs.items():
        st = rq.wait()
        if st.tag != t or st.source != prv or st.bytes != sizes[t]:
            return False, f"tag {t}: status {st}"
        ok, msg = eq(host(rbufs[t]), payload(prv, salt + t, sizes[t]), f"tag {t}")
        if not ok:
            return ok, msg
        rq.free()
    for rq in reqs:
        rq.wait()
        rq.free()
    return True, ""


def case_same_tag_order(comm, rank, n, salt, k=40):
    """k messages with one tag: received in sending order (non-overtaking)."""
    nxt, prv = (rank + 1) % n, (rank - 1) % n
    sends = [dev(payload(rank, salt + i, 257 + i)) for i in range(k)]
    reqs = [pml.isend(comm, sends[i], nxt, 9, stream=STREAM) for i in range(k)]
    fails = []
    for i in range(k):
        r = zeros(257 + i)
        st = pml.recv(comm, r, prv, 9, stream=STREAM)
        if st.bytes != 257 + i:
            fails.append(f"msg {i}: {st.bytes} bytes")
            continue
        ok, msg = eq(host(r), payload(prv, salt + i, 257 + i), f"msg {i}")
        if not ok:
            fails.append(msg)
    for rq in reqs:
        rq.wait()
        rq.free()
    return not fails, "; ".join(fails[:3])


def case_ring_wraps(comm, rank, n, salt, k=150):
    """k isends to the next rank before any receive is posted, alternating
    eager (<= 4 KiB) and staged sizes from device buffers: the 64-slot
    ring wraps twice, so eager cells, their flag words (seq + 1) and the
    staged copies' completion counters are reused while earlier messages'
    copy kernels may still run (a sender waits for its slot's FIN).  The
    receives come in sending order; every byte checked."""
    nxt, prv = (rank + 1) % n, (rank - 1) % n
    sizes = [3001 if i % 2 == 0 else 96 * 1024 + 7 * i for i in range(k)]
    sends = [dev(payload(rank, salt + i, b)) for i, b in enumerate(sizes)]
    reqs = []
    fails = []
    got = 0
    rbufs = [zeros(b) for b in sizes]
    rreqs = []
    for i in range(k):
        reqs.append(pml.isend(comm, sends[i], nxt, 11, stream=STREAM))
        # keep receives ~48 behind: the 65th unmatched send would wait for a slot
        if i >= 48:
            rreqs.append(pml.irecv(comm, rbufs[got], prv, 11, stream=STREAM))
            got += 1
    while got < k:
        rreqs.append(pml.irecv(comm, rbufs[got], prv, 11, stream=STREAM))
        got += 1
    for i, rq in enumerate(rreqs):
        try:
            st = rq.wait()
        except _lib.OmpiAmdError as e:
            return False, f"receive {i} of {k} ({sizes[i]} B): {e}"
        if st.bytes != sizes[i]:
            fails.append(f"msg {i}: {st.bytes} bytes")
            continue
        ok, msg = eq(host(rbufs[i]), payload(prv, salt + i, sizes[i]), f"msg {i}")
        if not ok:
            fails.append(msg)
        rq.free()
    for rq in reqs:
        rq.wait()
        rq.free()
    return not fails, "; ".join(fails[:3])


# STRESS_SEED (env): shifts the seeds of the randomized cases (more plans
# than the committed ones, same checks)
STRESS_SEED = int(os.environ.get("STRESS_SEED", "0"))


def case_random_channels(comm, rank, n, salt, per_rank=36, wild=0.0):
    """A seeded random message plan shared by every rank: per_rank x n
    messages between random (source, destination) pairs, self included, on
    three tags, sizes from 0 B to 2 MiB across the eager, staged and direct
    paths, standard or synchronous mode.  Each rank posts its sends and its
    receives (buffers sometimes larger than the message) in a random
    interleaving of its own that keeps plan order on every (source, tag)
    channel, then waits for its receives in a random order and for its
    sends.  MPI's non-overtaking rule fixes which message each receive gets:
    the i-th receive of a channel gets the channel's i-th send; every byte
    and every status checked.  wild > 0: that share of the messages travel
    on tag 40 and are received with MPI_ANY_SOURCE (buffers of the largest
    size); non-overtaking then fixes only the order per source, so the j-th
    wildcard receive that a source's message matched (in posting order)
    must hold that source's j-th tag-40 message to this rank."""
    rng = np.random.default_rng(SEED + salt)
    sizes = [0, 1, 17, 4096, 4097, 65536 + 13, 300001, (2 << 20) + 5]
    plan = []
    for k in range(per_rank * n):
        src, dst = int(rng.integers(n)), int(rng.integers(n))
        tag = 40 if rng.random() < wild else 31 + int(rng.integers(3))
        plan.append((src, dst, tag, int(rng.choice(sizes)), int(rng.integers(4)) == 0))
    wild_from = {}  # source -> [(k, bytes)] of its tag-40 messages to this rank, in plan order
    for k, (src, dst, tag, nb, _) in enumerate(plan):
        if dst == rank and tag == 40:
            wild_from.setdefault(src, []).append((k, nb))
    wild_seen = {}
    mine_s = [(k, m) for k, m in enumerate(plan) if m[0] == rank]
    mine_r = [(k, m) for k, m in enumerate(plan) if m[1] == rank]
    local = np.random.default_rng(SEED + salt + 1000 + rank)
    order = ["s"] * len(mine_s) + ["r"] * len(mine_r)
    local.shuffle(order)
    sreqs, rreqs, keep = [], [], []
    si = ri = 0
    for kind in order:
        if kind == "s":
            k, (src, dst, tag, nb, sync) = mine_s[si]
            si += 1
            buf = dev(payload(rank, salt + k, nb)) if nb else zeros(16)
            keep.append(buf)
            mode = pml.SEND_SYNCHRONOUS if sync else pml.SEND_STANDARD
            sreqs.append(pml.isend(comm, buf, dst, tag, nbytes=nb, mode=mode, stream=STREAM))
        else:
            k, (src, dst, tag, nb, _) = mine_r[ri]
            ri += 1
            extra = int(local.choice([0, 0, 16, 4096]))
            if tag == 40:  # any source: room for the largest message
                nb, src, k = max(sizes), pml.ANY_SOURCE, -1
            buf = zeros(nb + extra + 1)
            rreqs.append((k, src, tag, nb, buf, pml.irecv(comm, buf, src, tag, nbytes=nb + extra,
                                                          stream=STREAM)))
    fails = []
    waited = {}
    for i in local.permutation(len(rreqs)):
        k, src, tag, nb, buf, rq = rreqs[i]
        try:
            waited[i] = rq.wait()
        except _lib.OmpiAmdError as e:
            return False, f"receive of message {k} ({nb} B from {src}, tag {tag}): {e}"
    for i, (k, src, tag, nb, buf, rq) in enumerate(rreqs):  # posting order
        st = waited[i]
        if tag == 40:  # the j-th match from st.source is that source's j-th message
            j = wild_seen.get(st.source, 0)
            wild_seen[st.source] = j + 1
            if st.tag != 40 or j >= len(wild_from.get(st.source, [])):
                fails.append(f"wildcard receive {i}: unexpected ({st.source}, {st.tag})")
                rq.free()
                continue
            k, nb = wild_from[st.source][j]
            src = st.source
        if st.bytes != nb or st.source != src or st.tag != tag:
            fails.append(f"message {k}: status ({st.source}, {st.tag}, {st.bytes} B), "
                         f"expected ({src}, {tag}, {nb} B)")
        else:
            got = host(buf)
            ok, msg = eq(got[:nb], payload(src, salt + k, nb), f"message {k} ({nb} B from {src})")
            if ok and got[nb] != 0:
                ok, msg = False, f"message {k}: byte past the message written"
            if not ok:
                fails.append(msg)
        rq.free()
    for rq in sreqs:
        rq.wait()
        rq.free()
    return not fails, "; ".join(fails[:3])


def case_recv_timeout_cancel(comm, rank, n, salt):
    """A receive that times out is withdrawn: the message sent
    after the timeout is not copied into the abandoned buffer, and the next
    receive with the same (source, tag) gets it."""
    nxt, prv = (rank + 1) % n, (rank - 1) % n
    nbytes = 70001
    first = zeros(nbytes)
    comm.set_param("timeout_ms", 300)
    timed_out = False
    try:
        pml.recv(comm, first, prv, 300 + salt, stream=STREAM)
    except _lib.OmpiAmdError:
        timed_out = True
    finally:
        comm.set_param("timeout_ms", 20000)
    comm_barrier()
    s = dev(payload(rank, salt, nbytes))
    rq = pml.isend(comm, s, nxt, 300 + salt, stream=STREAM)
    second = zeros(nbytes)
    st = pml.recv(comm, second, prv, 300 + salt, stream=STREAM)
    rq.wait()
    rq.free()
    if not timed_out:
        return False, "the first receive did not time out"
    if host(first).any():
        return False, "the withdrawn receive's buffer was written"
    if st.bytes != nbytes:
        return False, f"status {st}"
    return eq(host(second), payload(prv, salt, nbytes), "second receive")


def case_any_source(comm, rank, n, salt):
    """Every rank but 0 sends to 0 with tag = its rank; rank 0 receives with
    ANY_SOURCE / ANY_TAG and checks each status against the data."""
    if rank != 0:
        pml.send(comm, dev(payload(rank, salt, 4096 + rank)), 0, rank, stream=STREAM)
        return True, ""
    seen = set()
    for _ in range(n - 1):
        r = zeros(8192)
        st = pml.recv(comm, r, pml.ANY_SOURCE, pml.ANY_TAG, stream=STREAM)
        if st.tag != st.source or st.bytes != 4096 + st.source or st.source in seen:
            return False, f"status {st}"
        seen.add(st.source)
        ok, msg = eq(host(r)[:st.bytes], payload(st.source, salt, st.bytes), f"from {st.source}")
        if not ok:
            return ok, msg
    return seen == set(range(1, n)), f"sources {sorted(seen)}"


def case_fan_in_any_source(comm, rank, n, salt, k=40):
    """Every rank but 0 isends k messages to rank 0 (eager and staged sizes
    alternating, tags cycling 0..2); rank 0 posts all (n-1)*k receives as
    ANY_SOURCE / ANY_TAG at once, while the senders publish: every message
    arrives exactly once, intact, and per source in sending order
    (MPI's non-overtaking rule across wildcard receives)."""
    size_of = lambda i: 1000 + i if i % 2 == 0 else 70000 + i
    if rank != 0:
        sends = [dev(payload(rank, salt + i, size_of(i))) for i in range(k)]
        reqs = [pml.isend(comm, sends[i], 0, i % 3, stream=STREAM) for i in range(k)]
        for rq in reqs:
            rq.wait()
            rq.free()
        return True, ""
    total = (n - 1) * k
    bufs = [zeros(80000) for _ in range(total)]
    rreqs = [pml.irecv(comm, bufs[j], pml.ANY_SOURCE, pml.ANY_TAG, stream=STREAM) for j in range(total)]
    last = {}
    seen = set()
    for j, rq in enumerate(rreqs):
        st = rq.wait()
        i = st.bytes - 1000 if st.bytes < 70000 else st.bytes - 70000
        if not 0 <= i < k or size_of(i) != st.bytes or st.tag != i % 3 or (st.source, i) in seen:
            return False, f"receive {j}: status {st}"
        if last.get(st.source, -1) >= i:
            return False, f"receive {j}: message {i} of rank {st.source} after message {last[st.source]}"
        last[st.source] = i
        seen.add((st.source, i))
        ok, msg = eq(host(bufs[j])[:st.bytes], payload(st.source, salt + i, st.bytes), f"{st.source}:{i}")
        if not ok:
            return ok, msg
        rq.free()
    return len(seen) == total, f"{len(seen)} of {total} messages"


def case_probe_truncate(comm, rank, n, salt):
    """probe reports the size; a short receive raises MPI_ERR_TRUNCATE with
    the prefix delivered; traffic continues afterwards."""
    nxt, prv = (rank + 1) % n, (rank - 1) % n
    a = dev(payload(rank, salt, 1000))
    b = dev(payload(rank, salt + 1, 77))
    r1 = pml.isend(comm, a, nxt, 3, stream=STREAM)
    r2 = pml.isend(comm, b, nxt, 4, stream=STREAM)
    st = pml.probe(comm, prv, 3)
    if (st.source, st.tag, st.bytes) != (prv, 3, 1000):
        return False, f"probe {st}"
    if pml.iprobe(comm, prv, 99) is not None:
        return False, "iprobe matched a tag nobody sent"
    short = zeros(600)
    try:
        pml.recv(comm, short, prv, 3, stream=STREAM)
        return False, "no truncation error"
    except _lib.OmpiAmdError as e:
        if e.code != _lib.ERR_TRUNCATE:
            return False, f"error {e}"
    ok, msg = eq(host(short), payload(prv, salt, 1000)[:600], "truncated prefix")
    if not ok:
        return ok, msg
    rb = zeros(77)
    st = pml.recv(comm, rb, prv, 4, stream=STREAM)
    for rq in (r1, r2):
        rq.wait()
        rq.free()
    return eq(host(rb), payload(prv, salt + 1, 77), "after truncation")


def case_self(comm, rank, n, salt):
    a = dev(payload(rank, salt, 123457))
    rq = pml.isend(comm, a, rank, 11, stream=STREAM)
    r = zeros(123457)
    st = pml.recv(comm, r, rank, 11, stream=STREAM)
    rq.wait()
    rq.free()
    if st.source != rank:
        return False, f"status {st}"
    return eq(host(r), payload(rank, salt, 123457), "self")


def case_eager_send_first(comm, rank, n, salt, k=50):
    """Every rank first MPI_Sends k small messages (<= 4 KiB, eager) to the
    next rank, overwriting its buffer after each send returns, and only then
    receives: completes only because small sends do not wait for the
    receiver; the data is what the buffer held at the send."""
    nxt, prv = (rank + 1) % n, (rank - 1) % n
    buf = zeros(4096)
    for i in range(k):
        nb = 1 + (i * 97) % 4096
        src = dev(payload(rank, salt + i, nb))
        with torch.cuda.stream(STREAM):
            buf[:nb].copy_(src)
        pml.send(comm, buf, nxt, 20 + i % 3, nbytes=nb, stream=STREAM)
        with torch.cuda.stream(STREAM):
            buf.zero_()  # the send already returned: its data was staged
    fails = []
    for i in range(k):
        nb = 1 + (i * 97) % 4096
        r = zeros(4096)
        st = pml.recv(comm, r, prv, 20 + i % 3, stream=STREAM)
        if st.bytes != nb:
            fails.append(f"msg {i}: {st.bytes} bytes, expected {nb}")
            continue
        ok, msg = eq(host(r)[:nb], payload(prv, salt + i, nb), f"msg {i}")
        if not ok:
            fails.append(msg)
    return not fails, "; ".join(fails[:3])


def case_ssend_small(comm, rank, n, salt):
    """MPI_Ssend of a small message takes the rendezvous: the isend is not
    complete before the receive is posted; data arrives intact."""
    nxt, prv = (rank + 1) % n, (rank - 1) % n
    a = dev(payload(rank, salt, 100))
    rq = pml.isend(comm, a, nxt, 31, mode=pml.SEND_SYNCHRONOUS, stream=STREAM)
    early = rq.test()
    comm_barrier()  # nobody has posted its receive yet
    r = zeros(100)
    pml.recv(comm, r, prv, 31, stream=STREAM)
    rq.wait()
    rq.free()
    if early:
        return False, "synchronous send completed before the receive was posted"
    return eq(host(r), payload(prv, salt, 100), "ssend")


# ----------------------------------------------------------------- osc cases
def fp_inputs(dt, count, rank, salt, kind="R"):
    rng = np.random.default_rng(SEED + 1000 * salt + rank)
    nd = dt.np_dtype
    if nd.names:
        a = np.zeros(count, dtype=nd)
        a["v"] = np.round(rng.random(count) * 64) / 64
        a["k"] = rank * count + np.arange(count)
        return a
    if nd.kind == "f":
        if kind == "E":
            return (rng.integers(-1024, 1025, count) * 2.0 ** -8).astype(nd)
        a = rng.uniform(-1, 1, count).astype(nd)
        if kind == "S":
            idx = rng.integers(0, count, max(1, count // 8))
            a[idx] = rng.choice(np.array([np.nan, 0.0, -0.0, np.inf, -np.inf], dtype=nd), len(idx))
        return a
    info = np.iinfo(nd)
    lo, hi = (-(1 << 20), 1 << 20) if nd.itemsize >= 4 else (info.min, info.max)
    return rng.integers(max(lo, info.min), hi, count, dtype=nd, endpoint=True)


def case_put_get(comm, rank, n, nbytes, salt):
    nxt, prv = (rank + 1) % n, (rank - 1) % n
    win = osc.Window.allocate(comm, nbytes + 64, disp_unit=1)
    try:
        src = dev(payload(rank, salt, nbytes))
        win.fence(stream=STREAM)
        win.put(src, nxt, 13, nbytes, stream=STREAM)
        win.fence(stream=STREAM, blocking=True)
        local = torch.empty(nbytes + 64, dtype=torch.uint8, device="cuda")
        win.get(local, rank, 0, stream=STREAM)  # own window through the same path
        got = host(local)
        exp = np.zeros(nbytes + 64, np.uint8)
        exp[13:13 + nbytes] = payload(prv, salt, nbytes)
        ok, msg = eq(got, exp, "put")
        if not ok:
            return ok, msg
        back = zeros(nbytes)
        win.get(back, nxt, 13, stream=STREAM)  # next rank's window holds my data
        win.fence(stream=STREAM, blocking=True)
        return eq(host(back), payload(rank, salt, nbytes), "get")
    finally:
        win.free()


def case_cross_layer(comm, rank, n, salt, k=4):
    """MPI's progress rule across layers and communicators, on the MPI path
    (coll/rocm, pml/rocm and osc/rocm each give a communicator a queue of its
    own: param own_stream): every rank interleaves, in its OWN random order,
    nonblocking collectives on communicator A (in A's order on every rank) (iallreduce at the fused,
    staged and zero-copy sizes, ireduce_scatter_block, iallgather) and a ring
    of isends / irecvs on communicator B (eager and rendezvous sizes, one tag
    each); then, with all of that outstanding, a fence epoch of puts on a
    window of communicator C (blocking, every rank alike); then waits for
    the requests in its own random order. Every result is checked."""
    F = mop.MPI_FLOAT
    nxt, prv = (rank + 1) % n, (rank - 1) % n
    comms = []
    for _ in range(3):
        cc = coll.Communicator.from_torch_distributed(device=comm.device)
        cc.set_param("timeout_ms", 20000)
        cc.set_param("own_stream", 1)
        comms.append(cc)
    ca, cb, cw = comms
    mine = np.random.default_rng(SEED + salt + 1000 * (rank + 1))
    win = None
    try:
        posts = []  # (go, check)
        for i, (kind, count) in enumerate([("ar", 7), ("ar", 70001), ("ar", (1 << 20) + 3),
                                           ("rsb", 50001), ("ag", 40001)]):
            xs = [np.random.default_rng(SEED + salt + 31 * i + r).standard_normal(
                count * (n if kind == "rsb" else 1)).astype(np.float32) for r in range(n)]
            s = dev(xs[rank])
            if kind == "ar":
                exp = orc.allreduce([x.copy() for x in xs], count, mop.MPI_SUM.index, F.code)[0][rank]
                o = zeros(count * 4)
                go = functools.partial(ca.iallreduce, s, o, count, F, mop.MPI_SUM)
            elif kind == "rsb":
                exp = orc.reduce_scatter_block([x.copy() for x in xs], count, mop.MPI_SUM.index,
                                               F.code)[rank].view(np.float32)
                o = zeros(count * 4)
                go = functools.partial(ca.ireduce_scatter_block, s, o, count, F, mop.MPI_SUM)
            else:
                exp = np.concatenate(xs)
                o = zeros(n * count * 4)
                go = functools.partial(ca.iallgather, s, o, count * 4)
            posts.append((go, (o, exp, f"A {kind} {count}"), s))
        for j in range(k):
            nb = (17, 4099, (1 << 20) + 5, (8 << 20) + 1)[j % 4]
            s = dev(payload(rank, salt + 50 + j, nb))
            r = zeros(nb)
            posts.append((functools.partial(pml.isend, cb, s, nxt, 900 + j, nb, stream=STREAM), None, s))
            posts.append((functools.partial(pml.irecv, cb, r, prv, 900 + j, nb, stream=STREAM),
                          (r, payload(prv, salt + 50 + j, nb), f"B recv {nb}"), r))
        wbytes = (3 << 20) + 44
        wbase = zeros(wbytes)
        win = osc.Window.create(cw, wbase, wbytes)
        wsrc = dev(payload(rank, salt + 90, wbytes - 40))
        torch.cuda.synchronize()
        # this rank's own interleaving of A's calls (in A's order: MPI orders
        # a communicator's collectives) with B's isends / irecvs (any order:
        # they match by tag)
        acalls, bcalls = posts[:5], posts[5:]
        mine.shuffle(bcalls)
        lanes = ["A"] * len(acalls) + ["B"] * len(bcalls)
        mine.shuffle(lanes)
        ai, bi = iter(acalls), iter(bcalls)
        posts = [next(ai) if ln == "A" else next(bi) for ln in lanes]
        reqs = [(go(), chk) for go, chk, _ in posts]
        win.fence(stream=STREAM)
        win.put(wsrc, nxt, 40, wbytes - 40, stream=STREAM)
        win.fence(stream=STREAM, blocking=True)
        order = list(range(len(reqs)))
        mine.shuffle(order)
        for i in order:
            reqs[i][0].wait()
        torch.cuda.synchronize()
        msgs = []
        for req, chk in reqs:
            req.free()
            if chk is None:
                continue
            buf, exp, what = chk
            ok, msg = eq(host(buf)[:exp.nbytes], exp, what)
            if not ok:
                msgs.append(msg)
        want = np.zeros(wbytes, np.uint8)
        want[40:] = payload(prv, salt + 90, wbytes - 40)
        ok, msg = eq(host(wbase), want, "C put")
        if not ok:
            msgs.append(msg)
        for cc in comms:
            if cc.error():
                msgs.append(f"device error {cc.error()}")
        return not msgs, "; ".join(msgs[:3])
    finally:
        if win is not None:
            win.free()
        for cc in comms:
            cc.free()


def case_acc_disjoint(comm, rank, n, dt, op, count, salt, kind="R"):
    """Each rank accumulates into the next rank's window (one origin per
    target): deterministic, bit-exact vs op/base incl. NaN / ±0 selection."""
    nxt, prv = (rank + 1) % n, (rank - 1) % n
    ext = dt.extent
    win_init = [fp_inputs(dt, count, r, salt, kind) for r in range(n)]
    origins = [fp_inputs(dt, count, r, salt + 1, kind) for r in range(n)]
    base = dev(win_init[rank], extra=16)
    win = osc.Window.create(comm, base, count * ext + 16, disp_unit=ext)
    try:
        o = dev(origins[rank])
        win.fence(stream=STREAM)
        win.accumulate(o, count, dt, nxt, 0, op, stream=STREAM)
        win.fence(stream=STREAM, blocking=True)
        exp = win_init[rank].copy()
        orc.op_2buff(op.index, dt.code, origins[prv].copy(), exp, count)
        got = host(base)[:count * ext].view(dt.np_dtype)
        if dt.np_dtype.names:  # gap bytes carry no data
            ok1, m1 = eq(got["v"], exp["v"], "v")
            ok2, m2 = eq(got["k"], exp["k"], "k")
            return ok1 and ok2, m1 + m2
        return eq(got, exp, op.name)
    finally:
        win.free()


def case_acc_concurrent(comm, rank, n, dt, op, count, salt, kind="E"):
    """Every rank accumulates into the SAME region of rank 0 at once: the
    accumulate lock serialises them; with exact data every order agrees."""
    ext = dt.extent
    init = fp_inputs(dt, count, 99, salt, kind)
    origins = [fp_inputs(dt, count, r, salt + 1, kind) for r in range(n)]
    base = dev(init if rank == 0 else np.zeros(0, np.uint8), extra=16)
    win = osc.Window.create(comm, base, base.numel(), disp_unit=ext)
    try:
        o = dev(origins[rank])
        win.fence(stream=STREAM)
        for _ in range(2):
            win.accumulate(o, count, dt, 0, 0, op, stream=STREAM)
        win.fence(stream=STREAM, blocking=True)
        if rank != 0:
            return True, ""
        exp = init.copy()
        for r in range(n):
            for _ in range(2):
                orc.op_2buff(op.index, dt.code, origins[r].copy(), exp, count)
        got = host(base)[:count * ext].view(dt.np_dtype)
        if dt.np_dtype.names:
            ok1, m1 = eq(got["v"], exp["v"], "v")
            ok2, m2 = eq(got["k"], exp["k"], "k")
            return ok1 and ok2, m1 + m2
        return eq(got, exp, op.name)
    finally:
        win.free()


def case_get_accumulate(comm, rank, n, salt, count=50001):
    """result = old target; target = old + origin (fp64, exact data); then
    REPLACE and NO_OP."""
    D = mop.MPI_DOUBLE
    nxt, prv = (rank + 1) % n, (rank - 1) % n
    init = [fp_inputs(D, count, r, salt, "E") for r in range(n)]
    org = [fp_inputs(D, count, r, salt + 1, "E") for r in range(n)]
    base = dev(init[rank])
    win = osc.Window.create(comm, base, count * 8, disp_unit=8)
    try:
        o = dev(org[rank])
        res = zeros(count * 8)
        win.fence(stream=STREAM)
        win.get_accumulate(o, res, count, D, nxt, 0, mop.MPI_SUM, stream=STREAM)
        win.fence(stream=STREAM, blocking=True)
        ok, msg = eq(host(res).view(np.float64), init[nxt], "fetched")
        if not ok:
            return ok, msg
        ok, msg = eq(host(base).view(np.float64), init[rank] + org[prv], "summed")
        if not ok:
            return ok, msg
        comm_barrier()  # every rank checked its window before the next epoch writes it
        # REPLACE via get_accumulate, then NO_OP fetch
        win.get_accumulate(o, res, count, D, nxt, 0, mop.MPI_REPLACE, stream=STREAM)
        win.fence(stream=STREAM, blocking=True)
        ok, msg = eq(host(res).view(np.float64), init[nxt] + org[rank], "fetched before replace")
        if not ok:
            return ok, msg
        res2 = zeros(count * 8)
        win.get_accumulate(None, res2, count, D, nxt, 0, mop.MPI_NO_OP, stream=STREAM)
        win.fence(stream=STREAM, blocking=True)
        ok, msg = eq(host(res2).view(np.float64), org[rank], "no_op fetch after replace")
        if not ok:
            return ok, msg
        return eq(host(base).view(np.float64), org[prv], "replaced")
    finally:
        win.free()


def _slots(dt, count, elem):
    """Byte offsets of the `elem`-byte primitive slots of count x dt, in
    type-map order (what ompi_osc_base_sndrcv_op walks)."""
    offs = []
    for i in range(count):
        for d, bl in dt.runs:
            offs.extend(i * dt.extent + d + b for b in range(0, bl, elem))
    return np.array(offs, dtype=np.int64)


def _pairs(prim, m, r, salt, seed_junk):
    """m memory pairs of `prim` (DOUBLE_INT 16 B, SHORT_INT 8 B): small
    integer values (ties exercise the lowest-index rule), random indices,
    junk in the padding."""
    g = np.random.default_rng(SEED + 131 * salt + r)
    mem = np.frombuffer(payload(r, seed_junk, m * prim.extent), np.uint8).copy().reshape(m, prim.extent)
    v = g.integers(-8, 9, m)
    k = g.integers(0, 1 << 20, m).astype(np.int32)
    if prim is mop.MPI_DOUBLE_INT:
        mem[:, 0:8] = v.astype(np.float64).view(np.uint8).reshape(m, 8)
        mem[:, 8:12] = k.view(np.uint8).reshape(m, 4)
    else:  # SHORT_INT: short at 0, int at 4 (bytes 2-3 padding)
        mem[:, 0:2] = v.astype(np.int16).view(np.uint8).reshape(m, 2)
        mem[:, 4:8] = k.view(np.uint8).reshape(m, 4)
    return mem


def _member_bytes(prim):
    """Byte ranges of a pair's members (what MPI owns; the rest is padding)."""
    return [(0, 8), (8, 12)] if prim is mop.MPI_DOUBLE_INT else [(0, 2), (4, 8)]


def case_acc_ddt_pair(comm, rank, n, salt):
    """MPI_Accumulate / MPI_Get_accumulate of pair types (MAXLOC / MINLOC
    operands) with derived datatypes (ompi_osc_base_sndrcv_op,
    osc_base_obj_convert.c:73-245): a vector of MPI_DOUBLE_INT at the
    target from a contiguous or a strided origin (12-byte packed pairs into
    16-byte slots), REPLACE, a contiguous MPI_SHORT_INT target (int at
    offset 4) from a strided origin, and get_accumulate into a strided
    result; expected from the oracle's op/base LOC rule pair by pair in
    type-map order, bit-exact, every padding and gap byte of the window (and
    of the result) untouched."""
    from ompi_amd import datatype as dd
    DI, SI = mop.MPI_DOUBLE_INT, mop.MPI_SHORT_INT
    nxt, prv = (rank + 1) % n, (rank - 1) % n
    di = dd.from_runs("double_int", [(0, 12)], 16)
    si = dd.from_runs("short_int", [(0, 2), (4, 4)], 8)
    runs = [
        # (name, prim, target type, tcount, origin type or None, op)
        ("double_int_vector_maxloc", DI, dd.type_vector(300, 1, 2, di), 2, None, mop.MPI_MAXLOC),
        ("double_int_vector_minloc_strided_origin", DI, dd.type_vector(150, 2, 3, di), 2,
         dd.type_vector(600, 1, 3, di), mop.MPI_MINLOC),
        ("double_int_vector_replace", DI, dd.type_vector(200, 1, 3, di), 1, dd.type_vector(200, 1, 2, di),
         mop.MPI_REPLACE),
        ("short_int_contig_target_minloc", SI, None, 500, dd.type_vector(500, 1, 2, si), mop.MPI_MINLOC),
    ]
    disp_unit, disp = 8, 3
    for k, (name, prim, tdt, tcount, odt, op) in enumerate(runs):
        E, mem_b = prim.extent, _member_bytes(prim)
        m = (tdt.size // prim.size) * tcount if tdt else tcount  # pairs
        span = ((tcount - 1) * tdt.extent + tdt.true_span) if tdt else m * E
        wbytes = disp * disp_unit + span + 64
        init = [np.frombuffer(payload(r, salt + k, wbytes), np.uint8).copy() for r in range(n)]
        tslots = disp * disp_unit + (np.array([i * tdt.extent + d for i in range(tcount) for d, _ in tdt.runs
                                               if d % E == 0], np.int64) if tdt else np.arange(m) * E)
        assert len(tslots) == m
        for r in range(n):  # real pairs in the window's target slots (gaps keep payload bytes)
            pr = _pairs(prim, m, r, salt + 10 + k, salt + 11 + k)
            for j, t in enumerate(tslots):
                init[r][t:t + E] = pr[j]
        org_mem = [_pairs(prim, m, r, salt + 20 + k, salt + 21 + k) for r in range(n)]
        if odt is None:
            org_buf, ocount = [om.reshape(-1) for om in org_mem], m
        else:  # the pairs at the origin type's slots, junk between
            ocount = 1
            oslots = np.array([d for d, _ in odt.runs if d % E == 0], np.int64)
            assert len(oslots) == m
            org_buf = []
            for r in range(n):
                b = np.frombuffer(payload(r, salt + 30 + k, int(oslots.max()) + E), np.uint8).copy()
                for j, o in enumerate(oslots):
                    b[o:o + E] = org_mem[r][j]
                org_buf.append(b)
        base = dev(init[rank])
        win = osc.Window.create(comm, base, wbytes, disp_unit=disp_unit)
        try:
            o = dev(org_buf[rank])
            win.fence(stream=STREAM)
            win.accumulate_ddt(o, ocount, odt, nxt, disp, tcount, tdt, prim, op, stream=STREAM)
            win.fence(stream=STREAM, blocking=True)
            exp = init[rank].copy()
            cur = np.stack([exp[t:t + E] for t in tslots]).copy()
            if op is mop.MPI_REPLACE:
                new = org_mem[prv].copy()
            else:
                new = cur.copy()
                orc.op_2buff(op.index, prim.code, org_mem[prv].reshape(-1).copy(), new.reshape(-1), m)
            for j, t in enumerate(tslots):
                for a, b in mem_b:  # only the members; the padding keeps the window's bytes
                    exp[t + a:t + b] = new[j, a:b]
            ok, msg = eq(host(base), exp, f"{name}: window")
            if not ok:
                return ok, msg
        finally:
            win.free()
        comm_barrier()
    # get_accumulate MAXLOC: the old target pairs into a strided result
    prim, E = DI, 16
    tdt, tcount = dd.type_vector(120, 1, 2, di), 3
    rdt = dd.type_vector(360, 1, 2, di)
    m = 360
    span = (tcount - 1) * tdt.extent + tdt.true_span
    wbytes = span + 64
    tslots = np.array([i * tdt.extent + d for i in range(tcount) for d, _ in tdt.runs], np.int64)
    init = [np.frombuffer(payload(r, salt + 50, wbytes), np.uint8).copy() for r in range(n)]
    for r in range(n):
        pr = _pairs(prim, m, r, salt + 51, salt + 52)
        for j, t in enumerate(tslots):
            init[r][t:t + E] = pr[j]
    org = [_pairs(prim, m, r, salt + 53, salt + 54) for r in range(n)]
    base = dev(init[rank])
    win = osc.Window.create(comm, base, wbytes, disp_unit=1)
    try:
        o = dev(org[rank].reshape(-1))
        res = zeros(2 * m * E)
        win.fence(stream=STREAM)
        win.get_accumulate_ddt(o, m, None, res, 1, rdt, nxt, 0, tcount, tdt, prim, mop.MPI_MAXLOC,
                               stream=STREAM)
        win.fence(stream=STREAM, blocking=True)
        got = host(res).reshape(2 * m, E)
        old = np.stack([init[nxt][t:t + E] for t in tslots])
        exp = np.zeros((2 * m, E), np.uint8)
        exp[0::2, 0:12] = old[:, 0:12]  # the fetched members; padding and odd slots stay zero
        ok, msg = eq(got, exp, "get_accumulate MAXLOC: fetched into the strided result")
        if not ok:
            return ok, msg
        cur = np.stack([init[rank][t:t + E] for t in tslots]).copy()
        new = cur.copy()
        orc.op_2buff(mop.MPI_MAXLOC.index, prim.code, org[prv].reshape(-1).copy(), new.reshape(-1), m)
        expw = init[rank].copy()
        for j, t in enumerate(tslots):
            expw[t:t + 12] = new[j, 0:12]
        return eq(host(base), expw, "get_accumulate MAXLOC: window")
    finally:
        win.free()


def case_acc_ddt(comm, rank, n, salt):
    """MPI_Accumulate / MPI_Get_accumulate with derived datatypes
    (osc_sm_comm.c:301, 350 -> ompi_osc_base_sndrcv_op): each rank updates
    the next rank's window through a target datatype (vector, blacs-style
    indexed), from a contiguous or a strided origin, with SUM, MAX (specials),
    REPLACE, and get_accumulate into a strided result; expected values from
    the oracle's op/base restatement applied slot by slot in type-map order
    (bit-exact), gaps of the window untouched."""
    from ompi_amd import datatype as dd
    F, D = mop.MPI_FLOAT, mop.MPI_DOUBLE
    nxt, prv = (rank + 1) % n, (rank - 1) % n
    f32, f64 = dd.predefined("MPI_FLOAT"), dd.predefined("MPI_DOUBLE")
    lens = [13, 13, 13, 13, 13, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1]
    disps = [286, 308, 330, 352, 374, 396, 419, 442, 465, 488, 511, 534, 557, 580, 603, 626, 649, 672]
    runs = [
        # (name, prim, target type, tcount, origin type or None, op, kind)
        ("vector_sum", F, dd.type_vector(997, 3, 7, f32), 3, None, mop.MPI_SUM, "R"),
        ("indexed_max", F, dd.type_indexed(lens, disps, f32), 40, dd.type_vector(40 * 156, 1, 2, f32),
         mop.MPI_MAX, "S"),
        ("vector_replace", D, dd.type_vector(501, 2, 5, f64), 2, dd.type_vector(1002, 2, 3, f64),
         mop.MPI_REPLACE, "R"),
        ("contig_target_min", D, None, 4001, dd.type_vector(4001, 1, 3, f64), mop.MPI_MIN, "S"),
    ]
    disp_unit, disp = 4, 6  # the target region starts 24 B into the window
    for k, (name, prim, tdt, tcount, odt, op, kind) in enumerate(runs):
        el = prim.extent
        m = (tdt.size * tcount if tdt else el * tcount) // el  # primitive elements
        span = ((tcount - 1) * tdt.extent + tdt.true_span) if tdt else m * el
        wbytes = disp * disp_unit + span + 64
        init = [np.frombuffer(payload(r, salt + k, wbytes), np.uint8).copy() for r in range(n)]
        for r in range(n):  # real values in the window (gaps keep their payload bytes)
            vals = fp_inputs(prim, wbytes // el, r, salt + 10 + k, kind)
            init[r][:(wbytes // el) * el] = vals.view(np.uint8)
        org_packed = [fp_inputs(prim, m, r, salt + 20 + k, kind) for r in range(n)]
        if odt is None:
            org_buf = [p_.view(np.uint8) for p_ in org_packed]
            ocount = m
        else:  # the packed values at the origin type's slots, junk between
            ocount = 1
            assert odt.size == m * el
            oslots = _slots(odt, 1, el)
            org_buf = []
            for r in range(n):
                b = np.frombuffer(payload(r, salt + 30 + k, int(oslots.max()) + el), np.uint8).copy()
                for j, o in enumerate(oslots):
                    b[o:o + el] = org_packed[r][j:j + 1].view(np.uint8)
                org_buf.append(b)
        base = dev(init[rank])
        win = osc.Window.create(comm, base, wbytes, disp_unit=disp_unit)
        try:
            o = dev(org_buf[rank])
            win.fence(stream=STREAM)
            win.accumulate_ddt(o, ocount, odt, nxt, disp, tcount, tdt, prim, op, stream=STREAM)
            win.fence(stream=STREAM, blocking=True)
            exp = init[rank].copy()
            tslots = disp * disp_unit + (_slots(tdt, tcount, el) if tdt else np.arange(m) * el)
            cur = np.concatenate([exp[t:t + el] for t in tslots]).view(prim.np_dtype).copy()
            if op is mop.MPI_REPLACE:
                cur = org_packed[prv].copy()
            else:
                orc.op_2buff(op.index, prim.code, org_packed[prv].copy(), cur, m)
            cb = cur.view(np.uint8)
            for j, t in enumerate(tslots):
                exp[t:t + el] = cb[j * el:(j + 1) * el]
            ok, msg = eq(host(base), exp, f"{name}: window")
            if not ok:
                return ok, msg
        finally:
            win.free()
        comm_barrier()
    # get_accumulate: the old target slots into a strided result, then SUM
    tdt, tcount, prim = dd.type_vector(333, 2, 5, f32), 4, F
    rdt = dd.type_vector(333 * 2 * 4, 1, 2, f32)
    el, m = 4, 333 * 2 * 4
    span = (tcount - 1) * tdt.extent + tdt.true_span
    wbytes = span + 64
    init = [fp_inputs(prim, wbytes // 4, r, salt + 50, "E").view(np.uint8).copy() for r in range(n)]
    org = [fp_inputs(prim, m, r, salt + 51, "E") for r in range(n)]
    base = dev(init[rank])
    win = osc.Window.create(comm, base, wbytes, disp_unit=1)
    try:
        o = dev(org[rank])
        res = zeros(2 * m * 4)
        win.fence(stream=STREAM)
        win.get_accumulate_ddt(o, m, None, res, 1, rdt, nxt, 0, tcount, tdt, prim, mop.MPI_SUM,
                               stream=STREAM)
        win.fence(stream=STREAM, blocking=True)
        tslots = _slots(tdt, tcount, 4)
        old = np.concatenate([init[nxt][t:t + 4] for t in tslots]).view(np.float32)
        got = host(res).view(np.float32)
        ok, msg = eq(got[0::2], old, "get_accumulate: fetched into the strided result")
        if not ok:
            return ok, msg
        ok, msg = eq(got[1::2], np.zeros(m, np.float32), "get_accumulate: result gaps untouched")
        if not ok:
            return ok, msg
        exp = init[rank].copy()
        mine_old = np.concatenate([exp[t:t + 4] for t in tslots]).view(np.float32) + org[prv]
        for j, t in enumerate(tslots):
            exp[t:t + 4] = mine_old[j:j + 1].view(np.uint8)
        return eq(host(base), exp, "get_accumulate: window")
    finally:
        win.free()


def case_put_get_ddt(comm, rank, n, salt):
    """MPI_Put / MPI_Get with derived datatypes (osc_sm_comm.c:24-100,
    209-270: ompi_datatype_sndrcv of any origin / target pair): each rank
    puts into the next rank's window through a target datatype (vector of
    single doubles, blacs-style indexed floats, struct {int, double} with its
    4-byte hole), from a contiguous or a strided origin, then gets it back
    into a gapped origin layout; request-based rput / rget under lock_all.
    Expected bytes: the origin's bytes in type-map order at the target type's
    byte slots; every other byte of the window and of the origin buffer
    untouched (byte-exact)."""
    from ompi_amd import datatype as dd
    nxt, prv = (rank + 1) % n, (rank - 1) % n
    f32, f64, i32 = dd.predefined("MPI_FLOAT"), dd.predefined("MPI_DOUBLE"), dd.predefined("MPI_INT32_T")
    lens = [13, 13, 13, 13, 13, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1]
    disps = [286, 308, 330, 352, 374, 396, 419, 442, 465, 488, 511, 534, 557, 580, 603, 626, 649, 672]
    pair = dd.type_struct([1, 1], [0, 8], [i32, f64])
    runs = [
        # (name, target type, tcount, origin type or None (contiguous bytes), request-based)
        ("vector_bl1_f64", dd.type_vector(20011, 1, 2, f64), 3, None, False),
        ("blacs_indexed_f32", dd.type_indexed(lens, disps, f32), 37, dd.type_vector(37 * 156, 1, 3, f32), False),
        ("struct_int_double", pair, 50003, dd.type_vector(50003, 1, 2, pair), False),
        ("vector_bl3_f32_requests", dd.type_vector(4099, 3, 7, f32), 5, None, True),
    ]
    disp_unit, disp = 8, 3  # the target region starts 24 B into the window
    for k, (name, tdt, tcount, odt, req) in enumerate(runs):
        tbytes = tdt.size * tcount
        span = (tcount - 1) * tdt.extent + tdt.true_span
        wbytes = disp * disp_unit + span + 64
        init = [np.frombuffer(payload(r, salt + k, wbytes), np.uint8).copy() for r in range(n)]
        data = [np.frombuffer(payload(r, salt + 10 + k, tbytes), np.uint8).copy() for r in range(n)]
        tslots = disp * disp_unit + _slots(tdt, tcount, 1)
        if odt is None:
            ocount, oslots, obytes = tbytes, np.arange(tbytes), tbytes
        else:
            ocount = 1
            assert odt.size == tbytes
            oslots = _slots(odt, 1, 1)
            obytes = int(oslots.max()) + 1
        org = []
        for r in range(n):  # the data at the origin type's byte slots, junk between
            b = np.frombuffer(payload(r, salt + 20 + k, obytes), np.uint8).copy()
            b[oslots] = data[r]
            org.append(b)
        base = dev(init[rank])
        win = osc.Window.create(comm, base, wbytes, disp_unit=disp_unit)
        try:
            o = dev(org[rank])
            if req:
                win.lock_all(stream=STREAM)
                r1 = win.rput_ddt(o, ocount, odt, nxt, disp, tcount, tdt, stream=STREAM)
                r1.wait()
                r1.free()
                win.unlock_all(stream=STREAM)
                comm_barrier()
                win.sync(stream=STREAM)  # MPI_Win_sync: the separate model's private copy
            else:
                win.fence(stream=STREAM)
                win.put_ddt(o, ocount, odt, nxt, disp, tcount, tdt, stream=STREAM)
                win.fence(stream=STREAM, blocking=True)
            exp = init[rank].copy()
            exp[tslots] = data[prv]
            ok, msg = eq(host(base), exp, f"{name}: put into the window")
            if not ok:
                return ok, msg
            # get it back from the next rank (which now holds my data) into a
            # fresh origin layout whose gaps must survive
            junk = np.frombuffer(payload(rank, salt + 40 + k, obytes), np.uint8).copy()
            back = dev(junk)
            if req:
                win.lock_all(stream=STREAM)
                r2 = win.rget_ddt(back, ocount, odt, nxt, disp, tcount, tdt, stream=STREAM)
                r2.wait()
                r2.free()
                win.unlock_all(stream=STREAM)
            else:
                win.get_ddt(back, ocount, odt, nxt, disp, tcount, tdt, stream=STREAM)
                win.fence(stream=STREAM, blocking=True)
            expo = junk.copy()
            expo[oslots] = data[rank]
            ok, msg = eq(host(back), expo, f"{name}: get into the origin layout")
            if not ok:
                return ok, msg
        finally:
            win.free()
        comm_barrier()
    # mismatched signatures are refused
    win = osc.Window.allocate(comm, 4096, disp_unit=1)
    try:
        src = dev(payload(rank, salt, 64))
        try:
            win.put_ddt(src, 64, None, nxt, 0, 7, dd.type_vector(4, 2, 3, f32), stream=STREAM)
            return False, "a put with unequal origin / target byte counts was accepted"
        except _lib.OmpiAmdError:
            pass
    finally:
        win.free()
    return True, ""


def case_separate_window(comm, rank, n, salt, nbytes=100003, force=False):
    """MPI_Win_create over memory peers cannot map reliably (a torch tensor
    of a small-pool 2 MiB segment: not an IPC-safe size) runs
    in the separate model (include/ompi_amd_osc.h): MPI_WIN_MODEL is
    SEPARATE on every rank; a fence brings the peers' puts into the caller's
    memory and the caller's own stores to the peers; passive-target puts
    reach it at MPI_Win_sync and at a lock of its own window.  force: the
    osc_win_shadow hook on a 64 MiB + 12 B tensor (IPC-safe segment)."""
    nxt, prv = (rank + 1) % n, (rank - 1) % n
    if force:
        comm.set_param("osc_win_shadow", 1)
    w0 = comm.get_param("osc_shadow_windows")
    try:
        base = dev(payload(rank, salt, nbytes))
        win = osc.Window.create(comm, base, nbytes)
    finally:
        if force:
            comm.set_param("osc_win_shadow", 0)
    try:
        if win.model != osc.WIN_SEPARATE or comm.get_param("osc_shadow_windows") != w0 + 1:
            return False, f"model {win.model}, shadow windows {comm.get_param('osc_shadow_windows') - w0}"
        half = nbytes // 2
        # 1. fence epoch: put into the next rank's first half
        src = dev(payload(rank, salt + 1, half))
        win.fence(stream=STREAM)
        win.put(src, nxt, 0, half, stream=STREAM)
        win.fence(stream=STREAM, blocking=True)
        exp = payload(rank, salt, nbytes).copy()
        exp[:half] = payload(prv, salt + 1, half)
        ok, msg = eq(host(base), exp, "fence: peer's put in the private copy")
        if not ok:
            return ok, msg
        # 2. my own stores between fences reach the peers' gets
        mine = payload(rank, salt + 2, nbytes - half)
        with torch.cuda.stream(STREAM):
            base[half:].copy_(torch.from_numpy(mine.copy()).to("cuda", non_blocking=False))
        STREAM.synchronize()
        win.fence(stream=STREAM)
        back = zeros(nbytes - half)
        win.get(back, prv, half, stream=STREAM)
        win.fence(stream=STREAM, blocking=True)
        ok, msg = eq(host(back), payload(prv, salt + 2, nbytes - half), "fence: peer's local stores in the public copy")
        if not ok:
            return ok, msg
        # 3. passive target: a put under lock_all, seen after MPI_Win_sync
        tail = dev(payload(rank, salt + 3, 4099))
        win.lock_all(stream=STREAM)
        win.put(tail, nxt, 7, 4099, stream=STREAM)
        win.unlock_all(stream=STREAM, blocking=True)
        comm_barrier()
        win.sync(stream=STREAM)
        exp[half:] = payload(rank, salt + 2, nbytes - half)
        exp[7:7 + 4099] = payload(prv, salt + 3, 4099)
        ok, msg = eq(host(base), exp, "win_sync: passive put in the private copy")
        if not ok:
            return ok, msg
        comm_barrier()
        # 4. a lock of my own window synchronises too
        tail2 = dev(payload(rank, salt + 4, 999))
        win.lock(nxt, osc.LOCK_EXCLUSIVE, stream=STREAM)
        win.put(tail2, nxt, nbytes - 999, 999, stream=STREAM)
        win.unlock(nxt, stream=STREAM, blocking=True)
        comm_barrier()
        win.lock(rank, osc.LOCK_SHARED, stream=STREAM)
        win.unlock(rank, stream=STREAM, blocking=True)
        exp[nbytes - 999:] = payload(prv, salt + 4, 999)
        ok, msg = eq(host(base), exp, "lock of the own window: passive put in the private copy")
        comm_barrier()
        return ok, msg
    finally:
        win.free()


def case_fetch_and_op_counter(comm, rank, n, k=25):
    """Shared counter on rank 0: k fetch_and_op(+1) per rank; the fetched
    values over all ranks are exactly 0 .. n*k-1 (each increment atomic)."""
    I64 = mop.MPI_INT64_T
    win = osc.Window.allocate(comm, 64 if rank == 0 else 0, disp_unit=8)
    try:
        one = dev(np.array([1], np.int64))
        res = zeros(8 * k)
        win.fence(stream=STREAM)
        for i in range(k):
            win.fetch_and_op(one, res[8 * i:8 * i + 8], I64, 0, 0, mop.MPI_SUM, stream=STREAM)
        win.fence(stream=STREAM, blocking=True)
        mine = host(res).view(np.int64).tolist()
        everyone = [None] * n
        dist.all_gather_object(everyone, mine)
        allv = sorted(v for lst in everyone for v in lst)
        if allv != list(range(n * k)):
            return False, f"fetched values not a permutation: {allv[:10]}..."
        if rank == 0:
            t = torch.empty(8, dtype=torch.uint8, device="cuda")
            win.get(t, 0, 0, stream=STREAM)
            if int(host(t).view(np.int64)[0]) != n * k:
                return False, f"counter {host(t).view(np.int64)[0]}"
        return True, ""
    finally:
        win.free()


def case_cas(comm, rank, n):
    """compare_and_swap(-1 -> rank) on rank 0: exactly one winner."""
    I32 = mop.MPI_INT32_T
    base = dev(np.array([-1, 0, 0, 0], np.int32))
    win = osc.Window.create(comm, base, 16, disp_unit=4)
    try:
        org = dev(np.array([rank], np.int32))
        cmp = dev(np.array([-1], np.int32))
        res = zeros(4)
        win.fence(stream=STREAM)
        win.compare_and_swap(org, cmp, res, I32, 0, 0, stream=STREAM)
        win.fence(stream=STREAM, blocking=True)
        got = int(host(res).view(np.int32)[0])
        everyone = [None] * n
        dist.all_gather_object(everyone, got)
        winners = [r for r, v in enumerate(everyone) if v == -1]
        if len(winners) != 1:
            return False, f"results {everyone}"
        w = winners[0]
        if any(v != w for r, v in enumerate(everyone) if r != w):
            return False, f"losers must see the winner {w}: {everyone}"
        if rank == 0 and int(host(base).view(np.int32)[0]) != w:
            return False, f"target holds {host(base).view(np.int32)[0]}, winner {w}"
        return True, ""
    finally:
        win.free()


def case_passive_acc_all_to_all(comm, rank, n, salt, count=20011, rounds=6, small=1001):
    """Passive target under contention: every round, every rank opens
    lock_all and accumulates (SUM, exact data) its origin into the SAME
    region of EVERY rank's window — the whole region (kernels behind a lock
    kernel) and its first `small` elements (the single-launch form that
    takes the lock inside its kernel), so both forms contend for each
    target's accumulate lock — flushes, closes; a second region takes a
    put from the next rank under an exclusive lock of that target.  Every
    target's accumulate lock serialises the n concurrent updates; after the
    last round each window holds init + rounds x sum of the origins
    (bit-exact: exact data) and the last put, checked after MPI_Win_sync."""
    F = mop.MPI_FLOAT
    nxt, prv = (rank + 1) % n, (rank - 1) % n
    init = fp_inputs(F, count, 99, salt, "E")
    org = [fp_inputs(F, count, r, salt + 1, "E") for r in range(n)]
    base = dev(np.concatenate([init, np.zeros(count, np.float32)]))
    win = osc.Window.create(comm, base, base.numel(), disp_unit=4)
    try:
        o = dev(org[rank])
        comm_barrier()
        for rd in range(rounds):
            win.lock_all(stream=STREAM)
            for t in range(n):
                win.accumulate(o, count, F, (rank + t) % n, 0, mop.MPI_SUM, stream=STREAM)
                win.accumulate(o, small, F, (rank + t) % n, 0, mop.MPI_SUM, stream=STREAM)
            for t in range(n):
                win.flush(t, stream=STREAM)
            win.unlock_all(stream=STREAM)
            mark = dev(np.full(count, rd * 1000 + rank, np.float32))
            win.lock(nxt, osc.LOCK_EXCLUSIVE, stream=STREAM)
            win.put(mark, nxt, count, count * 4, stream=STREAM)
            win.unlock(nxt, stream=STREAM, blocking=True)
        comm_barrier()
        win.sync(stream=STREAM)
        got = host(base).view(np.float32)
        exp = init.copy()
        total = np.zeros(count, np.float32)
        for r in range(n):
            orc.op_2buff(mop.MPI_SUM.index, F.code, org[r].copy(), total, count)
        for _ in range(rounds):
            orc.op_2buff(mop.MPI_SUM.index, F.code, total.copy(), exp, count)
            head = exp[:small].copy()
            orc.op_2buff(mop.MPI_SUM.index, F.code, total[:small].copy(), head, small)
            exp[:small] = head
        ok, msg = eq(got[:count], exp, "accumulated region")
        if not ok:
            # exact data: any order gives the same bits; a difference is a lost or doubled update
            return ok, msg
        return eq(got[count:], np.full(count, (rounds - 1) * 1000 + prv, np.float32), "last put")
    finally:
        win.free()


def case_passive_exclusive(comm, rank, n, k=10):
    """Read-modify-write of a counter under MPI_Win_lock(EXCLUSIVE): get,
    +1 on the device, put, unlock — k times per rank; final = n*k."""
    win = osc.Window.allocate(comm, 8 if rank == 0 else 0, disp_unit=8)
    try:
        comm_barrier()
        buf = zeros(8).view(torch.int64)
        for _ in range(k):
            win.lock(0, osc.LOCK_EXCLUSIVE, stream=STREAM)
            win.get(buf, 0, 0, 8, stream=STREAM)
            with torch.cuda.stream(STREAM):
                buf.add_(1)
            win.put(buf, 0, 0, 8, stream=STREAM)
            win.unlock(0, stream=STREAM, blocking=True)
        comm_barrier()
        if rank == 0:
            win.lock(0, osc.LOCK_SHARED, stream=STREAM)
            win.get(buf, 0, 0, 8, stream=STREAM)
            win.unlock(0, stream=STREAM, blocking=True)
            if int(host(buf)[0]) != n * k:
                return False, f"counter {int(host(buf)[0])} != {n * k}"
        return True, ""
    finally:
        win.free()


def case_lock_all(comm, rank, n, salt, nbytes=100003):
    """lock_all (shared), get every rank's window, flush, unlock_all."""
    base = dev(payload(rank, salt, nbytes))
    win = osc.Window.create(comm, base, nbytes)
    try:
        comm_barrier()
        outs = [zeros(nbytes) for _ in range(n)]
        win.lock_all(stream=STREAM)
        for p in range(n):
            win.get(outs[p], p, 0, stream=STREAM)
        win.flush(0, stream=STREAM)
        win.unlock_all(stream=STREAM)
        for p in range(n):
            ok, msg = eq(host(outs[p]), payload(p, salt, nbytes), f"rank {p}")
            if not ok:
                return ok, msg
        return True, ""
    finally:
        win.free()


def case_pscw_ring(comm, rank, n, salt, nbytes=200003, epochs=3, use_test=False):
    """General active target (osc_sm_active_target.c:126-335): each rank
    exposes its window to the previous rank (post [prv]) and accesses the
    next one (start [nxt]), puts, completes and waits; `epochs` epochs in a
    row (the counters are cumulative), the last one closed by MPI_Win_test
    when use_test."""
    nxt, prv = (rank + 1) % n, (rank - 1) % n
    base = zeros(nbytes)
    win = osc.Window.create(comm, base, nbytes)
    try:
        for e in range(epochs):
            src = dev(payload(rank, salt + e, nbytes))
            win.post([prv], stream=STREAM)
            win.start([nxt], stream=STREAM)
            win.put(src, nxt, 0, nbytes, stream=STREAM)
            win.complete(stream=STREAM)
            if use_test and e == epochs - 1:
                STREAM.synchronize()
                import time
                t0, done = time.time(), False
                while not done and time.time() - t0 < 20:
                    done = win.test()
                if not done:
                    return False, "MPI_Win_test never saw the origin complete"
                torch.cuda.synchronize()
            else:
                win.wait(stream=STREAM, blocking=True)
            ok, msg = eq(host(base), payload(prv, salt + e, nbytes), f"epoch {e}")
            if not ok:
                return ok, msg
            comm_barrier()  # the next epoch overwrites what was just checked
        return True, ""
    finally:
        win.free()


def case_osc_random_epochs(comm, rank, n, salt, epochs=10, separate=False):
    """A seeded random sequence of access epochs of every kind (fence, a
    lock_all passive epoch closed by unlock_all and a barrier, a PSCW ring
    epoch, an exclusive lock of one target), each with a random set of
    operations per origin — puts into the slots of each target's put area
    this origin owns (slot s belongs to origin s mod N: no two origins write
    one slot in an epoch), gets of owned slots it does not put to in the
    same epoch (their value is the one from before the epoch), accumulates
    (SUM, exact small integers) anywhere in the accumulate area, sizes from
    one element to 64 Ki — replayed on a CPU model of every window.  Gets
    checked when their epoch closes; every window checked at the end."""
    F = mop.MPI_FLOAT
    slot, nslots = 1024, 8 * n  # floats per put slot; slots per window
    put_n, acc_n = slot * nslots, 1 << 17
    W = put_n + acc_n
    rng = np.random.default_rng(SEED + salt)  # the plan: the same on every rank
    model = [np.zeros(W, np.float32) for _ in range(n)]
    base = zeros(W * 4)
    w0 = comm.get_param("osc_shadow_windows")
    if separate:  # every window through a public copy (the separate model)
        comm.set_param("osc_win_shadow", 1)
    try:
        win = osc.Window.create(comm, base, W * 4, disp_unit=4)
    finally:
        if separate:
            comm.set_param("osc_win_shadow", 0)
    shadowed = comm.get_param("osc_shadow_windows") - w0  # this rank's window through a public copy
    fails = []
    diag = os.environ.get("OSC_DIAG") == "1"  # every copy checked at every epoch close
    diag_end = os.environ.get("OSC_DIAG") == "2"  # the copies checked once, at the end (no extra syncs)
    mine_ops = []  # (epoch, kind, origin, what, disp, count) aimed at this rank
    all_ops = []   # (epoch, kind, origin, what, target, disp, count, seed): the whole plan so far

    def raw(addr):
        out = np.empty(W * 4, np.uint8)
        _lib.check(_lib.load().ompi_amd_memcpy(out.ctypes.data, addr, W * 4), "memcpy")
        return out

    def check_copies(e, kind):
        STREAM.synchronize()
        torch.cuda.synchronize()
        priv, pub, snap = win.copies()
        want = model[rank].view(np.uint8)
        got = {"priv": raw(priv)}
        if pub:
            got["pub"], got["snap"] = raw(pub), raw(snap)
        notes = []
        if pub and not np.array_equal(got["pub"], want):
            bad = np.flatnonzero(got["pub"] != want)
            notes.append(f"public != model: {bad.size} bytes from {bad[0]}")
        if pub and not np.array_equal(got["priv"], got["snap"]):
            bad = np.flatnonzero(got["priv"] != got["snap"])
            notes.append(f"private != snapshot: {bad.size} bytes from {bad[0]}")
        if not pub and not np.array_equal(got["priv"], want):
            bad = np.flatnonzero(got["priv"] != want)
            notes.append(f"unified window != model: {bad.size} bytes from {bad[0]}")
        if notes:
            first = int(bad[0]) // 4
            near = [op for op in mine_ops if op[4] <= first < op[4] + op[5]]
            src = got["pub"] if pub else got["priv"]
            gv = float(src.view(np.float32)[first])
            mv = float(model[rank][first])
            # which planned operation (any target) puts gv at this offset?
            cands = []
            for (ee, kk, oo, ww, tt, dd, cc, sd) in all_ops:
                if ww == "put" and dd <= first < dd + cc:
                    v = np.random.default_rng(sd).integers(-64, 65, cc).astype(np.float32)[first - dd]
                    if float(v) == gv:
                        cands.append((ee, kk, oo, tt, dd, cc))
            notes.append(f"at float {first}: public {gv} model {mv}; puts of that value there: {cands[:6]}")
            line = (f"DIAG rank {rank} epoch {e} ({kind}, shadowed {shadowed}): " + "; ".join(notes) +
                    f"; ops on float {first}: {near[-6:]}")
            print(line, file=sys.stderr, flush=True)
            fails.append(line)
            return False
        return True
    if separate and win.model != osc.WIN_SEPARATE:
        fails.append(f"model {win.model}, want WIN_SEPARATE")
    try:
        comm_barrier()
        if diag:  # a failed check is recorded; every rank goes on (the epochs are collective)
            check_copies(-1, "create")
            # every rank's mapping of every peer's window reaches that peer's
            # RMA target: each rank stamps its own (public) copy, peers read
            lib = _lib.load()
            priv, pub, snap = win.copies()
            mine = pub or priv
            stamp = np.full(64, rank + 1, np.uint8)
            _lib.check(lib.ompi_amd_memcpy(mine, stamp.ctypes.data, 64), "stamp")
            torch.cuda.synchronize()
            comm_barrier()
            for p in range(n):
                got = np.zeros(64, np.uint8)
                _lib.check(lib.ompi_amd_memcpy(got.ctypes.data, win.peer_base(p), 64), "read stamp")
                if not np.all(got == p + 1):
                    line = f"DIAG rank {rank}: mapping of rank {p}'s window holds stamp {got[:4].tolist()}"
                    print(line, file=sys.stderr, flush=True)
                    fails.append(line)
            comm_barrier()
            _lib.check(lib.ompi_amd_memcpy(mine, np.zeros(64, np.uint8).ctypes.data, 64), "unstamp")
            torch.cuda.synchronize()
            comm_barrier()
        for e in range(epochs):
            kind = ["fence", "lock_all", "pscw", "lock_one"][int(rng.integers(4))]
            excl = int(rng.integers(n))  # lock_one: every origin's target
            ops = []  # (origin, what, target, disp, count, data seed)
            for o in range(n):
                targets = ([(o + 1) % n] if kind == "pscw" else [excl] if kind == "lock_one"
                           else list(range(n)))
                owned = [sl for sl in range(nslots) if sl % n == o]
                for _ in range(int(rng.integers(1, 5))):
                    t = targets[int(rng.integers(len(targets)))]
                    what = ["put", "get", "acc", "acc"][int(rng.integers(4))]
                    if what == "acc":
                        cnt = int(rng.choice([1, 7, 1000, 65536]))
                        ops.append((o, "acc", t, put_n + int(rng.integers(acc_n - cnt + 1)), cnt,
                                    int(rng.integers(1 << 30))))
                    else:
                        sl = owned[int(rng.integers(len(owned)))]
                        cnt = int(rng.integers(1, slot + 1))
                        ops.append((o, what, t, sl * slot, cnt, int(rng.integers(1 << 30))))
            # two puts, or a get and a put, of one (origin, target, slot) in
            # one epoch would conflict (unordered): keep the first put, drop the get
            puts, kept = set(), []
            for op in ops:
                key = (op[0], op[2], op[3] // slot)
                if op[1] == "put":
                    if key in puts:
                        continue
                    puts.add(key)
                kept.append(op)
            ops = [op for op in kept if not (op[1] == "get" and (op[0], op[2], op[3] // slot) in puts)]
            before = [m.copy() for m in model]
            mine, keep = [], []
            if kind == "fence":
                win.fence(stream=STREAM)
            elif kind == "lock_all":
                win.lock_all(stream=STREAM)
            elif kind == "pscw":
                win.post([(rank - 1) % n], stream=STREAM)
                win.start([(rank + 1) % n], stream=STREAM)
            else:
                win.lock(excl, osc.LOCK_EXCLUSIVE, stream=STREAM)
            for o, what, t, d, cnt, sd in ops:
                vals = np.random.default_rng(sd).integers(-64, 65, cnt).astype(np.float32)
                if t == rank and what != "get":
                    mine_ops.append((e, kind, o, what, d, cnt))
                all_ops.append((e, kind, o, what, t, d, cnt, sd))
                if what == "put":
                    model[t][d:d + cnt] = vals
                elif what == "acc":
                    model[t][d:d + cnt] += vals
                if o != rank:
                    continue
                if what == "get":
                    buf = zeros(cnt * 4)
                    win.get(buf, t, d, cnt * 4, stream=STREAM)
                    mine.append((buf, before[t][d:d + cnt].copy(), f"epoch {e} ({kind}) get from {t}@{d}"))
                else:
                    src = dev(vals)
                    keep.append(src)
                    if what == "put":
                        win.put(src, t, d, cnt * 4, stream=STREAM)
                    else:
                        win.accumulate(src, cnt, F, t, d, mop.MPI_SUM, stream=STREAM)
            if kind == "fence":
                win.fence(stream=STREAM, blocking=True)
            elif kind == "lock_all":
                win.unlock_all(stream=STREAM)
                comm_barrier()
            elif kind == "pscw":
                win.complete(stream=STREAM)
                win.wait(stream=STREAM, blocking=True)
                comm_barrier()  # every origin's epoch closed before the next one starts
            else:
                win.unlock(excl, stream=STREAM)
                comm_barrier()
            for buf, exp, what in mine:
                ok, msg = eq(host(buf).view(np.float32), exp, f"{what} (model {win.model})")
                if not ok:
                    fails.append(msg)
            if diag:  # every rank's check between two barriers: passive epochs start at once
                comm_barrier()
                check_copies(e, kind)
                comm_barrier()
        win.fence(stream=STREAM, blocking=True)
        comm_barrier()
        win.sync(stream=STREAM)  # MPI_Win_sync: the private copy of a separate-model window
        STREAM.synchronize()
        ok, msg = eq(host(base).view(np.float32), model[rank],
                     f"window of rank {rank} (model {win.model}, shadowed here {shadowed})")
        if not ok:
            fails.append(msg)
        if diag_end and not ok:
            torch.cuda.synchronize()
            priv, pub, snap = win.copies()
            cp = {"priv": raw(priv)}
            if pub:
                cp["pub"], cp["snap"] = raw(pub), raw(snap)
            want = model[rank].view(np.uint8)
            parts = []
            for k, v in cp.items():
                badk = np.flatnonzero(v != want)
                parts.append(f"{k}: {badk.size} bad" + (f" from {badk[0]}" if badk.size else ""))
            bad = np.flatnonzero(cp["priv"] != want)
            fl = sorted(set((bad // 4).tolist()))
            first = fl[0]
            runs, st = [], fl[0]
            for a, b in zip(fl, fl[1:] + [None]):
                if b != a + 1:
                    runs.append((st, a))
                    st = b
            gotv = cp["priv"].view(np.float32)
            near = [op for op in mine_ops if any(op[4] <= r0 < op[4] + op[5] or r0 <= op[4] <= r1
                                                 for r0, r1 in runs[:4])]
            line = (f"DIAG2 rank {rank}: " + "; ".join(parts) + f"; bad float runs {runs[:6]}; "
                    f"priv {gotv[first]} model {model[rank][first]}; ops there {near[:8]}")
            print(line, file=sys.stderr, flush=True)
            fails.append(line)
    finally:
        win.free()
    return not fails, "; ".join(fails[:3])


def case_separate_refused(comm, rank, n):
    """osc_win_separate 0 (osc/rocm's osc_rocm_separate_model 0): an
    MPI_Win_create window over memory peers cannot map as it is (a small
    tensor: not an IPC-safe size) fails on every rank with
    OMPI_AMD_ERR_UNSUPPORTED instead of running through a public copy; a
    window over an exportable allocation still works (unified)."""
    comm.set_param("osc_win_separate", 0)
    try:
        small = zeros(4096 + 12)
        try:
            w = osc.Window.create(comm, small, small.numel(), disp_unit=1)
            w.free()
            return False, "a window needing a public copy was created with the separate model off"
        except _lib.OmpiAmdError as e:
            if e.code != _lib.ERR_UNSUPPORTED:
                return False, f"refusal code {e.code}"
        w = osc.Window.allocate(comm, 4096, disp_unit=1)
        try:
            if w.model != osc.WIN_UNIFIED:
                return False, f"allocated window model {w.model}"
        finally:
            w.free()
        return True, ""
    finally:
        comm.set_param("osc_win_separate", 1)


def case_dynamic_window(comm, rank, n, salt):
    """MPI_Win_create_dynamic / MPI_Win_attach / MPI_Win_detach over device
    memory (osc/rdma's flavor, osc_rdma_dynamic.c:162-300): each rank
    attaches a 4 MiB hipMalloc region and shares its address; puts,
    accumulates (SUM fp32) and gets at absolute addresses under fence and
    lock_all epochs reach exactly the attached regions; a second region
    attached later is found; host memory and memory peers cannot map (a small
    tensor) are refused at attach; an access outside every attached region
    and one into a detached region are refused at the call."""
    lib = _lib.load()
    F = mop.MPI_FLOAT
    nxt, prv = (rank + 1) % n, (rank - 1) % n
    R = 4 << 20
    regions, failures = [], []

    def region(seed):
        for _ in range(3):  # a fresh address (never exported before) is exportable
            p = ctypes.c_void_p()
            _lib.check(lib.ompi_amd_device_alloc(ctypes.byref(p), R), "device_alloc")
            regions.append(p.value)
            init = payload(rank, seed, R)
            _lib.check(lib.ompi_amd_memcpy(p.value, init.ctypes.data, R), "fill")
            try:
                win.attach(p.value, R)
                return p.value, init
            except _lib.OmpiAmdError as e:
                if e.code != _lib.ERR_UNSUPPORTED:
                    raise
        raise RuntimeError("no exportable 4 MiB region in three tries")

    def raw(addr, nb):
        out = np.empty(nb, np.uint8)
        _lib.check(lib.ompi_amd_memcpy(out.ctypes.data, addr, nb), "read")
        return out

    win = osc.Window.create_dynamic(comm)
    try:
        a, init = region(salt)
        addrs = [None] * n
        dist.all_gather_object(addrs, a)  # the application shares the address (MPI_Get_address + a send)
        inits = [payload(r, salt, R) for r in range(n)]
        pb, acc_n, gb = 65536 + 13, 100001, 4096
        src = dev(payload(rank, salt + 1, pb))
        accv = fp_inputs(F, acc_n, rank, salt + 2, "E")
        acc = dev(accv)
        got = zeros(gb)
        comm_barrier()
        win.fence(stream=STREAM)
        win.put(src, nxt, addrs[nxt] + 1000, pb, stream=STREAM)
        win.accumulate(acc, acc_n, F, nxt, addrs[nxt] + (2 << 20), mop.MPI_SUM, stream=STREAM)
        win.get(got, nxt, addrs[nxt] + (3 << 20), gb, stream=STREAM)
        win.fence(stream=STREAM, blocking=True)
        comm_barrier()
        exp = init.copy()
        exp[1000:1000 + pb] = payload(prv, salt + 1, pb)
        cur = exp[2 << 20:(2 << 20) + acc_n * 4].view(np.float32).copy()
        orc.op_2buff(mop.MPI_SUM.index, F.code, fp_inputs(F, acc_n, prv, salt + 2, "E").copy(), cur, acc_n)
        exp[2 << 20:(2 << 20) + acc_n * 4] = cur.view(np.uint8)
        ok, msg = eq(raw(a, R), exp, "fence epoch: attached region")
        if not ok:
            failures.append(msg)
        ok, msg = eq(host(got), inits[nxt][3 << 20:(3 << 20) + gb], "fence epoch: get")
        if not ok:
            failures.append(msg)
        # a second region, attached later, under lock_all
        b, init_b = region(salt + 5)
        addrs_b = [None] * n
        dist.all_gather_object(addrs_b, b)
        src2 = dev(payload(rank, salt + 6, 12345))
        comm_barrier()
        win.lock_all(stream=STREAM)
        win.put(src2, nxt, addrs_b[nxt] + 777, 12345, stream=STREAM)
        win.unlock_all(stream=STREAM)
        comm_barrier()
        exp_b = init_b.copy()
        exp_b[777:777 + 12345] = payload(prv, salt + 6, 12345)
        ok, msg = eq(raw(b, R), exp_b, "lock_all epoch: second region")
        if not ok:
            failures.append(msg)
        # refusals at attach and at the access
        hostbuf = np.zeros(1 << 22, np.uint8)
        small = zeros(4096 + 12)
        for what, fn, code in (
                ("attach of host memory", lambda: win.attach(hostbuf.ctypes.data, hostbuf.nbytes),
                 _lib.ERR_NOT_DEVICE),
                ("attach of memory peers cannot map", lambda: win.attach(small), _lib.ERR_UNSUPPORTED),
                ("put outside every attached region",
                 lambda: win.put(src2, nxt, addrs[nxt] + R + 64, 256, stream=STREAM), _lib.ERR_BAD_PARAM),
                ("put across a region's end",
                 lambda: win.put(src2, nxt, addrs[nxt] + R - 100, 256, stream=STREAM), _lib.ERR_BAD_PARAM)):
            try:
                fn()
                failures.append(what + " accepted")
            except _lib.OmpiAmdError as e:
                if e.code != code:
                    failures.append(f"{what}: code {e.code}, want {code}")
        win.detach(b)
        comm_barrier()  # every rank detached its second region
        try:
            win.put(src2, nxt, addrs_b[nxt] + 777, 64, stream=STREAM)
            failures.append("put into a detached region accepted")
        except _lib.OmpiAmdError as e:
            if e.code != _lib.ERR_BAD_PARAM:
                failures.append(f"put into a detached region: code {e.code}")
        win.detach(a)
        STREAM.synchronize()
    finally:
        comm_barrier()
        win.free()
        for p_ in regions:
            lib.ompi_amd_device_free(p_)
    return not failures, "; ".join(failures[:3])


def case_pscw_all_to_one(comm, rank, n, salt, count=100003):
    """Rank 0 posts to every other rank; each origin accumulates (SUM, exact
    data) into its own slice of rank 0's window, then rank 0 waits: every
    slice is bit-exact vs op/base, with rank 0 reading right after wait."""
    F = mop.MPI_FLOAT
    init = fp_inputs(F, count * n, 99, salt, "E")
    org = [fp_inputs(F, count, r, salt + 1, "E") for r in range(n)]
    base = dev(init if rank == 0 else np.zeros(0, np.float32), extra=16)
    win = osc.Window.create(comm, base, base.numel(), disp_unit=4)
    try:
        if rank == 0:
            win.post(range(1, n), stream=STREAM)
            win.wait(stream=STREAM, blocking=True)
            exp = init.copy()
            for r in range(1, n):
                sl = exp[r * count:(r + 1) * count]
                orc.op_2buff(mop.MPI_SUM.index, F.code, org[r].copy(), sl, count)
            return eq(host(base)[:count * n * 4].view(np.float32), exp, "slices")
        o = dev(org[rank])
        win.start([0], stream=STREAM)
        win.accumulate(o, count, F, 0, rank * count, mop.MPI_SUM, stream=STREAM)
        win.complete(stream=STREAM, blocking=True)
        return True, ""
    finally:
        win.free()


def case_pscw_errors(comm, rank, n):
    """Epoch calls out of order return OMPI_AMD_ERR_RMA_SYNC
    (osc_sm_active_target.c:137-140, 191-193, 230-233, 279-282, 314-317)."""
    win = osc.Window.allocate(comm, 64, disp_unit=1)
    bad = []
    try:
        for what, fn in (("complete without start", lambda: win.complete(stream=STREAM)),
                         ("wait without post", lambda: win.wait(stream=STREAM)),
                         ("test without post", lambda: win.test())):
            try:
                fn()
                bad.append(what + " accepted")
            except _lib.OmpiAmdError as e:
                if e.code != _lib.ERR_RMA_SYNC:
                    bad.append(f"{what}: code {e.code}")
        # an epoch of the empty group: post / start / complete / wait pass
        win.post([], stream=STREAM)
        try:
            win.post([], stream=STREAM)
            bad.append("second post accepted")
        except _lib.OmpiAmdError as e:
            if e.code != _lib.ERR_RMA_SYNC:
                bad.append(f"second post: code {e.code}")
        win.start([], stream=STREAM)
        win.complete(stream=STREAM)
        win.wait(stream=STREAM, blocking=True)
        return not bad, "; ".join(bad)
    finally:
        win.free()


def case_request_rma(comm, rank, n, salt, count=65537):
    """MPI_Rput / _Raccumulate / _Rget / _Rget_accumulate under lock_all:
    each request completes (test / wait) once its kernels ran; the windows
    then hold exactly the puts and the op/base sums."""
    F = mop.MPI_FLOAT
    nxt, prv = (rank + 1) % n, (rank - 1) % n
    init = [fp_inputs(F, 3 * count, r, salt, "E") for r in range(n)]
    org = [fp_inputs(F, count, r, salt + 1, "E") for r in range(n)]
    org2 = [fp_inputs(F, count, r, salt + 2, "E") for r in range(n)]
    src = [fp_inputs(F, count, r, salt + 3, "E") for r in range(n)]
    base = dev(init[rank])
    win = osc.Window.create(comm, base, 3 * count * 4, disp_unit=4)
    try:
        comm_barrier()
        s, o, o2 = dev(src[rank]), dev(org[rank]), dev(org2[rank])
        back, res = zeros(count * 4), zeros(count * 4)
        win.lock_all(stream=STREAM)
        r1 = win.rput(s, nxt, 0, count * 4, stream=STREAM)
        r2 = win.raccumulate(o, count, F, nxt, count, mop.MPI_SUM, stream=STREAM)
        r3 = win.rget(back, nxt, 2 * count, count * 4, stream=STREAM)
        r4 = win.rget_accumulate(o2, res, count, F, nxt, count, mop.MPI_SUM, stream=STREAM)
        import time
        t0, done = time.time(), False
        while not done and time.time() - t0 < 20:
            done = r1.test()
        for r in (r2, r3, r4):
            r.wait()
        if not (done and r2.test() and r3.test() and r4.test()):
            return False, "a request never completed"
        for r in (r1, r2, r3, r4):
            r.free()
        win.unlock_all(stream=STREAM)
        comm_barrier()
        win.sync(stream=STREAM)  # MPI_Win_sync: the separate model's private copy
        mine = host(base).view(np.float32)
        ok, msg = eq(mine[:count], src[prv], "rput")
        if not ok:
            return ok, msg
        b = init[rank][count:2 * count].copy()
        orc.op_2buff(mop.MPI_SUM.index, F.code, org[prv].copy(), b, count)
        exp_res = init[nxt][count:2 * count].copy()
        orc.op_2buff(mop.MPI_SUM.index, F.code, org[rank].copy(), exp_res, count)
        orc.op_2buff(mop.MPI_SUM.index, F.code, org2[prv].copy(), b, count)
        ok, msg = eq(mine[count:2 * count], b, "raccumulate + rget_accumulate")
        if not ok:
            return ok, msg
        ok, msg = eq(host(back).view(np.float32), init[nxt][2 * count:], "rget")
        if not ok:
            return ok, msg
        return eq(host(res).view(np.float32), exp_res, "rget_accumulate fetched")
    finally:
        win.free()


def case_shared_window(comm, rank, n, salt, noncontig=False):
    """MPI_Win_allocate_shared (osc_sm_component.c:244-360): segments of
    different sizes (one empty), each written by its owner with plain
    device copies and read by every rank through MPI_Win_shared_query's
    address; contiguous unless noncontig; MPI_PROC_NULL = the first
    nonzero segment; put into a shared window; shared_query on a window of
    another flavor is refused."""
    lib = _lib.load()
    sizes = [0 if (n > 2 and r == 1) else 1000 * (r + 1) + 3 * (r % 2) for r in range(n)]
    seg = [((z + 4095) // 4096 * 4096 if noncontig else z) for z in sizes]
    win = osc.Window.allocate_shared(comm, sizes[rank], disp_unit=1, noncontig=noncontig)
    try:
        mine = payload(rank, salt, sizes[rank])
        if sizes[rank]:
            _lib.check(lib.ompi_amd_memcpy(win.base_ptr, mine.ctypes.data, sizes[rank]), "memcpy")
        comm_barrier()
        addrs = []
        for p in range(n):
            size, du, addr = win.shared_query(p)
            if size != seg[p] or du != 1:
                return False, f"rank {p}: size {size} disp {du}, expected {seg[p]} / 1"
            if p == rank and addr != win.base_ptr:
                return False, "own segment address differs from the allocation's base"
            addrs.append(addr)
            if sizes[p]:
                got = np.empty(sizes[p], np.uint8)
                _lib.check(lib.ompi_amd_memcpy(got.ctypes.data, addr, sizes[p]), "memcpy back")
                ok, msg = eq(got, payload(p, salt, sizes[p]), f"segment {p}")
                if not ok:
                    return ok, msg
        for p in range(n - 1):
            if addrs[p + 1] != addrs[p] + seg[p]:
                return False, f"segments {p}, {p + 1} not back to back"
        first = next(p for p in range(n) if sizes[p])
        if win.shared_query(-1) != (seg[first], 1, addrs[first]):
            return False, f"MPI_PROC_NULL query {win.shared_query(-1)}"
        # RMA into the shared window: put into the next nonempty segment
        tgt = next(p for p in [(rank + k) % n for k in range(1, n + 1)] if sizes[p])
        src_rank = [r for r in range(n) if next(p for p in [(r + k) % n for k in range(1, n + 1)]
                                                 if sizes[p]) == rank]
        m = min(sizes[tgt], 512)
        src = dev(payload(rank, salt + 1, m))
        win.fence(stream=STREAM)
        if m:
            win.put(src, tgt, 0, m, stream=STREAM)
        win.fence(stream=STREAM, blocking=True)
        if sizes[rank] and src_rank:
            got = np.empty(sizes[rank], np.uint8)
            _lib.check(lib.ompi_amd_memcpy(got.ctypes.data, win.base_ptr, sizes[rank]), "memcpy")
            w = max(src_rank)  # several writers: the last fence orders nothing among them
            if len(src_rank) == 1:
                mm = min(sizes[rank], 512)
                exp = mine.copy()
                exp[:mm] = payload(w, salt + 1, mm)
                ok, msg = eq(got, exp, "put into the shared window")
                if not ok:
                    return ok, msg
        other = osc.Window.allocate(comm, 64, disp_unit=1)
        try:
            other.shared_query(0)
            return False, "shared_query on an MPI_Win_allocate window accepted"
        except _lib.OmpiAmdError as e:
            if e.code != _lib.ERR_UNSUPPORTED:
                return False, f"shared_query on another flavor: code {e.code}"
        finally:
            other.free()
        return True, ""
    finally:
        win.free()


def comm_barrier():
    STREAM.synchronize()
    dist.barrier()


def main():
    # a hung rank's Python stack, on the launcher's SIGUSR1 (test_coll_gpu.run_ranks)
    faulthandler.register(signal.SIGUSR1, all_threads=True)
    # a rank stuck for a minute prints every thread's stack (then again each
    # minute), as coll_worker.py does
    faulthandler.dump_traceback_later(60, repeat=True, file=sys.stderr)
    if os.environ.get("OMPI_AMD_BACKTRACE") == "1":  # ... and its native stack
        import threading

        def native_dumps():
            while True:
                time.sleep(60)
                os.kill(os.getpid(), signal.SIGUSR2)
        threading.Thread(target=native_dumps, daemon=True).start()
    global STREAM
    rank, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    device = int(os.environ.get("OMPI_AMD_DEVICE", "0"))
    torch.cuda.set_device(device)
    STREAM = torch.cuda.Stream()
    dist.init_process_group("gloo", rank=rank, world_size=n)
    comm = coll.Communicator.from_torch_distributed(device=device)
    comm.set_param("timeout_ms", 20000)
    F, D, I32, I64, DI, U8 = (mop.MPI_FLOAT, mop.MPI_DOUBLE, mop.MPI_INT32_T, mop.MPI_INT64_T,
                              mop.MPI_DOUBLE_INT, mop.MPI_UINT8_T)
    cases = [
        ("p2p_ring_0B", lambda: case_ring(comm, rank, n, 0, 1)),
        ("p2p_ring_1B", lambda: case_ring(comm, rank, n, 1, 2)),
        ("p2p_ring_4099B_misaligned", lambda: case_ring(comm, rank, n, 4099, 3, soff=3, roff=5)),
        ("p2p_ring_64MiB", lambda: case_ring(comm, rank, n, 64 << 20, 4)),
        ("p2p_ring_16MiB_plus_odd", lambda: case_ring(comm, rank, n, (16 << 20) + 13, 5, 16, 16)),
        ("p2p_aged_buffer_staged", lambda: case_aged_buffer_staged(comm, rank, n, 6)),
        ("p2p_stage_cap_aged", lambda: case_stage_cap_aged(comm, rank, n, 8)),
        ("p2p_tags_out_of_order", lambda: case_tags_out_of_order(comm, rank, n, 6)),
        ("p2p_same_tag_order", lambda: case_same_tag_order(comm, rank, n, 20)),
        ("p2p_ring_wraps_eager_and_staged", lambda: case_ring_wraps(comm, rank, n, 400)),
        ("p2p_any_source_any_tag", lambda: case_any_source(comm, rank, n, 70)),
        ("p2p_fan_in_any_source_order", lambda: case_fan_in_any_source(comm, rank, n, 500)),
        ("p2p_random_channels", lambda: case_random_channels(comm, rank, n, 600 + STRESS_SEED)),
        ("p2p_random_channels_b", lambda: case_random_channels(comm, rank, n, 601 + STRESS_SEED)),
        ("p2p_random_channels_any_source", lambda: case_random_channels(comm, rank, n, 602 + STRESS_SEED, wild=0.3)),
        # right after the random point-to-point traffic (which ages the
        # allocator's blocks, so MPI_Win_create windows get public copies):
        # the plans that lost epoch-0 puts in round 5 (the window's initial
        # copies completing after peers' first RMA)
        ("osc_random_epochs_after_p2p_s3000", lambda: case_osc_random_epochs(comm, rank, n, 3700 + STRESS_SEED)),
        ("osc_random_epochs_after_p2p_s5000", lambda: case_osc_random_epochs(comm, rank, n, 5700 + STRESS_SEED)),
        ("p2p_probe_truncate", lambda: case_probe_truncate(comm, rank, n, 71)),
        ("p2p_self", lambda: case_self(comm, rank, n, 72)),
        ("p2p_recv_timeout_cancel", lambda: case_recv_timeout_cancel(comm, rank, n, 75)),
        ("p2p_eager_send_before_recv", lambda: case_eager_send_first(comm, rank, n, 73)),
        ("p2p_ssend_small_rendezvous", lambda: case_ssend_small(comm, rank, n, 74)),
        ("osc_put_get_small", lambda: case_put_get(comm, rank, n, 1001, 80)),
        ("osc_put_get_32MiB", lambda: case_put_get(comm, rank, n, 32 << 20, 81)),
        ("osc_acc_sum_f32", lambda: case_acc_disjoint(comm, rank, n, F, mop.MPI_SUM, 1000003, 82)),
        # MPIX_C_FLOAT16 accumulates (acc_kernel<_Float16>): 8 halves per 16-B vector
        ("osc_acc_sum_f16", lambda: case_acc_disjoint(comm, rank, n, mop.MPIX_C_FLOAT16, mop.MPI_SUM,
                                                      100003, 140)),
        ("osc_acc_max_f16_specials",
         lambda: case_acc_disjoint(comm, rank, n, mop.MPIX_C_FLOAT16, mop.MPI_MAX, 70001, 141, "S")),
        ("osc_acc_prod_f64", lambda: case_acc_disjoint(comm, rank, n, D, mop.MPI_PROD, 30001, 83)),
        ("osc_acc_max_f32_specials",
         lambda: case_acc_disjoint(comm, rank, n, F, mop.MPI_MAX, 100001, 84, "S")),
        ("osc_acc_min_f64_specials",
         lambda: case_acc_disjoint(comm, rank, n, D, mop.MPI_MIN, 20001, 85, "S")),
        ("osc_acc_band_i64", lambda: case_acc_disjoint(comm, rank, n, I64, mop.MPI_BAND, 7777, 86)),
        ("osc_acc_bxor_u8_odd", lambda: case_acc_disjoint(comm, rank, n, U8, mop.MPI_BXOR, 1237, 87)),
        ("osc_acc_maxloc_double_int",
         lambda: case_acc_disjoint(comm, rank, n, DI, mop.MPI_MAXLOC, 40001, 88)),
        ("osc_acc_concurrent_sum_f32_exact",
         lambda: case_acc_concurrent(comm, rank, n, F, mop.MPI_SUM, 262147, 89)),
        ("osc_acc_concurrent_sum_i32",
         lambda: case_acc_concurrent(comm, rank, n, I32, mop.MPI_SUM, 65537, 90)),
        ("osc_acc_concurrent_maxloc",
         lambda: case_acc_concurrent(comm, rank, n, DI, mop.MPI_MAXLOC, 30001, 91)),
        ("osc_get_accumulate", lambda: case_get_accumulate(comm, rank, n, 92)),
        ("osc_accumulate_derived_datatypes", lambda: case_acc_ddt(comm, rank, n, 150)),
        ("osc_put_get_derived_datatypes", lambda: case_put_get_ddt(comm, rank, n, 160)),
        ("osc_accumulate_derived_pair_types", lambda: case_acc_ddt_pair(comm, rank, n, 165)),
        ("osc_separate_model_small_tensor", lambda: case_separate_window(comm, rank, n, 170)),
        ("osc_separate_model_refused", lambda: case_separate_refused(comm, rank, n)),
        ("osc_separate_model_forced_64MiB",
         lambda: case_separate_window(comm, rank, n, 171, nbytes=(64 << 20) + 12, force=True)),
        ("osc_fetch_and_op_counter", lambda: case_fetch_and_op_counter(comm, rank, n)),
        ("osc_compare_and_swap", lambda: case_cas(comm, rank, n)),
        ("osc_passive_exclusive_rmw", lambda: case_passive_exclusive(comm, rank, n)),
        ("osc_passive_acc_all_to_all", lambda: case_passive_acc_all_to_all(comm, rank, n, 180)),
        ("osc_lock_all_get", lambda: case_lock_all(comm, rank, n, 93)),
        ("osc_pscw_ring", lambda: case_pscw_ring(comm, rank, n, 94)),
        ("osc_pscw_ring_test", lambda: case_pscw_ring(comm, rank, n, 95, epochs=2, use_test=True)),
        ("osc_pscw_all_to_one_acc", lambda: case_pscw_all_to_one(comm, rank, n, 96)),
        ("osc_pscw_errors", lambda: case_pscw_errors(comm, rank, n)),
        ("osc_random_epochs", lambda: case_osc_random_epochs(comm, rank, n, 700 + STRESS_SEED,
                                                             separate=os.environ.get("OSC_FORCE_SHADOW") == "1")),
        ("osc_random_epochs_b", lambda: case_osc_random_epochs(comm, rank, n, 701 + STRESS_SEED, epochs=16)),
        ("osc_random_epochs_separate", lambda: case_osc_random_epochs(comm, rank, n, 702 + STRESS_SEED,
                                                                      separate=True)),
        ("osc_request_rma", lambda: case_request_rma(comm, rank, n, 97)),
        ("osc_dynamic_window", lambda: case_dynamic_window(comm, rank, n, 99)),
        ("osc_shared_window", lambda: case_shared_window(comm, rank, n, 98)),
        ("osc_shared_window_noncontig", lambda: case_shared_window(comm, rank, n, 99, noncontig=True)),
        ("cross_layer_progress", lambda: case_cross_layer(comm, rank, n, 2100 + STRESS_SEED)),
    ]
    only = os.environ.get("P2P_OSC_ONLY")
    pick = os.environ.get("P2P_OSC_CASES")  # exact names, comma-separated, run in list order
    if pick:
        byname = dict(cases)
        cases = [(nm, byname[nm]) for nm in pick.split(",")]
    all_ok = True
    for name, fn in cases:
        if only and only not in name:
            continue
        comm_barrier()
        try:
            ok, msg = fn()
        except Exception as e:  # noqa: BLE001 - reported per case
            ok, msg = False, f"{type(e).__name__}: {e}\n{traceback.format_exc()[-1200:]}"
        all_ok &= bool(ok)
        # process resources after the case (diagnostics for IPC open failures)
        try:
            fds = len(os.listdir("/proc/self/fd"))
        except OSError:
            fds = -1
        line = json.dumps({"rank": rank, "case": name, "ok": bool(ok), "msg": msg, "fds": fds,
                           "ipc_live": comm.get_param("ipc_live"),
                           "ipc_opens": comm.get_param("ipc_opens"),
                           "ipc_refusals": comm.get_param("ipc_refusals")})
        print(line, flush=True)
        if os.environ.get("COLL_LOG_DIR"):  # progress visible while the test runs
            os.makedirs(os.environ["COLL_LOG_DIR"], exist_ok=True)
            with open(os.path.join(os.environ["COLL_LOG_DIR"], f"p2p_osc_n{n}_rank{rank}.jsonl"), "a") as f:
                f.write(line + "\n")
        if comm.error():
            print(json.dumps({"rank": rank, "case": name + "/sticky", "ok": False,
                              "msg": f"device error {comm.error()}"}), flush=True)
            all_ok = False
            break
    comm_barrier()
    comm.free()
    dist.destroy_process_group()
    sys.exit(0 if all_ok else 1)


if __name__ == "__main__":
    main()
