"""Reduce / reduce_scatter_block / scan operand orders (CPU only).

The device folds each element in closed form (coll_ipc.hip fold(): chain,
in-order binomial and binary trees in virtual-rank order).  Here that closed
form is restated in Python and checked bit-exactly against the oracle's
independent message-flow simulation of coll_base_reduce.c's generic tree
reduce + coll_base_topo.c's trees, for every comm size 2..16, every root,
with and without MPI_IN_PLACE at the root, on inputs where operand order
changes fp bits (signed random sums, MAX over NaN/±0).  The library's host
decision (ompi_amd_coll_reduce_order) is checked against the oracle's
restatement of coll_tuned_decision_fixed.c:354-428.

No reference execution of coll_base_reduce.c is available in this container
(it needs the configure-generated headers), so these orders are pinned by
the restated source only: see DESIGN.md §5.
"""
import numpy as np
import pytest

MAX, SUM = 1, 3
F32 = 15
CHAIN, BINOMIAL, BINARY = "chain", "binomial", "binary"


def f(orc, op, out, inb):
    """2-buffer rule f(out, in) through the oracle's op/base loop."""
    r = out.copy()
    orc.op_2buff(op, F32, inb, r, r.size)
    return r


def fold(orc, op, v, order, swap):
    """Python twin of coll_ipc.hip fold() for the reduce orders."""
    n = len(v)
    if order == CHAIN:
        acc = v[n - 1]
        for j in range(n - 2, -1, -1):
            acc = f(orc, op, v[0], acc) if (j == 0 and swap) else f(orc, op, acc, v[j])
        return acc
    w = list(v)
    if order == BINOMIAL:
        for u in range(0, n - 1, 2):
            w[u] = f(orc, op, w[0], w[1]) if (u == 0 and swap) else f(orc, op, w[u + 1], w[u])
        m = 2
        while m < n:
            for u in range(0, n - m, 2 * m):
                w[u] = f(orc, op, w[u], w[u + m])
            m *= 2
        return w[0]
    assert order == BINARY
    for s in range(n - 1, -1, -1):
        d = 1
        while 2 * d <= s + 1:
            d *= 2
        c0, c1 = s + d, s + 2 * d
        if c0 < n:
            w[s] = f(orc, op, w[0], w[c0]) if (s == 0 and swap) else f(orc, op, w[c0], w[s])
        if c1 < n:
            w[s] = f(orc, op, w[s], w[c1])
    return w[0]


def _inputs(n, count, seed, specials):
    rng = np.random.default_rng(seed)
    xs = [rng.uniform(-1, 1, count).astype(np.float32) for _ in range(n)]
    if specials:
        sp = np.array([np.nan, 0.0, -0.0, 1.0], dtype=np.float32)
        for x in xs:
            idx = rng.integers(0, count, count // 2)
            x[idx] = rng.choice(sp, idx.size)
    return xs


def _bits_equal(a, b):
    nan = np.isnan(a) & np.isnan(b)
    return np.array_equal(a[~nan].view(np.uint32), b[~nan].view(np.uint32)) and \
        np.array_equal(np.isnan(a), np.isnan(b))


ALGS = [(CHAIN, 3), (BINOMIAL, 5), (BINARY, 4)]


@pytest.mark.parametrize("n", list(range(2, 17)))
def test_closed_form_fold_equals_message_flow(orc, n):
    count = 257
    for op, specials in ((SUM, False), (MAX, True)):
        xs = _inputs(n, count, 1000 + n, specials)
        for root in range(n):
            for inplace in (False, True):
                v = [xs[(root + j) % n] for j in range(n)]
                for name, alg in ALGS:
                    exp, ran = orc.reduce(xs, count, op, F32, root, inplace, algorithm=alg)
                    assert ran == alg
                    got = fold(orc, op, v, name, inplace)
                    assert _bits_equal(got, exp), (n, root, inplace, name, op)
                # basic_linear = chain rooted at 0 without the swap, any root
                exp, ran = orc.reduce(xs, count, op, F32, root, inplace, algorithm=1)
                assert ran == 1
                assert _bits_equal(fold(orc, op, list(xs), CHAIN, False), exp)


def test_orders_differ_on_fp(orc):
    """The orders are distinguishable on these inputs (the test above is not
    vacuous)."""
    xs = _inputs(8, 4096, 5, False)
    outs = {alg: orc.reduce(xs, 4096, SUM, F32, 0, False, algorithm=alg)[0].view(np.uint32)
            for alg in (1, 3, 4, 5)}
    assert not np.array_equal(outs[1], outs[5])
    assert not np.array_equal(outs[5], outs[4])
    assert np.array_equal(outs[1], outs[3])  # pipeline rooted at 0 == basic_linear


def test_reduce_decision_matches_reference_table(orc):
    """Spot values of coll_tuned_decision_fixed.c:395-428 for commutative ops."""
    d = orc.reduce_decision
    assert d(4, 511, 100) == 1            # n < 8 and msg < 512: linear
    assert d(4, 512, 128) == 5            # n < 8 and msg < 20480: binomial
    assert d(8, 511, 100) == 5            # msg < 2048: binomial
    assert d(8, 4096, 1024) == 5          # 8 > 0.6016/1024*4096 + 1.3496
    assert d(8, 16384, 4096) == 4         # binary: 8 > 0.0422/1024*m + 1.1614
    assert d(8, 64 << 20, 16 << 20) == 3  # pipeline 64K
    assert d(2, 1 << 20, 262144) == 3
    assert d(4, 40000, 10000) == 4
    assert d(4, 80000, 20000) == 3
    assert d(16, 1 << 30, 1) == 5         # count <= 1


def test_library_decision_matches_oracle(orc):
    from ompi_amd import coll
    names = {1: "chain", 3: "chain", 4: "binary", 5: "binomial"}
    for n in (2, 3, 4, 5, 7, 8, 9, 12, 16):
        for msg in (4, 500, 512, 2000, 2048, 4096, 9000, 11000, 12000, 20000, 20480, 40000,
                    100000, 165000, 170000, 1 << 20, 256 << 20):
            for tsize in (4, 8, 12):
                count = max(1, msg // tsize)
                alg = orc.reduce_decision(n, count * tsize, count)
                for root in (0, n - 1):
                    name, first = coll.reduce_order(n, count * tsize, count, root)
                    assert name == names[alg], (n, msg, tsize)
                    assert first == (0 if alg == 1 else root)


def test_rsb_is_tuned_reduce_then_scatter(orc):
    for n, rcount in ((8, 300), (8, 4000), (8, 100000), (3, 2000), (4, 5000)):
        xs = _inputs(n, rcount * n, 77 + n, False)
        rb = orc.reduce_scatter_block(xs, rcount, SUM, F32)
        full, _ = orc.reduce(xs, rcount * n, SUM, F32, 0)
        for r in range(n):
            assert np.array_equal(rb[r].view(np.float32), full[r * rcount:(r + 1) * rcount])


@pytest.mark.parametrize("exclusive", [False, True])
def test_scan_linear_order(orc, exclusive):
    n, count = 7, 1001
    xs = _inputs(n, count, 9, False)
    res = orc.scan(xs, count, SUM, F32, exclusive)
    acc = xs[0].copy()
    if not exclusive:
        assert np.array_equal(res[0], acc)
    else:
        assert not res[0].any()
    for r in range(1, n):
        nxt = f(orc, SUM, xs[r], acc)          # P_r = f(out = x_r, in = P_(r-1))
        assert np.array_equal(res[r], acc if exclusive else nxt), r
        acc = nxt


def halving_fold(orc, op, v, tb):
    """Python twin of coll_ipc.hip fold() ORDER_HALVING (recursive halving
    reduce_scatter, coll_base_reduce_scatter.c:132-391) for tmp rank tb."""
    n = len(v)
    adj = 1
    while adj * 2 <= n:
        adj *= 2
    remain = n - adj
    w = [f(orc, op, v[2 * u + 1], v[2 * u]) if u < remain else v[u + remain] for u in range(adj)]
    m = adj // 2
    while m >= 1:
        for u in range(adj):
            if (u & m) == (tb & m):
                w[u] = f(orc, op, w[u], w[u ^ m])
        m //= 2
    return w[tb]


@pytest.mark.parametrize("n", list(range(2, 17)))
def test_reduce_scatter_closed_forms(orc, n):
    """Ring (block b folded from x[b+1] around to x[b]) and recursive-halving
    closed forms against the oracle's message-flow simulations, uneven and
    zero counts included."""
    rng = np.random.default_rng(n)
    rcounts = [int(c) for c in rng.integers(0, 40, n)]
    rcounts[n // 2] = 0
    total = sum(rcounts)
    for op, specials in ((SUM, False), (MAX, True)):
        xs = _inputs(n, total, 300 + n, specials)
        disps = np.concatenate([[0], np.cumsum(rcounts)[:-1]]).astype(int)
        adj = 1
        while adj * 2 <= n:
            adj *= 2
        remain = n - adj
        for alg in (1, 2):
            res, ran = orc.reduce_scatter(xs, rcounts, op, F32, algorithm=alg)
            assert ran == alg
            for b in range(n):
                if rcounts[b] == 0:
                    continue
                sl = [x[disps[b]:disps[b] + rcounts[b]].copy() for x in xs]
                if alg == 2:   # ring: v[j] = x[(b + 1 + j) % n], acc = f(v[j], acc)
                    acc = sl[(b + 1) % n]
                    for j in range(1, n):
                        acc = f(orc, op, sl[(b + 1 + j) % n], acc)
                else:
                    tb = b // 2 if b < 2 * remain else b - remain
                    acc = halving_fold(orc, op, sl, tb)
                assert _bits_equal(res[b], acc), (n, alg, b, op)


def test_reduce_scatter_decision(orc):
    d = orc.reduce_scatter_decision
    assert d(8, 12 * 1024) == 1 and d(3, 12 * 1024) == 1
    assert d(8, 256 * 1024) == 1 and d(8, 256 * 1024 + 4) == 2
    assert d(3, 12 * 1024 + 4) == 2 and d(4, 100000) == 1 and d(6, 100000) == 2


# ---- forced allreduce algorithms (coll_tuned_allreduce_algorithm) ----

def raben_piece(count, n, o):
    """Twin of coll_ipc.hip raben_piece: the part of the vector vrank o owns."""
    adj = 1
    while adj * 2 <= n:
        adj *= 2
    lo, w, m = 0, count, 1
    while m < adj:
        half = w // 2
        if o & m:
            lo, w = lo + half, w - half
        else:
            w = half
        m *= 2
    return lo, w


def raben_fold(orc, op, v, o):
    """Twin of coll_ipc.hip fold() ORDER_RABEN for an element owned by vrank o."""
    n = len(v)
    adj = 1
    while adj * 2 <= n:
        adj *= 2
    rem = n - adj
    right = o & 1
    w = [None] * adj
    for u in range(adj):
        if u < rem:
            w[u] = f(orc, op, v[2 * u + 1], v[2 * u]) if right else f(orc, op, v[2 * u], v[2 * u + 1])
        else:
            w[u] = v[u + rem]
    m = 1
    while m < adj:
        for u in range(adj):
            if (u & m) == (o & m):
                w[u] = f(orc, op, w[u], w[u ^ m])
        m *= 2
    return w[o]


@pytest.mark.parametrize("n", list(range(2, 17)))
def test_rabenseifner_closed_form_matches_message_flow(orc, n):
    """The device's per-element Rabenseifner fold (pieces by recursive
    halving, step-1 pair order by half) equals the oracle's message-flow
    simulation of coll_base_allreduce.c:970-1243, bit for bit, for every
    comm size 2..16 — including the non-power-of-two fold of step 1."""
    rng = np.random.default_rng(100 + n)
    count = 61 * n + 7
    xs = [rng.uniform(-1, 1, count).astype(np.float32) for _ in range(n)]
    res, alg = orc.allreduce_forced([x.copy() for x in xs], count, SUM, F32, orc.ALG_REDSCAT_ALLGATHER)
    assert alg == orc.ALG_REDSCAT_ALLGATHER
    adj = 1
    while adj * 2 <= n:
        adj *= 2
    exp = np.empty(count, dtype=np.float32)
    covered = 0
    for o in range(adj):
        lo, w = raben_piece(count, n, o)
        covered += w
        v = [x[lo:lo + w] for x in xs]
        exp[lo:lo + w] = raben_fold(orc, SUM, v, o)
    assert covered == count
    for r in range(n):
        assert np.array_equal(res[r].view(np.uint32), exp.view(np.uint32)), (n, r)
    # and the order matters on this data: the ring's result differs somewhere
    ring, _ = orc.allreduce([x.copy() for x in xs], count, SUM, F32, orc.ALG_RING)
    if n > 2:
        assert not np.array_equal(ring[0].view(np.uint32), exp.view(np.uint32))


@pytest.mark.parametrize("n", [2, 3, 5, 6, 8])
def test_forced_small_fallbacks(orc, n):
    """Each forced algorithm's own fallback: Rabenseifner below p' elements
    runs basic_linear (:988-995), ring below n elements recursive doubling
    (:371-377); basic_linear = the linear reduce's chain order."""
    rng = np.random.default_rng(7 + n)
    count = n - 1
    xs = [rng.uniform(-1, 1, count).astype(np.float32) for _ in range(n)]
    adj = 1
    while adj * 2 <= n:
        adj *= 2
    _, alg = orc.allreduce_forced([x.copy() for x in xs], adj - 1, SUM, F32, orc.ALG_REDSCAT_ALLGATHER)
    assert alg == orc.ALG_BASIC_LINEAR
    _, alg = orc.allreduce_forced([x.copy() for x in xs], count, SUM, F32, orc.ALG_RING)
    assert alg == orc.ALG_RECURSIVE_DOUBLING
    res, _ = orc.allreduce_forced([x.copy() for x in xs], count, SUM, F32, orc.ALG_BASIC_LINEAR)
    assert np.array_equal(res[0].view(np.uint32), fold(orc, SUM, xs, CHAIN, False).view(np.uint32))


@pytest.mark.parametrize("n", [2, 3, 4, 7])
@pytest.mark.parametrize("inplace", [False, True])
def test_forced_nonoverlapping_is_tuned_reduce_then_bcast(orc, n, inplace):
    """nonoverlapping = tuned reduce to rank 0 (with rank 0's MPI_IN_PLACE)
    + bcast (:54-86): every rank gets the reduce's result."""
    rng = np.random.default_rng(11 + n)
    count = 3001
    xs = [rng.uniform(-1, 1, count).astype(np.float32) for _ in range(n)]
    res, alg = orc.allreduce_forced([x.copy() for x in xs], count, SUM, F32, orc.ALG_NONOVERLAPPING,
                                    root0_inplace=inplace)
    assert alg == orc.ALG_NONOVERLAPPING
    red, _ = orc.reduce([x.copy() for x in xs], count, SUM, F32, 0, inplace)
    for r in range(n):
        assert np.array_equal(res[r].view(np.uint32), red.view(np.uint32))


def test_library_forced_reduce_orders(orc):
    """coll_tuned_reduce_algorithm forced (dynamic rules on): the library's
    order for 1 / 3 / 4 / 5 is the one the oracle runs for that algorithm
    whatever the fixed decision would say; 2 / 6 / 7 are refused (coll/rocm
    then leaves the reduction to coll/tuned)."""
    from ompi_amd import _lib, coll
    names = {1: "chain", 3: "chain", 4: "binary", 5: "binomial"}
    for n in (2, 3, 4, 8, 9):
        for msg in (4, 511, 4096, 1 << 20):
            count = max(1, msg // 4)
            for forced, name in names.items():
                for root in (0, n - 1):
                    got, first = coll.reduce_order(n, count * 4, count, root, forced=forced)
                    assert got == name, (n, msg, forced)
                    assert first == (0 if forced == 1 else root)
            for forced in (2, 6, 7):
                with pytest.raises(_lib.OmpiAmdError) as e:
                    coll.reduce_order(n, count * 4, count, 0, forced=forced)
                assert e.value.code == _lib.ERR_UNSUPPORTED


@pytest.mark.parametrize("n", [2, 3, 5, 8])
def test_oracle_forced_rsb_and_rs_nonoverlapping(orc, n):
    """rsb basic_linear and reduce_scatter non-overlapping call coll/tuned's
    reduce to rank 0 (coll_base_reduce_scatter_block.c:95-97,
    coll_base_reduce_scatter.c:42-92), so a forced reduce algorithm changes
    their fp order: the oracle's forms equal its reduce with that algorithm,
    cut into the blocks."""
    rcount = 300
    xs = _inputs(n, n * rcount, 77 + n, False)
    for alg in (0, 1, 3, 4, 5):
        full, _ = orc.reduce(xs, n * rcount, SUM, F32, 0, False, algorithm=alg)
        rb = orc.reduce_scatter_block([x.copy() for x in xs], rcount, SUM, F32, red_alg=alg)
        for r in range(n):
            assert _bits_equal(rb[r].view(np.float32), full[r * rcount:(r + 1) * rcount]), (alg, r)
        rcounts = [rcount + (r % 3) - 1 for r in range(n)]
        tot = sum(rcounts)
        ys = [x[:tot].copy() for x in xs]
        for inplace in (False, True):
            full2, _ = orc.reduce(ys, tot, SUM, F32, 0, inplace, algorithm=alg)
            got, ran = orc.reduce_scatter(ys, rcounts, SUM, F32, algorithm=orc.RS_NONOVERLAPPING,
                                          red_alg=alg, inplace=inplace)
            assert ran == orc.RS_NONOVERLAPPING
            off = 0
            for r in range(n):
                assert _bits_equal(got[r], full2[off:off + rcounts[r]]), (alg, inplace, r)
                off += rcounts[r]
    # the forced orders really differ from the fixed one on these inputs
    a = orc.reduce_scatter_block([x.copy() for x in xs], rcount, SUM, F32, red_alg=1)
    b = orc.reduce_scatter_block([x.copy() for x in xs], rcount, SUM, F32, red_alg=5)
    assert n == 2 or any(not _bits_equal(a[r].view(np.float32), b[r].view(np.float32)) for r in range(n))
