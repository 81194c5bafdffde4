"""Pin the CPU oracle against the reference's own known answers (CPU only).

The oracle is the checker for every GPU parity test, so it is checked first
against fixtures restated from the reference's tests (tests/golden/*.json,
see make_golden.py for the file:line of each).
"""
import numpy as np
import pytest

from ompi_amd import op as mop

MAX, MIN, SUM, PROD, LAND, BAND, LOR, BOR, LXOR, BXOR, MAXLOC, MINLOC = range(1, 13)


def test_reduce_local_kat(orc, golden):
    kat = golden("op_kat.json")
    for case in kat["cases"]:
        dt = np.dtype(case["dtype"])
        for count in case["counts"] + kat["sweep_counts"][:12]:
            src = np.full(count, case["source"], dtype=dt)
            tgt = np.full(count, case["target"], dtype=dt)
            orc.op_2buff(case["op"], case["type_code"], src, tgt, count)
            exp = np.array(case["expected_target"], dtype=dt)
            assert (tgt == exp).all(), (case, count)


def test_op_edge_cases(orc, golden):
    edge = golden("op_edge.json")
    for c in edge["max_float_2buff"]:
        out = np.array([c["out"]], dtype=np.uint32).view(np.float32)
        inb = np.array([c["in"]], dtype=np.uint32).view(np.float32)
        orc.op_2buff(MAX, 15, inb, out, 1)
        got = out.view(np.uint32)[0]
        exp = c["result"]
        if np.isnan(np.array([exp], dtype=np.uint32).view(np.float32)[0]):
            assert np.isnan(out[0])
        else:
            assert got == exp, c
    dt = mop.MPI_DOUBLE_INT.np_dtype
    assert dt.itemsize == edge["double_int_sizeof"]
    for c in edge["maxloc_double_int_2buff"]:
        out = np.zeros(1, dtype=dt)
        inb = np.zeros(1, dtype=dt)
        out["v"], out["k"] = c["out"]
        inb["v"], inb["k"] = c["in"]
        orc.op_2buff(MAXLOC, 35, inb, out, 1)
        assert [out["v"][0], out["k"][0]] == c["result"]


def test_op_table_pattern(orc):
    """The (op,type) slots the oracle restates match the product's table
    (both follow op_base_functions.c:1485-1569)."""
    lib = pytest.importorskip("ompi_amd._lib").load()
    for op in range(15):
        for t in range(41):
            assert bool(lib.ompi_amd_op_supported(op, t)) == orc.defined(op, t), (op, t)


def _np_ref_2buff(op, a, b):
    """numpy restatement of the 2-buffer rule for plain numeric arrays."""
    with np.errstate(over="ignore", invalid="ignore"):
        if op == SUM:
            return (b + a).astype(b.dtype)
        if op == PROD:
            return (b * a).astype(b.dtype)
        if op == MAX:
            return np.where(b > a, b, a)
        if op == MIN:
            return np.where(b < a, b, a)
        if op == BAND:
            return b & a
        if op == BOR:
            return b | a
        if op == BXOR:
            return b ^ a
        if op == LAND:
            return ((b != 0) & (a != 0)).astype(b.dtype)
        if op == LOR:
            return ((b != 0) | (a != 0)).astype(b.dtype)
        if op == LXOR:
            return ((b != 0) ^ (a != 0)).astype(b.dtype)


@pytest.mark.parametrize("dtype", [mop.MPI_INT8_T, mop.MPI_UINT16_T, mop.MPI_INT32_T,
                                   mop.MPI_UINT64_T, mop.MPI_FLOAT, mop.MPI_DOUBLE])
def test_oracle_vs_numpy(orc, dtype):
    rng = np.random.default_rng(7)
    n = 10007
    nd = dtype.np_dtype
    if nd.kind == "f":
        a = rng.standard_normal(n).astype(nd)
        b = rng.standard_normal(n).astype(nd)
        a[::97] = np.nan
        b[::89] = -0.0
        a[::83] = 0.0
    else:
        info = np.iinfo(nd)
        a = rng.integers(info.min, info.max, n, dtype=nd, endpoint=True)
        b = rng.integers(info.min, info.max, n, dtype=nd, endpoint=True)
        b[::13] = a[::13]
    for op in (SUM, PROD, MAX, MIN, BAND, BOR, BXOR, LAND, LOR, LXOR):
        if not orc.defined(op, dtype.code):
            continue
        out = b.copy()
        orc.op_2buff(op, dtype.code, a, out, n)
        exp = _np_ref_2buff(op, a, b)
        assert np.array_equal(out.view(np.uint8), exp.astype(nd).view(np.uint8)), op
        # 3-buffer: out = in1 op in2 with in1 playing the out role
        out3 = np.zeros_like(b)
        orc.op_3buff(op, dtype.code, b, a, out3, n)
        assert np.array_equal(out3.view(np.uint8), exp.astype(nd).view(np.uint8)), op


def test_loc_2buff_vs_3buff_semantics(orc):
    """LOC_FUNC keeps out on an unordered compare; LOC_FUNC_3BUF takes in2
    (op_base_functions.c:88-104 vs :709-731)."""
    dt = mop.MPI_DOUBLE_INT.np_dtype
    a = np.zeros(3, dtype=dt)
    b = np.zeros(3, dtype=dt)
    a["v"] = [np.nan, 1.0, 2.0]
    a["k"] = [1, 9, 4]
    b["v"] = [5.0, 1.0, np.nan]
    b["k"] = [2, 3, 6]
    out = b.copy()
    orc.op_2buff(MAXLOC, 35, a, out, 3)      # in=a, inout=b
    assert list(out["k"]) == [2, 3, 6]
    out3 = np.zeros(3, dtype=dt)
    orc.op_3buff(MAXLOC, 35, a, b, out3, 3)  # in1=a, in2=b
    assert list(out3["k"]) == [2, 3, 6]
    out3 = np.zeros(3, dtype=dt)
    orc.op_3buff(MAXLOC, 35, b, a, out3, 3)  # in1=b, in2=a
    assert list(out3["k"]) == [1, 3, 4]


def test_allreduce_closed_forms(orc, golden):
    for c in golden("ring_closed_form.json")["cases"]:
        n, count = c["nranks"], c["count"]
        x = np.array(c["x_bits"], dtype=np.uint32).view(np.float32)
        sb = [x[r].copy() for r in range(n)]
        ring, alg = orc.allreduce(sb, count, SUM, 15, orc.ALG_RING)
        assert alg == orc.ALG_RING
        exp = np.array(c["ring_bits"], dtype=np.uint32)
        for r in range(n):
            assert np.array_equal(ring[r].view(np.uint32), exp), (n, r)
        tree, alg = orc.allreduce(sb, count, SUM, 15, orc.ALG_RECURSIVE_DOUBLING)
        exp = np.array(c["tree_bits"], dtype=np.uint32)
        for r in range(n):
            assert np.array_equal(tree[r].view(np.uint32), exp), (n, r)


def test_ring_segmented_equals_ring_order(orc):
    rng = np.random.default_rng(3)
    n, count = 4, 3 * 4096 + 5
    sb = [rng.standard_normal(count).astype(np.float32) for _ in range(n)]
    ring, _ = orc.allreduce(sb, count, SUM, 15, orc.ALG_RING)
    seg, alg = orc.allreduce(sb, count, SUM, 15, orc.ALG_RING_SEGMENTED, segsize=1024)
    assert alg == orc.ALG_RING_SEGMENTED
    for r in range(n):
        assert np.array_equal(ring[r], seg[r])


@pytest.mark.parametrize("n", [2, 3, 4, 5, 8])
def test_tuned_decision_and_agreement(orc, n):
    rng = np.random.default_rng(n)
    for count, expect in ((100, orc.ALG_RECURSIVE_DOUBLING), (50000, orc.ALG_RING),
                          (n * 262144 + 11, orc.ALG_RING_SEGMENTED)):
        sb = [rng.standard_normal(count).astype(np.float32) for _ in range(n)]
        res, alg = orc.allreduce(sb, count, SUM, 15, orc.ALG_TUNED)
        assert alg == expect
        for r in range(1, n):
            assert np.array_equal(res[0].view(np.uint32), res[r].view(np.uint32))
        exact = np.sum(np.stack(sb).astype(np.float64), axis=0)
        scale = np.sum(np.abs(np.stack(sb).astype(np.float64)), axis=0)
        assert (np.abs(res[0] - exact) <= 1e-6 * scale + 1e-30).all()


def test_maxloc_allreduce_exact(orc):
    dt = mop.MPI_DOUBLE_INT.np_dtype
    n, count = 8, 5000
    rng = np.random.default_rng(11)
    sb = []
    for r in range(n):
        a = np.zeros(count, dtype=dt)
        a["v"] = np.round(rng.random(count) * 1024) / 1024
        a["k"] = r * count + np.arange(count)
        sb.append(a)
    res, _ = orc.allreduce(sb, count, MAXLOC, 35)
    v = np.stack([s["v"] for s in sb])
    k = np.stack([s["k"] for s in sb])
    best = v.max(axis=0)
    kk = np.where(v == best, k, np.iinfo(np.int32).max).min(axis=0)
    for r in range(n):
        assert np.array_equal(res[r]["v"], best)
        assert np.array_equal(res[r]["k"], kk)


def _np_pack(blocks, extent, count, src):
    out = []
    for e in range(count):
        for d, ln in blocks:
            out.append(src[e * extent + d: e * extent + d + ln])
    return np.concatenate(out)


def test_ddt_pack_unpack_kat(orc, golden):
    for t in golden("ddt_kat.json")["types"]:
        blocks = [tuple(b) for b in t["blocks"]]
        assert sum(b[1] for b in blocks) == t["size"], t["name"]
        count = min(t["count"], 64)
        span = (count - 1) * t["extent"] + max(d + ln for d, ln in blocks)
        src = np.random.default_rng(1).integers(0, 255, span, dtype=np.uint8)
        full = _np_pack(blocks, t["extent"], count, src)
        assert full.nbytes == t["size"] * count
        for chunk in t["chunks"] + [t["size"] * count]:
            pieces = []
            pos = 0
            while pos < full.nbytes:
                p = orc.pack(blocks, t["extent"], count, src, pos, chunk)
                assert p.nbytes == min(chunk, full.nbytes - pos)
                pieces.append(p)
                pos += p.nbytes
            assert np.array_equal(np.concatenate(pieces), full), (t["name"], chunk)
            dst = np.zeros_like(src)
            pos = 0
            while pos < full.nbytes:
                n = orc.unpack(blocks, t["extent"], count, full[pos:pos + chunk].copy(), dst, pos)
                pos += n
            assert np.array_equal(_np_pack(blocks, t["extent"], count, dst), full)


def test_datatype_builders_match_reference_types(golden):
    """The host-side constructors (ompi_amd/datatype.py) reproduce the
    typemaps, sizes and extents of the reference tests' datatypes, and fold
    them the way opal's optimizer does (vector -> 1 element, blacs -> 13)."""
    from ompi_amd import datatype as dd
    d, i32 = dd.predefined("MPI_DOUBLE"), dd.predefined("MPI_INT")
    kat = {t["name"]: t for t in golden("ddt_kat.json")["types"]}
    lens = [13, 13, 13, 13, 13, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1]
    disps = [286, 308, 330, 352, 374, 396, 419, 442, 465, 488, 511, 534, 557, 580, 603,
             626, 649, 672]
    built = {
        "vector_450_10_11_double": (dd.type_vector(450, 10, 11, d), 1),
        "blacs_indexed_int": (dd.type_indexed(lens, disps, i32), 13),
        "upper_matrix_100": (dd.type_indexed([100 - k for k in range(100)],
                                             [k * 100 + k for k in range(100)], d), 100),
        "struct_char_double": (dd.type_struct([1, 1], [0, 8], [dd.predefined("MPI_CHAR"), d]), 2),
        "twice_two_doubles": (dd.type_vector(2, 2, 5, d), 1),
        "struct_int_double": (dd.type_struct([1, 1], [0, 8], [i32, d]), 2),
    }
    for name, (dt, nel) in built.items():
        t = kat[name]
        assert dt.runs == [tuple(b) for b in t["blocks"]], name
        assert dt.size == t["size"] and dt.extent == t["extent"], name
        assert len(dt.elems) == nel, (name, dt.elems[:4])


@pytest.mark.parametrize("table", ["test1", "test2", "test3", "test4"])
def test_oracle_unpack_out_of_order_fixture(orc, golden, table):
    """The oracle's unpack restatement against the reference's own
    out-of-order fixture (test/datatype/unpack_ooo.c, tests/golden/
    unpack_ooo.json): every (bytes, offset) fragment of the table unpacked at
    its offset, in the table's order, gives exactly the layout the test
    checks (:125-131) — gaps (i[1], d[1]) and padding untouched."""
    u = golden("unpack_ooo.json")
    packed = np.frombuffer(bytes.fromhex(u["packed_hex"]), dtype=np.uint8)
    typed = np.frombuffer(bytes.fromhex(u["bar_init_hex"]), dtype=np.uint8).copy()
    expected = np.frombuffer(bytes.fromhex(u["expected_hex"]), dtype=np.uint8)
    assert sum(b for b, _ in u["tables"][table]) == packed.nbytes == u["size"] * u["count"]
    for nbytes, off in u["tables"][table]:
        frag = packed[off:off + nbytes].copy()
        assert orc.unpack(u["blocks"], u["extent"], u["count"], frag, typed, off) == nbytes
    assert np.array_equal(typed, expected)


def test_short_float_restatement(orc):
    """binary16 in the oracle (MPIX_C_FLOAT16 / opal_short_float_t): the
    half <-> float conversions equal numpy's IEEE ones (every half, and
    floats around every half's midpoints), and SUM / PROD equal the exact
    double result rounded once to half — so the x86 float evaluation the
    oracle restates is correctly rounded for one +, *."""
    import ctypes
    L = orc.lib()
    L.orc_h2f.restype, L.orc_h2f.argtypes = ctypes.c_float, [ctypes.c_uint16]
    L.orc_f2h.restype, L.orc_f2h.argtypes = ctypes.c_uint16, [ctypes.c_float]
    allh = np.arange(65536, dtype=np.uint16)
    ref = allh.view(np.float16).astype(np.float32)
    got = np.array([L.orc_h2f(int(h)) for h in allh], dtype=np.float32)
    nan = np.isnan(ref)
    assert np.array_equal(ref[~nan].view(np.uint32), got[~nan].view(np.uint32))
    assert np.isnan(got[nan]).all()
    rng = np.random.default_rng(14)
    near = (ref[~nan][::7].view(np.uint32).astype(np.int64)[:, None] + np.arange(-2, 3)[None, :])
    fs = np.concatenate([rng.integers(0, 2**32, 20000, dtype=np.uint64).astype(np.uint32),
                         (near.ravel() & 0xffffffff).astype(np.uint32)]).view(np.float32)
    fs = fs[~np.isnan(fs)]
    with np.errstate(over="ignore"):
        exp = fs.astype(np.float16).view(np.uint16)
    assert np.array_equal(np.array([L.orc_f2h(float(f)) for f in fs], dtype=np.uint16), exp)
    a = rng.integers(0, 65536, 50000, dtype=np.uint64).astype(np.uint16)
    b = rng.integers(0, 65536, 50000, dtype=np.uint64).astype(np.uint16)
    for op, fn in ((SUM, np.add), (PROD, np.multiply)):
        out = b.copy()
        orc.op_2buff(op, 14, a, out, len(a))
        with np.errstate(over="ignore", invalid="ignore"):
            e = fn(b.view(np.float16).astype(np.float64),
                   a.view(np.float16).astype(np.float64)).astype(np.float16)
        ok = ~np.isnan(e)
        assert np.array_equal(out[ok], e.view(np.uint16)[ok]), op
        assert np.isnan(out.view(np.float16)[~ok]).all()
