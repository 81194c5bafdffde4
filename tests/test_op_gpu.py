"""GPU parity of the MPI_Op kernels against the CPU oracle (bit-exact).

Every (op, type) slot the library provides is run through both the C-ABI
entry points (2-/3-buffer) and the op-framework handler table, on random
data plus the edge values the reference's semantics hinge on (NaN, ±0,
±inf, denormals, ties), at ragged sizes that exercise the vector body, the
scalar tail and the unaligned path; and on the reference's own
known-answer tests (reduce_local.c / check_op.sh, tests/golden/op_kat.json).
"""
import ctypes

import numpy as np
import pytest

from ompi_amd import _lib
from ompi_amd import op as mop

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

DEV = "cuda:0"
SIZES = [1, 3, 17, 64, 1000, 4099, 65536 + 13, 1 << 20]


def to_dev(a: np.ndarray, offset: int = 0):
    """Copy bytes of `a` to a fresh device buffer at byte `offset`."""
    raw = a.view(np.uint8).reshape(-1)
    t = torch.empty(raw.nbytes + offset + 16, dtype=torch.uint8, device=DEV)
    t[offset:offset + raw.nbytes].copy_(torch.from_numpy(raw.copy()))
    return t, t.data_ptr() + offset


def from_dev(t, offset, nbytes) -> np.ndarray:
    return t[offset:offset + nbytes].cpu().numpy()


def gen(dtype: mop.Datatype, n: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    nd = dtype.np_dtype
    if nd.names == ("re", "im"):  # short float complex: a record of two halves
        h = np.dtype(np.float16)
        return _cplx(gen(Datatype_like(h), n, seed * 2 + 1), gen(Datatype_like(h), n, seed * 2 + 2), nd)
    if nd.names:  # pair
        a = np.zeros(n, dtype=nd)
        vt = nd.fields["v"][0]
        if vt.kind == "f":
            a["v"] = np.round(rng.random(n) * 64) / 64
            a["v"][::37] = np.nan
            a["v"][::41] = -0.0
        else:
            a["v"] = rng.integers(-8, 8, n)
        a["k"] = rng.integers(-1000, 1000, n)
        raw = a.view(np.uint8).reshape(n, nd.itemsize)
        # random gap bytes: the kernels must preserve / not write them
        for off in range(nd.itemsize):
            if off >= nd.fields["v"][1] + vt.itemsize and off < nd.fields["k"][1]:
                raw[:, off] = rng.integers(0, 255, n)
            if off >= nd.fields["k"][1] + 4:
                raw[:, off] = rng.integers(0, 255, n)
        return a
    if nd.kind == "c":
        # complex: independent real/imaginary parts through the fp generator,
        # so NaN / inf / ±0 / denormal components meet every recovery branch
        # of the C99 product (ISO C Annex G.5.1)
        rd = np.dtype(np.float32 if nd.itemsize == 8 else np.float64)
        re = gen(Datatype_like(rd), n, seed * 2 + 1)
        im = gen(Datatype_like(rd), n, seed * 2 + 2)
        return _cplx(re, im, nd)
    if nd.kind == "f":
        a = (rng.standard_normal(n) * 100).astype(nd)
        specials = np.array([np.nan, -np.nan, 0.0, -0.0, np.inf, -np.inf,
                             np.finfo(nd).tiny / 4, -np.finfo(nd).tiny / 8,
                             np.finfo(nd).max, 1.0], dtype=nd)
        a[rng.integers(0, n, max(1, n // 5))] = rng.choice(specials, max(1, n // 5))
        return a
    if nd.itemsize == 1 and dtype.code in (25,):
        return rng.integers(0, 2, n).astype(nd)
    info = np.iinfo(nd)
    a = rng.integers(info.min, info.max, n, dtype=nd, endpoint=True)
    a[::7] = rng.integers(-3, 3, len(a[::7])).astype(nd)
    return a


class Datatype_like:
    """Minimal stand-in carrying a numpy dtype for gen()."""
    def __init__(self, nd):
        self.np_dtype = nd
        self.code = -1


def _cplx(re: np.ndarray, im: np.ndarray, nd) -> np.ndarray:
    # interleave the parts bit-for-bit (re + 1j*im would turn inf*1j into nan)
    out = np.empty(len(re), dtype=nd)
    v = out.view(re.dtype).reshape(-1, 2)
    v[:, 0] = re
    v[:, 1] = im
    return out


def same_bits(got: np.ndarray, exp: np.ndarray, dtype: mop.Datatype) -> bool:
    nd = dtype.np_dtype
    if nd.names == ("re", "im"):
        return same_bits(got.view(np.float16), exp.view(np.float16), Datatype_like(np.dtype(np.float16)))
    if nd.names:
        # pair types: compare the value and index bytes.  Padding bytes of a
        # struct take unspecified values when a member is stored (C11
        # 6.2.6.1p6), so not even two builds of the reference agree on them.
        return all(np.array_equal(np.ascontiguousarray(got[f]).view(np.uint8),
                                  np.ascontiguousarray(exp[f]).view(np.uint8))
                   for f in ("v", "k"))
    g = got.view(np.uint8)
    e = exp.view(np.uint8)
    if np.array_equal(g, e):
        return True
    if nd.kind in "fc":
        # NaN payload/sign bits may differ only where both are NaN (complex:
        # per component)
        rd = nd if nd.kind == "f" else np.dtype(np.float32 if nd.itemsize == 8 else np.float64)
        gv, ev = got.view(rd), exp.view(rd)
        both_nan = np.isnan(gv) & np.isnan(ev)
        return bool(np.array_equal(gv[~both_nan].view(np.uint8), ev[~both_nan].view(np.uint8)))
    return False


SLOTS = [(op, dt) for op in mop.OPS for dt in mop.DATATYPES]


@pytest.mark.parametrize("op,dt", SLOTS, ids=[f"{o.name}-{d.name}" for o, d in SLOTS])
def test_op_parity(orc, op, dt):
    if not orc.defined(op.index, dt.code):
        assert not mop.supported(op, dt)
        return
    assert mop.supported(op, dt)
    for si, n in enumerate(SIZES):
        a = gen(dt, n, 100 + si)
        b = gen(dt, n, 200 + si)
        ext = dt.extent
        for off in ((0,) if n < 1000 else (0, ext if ext < 16 else 0)):
            # 2-buffer via the C ABI
            ta, pa = to_dev(a, off)
            tb, pb = to_dev(b, off)
            mop.reduce_local_async(pa, pb, n, dt, op)
            torch.cuda.synchronize()
            exp = b.copy()
            orc.op_2buff(op.index, dt.code, a, exp, n)
            got = from_dev(tb, off, n * ext).view(dt.np_dtype)
            assert same_bits(got, exp, dt), (op.name, dt.name, n, off)
            # 3-buffer via the C ABI; out pre-filled so gap bytes are checked
            out0 = gen(dt, n, 300 + si)
            to, po = to_dev(out0, off)
            ta, pa = to_dev(a, off)
            tb, pb = to_dev(b, off)
            mop.reduce_local_3buff_async(pa, pb, po, n, dt, op)
            torch.cuda.synchronize()
            exp3 = out0.copy()
            orc.op_3buff(op.index, dt.code, a, b, exp3, n)
            got3 = from_dev(to, off, n * ext).view(dt.np_dtype)
            assert same_bits(got3, exp3, dt), (op.name, dt.name, n, off, "3buff")


@pytest.mark.parametrize("op,dt", [(mop.MPI_SUM, mop.MPI_FLOAT), (mop.MPI_MAX, mop.MPI_DOUBLE),
                                   (mop.MPI_BAND, mop.MPI_INT32_T),
                                   (mop.MPI_MAXLOC, mop.MPI_DOUBLE_INT)])
def test_handler_table_path(orc, op, dt):
    """Call through the op-framework slot with the reference's handler
    signature (fns[type](in, inout, &count, &dtype, module))."""
    n = 12345
    a, b = gen(dt, n, 5), gen(dt, n, 6)
    ta, pa = to_dev(a)
    tb, pb = to_dev(b)
    mop.reduce_local(pa, pb, n, dt, op)          # blocking handler
    exp = b.copy()
    orc.op_2buff(op.index, dt.code, a, exp, n)
    assert same_bits(from_dev(tb, 0, n * dt.extent).view(dt.np_dtype), exp, dt)
    out0 = gen(dt, n, 7)
    to, po = to_dev(out0)
    ta, pa = to_dev(a)
    tb, pb = to_dev(b)
    mop.reduce_local_3buff(pa, pb, po, n, dt, op)
    exp3 = out0.copy()
    orc.op_3buff(op.index, dt.code, a, b, exp3, n)
    assert same_bits(from_dev(to, 0, n * dt.extent).view(dt.np_dtype), exp3, dt)


@pytest.mark.parametrize("op,dt", [(mop.MPI_SUM, mop.MPI_FLOAT), (mop.MPI_MAX, mop.MPI_DOUBLE),
                                   (mop.MPI_MAXLOC, mop.MPI_DOUBLE_INT),
                                   (mop.MPI_PROD, mop.MPI_C_DOUBLE_COMPLEX)])
def test_handler_mixed_residency(orc, op, dt):
    """Host and device operands in one handler call: coll/tuned's ring
    reduces a malloc'd host inbuf into the device rbuf
    (coll_base_allreduce.c:688-693) when coll/rocm declines.  The handler
    stages the host operands on the device and returns the oracle's bits —
    for every placement of the operands, 2- and 3-buffer."""
    n = 70001
    a, b = gen(dt, n, 15), gen(dt, n, 16)
    ext = dt.extent
    h2 = mop.handler(op, dt)
    h3 = mop.handler3(op, dt)
    cnt = ctypes.c_int(n)
    for in_dev, inout_dev in ((False, True), (True, False)):
        ha, hb = a.copy(), b.copy()
        ta, pa = to_dev(ha)
        tb, pb = to_dev(hb)
        src = pa if in_dev else ha.ctypes.data
        dst = pb if inout_dev else hb.ctypes.data
        h2(src, dst, ctypes.byref(cnt), None, None)
        exp = b.copy()
        orc.op_2buff(op.index, dt.code, a, exp, n)
        got = from_dev(tb, 0, n * ext).view(dt.np_dtype) if inout_dev else hb
        assert same_bits(got, exp, dt), ("2buff", in_dev, inout_dev)
    for mask in range(1, 7):  # not all-device (0 is the plain path), not all-host (7)
        ha, hb = a.copy(), b.copy()
        hout = gen(dt, n, 17)
        ta, pa = to_dev(ha)
        tb, pb = to_dev(hb)
        to, po = to_dev(hout)
        p1 = ha.ctypes.data if mask & 1 else pa
        p2 = hb.ctypes.data if mask & 2 else pb
        p3 = hout.ctypes.data if mask & 4 else po
        h3(p1, p2, p3, ctypes.byref(cnt), None, None)
        exp3 = gen(dt, n, 17)
        orc.op_3buff(op.index, dt.code, a, b, exp3, n)
        got3 = hout if mask & 4 else from_dev(to, 0, n * ext).view(dt.np_dtype)
        assert same_bits(got3, exp3, dt), ("3buff", mask)


def test_handler_host_fallback(orc):
    """Host buffers go to the registered lower-priority handler, never to a
    device kernel (op_example_module_max.c fallback pattern)."""
    lib = _lib.load()
    calls = []

    @_lib.HANDLER_FN
    def base_sum_float(inp, inout, count, dtype, module):
        n = count[0]
        a = np.ctypeslib.as_array(ctypes.cast(inp, ctypes.POINTER(ctypes.c_float)), (n,))
        b = np.ctypeslib.as_array(ctypes.cast(inout, ctypes.POINTER(ctypes.c_float)), (n,))
        b += a
        calls.append(n)

    lib.ompi_amd_op_set_fallback(3, 15, ctypes.cast(base_sum_float, ctypes.c_void_p), None,
                                 None, None)
    a = np.arange(10, dtype=np.float32)
    b = np.ones(10, dtype=np.float32)
    fn = mop.handler(mop.MPI_SUM, mop.MPI_FLOAT)
    c = ctypes.c_int(10)
    fn(a.ctypes.data, b.ctypes.data, ctypes.byref(c), None, None)
    assert calls == [10]
    assert np.array_equal(b, np.arange(10, dtype=np.float32) + 1)
    lib.ompi_amd_op_set_fallback(3, 15, None, None, None, None)


def test_reduce_local_kat(golden):
    """reduce_local.c known answers at check_op.sh sizes, on the GPU."""
    kat = golden("op_kat.json")
    for case in kat["cases"]:
        dt = mop.BY_CODE[case["type_code"]]
        op = next(o for o in mop.OPS if o.index == case["op"])
        nd = np.dtype(case["dtype"])
        n = max(case["counts"])
        src = torch.from_numpy(np.full(n, case["source"], dtype=nd).view(np.uint8)).to(DEV)
        tgt = torch.from_numpy(np.full(n, case["target"], dtype=nd).view(np.uint8)).to(DEV)
        for count in case["counts"]:
            t = tgt.clone()
            mop.reduce_local(src, t, count, dt, op)
            got = t.cpu().numpy().view(nd)
            exp = np.array(case["expected_target"], dtype=nd)
            assert (got[:count] == exp).all(), (case["dtype"], case["op_name"], count)
            assert (got[count:] == nd.type(case["target"])).all()


def test_large_buffer_sum_float(orc):
    """1 GiB-class run (BASELINE config 2 top size), checked exactly."""
    n = (256 << 20) // 4 + 5
    rng = np.random.default_rng(0)
    a = rng.standard_normal(n, dtype=np.float32)
    b = rng.standard_normal(n, dtype=np.float32)
    da, db = torch.from_numpy(a).to(DEV), torch.from_numpy(b).to(DEV)
    out = torch.empty_like(da)
    mop.reduce_local_3buff_async(da, db, out, n, mop.MPI_FLOAT, mop.MPI_SUM)
    torch.cuda.synchronize()
    exp = np.empty_like(a)
    orc.op_3buff(3, 15, a, b, exp, n)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), exp.view(np.uint32))


MISALIGNED = [(mop.MPI_SUM, mop.MPI_FLOAT), (mop.MPI_MAX, mop.MPI_DOUBLE),
              (mop.MPI_BXOR, mop.MPI_UINT8_T), (mop.MPI_PROD, mop.MPI_INT16_T),
              (mop.MPI_MAXLOC, mop.MPI_FLOAT_INT)]


@pytest.mark.parametrize("op,dt", MISALIGNED, ids=[f"{o.name}-{d.name}" for o, d in MISALIGNED])
def test_misaligned_operands(orc, op, dt):
    """Operands displaced inside their 16-B vectors: all by the same amount
    (head peeled, vectors after it) and by different amounts (element path),
    sizes around the head / tail boundaries; the bytes around the result stay
    untouched."""
    ext = dt.extent
    for n in (1, 3, 5, 17, 1000, 65537, 1 << 20):
        for offs in ((ext, ext, ext), (3 * ext, 3 * ext, 3 * ext), (ext, 0, ext), (0, 2 * ext, ext)):
            a = gen(dt, n, 400 + n % 97)
            b = gen(dt, n, 500 + n % 89)
            out0 = gen(dt, n + 8, 600)
            xo, yo, do = offs
            ta, pa = to_dev(a, xo)
            tb, pb = to_dev(b, yo)
            raw_out = np.ascontiguousarray(out0).view(np.uint8)
            to, po = to_dev(out0, do)  # guard bytes: the rest of out0 after n elements
            mop.reduce_local_3buff_async(pa, pb, po, n, dt, op)
            torch.cuda.synchronize()
            exp3 = out0[:n].copy()
            orc.op_3buff(op.index, dt.code, a, b, exp3, n)
            got = from_dev(to, do, raw_out.nbytes)
            assert same_bits(got[:n * ext].view(dt.np_dtype), exp3, dt), (op.name, dt.name, n, offs)
            assert np.array_equal(got[n * ext:], raw_out[n * ext:]), ("guard bytes", n, offs)
            # 2-buffer (inout shares the in operand's offset or not)
            ta, pa = to_dev(a, xo)
            tb, pb = to_dev(b, do)
            mop.reduce_local_async(pa, pb, n, dt, op)
            torch.cuda.synchronize()
            exp = b.copy()
            orc.op_2buff(op.index, dt.code, a, exp, n)
            got2 = from_dev(tb, do, n * ext).view(dt.np_dtype)
            assert same_bits(got2, exp, dt), (op.name, dt.name, n, offs, "2buff")
