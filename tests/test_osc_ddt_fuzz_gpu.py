"""Randomized one-sided operations with derived datatypes (osc_sm_comm.c:
24-100, 209-270: MPI_Put / MPI_Get through ompi_datatype_sndrcv of any
origin / target pair; ompi_osc_base_sndrcv_op for MPI_Accumulate /
MPI_Get_accumulate): random nested target types, origin types that are
contiguous or vectors of the same element, random displacements into a
window created over a caller's device buffer (a communicator of one rank:
the target is this GPU).  Put and get are checked byte-exact against the
oracle's pack + unpack; accumulate and get_accumulate (fp64 SUM: one IEEE
add per element, doubles at any byte offset, so bit-exact) against the
oracle's op on the packed streams; window bytes outside the target typemap
untouched."""
import numpy as np
import pytest

from ddt_random import rand_type, span_of
from ompi_amd import coll, osc
from ompi_amd import datatype as dd
from ompi_amd import op as mop

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def comm():
    c = coll.Communicator(f"oscfuzz_{np.random.randint(1 << 30)}", 0, 1, 0)
    yield c
    c.free()


def origin_type(rng, nelem, prim):
    """None (contiguous) or a vector of `prim` with a random block length
    dividing `nelem` and a random gap."""
    if rng.random() < 0.3:
        return None, nelem * prim.size
    divs = [b for b in range(1, 65) if nelem % b == 0]
    bl = int(rng.choice(divs))
    return dd.type_vector(nelem // bl, bl, bl + int(rng.integers(0, 5)), prim), 1


def pick_target(rng, bases):
    while True:
        tdt = rand_type(rng, int(rng.integers(1, 4)), bases)
        if 0 < tdt.size <= (1 << 20) and tdt.extent > 0 and len(tdt.runs) <= 20000:
            break
    tcount = max(1, int(rng.choice([1, 3, 17, 200, 2000])) * 64 // max(tdt.size, 64))
    tcount = min(tcount, max(1, (2 << 20) // tdt.size))
    return tdt, tcount


def make_window(comm, nbytes, seed):
    base = torch.empty(nbytes, dtype=torch.uint8, device=DEV)
    g = torch.Generator(device=DEV).manual_seed(seed)
    base.random_(0, 256, generator=g)
    torch.cuda.synchronize()
    return base, osc.Window.create(comm, base, nbytes, disp_unit=1)


def origin_bytes(odt, ocount, stream_np, seed, orc):
    """An origin buffer (random fill) whose odt typemap holds `stream_np`."""
    span = span_of(odt, ocount) if odt is not None else stream_np.nbytes
    fill = np.random.default_rng(seed).integers(0, 256, span, dtype=np.uint8)
    if odt is None:
        fill[:] = stream_np
    else:
        orc.unpack(odt.runs, odt.extent, ocount, stream_np, fill, 0)
    return fill


@pytest.mark.parametrize("seed", range(40))
def test_put_get_random_types(orc, comm, seed):
    rng = np.random.default_rng(11000 + seed)
    tdt, tcount = pick_target(rng, ["MPI_CHAR", "MPI_SHORT", "MPI_INT", "MPI_DOUBLE"])
    total = tdt.size * tcount
    disp = int(rng.integers(0, 64))
    W = disp + span_of(tdt, tcount) + 64
    prim = dd.predefined("MPI_CHAR")
    odt, ocount = origin_type(rng, total, prim)
    if odt is not None:
        ocount = 1
    what = f"seed {seed}: target {tdt.name} x {tcount} ({total} B) at {disp}, origin {odt.name if odt else 'bytes'}"
    base, win = make_window(comm, W, 600 + seed)
    try:
        stream = np.random.default_rng(700 + seed).integers(0, 256, total, dtype=np.uint8)
        org_np = origin_bytes(odt, ocount, stream, 800 + seed, orc)
        org = torch.from_numpy(org_np).to(DEV)
        before = base.cpu().numpy().copy()
        win.lock(0, osc.LOCK_EXCLUSIVE)
        win.put_ddt(org, ocount if odt else total, odt, 0, disp, tcount, tdt)
        win.unlock(0)
        win.sync()
        torch.cuda.synchronize()
        exp = before.copy()
        view = exp[disp:]
        orc.unpack(tdt.runs, tdt.extent, tcount, stream, view, 0)
        exp[disp:] = view
        bad = np.flatnonzero(base.cpu().numpy() != exp)
        assert bad.size == 0, f"{what}: put differs first at window byte {bad[:1]}"
        # get it back into a freshly filled origin buffer
        back = torch.from_numpy(np.random.default_rng(900 + seed).integers(
            0, 256, org_np.nbytes, dtype=np.uint8)).to(DEV)
        exp_back = back.cpu().numpy().copy()
        if odt is None:
            exp_back[:] = stream
        else:
            orc.unpack(odt.runs, odt.extent, ocount, stream, exp_back, 0)
        win.lock(0, osc.LOCK_SHARED)
        win.get_ddt(back, ocount if odt else total, odt, 0, disp, tcount, tdt)
        win.unlock(0)
        torch.cuda.synchronize()
        bad = np.flatnonzero(back.cpu().numpy() != exp_back)
        assert bad.size == 0, f"{what}: get differs first at origin byte {bad[:1]}"
    finally:
        win.free()
        tdt.free()
        if odt is not None:
            odt.free()


@pytest.mark.parametrize("seed", range(40))
def test_accumulate_random_types(orc, comm, seed):
    rng = np.random.default_rng(12000 + seed)
    D = dd.predefined("MPI_DOUBLE")
    tdt, tcount = pick_target(rng, ["MPI_DOUBLE"])
    total = tdt.size * tcount
    n = total // 8
    disp = 8 * int(rng.integers(0, 8))
    W = disp + span_of(tdt, tcount) + 64
    odt, ocount = origin_type(rng, n, D)
    if odt is not None:
        ocount = 1
    what = f"seed {seed}: target {tdt.name} x {tcount} ({n} doubles) at {disp}, origin {odt.name if odt else 'contiguous'}"
    # every byte below 0x40: a double read at ANY byte offset (struct
    # members need not be 8-B aligned) is finite, so old + stream is exact
    # IEEE arithmetic on both sides, no NaN payloads to compare
    wbytes = torch.randint(0, 0x40, (W + 64,), dtype=torch.uint8, device=DEV)
    win = osc.Window.create(comm, wbytes, W, disp_unit=1)
    try:
        stream = np.random.default_rng(1300 + seed).integers(-1000, 1000, n).astype(np.float64)
        org_np = origin_bytes(odt, ocount, stream.view(np.uint8), 1400 + seed, orc)
        org = torch.from_numpy(org_np).to(DEV)
        before = wbytes.cpu().numpy()[:W].copy()
        result = torch.zeros(n, dtype=torch.float64, device=DEV)
        win.lock(0, osc.LOCK_EXCLUSIVE)
        if rng.random() < 0.5:
            win.accumulate_ddt(org, ocount if odt else n, odt, 0, disp, tcount, tdt, mop.MPI_DOUBLE,
                               mop.MPI_SUM)
            fetched = False
        else:
            win.get_accumulate_ddt(org, ocount if odt else n, odt, result, n, None, 0, disp, tcount, tdt,
                                   mop.MPI_DOUBLE, mop.MPI_SUM)
            fetched = True
        win.unlock(0)
        win.sync()
        torch.cuda.synchronize()
        old = orc.pack(tdt.runs, tdt.extent, tcount, before[disp:].copy(), 0, total).view(np.float64)
        new = (old + stream).view(np.uint8)
        exp = before.copy()
        view = exp[disp:]
        orc.unpack(tdt.runs, tdt.extent, tcount, new, view, 0)
        exp[disp:] = view
        bad = np.flatnonzero(wbytes.cpu().numpy()[:W] != exp)
        assert bad.size == 0, f"{what}: accumulate differs first at window byte {bad[:1]}"
        if fetched:
            assert np.array_equal(result.cpu().numpy().view(np.uint8), old.view(np.uint8)), \
                f"{what}: fetched values"
    finally:
        win.free()
        tdt.free()
        if odt is not None:
            odt.free()
