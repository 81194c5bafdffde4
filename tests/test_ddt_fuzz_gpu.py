"""Randomized convertor parity: random nested datatypes (contiguous /
vector / indexed / struct over char, short, int and double, up to three
levels), random counts from a few bytes to several MiB packed, typed bases
off alignment, packed buffers at odd offsets, and the stream moved in
random-length convertor calls (opal_convertor_pack / _unpack resumed at
bConverted, ddt_test.c:258-337) and in one random iovec train (fAdvance with
out_size > 1).  Every kernel the dispatcher can pick — the staged tile, the
16-B walk, the generic element search, the byte edges, the iovec kernels —
is reached by some seed.  Pack byte-exact against the oracle's pack; unpack
into a pre-filled typed buffer byte-exact against the oracle's unpack into
the same bytes (gap bytes untouched)."""
import numpy as np
import pytest

from ddt_random import rand_type, span_of
from ompi_amd import datatype as dd

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def make_case(seed):
    rng = np.random.default_rng(7000 + seed)
    while True:
        dt = rand_type(rng, int(rng.integers(1, 4)))
        if (dt.size == 0 or dt.extent <= 0 or dt.size > (4 << 20) or len(dt.elems) > 2048
                or len(dt.runs) > 20000):
            continue
        break
    target = int(rng.choice([1 << 10, 60 << 10, 700 << 10, 3 << 20]))
    count = max(1, target // dt.size)
    count = min(count, max(1, (48 << 20) // max(dt.extent, 1)))
    return rng, dt, count


def dev_rand(n, seed):
    t = torch.empty(n + 64, dtype=torch.uint8, device=DEV)
    g = torch.Generator(device=DEV).manual_seed(seed)
    t.random_(0, 256, generator=g)
    return t


def chunk_lengths(rng, total, max_calls=400):
    """Random call lengths covering `total` bytes in at most max_calls calls."""
    kind = int(rng.integers(4))
    if kind == 0 or total <= 16:
        return [total]
    if kind == 1:
        c = int(rng.choice([12, 4099, 65536]))
        c = max(c, -(-total // max_calls))
        k = -(-total // c)
        return [c] * (k - 1) + [total - c * (k - 1)]
    lens, left = [], total
    lo = max(1, total // max_calls)
    while left > 0:
        n = min(left, int(rng.integers(lo, max(lo + 1, 2 * total // max(1, max_calls // 4)))))
        lens.append(n)
        left -= n
    return lens


@pytest.mark.parametrize("seed", range(200))
def test_convertor_random_types(orc, seed):
    rng, dt, count = make_case(seed)
    total = dt.size * count
    span = span_of(dt, count)
    shift = int(rng.choice([0, 0, 0, 1, 2, 4, 8, 12]))  # 16-B granules need 0
    runs = dt.runs
    src = dev_rand(span + shift, 100 + seed)
    src_np = src.cpu().numpy()[shift:shift + span].copy()
    exp = orc.pack(runs, dt.extent, count, src_np, 0, total)
    assert exp.nbytes == total
    what = f"seed {seed}: {dt.name} x {count} ({len(dt.elems)} elems, {total} B, shift {shift})"

    # pack in random-length calls into a buffer at an odd offset
    poff = int(rng.choice([0, 0, 16, 1, 3, 8]))
    packed = torch.zeros(total + poff + 64, dtype=torch.uint8, device=DEV)
    conv = dd.Convertor()
    conv.prepare_for_send(dt, count, src.data_ptr() + shift)
    pos = 0
    for n in chunk_lengths(rng, total):
        done, moved = conv.pack(packed.data_ptr() + poff + pos, n)
        assert moved == min(n, total - pos), what
        pos += moved
    assert pos == total and done == 1, what
    torch.cuda.synchronize()
    got = packed.cpu().numpy()[poff:poff + total]
    bad = np.flatnonzero(got != exp)
    assert bad.size == 0, f"{what}: pack differs first at {bad[:1]}"

    # unpack in other random-length calls into a pre-filled typed buffer
    fill = dev_rand(span + shift, 200 + seed)
    exp_dst = fill.cpu().numpy()[shift:shift + span].copy()
    orc.unpack(runs, dt.extent, count, exp, exp_dst, 0)
    conv = dd.Convertor()
    conv.prepare_for_recv(dt, count, fill.data_ptr() + shift)
    pos = 0
    for n in chunk_lengths(rng, total):
        _, moved = conv.unpack(packed.data_ptr() + poff + pos, n)
        pos += moved
    assert pos == total, what
    torch.cuda.synchronize()
    got_dst = fill.cpu().numpy()[shift:shift + span]
    bad = np.flatnonzero(got_dst != exp_dst)
    assert bad.size == 0, f"{what}: unpack differs first at typed byte {bad[:1]}"

    # one iovec train: random fragment lengths at random gaps, two calls
    lens = chunk_lengths(rng, total, max_calls=120)
    gaps = rng.integers(0, 24, len(lens))
    offs = np.concatenate([[0], np.cumsum(np.array(lens) + gaps)[:-1]]).astype(np.int64)
    train = torch.zeros(int(offs[-1]) + lens[-1] + 64, dtype=torch.uint8, device=DEV)
    iovs = [(train.data_ptr() + int(o), int(n)) for o, n in zip(offs, lens)]
    half = max(1, len(iovs) // 2)
    conv = dd.Convertor()
    conv.prepare_for_send(dt, count, src.data_ptr() + shift)
    moved_all = 0
    for part in (iovs[:half], iovs[half:]):
        if part:
            _, _, _, moved = conv.pack_iov(part)
            moved_all += moved
    assert moved_all == total, what
    torch.cuda.synchronize()
    t_np = train.cpu().numpy()
    got = np.concatenate([t_np[o:o + n] for o, n in zip(offs, lens)])
    bad = np.flatnonzero(got != exp)
    assert bad.size == 0, f"{what}: iovec pack differs first at {bad[:1]}"
    fill2 = dev_rand(span + shift, 300 + seed)
    exp_dst2 = fill2.cpu().numpy()[shift:shift + span].copy()
    orc.unpack(runs, dt.extent, count, exp, exp_dst2, 0)
    conv = dd.Convertor()
    conv.prepare_for_recv(dt, count, fill2.data_ptr() + shift)
    for part in (iovs[:half], iovs[half:]):
        if part:
            conv.unpack_iov(part)
    torch.cuda.synchronize()
    got_dst = fill2.cpu().numpy()[shift:shift + span]
    bad = np.flatnonzero(got_dst != exp_dst2)
    assert bad.size == 0, f"{what}: iovec unpack differs first at typed byte {bad[:1]}"
    dt.free()


@pytest.mark.parametrize("seed", range(24))
def test_walk16_random_vectors(orc, seed):
    """The 16-B walk (ddt_vec_kernel's chunked persistent form: a pack whose
    gaps exceed the tile's 128 B, an unpack whose gaps exceed 4 KiB, windows
    under 256 KiB): vectors of 16-B-multiple double runs at random strides
    and counts, 16-B-aligned bases, windows of random length (head / tail
    bytes off the granule grid when a length is not a multiple of 16)."""
    rng = np.random.default_rng(9000 + seed)
    d = dd.predefined("MPI_DOUBLE")
    bl = 2 * int(rng.integers(1, 41))
    gap = int(rng.choice([2, 18, 66, 520, 700]))
    count = max(1, int(rng.integers(100 << 10, 4 << 20)) // (8 * bl))
    dt = dd.type_vector(count, bl, bl + gap, d)
    total, span = dt.size, span_of(dt, 1)
    src = dev_rand(span, 400 + seed)
    exp = orc.pack(dt.runs, dt.extent, 1, src.cpu().numpy()[:span].copy(), 0, total)
    what = f"seed {seed}: vector({count}, {bl}, {bl + gap}) doubles, {total} B"
    packed = torch.zeros(total + 64, dtype=torch.uint8, device=DEV)
    conv = dd.Convertor()
    conv.prepare_for_send(dt, 1, src)
    pos = 0
    for n in chunk_lengths(rng, total, max_calls=64):
        pos += conv.pack(packed.data_ptr() + pos, n)[1]
    assert pos == total, what
    torch.cuda.synchronize()
    bad = np.flatnonzero(packed.cpu().numpy()[:total] != exp)
    assert bad.size == 0, f"{what}: pack differs first at {bad[:1]}"
    fill = dev_rand(span, 500 + seed)
    exp_dst = fill.cpu().numpy()[:span].copy()
    orc.unpack(dt.runs, dt.extent, 1, exp, exp_dst, 0)
    conv = dd.Convertor()
    conv.prepare_for_recv(dt, 1, fill)
    pos = 0
    for n in chunk_lengths(rng, total, max_calls=64):
        pos += conv.unpack(packed.data_ptr() + pos, n)[1]
    torch.cuda.synchronize()
    bad = np.flatnonzero(fill.cpu().numpy()[:span] != exp_dst)
    assert bad.size == 0, f"{what}: unpack differs first at typed byte {bad[:1]}"
    dt.free()
