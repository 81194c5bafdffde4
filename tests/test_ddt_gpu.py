"""GPU parity of the datatype pack/unpack offload against the oracle
(byte-exact), driven the way the reference's own tests drive the convertor
(ddt_test.c local_copy_with_convertor: pack in fixed-size chunks, then
unpack in chunks, test/datatype/ddt_test.c:258-337)."""
import numpy as np
import pytest

from ompi_amd import datatype as dd

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def dev_bytes(n, seed=None, offset=0):
    t = torch.zeros(n + offset + 64, dtype=torch.uint8, device=DEV)
    if seed is not None:
        g = torch.Generator(device=DEV).manual_seed(seed)
        t.random_(0, 256, generator=g)
    return t


def span_of(dt, count):
    return (count - 1) * dt.extent + dt.true_span


def kat_types(golden):
    out = []
    for t in golden("ddt_kat.json")["types"]:
        blocks = [tuple(b) for b in t["blocks"]]
        dt = dd.from_runs(t["name"], blocks, t["extent"])
        out.append((dt, t["count"], t["chunks"], blocks))
    return out


def chunked(conv, fn, buf_ptr, total, chunk):
    pos = 0
    while True:
        done, n = fn(buf_ptr + pos, chunk)
        pos += n
        if done:
            break
        assert n > 0
    assert pos == total


def test_ddt_kat_types_pack_unpack(orc, golden):
    for dt, count, chunks, blocks in kat_types(golden):
        span = span_of(dt, count)
        src = dev_bytes(span, seed=1)
        src_np = src.cpu().numpy()
        total = dt.size * count
        exp = orc.pack(blocks, dt.extent, count, src_np, 0, total)
        assert exp.nbytes == total
        for chunk in chunks + [total]:
            packed = dev_bytes(total)
            conv = dd.Convertor()
            conv.prepare_for_send(dt, count, src)
            chunked(conv, conv.pack, packed.data_ptr(), total, chunk)
            torch.cuda.synchronize()
            got = packed[:total].cpu().numpy()
            assert np.array_equal(got, exp), (dt.name, chunk)
            # unpack into a zeroed typed buffer, in chunks
            dst = dev_bytes(span)
            conv = dd.Convertor()
            conv.prepare_for_recv(dt, count, dst)
            chunked(conv, conv.unpack, packed.data_ptr(), total, chunk)
            torch.cuda.synchronize()
            dst_np = dst.cpu().numpy()
            exp_dst = np.zeros_like(dst_np)
            orc.unpack(blocks, dt.extent, count, exp, exp_dst, 0)
            assert np.array_equal(dst_np, exp_dst), (dt.name, chunk, "unpack")


@pytest.mark.parametrize("bl", [1, 2, 8, 64])
def test_vector_config3(orc, bl):
    """BASELINE config 3: vector(count, bl doubles, stride 2*bl), chunk sizes
    whole / 64 KiB / 12 B (12 B splits doubles, ddt_test.c:479-483)."""
    d = dd.predefined("MPI_DOUBLE")
    count = (256 * 1024) // (8 * bl)   # 256 KiB packed
    dt = dd.type_vector(count, bl, 2 * bl, d)
    assert dt.nelems == 1  # folded to one {count, blocklen, stride} element
    span = span_of(dt, 1)
    src = dev_bytes(span, seed=bl)
    src_np = src.cpu().numpy()
    exp = orc.pack(dt.runs, dt.extent, 1, src_np, 0, dt.size)
    for chunk in (dt.size, 65536, 12):
        if chunk == 12 and bl > 2:
            continue  # 12-byte chunks over 256 KiB = 21k launches: keep for small
        packed = dev_bytes(dt.size)
        conv = dd.Convertor()
        conv.prepare_for_send(dt, 1, src)
        chunked(conv, conv.pack, packed.data_ptr(), dt.size, chunk)
        torch.cuda.synchronize()
        assert np.array_equal(packed[:dt.size].cpu().numpy(), exp), (bl, chunk)


@pytest.mark.parametrize("bl,stride,shift", [(8, 16, 0), (8, 16, 8), (9, 19, 8), (16, 32, 24),
                                             (5, 13, 4)])
def test_vector_gapped_tile_pack(orc, bl, stride, shift):
    """The staged tile pack of vector runs with gaps of 64-128 B (read
    through into LDS, batched): run phases that drift across 16 B (stride
    19 / 13 doubles), a typed base off 16-B alignment by `shift` bytes, and
    a 64 KiB-fragment train whose windows start mid-period; the gap bytes
    hold random data that must never reach the packed stream."""
    d = dd.predefined("MPI_DOUBLE")
    count = (512 * 1024) // (8 * bl) + 3
    dt = dd.type_vector(count, bl, stride, d)
    span = span_of(dt, 1)
    src = dev_bytes(span + shift, seed=stride)
    src_np = src.cpu().numpy()[shift:shift + span]
    exp = orc.pack(dt.runs, dt.extent, 1, src_np, 0, dt.size)
    for chunk in (dt.size, 65536 + 8):
        packed = dev_bytes(dt.size)
        conv = dd.Convertor()
        conv.prepare_for_send(dt, 1, src.data_ptr() + shift)
        chunked(conv, conv.pack, packed.data_ptr(), dt.size, chunk)
        torch.cuda.synchronize()
        assert np.array_equal(packed[:dt.size].cpu().numpy(), exp), (bl, stride, shift, chunk)


def test_struct_int_double_offsets(orc):
    i32, f64 = dd.predefined("MPI_INT"), dd.predefined("MPI_DOUBLE")
    dt = dd.type_struct([1, 1], [0, 8], [i32, f64])
    assert (dt.size, dt.extent) == (12, 16)
    count = 3001
    for base_off in (0, 4, 8):
        src = dev_bytes(span_of(dt, count), seed=5, offset=base_off)
        ptr = src.data_ptr() + base_off
        src_np = src.cpu().numpy()[base_off:]
        exp = orc.pack(dt.runs, dt.extent, count, src_np.copy(), 0, dt.size * count)
        for pos, chunk in ((0, 12 * count), (5, 1000), (7, 12), (12 * count - 3, 64)):
            packed = dev_bytes(chunk, offset=3)
            conv = dd.Convertor()
            conv.prepare_for_send(dt, count, ptr)
            conv.set_position(pos)
            done, n = conv.pack(packed.data_ptr() + 3, chunk)
            torch.cuda.synchronize()
            assert n == min(chunk, 12 * count - pos)
            assert np.array_equal(packed[3:3 + n].cpu().numpy(), exp[pos:pos + n]), (base_off, pos)


def test_indexed_upper_triangular_large(orc):
    """Size-independent property at 64 MiB-class: pack -> unpack round trip
    restores exactly the typemap bytes and nothing else."""
    d = dd.predefined("MPI_DOUBLE")
    n = 2048
    dt = dd.type_indexed([n - i for i in range(n)], [i * n + i for i in range(n)], d)
    span = span_of(dt, 1)
    src = dev_bytes(span, seed=9)
    packed = dev_bytes(dt.size)
    conv = dd.Convertor()
    conv.prepare_for_send(dt, 1, src)
    done, nb = conv.pack(packed, dt.size)
    assert done == 1 and nb == dt.size
    dst = dev_bytes(span)
    conv = dd.Convertor()
    conv.prepare_for_recv(dt, 1, dst)
    conv.unpack(packed, dt.size)
    torch.cuda.synchronize()
    mask = np.zeros(span, dtype=bool)
    for dsp, ln in dt.runs:
        mask[dsp:dsp + ln] = True
    s, t = src[:span].cpu().numpy(), dst[:span].cpu().numpy()
    assert np.array_equal(s[mask], t[mask])
    assert not t[~mask].any()


@pytest.mark.parametrize("layout", ["struct_int_double", "blacs", "vector_bl1_single",
                                    "vector5_bl1_tiled", "struct_neg_lb", "contig_resized"])
def test_tile_pack_layouts(orc, layout):
    """Layouts the staged LDS tile pack takes (periodic, sub-16-B granules,
    small gaps), many tiles, whole-stream and odd-chunk windows, misaligned
    packed destination: byte-exact vs the oracle."""
    i32, f64 = dd.predefined("MPI_INT"), dd.predefined("MPI_DOUBLE")
    if layout == "struct_int_double":
        dt, count = dd.type_struct([1, 1], [0, 8], [i32, f64]), 200003
    elif layout == "blacs":
        lens = [13, 13, 13, 13, 13, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1]
        disps = [286, 308, 330, 352, 374, 396, 419, 442, 465, 488, 511, 534, 557, 580, 603,
                 626, 649, 672]
        dt, count = dd.type_indexed(lens, disps, i32), 4001
    elif layout == "vector_bl1_single":
        dt, count = dd.type_vector(300007, 1, 2, f64), 1
    elif layout == "vector5_bl1_tiled":
        dt, count = dd.type_vector(5, 1, 2, f64), 50001
    elif layout == "struct_neg_lb":
        dt, count = dd.type_struct([1, 2], [-8, 4], [f64, i32]), 70001
    else:
        dt, count = dd.type_struct([3], [4], [i32]), 100001   # 12 B at +4, extent 16
    total = dt.size * count
    lb = min(d for d, _ in dt.runs)
    src = dev_bytes(span_of(dt, count) + max(0, -lb), seed=11)
    base = src.data_ptr() + max(0, -lb)
    src_np = src.cpu().numpy()[max(0, -lb):]
    if lb < 0:  # oracle indexes from the typed base: shift the runs
        runs = [(d - lb, n) for d, n in dt.runs]
        exp = orc.pack(runs, dt.extent, count, src.cpu().numpy().copy(), 0, total)
    else:
        exp = orc.pack(dt.runs, dt.extent, count, src_np.copy(), 0, total)
    for chunk, dst_off in ((total, 0), (300007, 5), (262147, 0), (65536, 0), (7777, 8)):
        packed = dev_bytes(total, offset=dst_off)
        conv = dd.Convertor()
        conv.prepare_for_send(dt, count, base)
        chunked(conv, conv.pack, packed.data_ptr() + dst_off, total, chunk)
        torch.cuda.synchronize()
        got = packed[dst_off:dst_off + total].cpu().numpy()
        assert np.array_equal(got, exp), (layout, chunk, dst_off)


@pytest.mark.parametrize("layout", ["struct_int_double", "blacs", "vector_bl1_single",
                                    "vector5_bl1_tiled", "struct_neg_lb", "contig_resized",
                                    "vector_bl2_single"])
def test_tile_unpack_layouts(orc, layout):
    """Staged LDS tile unpack over the same layouts: chunked windows with
    partial periods at both ends, misaligned packed source, typed buffer
    pre-filled so that any write into a gap byte shows: byte-exact vs the
    oracle's unpack into the same pre-filled buffer."""
    i32, f64 = dd.predefined("MPI_INT"), dd.predefined("MPI_DOUBLE")
    if layout == "struct_int_double":
        dt, count = dd.type_struct([1, 1], [0, 8], [i32, f64]), 200003
    elif layout == "blacs":
        lens = [13, 13, 13, 13, 13, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1]
        disps = [286, 308, 330, 352, 374, 396, 419, 442, 465, 488, 511, 534, 557, 580, 603,
                 626, 649, 672]
        dt, count = dd.type_indexed(lens, disps, i32), 4001
    elif layout == "vector_bl1_single":
        dt, count = dd.type_vector(300007, 1, 2, f64), 1
    elif layout == "vector_bl2_single":
        dt, count = dd.type_vector(100003, 2, 4, f64), 1
    elif layout == "vector5_bl1_tiled":
        dt, count = dd.type_vector(5, 1, 2, f64), 50001
    elif layout == "struct_neg_lb":
        dt, count = dd.type_struct([1, 2], [-8, 4], [f64, i32]), 70001
    else:
        dt, count = dd.type_struct([3], [4], [i32]), 100001   # 12 B at +4, extent 16
    total = dt.size * count
    lb = min(d for d, _ in dt.runs)
    shift = max(0, -lb)
    runs = [(d + shift, n) for d, n in dt.runs]
    span = span_of(dt, count) + shift
    packed_np = np.random.default_rng(3).integers(0, 256, total + 64, dtype=np.uint8)
    fill = dev_bytes(span, seed=13)
    fill_np = fill.cpu().numpy()
    exp = fill_np.copy()
    orc.unpack(runs, dt.extent, count, packed_np[:total].copy(), exp, 0)
    for chunk, src_off in ((total, 0), (300007, 5), (262147, 0), (65536, 0), (7777, 8)):
        packed = torch.from_numpy(packed_np[:total].copy())
        pbuf = torch.zeros(total + src_off + 64, dtype=torch.uint8, device=DEV)
        pbuf[src_off:src_off + total] = packed.to(DEV)
        dst = fill.clone()
        conv = dd.Convertor()
        conv.prepare_for_recv(dt, count, dst.data_ptr() + shift)
        chunked(conv, conv.unpack, pbuf.data_ptr() + src_off, total, chunk)
        torch.cuda.synchronize()
        got = dst.cpu().numpy()
        assert np.array_equal(got, exp), (layout, chunk, src_off,
                                          int(np.flatnonzero(got != exp)[:1].sum()))


def tile_layout(layout, count_cap=None):
    i32, f64 = dd.predefined("MPI_INT"), dd.predefined("MPI_DOUBLE")
    lens = [13, 13, 13, 13, 13, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1]
    disps = [286, 308, 330, 352, 374, 396, 419, 442, 465, 488, 511, 534, 557, 580, 603,
             626, 649, 672]
    mk = {
        "struct_int_double": (lambda c: dd.type_struct([1, 1], [0, 8], [i32, f64]), 200003, True),
        "blacs": (lambda c: dd.type_indexed(lens, disps, i32), 4001, True),
        "vector_bl1_single": (lambda c: dd.type_vector(c, 1, 2, f64), 300007, False),
        "vector_bl8_single": (lambda c: dd.type_vector(c, 8, 16, f64), 40009, False),
        "vector5_bl1_tiled": (lambda c: dd.type_vector(5, 1, 2, f64), 50001, True),
        "struct_neg_lb": (lambda c: dd.type_struct([1, 2], [-8, 4], [f64, i32]), 70001, True),
        "contig_resized": (lambda c: dd.type_struct([3], [4], [i32]), 100001, True),
    }
    fn, count, tiled_count = mk[layout]
    if count_cap:
        count = max(3, min(count, count_cap))
    if tiled_count:
        return fn(None), count
    return fn(count), 1


IOV_LAYOUTS = ["struct_int_double", "blacs", "vector_bl1_single", "vector_bl8_single",
               "vector5_bl1_tiled", "struct_neg_lb", "contig_resized"]


@pytest.mark.parametrize("layout", IOV_LAYOUTS)
@pytest.mark.parametrize("frag", [65536, 4099, 12])
def test_iov_train_layouts(orc, layout, frag):
    """fAdvance over iovec trains (ompi_amd_ddt_pack_iov / _unpack_iov, one
    launch per call; periodic layouts run the staged tile kernels per iovec,
    partial periods at each fragment's ends byte by byte): the stream in
    `frag`-byte fragments at odd offsets (64 KiB ones aligned) of one device buffer, several calls
    of up to 97 iovecs each, resumed at bConverted.  Pack byte-exact vs the
    oracle; unpack into a pre-filled typed buffer byte-exact vs the oracle's
    unpack into the same buffer (gap bytes untouched)."""
    probe, _ = tile_layout(layout)
    cap = None if frag >= 4096 else max(3, (frag * 6000) // probe.size)
    dt, count = tile_layout(layout, cap)
    total = dt.size * count
    lb = min(d for d, _ in dt.runs)
    shift = max(0, -lb)
    runs = [(d + shift, n) for d, n in dt.runs]
    span = span_of(dt, count) + shift
    src = dev_bytes(span, seed=21)
    exp = orc.pack(runs, dt.extent, count, src.cpu().numpy()[:span].copy(), 0, total)
    nfrag = (total + frag - 1) // frag
    # 64 KiB fragments 16-B aligned (the type's own granule), the others at
    # odd offsets (byte granules)
    off, pitch = (0, frag + 16) if frag == 65536 else (1, frag + 3)
    packed = dev_bytes(nfrag * pitch + 16, seed=22)
    base = packed.data_ptr() + off
    iovs = [(base + i * pitch, frag) for i in range(nfrag)]
    per_call = 97
    conv = dd.Convertor()
    conv.prepare_for_send(dt, count, src.data_ptr() + shift)
    pos = 0
    for c0 in range(0, nfrag, per_call):
        rc, lens, used, moved = conv.pack_iov(iovs[c0:c0 + per_call])
        want = min(per_call * frag, total - pos)
        assert moved == want and sum(lens) == want, (layout, frag, c0)
        pos += moved
        assert rc == (1 if pos == total else 0)
    torch.cuda.synchronize()
    got_all = packed.cpu().numpy()
    got = np.concatenate([got_all[off + i * pitch:off + i * pitch + min(frag, total - i * frag)]
                          for i in range(nfrag)])
    assert np.array_equal(got, exp), (layout, frag, int(np.flatnonzero(got != exp)[:1].sum()))
    # unpack the same fragments into a pre-filled typed buffer
    fill = dev_bytes(span, seed=23)
    want_typed = fill.cpu().numpy().copy()
    orc.unpack(runs, dt.extent, count, exp.copy(), want_typed, 0)
    conv = dd.Convertor()
    conv.prepare_for_recv(dt, count, fill.data_ptr() + shift)
    pos = 0
    for c0 in range(0, nfrag, per_call):
        rc, lens, used, moved = conv.unpack_iov(iovs[c0:c0 + per_call])
        pos += moved
        assert rc == (1 if pos == total else 0)
    torch.cuda.synchronize()
    out = fill.cpu().numpy()
    assert np.array_equal(out, want_typed), (layout, frag, "unpack",
                                             int(np.flatnonzero(out != want_typed)[:1].sum()))
