"""CPU coverage of the multi-rank path (no GPU): the shared-memory
rendezvous across processes, and — over a world_size 2/3 gloo group — the
block partition / ring ownership the GPU allreduce uses, reassembled and
checked bit-exactly against the oracle's simulation of coll/tuned."""
import os
import shutil
import subprocess
import sys
import uuid

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    from ompi_amd import _lib
    _lib.load()
    out = tmp_path_factory.mktemp("h") / "boot_harness"
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no g++")
    libdir = os.path.join(ROOT, "ompi_amd")
    subprocess.run([cxx, "-O1", "-std=c++17", os.path.join(ROOT, "tests", "harness", "boot_harness.cpp"),
                    "-o", str(out), f"-L{libdir}", "-lompi_amd", f"-Wl,-rpath,{libdir}"],
                   check=True)
    return str(out)


@pytest.mark.parametrize("n", [2, 5])
def test_shm_rendezvous_multiprocess(harness, n):
    name = f"test_{uuid.uuid4().hex[:10]}"
    procs = [subprocess.Popen([harness, name, str(r), str(n), "200"], stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(n)]
    for p in procs:
        out, err = p.communicate(timeout=60)
        assert p.returncode == 0, (p.returncode, out, err)
    assert not os.path.exists(f"/dev/shm/ompi_amd_{name}")  # unlinked after attach


def _plan_worker(rank, world, port, q):
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch

    from ompi_amd import coll
    from oracle import oracle as orc
    try:
        for count in (10007, 3 * 262144 + 5, 2500):
            xs = [np.random.default_rng(100 + r).uniform(-1, 1, count).astype(np.float32)
                  for r in range(world)]
            # the block this rank produces and its offsets, as the library plans them
            block = next(b for b in range(world) if coll.block_owner(world, b) == rank)
            off, cnt = coll.block_partition(count, world, block)
            # ring operand order: acc = x[b]; acc = x[b+j] (+) acc
            acc = xs[block][off:off + cnt].copy()
            for j in range(1, world):
                out = xs[(block + j) % world][off:off + cnt].copy()
                orc.op_2buff(3, 15, acc, out, cnt)  # out = out + acc
                acc = out
            pieces = [None] * world
            dist.all_gather_object(pieces, (block, off, acc.tobytes()))
            full = np.zeros(count, dtype=np.float32)
            for b, o, data in pieces:
                arr = np.frombuffer(data, dtype=np.float32)
                full[o:o + arr.size] = arr
            exp, alg = orc.allreduce(xs, count, 3, 15, orc.ALG_RING)
            assert np.array_equal(full.view(np.uint32), exp[rank].view(np.uint32)), count
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()
        del torch


@pytest.mark.parametrize("world", [2, 3])
def test_ring_plan_gloo(world):
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_plan_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(v == "ok" for v in res.values()), res


def test_block_partition_matches_oracle():
    from ompi_amd import coll
    from oracle import oracle as orc
    for count in (1, 7, 8, 9, 1000003):
        for n in (2, 3, 8, 16):
            split, early, late = orc.blockcount(count, n)
            tot = 0
            for b in range(n):
                off, cnt = coll.block_partition(count, n, b)
                assert off == tot and cnt == (early if b < split else late)
                tot += cnt
            assert tot == count
            assert sorted(coll.block_owner(n, b) for b in range(n)) == list(range(n))


@pytest.mark.parametrize("n", [2, 4, 8])
def test_cpu_ring_baseline_matches_oracle(tmp_path, n):
    """The N-process CPU baseline (tools/cpu_ring_baseline.c, the bench's
    `cpu_baseline` for the allreduce and for BASELINE configs[0]) computes
    exactly what the oracle's ring_segmented does: dataset R (U(-1,1), where
    summation orders round differently) at several phases and ragged
    blocks, every rank, every element bit-exact."""
    from oracle import oracle as orc
    exe = os.path.join(ROOT, "tools", "cpu_ring_baseline")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.join(ROOT, "tools"), "cpu_ring_baseline"], check=True,
                       capture_output=True)
    seg = (1 << 20) // 4
    count = 3 * n * seg + 1001  # three phases plus a ragged tail
    xs = [np.random.default_rng(20261015 + r).uniform(-1, 1, count).astype(np.float32) for r in range(n)]
    for r, x in enumerate(xs):
        x.tofile(tmp_path / f"in.{r}")
    subprocess.run([exe, str(n), str(count * 4), "0", "1", str(tmp_path / "in"), str(tmp_path / "out")],
                   check=True, capture_output=True, timeout=300)
    exp, alg = orc.allreduce_forced(xs, count, 3, 15, orc.ALG_RING_SEGMENTED, segsize=1 << 20)
    assert alg == orc.ALG_RING_SEGMENTED
    differs = False
    for r in range(n):
        got = np.fromfile(tmp_path / f"out.{r}", dtype=np.float32)
        assert np.array_equal(got.view(np.uint32), exp[r].view(np.uint32)), r
        # the data really distinguishes orders (N > 2: a left-to-right sum
        # rounds differently somewhere)
        differs = differs or not np.array_equal(got, sum(xs[1:], xs[0].copy()))
    assert differs or n == 2
