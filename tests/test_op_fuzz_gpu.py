"""Randomized MPI_Op parity: random (op, type) slots, element counts from 1
to 300k and independent element-granular displacements of the three
operands inside their 16-B vectors (the vector body, the peeled head, the
per-element path and every mix), 3-buffer and 2-buffer, bit-exact against
the oracle's op/base restatement, guard bytes after the result untouched.
Data and helpers as tests/test_op_gpu.py (NaN, ±0, ±inf, denormals, ties)."""
import numpy as np
import pytest

from ompi_amd import op as mop
from test_op_gpu import SLOTS, from_dev, gen, same_bits, to_dev

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", range(120))
def test_op_random_slots_offsets(orc, seed):
    rng = np.random.default_rng(31000 + seed)
    slots = [(o, d) for o, d in SLOTS if orc.defined(o.index, d.code)]  # op/base's non-NULL slots
    op, dt = slots[int(rng.integers(len(slots)))]
    ext = dt.extent
    n = int(rng.choice([1, 2, 7, 63, 1000, 4097, 65536 + 5, 300001]))
    offs = [ext * int(rng.integers(0, 16 // ext + 1)) if ext <= 16 else 0 for _ in range(3)]
    what = f"seed {seed}: {op.name} {dt.name} n={n} offsets={offs}"
    a = gen(dt, n, 700 + seed)
    b = gen(dt, n, 800 + seed)
    out0 = gen(dt, n + 4, 900 + seed)
    ta, pa = to_dev(a, offs[0])
    tb, pb = to_dev(b, offs[1])
    raw_out = np.ascontiguousarray(out0).view(np.uint8)
    to, po = to_dev(out0, offs[2])
    mop.reduce_local_3buff_async(pa, pb, po, n, dt, op)
    torch.cuda.synchronize()
    exp3 = out0[:n].copy()
    orc.op_3buff(op.index, dt.code, a, b, exp3, n)
    got = from_dev(to, offs[2], raw_out.nbytes)
    assert same_bits(got[:n * ext].view(dt.np_dtype), exp3, dt), what + " (3-buffer)"
    assert np.array_equal(got[n * ext:], raw_out[n * ext:]), what + " (guard bytes)"
    ta, pa = to_dev(a, offs[0])
    tb, pb = to_dev(b, offs[2])
    mop.reduce_local_async(pa, pb, n, dt, op)
    torch.cuda.synchronize()
    exp = b.copy()
    orc.op_2buff(op.index, dt.code, a, exp, n)
    got2 = from_dev(tb, offs[2], n * ext).view(dt.np_dtype)
    assert same_bits(got2, exp, dt), what + " (2-buffer)"
