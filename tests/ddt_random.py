"""Random nested MPI datatypes for the fuzz tests (contiguous / vector /
indexed / struct, non-overlapping typemaps, non-negative displacements)."""
from ompi_amd import datatype as dd

BASES = ["MPI_CHAR", "MPI_SHORT", "MPI_INT", "MPI_DOUBLE", "MPI_DOUBLE"]


def rand_type(rng, depth, bases=BASES):
    """A random datatype over the predefined `bases`, up to `depth` levels."""
    if depth == 0 or rng.random() < 0.2:
        return dd.predefined(bases[rng.integers(len(bases))])
    old = rand_type(rng, depth - 1, bases)
    k = int(rng.integers(4))
    if k == 0:
        return dd.type_contiguous(int(rng.integers(1, 6)), old)
    if k == 1:
        bl = int(rng.integers(1, 9))
        stride = bl + int(rng.choice([0, 1, 3, bl, 40]))
        return dd.type_vector(int(rng.integers(1, 60)), bl, stride, old)
    if k == 2:
        nb = int(rng.integers(1, 9))
        bls, disps, pos = [], [], int(rng.integers(0, 5))
        for _ in range(nb):
            b = int(rng.integers(0, 7))
            bls.append(b)
            disps.append(pos)
            pos += b + int(rng.integers(0, 7))
        return dd.type_indexed(bls, disps, old)
    m = int(rng.integers(2, 4))
    types = [old] + [rand_type(rng, depth - 1, bases) for _ in range(m - 1)]
    bls, disps, pos = [], [], int(rng.integers(0, 9))
    for t in types:
        b = int(rng.integers(1, 4))
        bls.append(b)
        disps.append(pos)
        # past the member's last byte (typemaps must not overlap: an
        # overlapping receive type is erroneous, its unpack order-dependent)
        pos += (b - 1) * t.extent + max(t.true_span, t.ub) + int(rng.integers(0, 13))
    return dd.type_struct(bls, disps, types)


def span_of(dt, count):
    """Bytes from the buffer base to the last typed byte of `count` elements."""
    return (count - 1) * dt.extent + dt.true_span
