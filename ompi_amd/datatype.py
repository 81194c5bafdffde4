"""Derived datatypes and the convertor for device buffers.

Mirrors the reference's constructors and convertor contract for this path:

* ``type_vector`` / ``type_indexed`` / ``type_struct`` / ``type_contiguous``
  (ompi/datatype/ompi_datatype_create_vector.c:31, _indexed.c:34,
  _struct.c:31, _contiguous.c) build the optimized description directly: a
  list of ``{count, blocklen, stride, disp}`` byte elements in typemap order
  — the shape of opal's ``ddt_elem_desc`` after opal_datatype_optimize.c (a
  vector of a predefined type is ONE element) — plus lb / ub / extent.
* ``Convertor`` is opal_convertor_t's pack/unpack protocol
  (opal/datatype/opal_convertor.h:88-146, opal_convertor.c:218-325):
  ``prepare_for_send`` / ``prepare_for_recv`` then repeated ``pack`` /
  ``unpack`` calls each moving at most ``max_data`` bytes and advancing
  ``bConverted``; the return value is 1 when the whole stream is done, 0
  when data remains (convertor_advance_fct_t, opal_convertor.h:64-67).
  Device buffers only: every call is one libompi_amd kernel launch (the
  reference issues one cuMemcpy per run, opal_datatype_cuda.c:121-145).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

from . import _lib

# predefined element types used by the builders: size (= alignment)
PREDEFINED = {
    "MPI_CHAR": 1, "MPI_BYTE": 1, "MPI_SHORT": 2, "MPI_INT": 4, "MPI_FLOAT": 4,
    "MPI_LONG": 8, "MPI_DOUBLE": 8, "MPI_INT8_T": 1, "MPI_INT16_T": 2, "MPI_INT32_T": 4,
    "MPI_INT64_T": 8,
}


def _normalize(elems):
    """Drop empty elements, give count-1 elements stride = blocklen, and
    merge an element into its predecessor when the runs touch."""
    out = []
    for c, bl, st, d in elems:
        if c <= 0 or bl <= 0:
            continue
        if c == 1:
            st = bl
        elif st == bl:  # contiguous repetitions: one run
            c, bl, st = 1, c * bl, c * bl
        if out:
            pc, pbl, pst, pd = out[-1]
            if pc == 1 and c == 1 and pd + pbl == d:
                out[-1] = (1, pbl + bl, pbl + bl, pd)
                continue
            if pc > 1 and c == 1 and bl == pbl and d == pd + pc * pst:
                out[-1] = (pc + 1, pbl, pst, pd)
                continue
            if pc == 1 and c == 1 and bl == pbl:
                out[-1] = (2, bl, d - pd, pd)
                continue
        out.append((c, bl, st, d))
    return out


@dataclass
class Datatype:
    """A committed datatype: elements (count, blocklen, stride, disp) in
    typemap order, byte units, plus lb/ub."""
    name: str
    elems: list = field(default_factory=list)
    lb: int = 0
    ub: int = 0
    align: int = 1
    _handle: object = None

    def __post_init__(self):
        self.elems = _normalize(self.elems)
        self._size = sum(c * bl for c, bl, _, _ in self.elems)

    @property
    def size(self) -> int:
        return self._size

    @property
    def extent(self) -> int:
        return self.ub - self.lb

    @property
    def runs(self) -> list:
        """Flattened typemap (disp, len) — small types / tests only."""
        return [(d + i * st, bl) for c, bl, st, d in self.elems for i in range(c)]

    @property
    def true_span(self) -> int:
        """Bytes from the element base to the end of its last byte."""
        return max(d + (c - 1) * st + bl for c, bl, st, d in self.elems)

    def commit(self) -> "Datatype":
        """ompi_datatype_commit: build the device program."""
        if self._handle is None:
            lib = _lib.load()
            arr = (_lib.DdtElem * len(self.elems))(
                *[_lib.DdtElem(c, bl, st, d) for c, bl, st, d in self.elems])
            h = ctypes.c_void_p()
            _lib.check(lib.ompi_amd_ddt_create_elems(arr, len(self.elems), self.extent,
                                                     ctypes.byref(h)), f"commit {self.name}")
            self._handle = h
        return self

    @property
    def nelems(self) -> int:
        self.commit()
        return _lib.load().ompi_amd_ddt_nelems(self._handle)

    def free(self) -> None:
        if self._handle is not None:
            _lib.load().ompi_amd_ddt_destroy(self._handle)
            self._handle = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def predefined(name: str) -> Datatype:
    size = PREDEFINED[name]
    return Datatype(name, [(1, size, size, 0)], 0, size, size)


def from_runs(name: str, runs, extent: int, lb: int = 0) -> Datatype:
    """A datatype given by its flattened typemap."""
    return Datatype(name, [(1, n, n, d) for d, n in runs], lb, lb + extent)


def _shift(old: Datatype, disp: int):
    return [(c, bl, st, d + disp) for c, bl, st, d in old.elems]


def _repeat(old: Datatype, disp: int, count: int, step: int):
    """`count` copies of old, `step` bytes apart, starting at `disp`."""
    if count <= 0:
        return []
    if len(old.elems) == 1:
        c, bl, st, d = old.elems[0]
        if c == 1:  # a single run per copy: one strided element
            return [(count, bl, step, d + disp)]
    out = []
    for i in range(count):
        out.extend(_shift(old, disp + i * step))
    return out


def type_contiguous(count: int, old: Datatype) -> Datatype:
    return Datatype(f"contiguous({count},{old.name})", _repeat(old, 0, count, old.extent),
                    old.lb, old.lb + count * old.extent, old.align)


def type_vector(count: int, blocklength: int, stride: int, old: Datatype) -> Datatype:
    """MPI_Type_vector (stride in elements of old)."""
    block = type_contiguous(blocklength, old)
    elems = _repeat(block, 0, count, stride * old.extent)
    lo = min(0, (count - 1) * stride * old.extent) + old.lb
    hi = max(0, (count - 1) * stride * old.extent) + blocklength * old.extent + old.lb
    return Datatype(f"vector({count},{blocklength},{stride},{old.name})", elems, lo, hi,
                    old.align)


def type_indexed(blocklengths, displacements, old: Datatype) -> Datatype:
    """MPI_Type_indexed (displacements in elements of old)."""
    elems = []
    lo, hi = None, None
    for bl, dp in zip(blocklengths, displacements):
        if bl == 0:
            continue
        elems.extend(_repeat(old, dp * old.extent, bl, old.extent))
        b0, b1 = dp * old.extent + old.lb, (dp + bl) * old.extent + old.lb
        lo = b0 if lo is None else min(lo, b0)
        hi = b1 if hi is None else max(hi, b1)
    return Datatype(f"indexed({len(blocklengths)},{old.name})", elems, lo or 0, hi or 0,
                    old.align)


def type_struct(blocklengths, displacements, types) -> Datatype:
    """MPI_Type_struct (byte displacements); ub padded to the largest
    member alignment (the standard's epsilon rule)."""
    elems = []
    lo, hi, align = None, None, 1
    for bl, dp, t in zip(blocklengths, displacements, types):
        if bl == 0:
            continue
        elems.extend(_repeat(t, dp, bl, t.extent))
        b0, b1 = dp + t.lb, dp + t.lb + bl * t.extent
        lo = b0 if lo is None else min(lo, b0)
        hi = b1 if hi is None else max(hi, b1)
        align = max(align, t.align)
    hi = hi or 0
    if hi % align:
        hi += align - hi % align
    return Datatype("struct", elems, lo or 0, hi, align)


def _addr(buf) -> int:
    if isinstance(buf, int):
        return buf
    if hasattr(buf, "data_ptr"):
        if not buf.is_cuda:
            raise _lib.OmpiAmdError(_lib.ERR_NOT_DEVICE, "convertor on a host tensor")
        return buf.data_ptr()
    raise TypeError(type(buf))


class Convertor:
    """opal_convertor_t restricted to homogeneous device-buffer conversions."""

    def __init__(self):
        self.datatype = None
        self.count = 0
        self.base = 0
        self.bConverted = 0
        self.local_size = 0
        self.stream = None

    def _prepare(self, datatype: Datatype, count: int, buf, stream):
        datatype.commit()
        self.datatype, self.count, self.base = datatype, count, _addr(buf)
        self.bConverted = 0
        self.local_size = datatype.size * count
        self.stream = stream
        return 0

    def prepare_for_send(self, datatype: Datatype, count: int, buf, stream=None) -> int:
        """opal_convertor_prepare_for_send (opal_convertor.c:608)."""
        return self._prepare(datatype, count, buf, stream)

    def prepare_for_recv(self, datatype: Datatype, count: int, buf, stream=None) -> int:
        """opal_convertor_prepare_for_recv (opal_convertor.c:565)."""
        return self._prepare(datatype, count, buf, stream)

    def set_position(self, position: int) -> int:
        """opal_convertor_set_position: resume at any stream byte."""
        self.bConverted = max(0, min(int(position), self.local_size))
        return 0

    def _run(self, fn, src, dst, max_data):
        want = min(int(max_data), self.local_size - self.bConverted)
        done = ctypes.c_size_t(0)
        sp = None if self.stream is None else (
            self.stream if isinstance(self.stream, int) else self.stream.cuda_stream)
        rc = fn(self.datatype._handle, self.count, src, dst, self.bConverted,
                want, ctypes.byref(done), sp)
        _lib.check(rc, "convertor")
        self.bConverted += done.value
        return (1 if self.bConverted == self.local_size else 0), done.value

    def _run_iov(self, fn, iovs):
        """fAdvance over an iovec array (convertor_advance_fct_t,
        opal_convertor.h:64-67): iovs = [(device address, capacity)...].
        Returns (completed, [bytes used per entry], entries used, max_data);
        one kernel launch for all entries."""
        n = len(iovs)
        arr = (_lib.Iovec * max(1, n))(*[_lib.Iovec(_addr(b), int(l)) for b, l in iovs])
        out = ctypes.c_uint32(n)
        max_data = ctypes.c_size_t(0)
        sp = None if self.stream is None else (
            self.stream if isinstance(self.stream, int) else self.stream.cuda_stream)
        rc = fn(self.datatype._handle, self.count, self.base, self.bConverted, arr,
                ctypes.byref(out), ctypes.byref(max_data), sp)
        if rc < 0:
            _lib.check(rc, "convertor (iovec)")
        self.bConverted += max_data.value
        return rc, [arr[i].iov_len for i in range(out.value)], out.value, max_data.value

    def pack_iov(self, iovs):
        """opal_convertor_pack with an iovec array (packed bytes into each entry)."""
        return self._run_iov(_lib.load().ompi_amd_ddt_pack_iov, iovs)

    def unpack_iov(self, iovs):
        """opal_convertor_unpack with an iovec array (packed bytes from each entry)."""
        return self._run_iov(_lib.load().ompi_amd_ddt_unpack_iov, iovs)

    def pack(self, iov, max_data: int):
        """opal_convertor_pack: returns (completed, bytes written into iov)."""
        return self._run(_lib.load().ompi_amd_ddt_pack, self.base, _addr(iov), max_data)

    def unpack(self, iov, max_data: int):
        """opal_convertor_unpack: returns (completed, bytes consumed from iov)."""
        return self._run(_lib.load().ompi_amd_ddt_unpack, _addr(iov), self.base, max_data)
