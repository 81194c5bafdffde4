"""Derived datatypes and the convertor for device buffers.

Mirrors the reference's constructors and convertor contract for this path:

* ``type_vector`` / ``type_indexed`` / ``type_struct`` / ``type_contiguous``
  (ompi/datatype/ompi_datatype_create_vector.c:31, _indexed.c:34,
  _struct.c:31, _contiguous.c) build the flattened typemap (a list of
  contiguous byte runs {disp, len} in typemap order plus lb/ub/extent).
* ``Convertor`` is opal_convertor_t's pack/unpack protocol
  (opal/datatype/opal_convertor.h:88-146, opal_convertor.c:218-325):
  ``prepare_for_send`` / ``prepare_for_recv`` then repeated ``pack`` /
  ``unpack`` calls each moving at most ``max_data`` bytes and advancing
  ``bConverted``; the return value is 1 when the whole stream is done, 0
  when data remains (convertor_advance_fct_t, opal_convertor.h:64-67).
  Device buffers only: every byte moves in one libompi_amd kernel launch
  per call (the reference issues one cuMemcpy per run,
  opal_datatype_cuda.c:121-145).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

from . import _lib

# predefined element types used by the builders: (size, alignment)
PREDEFINED = {
    "MPI_CHAR": 1, "MPI_BYTE": 1, "MPI_SHORT": 2, "MPI_INT": 4, "MPI_FLOAT": 4,
    "MPI_LONG": 8, "MPI_DOUBLE": 8, "MPI_INT8_T": 1, "MPI_INT16_T": 2, "MPI_INT32_T": 4,
    "MPI_INT64_T": 8,
}


@dataclass
class Datatype:
    """A committed datatype as its typemap: runs of (disp, len) bytes."""
    name: str
    runs: list = field(default_factory=list)  # [(disp, len)] in typemap order
    lb: int = 0
    ub: int = 0
    align: int = 1
    _handle: object = None

    @property
    def size(self) -> int:
        return sum(n for _, n in self.runs)

    @property
    def extent(self) -> int:
        return self.ub - self.lb

    def commit(self) -> "Datatype":
        """ompi_datatype_commit: build the device program (opt_desc)."""
        if self._handle is None:
            lib = _lib.load()
            blocks = (_lib.DdtBlock * len(self.runs))(*[_lib.DdtBlock(d, n) for d, n in self.runs])
            h = ctypes.c_void_p()
            _lib.check(lib.ompi_amd_ddt_create(blocks, len(self.runs), self.extent,
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
    return Datatype(name, [(0, size)], 0, size, size)


def _merge(runs):
    out = []
    for d, n in runs:
        if out and out[-1][0] + out[-1][1] == d:
            out[-1] = (out[-1][0], out[-1][1] + n)
        else:
            out.append((d, n))
    return out


def _replicate(old: Datatype, disp: int, count: int):
    """`count` consecutive copies of old starting at byte `disp`."""
    runs = []
    for i in range(count):
        base = disp + i * old.extent
        runs.extend((base + d, n) for d, n in old.runs)
    return runs


def type_contiguous(count: int, old: Datatype) -> Datatype:
    runs = _merge(_replicate(old, 0, count))
    return Datatype(f"contiguous({count},{old.name})", runs, old.lb,
                    old.lb + count * old.extent, old.align)


def type_vector(count: int, blocklength: int, stride: int, old: Datatype) -> Datatype:
    """MPI_Type_vector (stride in elements of old)."""
    runs = []
    for i in range(count):
        runs.extend(_replicate(old, i * stride * old.extent, blocklength))
    runs = _merge(runs)
    span_lo = min(0, (count - 1) * stride * old.extent) + old.lb
    last = (count - 1) * stride * old.extent
    ub = max(last, 0) + blocklength * old.extent + old.lb
    return Datatype(f"vector({count},{blocklength},{stride},{old.name})", runs, span_lo,
                    ub, old.align)


def type_indexed(blocklengths, displacements, old: Datatype) -> Datatype:
    """MPI_Type_indexed (displacements in elements of old)."""
    runs = []
    lo, hi = None, None
    for bl, dp in zip(blocklengths, displacements):
        if bl == 0:
            continue
        runs.extend(_replicate(old, dp * old.extent, bl))
        b0, b1 = dp * old.extent + old.lb, (dp + bl) * old.extent + old.lb
        lo = b0 if lo is None else min(lo, b0)
        hi = b1 if hi is None else max(hi, b1)
    return Datatype(f"indexed({len(runs)},{old.name})", _merge(runs), lo or 0, hi or 0,
                    old.align)


def type_struct(blocklengths, displacements, types) -> Datatype:
    """MPI_Type_struct (byte displacements); ub padded to the largest
    member alignment, as the standard's epsilon rule prescribes."""
    runs = []
    lo, hi, align = None, None, 1
    for bl, dp, t in zip(blocklengths, displacements, types):
        if bl == 0:
            continue
        runs.extend(_replicate(t, dp, bl))
        b0, b1 = dp + t.lb, dp + t.lb + bl * t.extent
        lo = b0 if lo is None else min(lo, b0)
        hi = b1 if hi is None else max(hi, b1)
        align = max(align, t.align)
    hi = hi or 0
    if hi % align:
        hi += align - hi % align
    return Datatype("struct", _merge(runs), lo or 0, hi, align)


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
        lib = _lib.load()
        want = min(int(max_data), self.local_size - self.bConverted)
        done = ctypes.c_size_t(0)
        sp = None if self.stream is None else (
            self.stream if isinstance(self.stream, int) else self.stream.cuda_stream)
        rc = fn(self.datatype._handle, self.count, src, dst, self.bConverted,
                want, ctypes.byref(done), sp)
        _lib.check(rc, "convertor")
        self.bConverted += done.value
        return (1 if self.bConverted == self.local_size else 0), done.value

    def pack(self, iov, max_data: int):
        """opal_convertor_pack: returns (completed, bytes written into iov)."""
        return self._run(_lib.load().ompi_amd_ddt_pack, self.base, _addr(iov), max_data)

    def unpack(self, iov, max_data: int):
        """opal_convertor_unpack: returns (completed, bytes consumed from iov)."""
        return self._run(_lib.load().ompi_amd_ddt_unpack, _addr(iov), self.base, max_data)
