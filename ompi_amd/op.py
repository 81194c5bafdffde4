"""MPI_Op surface of the MI355X path: predefined ops and datatypes, and
``reduce_local`` (MPI_Reduce_local, ompi/mpi/c/reduce_local.c:47 ->
coll_base_reduce.c:42 -> ompi_op_reduce, ompi/op/op.h:547).

Buffers are device tensors (or raw device addresses).  Every call goes
through libompi_amd.so; host buffers are rejected, not reduced on the CPU.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib


@dataclass(frozen=True)
class Op:
    """A predefined MPI_Op; `index` is OMPI_OP_BASE_FORTRAN_* (op.h:203-237)."""
    name: str
    index: int


@dataclass(frozen=True)
class Datatype:
    """A predefined datatype; `code` is OMPI_OP_BASE_TYPE_* (op.h:104-190).

    `size` is the MPI type size (bytes of data), `extent` the element stride
    (MPI_DOUBLE_INT: size 12, extent 16 — ompi_datatype_module.c:404-430).
    """
    name: str
    code: int
    size: int
    extent: int
    np_dtype: object  # numpy dtype of one element (structured for pairs)


MPI_MAX = Op("MPI_MAX", 1)
MPI_MIN = Op("MPI_MIN", 2)
MPI_SUM = Op("MPI_SUM", 3)
MPI_PROD = Op("MPI_PROD", 4)
MPI_LAND = Op("MPI_LAND", 5)
MPI_BAND = Op("MPI_BAND", 6)
MPI_LOR = Op("MPI_LOR", 7)
MPI_BOR = Op("MPI_BOR", 8)
MPI_LXOR = Op("MPI_LXOR", 9)
MPI_BXOR = Op("MPI_BXOR", 10)
MPI_MAXLOC = Op("MPI_MAXLOC", 11)
MPI_MINLOC = Op("MPI_MINLOC", 12)
# one-sided only (MPI_Accumulate / MPI_Get_accumulate, ompi/mca/op/op.h:232-235)
MPI_REPLACE = Op("MPI_REPLACE", 13)
MPI_NO_OP = Op("MPI_NO_OP", 14)
OPS = [MPI_MAX, MPI_MIN, MPI_SUM, MPI_PROD, MPI_LAND, MPI_BAND, MPI_LOR,
       MPI_BOR, MPI_LXOR, MPI_BXOR, MPI_MAXLOC, MPI_MINLOC]


def _pair(vt, pad):
    fields = [("v", vt), ("k", np.int32)]
    names = ["v", "k"]
    formats = [np.dtype(vt), np.dtype(np.int32)]
    vsz = np.dtype(vt).itemsize
    offsets = [0, vsz if vsz >= 4 else 4]
    itemsize = offsets[1] + 4 + pad
    del fields
    return np.dtype({"names": names, "formats": formats, "offsets": offsets,
                     "itemsize": itemsize})


MPI_INT8_T = Datatype("MPI_INT8_T", 0, 1, 1, np.dtype(np.int8))
MPI_UINT8_T = Datatype("MPI_UINT8_T", 1, 1, 1, np.dtype(np.uint8))
MPI_INT16_T = Datatype("MPI_INT16_T", 2, 2, 2, np.dtype(np.int16))
MPI_UINT16_T = Datatype("MPI_UINT16_T", 3, 2, 2, np.dtype(np.uint16))
MPI_INT32_T = Datatype("MPI_INT32_T", 4, 4, 4, np.dtype(np.int32))
MPI_UINT32_T = Datatype("MPI_UINT32_T", 5, 4, 4, np.dtype(np.uint32))
MPI_INT64_T = Datatype("MPI_INT64_T", 6, 8, 8, np.dtype(np.int64))
MPI_UINT64_T = Datatype("MPI_UINT64_T", 7, 8, 8, np.dtype(np.uint64))
# MPIX_C_FLOAT16 (opal_short_float_t = _Float16) and its complex,
# opal_short_float_t[2] (no numpy complex32: a (re, im) record of halves)
MPIX_C_FLOAT16 = Datatype("MPIX_C_FLOAT16", 14, 2, 2, np.dtype(np.float16))
MPIX_C_FLOAT16_COMPLEX = Datatype("MPIX_C_FLOAT16_COMPLEX", 26, 4, 4,
                                  np.dtype([("re", np.float16), ("im", np.float16)]))
MPI_FLOAT = Datatype("MPI_FLOAT", 15, 4, 4, np.dtype(np.float32))
MPI_DOUBLE = Datatype("MPI_DOUBLE", 16, 8, 8, np.dtype(np.float64))
MPI_C_BOOL = Datatype("MPI_C_BOOL", 25, 1, 1, np.dtype(np.uint8))
MPI_C_FLOAT_COMPLEX = Datatype("MPI_C_FLOAT_COMPLEX", 27, 8, 8, np.dtype(np.complex64))
MPI_C_DOUBLE_COMPLEX = Datatype("MPI_C_DOUBLE_COMPLEX", 28, 16, 16, np.dtype(np.complex128))
MPI_BYTE = Datatype("MPI_BYTE", 30, 1, 1, np.dtype(np.uint8))
MPI_FLOAT_INT = Datatype("MPI_FLOAT_INT", 34, 8, 8, _pair(np.float32, 0))
MPI_DOUBLE_INT = Datatype("MPI_DOUBLE_INT", 35, 12, 16, _pair(np.float64, 4))
MPI_LONG_INT = Datatype("MPI_LONG_INT", 36, 12, 16, _pair(np.int64, 4))
MPI_2INT = Datatype("MPI_2INT", 37, 8, 8, _pair(np.int32, 0))
MPI_SHORT_INT = Datatype("MPI_SHORT_INT", 38, 6, 8, _pair(np.int16, 0))
# MPI_INT aliases INT32_T by size (ompi_datatype_internal.h:166-175)
MPI_INT = MPI_INT32_T
MPI_LONG = MPI_INT64_T

DATATYPES = [MPI_INT8_T, MPI_UINT8_T, MPI_INT16_T, MPI_UINT16_T, MPI_INT32_T,
             MPI_UINT32_T, MPI_INT64_T, MPI_UINT64_T, MPIX_C_FLOAT16, MPI_FLOAT, MPI_DOUBLE,
             MPI_C_BOOL, MPIX_C_FLOAT16_COMPLEX, MPI_C_FLOAT_COMPLEX, MPI_C_DOUBLE_COMPLEX, MPI_BYTE, MPI_FLOAT_INT, MPI_DOUBLE_INT, MPI_LONG_INT,
             MPI_2INT, MPI_SHORT_INT]
BY_CODE = {d.code: d for d in DATATYPES}


def _ptr(buf) -> int:
    if isinstance(buf, int):
        return buf
    if hasattr(buf, "data_ptr"):
        if not buf.is_cuda:
            raise _lib.OmpiAmdError(_lib.ERR_NOT_DEVICE, "host tensor passed to a device op")
        return buf.data_ptr()
    raise TypeError(f"unsupported buffer type {type(buf)!r}")


def _stream_ptr(stream) -> int | None:
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream  # torch.cuda.Stream


def supported(op: Op, dtype: Datatype) -> bool:
    return bool(_lib.load().ompi_amd_op_supported(op.index, dtype.code))


def reduce_local_async(inbuf, inoutbuf, count: int, datatype: Datatype, op: Op,
                       stream=None) -> None:
    """inout = inout (op) in on `stream` (2-buffer handler semantics)."""
    lib = _lib.load()
    rc = lib.ompi_amd_op_reduce(op.index, datatype.code, _ptr(inbuf), _ptr(inoutbuf),
                                count, _stream_ptr(stream))
    _lib.check(rc, f"reduce_local({op.name}, {datatype.name})")


def reduce_local_3buff_async(in1, in2, out, count: int, datatype: Datatype, op: Op,
                             stream=None) -> None:
    """out = in1 (op) in2 on `stream` (3-buffer handler semantics)."""
    lib = _lib.load()
    rc = lib.ompi_amd_op_reduce_3buff(op.index, datatype.code, _ptr(in1), _ptr(in2),
                                      _ptr(out), count, _stream_ptr(stream))
    _lib.check(rc, f"reduce_local_3buff({op.name}, {datatype.name})")


def reduce_local(inbuf, inoutbuf, count: int, datatype: Datatype, op: Op) -> None:
    """MPI_Reduce_local: blocking, through the op framework's handler slot
    exactly as ompi_op_reduce calls it (fns[type](in, inout, &count, &dtype,
    module), ompi/op/op.h:585-587)."""
    fn = handler(op, datatype)
    c = ctypes.c_int(count)
    fn(_ptr(inbuf), _ptr(inoutbuf), ctypes.byref(c), None, None)


def reduce_local_3buff(in1, in2, out, count: int, datatype: Datatype, op: Op) -> None:
    """ompi_3buff_op_reduce (ompi/op/op.h:642-661), blocking."""
    fn = handler3(op, datatype)
    c = ctypes.c_int(count)
    fn(_ptr(in1), _ptr(in2), _ptr(out), ctypes.byref(c), None, None)


def handler(op: Op, datatype: Datatype):
    """The 2-buffer handler the op component installs for (op, type)."""
    lib = _lib.load()
    row = lib.ompi_amd_op_handler_row(op.index)
    addr = row[datatype.code] if row else None
    if not addr:
        raise _lib.OmpiAmdError(_lib.ERR_UNSUPPORTED, f"no handler for {op.name}/{datatype.name}")
    return _lib.HANDLER_FN(addr)


def handler3(op: Op, datatype: Datatype):
    lib = _lib.load()
    row = lib.ompi_amd_op_3buff_handler_row(op.index)
    addr = row[datatype.code] if row else None
    if not addr:
        raise _lib.OmpiAmdError(_lib.ERR_UNSUPPORTED, f"no handler for {op.name}/{datatype.name}")
    return _lib.HANDLER3_FN(addr)
