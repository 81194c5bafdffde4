"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes front-end of oracle/liboracle.so, the CPU restatement of the
reference's op/base loops, coll/base allreduce orders and convertor byte
stream (see oracle.h for the file:line map).  Imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

ALG_TUNED, ALG_RECURSIVE_DOUBLING, ALG_RING, ALG_RING_SEGMENTED = 0, 3, 4, 5
ALG_BASIC_LINEAR, ALG_NONOVERLAPPING, ALG_REDSCAT_ALLGATHER = 1, 2, 6


class Block(ctypes.Structure):
    _fields_ = [("disp", ctypes.c_int64), ("len", ctypes.c_int64)]


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        c = ctypes
        L.orc_op_defined.restype = c.c_int
        L.orc_op_defined.argtypes = [c.c_int, c.c_int]
        L.orc_type_extent.restype = c.c_size_t
        L.orc_type_extent.argtypes = [c.c_int]
        L.orc_op_2buff.argtypes = [c.c_int, c.c_int, c.c_void_p, c.c_void_p, c.c_size_t]
        L.orc_op_3buff.argtypes = [c.c_int, c.c_int, c.c_void_p, c.c_void_p, c.c_void_p, c.c_size_t]
        L.orc_allreduce.argtypes = [c.c_int, c.c_int, c.POINTER(c.c_void_p),
                                    c.POINTER(c.c_void_p), c.c_size_t, c.c_int, c.c_int,
                                    c.c_size_t]
        L.orc_allreduce_forced.argtypes = [c.c_int, c.c_int, c.POINTER(c.c_void_p),
                                           c.POINTER(c.c_void_p), c.c_size_t, c.c_int, c.c_int,
                                           c.c_size_t, c.c_int]
        L.orc_reduce_scatter_block.argtypes = [c.c_int, c.POINTER(c.c_void_p),
                                               c.POINTER(c.c_void_p), c.c_size_t, c.c_int, c.c_int]
        L.orc_reduce_scatter_block_alg.argtypes = [c.c_int, c.POINTER(c.c_void_p),
                                                   c.POINTER(c.c_void_p), c.c_size_t, c.c_int,
                                                   c.c_int, c.c_int]
        L.orc_reduce_scatter_nonoverlapping.argtypes = [c.c_int, c.POINTER(c.c_void_p),
                                                        c.POINTER(c.c_void_p), c.POINTER(c.c_size_t),
                                                        c.c_int, c.c_int, c.c_int, c.c_int]
        L.orc_reduce_decision.argtypes = [c.c_int, c.c_size_t, c.c_size_t]
        L.orc_reduce.argtypes = [c.c_int, c.c_int, c.POINTER(c.c_void_p), c.c_void_p,
                                 c.c_size_t, c.c_int, c.c_int, c.c_int, c.c_int]
        L.orc_reduce_scatter_decision.argtypes = [c.c_int, c.c_size_t]
        L.orc_reduce_scatter.argtypes = [c.c_int, c.c_int, c.POINTER(c.c_void_p),
                                         c.POINTER(c.c_void_p), c.POINTER(c.c_size_t), c.c_int,
                                         c.c_int]
        L.orc_scan.argtypes = [c.c_int, c.c_int, c.POINTER(c.c_void_p), c.POINTER(c.c_void_p),
                               c.c_size_t, c.c_int, c.c_int]
        L.orc_allgather.argtypes =[c.c_int, c.POINTER(c.c_void_p), c.POINTER(c.c_void_p),
                                    c.c_size_t]
        L.orc_bcast.argtypes = [c.c_int, c.c_int, c.POINTER(c.c_void_p), c.c_size_t]
        L.orc_blockcount.argtypes = [c.c_size_t, c.c_int, c.POINTER(c.c_size_t),
                                     c.POINTER(c.c_size_t), c.POINTER(c.c_size_t)]
        for f in (L.orc_pack, L.orc_unpack):
            f.restype = c.c_size_t
            f.argtypes = [c.POINTER(Block), c.c_int, c.c_int64, c.c_size_t, c.c_void_p,
                          c.c_void_p, c.c_size_t, c.c_size_t]
        L.orc_time_op_3buff.restype = c.c_double
        L.orc_time_op_3buff.argtypes = [c.c_int, c.c_int, c.c_void_p, c.c_void_p, c.c_void_p,
                                        c.c_size_t, c.c_int]
        _lib = L
    return _lib


def _p(a: np.ndarray) -> int:
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def defined(op: int, type_code: int) -> bool:
    return bool(lib().orc_op_defined(op, type_code))


def op_2buff(op: int, type_code: int, inbuf: np.ndarray, inout: np.ndarray, count: int) -> None:
    rc = lib().orc_op_2buff(op, type_code, _p(inbuf), _p(inout), count)
    if rc != 0:
        raise ValueError(f"oracle: (op {op}, type {type_code}) undefined")


def op_3buff(op: int, type_code: int, in1: np.ndarray, in2: np.ndarray, out: np.ndarray,
             count: int) -> None:
    rc = lib().orc_op_3buff(op, type_code, _p(in1), _p(in2), _p(out), count)
    if rc != 0:
        raise ValueError(f"oracle: (op {op}, type {type_code}) undefined")


def allreduce(sbufs: list[np.ndarray], count: int, op: int, type_code: int,
              algorithm: int = ALG_TUNED, segsize: int = 0) -> tuple[list[np.ndarray], int]:
    n = len(sbufs)
    rbufs = [np.zeros_like(s) for s in sbufs]
    sp = (ctypes.c_void_p * n)(*[_p(s) for s in sbufs])
    rp = (ctypes.c_void_p * n)(*[_p(r) for r in rbufs])
    alg = lib().orc_allreduce(algorithm, n, sp, rp, count, op, type_code, segsize)
    if alg < 0:
        raise ValueError(f"oracle allreduce failed ({alg})")
    return rbufs, alg


def allreduce_forced(sbufs: list[np.ndarray], count: int, op: int, type_code: int, algorithm: int,
                     segsize: int = 0, root0_inplace: bool = False) -> tuple[list[np.ndarray], int]:
    """coll/tuned allreduce with coll_tuned_allreduce_algorithm forced to
    `algorithm` (1..6, coll_tuned_allreduce_decision.c:37-47 numbering)."""
    n = len(sbufs)
    rbufs = [np.zeros_like(s) for s in sbufs]
    sp = (ctypes.c_void_p * n)(*[_p(s) for s in sbufs])
    rp = (ctypes.c_void_p * n)(*[_p(r) for r in rbufs])
    alg = lib().orc_allreduce_forced(algorithm, n, sp, rp, count, op, type_code, segsize,
                                     1 if root0_inplace else 0)
    if alg < 0:
        raise ValueError(f"oracle allreduce (forced {algorithm}) failed ({alg})")
    return rbufs, alg


def reduce_scatter_block(sbufs: list[np.ndarray], rcount: int, op: int,
                         type_code: int, red_alg: int = 0) -> list[np.ndarray]:
    """basic_linear rsb; red_alg: coll/tuned's forced reduce algorithm
    (RED_*, 0 = its fixed decision) for the reduce it calls."""
    n = len(sbufs)
    ext = lib().orc_type_extent(type_code)
    rbufs = [np.zeros(rcount * ext, dtype=np.uint8) for _ in range(n)]
    sp = (ctypes.c_void_p * n)(*[_p(s) for s in sbufs])
    rp = (ctypes.c_void_p * n)(*[_p(r) for r in rbufs])
    if lib().orc_reduce_scatter_block_alg(n, sp, rp, rcount, op, type_code, red_alg) < 0:
        raise ValueError("oracle rsb failed")
    return rbufs


RED_TUNED, RED_LINEAR, RED_PIPELINE, RED_BINARY, RED_BINOMIAL = 0, 1, 3, 4, 5


def reduce_decision(n: int, msg: int, count: int) -> int:
    return lib().orc_reduce_decision(n, msg, count)


def reduce(sbufs: list[np.ndarray], count: int, op: int, type_code: int, root: int,
           root_inplace: bool = False, algorithm: int = RED_TUNED) -> tuple[np.ndarray, int]:
    """coll/tuned reduce of sbufs to `root`: (root's result, algorithm run)."""
    n = len(sbufs)
    out = np.zeros_like(sbufs[root])
    sp = (ctypes.c_void_p * n)(*[_p(s) for s in sbufs])
    alg = lib().orc_reduce(algorithm, n, sp, _p(out), count, op, type_code, root,
                           1 if root_inplace else 0)
    if alg < 0:
        raise ValueError(f"oracle reduce failed ({alg})")
    return out, alg


RS_TUNED, RS_HALVING, RS_RING = 0, 1, 2
RS_NONOVERLAPPING = 3  # reduce to rank 0 (coll/tuned's, red_alg) + scatterv


def reduce_scatter_decision(n: int, total_bytes: int) -> int:
    return lib().orc_reduce_scatter_decision(n, total_bytes)


def reduce_scatter(sbufs: list[np.ndarray], rcounts: list[int], op: int, type_code: int,
                   algorithm: int = RS_TUNED, red_alg: int = 0,
                   inplace: bool = False) -> tuple[list[np.ndarray], int]:
    """coll/tuned reduce_scatter: (per-rank results, algorithm run)."""
    n = len(sbufs)
    rbufs = [np.zeros(max(1, rc), dtype=sbufs[0].dtype)[:rc] for rc in rcounts]
    rbufs = [np.ascontiguousarray(r) if r.size else np.zeros(1, dtype=sbufs[0].dtype)
             for r in rbufs]
    sp = (ctypes.c_void_p * n)(*[_p(s) for s in sbufs])
    rp = (ctypes.c_void_p * n)(*[_p(r) for r in rbufs])
    rc = (ctypes.c_size_t * n)(*rcounts)
    if algorithm == RS_NONOVERLAPPING:
        alg = lib().orc_reduce_scatter_nonoverlapping(n, sp, rp, rc, op, type_code, red_alg,
                                                      1 if inplace else 0)
        alg = RS_NONOVERLAPPING if alg >= 0 else alg
    else:
        alg = lib().orc_reduce_scatter(algorithm, n, sp, rp, rc, op, type_code)
    if alg < 0:
        raise ValueError(f"oracle reduce_scatter failed ({alg})")
    return [r[:c] for r, c in zip(rbufs, rcounts)], alg


def scan(sbufs: list[np.ndarray], count: int, op: int, type_code: int,
         exclusive: bool = False) -> list[np.ndarray]:
    """Linear scan / exscan; exscan's rank-0 result stays all-zero bytes."""
    n = len(sbufs)
    rbufs = [np.zeros_like(s) for s in sbufs]
    sp = (ctypes.c_void_p * n)(*[_p(s) for s in sbufs])
    rp = (ctypes.c_void_p * n)(*[_p(r) for r in rbufs])
    if lib().orc_scan(1 if exclusive else 0, n, sp, rp, count, op, type_code) != 0:
        raise ValueError("oracle scan failed")
    return rbufs


def blockcount(count: int, nblocks: int) -> tuple[int, int, int]:
    s, e, l_ = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
    lib().orc_blockcount(count, nblocks, ctypes.byref(s), ctypes.byref(e), ctypes.byref(l_))
    return s.value, e.value, l_.value


def _blocks(blocks):
    arr = (Block * len(blocks))(*[Block(d, n) for d, n in blocks])
    return arr


def pack(blocks, extent: int, count: int, src: np.ndarray, offset: int, nbytes: int) -> np.ndarray:
    dst = np.zeros(nbytes, dtype=np.uint8)
    done = lib().orc_pack(_blocks(blocks), len(blocks), extent, count, _p(src), _p(dst),
                          offset, nbytes)
    return dst[:done]


def unpack(blocks, extent: int, count: int, packed: np.ndarray, dst: np.ndarray,
           offset: int) -> int:
    return lib().orc_unpack(_blocks(blocks), len(blocks), extent, count, _p(packed), _p(dst),
                            offset, packed.nbytes)


def time_op_3buff(op: int, type_code: int, in1, in2, out, count: int, iters: int) -> float:
    return lib().orc_time_op_3buff(op, type_code, _p(in1), _p(in2), _p(out), count, iters)
