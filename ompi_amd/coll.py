"""Device-buffer collectives of the MI355X path (the coll module surface).

Mirrors the coll framework's entry points this path provides
(ompi/mca/coll/coll.h:200-250):

    coll_allreduce(sbuf, rbuf, count, dtype, op, comm, module)
    coll_iallreduce(sbuf, rbuf, count, dtype, op, comm, request, module)
    coll_allreduce_init(sbuf, rbuf, count, dtype, op, comm, info, request, module)
    coll_reduce(sbuf, rbuf, count, dtype, op, root, comm, module)
    coll_reduce_scatter(sbuf, rbuf, rcounts, dtype, op, comm, module)
    coll_reduce_scatter_block(sbuf, rbuf, rcount, dtype, op, comm, module)
    coll_scan / coll_exscan(sbuf, rbuf, count, dtype, op, comm, module)
    coll_allgather(sbuf, scount, sdtype, rbuf, rcount, rdtype, comm, module)
    coll_bcast(buf, count, dtype, root, comm, module)

with the communicator object holding the module state (IPC mappings, flags,
epoch).  One process per GPU on one node.  All calls are stream-ordered;
``blocking=True`` (the MPI semantics the MCA glue uses) synchronises the
stream and raises on a device-side error.  Every byte moves through
libompi_amd.so; there is no host fallback for device buffers.
"""
from __future__ import annotations

import ctypes
import os
import secrets

from . import _lib
from .op import Datatype, Op

IN_PLACE = object()  # MPI_IN_PLACE
_IN_PLACE_PTR = 1


def _ptr(buf) -> int:
    if buf is IN_PLACE:
        return _IN_PLACE_PTR
    if isinstance(buf, int):
        return buf
    if hasattr(buf, "data_ptr"):
        if not buf.is_cuda:
            raise _lib.OmpiAmdError(_lib.ERR_NOT_DEVICE, "host tensor passed to a device collective")
        return buf.data_ptr()
    raise TypeError(type(buf))


def _stream(stream):
    """The stream a call is ordered on: None means torch's current stream, so
    a collective runs after the torch work that produced its buffers (the
    library's own NULL default is the per-thread stream, which is not
    ordered after torch's stream)."""
    if stream is None:
        try:
            import torch
            if torch.cuda.is_available():
                # torch's default stream is the legacy null stream (handle 0),
                # which the C ABI spells hipStreamLegacy (1): NULL there means
                # the per-thread stream
                return torch.cuda.current_stream().cuda_stream or 1
        except ImportError:
            pass
        return None
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


class Communicator:
    """A node-local communicator over `size` ranks, one GPU each."""

    def __init__(self, name: str, rank: int, size: int, device: int = 0):
        self._lib = _lib.load()
        h = ctypes.c_void_p()
        _lib.check(self._lib.ompi_amd_comm_create(name.encode(), rank, size, device,
                                                  ctypes.byref(h)), "comm_create")
        self._h = h
        self.rank, self.size, self.device = rank, size, device

    @classmethod
    def from_torch_distributed(cls, group=None, device: int | None = None) -> "Communicator":
        """Bootstrap from an initialised torch.distributed group (any
        backend): rank 0 draws a node-unique segment name and broadcasts it."""
        import torch.distributed as dist
        rank, size = dist.get_rank(group), dist.get_world_size(group)
        token = [f"{os.getpid()}_{secrets.token_hex(6)}" if rank == 0 else None]
        dist.broadcast_object_list(token, src=0, group=group)
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", rank))
        return cls(token[0], rank, size, device)

    # -- parameters / state ------------------------------------------------
    def set_param(self, key: str, value: int) -> None:
        _lib.check(self._lib.ompi_amd_comm_set_param(self._h, key.encode(), int(value)),
                   f"set_param({key})")

    def get_param(self, key: str) -> int:
        v = ctypes.c_int64()
        _lib.check(self._lib.ompi_amd_comm_get_param(self._h, key.encode(), ctypes.byref(v)),
                   f"get_param({key})")
        return v.value

    def error(self) -> int:
        return self._lib.ompi_amd_comm_error(self._h)

    def phase_ms(self, phase: int) -> tuple[float, int]:
        """(total kernel ms, calls) of a profiled allreduce phase (0 =
        reduce, 1 = gather) since the last read."""
        tot, n = ctypes.c_double(), ctypes.c_int()
        _lib.check(self._lib.ompi_amd_comm_phase_ms(self._h, phase, ctypes.byref(tot),
                                                    ctypes.byref(n)), "phase_ms")
        return tot.value, n.value

    def free(self) -> None:
        if getattr(self, "_h", None):
            _lib.check(self._lib.ompi_amd_comm_destroy(self._h), "comm_destroy")
            self._h = None

    def sync(self, stream=None) -> None:
        """ompi_amd_comm_sync: this communicator's calls on `stream` done
        (what coll/rocm's blocking collectives wait with); while it waits,
        the other communicators' ready nonblocking calls are launched."""
        _lib.check(self._lib.ompi_amd_comm_sync(self._h, _stream(stream)), "comm_sync")

    def _finish(self, rc: int, what: str, blocking: bool, stream) -> None:
        _lib.check(rc, what)
        if blocking:
            import torch
            if stream is None:
                torch.cuda.synchronize(self.device)
            else:
                stream.synchronize()
            err = self.error()
            if err:
                raise _lib.OmpiAmdError(err, what)

    # -- collectives ---------------------------------------------------------
    def allreduce(self, sbuf, rbuf, count: int, datatype: Datatype, op: Op, stream=None,
                  blocking: bool = False) -> None:
        rc = self._lib.ompi_amd_allreduce(self._h, _ptr(sbuf), _ptr(rbuf), count, datatype.code,
                                          op.index, _stream(stream))
        self._finish(rc, f"allreduce({op.name},{datatype.name})", blocking, stream)

    def allreduce_wait(self, sbuf, rbuf, count: int, datatype: Datatype, op: Op) -> None:
        """MPI_Allreduce's blocking form on the per-thread stream
        (ompi_amd_allreduce_wait: a fused small call stores its own
        completion mark)."""
        _lib.check(self._lib.ompi_amd_allreduce_wait(self._h, _ptr(sbuf), _ptr(rbuf), count,
                                                     datatype.code, op.index),
                   f"allreduce_wait({op.name},{datatype.name})")

    def iallreduce(self, sbuf, rbuf, count: int, datatype: Datatype, op: Op,
                   stream=None) -> "Request":
        """MPI_Iallreduce: returns without waiting for any peer."""
        h = ctypes.c_void_p()
        _lib.check(self._lib.ompi_amd_iallreduce(self._h, _ptr(sbuf), _ptr(rbuf), count,
                                                 datatype.code, op.index, _stream(stream),
                                                 ctypes.byref(h)),
                   f"iallreduce({op.name},{datatype.name})")
        return Request(self, h, f"iallreduce({op.name},{datatype.name})")

    def allreduce_init(self, sbuf, rbuf, count: int, datatype: Datatype, op: Op) -> "Plan":
        """MPI_Allreduce_init: a persistent allreduce (collective); start()
        enqueues it without any host rendezvous."""
        h = ctypes.c_void_p()
        _lib.check(self._lib.ompi_amd_allreduce_init(self._h, _ptr(sbuf), _ptr(rbuf), count,
                                                     datatype.code, op.index, ctypes.byref(h)),
                   f"allreduce_init({op.name},{datatype.name})")
        return Plan(self, h, f"allreduce({op.name},{datatype.name})")

    def reduce(self, sbuf, rbuf, count: int, datatype: Datatype, op: Op, root: int,
               stream=None, blocking: bool = False) -> None:
        """MPI_Reduce; rbuf may be None off the root, sbuf IN_PLACE at the root."""
        rc = self._lib.ompi_amd_reduce(self._h, _ptr(sbuf), _ptr(rbuf) if rbuf is not None else None,
                                       count, datatype.code, op.index, root, _stream(stream))
        self._finish(rc, f"reduce({op.name},{datatype.name},root={root})", blocking, stream)

    def scan(self, sbuf, rbuf, count: int, datatype: Datatype, op: Op, stream=None,
             blocking: bool = False) -> None:
        rc = self._lib.ompi_amd_scan(self._h, _ptr(sbuf), _ptr(rbuf), count, datatype.code,
                                     op.index, _stream(stream))
        self._finish(rc, f"scan({op.name},{datatype.name})", blocking, stream)

    def exscan(self, sbuf, rbuf, count: int, datatype: Datatype, op: Op, stream=None,
               blocking: bool = False) -> None:
        rc = self._lib.ompi_amd_exscan(self._h, _ptr(sbuf), _ptr(rbuf), count, datatype.code,
                                       op.index, _stream(stream))
        self._finish(rc, f"exscan({op.name},{datatype.name})", blocking, stream)

    def reduce_scatter(self, sbuf, rbuf, rcounts, datatype: Datatype, op: Op, stream=None,
                       blocking: bool = False) -> None:
        """MPI_Reduce_scatter: rbuf gets rcounts[rank] elements of the reduction."""
        arr = (ctypes.c_size_t * self.size)(*[int(c) for c in rcounts])
        rc = self._lib.ompi_amd_reduce_scatter(self._h, _ptr(sbuf), _ptr(rbuf), arr, datatype.code,
                                               op.index, _stream(stream))
        self._finish(rc, f"reduce_scatter({op.name},{datatype.name})", blocking, stream)

    def reduce_scatter_block(self, sbuf, rbuf, rcount: int, datatype: Datatype, op: Op,
                             stream=None, blocking: bool = False) -> None:
        rc = self._lib.ompi_amd_reduce_scatter_block(self._h, _ptr(sbuf), _ptr(rbuf), rcount,
                                                     datatype.code, op.index, _stream(stream))
        self._finish(rc, f"reduce_scatter_block({op.name},{datatype.name})", blocking, stream)

    def allgather(self, sbuf, rbuf, nbytes: int, stream=None, blocking: bool = False) -> None:
        """`nbytes` per rank (scount * extent of a contiguous sdtype)."""
        rc = self._lib.ompi_amd_allgather(self._h, _ptr(sbuf), _ptr(rbuf), nbytes, _stream(stream))
        self._finish(rc, "allgather", blocking, stream)

    def bcast(self, buf, nbytes: int, root: int, stream=None, blocking: bool = False) -> None:
        rc = self._lib.ompi_amd_bcast(self._h, _ptr(buf), nbytes, root, _stream(stream))
        self._finish(rc, "bcast", blocking, stream)

    # -- nonblocking forms (coll.h:261-410) -----------------------------------
    def ireduce_scatter_block(self, sbuf, rbuf, rcount: int, datatype: Datatype, op: Op,
                              stream=None) -> "Request":
        h = ctypes.c_void_p()
        what = f"ireduce_scatter_block({op.name},{datatype.name})"
        _lib.check(self._lib.ompi_amd_ireduce_scatter_block(self._h, _ptr(sbuf), _ptr(rbuf), rcount,
                                                            datatype.code, op.index,
                                                            _stream(stream), ctypes.byref(h)), what)
        return Request(self, h, what)

    def iallgather(self, sbuf, rbuf, nbytes: int, stream=None) -> "Request":
        h = ctypes.c_void_p()
        _lib.check(self._lib.ompi_amd_iallgather(self._h, _ptr(sbuf), _ptr(rbuf), nbytes,
                                                 _stream(stream), ctypes.byref(h)), "iallgather")
        return Request(self, h, "iallgather")

    def ibcast(self, buf, nbytes: int, root: int, stream=None) -> "Request":
        h = ctypes.c_void_p()
        _lib.check(self._lib.ompi_amd_ibcast(self._h, _ptr(buf), nbytes, root, _stream(stream),
                                             ctypes.byref(h)), "ibcast")
        return Request(self, h, "ibcast")

    def ireduce(self, sbuf, rbuf, count: int, datatype: Datatype, op: Op, root: int,
                stream=None) -> "Request":
        """MPI_Ireduce (rbuf may be None off the root, sbuf IN_PLACE at it)."""
        h = ctypes.c_void_p()
        what = f"ireduce({op.name},{datatype.name},root={root})"
        _lib.check(self._lib.ompi_amd_ireduce(self._h, _ptr(sbuf), _ptr(rbuf) if rbuf is not None else None,
                                              count, datatype.code, op.index, root, _stream(stream),
                                              ctypes.byref(h)), what)
        return Request(self, h, what)

    def iscan(self, sbuf, rbuf, count: int, datatype: Datatype, op: Op, stream=None,
              exclusive: bool = False) -> "Request":
        """MPI_Iscan (exclusive: MPI_Iexscan)."""
        h = ctypes.c_void_p()
        fn = self._lib.ompi_amd_iexscan if exclusive else self._lib.ompi_amd_iscan
        what = f"{'iexscan' if exclusive else 'iscan'}({op.name},{datatype.name})"
        _lib.check(fn(self._h, _ptr(sbuf), _ptr(rbuf), count, datatype.code, op.index, _stream(stream),
                      ctypes.byref(h)), what)
        return Request(self, h, what)

    def ireduce_scatter(self, sbuf, rbuf, rcounts, datatype: Datatype, op: Op,
                        stream=None) -> "Request":
        h = ctypes.c_void_p()
        arr = (ctypes.c_size_t * self.size)(*[int(c) for c in rcounts])
        what = f"ireduce_scatter({op.name},{datatype.name})"
        _lib.check(self._lib.ompi_amd_ireduce_scatter(self._h, _ptr(sbuf), _ptr(rbuf), arr,
                                                      datatype.code, op.index, _stream(stream),
                                                      ctypes.byref(h)), what)
        return Request(self, h, what)

    # -- persistent forms (MPI-4 *_init, coll.h:545-566) ----------------------
    def reduce_scatter_block_init(self, sbuf, rbuf, rcount: int, datatype: Datatype,
                                  op: Op) -> "Plan":
        h = ctypes.c_void_p()
        _lib.check(self._lib.ompi_amd_reduce_scatter_block_init(self._h, _ptr(sbuf), _ptr(rbuf), rcount,
                                                                datatype.code, op.index, ctypes.byref(h)),
                   "reduce_scatter_block_init")
        return Plan(self, h, f"reduce_scatter_block({op.name},{datatype.name})")

    def allgather_init(self, sbuf, rbuf, nbytes: int) -> "Plan":
        h = ctypes.c_void_p()
        _lib.check(self._lib.ompi_amd_allgather_init(self._h, _ptr(sbuf), _ptr(rbuf), nbytes,
                                                     ctypes.byref(h)), "allgather_init")
        return Plan(self, h, "allgather")

    def bcast_init(self, buf, nbytes: int, root: int) -> "Plan":
        h = ctypes.c_void_p()
        _lib.check(self._lib.ompi_amd_bcast_init(self._h, _ptr(buf), nbytes, root, ctypes.byref(h)),
                   "bcast_init")
        return Plan(self, h, "bcast")

    def reduce_init(self, sbuf, rbuf, count: int, datatype: Datatype, op: Op, root: int) -> "Plan":
        """MPI_Reduce_init (coll.h:561 coll_reduce_init): every start posts ireduce."""
        h = ctypes.c_void_p()
        what = f"reduce({op.name},{datatype.name},root={root})"
        _lib.check(self._lib.ompi_amd_reduce_init(self._h, _ptr(sbuf),
                                                  _ptr(rbuf) if rbuf is not None else None, count,
                                                  datatype.code, op.index, root, ctypes.byref(h)),
                   what + "_init")
        return Plan(self, h, what)

    def reduce_scatter_init(self, sbuf, rbuf, rcounts, datatype: Datatype, op: Op) -> "Plan":
        """MPI_Reduce_scatter_init (coll.h:562 coll_reduce_scatter_init)."""
        h = ctypes.c_void_p()
        arr = (ctypes.c_size_t * self.size)(*[int(c) for c in rcounts])
        what = f"reduce_scatter({op.name},{datatype.name})"
        _lib.check(self._lib.ompi_amd_reduce_scatter_init(self._h, _ptr(sbuf), _ptr(rbuf), arr,
                                                          datatype.code, op.index, ctypes.byref(h)),
                   what + "_init")
        return Plan(self, h, what)

    def scan_init(self, sbuf, rbuf, count: int, datatype: Datatype, op: Op,
                  exclusive: bool = False) -> "Plan":
        """MPI_Scan_init / MPI_Exscan_init (coll.h:558, 564)."""
        h = ctypes.c_void_p()
        fn = self._lib.ompi_amd_exscan_init if exclusive else self._lib.ompi_amd_scan_init
        what = f"{'exscan' if exclusive else 'scan'}({op.name},{datatype.name})"
        _lib.check(fn(self._h, _ptr(sbuf), _ptr(rbuf), count, datatype.code, op.index, ctypes.byref(h)),
                   what + "_init")
        return Plan(self, h, what)

    def __del__(self):
        # destroy is collective; only an explicit free() releases the comm
        pass


class Plan:
    """A persistent collective (ompi_amd_plan_t)."""

    def __init__(self, comm: Communicator, handle, what: str):
        self._comm, self._h, self._what = comm, handle, what

    def start(self, stream=None, blocking: bool = False) -> None:
        rc = self._comm._lib.ompi_amd_plan_start(self._h, _stream(stream))
        self._comm._finish(rc, "start " + self._what, blocking, stream)

    def test(self) -> bool:
        done = ctypes.c_int()
        _lib.check(self._comm._lib.ompi_amd_plan_test(self._h, ctypes.byref(done)),
                   "test " + self._what)
        return bool(done.value)

    def wait(self) -> None:
        _lib.check(self._comm._lib.ompi_amd_plan_wait(self._h), "wait " + self._what)

    @property
    def kind(self) -> int:
        """0 re-run of the plain call (fused / staged / push-gather), 1 pull,
        2 pull+push, 3 push on the caller's mapped buffers."""
        return self._comm._lib.ompi_amd_plan_kind(self._h)

    def free(self) -> None:
        if self._h:
            _lib.check(self._comm._lib.ompi_amd_plan_free(self._h), "plan_free")
            self._h = None


class Request:
    """A nonblocking collective (ompi_amd_request_t): test / wait / free."""

    def __init__(self, comm: Communicator, handle, what: str):
        self._comm, self._h, self._what = comm, handle, what

    def test(self) -> bool:
        done = ctypes.c_int()
        _lib.check(self._comm._lib.ompi_amd_request_test(self._h, ctypes.byref(done)),
                   "test " + self._what)
        return bool(done.value)

    def wait(self) -> None:
        _lib.check(self._comm._lib.ompi_amd_request_wait(self._h), "wait " + self._what)

    def free(self) -> None:
        if self._h:
            h, self._h = self._h, None
            _lib.check(self._comm._lib.ompi_amd_request_free(h), "free " + self._what)


def block_partition(count: int, nranks: int, block: int) -> tuple[int, int]:
    """(offset, count) of ring block `block` (COLL_BASE_COMPUTE_BLOCKCOUNT,
    coll_base_functions.h:425-431) as the library computes it."""
    lib = _lib.load()
    off, cnt = ctypes.c_size_t(), ctypes.c_size_t()
    _lib.check(lib.ompi_amd_coll_block(count, nranks, block, ctypes.byref(off), ctypes.byref(cnt)),
               "coll_block")
    return off.value, cnt.value


ORDER_NAMES = {0: "ring", 1: "recursive_doubling", 2: "chain", 3: "binomial", 4: "binary"}


def reduce_order(nranks: int, msg_bytes: int, count: int, root: int,
                 root_inplace: bool = False, forced: int = 0) -> tuple[str, int]:
    """(operand order, virtual-rank-0) the library folds a reduce / rsb in:
    coll/tuned's fixed reduce decision (coll_tuned_decision_fixed.c:354-428),
    or its forced algorithm `forced` (coll_tuned_reduce_decision.c:146-179;
    OmpiAmdError ERR_UNSUPPORTED for the ones the device path leaves to tuned)."""
    o, f = ctypes.c_int(), ctypes.c_int()
    _lib.check(_lib.load().ompi_amd_coll_reduce_order_forced(nranks, msg_bytes, count, root,
                                                             1 if root_inplace else 0, forced,
                                                             ctypes.byref(o), ctypes.byref(f)),
               "coll_reduce_order")
    return ORDER_NAMES[o.value], f.value


def block_owner(nranks: int, block: int) -> int:
    """Rank that produces ring block `block` (the rank where the
    reference's ring finishes it: block - 1 mod N)."""
    return _lib.load().ompi_amd_coll_owner(nranks, block)
