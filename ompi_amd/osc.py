"""One-sided communication on device windows (the osc surface for device
memory).

Mirrors osc/sm's module functions (ompi/mca/osc/sm/osc_sm_comm.c,
osc_sm_active_target.c, osc_sm_passive_target.c):

    put / get                      osc_sm_comm.c:209-268
    accumulate                     osc_sm_comm.c:271-309
    get_accumulate                 osc_sm_comm.c:312-360
    compare_and_swap               osc_sm_comm.c:363-400
    fetch_and_op                   osc_sm_comm.c:403-441
    allocate_shared / shared_query osc_sm_component.c:244-360, 455-485
    fence                          osc_sm_active_target.c:95-115
    post / start / complete / wait / test
                                   osc_sm_active_target.c:126-335
    rput / rget / raccumulate / rget_accumulate
                                   osc_sm_comm.c:23-206
    lock / unlock / lock_all / unlock_all / flush
                                   osc_sm_passive_target.c:113-270

Displacements are in the target's disp_unit, counts in elements of the
datatype.  Every call is stream-ordered on the origin's stream; the RMA
kernels load and store the target's memory over xGMI
(include/ompi_amd_osc.h).  There is no host fallback.
"""
from __future__ import annotations

import ctypes

from . import _lib
from .coll import Communicator, _ptr, _stream
from .op import Datatype, Op

LOCK_EXCLUSIVE = 1   # MPI_LOCK_EXCLUSIVE (mpi.h.in:548)
LOCK_SHARED = 2      # MPI_LOCK_SHARED (mpi.h.in:549)
MODE_NOCHECK = 1     # MPI_MODE_NOCHECK (mpi.h.in:542)
WIN_UNIFIED = 0      # MPI_WIN_UNIFIED (mpi.h.in:556)
WIN_SEPARATE = 1     # MPI_WIN_SEPARATE (mpi.h.in:557)


class RmaRequest:
    """The request of MPI_Rput / _Rget / _Raccumulate / _Rget_accumulate:
    complete when the call's kernels have finished."""

    def __init__(self, lib, handle):
        self._lib, self._h = lib, handle

    def test(self) -> bool:
        done = ctypes.c_int(0)
        _lib.check(self._lib.ompi_amd_rma_test(self._h, ctypes.byref(done)), "rma_test")
        return bool(done.value)

    def wait(self) -> None:
        _lib.check(self._lib.ompi_amd_rma_wait(self._h), "rma_wait")

    def free(self) -> None:
        if self._h:
            h, self._h = self._h, None
            _lib.check(self._lib.ompi_amd_rma_free(h), "rma_free")


def _ranks(ranks):
    ranks = list(ranks)
    return (ctypes.c_int * max(1, len(ranks)))(*ranks), len(ranks)


class Window:
    """MPI_Win over device memory of every rank of `comm`."""

    def __init__(self, comm: Communicator, handle, base_ptr: int, nbytes: int):
        self.comm, self._h, self.base_ptr, self.nbytes = comm, handle, base_ptr, nbytes
        self._lib = comm._lib

    @classmethod
    def create(cls, comm: Communicator, base, nbytes: int | None = None,
               disp_unit: int = 1) -> "Window":
        """MPI_Win_create (collective) over a device tensor / pointer."""
        if nbytes is None:
            nbytes = base.numel() * base.element_size() if base is not None else 0
        ptr = _ptr(base) if nbytes else None
        h = ctypes.c_void_p()
        _lib.check(comm._lib.ompi_amd_win_create(comm._h, ptr, nbytes, disp_unit,
                                                 ctypes.byref(h)), "win_create")
        return cls(comm, h, ptr or 0, nbytes)

    @classmethod
    def allocate(cls, comm: Communicator, nbytes: int, disp_unit: int = 1) -> "Window":
        """MPI_Win_allocate (collective): zeroed device memory owned by the
        window; `base_ptr` is its address."""
        h, b = ctypes.c_void_p(), ctypes.c_void_p()
        _lib.check(comm._lib.ompi_amd_win_allocate(comm._h, nbytes, disp_unit, ctypes.byref(b),
                                                   ctypes.byref(h)), "win_allocate")
        return cls(comm, h, b.value or 0, nbytes)

    @classmethod
    def allocate_shared(cls, comm: Communicator, nbytes: int, disp_unit: int = 1,
                        noncontig: bool = False) -> "Window":
        """MPI_Win_allocate_shared (collective): every rank's segment in one
        device allocation of rank 0, contiguous in every process unless
        `noncontig`; `base_ptr` is this rank's segment."""
        h, b = ctypes.c_void_p(), ctypes.c_void_p()
        _lib.check(comm._lib.ompi_amd_win_allocate_shared(comm._h, nbytes, disp_unit,
                                                          int(noncontig), ctypes.byref(b),
                                                          ctypes.byref(h)), "win_allocate_shared")
        return cls(comm, h, b.value or 0, nbytes)

    @classmethod
    def create_dynamic(cls, comm: Communicator) -> "Window":
        """MPI_Win_create_dynamic (collective): no memory until attach();
        displacements are the target's absolute addresses."""
        h = ctypes.c_void_p()
        _lib.check(comm._lib.ompi_amd_win_create_dynamic(comm._h, ctypes.byref(h)),
                   "win_create_dynamic")
        return cls(comm, h, 0, 0)

    def attach(self, base, nbytes: int | None = None) -> int:
        """MPI_Win_attach (local) of device memory; returns its address (the
        displacement peers use, after the application shares it)."""
        if nbytes is None:
            nbytes = base.numel() * base.element_size()
        ptr = _ptr(base)
        _lib.check(self._lib.ompi_amd_win_attach(self._h, ptr, nbytes), "win_attach")
        return ptr

    def detach(self, base) -> None:
        """MPI_Win_detach (local)."""
        _lib.check(self._lib.ompi_amd_win_detach(self._h, _ptr(base)), "win_detach")

    def shared_query(self, rank: int):
        """MPI_Win_shared_query: (size, disp_unit, address in this process)
        of `rank`'s segment; rank < 0 (MPI_PROC_NULL) = the first nonzero one."""
        size, du, base = ctypes.c_size_t(), ctypes.c_int(), ctypes.c_void_p()
        _lib.check(self._lib.ompi_amd_win_shared_query(self._h, rank, ctypes.byref(size),
                                                       ctypes.byref(du), ctypes.byref(base)),
                   "win_shared_query")
        return size.value, du.value, base.value or 0

    def free(self) -> None:
        if self._h:
            h, self._h = self._h, None
            _lib.check(self._lib.ompi_amd_win_free(h), "win_free")

    # -- synchronisation -----------------------------------------------------
    def _done(self, rc: int, what: str, blocking: bool, stream) -> None:
        self.comm._finish(rc, what, blocking, stream)

    def fence(self, assert_: int = 0, stream=None, blocking: bool = False) -> None:
        self._done(self._lib.ompi_amd_win_fence(self._h, assert_, _stream(stream)), "win_fence",
                   blocking, stream)

    def lock(self, target: int, lock_type: int = LOCK_EXCLUSIVE, assert_: int = 0,
             stream=None) -> None:
        _lib.check(self._lib.ompi_amd_win_lock(self._h, lock_type, target, assert_,
                                               _stream(stream)), "win_lock")

    def unlock(self, target: int, stream=None, blocking: bool = True) -> None:
        self._done(self._lib.ompi_amd_win_unlock(self._h, target, _stream(stream)), "win_unlock",
                   blocking, stream)

    def lock_all(self, assert_: int = 0, stream=None) -> None:
        _lib.check(self._lib.ompi_amd_win_lock_all(self._h, assert_, _stream(stream)),
                   "win_lock_all")

    def unlock_all(self, stream=None, blocking: bool = True) -> None:
        self._done(self._lib.ompi_amd_win_unlock_all(self._h, _stream(stream)), "win_unlock_all",
                   blocking, stream)

    @property
    def model(self) -> int:
        """MPI_WIN_MODEL: WIN_SEPARATE when some rank's MPI_Win_create
        memory is reached through a public copy (include/ompi_amd_osc.h)."""
        m = self._lib.ompi_amd_win_model(self._h)
        if m < 0:
            _lib.check(m, "win_model")
        return m

    def copies(self):
        """Diagnostics: (private, public, snapshot) device addresses of this
        rank's copies; public and snapshot are 0 where the window is unified."""
        p, q, s = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        _lib.check(self._lib.ompi_amd_win_copies(self._h, ctypes.byref(p), ctypes.byref(q),
                                                 ctypes.byref(s)), "win_copies")
        return p.value or 0, q.value or 0, s.value or 0

    def peer_base(self, peer: int) -> int:
        """Diagnostics: the address RMA toward `peer` targets in this process."""
        b = ctypes.c_void_p()
        _lib.check(self._lib.ompi_amd_win_peer_base(self._h, peer, ctypes.byref(b)), "win_peer_base")
        return b.value or 0

    def sync(self, stream=None) -> None:
        """MPI_Win_sync: the public and private copies merged."""
        _lib.check(self._lib.ompi_amd_win_sync(self._h, _stream(stream)), "win_sync")

    def flush(self, target: int, stream=None) -> None:
        _lib.check(self._lib.ompi_amd_win_flush(self._h, target, _stream(stream)), "win_flush")

    def post(self, ranks, assert_: int = 0, stream=None) -> None:
        """MPI_Win_post: open an exposure epoch to the origins `ranks`."""
        arr, n = _ranks(ranks)
        _lib.check(self._lib.ompi_amd_win_post(self._h, arr, n, assert_, _stream(stream)),
                   "win_post")

    def start(self, ranks, assert_: int = 0, stream=None) -> None:
        """MPI_Win_start: open an access epoch to the targets `ranks`
        (the stream waits until each of them posted)."""
        arr, n = _ranks(ranks)
        _lib.check(self._lib.ompi_amd_win_start(self._h, arr, n, assert_, _stream(stream)),
                   "win_start")

    def complete(self, stream=None, blocking: bool = False) -> None:
        self._done(self._lib.ompi_amd_win_complete(self._h, _stream(stream)), "win_complete",
                   blocking, stream)

    def wait(self, stream=None, blocking: bool = False) -> None:
        self._done(self._lib.ompi_amd_win_wait(self._h, _stream(stream)), "win_wait",
                   blocking, stream)

    def test(self) -> bool:
        flag = ctypes.c_int(0)
        _lib.check(self._lib.ompi_amd_win_test(self._h, ctypes.byref(flag)), "win_test")
        return bool(flag.value)

    # -- communication -------------------------------------------------------
    def put(self, origin, target: int, disp: int, nbytes: int | None = None, stream=None) -> None:
        n = origin.numel() * origin.element_size() if nbytes is None else nbytes
        _lib.check(self._lib.ompi_amd_put(self._h, _ptr(origin), n, target, disp,
                                          _stream(stream)), "put")

    def get(self, origin, target: int, disp: int, nbytes: int | None = None, stream=None) -> None:
        n = origin.numel() * origin.element_size() if nbytes is None else nbytes
        _lib.check(self._lib.ompi_amd_get(self._h, _ptr(origin), n, target, disp,
                                          _stream(stream)), "get")

    def accumulate(self, origin, count: int, datatype: Datatype, target: int, disp: int, op: Op,
                   stream=None) -> None:
        _lib.check(self._lib.ompi_amd_accumulate(self._h, _ptr(origin), count, datatype.code,
                                                 target, disp, op.index, _stream(stream)),
                   f"accumulate({op.name}, {datatype.name})")

    def get_accumulate(self, origin, result, count: int, datatype: Datatype, target: int,
                       disp: int, op: Op, stream=None) -> None:
        optr = _ptr(origin) if origin is not None else None
        _lib.check(self._lib.ompi_amd_get_accumulate(self._h, optr, _ptr(result), count,
                                                     datatype.code, target, disp, op.index,
                                                     _stream(stream)),
                   f"get_accumulate({op.name}, {datatype.name})")

    @staticmethod
    def _ddt(dt):
        return None if dt is None else dt.commit()._handle

    def put_ddt(self, origin, ocount: int, odt, target: int, disp: int, tcount: int, tdt,
                stream=None) -> None:
        """MPI_Put with derived datatypes (osc_sm_comm.c:24-100): odt / tdt
        are ompi_amd.datatype.Datatype, None meaning `ocount` / `tcount`
        contiguous bytes."""
        _lib.check(self._lib.ompi_amd_put_ddt(self._h, _ptr(origin), ocount, self._ddt(odt), target, disp,
                                              tcount, self._ddt(tdt), _stream(stream)), "put_ddt")

    def get_ddt(self, origin, ocount: int, odt, target: int, disp: int, tcount: int, tdt,
                stream=None) -> None:
        """MPI_Get with derived datatypes (osc_sm_comm.c:209-270)."""
        _lib.check(self._lib.ompi_amd_get_ddt(self._h, _ptr(origin), ocount, self._ddt(odt), target, disp,
                                              tcount, self._ddt(tdt), _stream(stream)), "get_ddt")

    def accumulate_ddt(self, origin, ocount: int, odt, target: int, disp: int, tcount: int, tdt,
                       prim: Datatype, op: Op, stream=None) -> None:
        """MPI_Accumulate with derived datatypes (ompi_osc_base_sndrcv_op):
        odt / tdt are ompi_amd.datatype.Datatype (None: `prim` contiguous)
        built from the predefined `prim`."""
        _lib.check(self._lib.ompi_amd_accumulate_ddt(self._h, _ptr(origin), ocount, self._ddt(odt),
                                                     target, disp, tcount, self._ddt(tdt), prim.code,
                                                     op.index, _stream(stream)),
                   f"accumulate_ddt({op.name}, {prim.name})")

    def get_accumulate_ddt(self, origin, ocount: int, odt, result, rcount: int, rdt, target: int,
                           disp: int, tcount: int, tdt, prim: Datatype, op: Op,
                           stream=None) -> None:
        optr = _ptr(origin) if origin is not None else None
        _lib.check(self._lib.ompi_amd_get_accumulate_ddt(
            self._h, optr, ocount, self._ddt(odt), _ptr(result), rcount, self._ddt(rdt), target,
            disp, tcount, self._ddt(tdt), prim.code, op.index, _stream(stream)),
            f"get_accumulate_ddt({op.name}, {prim.name})")

    def fetch_and_op(self, origin, result, datatype: Datatype, target: int, disp: int, op: Op,
                     stream=None) -> None:
        optr = _ptr(origin) if origin is not None else None
        _lib.check(self._lib.ompi_amd_fetch_and_op(self._h, optr, _ptr(result), datatype.code,
                                                   target, disp, op.index, _stream(stream)),
                   f"fetch_and_op({op.name}, {datatype.name})")

    def compare_and_swap(self, origin, compare, result, datatype: Datatype, target: int,
                         disp: int, stream=None) -> None:
        _lib.check(self._lib.ompi_amd_compare_and_swap(self._h, _ptr(origin), _ptr(compare),
                                                       _ptr(result), datatype.code, target, disp,
                                                       _stream(stream)), "compare_and_swap")

    # -- request-based communication ------------------------------------------
    def _req(self, fn, what, *args) -> RmaRequest:
        h = ctypes.c_void_p()
        _lib.check(fn(self._h, *args, ctypes.byref(h)), what)
        return RmaRequest(self._lib, h)

    def rput(self, origin, target: int, disp: int, nbytes: int | None = None,
             stream=None) -> RmaRequest:
        n = origin.numel() * origin.element_size() if nbytes is None else nbytes
        return self._req(self._lib.ompi_amd_rput, "rput", _ptr(origin), n, target, disp,
                         _stream(stream))

    def rput_ddt(self, origin, ocount: int, odt, target: int, disp: int, tcount: int, tdt,
                 stream=None) -> RmaRequest:
        return self._req(self._lib.ompi_amd_rput_ddt, "rput_ddt", _ptr(origin), ocount, self._ddt(odt),
                         target, disp, tcount, self._ddt(tdt), _stream(stream))

    def rget_ddt(self, origin, ocount: int, odt, target: int, disp: int, tcount: int, tdt,
                 stream=None) -> RmaRequest:
        return self._req(self._lib.ompi_amd_rget_ddt, "rget_ddt", _ptr(origin), ocount, self._ddt(odt),
                         target, disp, tcount, self._ddt(tdt), _stream(stream))

    def rget(self, origin, target: int, disp: int, nbytes: int | None = None,
             stream=None) -> RmaRequest:
        n = origin.numel() * origin.element_size() if nbytes is None else nbytes
        return self._req(self._lib.ompi_amd_rget, "rget", _ptr(origin), n, target, disp,
                         _stream(stream))

    def raccumulate(self, origin, count: int, datatype: Datatype, target: int, disp: int,
                    op: Op, stream=None) -> RmaRequest:
        return self._req(self._lib.ompi_amd_raccumulate, f"raccumulate({op.name})", _ptr(origin),
                         count, datatype.code, target, disp, op.index, _stream(stream))

    def rget_accumulate(self, origin, result, count: int, datatype: Datatype, target: int,
                        disp: int, op: Op, stream=None) -> RmaRequest:
        optr = _ptr(origin) if origin is not None else None
        return self._req(self._lib.ompi_amd_rget_accumulate, f"rget_accumulate({op.name})", optr,
                         _ptr(result), count, datatype.code, target, disp, op.index,
                         _stream(stream))
