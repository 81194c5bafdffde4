"""Point-to-point messages between device buffers (the PML surface for
device memory).

Mirrors the PML module entry points (ompi/mca/pml/pml.h):

    pml_isend(buf, count, dtype, dst, tag, mode, comm, request)   pml.h:317-326
    pml_irecv(buf, count, dtype, src, tag, comm, request)         pml.h:233-241
    pml_send / pml_recv                                           pml.h:341-349, 262-270
    pml_iprobe / pml_probe                                        pml.h:371-377, 398-403

with the message size in bytes (contiguous data; non-contiguous datatypes
go through ompi_amd.datatype's convertor first).  The receiver pulls the
sender's buffer over xGMI through its IPC mapping (include/ompi_amd_p2p.h);
there is no host fallback for device buffers.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

from . import _lib
from .coll import Communicator, _ptr, _stream

ANY_SOURCE = -1   # MPI_ANY_SOURCE
ANY_TAG = -1      # MPI_ANY_TAG

# mca_pml_base_send_mode_t (ompi/mca/pml/pml_constants.h:30-37)
SEND_SYNCHRONOUS, SEND_COMPLETE, SEND_BUFFERED, SEND_READY, SEND_STANDARD = range(5)


@dataclass
class Status:
    """MPI_Status of a receive / probe: MPI_SOURCE, MPI_TAG, MPI_ERROR and
    the message size in bytes (MPI_Get_count's numerator)."""
    source: int
    tag: int
    error: int
    bytes: int


def _status(st: _lib.Status) -> Status:
    return Status(st.source, st.tag, st.error, st.bytes)


def _nbytes(buf, nbytes):
    if nbytes is not None:
        return int(nbytes)
    return buf.numel() * buf.element_size()


class P2PRequest:
    """MPI_Request of an isend / irecv."""

    def __init__(self, comm: Communicator, handle, what: str):
        self._comm, self._h, self._what = comm, handle, what
        self.status: Status | None = None

    def test(self) -> bool:
        done, st = ctypes.c_int(), _lib.Status()
        _lib.check(self._comm._lib.ompi_amd_p2p_test(self._h, ctypes.byref(done),
                                                     ctypes.byref(st)), "test " + self._what)
        if done.value:
            self.status = _status(st)
        return bool(done.value)

    def wait(self) -> Status:
        st = _lib.Status()
        rc = self._comm._lib.ompi_amd_p2p_wait(self._h, ctypes.byref(st))
        self.status = _status(st)
        _lib.check(rc, "wait " + self._what)
        return self.status

    def free(self) -> None:
        if self._h:
            h, self._h = self._h, None
            _lib.check(self._comm._lib.ompi_amd_p2p_free(h), "free " + self._what)


def isend(comm: Communicator, buf, dst: int, tag: int, nbytes: int | None = None,
          mode: int = SEND_STANDARD, stream=None) -> P2PRequest:
    h = ctypes.c_void_p()
    _lib.check(comm._lib.ompi_amd_isend(comm._h, _ptr(buf), _nbytes(buf, nbytes), dst, tag, mode,
                                        _stream(stream), ctypes.byref(h)), "isend")
    return P2PRequest(comm, h, f"isend(to {dst}, tag {tag})")


def irecv(comm: Communicator, buf, src: int = ANY_SOURCE, tag: int = ANY_TAG,
          nbytes: int | None = None, stream=None) -> P2PRequest:
    h = ctypes.c_void_p()
    _lib.check(comm._lib.ompi_amd_irecv(comm._h, _ptr(buf), _nbytes(buf, nbytes), src, tag,
                                        _stream(stream), ctypes.byref(h)), "irecv")
    return P2PRequest(comm, h, f"irecv(from {src}, tag {tag})")


def send(comm: Communicator, buf, dst: int, tag: int, nbytes: int | None = None,
         mode: int = SEND_STANDARD, stream=None) -> None:
    _lib.check(comm._lib.ompi_amd_send(comm._h, _ptr(buf), _nbytes(buf, nbytes), dst, tag, mode,
                                       _stream(stream)), "send")


def recv(comm: Communicator, buf, src: int = ANY_SOURCE, tag: int = ANY_TAG,
         nbytes: int | None = None, stream=None) -> Status:
    st = _lib.Status()
    _lib.check(comm._lib.ompi_amd_recv(comm._h, _ptr(buf), _nbytes(buf, nbytes), src, tag,
                                       _stream(stream), ctypes.byref(st)), "recv")
    return _status(st)


def sendrecv(comm: Communicator, sbuf, dst: int, stag: int, rbuf, src: int, rtag: int,
             sbytes: int | None = None, rbytes: int | None = None, stream=None) -> Status:
    st = _lib.Status()
    _lib.check(comm._lib.ompi_amd_sendrecv(comm._h, _ptr(sbuf), _nbytes(sbuf, sbytes), dst, stag,
                                           _ptr(rbuf), _nbytes(rbuf, rbytes), src, rtag,
                                           _stream(stream), ctypes.byref(st)), "sendrecv")
    return _status(st)


def iprobe(comm: Communicator, src: int = ANY_SOURCE, tag: int = ANY_TAG) -> Status | None:
    flag, st = ctypes.c_int(), _lib.Status()
    _lib.check(comm._lib.ompi_amd_iprobe(comm._h, src, tag, ctypes.byref(flag), ctypes.byref(st)),
               "iprobe")
    return _status(st) if flag.value else None


def probe(comm: Communicator, src: int = ANY_SOURCE, tag: int = ANY_TAG) -> Status:
    st = _lib.Status()
    _lib.check(comm._lib.ompi_amd_probe(comm._h, src, tag, ctypes.byref(st)), "probe")
    return _status(st)
