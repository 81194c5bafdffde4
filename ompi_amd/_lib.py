"""ctypes binding of libompi_amd.so (the C ABI declared in include/ompi_amd.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (or
``make -C ompi_amd/csrc``).  There is no fallback: if the library is missing
every entry point raises, so a test or bench can never silently run on a
CPU path.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libompi_amd.so")

# status codes (include/ompi_amd.h)
SUCCESS = 0
ERR_UNSUPPORTED = -1
ERR_BAD_PARAM = -2
ERR_HIP = -3
ERR_TIMEOUT = -4
ERR_NOT_DEVICE = -5
ERR_BOOTSTRAP = -6
ERR_RMA_SYNC = -7
ERR_TRUNCATE = -7

_ERRNAMES = {
    ERR_UNSUPPORTED: "unsupported (op,type)",
    ERR_BAD_PARAM: "bad parameter",
    ERR_HIP: "HIP error",
    ERR_TIMEOUT: "timeout waiting for a peer",
    ERR_NOT_DEVICE: "buffer is not device memory",
    ERR_BOOTSTRAP: "bootstrap failure",
    ERR_RMA_SYNC: "RMA synchronisation call out of order",
    ERR_TRUNCATE: "message truncated",
}


class OmpiAmdError(RuntimeError):
    def __init__(self, code: int, what: str):
        detail = ""
        if _lib is not None:
            detail = _lib.ompi_amd_last_error().decode(errors="replace")
        super().__init__(f"{what}: {_ERRNAMES.get(code, code)} {detail}".strip())
        self.code = code


_lib = None

HANDLER_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p,
                              ctypes.POINTER(ctypes.c_int), ctypes.c_void_p,
                              ctypes.c_void_p)
HANDLER3_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                               ctypes.c_void_p, ctypes.c_void_p)


class DdtBlock(ctypes.Structure):
    _fields_ = [("disp", ctypes.c_int64), ("len", ctypes.c_int64)]


class Iovec(ctypes.Structure):
    """ompi_amd_iovec_t (layout of struct iovec)."""
    _fields_ = [("iov_base", ctypes.c_void_p), ("iov_len", ctypes.c_size_t)]


class DdtElem(ctypes.Structure):
    _fields_ = [("count", ctypes.c_int64), ("blocklen", ctypes.c_int64),
                ("stride", ctypes.c_int64), ("disp", ctypes.c_int64)]


class Status(ctypes.Structure):
    """ompi_amd_status_t (include/ompi_amd_p2p.h)."""
    _fields_ = [("source", ctypes.c_int), ("tag", ctypes.c_int), ("error", ctypes.c_int),
                ("bytes", ctypes.c_size_t)]


# (name, restype, argtypes) for every symbol include/ompi_amd*.h declares
_C = ctypes
PROTOTYPES = [
    ("ompi_amd_version", _C.c_char_p, []),
    ("ompi_amd_device_count", _C.c_int, []),
    ("ompi_amd_last_error", _C.c_char_p, []),
    ("ompi_amd_op_supported", _C.c_int, [_C.c_int, _C.c_int]),
    ("ompi_amd_type_extent", _C.c_size_t, [_C.c_int]),
    ("ompi_amd_op_reduce", _C.c_int,
     [_C.c_int, _C.c_int, _C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_void_p]),
    ("ompi_amd_op_reduce_3buff", _C.c_int,
     [_C.c_int, _C.c_int, _C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_void_p]),
    ("ompi_amd_op_handler_row", _C.POINTER(_C.c_void_p), [_C.c_int]),
    ("ompi_amd_op_3buff_handler_row", _C.POINTER(_C.c_void_p), [_C.c_int]),
    ("ompi_amd_op_set_fallback", _C.c_int,
     [_C.c_int, _C.c_int, _C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_void_p]),
    ("ompi_amd_set_thread_stream", _C.c_int, [_C.c_void_p]),
    ("ompi_amd_set_tuning", _C.c_int, [_C.c_char_p, _C.c_int64]),
    ("ompi_amd_ddt_create", _C.c_int,
     [_C.POINTER(DdtBlock), _C.c_int, _C.c_int64, _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_ddt_create_elems", _C.c_int,
     [_C.POINTER(DdtElem), _C.c_int, _C.c_int64, _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_ddt_destroy", _C.c_int, [_C.c_void_p]),
    ("ompi_amd_ddt_size", _C.c_size_t, [_C.c_void_p]),
    ("ompi_amd_ddt_nelems", _C.c_int, [_C.c_void_p]),
    ("ompi_amd_ddt_pack", _C.c_int,
     [_C.c_void_p, _C.c_size_t, _C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_size_t,
      _C.POINTER(_C.c_size_t), _C.c_void_p]),
    ("ompi_amd_ddt_unpack", _C.c_int,
     [_C.c_void_p, _C.c_size_t, _C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_size_t,
      _C.POINTER(_C.c_size_t), _C.c_void_p]),
    ("ompi_amd_ddt_pack_iov", _C.c_int,
     [_C.c_void_p, _C.c_size_t, _C.c_void_p, _C.c_size_t, _C.c_void_p, _C.POINTER(_C.c_uint32),
      _C.POINTER(_C.c_size_t), _C.c_void_p]),
    ("ompi_amd_ddt_unpack_iov", _C.c_int,
     [_C.c_void_p, _C.c_size_t, _C.c_void_p, _C.c_size_t, _C.c_void_p, _C.POINTER(_C.c_uint32),
      _C.POINTER(_C.c_size_t), _C.c_void_p]),
    ("ompi_amd_is_device_pointer", _C.c_int, [_C.c_void_p]),
    ("ompi_amd_pointer_range", _C.c_int, [_C.c_void_p, _C.POINTER(_C.c_void_p), _C.POINTER(_C.c_size_t)]),
    ("ompi_amd_memcpy_async", _C.c_int, [_C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_void_p]),
    ("ompi_amd_memcpy", _C.c_int, [_C.c_void_p, _C.c_void_p, _C.c_size_t]),
    ("ompi_amd_memmove", _C.c_int, [_C.c_void_p, _C.c_void_p, _C.c_size_t]),
    ("ompi_amd_device_alloc", _C.c_int, [_C.POINTER(_C.c_void_p), _C.c_size_t]),
    ("ompi_amd_host_alloc", _C.c_int, [_C.POINTER(_C.c_void_p), _C.c_size_t]),
    ("ompi_amd_host_free", _C.c_int, [_C.c_void_p]),
    ("ompi_amd_event_record", _C.c_int, [_C.POINTER(_C.c_void_p), _C.c_void_p]),
    ("ompi_amd_event_query", _C.c_int, [_C.c_void_p]),
    ("ompi_amd_event_synchronize", _C.c_int, [_C.c_void_p]),
    ("ompi_amd_event_destroy", _C.c_int, [_C.c_void_p]),
    ("ompi_amd_device_free", _C.c_int, [_C.c_void_p]),
    ("ompi_amd_stream_synchronize", _C.c_int, [_C.c_void_p]),
    ("ompi_amd_comm_create", _C.c_int,
     [_C.c_char_p, _C.c_int, _C.c_int, _C.c_int, _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_comm_destroy", _C.c_int, [_C.c_void_p]),
    ("ompi_amd_comm_rank", _C.c_int, [_C.c_void_p]),
    ("ompi_amd_comm_size", _C.c_int, [_C.c_void_p]),
    ("ompi_amd_comm_set_param", _C.c_int, [_C.c_void_p, _C.c_char_p, _C.c_int64]),
    ("ompi_amd_comm_get_param", _C.c_int, [_C.c_void_p, _C.c_char_p, _C.POINTER(_C.c_int64)]),
    ("ompi_amd_comm_error", _C.c_int, [_C.c_void_p]),
    ("ompi_amd_comm_agree", _C.c_int, [_C.c_void_p, _C.c_int, _C.POINTER(_C.c_int)]),
    ("ompi_amd_comm_vote", _C.c_int, [_C.c_void_p, _C.c_int, _C.POINTER(_C.c_int)]),
    ("ompi_amd_comm_abort", _C.c_int, [_C.c_void_p, _C.c_int]),
    ("ompi_amd_allreduce_wait", _C.c_int, [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_size_t,
                                           _C.c_int, _C.c_int]),
    ("ompi_amd_comm_sync", _C.c_int, [_C.c_void_p, _C.c_void_p]),
    ("ompi_amd_comm_phase_ms", _C.c_int,
     [_C.c_void_p, _C.c_int, _C.POINTER(_C.c_double), _C.POINTER(_C.c_int)]),
    ("ompi_amd_coll_block", _C.c_int,
     [_C.c_size_t, _C.c_int, _C.c_int, _C.POINTER(_C.c_size_t), _C.POINTER(_C.c_size_t)]),
    ("ompi_amd_coll_owner", _C.c_int, [_C.c_int, _C.c_int]),
    ("ompi_amd_coll_reduce_order", _C.c_int,
     [_C.c_int, _C.c_size_t, _C.c_size_t, _C.c_int, _C.c_int, _C.POINTER(_C.c_int),
      _C.POINTER(_C.c_int)]),
    ("ompi_amd_coll_reduce_order_forced", _C.c_int,
     [_C.c_int, _C.c_size_t, _C.c_size_t, _C.c_int, _C.c_int, _C.c_int, _C.POINTER(_C.c_int),
      _C.POINTER(_C.c_int)]),
    ("ompi_amd_allreduce", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_int, _C.c_void_p]),
    ("ompi_amd_allreduce_init", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_int,
      _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_plan_start", _C.c_int, [_C.c_void_p, _C.c_void_p]),
    ("ompi_amd_plan_test", _C.c_int, [_C.c_void_p, _C.POINTER(_C.c_int)]),
    ("ompi_amd_plan_wait", _C.c_int, [_C.c_void_p]),
    ("ompi_amd_plan_free", _C.c_int, [_C.c_void_p]),
    ("ompi_amd_plan_kind", _C.c_int, [_C.c_void_p]),
    ("ompi_amd_iallreduce", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_int, _C.c_void_p,
      _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_ireduce_scatter_block", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_int, _C.c_void_p,
      _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_iallgather", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_void_p, _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_ibcast", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_void_p, _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_ireduce", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_int, _C.c_int, _C.c_void_p,
      _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_iscan", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_int, _C.c_void_p,
      _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_iexscan", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_int, _C.c_void_p,
      _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_ireduce_scatter", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.POINTER(_C.c_size_t), _C.c_int, _C.c_int, _C.c_void_p,
      _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_reduce_scatter_block_init", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_int, _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_allgather_init", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_size_t, _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_bcast_init", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_reduce_init", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_int, _C.c_int,
      _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_reduce_scatter_init", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.POINTER(_C.c_size_t), _C.c_int, _C.c_int,
      _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_scan_init", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_int, _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_exscan_init", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_int, _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_request_test", _C.c_int, [_C.c_void_p, _C.POINTER(_C.c_int)]),
    ("ompi_amd_request_wait", _C.c_int, [_C.c_void_p]),
    ("ompi_amd_request_free", _C.c_int, [_C.c_void_p]),
    ("ompi_amd_reduce", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_int, _C.c_int,
      _C.c_void_p]),
    ("ompi_amd_reduce_scatter_block", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_int, _C.c_void_p]),
    ("ompi_amd_reduce_scatter", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.POINTER(_C.c_size_t), _C.c_int, _C.c_int,
      _C.c_void_p]),
    ("ompi_amd_scan", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_int, _C.c_void_p]),
    ("ompi_amd_exscan", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_int, _C.c_void_p]),
    ("ompi_amd_allgather", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_void_p]),
    ("ompi_amd_bcast", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_void_p]),
    # point-to-point (include/ompi_amd_p2p.h)
    ("ompi_amd_isend", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_int, _C.c_int, _C.c_void_p,
      _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_irecv", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_int, _C.c_void_p,
      _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_send", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_int, _C.c_int, _C.c_void_p]),
    ("ompi_amd_recv", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_int, _C.c_void_p,
      _C.POINTER(Status)]),
    ("ompi_amd_sendrecv", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_int, _C.c_void_p, _C.c_size_t,
      _C.c_int, _C.c_int, _C.c_void_p, _C.POINTER(Status)]),
    ("ompi_amd_p2p_test", _C.c_int, [_C.c_void_p, _C.POINTER(_C.c_int), _C.POINTER(Status)]),
    ("ompi_amd_p2p_wait", _C.c_int, [_C.c_void_p, _C.POINTER(Status)]),
    ("ompi_amd_p2p_free", _C.c_int, [_C.c_void_p]),
    ("ompi_amd_iprobe", _C.c_int,
     [_C.c_void_p, _C.c_int, _C.c_int, _C.POINTER(_C.c_int), _C.POINTER(Status)]),
    ("ompi_amd_probe", _C.c_int, [_C.c_void_p, _C.c_int, _C.c_int, _C.POINTER(Status)]),
    # one-sided (include/ompi_amd_osc.h)
    ("ompi_amd_win_create", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_win_allocate", _C.c_int,
     [_C.c_void_p, _C.c_size_t, _C.c_int, _C.POINTER(_C.c_void_p), _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_win_free", _C.c_int, [_C.c_void_p]),
    ("ompi_amd_win_fence", _C.c_int, [_C.c_void_p, _C.c_int, _C.c_void_p]),
    ("ompi_amd_win_lock", _C.c_int, [_C.c_void_p, _C.c_int, _C.c_int, _C.c_int, _C.c_void_p]),
    ("ompi_amd_win_unlock", _C.c_int, [_C.c_void_p, _C.c_int, _C.c_void_p]),
    ("ompi_amd_win_lock_all", _C.c_int, [_C.c_void_p, _C.c_int, _C.c_void_p]),
    ("ompi_amd_win_unlock_all", _C.c_int, [_C.c_void_p, _C.c_void_p]),
    ("ompi_amd_win_flush", _C.c_int, [_C.c_void_p, _C.c_int, _C.c_void_p]),
    ("ompi_amd_put", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_size_t, _C.c_void_p]),
    ("ompi_amd_get", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_size_t, _C.c_void_p]),
    ("ompi_amd_accumulate", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_int, _C.c_size_t, _C.c_int,
      _C.c_void_p]),
    ("ompi_amd_get_accumulate", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_int, _C.c_size_t,
      _C.c_int, _C.c_void_p]),
    ("ompi_amd_win_sync", _C.c_int, [_C.c_void_p, _C.c_void_p]),
    ("ompi_amd_win_model", _C.c_int, [_C.c_void_p]),
    ("ompi_amd_win_peer_base", _C.c_int, [_C.c_void_p, _C.c_int, _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_win_create_dynamic", _C.c_int, [_C.c_void_p, _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_win_attach", _C.c_int, [_C.c_void_p, _C.c_void_p, _C.c_size_t]),
    ("ompi_amd_win_detach", _C.c_int, [_C.c_void_p, _C.c_void_p]),
    ("ompi_amd_win_copies", _C.c_int, [_C.c_void_p, _C.POINTER(_C.c_void_p), _C.POINTER(_C.c_void_p),
                                       _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_put_ddt", _C.c_int, [_C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_void_p, _C.c_int,
                                    _C.c_size_t, _C.c_size_t, _C.c_void_p, _C.c_void_p]),
    ("ompi_amd_get_ddt", _C.c_int, [_C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_void_p, _C.c_int,
                                    _C.c_size_t, _C.c_size_t, _C.c_void_p, _C.c_void_p]),
    ("ompi_amd_rput_ddt", _C.c_int, [_C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_void_p, _C.c_int,
                                     _C.c_size_t, _C.c_size_t, _C.c_void_p, _C.c_void_p,
                                     _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_rget_ddt", _C.c_int, [_C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_void_p, _C.c_int,
                                     _C.c_size_t, _C.c_size_t, _C.c_void_p, _C.c_void_p,
                                     _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_accumulate_ddt", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_void_p, _C.c_int, _C.c_size_t, _C.c_size_t,
      _C.c_void_p, _C.c_int, _C.c_int, _C.c_void_p]),
    ("ompi_amd_get_accumulate_ddt", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_void_p,
      _C.c_int, _C.c_size_t, _C.c_size_t, _C.c_void_p, _C.c_int, _C.c_int, _C.c_void_p]),
    ("ompi_amd_raccumulate_ddt", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_void_p, _C.c_int, _C.c_size_t, _C.c_size_t,
      _C.c_void_p, _C.c_int, _C.c_int, _C.c_void_p, _C.c_void_p]),
    ("ompi_amd_rget_accumulate_ddt", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_void_p,
      _C.c_int, _C.c_size_t, _C.c_size_t, _C.c_void_p, _C.c_int, _C.c_int, _C.c_void_p,
      _C.c_void_p]),
    ("ompi_amd_fetch_and_op", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_int, _C.c_int, _C.c_size_t, _C.c_int,
      _C.c_void_p]),
    ("ompi_amd_compare_and_swap", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_int, _C.c_int, _C.c_size_t,
      _C.c_void_p]),
    ("ompi_amd_win_allocate_shared", _C.c_int,
     [_C.c_void_p, _C.c_size_t, _C.c_int, _C.c_int, _C.POINTER(_C.c_void_p),
      _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_win_shared_query", _C.c_int,
     [_C.c_void_p, _C.c_int, _C.POINTER(_C.c_size_t), _C.POINTER(_C.c_int),
      _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_win_post", _C.c_int,
     [_C.c_void_p, _C.POINTER(_C.c_int), _C.c_int, _C.c_int, _C.c_void_p]),
    ("ompi_amd_win_start", _C.c_int,
     [_C.c_void_p, _C.POINTER(_C.c_int), _C.c_int, _C.c_int, _C.c_void_p]),
    ("ompi_amd_win_complete", _C.c_int, [_C.c_void_p, _C.c_void_p]),
    ("ompi_amd_win_wait", _C.c_int, [_C.c_void_p, _C.c_void_p]),
    ("ompi_amd_win_test", _C.c_int, [_C.c_void_p, _C.POINTER(_C.c_int)]),
    ("ompi_amd_rput", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_size_t, _C.c_void_p,
      _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_rget", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_size_t, _C.c_void_p,
      _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_raccumulate", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_int, _C.c_size_t, _C.c_int,
      _C.c_void_p, _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_rget_accumulate", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_size_t, _C.c_int, _C.c_int, _C.c_size_t,
      _C.c_int, _C.c_void_p, _C.POINTER(_C.c_void_p)]),
    ("ompi_amd_rma_test", _C.c_int, [_C.c_void_p, _C.POINTER(_C.c_int)]),
    ("ompi_amd_rma_wait", _C.c_int, [_C.c_void_p]),
    ("ompi_amd_rma_free", _C.c_int, [_C.c_void_p]),
]


def load(path: str = LIB_PATH):
    """Load libompi_amd.so once; raise loudly if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(
            f"libompi_amd.so not built at {path}: run __graft_entry__.build() "
            "(or make -C ompi_amd/csrc). There is no CPU fallback.")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    for name, res, args in PROTOTYPES:
        fn = getattr(lib, name, None)
        if fn is None:
            continue  # checked explicitly by tests/test_abi.py
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != SUCCESS:
        raise OmpiAmdError(rc, what)
