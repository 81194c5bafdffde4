"""Which device allocations can hipIpcGetMemHandle export?

tests/coll_worker.py saw `hipIpcGetMemHandle: invalid argument` for a torch
tensor allocated after earlier segments had been returned with
torch.cuda.empty_cache() (3 ranks on one GPU, round 2).  This probe replays
that allocation pattern in one process: torch tensors of the sizes the
collective tests use, freed and re-allocated with empty_cache() between
rounds, each exported the way coll_ipc.hip's export_buf does (allocation
base from hipMemGetAddressRange, then hipIpcGetMemHandle(base)).  Prints one
JSON line per export; the failures say which pattern the runtime rejects.
"""
import ctypes
import json
import sys

import torch

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemGetAddressRange.argtypes = [ctypes.POINTER(ctypes.c_void_p),
                                      ctypes.POINTER(ctypes.c_size_t), ctypes.c_void_p]
hip.hipIpcGetMemHandle.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
hip.hipGetErrorString.restype = ctypes.c_char_p


def export(t):
    base, size = ctypes.c_void_p(), ctypes.c_size_t()
    e1 = hip.hipMemGetAddressRange(ctypes.byref(base), ctypes.byref(size), ctypes.c_void_p(t.data_ptr()))
    h = (ctypes.c_char * 64)()
    e2 = hip.hipIpcGetMemHandle(h, base) if e1 == 0 else -1
    return {"ptr": hex(t.data_ptr()), "bytes": t.numel(), "base": hex(base.value or 0),
            "range": size.value, "range_rc": e1, "export_rc": e2,
            "err": hip.hipGetErrorString(e2).decode() if e2 > 0 else ""}


def main():
    torch.cuda.init()
    fails = 0
    sizes = [16 << 20, (16 << 20) + 24, (4 << 20) + 28, 12 << 20, 1 << 20, 300007 * 4,
             (2 << 20) + 24, 64 << 20, 9000011 * 4, 8 << 20]
    for rnd in range(6):
        live = []
        for i, b in enumerate(sizes):
            t = torch.empty(b + 4096 * rnd, dtype=torch.uint8, device="cuda")
            r = export(t)
            r.update({"round": rnd, "i": i})
            fails += r["export_rc"] != 0
            print(json.dumps(r), flush=True)
            live.append(t)
            if i % 3 == 2:  # free some, keep others, as the tests do
                del live[0]
        del live
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    print(json.dumps({"failures": fails}), flush=True)
    sys.exit(0)


if __name__ == "__main__":
    main()
