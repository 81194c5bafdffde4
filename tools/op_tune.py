#!/usr/bin/env python3
"""Sweep the op kernel's build variants (unroll x nt policy, built by
`make -C ompi_amd/csrc tune`) and grid caps on fp32 3-buffer SUM, 1 GiB per
buffer.  One subprocess per variant; prints one JSON line per point."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TUNE = os.path.join(ROOT, "ompi_amd", "tune")


def run_variant(path, blocks_list, nbytes, iters):
    import ctypes

    import torch
    sys.path.insert(0, ROOT)
    from ompi_amd import _lib
    lib = _lib.load(path)
    n = nbytes // 4
    a = torch.randn(n, device="cuda")
    b = torch.randn(n, device="cuda")
    o = torch.empty_like(a)
    s = torch.cuda.current_stream()
    for blocks in blocks_list:
        lib.ompi_amd_set_tuning(b"op_max_blocks", blocks)
        for _ in range(3):
            lib.ompi_amd_op_reduce_3buff(3, 15, a.data_ptr(), b.data_ptr(), o.data_ptr(), n,
                                         ctypes.c_void_p(s.cuda_stream))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(iters):
            lib.ompi_amd_op_reduce_3buff(3, 15, a.data_ptr(), b.data_ptr(), o.data_ptr(), n,
                                         ctypes.c_void_p(s.cuda_stream))
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / iters
        print(json.dumps({"variant": os.path.basename(path), "blocks": blocks, "bytes": nbytes,
                          "ms": round(ms, 4), "GBps": round(3 * nbytes / ms / 1e6, 1)}),
              flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--one":
        run_variant(sys.argv[2], [int(x) for x in sys.argv[3].split(",")], int(sys.argv[4]),
                    int(sys.argv[5]))
        sys.exit(0)
    blocks = os.environ.get("TUNE_BLOCKS", "16777216,8192,2048")
    nbytes = int(os.environ.get("TUNE_BYTES", 1 << 30))
    for lib in sorted(os.listdir(TUNE)):
        if lib.endswith(".so"):
            subprocess.run([sys.executable, __file__, "--one", os.path.join(TUNE, lib), blocks,
                            str(nbytes), "20"], check=False)
