#!/usr/bin/env python3
"""Is the N = 1 headline kernel (3-buffer fp32 SUM, 1 GiB per buffer)
slower in the first milliseconds of a process than seconds later, and does
it depend on which buffers it runs on?  Times batches of 20 launches, event
to event on one stream, for ~`seconds` of continuous work: the bench's
buffers (torch.randn, allocated first) and a second set (random bytes,
allocated later) alternately.  One JSON line per batch."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from ompi_amd import op as mop  # noqa: E402


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
    n = (1 << 30) // 4
    g = torch.Generator(device="cuda").manual_seed(20261015)
    a = torch.randn(n, device="cuda", generator=g)
    b = torch.randn(n, device="cuda", generator=g)
    out = torch.empty_like(a)
    a2 = torch.empty(n, device="cuda").random_()
    b2 = torch.empty(n, device="cuda").random_()
    out2 = torch.empty_like(a2)
    s = torch.cuda.current_stream()
    torch.cuda.synchronize()
    t0 = time.time()
    k = 0
    while time.time() - t0 < seconds:
        for name, (x, y, o) in (("bench_buffers", (a, b, out)), ("later_buffers", (a2, b2, out2))):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(20):
                mop.reduce_local_3buff_async(x, y, o, n, mop.MPI_FLOAT, mop.MPI_SUM, stream=s)
            e1.record(s)
            e1.synchronize()
            ms = e0.elapsed_time(e1) / 20
            print(json.dumps({"batch": k, "t_s": round(time.time() - t0, 3), "buffers": name,
                              "kernel_ms": round(ms, 4),
                              "frac_of_8TBs": round(3 * n * 4 / (ms * 1e-3) / 8e12, 4)}), flush=True)
        k += 1


if __name__ == "__main__":
    main()
