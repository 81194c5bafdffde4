#!/usr/bin/env python3
"""Op kernel on displaced operands: 3-buffer SUM over
256 MiB per buffer with the three operands at byte offsets (x, y, dst)
inside their 16-B vectors — aligned, all displaced alike (head-peel + 16-B
vectors) and displaced differently (element path) — fp32 and fp64.  One JSON
line per point: HIP-event kernel time on the launch stream (median of 5
batches), algorithmic GB/s = 3 * bytes / t, fraction of 8 TB/s."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from ompi_amd import op as mop  # noqa: E402
from op_sweep import time_op  # noqa: E402

PEAK = 8000.0


def main():
    nbytes = int(os.environ.get("PROBE_BYTES", 256 << 20))
    a = torch.empty(nbytes + 64, dtype=torch.uint8, device="cuda").random_()
    b = torch.empty(nbytes + 64, dtype=torch.uint8, device="cuda").random_()
    o = torch.empty(nbytes + 64, dtype=torch.uint8, device="cuda")
    for dt in (mop.MPI_FLOAT, mop.MPI_DOUBLE):
        e = dt.extent
        for offs in ((0, 0, 0), (e, e, e), (3 * e if e < 8 else e, 3 * e if e < 8 else e, 3 * e if e < 8 else e),
                     (e, 0, e), (0, e, 0), (e, 2 * e if e < 8 else 0, 0)):
            n = nbytes // e - 4
            pa, pb, po = a.data_ptr() + offs[0], b.data_ptr() + offs[1], o.data_ptr() + offs[2]
            ms = time_op(lambda s: mop.reduce_local_3buff_async(pa, pb, po, n, dt, mop.MPI_SUM,
                                                                stream=s), 20)
            gbs = 3 * n * e / (ms * 1e-3) / 1e9
            print(json.dumps({"type": dt.name, "offsets": offs, "bytes": n * e, "ms": round(ms, 5),
                              "GBps": round(gbs, 1), "frac_of_8TBps": round(gbs / PEAK, 3),
                              "path": "vector" if len(set(o_ % 16 for o_ in offs)) == 1 else "element"}),
                  flush=True)


if __name__ == "__main__":
    main()
