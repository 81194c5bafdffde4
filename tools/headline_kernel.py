"""The N=1 headline kernel's launches from a rocprofv3 kernel trace (the
bench's timed op_vec_kernel launches at the headline grid), as the JSON
committed beside the bench line under profiles/.

    python tools/headline_kernel.py <kernel_trace.csv> [out.json]
"""
import csv
import json
import statistics
import sys

KERNEL = "op_vec_kernel<float,3,true>"
ALG_BYTES = 3 * (1 << 30)  # two 1 GiB inputs read, one 1 GiB result written


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    durs, grids = [], {}
    for r in rows:
        if KERNEL not in r["Kernel_Name"].replace(" ", "").replace("ompi_amd::", ""):
            continue
        g = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
        grids.setdefault(g, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    g, durs = max(grids.items(), key=lambda kv: (kv[0], len(kv[1])))
    avg = statistics.mean(durs)
    out = {"kernel": KERNEL, "grid_threads": g, "launches": len(durs), "avg_ns": avg,
           "min_ns": min(durs), "max_ns": max(durs), "algorithmic_bytes": ALG_BYTES,
           "achieved_GBps": ALG_BYTES / avg, "frac_of_8TBs": ALG_BYTES / avg / 8000.0,
           "source": "rocprofv3 --kernel-trace of python3 bench.py --no-cpu-baseline, "
                     "headline-grid launches only"}
    text = json.dumps(out)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
