"""Per-kernel summary (calls, avg/min/max/total µs) of a rocprofv3 rocpd
database (ROCm 7.2 writes `*_results.db` by default), in the layout of
rocprofv3's kernel_stats.csv.  usage: python tools/rocpd_stats.py DB [OUT.csv]"""
import csv
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    rows = db.execute("select name, count(*), avg(end-start), min(end-start), max(end-start), "
                      "sum(end-start) from kernels group by name order by sum(end-start) desc")
    out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.writer(out)
    w.writerow(["Name", "Calls", "AverageNs", "MinNs", "MaxNs", "TotalDurationNs"])
    for name, n, avg, mn, mx, tot in rows:
        w.writerow([name, n, round(avg, 1), mn, mx, tot])


if __name__ == "__main__":
    main()
