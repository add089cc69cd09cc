"""Turn a rocprofv3 rocpd database (`--kernel-trace` without `--output-format csv`), or a
`*_kernel_trace.csv`, into the kernel_stats.csv layout `--stats` writes: Name, Calls,
TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs, StdDev, one row per kernel name, ordered
by total time.

usage: python tools/rocpd_stats.py RUN_results.db|RUN_kernel_trace.csv OUT.csv
"""
import csv
import math
import sqlite3
import sys
from collections import defaultdict


def stats(src):
    dur = defaultdict(list)
    if src.endswith(".csv"):
        for r in csv.DictReader(open(src)):
            dur[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    else:
        for name, d in sqlite3.connect(src).execute("select name, duration from kernels"):
            dur[name].append(int(d))
    total = sum(sum(v) for v in dur.values()) or 1
    rows = []
    for name, v in dur.items():
        n, s = len(v), sum(v)
        mean = s / n
        sd = math.sqrt(sum((x - mean) ** 2 for x in v) / n)
        rows.append([name, n, s, f"{mean:.6f}", f"{100.0 * s / total:.2f}", min(v), max(v), f"{sd:.6f}"])
    rows.sort(key=lambda r: -r[2])
    return rows


def main(db, out):
    with open(out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_ALL)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        w.writerows(stats(db))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
