#!/usr/bin/env python3
"""Write a rocprofv3 `--stats`-style kernel_stats.csv from a rocprofv3 results database.

usage: db2stats.py <run_results.db> <out.csv>
(rocprofv3 on this image writes its results as a rocpd SQLite database by default.)
"""
import csv
import math
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    rows = c.execute("select name, end - start from kernels").fetchall()
    agg = {}
    for name, d in rows:
        agg.setdefault(name, []).append(d)
    total = sum(sum(v) for v in agg.values())
    with open(sys.argv[2], "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
            n, s = len(v), sum(v)
            avg = s / n
            sd = math.sqrt(sum((x - avg) ** 2 for x in v) / n)
            w.writerow([name, n, s, round(avg, 3), round(100.0 * s / total, 2), min(v), max(v), round(sd, 3)])


if __name__ == "__main__":
    main()
