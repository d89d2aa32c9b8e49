#!/usr/bin/env python3
"""Per-kernel duration summary from a rocprofv3 results database (dev tool).

usage: kstats.py <run_results.db> [name-substring]
"""
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    rows = c.execute("select name, count(*), avg(end - start), min(end - start), sum(end - start) "
                     "from kernels group by name order by sum(end - start) desc").fetchall()
    for name, n, avg, mn, tot in rows:
        if sub in name:
            print(f"{n:7d}  avg {avg / 1e3:9.2f} us  min {mn / 1e3:9.2f} us  total {tot / 1e6:9.3f} ms  {name[:90]}")


if __name__ == "__main__":
    main()
