#!/usr/bin/env python3
"""Kernel timeline of the initialisation's RANSAC frames from a rocprofv3
kernel-trace database (dev tool): for each h_hyp_kernel dispatch (a frame
past the 2D-2D gate), every kernel from the klt_kernel before it to the
select kernel after it, with start / end relative to that KLT launch, the
queue and the idle gap before it on its queue.

usage: init_timeline.py <results.db> [max_frames=4]
"""
import re
import sqlite3
import sys


def short(name):
    m = re.search(r"(\w+_kernel|__amd_rocclr_\w+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or ""))[:36] if m else name[:36]


def main():
    c = sqlite3.connect(sys.argv[1])
    cap = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    rows = c.execute("select name, start, end, queue_id from kernels order by start").fetchall()
    rows = [(short(n), s, e, q) for n, s, e, q in rows]
    hyp = [i for i, r in enumerate(rows) if r[0].startswith("h_hyp_kernel")]
    for fi, h in enumerate(hyp[:cap]):
        k = h
        while k > 0 and not rows[k][0].startswith("klt_kernel"):
            k -= 1
        e = h
        while e < len(rows) - 1 and not rows[e][0].startswith("select_finish") and \
                not rows[e][0].startswith("select_output"):
            e += 1
        t0 = rows[k][1]
        print(f"RANSAC frame {fi}: klt .. select = {(rows[e][2] - t0) / 1e3:.1f} us")
        last = {}
        for n, s, en, q in rows[k:e + 1]:
            gap = (s - last[q]) / 1e3 if q in last else float("nan")
            last[q] = en
            print(f"  q{q} {n:36s} {(s - t0) / 1e3:8.1f} .. {(en - t0) / 1e3:8.1f}  ({(en - s) / 1e3:6.1f})  gap {gap:6.1f}")


if __name__ == "__main__":
    main()
