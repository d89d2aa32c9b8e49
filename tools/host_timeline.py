#!/usr/bin/env python3
"""Timeline of the host-frame path (viso_process_frame per frame) from a
rocprofv3 --kernel-trace --memory-copy-trace database (dev tool): for frames
[F, F + N) of the run (the k-th direct_level_kernel L(3) launch starts frame
k), every kernel and copy with its queue, start / end relative to frame F's
L(3) start, and per frame the chain (L(3) start -> L(0) end), the gap before
its L(3), and when its pyramid and upload ended.

usage: host_timeline.py <results.db> [F=20] [N=4]"""
import re
import sqlite3
import sys


def main():
    db = sys.argv[1]
    F = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    N = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    c = sqlite3.connect(db)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table', 'view')")]
    kcols = [r[1] for r in c.execute("pragma table_info(kernels)").fetchall()]
    qcol = next((k for k in ("queue_id", "stream_id", "queue") if k in kcols), "0")
    ev = [(r[1], r[2], f"q{r[3]}", r[0]) for r in c.execute(f"select name, start, end, {qcol} from kernels")]
    mt = next((t for t in tabs if "memory_cop" in t), None)
    if mt:
        mcols = [r[1] for r in c.execute(f"pragma table_info({mt})").fetchall()]
        nm = next((k for k in ("name", "operation", "kind") if k in mcols), None)
        sz = next((k for k in ("size", "bytes") if k in mcols), None)
        q = next((k for k in ("queue_id", "stream_id") if k in mcols), None)
        for r in c.execute(f"select start, end, {q or 0}, {nm or repr('copy')}, {sz or 0} from {mt}"):
            ev.append((r[0], r[1], f"c{r[2]}", f"COPY {r[3]} {r[4]} B"))
    ev.sort()
    d3 = [e for e in ev if "direct_level_kernel" in e[3]]
    # a frame's L(3): the direct launch after a non-direct event or the first of four
    starts = [i for i, e in enumerate(d3) if i % 4 == 0]
    if len(starts) < F + N + 1:
        print(f"only {len(starts)} frames")
        return
    t0 = d3[starts[F]][0]
    t1 = d3[starts[F + N]][0]
    print(f"tables: {tabs}")
    for s, e, q, name in ev:
        if e < t0 - 150_000 or s > t1:
            continue
        m = re.search(r"(\w+_kernel|__amd_rocclr_\w+|COPY.*)(<[^>]*>)?", name)
        short = ((m.group(1) + (m.group(2) or "")) if m else name)[:40]
        print(f"  {q:>4s} {short:40s} {(s - t0) / 1e3:9.1f} .. {(e - t0) / 1e3:9.1f} us ({(e - s) / 1e3:6.1f})")
    for k in range(F, F + N):
        a, b = d3[starts[k]], d3[starts[k] + 3]
        prev_end = d3[starts[k] - 1][1]
        print(f"frame {k}: chain {(b[1] - a[0]) / 1e3:.1f} us, gap before L3 {(a[0] - prev_end) / 1e3:.1f} us, "
              f"period {(d3[starts[k + 1]][0] - a[0]) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
