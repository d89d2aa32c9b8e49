#!/usr/bin/env python3
"""Timeline of one device-ingest chunk from a rocprofv3 kernel-trace database
(dev tool).  Finds the background LK grid's dispatches (lk_item_kernel with a
grid of one workgroup per CU) and, for the chosen one, prints every kernel
that overlaps [its start - 100 us, its end + 100 us]: start / end relative
to the grid's start and the idle gap before each kernel on the same queue.

usage: chunk_timeline.py <results.db> [which=0] [--all]
"""
import re
import sqlite3
import sys


def main():
    db = sys.argv[1]
    which = int(sys.argv[2]) if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else 0
    full = "--all" in sys.argv
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)").fetchall()]
    qcol = next((k for k in ("queue_id", "stream_id", "queue") if k in cols), None)
    gcol = next((k for k in ("grid_size", "grid_size_x", "grid_x") if k in cols), None)
    wcol = next((k for k in ("workgroup_size", "workgroup_size_x", "workgroup_x") if k in cols), None)
    sel = "name, start, end" + (f", {qcol}" if qcol else ", 0") + (f", {gcol}" if gcol else ", 0") + \
        (f", {wcol}" if wcol else ", 0")
    rows = c.execute(f"select {sel} from kernels order by start").fetchall()
    print("columns:", cols)
    bg = [r for r in rows if "lk_item_kernel" in r[0]]
    print(f"{len(rows)} kernels, {len(bg)} lk_item_kernel dispatches (grid sizes: "
          f"{sorted(set(r[4] for r in bg))})")
    if not bg:
        return
    # the resident grid: the longest lk_item dispatches
    grids = sorted([r for r in bg if r[2] - r[1] > 200_000], key=lambda r: r[1])
    if not grids:
        grids = bg
    g = grids[min(which, len(grids) - 1)]
    t0, t1 = g[1], g[2]
    print(f"grid {which}: {(t1 - t0) / 1e3:.1f} us, grid size {g[4]}")
    last_end = {}
    prev_any = None
    for name, s, e, q, gs, ws in rows:
        if e < t0 - 100_000 or s > t1 + 100_000:
            last_end[q] = e
            continue
        m = re.search(r"(\w+_kernel|__amd_rocclr_\w+)(<[^>]*>)?", name)
        short = (m.group(1) + (m.group(2) or ""))[:34] if m else name[:34]
        gap = (s - last_end[q]) / 1e3 if q in last_end else float("nan")
        last_end[q] = e
        if full or "direct_level" not in short or prev_any is None or gap > 3.0:
            print(f"  q{q} {short:34s} {(s - t0) / 1e3:9.1f} .. {(e - t0) / 1e3:9.1f} us  "
                  f"({(e - s) / 1e3:7.1f})  gap {gap:6.1f}  grid {gs}")
        prev_any = e
    d = [r for r in rows if "direct_level" in r[0] and t0 <= r[1] <= t1]
    if d:
        durs = [(r[2] - r[1]) / 1e3 for r in d]
        gaps = [(d[i + 1][1] - d[i][2]) / 1e3 for i in range(len(d) - 1)]
        print(f"direct_level_kernel in the grid's span: {len(d)} launches, first start "
              f"{(d[0][1] - t0) / 1e3:.1f} us, last end {(d[-1][2] - t0) / 1e3:.1f} us, "
              f"avg {sum(durs) / len(durs):.2f} us, avg gap {sum(gaps) / max(len(gaps), 1):.2f} us, "
              f"tail after last direct {(t1 - d[-1][2]) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
