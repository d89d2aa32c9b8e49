#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes for the image pass.

Usage: tools/pmc_traffic.py FETCH_DIR WRITE_DIR [OUT_JSON]

Each directory holds a run_counter_collection.csv of one `rocprofv3 --pmc`
pass over `bench.py`.  MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reports half
the bytes of 16-byte-per-lane streaming reads on gfx950; other widths are
uncalibrated.  pyr_down_stream_kernel reads 8 bytes per lane.  Its raw
FETCH_SIZE for a 100-image chunk (39.9 MB for the level-0 pass) is below the
46.6 MB of level 0 it must read at least once, while the doubled value (79.8
MB) lies between that and the 87.6 MB of 128-byte lines its loads touch, so
the same factor 2 is applied (FETCH_SCALE overrides).  WRITE_SIZE (KB) is
taken as is.  The per-chunk traffic of the image pass is the sum over its
three launches, averaged over the full-size chunks.
"""
from __future__ import annotations

import collections
import csv
import json
import os
import sys


def per_dispatch(path, counter):
    vals = collections.defaultdict(float)
    grid = {}
    for r in csv.DictReader(open(os.path.join(path, "run_counter_collection.csv"))):
        if "pyr_down_stream" not in r["Kernel_Name"] or r["Counter_Name"] != counter:
            continue
        d = int(r["Dispatch_Id"])
        vals[d] += float(r["Counter_Value"])
        grid[d] = (int(r["Grid_Size"]), r["Kernel_Name"])
    return vals, grid


def main():
    fdir, wdir = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else None
    f, fg = per_dispatch(fdir, "FETCH_SIZE")
    w, wg = per_dispatch(wdir, "WRITE_SIZE")

    def chunks(vals, grid):
        # group consecutive dispatches in threes (L1, L2, L3 of one chunk)
        ids = sorted(vals)
        groups = [ids[i:i + 3] for i in range(0, len(ids) - len(ids) % 3, 3)]
        sums = [(sum(vals[d] for d in g), grid[g[0]][0]) for g in groups]
        big = max(s[1] for s in sums)
        return [s[0] for s in sums if s[1] == big]

    fc, wc = chunks(f, fg), chunks(w, wg)
    scale = float(os.environ.get("FETCH_SCALE", "2"))
    fetch = scale * 1024 * sum(fc) / len(fc)
    write = 1024.0 * sum(wc) / len(wc)
    res = {"width": int(os.environ.get("WIDTH", "1242")), "height": int(os.environ.get("HEIGHT", "375")),
           "images_per_launch": 100,
           "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
           "traffic_bytes_per_launch": fetch + write, "chunks": len(fc),
           "fetch_scale": scale,
           "note": "FETCH_SIZE x fetch_scale + WRITE_SIZE (KB -> bytes) summed over the three "
                   "pyr_down_stream_kernel launches of one 100-image chunk (tools/pmc_traffic.py)"}
    print(json.dumps(res, indent=1))
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
