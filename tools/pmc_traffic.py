#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes for the image pass.

Usage: [IMAGES=n SOURCE=... SRC_HASH=...] tools/pmc_traffic.py FETCH_DIR WRITE_DIR [OUT_JSON]
(OUT_JSON is a table of entries keyed by frame size and images per launch,
profiles/pyramid_traffic.json for bench.py)

Each directory holds a run_counter_collection.csv of one `rocprofv3 --pmc`
pass over `bench.py`.  MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reports half
the bytes of 16-byte-per-lane streaming reads on gfx950; other widths are
uncalibrated.  The level-1 kernel reads 8 bytes per lane, the tail kernel
(levels 2-3) 16 bytes.  The raw
FETCH_SIZE of the level-0 pass of a 100-image chunk is below the 46.6 MB of
level 0 it must read at least once (round 1: 39.9 MB for the first streaming
kernel), while the doubled value lies between that and the bytes of the
128-byte lines its loads touch, so the same factor 2 is applied (FETCH_SCALE
overrides; the per-launch raw values are printed for the check).  WRITE_SIZE (KB) is
taken as is.  The per-chunk traffic of the image pass is the sum over its
launches (LAUNCHES, default 2: level 1 + tail; 3 for the round-1 per-level
form), averaged over the full-size chunks.
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
    f = os.path.join(path, "run_counter_collection.csv")
    if not os.path.exists(f):
        f = next(os.path.join(d, x) for d, _, xs in os.walk(path) for x in xs if x.endswith("counter_collection.csv"))
    for r in csv.DictReader(open(f)):
        if ("pyr_down_" not in r["Kernel_Name"] and "pyr_tail_" not in r["Kernel_Name"]) or \
                r["Counter_Name"] != counter:
            continue
        d = int(r["Dispatch_Id"])
        vals[d] += float(r["Counter_Value"])
        grid[d] = (int(r["Grid_Size"]), r["Kernel_Name"])
    return vals, grid


LAUNCHES = int(os.environ.get("LAUNCHES", "2"))


def big_groups(vals, grid):
    """Dispatch-id groups (the launches of one chunk) of the full-size chunks."""
    ids = sorted(vals)
    groups = [ids[i:i + LAUNCHES] for i in range(0, len(ids) - len(ids) % LAUNCHES, LAUNCHES)]
    big = max(grid[g[0]][0] for g in groups)
    return [g for g in groups if grid[g[0]][0] == big]


def per_level(vals, grid):
    """Mean raw counter value (KB) per launch of each level over the full-size chunks."""
    gs = big_groups(vals, grid)
    return [round(sum(vals[g[k]] for g in gs) / len(gs), 1) for k in range(LAUNCHES)]


def main():
    fdir, wdir = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else None
    f, fg = per_dispatch(fdir, "FETCH_SIZE")
    w, wg = per_dispatch(wdir, "WRITE_SIZE")

    def chunks(vals, grid):
        return [sum(vals[d] for d in g) for g in big_groups(vals, grid)]

    fc, wc = chunks(f, fg), chunks(w, wg)
    scale = float(os.environ.get("FETCH_SCALE", "2"))
    fetch = scale * 1024 * sum(fc) / len(fc)
    write = 1024.0 * sum(wc) / len(wc)
    imgs = int(os.environ.get("IMAGES", "100"))
    res = {"width": int(os.environ.get("WIDTH", "1242")), "height": int(os.environ.get("HEIGHT", "375")),
           "images_per_launch": imgs, "source": os.environ.get("SOURCE", fdir),
           "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
           "traffic_bytes_per_launch": fetch + write, "chunks": len(fc),
           "fetch_scale": scale,
           "note": f"FETCH_SIZE x fetch_scale + WRITE_SIZE (KB -> bytes) summed over the {LAUNCHES} "
                   f"image-pass launches of one {imgs}-image chunk (tools/pmc_traffic.py)",
           "raw_fetch_kb_per_launch": per_level(f, fg), "raw_write_kb_per_launch": per_level(w, wg),
           # the library the passes ran (viso_version "src:"): bench.py uses
           # an entry only for the library it loads
           "src": os.environ.get("SRC_HASH", "")}
    print(json.dumps(res, indent=1))
    if out:
        # a table of entries (bench.py pyramid_traffic looks up its own size
        # and chunk): replace the entry of this size / chunk, keep the others
        table = {"entries": []}
        base = os.environ.get("BASE_TABLE", out)
        if os.path.exists(base):
            old = json.load(open(base))
            table = old if "entries" in old else table
        table["entries"] = [e for e in table["entries"]
                            if (e["width"], e["height"], e["images_per_launch"]) !=
                            (res["width"], res["height"], res["images_per_launch"])] + [res]
        json.dump(table, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
