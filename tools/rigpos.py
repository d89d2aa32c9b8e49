#!/usr/bin/env python3
"""Per-position (L3..L0 or F) rig_level_kernel durations from a rocprofv3 results db.
usage: rigpos.py <run_results.db> <launches per timestep>"""
import sqlite3, sys
import numpy as np
c = sqlite3.connect(sys.argv[1])
per = int(sys.argv[2])
rows = c.execute("select name, start, end from kernels order by start").fetchall()
for fast in ("<false>", "<true>"):
    d = np.array([e - s for n, s, e in rows if "rig_level_kernel" + fast in n]) / 1e3
    print(fast, len(d), "launches")
    # sessions: the bench runs the warmup + timed call; align on whole timesteps from the start
    m = (len(d) // per) * per
    body = d[:m]
    for p in range(per):
        x = body[p::per]
        print(f"  pos {p}: mean {x.mean():6.1f} std {x.std():5.1f} min {x.min():6.1f} max {x.max():6.1f} us")
