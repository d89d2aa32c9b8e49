#!/usr/bin/env python3
"""Average rocprofv3 --pmc counters per kernel from a counter_collection.csv (dev tool).

usage: sqsum.py <run_counter_collection.csv> [name-substring]
"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
sub = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    if sub in r["Kernel_Name"]:
        agg[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:24s} {sum(v) / len(v):14.0f}  (n={len(v)})")
