#!/usr/bin/env python3
"""Per-kernel instructions per wave from a rocprofv3 --pmc run (SQ_INSTS_VALU,
SQ_INSTS_SALU, SQ_INSTS_LDS, SQ_WAVES); dev tool.  usage: pmc_insts.py DIR [DIR2]"""
import collections
import csv
import glob
import re
import sys


def load(d):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for r in csv.DictReader(open(f)):
        name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).split("(")[0]
        acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "SQ_WAVES":
            n[name] += 1
    return acc, n


for d in sys.argv[1:]:
    acc, n = load(d)
    print(d)
    for k in sorted(acc, key=lambda k: -acc[k]["SQ_INSTS_VALU"])[:8]:
        a = acc[k]
        w = max(a["SQ_WAVES"], 1)
        print(f"  {k[-55:]:55s} dispatches {n[k]:5d} waves/dispatch {w / max(n[k], 1):8.0f}  per wave: "
              f"VALU {a['SQ_INSTS_VALU'] / w:8.1f} SALU {a['SQ_INSTS_SALU'] / w:8.1f} LDS {a['SQ_INSTS_LDS'] / w:6.1f}")
