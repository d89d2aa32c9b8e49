#!/usr/bin/env python3
"""Per-kernel mean of every PMC counter in rocprofv3 --pmc csv directories
(dev tool): tools/pmc_summary.py DIR [DIR ...]"""
import collections
import csv
import glob
import os
import re
import sys


def short(name):
    m = re.search(r"(\w+_kernel)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def main():
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"])
                tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
    for k, c in sorted(tot.items()):
        print(k)
        for name, v in sorted(c.items()):
            n = len(disp[(k, name)])
            print(f"   {name:24s} {v / max(n, 1):14.1f}  (per dispatch, {n} dispatches)")


if __name__ == "__main__":
    main()
