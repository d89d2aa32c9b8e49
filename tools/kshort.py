#!/usr/bin/env python3
"""Print a kernel_stats.csv (db2stats.py / rocprofv3 --stats) with short kernel names.

usage: kshort.py <kernel_stats.csv> [max rows]
"""
import csv
import re
import sys


def short(name):
    n = name.replace("viso::(anonymous namespace)::", "").replace("void ", "")
    n = re.sub(r"\(viso::.*$|\(unsigned char.*$|\(HIP_vector.*$|\(int.*$|\(double.*$", "", n)
    return n


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    lim = int(sys.argv[2]) if len(sys.argv) > 2 else len(rows)
    for r in rows[:lim]:
        print(f"{short(r['Name'])[:58]:58s} {r['Calls']:>6} avg {float(r['AverageNs']) / 1e3:8.2f} "
              f"min {int(r['MinNs']) / 1e3:7.2f} max {int(r['MaxNs']) / 1e3:8.2f} us {r['Percentage']:>6}%")


if __name__ == "__main__":
    main()
