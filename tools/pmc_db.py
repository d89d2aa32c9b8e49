#!/usr/bin/env python3
"""Per-kernel averages of the PMC counters in a rocprofv3 results database.

usage: tools/pmc_db.py RUN_RESULTS_DB [KERNEL_SUBSTRING]
Prints, per kernel (name filter optional): dispatches, mean duration (ns) and
the mean per-dispatch value of every counter collected (summed over
instances).
"""
import collections
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    q = """select ks.kernel_name, kd.id, kd.end - kd.start, ip.name, pe.value
           from rocpd_pmc_event pe
           join rocpd_info_pmc ip on pe.pmc_id = ip.id
           join rocpd_kernel_dispatch kd on pe.event_id = kd.event_id
           join kernel_symbols ks on kd.kernel_id = ks.id"""
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    names = {}
    for kname, did, d, pname, v in c.execute(q):
        if filt and filt not in kname:
            continue
        per[did][pname] += v
        dur[did] = d
        names[did] = kname
    agg = collections.defaultdict(list)
    for did in per:
        agg[names[did]].append(did)
    for k, ids in agg.items():
        print(f"{k[:90]}  dispatches {len(ids)}  mean ns {sum(dur[i] for i in ids) / len(ids):.0f}")
        keys = sorted({p for i in ids for p in per[i]})
        for p in keys:
            print(f"    {p:28s} {sum(per[i][p] for i in ids) / len(ids):.4g}")


if __name__ == "__main__":
    main()
