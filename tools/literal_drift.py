#!/usr/bin/env python3
"""Measure the drift of the oracle's tree sums against the reference's literal
running sums (tests/drift.py) on the three 200-frame cases of
tests/test_literal_drift.py and write profiles/r02_literal_drift.json."""
import concurrent.futures as cf
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from tests import test_literal_drift as t
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r02_literal_drift.json")
    with cf.ThreadPoolExecutor(len(t.CASES)) as ex:
        futs = {k: ex.submit(t.run_case, k) for k in t.CASES}
        res = {k: f.result() for k, f in futs.items()}
    summary = {}
    for k, r in res.items():
        summary[k] = {"frames": r["frames"], "poses": r["poses"],
                      "discrete_mismatches": len(r["mismatch"]),
                      "pose_max_rel_frobenius": r["pose_max_rel_frobenius"],
                      "pose_mean_rel_frobenius": r["pose_mean_rel_frobenius"],
                      "map_points_max_abs_diff": r["map_points_max_abs"],
                      "init_frames": sum(1 for s in r["states"] if s == 0),
                      "direct_nGood_min_tracking": min(g for g, s in zip(r["nGood"], r["states"]) if s == 1
                                                       and g > 0)}
    doc = {"what": "oracle tree-sum order vs literal running-sum order (src/viso.cpp:199-201, 308-310, "
                   "622-625, 727-729, 888-890), same inputs, 200 frames each",
           "compared": "state, KLT-surviving tracks (kp1/kp2), SelectMotion inlier masks, direct nGood, "
                       "LK pairs and success flags per frame; poses rel-Frobenius; map points",
           "cases": summary}
    with open(out, "w") as fh:
        json.dump(doc, fh, indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
