#!/usr/bin/env python3
"""Algorithmic work of the stereo-VO kernels on tools/bench_svo.py's
workload (the 100-pair batch its rocprofv3 --pmc passes measure; the PMC
summary is profiles/rNN_gn_svo_pmc.json), from the CPU spec
(oracle/oracle_svo.cpp, single thread; deterministic):

* svo_circle_kernel: the candidates whose 32-byte SAD the spec evaluates in
  the four chained best-match searches of every feature (oracle_svo_sad_evals)
  over pairs 1..99 of the batch;
* svo_detect_kernel: per image (left and right of every pair) and interior
  response pixel, the two 5x5 filters' taps (blob 25, corner 16) and the four
  classes' (2n+1)^2 NMS windows evaluated separably (2 x 2n compares each).

Writes profiles/svo_algorithmic_ops.json; bench.py's matching_pass_hbm
divides these by the PMC pass's kernel durations and the VALU peak.
usage: python tools/svo_ops.py [PAIRS=100]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from tests import oracle_lib
    from viso_amd.synth import Sequence
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    W, H = 1242, 375
    seq = Sequence(W, H, seed=0)  # tools/bench_svo.py's sequence
    p = oracle_lib.svo_params(W, H, *seq.K, seq.p.baseline)
    lib = oracle_lib.load()
    S = oracle_lib.SvoSequence(p)
    lib.oracle_svo_sad_evals(1)
    feats = []
    for f in range(n):
        S.process(seq.image(f, 0), seq.image(f, 1))
        feats.append(S.stats[0] + S.stats[1])
    sad = int(lib.oracle_svo_sad_evals(1))
    # the matching pass's inputs read once: the feature sets of pairs k and
    # k - 1 (u, v, class as 3 x 4 bytes + the 32-byte descriptor each)
    in_bytes = sum(44 * (feats[k] + feats[k - 1]) for k in range(1, n))
    nms = p.nms_n
    px = (W - 4) * (H - 4)  # response domain: x in [2, w-2), y in [2, h-2)
    out = {"workload": f"tools/bench_svo.py: synthetic {W}x{H} stereo sequence seed 0, pairs 0-{n - 1} in one batch",
           "pairs": n,
           "sad_candidates": sad, "sad_bytes": 32 * sad,
           "sad_basis": "candidates whose 32-byte SAD the spec evaluates (same class, search window; four chained "
                        "best-match searches per feature; oracle/oracle_svo.cpp best_match) over pairs 1..n-1",
           "circle_input_bytes": int(in_bytes),
           "circle_input_basis": "feature sets of pairs k and k - 1 read once per pair k = 1..n-1: "
                                 "(u, v, class) 12 B + descriptor 32 B per feature",
           "detect_images": 2 * n, "detect_pixels_per_image": px,
           "detect_ops": 2 * n * px * (25 + 16 + 4 * 2 * (2 * nms)),
           "detect_basis": f"per image and response pixel: 25 + 16 filter taps and 4 classes x 2 x {2 * nms} "
                           "separable NMS compares"}
    path = os.path.join(ROOT, "profiles", "svo_algorithmic_ops.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
