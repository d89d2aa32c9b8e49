#!/usr/bin/env python3
"""Stereo VO (SVO) throughput (dev tool, GPU box): N synthetic 1242x375 pairs
resident in HBM through viso_svo_process_device; prints pairs/s and the last
pair's stats.  Run under rocprofv3 --kernel-trace --stats for per-kernel times."""
from __future__ import annotations

import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    from viso_amd import svo
    from viso_amd.synth import Sequence

    W, H = int(os.environ.get("WIDTH", "1242")), int(os.environ.get("HEIGHT", "375"))
    n = int(os.environ.get("PAIRS", "100"))
    seq = Sequence(W, H, seed=0)
    left = np.stack([seq.image(f, 0) for f in range(n)])
    right = np.stack([seq.image(f, 1) for f in range(n)])
    dl = torch.from_numpy(left).cuda()
    dr = torch.from_numpy(right).cuda()
    p = svo.default_params(W, H, *seq.K, seq.p.baseline)
    for k in ("gn_iters", "ransac_iters"):
        if k.upper() in os.environ:
            setattr(p, k, int(os.environ[k.upper()]))
    vo = svo.VisualOdometryStereo(p)
    vo.process_device(dl.data_ptr(), dr.data_ptr(), 10, W * H)  # warm-up
    vo.synchronize()
    vo2 = svo.VisualOdometryStereo(p)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    vo2.process_device(dl.data_ptr(), dr.data_ptr(), n, W * H)
    vo2.synchronize()
    dt = time.perf_counter() - t0
    print(f"pairs {n}  {n / dt:.1f} pairs/s  {dt / n * 1e6:.1f} us/pair  stats {vo2.stats().tolist()}")


if __name__ == "__main__":
    main()
