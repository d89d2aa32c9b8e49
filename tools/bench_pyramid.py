#!/usr/bin/env python3
"""Pyramid microbenchmark (dev tool, GPU box): the batched image pass alone.

Builds the 4-level pyramid of N synthetic 1242x375 images resident in HBM
with the product kernel (viso_process_frames_device would interleave it with
tracking; here it runs back to back) and reports the HIP-event time per
launch and the algorithmic bandwidth (level-0 read + levels 1..3 written).
Run under rocprofv3 for kernel durations / PMC counters.
"""
from __future__ import annotations

import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    import viso_amd
    from viso_amd.synth import Sequence

    W, H = 1242, 375
    n = int(os.environ.get("IMAGES", "100"))
    reps = int(os.environ.get("REPS", "20"))
    seq = Sequence(W, H, seed=0)
    frames = np.stack([seq.image(f % 16, f % 2) for f in range(n)])
    d = torch.from_numpy(frames).cuda()
    v = viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=0, batch_frames=n)
    # the initialisation state machine runs per frame; to time only the
    # pyramid use the per-launch kernel timer
    v.ctx.timing_enable(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        v.process_device(d.data_ptr(), None, n, W * H)
    v.synchronize()
    wall = time.perf_counter() - t0
    launches, ms = v.ctx.timing("pyramid")
    dims, _ = viso_amd.pyramid_dims(W, H)
    algo = sum(w * h for w, h in dims)
    per = ms / max(launches, 1)
    print(f"images/launch {n}  launches {launches}  avg {per * 1e3:.1f} us  "
          f"algorithmic {algo * n / (per * 1e-3) / 1e9:.1f} GB/s  wall/rep {wall / reps * 1e3:.2f} ms")


if __name__ == "__main__":
    main()
