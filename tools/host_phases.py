#!/usr/bin/env python3
"""Host-side phases of the driver's timed region (dev tool, GPU box): for
one 20-frame chunk (bench.py --steps 20 --warmup 5), the time to enqueue
(process_device returns), to synchronize, and to read the poses, over REPS
chunks."""
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
    warm, steps, reps = 5, int(os.environ.get("STEPS", "20")), int(os.environ.get("REPS", "8"))
    seq = Sequence(W, H, seed=0)
    n = warm + steps * reps
    left = np.stack([seq.image(f, 0) for f in range(n)])
    right = np.stack([seq.image(f, 1) for f in range(n)])
    d_left = torch.from_numpy(left).cuda()
    d_right = torch.from_numpy(right).cuda()
    v = viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=1, batch_frames=128, max_poses=4096)
    v.set_stereo(seq.p.baseline, 128, 1)
    v.process_device(d_left.data_ptr(), d_right.data_ptr(), warm, W * H)
    v.synchronize()
    rows = []
    for rep in range(reps):
        f0 = warm + rep * steps
        torch.cuda.synchronize()
        v.synchronize()
        t0 = time.perf_counter()
        v.process_device(d_left.data_ptr() + f0 * W * H, d_right.data_ptr() + f0 * W * H, steps, W * H)
        t1 = time.perf_counter()
        v.synchronize()
        t2 = time.perf_counter()
        p = v.poses
        t3 = time.perf_counter()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        rows.append([(t1 - t0) * 1e6, (t2 - t1) * 1e6, (t3 - t2) * 1e6, (t4 - t3) * 1e6, (t4 - t0) * 1e6])
    r = np.array(rows)
    print("per chunk (us): enqueue / sync / poses / torch sync / total")
    for x in r:
        print("   " + " ".join(f"{y:8.1f}" for y in x))
    print("median " + " ".join(f"{y:8.1f}" for y in np.median(r, 0)), f"({len(p)} poses)")


if __name__ == "__main__":
    main()
