#!/usr/bin/env python3
"""Host enqueue time vs GPU time of batched ingest (dev tool, GPU box): is the
per-frame path host-bound?  Times viso_process_frames_device's return (host
enqueue of a chunk) and the chunk's completion, per chunk size."""
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
    seq = Sequence(W, H, seed=0)
    n = 20 + 3 * 128
    left = np.stack([seq.image(f, 0) for f in range(n)])
    right = np.stack([seq.image(f, 1) for f in range(n)])
    dl = torch.from_numpy(left).cuda()
    dr = torch.from_numpy(right).cuda()
    fb = W * H
    for batch in (20, 128):
        v = viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=1, batch_frames=128, max_poses=4096)
        v.set_stereo(seq.p.baseline, 128, 1)
        v.process_device(dl.data_ptr(), dr.data_ptr(), 20, fb)
        v.synchronize()
        f = 20
        for rep in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            v.process_device(dl.data_ptr() + f * fb, dr.data_ptr() + f * fb, batch, fb)
            t1 = time.perf_counter()
            v.synchronize()
            t2 = time.perf_counter()
            f += batch
            print(f"batch {batch}: enqueue {1e6 * (t1 - t0) / batch:.1f} us/frame, "
                  f"complete {1e6 * (t2 - t0) / batch:.1f} us/frame", flush=True)


if __name__ == "__main__":
    main()
