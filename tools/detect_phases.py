#!/usr/bin/env python3
"""Host-side phases of the initialisation's first frames (dev tool, GPU box):
over REPS fresh contexts (after one warm-up initialisation, as bench.py's
init leg), the time to create the context, and per frame the time to
enqueue (process_device returns) and to synchronize, for the FAST frame and
the KLT frames after it."""
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
    from viso_amd.shard import sequence_seed
    from viso_amd.synth import Sequence

    W, H = 1242, 375
    reps, nf = int(os.environ.get("REPS", "8")), int(os.environ.get("FRAMES", "4"))
    seq = Sequence(W, H, seed=sequence_seed(0))
    left = np.stack([seq.image(f, 0) for f in range(12)])
    d_left = torch.from_numpy(left).cuda()
    torch.cuda.synchronize()
    fb = W * H

    def ctx():
        return viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=1, batch_frames=8, max_poses=1024)

    w = ctx()
    f = 0
    while w.state != 1 and f < 12:
        w.process_device(d_left.data_ptr() + f * fb, None, 1, fb)
        w.synchronize()
        f += 1
    rows = []
    for _ in range(reps):
        t0 = time.perf_counter()
        v = ctx()
        row = [(time.perf_counter() - t0) * 1e6]
        for f in range(nf):
            t0 = time.perf_counter()
            v.process_device(d_left.data_ptr() + f * fb, None, 1, fb)
            t1 = time.perf_counter()
            v.synchronize()
            t2 = time.perf_counter()
            row += [(t1 - t0) * 1e6, (t2 - t1) * 1e6]
        rows.append(row)
        v.close()
    r = np.array(rows)
    print("per fresh context (us): create | frame f: enqueue sync")
    for x in r:
        print(f"   {x[0]:9.1f} |" + " |".join(f" {x[1 + 2 * k]:7.1f} {x[2 + 2 * k]:7.1f}" for k in range(nf)))
    m = np.median(r, 0)
    print(f"median {m[0]:9.1f} |" + " |".join(f" {m[1 + 2 * k]:7.1f} {m[2 + 2 * k]:7.1f}" for k in range(nf)))


if __name__ == "__main__":
    main()
