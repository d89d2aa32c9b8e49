#!/usr/bin/env python3
"""Block timeline of the pyramid tail launch (dev tool, GPU box).

Loads the instrumented library (VISO_VARIANT=probe), builds the pyramids of
IMAGES synthetic 1242x375 images a few times and prints, for the last
pyr_tail_kernel launch: phase durations per workgroup (phase 1 = level-1
rows staged from HBM, phase 2 = level 2, phase 3 = level 3 including the
drain of its stores), start spread, workgroups per CU and the number of live
workgroups over time.
"""
from __future__ import annotations

import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("VISO_LIB", os.path.join(ROOT, "viso_amd", "libviso_amd_probe.so"))


def main():
    import numpy as np
    import torch

    import viso_amd
    from viso_amd import _lib
    from viso_amd.synth import Sequence

    W, H = 1242, 375
    n = int(os.environ.get("IMAGES", "50"))
    seq = Sequence(W, H, seed=0)
    frames = np.stack([seq.image(f % 16, f % 2) for f in range(n)])
    d = torch.from_numpy(frames).cuda()
    v = viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=0, batch_frames=n)
    for _ in range(5):
        v.process_device(d.data_ptr(), None, n, W * H)
    v.synchronize()
    lib = _lib.load()
    lib.viso_debug_pyr_timeline.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dims, _ = viso_amd.pyramid_dims(W, H)
    h3 = dims[3][1]
    band = max(2, -(-h3 // max(1, 512 // n)))  # image.hip pf_plan (uncapped at 1242 wide)
    nb = -(-h3 // band)
    blocks = nb * n
    buf = np.zeros((8192, 5), np.uint64)
    assert lib.viso_debug_pyr_timeline(buf.ctypes.data, 8192) == 0
    tl = buf[:blocks].astype(np.int64)
    t0 = tl[:, 0].min()
    us = lambda c: (tl[:, c] - t0) * 10 / 1000.0  # noqa: E731  (100 MHz ticks)
    st, p1, p2, en = us(0), us(1), us(2), us(3)
    pct = lambda x: np.round(np.percentile(x, [5, 25, 50, 75, 95, 100]), 2)  # noqa: E731
    print(f"blocks {blocks}  span {en.max():.2f} us  start spread {st.max():.2f} us")
    print("phase 1 us (5/25/50/75/95/max):", pct(p1 - st))
    print("phase 2 us:", pct(p2 - p1))
    print("phase 3 us:", pct(en - p2))
    print("total us:", pct(en - st))
    print("start us:", pct(st))
    hw, xcc = tl[:, 4] & 0xFFFFFFFF, (tl[:, 4] >> 32) & 0xF
    cu = (hw >> 8) & 0xF
    sh_ = (hw >> 12) & 1
    se = (hw >> 13) & 0x7
    cu_key = xcc * 1000 + se * 100 + sh_ * 16 + cu
    ucu, cnt = np.unique(cu_key, return_counts=True)
    print(f"distinct CUs {len(ucu)}  blocks per CU min/median/max {cnt.min()}/{int(np.median(cnt))}/{cnt.max()}")
    img = np.arange(blocks) // nb
    same = [len(np.unique(xcc[img == i])) for i in range(n)]
    print("XCDs per image (max):", max(same))
    for t in np.arange(0, en.max() + 0.5, 1.0):
        live = int(np.sum((st <= t) & (en > t)))
        print(f"  t={t:5.1f} us live blocks {live}")


if __name__ == "__main__":
    main()
