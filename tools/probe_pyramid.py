#!/usr/bin/env python3
"""Wave timeline of the level-1 pyrDown launch (dev tool, GPU box).

Loads the instrumented library (VISO_VARIANT=probe), builds the pyramids of
100 synthetic 1242x375 images a few times and prints, for the last level-1
launch: the span, per-wave durations, start-time spread, waves per CU and the
number of live waves over time.
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

    W, H, n = 1242, 375, int(os.environ.get("IMAGES", "100"))
    seq = Sequence(W, H, seed=0)
    frames = np.stack([seq.image(f % 16, f % 2) for f in range(n)])
    d = torch.from_numpy(frames).cuda()
    v = viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=0, batch_frames=n)
    for _ in range(5):
        v.process_device(d.data_ptr(), None, n, W * H)
    v.synchronize()
    lib = _lib.load()
    lib.viso_debug_pyr_timeline.argtypes = [ctypes.c_void_p, ctypes.c_int]
    bh = 4 if n <= 32 else 8  # image.hip kSkSmallBatch / kSkBHs / kSkBH1
    bands = -(-(H // 2) // bh)
    upi = 3 * bands
    units = min(upi * n, 8192)
    buf = np.zeros((8192, 5), np.uint64)
    assert lib.viso_debug_pyr_timeline(buf.ctypes.data, 8192) == 0
    tl = buf[:units].astype(np.int64)
    t0 = tl[:, 0].min()
    st = (tl[:, 0] - t0) * 10 / 1000.0  # us
    en = (tl[:, 1] - t0) * 10 / 1000.0
    dur = en - st
    ld = (tl[:, 4] - t0) * 10 / 1000.0 - st
    print("load wait us percentiles 5/25/50/75/95/max:",
          np.round(np.percentile(ld, [5, 25, 50, 75, 95, 100]), 2))
    print("compute+store us percentiles 5/25/50/75/95/max:",
          np.round(np.percentile(dur - ld, [5, 25, 50, 75, 95, 100]), 2))
    hw, xcc = tl[:, 2], tl[:, 3]
    cu = (hw >> 8) & 0xF
    sh_ = (hw >> 12) & 1
    se = (hw >> 13) & 0x7
    simd = (hw >> 4) & 3
    cu_key = (xcc & 0xF) * 1000 + se * 100 + sh_ * 16 + cu
    print(f"waves {units}  span {en.max():.2f} us  start spread {st.max():.2f} us")
    print("duration us percentiles 5/25/50/75/95/max:",
          np.round(np.percentile(dur, [5, 25, 50, 75, 95, 100]), 2))
    print("start us percentiles 5/25/50/75/95/max:",
          np.round(np.percentile(st, [5, 25, 50, 75, 95, 100]), 2))
    ucu, cnt = np.unique(cu_key, return_counts=True)
    print(f"distinct CUs {len(ucu)}  waves per CU min/median/max {cnt.min()}/{int(np.median(cnt))}/{cnt.max()}")
    print("distinct XCC:", np.unique(xcc & 0xF))
    for t in np.arange(0, en.max() + 0.5, 1.0):
        live = int(np.sum((st <= t) & (en > t)))
        print(f"  t={t:5.1f} us live waves {live}")
    # per XCC (HW_REG XCC_ID low bits): a late group on some XCCs would be a
    # clock offset between the XCDs' realtime counters, not a dispatch stall
    for x in np.unique(xcc & 0xF):
        m = (xcc & 0xF) == x
        print(f"xcc {x:2d}: waves {m.sum():5d}  start min/med/max {st[m].min():6.2f} {np.median(st[m]):6.2f} "
              f"{st[m].max():6.2f}  end max {en[m].max():6.2f}")
    late = st > 0.5 * st.max()
    if late.any():
        img = np.arange(units) // upi
        print("late waves:", int(late.sum()), "images", np.unique(img[late])[:40])
    # by strip (unit // bands): edge strips vs interior
    unit = np.arange(units) % upi
    strip = unit // bands
    for s in range(3):
        print(f"strip {s}: median duration {np.median(dur[strip == s]):.2f} us")


if __name__ == "__main__":
    main()
