#!/usr/bin/env python3
"""Dev timing of the FAST stage (viso_fast: fast_tile_kernel + fast_order_kernel)
at 1242x375 and 1920x1080 (synthetic frames); HIP-event region per call and
corner counts.  Run under rocprofv3 --kernel-trace --stats for kernel times.
VISO_LIB selects a variant library."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import viso_amd  # noqa: E402
from viso_amd.synth import Sequence  # noqa: E402

for (w, h, kw) in [(1242, 375, {}), (1920, 1080, {"block_m": 0.35})]:
    img = Sequence(w, h, seed=0, **kw).image(0)
    ctx = viso_amd.Context(viso_amd.default_params(width=w, height=h))
    xs, _, _ = ctx.fast(img, 50)
    ctx.timing_enable(True)
    n = 50
    for _ in range(n):
        ctx.fast(img, 50)
    launches, ms = ctx.timing("fast")
    print(f"{w}x{h}: {len(xs)} corners, HIP-event region {1e3 * ms / launches:.2f} us per call ({launches} calls)")
