#!/usr/bin/env python3
"""Phase timing of the direct-pose kernels (dev tool, GPU box).

Loads the instrumented library (VISO_VARIANT=probe python viso_amd/build.py
-> viso_amd/libviso_amd_probe.so), runs the bench workload for a few hundred
tracking frames and prints, per kernel phase, the mean time from kernel entry
(block 0, thread 0, s_memrealtime at 100 MHz), plus the last frame's launch
timeline (entry/exit stamps of every level's tiles and solve kernels).
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

    W, H, warm, steps, batch = 1242, 375, 20, int(os.environ.get("STEPS", "200")), 50
    seq = Sequence(W, H, seed=0)
    n = warm + steps
    left = np.stack([seq.image(f, 0) for f in range(n)])
    right = np.stack([seq.image(f, 1) for f in range(n)])
    d_left = torch.from_numpy(left).cuda()
    d_right = torch.from_numpy(right).cuda()
    prec = viso_amd.PRECISION_FAST if os.environ.get("PRECISION", "") == "fast" else viso_amd.PRECISION_FAITHFUL
    v = viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=1, batch_frames=batch,
                      max_poses=4096, precision=prec)
    stereo = os.environ.get("MONO", "0") != "1"
    if stereo:  # the bench path: stereo-initialised map
        v.set_stereo(seq.p.baseline, 128, 1)
    lib = _lib.load()
    lib.viso_debug_probe.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    buf = (ctypes.c_ulonglong * 128)()

    def run(f0, m):
        f = f0
        while f < f0 + m:
            k = min(batch, f0 + m - f)
            v.process_device(d_left.data_ptr() + f * W * H,
                             d_right.data_ptr() + f * W * H if stereo else None, k, W * H)
            f += k

    lib.viso_debug_probe_lk.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lkbuf = (ctypes.c_ulonglong * 16)()
    run(0, warm)
    v.synchronize()
    lib.viso_debug_probe(buf, 128, 1)
    lib.viso_debug_probe_lk(lkbuf, 1)
    run(warm, steps)
    v.synchronize()
    print(f"map points {len(v.GetPoints())}, state {v.state}")
    assert lib.viso_debug_probe(buf, 128, 0) == 0
    lib.viso_debug_probe_lk(lkbuf, 0)
    q = list(lkbuf)
    print("LK alignment: mean GN iterations per (pair, level):",
          ", ".join(f"L{l} {q[l] / max(q[4 + l], 1):.2f} ({q[4 + l]} calls)" for l in range(4)))
    print(f"  (pair, level) with >= 10 iterations: {q[8]}")
    calls = max(sum(q[4:8]), 1)
    print(f"  per (pair, level): template+window {10.0 * q[12] / calls / 1e3:.2f} us, "
          f"iterations {10.0 * q[13] / calls / 1e3:.2f} us; per pair (4 levels) "
          f"{10.0 * q[14] / max(q[15], 1) / 1e3:.2f} us")
    p = list(buf)
    us = lambda x, c: 10.0 * x / max(c, 1) / 1e3  # 100 MHz ticks -> us
    print("launch  count  prologue-done  block0-done   (us from entry, block 0)")
    for k, name in enumerate(["F", "L(0)", "L(1)", "L(2)", "L(3)"]):
        c = p[16 + k]
        print(f"{name:6s} {c:6d}  {us(p[k], c):12.2f}  {us(p[8 + k], c):11.2f}")
    print("prologue phases (us from entry): B1  S-combined  solved  prologue-done")
    for k, name in enumerate(["F", "L(0)", "L(1)", "L(2)", "L(3)"]):
        c = p[16 + k]
        ph = [us(p[32 + 6 * k + j], c) for j in range(3)]
        print(f"{name:6s} {ph[0]:8.2f} {ph[1]:8.2f} {ph[2]:8.2f} {us(p[k], c):8.2f}")
    c = p[16 + 2]
    print("L(1) solve_wave0 (us from entry): LU %.2f  inverse %.2f  update %.2f  exp %.2f" %
          tuple(us(p[90 + k], c) for k in range(4)))
    if p[96]:
        print("L(1) solve: %.0f shader clocks in %.2f us -> %.2f GHz" %
              (p[95] / max(c, 1), us(p[96], c), p[95] / (10.0 * p[96])))
    stamps = [x for x in p[64:84] if x]
    t0 = min(stamps)
    print("last frame timeline (us from the first launch entry):")
    for k, name in [(4, "L(3)"), (3, "L(2)"), (2, "L(1)"), (1, "L(0)"), (0, "F")]:
        a, b = (p[64 + 4 * k] - t0) * 0.01, (p[65 + 4 * k] - t0) * 0.01
        last = (p[100 + k] - t0) * 0.01
        print(f"  {name:5s} entry {a:7.2f}  block0 exit {b:7.2f}  last block exit {last:7.2f}")

if __name__ == "__main__":
    main()
