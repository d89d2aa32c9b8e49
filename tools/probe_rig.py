#!/usr/bin/env python3
"""Phase timing of rig_level_kernel (dev tool, GPU box; probe library,
VISO_VARIANT=probe python viso_amd/build.py).  Runs the bench's configs[4]
rig workload and prints, per level kind, block 0's phase stamps from kernel
entry and the per-block prologue / tile / exit spread."""
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
    from viso_amd.rig import VisoRig
    from viso_amd.synth import RigSequence

    W, H, nc, n = 1242, 375, 4, 64
    seq = RigSequence(W, H, seed=2000, n_cams=nc)
    frames = [seq.frame(f) for f in range(n)]
    dl = torch.from_numpy(np.stack([im for ls, _ in frames for im in ls])).cuda()
    dr = torch.from_numpy(np.stack([im for _, rs in frames for im in rs])).cuda()
    fb = W * H
    prec = viso_amd.PRECISION_FAST if os.environ.get("PRECISION", "") == "fast" else viso_amd.PRECISION_FAITHFUL
    g = VisoRig(*seq.K, W, H, seq.extrinsics(), precision=prec, max_poses=n + 8)
    g.set_stereo(seq.p.baseline, 128, 1)
    g.process_device(dl.data_ptr(), dr.data_ptr(), 1, fb)
    g.synchronize()
    lib = _lib.load()
    lib.viso_debug_probe_ring.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                          ctypes.c_int]
    cap = 4096
    log = np.zeros((cap, 16), np.uint64)
    exits = np.zeros(cap, np.uint64)
    nl = ctypes.c_int(0)
    assert lib.viso_debug_probe_ring(log.ctypes.data, exits.ctypes.data, cap, ctypes.byref(nl), 1) == 0
    g.process_device(dl.data_ptr() + nc * fb, None, n - 1, fb)
    g.synchronize()
    assert lib.viso_debug_probe_ring(log.ctypes.data, exits.ctypes.data, cap, ctypes.byref(nl), 0) == 0
    m = min(nl.value, cap)
    log, exits = log[:m].astype(np.int64), exits[:m].astype(np.int64)
    keep = log[:, 15] != 0
    print(f"map points {[len(g.points(c)) for c in range(nc)]}; {int(keep.sum())} launches")
    us = 0.01
    meta = log[:, 15]
    lvl = (meta & 0xff) - 1
    merged = (meta >> 8) & 0xff
    entry = log[:, 0]
    kinds = [("L3m", keep & (lvl == 3) & (merged == 1)), ("L2", keep & (lvl == 2)), ("L1", keep & (lvl == 1)),
             ("L0", keep & (lvl == 0)), ("F", keep & (lvl == -1))]
    print("phase (us from block 0 entry)       " + "  ".join(f"{k:>7s}" for k, _ in kinds))
    for k, name in [(3, "w0: its partial loads landed"), (4, "w0: camera 0 contribution"),
                    (1, "every contribution in (w0)"), (2, "fold done"), (7, "solve done"), (8, "after B2"), (11, "block 0 exit")]:
        row = []
        for _, sel0 in kinds:
            sel = sel0 & (log[:, k] > 0)
            row.append(f"{(log[sel, k] - entry[sel]).mean() * us:7.2f}" if sel.any() else "      -")
        print(f"  {name:32s}" + "  ".join(row))
    row = []
    for _, sel0 in kinds:
        sel = sel0 & (exits > 0)
        row.append(f"{(exits[sel] - entry[sel]).mean() * us:7.2f}" if sel.any() else "      -")
    print(f"  {'last block exit':32s}" + "  ".join(row))
    lib.viso_debug_probe_blocks.argtypes = [ctypes.c_void_p, ctypes.c_int]
    blk = np.zeros((512, 256, 4), np.uint64)
    mb = lib.viso_debug_probe_blocks(blk.ctypes.data, 512)
    blk = blk[:mb].astype(np.int64)
    lv_b, mg_b = lvl[m - mb:], merged[m - mb:]
    for L in (3, 2, 1, 0):
        sel = np.where((lv_b == L) & (meta[m - mb:] != 0))[0]
        if not len(sel):
            continue
        B = blk[sel]
        nb = int((B[0, :, 0] > 0).sum())
        B = B[:, :nb, :]
        e0 = B[:, :1, 0]
        rel = (B - e0[:, :, None]) * us
        pro = (B[:, :, 1] - B[:, :, 0]) * us
        til = (B[:, :, 2] - B[:, :, 1]) * us
        tree = (B[:, :, 3] - B[:, :, 2]) * us
        print(f"L({L}) {nb} blocks: entry skew max {rel[:, :, 0].max(axis=1).mean():.2f}; prologue p50 "
              f"{np.median(pro):.2f} max {pro.max(axis=1).mean():.2f}; tiles p50 {np.median(til):.2f} max "
              f"{til.max(axis=1).mean():.2f}; tree+store p50 {np.median(tree):.2f} max {tree.max(axis=1).mean():.2f}; "
              f"exit p50 {np.median(rel[:, :, 3]):.2f} max {rel[:, :, 3].max(axis=1).mean():.2f}")
    per = [(entry[i + 1] - entry[i]) * us for i in range(m - 1) if keep[i] and keep[i + 1]]
    print(f"entry-to-entry per launch: {np.mean(per):.2f} us")


if __name__ == "__main__":
    main()
