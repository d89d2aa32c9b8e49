#!/usr/bin/env python3
"""Per-item timeline of the background LK grid's last frame (dev tool, GPU
box; probe build: VISO_VARIANT=probe python viso_amd/build.py).

Runs the driver's bench workload (5 warm-up frames, then one chunk of
STEPS=20 tracking frames) and prints, for the chunk's last frame, when its
items were dequeued / started / ended relative to the first start, the
per-level GN time and iterations of the slowest items, and on which wave kind
(resident grid or drain), XCD and CU they ran.
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
    warm, steps = 5, int(os.environ.get("STEPS", "20"))
    reps = int(os.environ.get("REPS", "3"))
    seq = Sequence(W, H, seed=0)
    n = warm + steps * reps
    left = np.stack([seq.image(f, 0) for f in range(n)])
    right = np.stack([seq.image(f, 1) for f in range(n)])
    d_left = torch.from_numpy(left).cuda()
    d_right = torch.from_numpy(right).cuda()
    v = viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=1, batch_frames=128, max_poses=4096)
    v.set_stereo(seq.p.baseline, 128, 1)
    lib = _lib.load()
    lib.viso_debug_probe_items.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    lib.viso_debug_probe_waves.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    wv = np.zeros((8192, 4), np.uint64)
    cap = 16384
    rec = np.zeros((cap, 16), np.uint64)
    lib.viso_debug_probe_ring.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                          ctypes.c_int]
    rcap = 4096
    rlog = np.zeros((rcap, 16), np.uint64)
    rexit = np.zeros(rcap, np.uint64)
    nl = ctypes.c_int(0)

    def run(f0, m):
        v.process_device(d_left.data_ptr() + f0 * W * H, d_right.data_ptr() + f0 * W * H, m, W * H)

    run(0, warm)
    v.synchronize()
    us = 0.01
    for rep in range(reps):
        lib.viso_debug_probe_items(rec.ctypes.data, cap, 1)
        lib.viso_debug_probe_waves(wv.ctypes.data, 8192, 1)
        lib.viso_debug_probe_ring(rlog.ctypes.data, rexit.ctypes.data, rcap, ctypes.byref(nl), 1)
        torch.cuda.synchronize()
        import time
        th = time.perf_counter()
        run(warm + rep * steps, steps)
        v.synchronize()
        th = (time.perf_counter() - th) * 1e6
        lib.viso_debug_probe_items(rec.ctypes.data, cap, 0)
        lib.viso_debug_probe_waves(wv.ctypes.data, 8192, 0)
        lib.viso_debug_probe_ring(rlog.ctypes.data, rexit.ctypes.data, rcap, ctypes.byref(nl), 0)
        nr = min(nl.value, rcap)
        rl = rlog[:nr].astype(np.int64)
        rx = rexit[:nr].astype(np.int64)
        r = rec.astype(np.int64)
        ok = ((r[:, 12] >> 48) & 1) == 1
        idx = np.where(ok)[0]
        R = r[idx]
        t0 = R[:, 1].min()
        start = (R[:, 1] - t0) * us
        end = (R[:, 10] - t0) * us
        dur = end - start
        deq = (R[:, 14] - t0) * us
        drain = ((R[:, 12] >> 40) & 1) == 1
        xcc = (R[:, 12] >> 32) & 0xff
        hw = R[:, 12] & 0xffffffff
        cu = (hw >> 8) & 0xf
        se = (hw >> 13) & 0x7
        simd = (hw >> 4) & 0x3
        its = np.stack([(R[:, 11] >> (16 * k)) & 0xffff for k in range(4)], 1)  # L3, L2, L1, L0
        chain0 = rl[0, 0]
        print(f"== rep {rep}: host-timed chunk {th:.0f} us; {nr} direct launches: first entry -> last exit "
              f"{(rx[-1] - chain0) * us:.1f} us; last frame's first item start at {(t0 - chain0) * us:.1f} us, "
              f"its last item end at {(R[:, 10].max() - chain0) * us:.1f} us")
        print(f"== rep {rep}: last frame {len(idx)} items ({drain.sum()} by the drain); first start -> last end "
              f"{end.max():.1f} us; last start {start.max():.1f}; dequeue before first start: "
              f"{(deq < 0).sum()} items")
        src = R[:, 13] & 0xff
        print(f"   sources: head {(src == 0).sum()}, leftover list {(src == 1).sum()}, second of a dequeue "
              f"{(src == 2).sum()}")
        W_ = wv.astype(np.int64)
        dr = W_[1024:]
        dr = dr[dr[:, 0] > 0]
        if len(dr):
            ds = (dr[:, 0] - t0) * us
            de = np.where(dr[:, 1] > 0, (dr[:, 1] - t0) * us, np.nan)
            print(f"   drain waves {len(dr)}: start p0 {ds.min():.1f} p50 {np.median(ds):.1f} p100 {ds.max():.1f} us; "
                  f"end p50 {np.nanmedian(de):.1f} max {np.nanmax(de):.1f}; n_left {int(dr[:, 3].max())}; items "
                  f"run: total {int(dr[:, 2].sum())}, waves with none {(dr[:, 2] == 0).sum()}, max {int(dr[:, 2].max())}")
        rw = W_[:1024]
        rw = rw[rw[:, 0] > 0]
        if len(rw):
            re_ = np.where(rw[:, 1] > 0, (rw[:, 1] - t0) * us, np.nan)
            print(f"   resident waves {len(rw)}: end p50 {np.nanmedian(re_):.1f} max {np.nanmax(re_):.1f} us; "
                  f"left early (no end stamp) {(rw[:, 1] == 0).sum()}; items run total {int(rw[:, 2].sum())}")
        q = np.percentile(dur, [50, 90, 99, 100])
        print(f"   item duration p50 {q[0]:.1f} p90 {q[1]:.1f} p99 {q[2]:.1f} max {q[3]:.1f} us; "
              f"mean iterations {its.sum(1).mean():.1f}")
        for lo, hi in [(0, 20), (20, 50), (50, 100), (100, 200), (200, 1e9)]:
            m = (end >= lo) & (end < hi)
            print(f"   items ending in [{lo}, {hi}) us: {m.sum()}")
        order = np.argsort(-end)[:16]
        print("   latest-ending items: point kind xcc se cu simd | deq start end | per level (L3..L0) "
              "iters @ us (us/iter)")
        for j in order:
            lv = []
            for k in range(4):
                a, b = R[j, 2 + k], R[j, 6 + k]
                if a and b:
                    dt = (b - a) * us
                    lv.append(f"{its[j, k]}@{dt:.1f}({dt / max(its[j, k], 1):.2f})")
                else:
                    lv.append("-")
            gaps = []
            prev = R[j, 1]
            for k in range(4):
                if R[j, 2 + k]:
                    gaps.append(f"{(R[j, 2 + k] - prev) * us:.1f}")
                    prev = R[j, 6 + k]
            wl = ""
            if R[j, 15]:  # VISO_PROBE_WIN: the slowest window load of the item (issue -> data, -> LDS)
                w15 = int(R[j, 15])
                t_iss = ((w15 >> 40) - (int(R[j, 1]) & 0xffffff)) % (1 << 24)
                wl = (f" | window L{(w15 >> 32) & 3}: load {(w15 & 0xffff) * us:.1f} commit {((w15 >> 16) & 0xffff) * us:.1f}"
                      f" issued at {start[j] + t_iss * us:.1f}")
            print(f"   {idx[j]:5d} {'drain' if drain[j] else 'res  '} {xcc[j]} {se[j]} {cu[j]:2d} {simd[j]} | "
                  f"{deq[j]:6.1f} {start[j]:6.1f} {end[j]:6.1f} | {' '.join(lv)} | gaps {' '.join(gaps)}{wl}")
        # by iterations: time per iteration of long items vs their kind
        tot = its.sum(1)
        sel = tot >= 40
        if sel.any():
            print("   items with >= 40 iterations: " + ", ".join(
                f"{idx[j]}:{tot[j]}it/{dur[j]:.0f}us/{'d' if drain[j] else 'r'}" for j in np.where(sel)[0][:40]))


if __name__ == "__main__":
    main()
