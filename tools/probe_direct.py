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

    W, H, warm, steps, batch = 1242, 375, 20, int(os.environ.get("STEPS", "200")), int(os.environ.get("BATCH", "50"))
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
    lib.viso_debug_probe_ring.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                          ctypes.c_int]
    cap = 4096
    log = np.zeros((cap, 16), np.uint64)
    exits = np.zeros(cap, np.uint64)
    nl = ctypes.c_int(0)

    def run(f0, m):
        f = f0
        while f < f0 + m:
            k = min(batch, f0 + m - f)
            v.process_device(d_left.data_ptr() + f * W * H,
                             d_right.data_ptr() + f * W * H if stereo else None, k, W * H)
            f += k

    lib.viso_debug_probe_lk.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lkbuf = (ctypes.c_ulonglong * 32)()
    run(0, warm)
    v.synchronize()
    assert lib.viso_debug_probe_ring(log.ctypes.data, exits.ctypes.data, cap, ctypes.byref(nl), 1) == 0
    lib.viso_debug_probe_lk(lkbuf, 1)
    wm = (ctypes.c_ulonglong * 8)()
    has_wm = hasattr(lib, "viso_debug_probe_window_misses")
    if has_wm:
        lib.viso_debug_probe_window_misses(wm, 1)
    run(warm, steps)
    v.synchronize()
    if has_wm:
        lib.viso_debug_probe_window_misses(wm, 0)
        print("current-image samples outside their LDS window, per level (L0..L3): " +
              ", ".join(str(x) for x in list(wm)[:4]))
        print(f"merged L(3) points with a lane re-loading its `last` taps: {wm[4]} of {wm[5]}")
    print(f"map points {len(v.GetPoints())}, state {v.state}")
    assert lib.viso_debug_probe_ring(log.ctypes.data, exits.ctypes.data, cap, ctypes.byref(nl), 0) == 0
    n = min(nl.value, cap)
    log, exits = log[:n].astype(np.int64), exits[:n].astype(np.int64)
    lib.viso_debug_probe_lk(lkbuf, 0)
    q = list(lkbuf)
    print("LK alignment: mean GN iterations per (pair, level):",
          ", ".join(f"L{l} {q[l] / max(q[4 + l], 1):.2f} ({q[4 + l]} calls)" for l in range(4)))
    print(f"LK alignment: points {q[15]}, mean {q[14] / max(q[15], 1) * 0.01:.2f} us per point, slowest point "
          f"{q[9] * 0.01:.1f} us, most GN iterations of a point {q[10]}, points >= 20 us: {q[11]}, "
          f">= 10 iterations on a level: {q[8]}")
    print(f"LK alignment: slowest point {(q[24] >> 16) * 0.01:.1f} us with {q[24] & 0xffff} GN iterations; "
          f"most-iterated point {q[25] >> 40} iterations in {(q[25] & ((1 << 40) - 1)) * 0.01:.1f} us")
    if q[19]:  # background LK: the last frame of the (last) chunk
        first = (~q[16]) & 0xFFFFFFFFFFFFFFFF
        print(f"background LK last frame: {q[19]} items ({q[20]} by the drain), first ready sighting -> last "
              f"completion {(q[17] - first) * 0.01:.1f} us, last item start {(q[21] - first) * 0.01:.1f} us, "
              f"slowest item {q[18] * 0.01:.1f} us")
        if q[22]:
            d0 = (~q[22]) & 0xFFFFFFFFFFFFFFFF
            print(f"background LK drain: first drain wave -> last item of the chunk {(q[23] - d0) * 0.01:.1f} us; "
                  f"last frame first sighted {(first - d0) * 0.01:+.1f} us from the first drain wave")
    us = 0.01  # 100 MHz ticks -> us
    meta = log[:, 15]
    lvl = (meta & 0xff) - 1
    merged = (meta >> 8) & 0xff
    tiles = meta >> 16
    entry = log[:, 0]
    print(f"{n} launches; tiles per launch {int(np.median(tiles))}")
    names = ["partials reduced (w0)", "solver starts", "LU", "inverse", "update", "SE3 exp", "solve done",
             "after B2", "prefetch done (last wave)", "-", "block 0 exit", "first LU pass (VISO_LU_TWICE)"]
    print("phase (us from block 0 entry; mean over launches)      " +
          "  ".join(f"{x:>7s}" for x in ["F", "L0", "L1", "L2", "L3m", "L3"]))
    kinds = [(lvl == -1), (lvl == 0), (lvl == 1), (lvl == 2), (lvl == 3) & (merged == 1), (lvl == 3) & (merged == 0)]
    for k, name in enumerate(names, start=1):
        if name == "-":
            continue
        row = []
        for m in kinds:
            sel = m & (log[:, k] > 0)
            row.append(f"{(log[sel, k] - entry[sel]).mean() * us:7.2f}" if sel.any() else "      -")
        print(f"  {name:52s}" + "  ".join(row))
    row = []
    for m in kinds:
        sel = m & (exits > 0)
        row.append(f"{(exits[sel] - entry[sel]).mean() * us:7.2f}" if sel.any() else "      -")
    print(f"  {'last block exit':52s}" + "  ".join(row))
    # boundaries: consecutive launches of one frame's chain
    gaps = {}
    for i in range(n - 1):
        a, b = lvl[i], lvl[i + 1]
        if (a, b) in [(3, 2), (2, 1), (1, 0), (0, 3)] and exits[i] > 0:
            gaps.setdefault((a, b), []).append((entry[i + 1] - exits[i]) * us)
    print("boundary: last block exit -> next launch's block 0 entry (us): " +
          ", ".join(f"L{a}->L{b} {np.mean(g):.2f} (n={len(g)})" for (a, b), g in sorted(gaps.items())))
    # per-block stamps of the last launches: dispatch skew and phase durations
    lib.viso_debug_probe_blocks.argtypes = [ctypes.c_void_p, ctypes.c_int]
    blk = np.zeros((512, 256, 4), np.uint64)
    mb = lib.viso_debug_probe_blocks(blk.ctypes.data, 512)
    blk = blk[:mb].astype(np.int64)
    lv_b = lvl[n - mb:]
    nt = tiles[n - mb:]
    for L in (3, 2, 1, 0):
        sel = np.where(lv_b == L)[0]
        if not len(sel):
            continue
        T = int(nt[sel[0]])
        B = blk[sel, :T, :]
        e0 = B[:, :1, 0]
        rel = (B - e0[:, :, None]) * us  # us from block 0's entry
        pro = (B[:, :, 1] - B[:, :, 0]) * us
        til = (B[:, :, 2] - B[:, :, 1]) * us
        tree = (B[:, :, 3] - B[:, :, 2]) * us
        ex = rel[:, :, 3]
        print(f"L({L}) {T} blocks, mean over launches: entry skew max {rel[:, :, 0].max(axis=1).mean():.2f}; "
              f"prologue (entry -> B2) p50 {np.median(pro):.2f} max {pro.max(axis=1).mean():.2f}; "
              f"tiles (B2 -> wave 0's points) p50 {np.median(til):.2f} max {til.max(axis=1).mean():.2f}; "
              f"tile tree + store p50 {np.median(tree):.2f} max {tree.max(axis=1).mean():.2f}; "
              f"exit p50 {np.median(ex):.2f} max {ex.max(axis=1).mean():.2f}")
        for name, arr in [("prologue", pro), ("tiles", til), ("exit", ex)]:
            m = arr.mean(axis=0)
            print(f"      {name:8s} by block: first 8 {np.round(m[:8], 2).tolist()} last 8 {np.round(m[-8:], 2).tolist()} "
                  f"by XCD (b % 8) {np.round([m[x::8].mean() for x in range(8)], 2).tolist()}")
    # per wave: its point evaluated, relative to the block's B2; the last
    # arriver's trees stored (probe build, g_pwave)
    if hasattr(lib, "viso_debug_probe_waves_direct"):
        lib.viso_debug_probe_waves_direct.argtypes = [ctypes.c_void_p, ctypes.c_int]
        pw = np.zeros((512, 256, 16), np.uint64)
        mw = lib.viso_debug_probe_waves_direct(pw.ctypes.data, 512)
        pw = pw[:mw].astype(np.int64)
        blk2 = blk[-mw:] if len(blk) >= mw else blk
        for L in (3, 2, 1, 0):
            sel = np.where(lv_b[-mw:] == L)[0]
            if not len(sel):
                continue
            T = int(nt[-mw:][sel[0]])
            b2 = blk2[sel, :T, 1][:, :, None]
            rel = (pw[sel, :T, :] - b2) * us
            valid = pw[sel, :T, :] > 0
            row = []
            for w in range(16):
                v = rel[:, :, w][valid[:, :, w]]
                row.append(f"{np.median(v):5.2f}" if len(v) else "    -")
            print(f"L({L}) per wave, point(s) done after B2 (p50 us): " + " ".join(row[:15]) + f" | trees stored {row[15]}")
    # per wave, its point's phases (VISO_PROBE_PT builds): start after B2,
    # then quotients / samples / six sums / 28 sums, blocks < 32
    if hasattr(lib, "viso_debug_probe_points"):
        lib.viso_debug_probe_points.argtypes = [ctypes.c_void_p, ctypes.c_int]
        pp = np.zeros((128, 32, 16, 5), np.uint64)
        mp = lib.viso_debug_probe_points(pp.ctypes.data, 128)
        pp = pp[:mp].astype(np.int64)
        blk3 = blk[-mp:]
        for L in (3, 2, 1, 0):
            sel = np.where(lv_b[-mp:] == L)[0]
            if not len(sel):
                continue
            b2 = blk3[sel, :32, 1][:, :, None]
            st = pp[sel]  # launches x 32 x 16 x 5
            print(f"L({L}) per wave (blocks < 32, p50 us): start after B2 | quotients | samples | six sums | 28 sums")
            for w in range(12):
                ok = st[:, :, w, 0] > 0
                if not ok.any():
                    continue
                s0 = (st[:, :, w, 0] - b2[:, :, 0])[ok] * us
                d = [np.median((st[:, :, w, k] - st[:, :, w, k - 1])[ok]) * us for k in range(1, 5)]
                print(f"   wave {w:2d}: {np.median(s0):5.2f} | " + " | ".join(f"{x:5.2f}" for x in d))
    per = [(entry[i + 1] - entry[i]) * us for i in range(n - 1) if (lvl[i], lvl[i + 1]) in [(3, 2), (2, 1), (1, 0), (0, 3)]]
    print(f"entry-to-entry per launch in the chain: {np.mean(per):.2f} us")


if __name__ == "__main__":
    main()
