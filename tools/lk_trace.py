"""Analysis tool (CPU only): the per-iteration trajectories of LKAlignment on
the bench's synthetic sequence, from the oracle's trace hook
(oracle_lk_trace), with the device window's behaviour simulated per
iteration (track.hip load_window / window_follow: initial 24x24 window
clamped into the level, re-placed at (ix0 - 7, iy0 - 7) when a tap leaves
it).  Prints the points of frame F with the most iterations / refills.

  python tools/lk_trace.py [--frame 24] [--top 12]
"""
from __future__ import annotations

import argparse
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tests import oracle_lib  # noqa: E402
from viso_amd.synth import Sequence  # noqa: E402

W, H = 1242, 375
WIN = 24


def level_dims(w, h):
    from viso_amd import api
    return api.pyramid_dims(w, h)[0]


def simulate(rows, dims):
    """rows: (level, iter, X, Y) of one point in order -> per-iteration refill
    flags and the number of iterations whose taps left the window."""
    out = []
    cur_level = None
    x0 = y0 = 0
    for lv, it, X, Y in rows:
        w, h = dims[int(lv)]
        if lv != cur_level:
            cur_level = lv
            # load_window around the level's start position (clamped)
            x0 = min(max(int(math.floor(X)) - WIN // 2 + 1, 0), w - WIN)
            y0 = min(max(int(math.floor(Y)) - WIN // 2 + 1, 0), h - WIN)
        ix = [int(X + px) for px in range(-4, 4)]
        iy = [int(Y + py) for py in range(-4, 4)]
        inside = all(0 <= a - x0 < WIN - 1 for a in ix) and all(0 <= b - y0 < WIN - 1 for b in iy)
        refill = False
        if not inside:
            x0, y0 = ix[0] - 7, iy[0] - 7
            refill = True
        out.append(refill)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frame", type=int, default=24)
    ap.add_argument("--top", type=int, default=12)
    args = ap.parse_args()
    seq = Sequence(W, H, seed=0)
    ov = oracle_lib.Viso(seq.K, W, H, enable_tracking=1)
    ov.set_stereo(seq.p.baseline, 128, 1)
    lib = oracle_lib.load()
    for f in range(args.frame):
        ov.on_new_stereo(seq.image(f, 0), seq.image(f, 1))
    cap = 2_000_000
    buf = np.zeros((cap, 6))
    lib.oracle_lk_trace(oracle_lib.ptr(buf), cap)
    ov.on_new_stereo(seq.image(args.frame, 0), seq.image(args.frame, 1))
    n = lib.oracle_lk_trace_count()
    lib.oracle_lk_trace(None, 0)
    t = buf[:n]
    dims = level_dims(W, H)
    pts = np.unique(t[:, 0]).astype(int)
    stats = []
    for p in pts:
        r = t[t[:, 0] == p]
        ref = simulate([(a[1], a[2], a[3], a[4]) for a in r], dims)
        per_level = [int((r[:, 1] == lv).sum()) for lv in range(4)]
        stats.append((p, len(r), int(sum(ref)), per_level, r))
    print(f"frame {args.frame}: {len(pts)} points, {n} iterations, "
          f"refills {sum(s[2] for s in stats)}")
    stats.sort(key=lambda s: -(s[1] + 10 * s[2]))
    for p, it, rf, pl, r in stats[:args.top]:
        print(f"point {p}: {it} iterations (L3..L0 {pl[3]} {pl[2]} {pl[1]} {pl[0]}), refills {rf}")
        for lv in (3, 2, 1, 0):
            rr = r[r[:, 1] == lv]
            if len(rr):
                step = np.hypot(np.diff(rr[:, 3]), np.diff(rr[:, 4])) if len(rr) > 1 else np.zeros(1)
                print(f"   L{lv}: start ({rr[0, 3]:.1f}, {rr[0, 4]:.1f}) end ({rr[-1, 3]:.1f}, {rr[-1, 4]:.1f}) "
                      f"dims {dims[lv]} step mean {step.mean():.2f} max {step.max():.2f} "
                      f"cost {rr[0, 5]:.3g} -> {rr[-1, 5]:.3g}")


if __name__ == "__main__":
    main()
