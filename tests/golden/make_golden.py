#!/usr/bin/env python3
"""Generate tests/golden/golden_v2.npz: frozen input/output vectors of the
per-frame path, written by the CPU oracle (oracle/, compiled in this
container).

The reference ships no tests, fixtures or golden vectors, and it cannot be
built here (Eigen/Sophus/OpenCV are absent). So these vectors
pin the oracle against itself over time, not against the reference ("parity
unpinned"). They also give the GPU tests anchors that do not
need the oracle at run time. Every input is stored in the file, and no input is
regenerated from a seed at test time, except the synthetic sequence frames:
they are re-rendered by viso_amd.synth and checked against stored SHA-256
hashes before use.

    python tests/golden/make_golden.py      # rewrites golden_v2.npz

golden_v2 (round 6) is golden_v1 (rounds 1-5) regenerated after the direct
pose's per-point sums took the factored form (oracle_track.cpp
direct_point_partials); only the sequence's fp64 outputs moved, in their last
bits (tests/test_golden.py::test_factored_sums_vs_golden_v1 keeps v1 as the
per-pixel form's frozen outputs).
"""
from __future__ import annotations

import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

OUT = os.path.join(HERE, "golden_v2.npz")
SEQ_FRAMES = 10  # synthetic seq (seed 0) initialises at frame 5, then tracks


def synth_matches(n, seed):
    """Normalised correspondences of a rotation-dominated motion (the
    reference keeps parallax <= 1 deg, src/viso.cpp:570) with 10 % outliers."""
    rng = np.random.default_rng(seed)
    a, b, c = 0.002, 0.03, 0.001
    Rx = np.array([[1, 0, 0], [0, np.cos(a), -np.sin(a)], [0, np.sin(a), np.cos(a)]])
    Ry = np.array([[np.cos(b), 0, np.sin(b)], [0, 1, 0], [-np.sin(b), 0, np.cos(b)]])
    Rz = np.array([[np.cos(c), -np.sin(c), 0], [np.sin(c), np.cos(c), 0], [0, 0, 1]])
    R = Rz @ Ry @ Rx
    t = np.array([0.05, 0.0, 0.01])
    X = np.stack([rng.uniform(-8, 8, n), rng.uniform(-3, 3, n), rng.uniform(10, 40, n)], 1)
    Y = X @ R.T + t
    x1 = X / X[:, 2:3]
    x2 = Y / Y[:, 2:3]
    k = n // 10
    x2[:k, :2] += rng.uniform(-0.05, 0.05, (k, 2))
    return x1, x2


def main():
    from tests import images, oracle_lib
    from viso_amd.synth import Sequence

    g = {}
    # --- pyramid (include/keyframe.h:28-46): odd sizes exercise trunc(w*0.5)
    img = images.mixed(61, 97, seed=11)
    g["pyr_in"] = img
    g["pyr_out"] = oracle_lib.pyramid(img)

    # --- FAST-9 + NMS (src/viso.cpp:104), two thresholds
    img = images.mixed(120, 160, seed=5)
    g["fast_in"] = img
    for t in (20, 50):
        xs, ys, sc = oracle_lib.fast(img, t)
        g[f"fast_t{t}"] = np.stack([xs, ys, sc], 1).astype(np.int32)

    # --- KLT (src/viso.cpp:259-391): smooth image moved by (+3, +2) plus
    # points at the border (failures) and a NaN-free far point
    base = images.smooth(120, 160, seed=2, scale=6)
    shifted = np.roll(np.roll(base, 2, axis=0), 3, axis=1)
    kp1 = np.array([[60, 50], [80, 70], [100, 40], [40, 80], [2, 2], [158, 118], [5, 60]],
                   np.float32)
    g["klt_ref"] = base
    g["klt_cur"] = shifted
    g["klt_kp1"] = kp1
    kp2, succ = oracle_lib.klt(oracle_lib.pyramid(base), oracle_lib.pyramid(shifted), 160, 120,
                               kp1, kp1.copy())
    g["klt_kp2"] = kp2
    g["klt_success"] = succ

    # --- PoseEstimation2d2d + SelectMotion (src/viso.cpp:178-256, 520-638)
    K = np.array([718.856, 718.856, 607.1928, 185.2157])
    x1, x2 = synth_matches(300, seed=3)
    g["p2d_K"] = K
    g["p2d_p1"] = x1
    g["p2d_p2"] = x2
    out = oracle_lib.pose_2d2d(x1, x2, K)
    g["p2d_R"] = out["R"]
    g["p2d_T"] = out["T"]
    g["p2d_inliers"] = out["inliers"]
    g["p2d_stats"] = out["stats"]

    # --- whole OnNewFrame path (src/viso.cpp:7-145) on the synthetic sequence
    seq = Sequence(1242, 375, seed=0)
    frames = np.stack([seq.image(f, 0) for f in range(SEQ_FRAMES)])
    g["seq_K"] = np.array(seq.K)
    g["seq_frame_sha256"] = np.array(
        [hashlib.sha256(f.tobytes()).hexdigest() for f in frames])
    # the frames themselves (3.7 MB of noise-like texture) are not stored: the
    # tests re-render them and check these hashes first, so a renderer change
    # fails loudly instead of silently moving the anchor
    v = oracle_lib.Viso(seq.K, 1242, 375, enable_tracking=1)
    states, stats = [], []
    for f in range(SEQ_FRAMES):
        v.on_new_frame(frames[f])
        states.append(v.state)
        stats.append(v.stats())
    g["seq_states"] = np.array(states, np.int32)
    g["seq_stats"] = np.stack(stats)
    g["seq_poses"] = v.poses()
    g["seq_points"] = v.points()
    g["seq_kf_poses"] = v.keyframe_poses()
    pk, sc, ub, ua = v.alignment()
    g["seq_lk_pair"] = pk
    g["seq_lk_success"] = sc
    g["seq_lk_after"] = ua

    # --- stereo SAD stage (north-star; no reference counterpart)
    rng = np.random.default_rng(0)
    left = rng.integers(0, 256, (60, 200), dtype=np.uint8)
    right = np.roll(left, -7, axis=1)
    right[:, 120:] = rng.integers(0, 256, (60, 80), dtype=np.uint8)  # unmatched region
    xs = np.array([50, 100, 150, 3, 197, 119, 60], np.int32)
    ys = np.array([30, 20, 40, 30, 30, 10, 4], np.int32)
    d, s = oracle_lib.stereo_match(left, right, xs, ys, 32)
    g["st_left"], g["st_right"], g["st_xs"], g["st_ys"] = left, right, xs, ys
    g["st_disp"], g["st_sad"] = d, s

    np.savez_compressed(OUT, **g)
    print(f"wrote {OUT}: {os.path.getsize(OUT)} bytes, {len(g)} arrays")
    print("seq states", states, "poses", g["seq_poses"].shape, "points", g["seq_points"].shape)


if __name__ == "__main__":
    main()
