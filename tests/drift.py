"""TEST INFRASTRUCTURE ONLY — drift of the oracle's canonical tree sums
against a literal restatement of the reference's running sums.

The device reproduces the oracle bit for bit in its tree order (DESIGN.md §2
"Canonical reduction order"); the reference accumulates H, b and cost as
running sums in loop order (src/viso.cpp:308-310, 727-729, 888-890) and the
disparity / mean depth likewise (:199-201, :622-625).  `compare` runs one
sequence through the oracle twice — tree order and literal order
(oracle_set_sum_order), concurrently in two threads (the order is per calling
thread) — and reports, frame by frame, whether every discrete decision
matches and how far the poses drift."""
from __future__ import annotations

import concurrent.futures as cf

import numpy as np

from tests import oracle_lib


def _run(literal, K, w, h, frames, stereo_base, max_disp):
    lib = oracle_lib.load()
    lib.oracle_set_sum_order(1 if literal else 0)
    try:
        v = oracle_lib.Viso(K, w, h, enable_tracking=1)
        if stereo_base > 0:
            v.set_stereo(stereo_base, max_disp, 1)
        rec = []
        for left, right in frames:
            if stereo_base > 0:
                v.on_new_stereo(left, right)
            else:
                v.on_new_frame(left)
            k1, k2, succ = v.tracks()
            pk, sc, _, _ = v.alignment()
            rec.append({"state": v.state, "stats": v.stats(), "kp1": k1, "kp2": k2, "inliers": succ,
                        "lk_pair": pk, "lk_success": sc})
        return rec, v.poses(), v.points()
    finally:
        lib.oracle_set_sum_order(0)


def compare(K, w, h, frames, stereo_base=0.0, max_disp=128):
    """frames: list of (left, right) u8 images.  Returns a summary dict."""
    with cf.ThreadPoolExecutor(2) as ex:
        ft = ex.submit(_run, False, K, w, h, frames, stereo_base, max_disp)
        fl = ex.submit(_run, True, K, w, h, frames, stereo_base, max_disp)
        (rt, pt, mt), (rl, pl, ml) = ft.result(), fl.result()
    # stats: [state, n_tracked, nr_inliers, best_motion, n_cand, frame_cnt,
    # lk pairs, lk successes, disparity^2, direct nGood (level 0), cost, ...]
    discrete = (0, 1, 2, 3, 4, 5, 6, 7, 9)
    mismatch = []
    for f, (a, b) in enumerate(zip(rt, rl)):
        bad = []
        if a["state"] != b["state"]:
            bad.append("state")
        if any(a["stats"][k] != b["stats"][k] for k in discrete):
            bad.append("stats")
        for key in ("kp1", "kp2", "inliers", "lk_pair", "lk_success"):
            if a[key].shape != b[key].shape or not np.array_equal(a[key], b[key]):
                bad.append(key)
        if bad:
            mismatch.append((f, bad))
    n = min(len(pt), len(pl))
    rel = (np.linalg.norm(pt[:n] - pl[:n], axis=1) /
           np.maximum(np.linalg.norm(pl[:n], axis=1), 1e-300)) if n else np.zeros(0)
    return {
        "frames": len(frames), "poses": int(n), "pose_counts": (len(pt), len(pl)),
        "states": [r["state"] for r in rt],
        "mismatch": mismatch,
        "pose_max_rel_frobenius": float(rel.max()) if n else 0.0,
        "pose_mean_rel_frobenius": float(rel.mean()) if n else 0.0,
        "map_points_max_abs": float(np.abs(mt - ml).max()) if mt.shape == ml.shape and mt.size else
        (0.0 if mt.shape == ml.shape else None),
        "nGood": [int(r["stats"][9]) for r in rt],
        "nGood_literal": [int(r["stats"][9]) for r in rl],
    }
