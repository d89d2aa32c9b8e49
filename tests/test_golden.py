"""Golden vectors (tests/golden/golden_v2.npz, written by
tests/golden/make_golden.py from the CPU oracle; golden_v1.npz holds the
same vectors from before the direct pose's factored per-point sums, kept as
the per-pixel form's frozen outputs).

The reference ships no fixtures and cannot be built here, so parity with the
reference itself is unpinned. These vectors freeze the
oracle's outputs: the CPU tests check that the oracle still reproduces them
exactly, and the GPU tests check the HIP path against the same numbers
without calling the oracle. Bars: bit-exact for pixels, indices, keypoint
positions (float32 bits), masks and counts; fp64 poses and map points within
1e-10 relative Frobenius (north_star bar 1e-4)."""
from __future__ import annotations

import functools
import hashlib
import os

import numpy as np
import pytest

from tests import oracle_lib

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_v2.npz")
GOLDEN_V1 = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_v1.npz")
W, H = 1242, 375


@functools.lru_cache(maxsize=1)
def golden():
    with np.load(GOLDEN, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@functools.lru_cache(maxsize=1)
def seq_frames():
    from viso_amd.synth import Sequence

    g = golden()
    seq = Sequence(W, H, seed=0)
    frames = [seq.image(f, 0) for f in range(len(g["seq_frame_sha256"]))]
    for f, img in enumerate(frames):
        assert hashlib.sha256(img.tobytes()).hexdigest() == str(g["seq_frame_sha256"][f]), \
            f"synthetic renderer changed (frame {f}): regenerate tests/golden"
    return frames


def _rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def _pyr(img):
    return oracle_lib.pyramid(img)


# ------------------------------------------------------------------ CPU: oracle pinned
def test_golden_file_small_and_complete():
    assert os.path.getsize(GOLDEN) < 512 * 1024
    g = golden()
    for k in ("pyr_out", "fast_t20", "fast_t50", "klt_kp2", "p2d_R", "seq_poses", "seq_points",
              "st_disp"):
        assert k in g and g[k].size > 0, k


def test_oracle_pyramid_golden():
    g = golden()
    assert np.array_equal(oracle_lib.pyramid(g["pyr_in"]), g["pyr_out"])


@pytest.mark.parametrize("t", [20, 50])
def test_oracle_fast_golden(t):
    g = golden()
    xs, ys, sc = oracle_lib.fast(g["fast_in"], t)
    assert np.array_equal(np.stack([xs, ys, sc], 1), g[f"fast_t{t}"])


def test_oracle_klt_golden():
    g = golden()
    kp2, succ = oracle_lib.klt(_pyr(g["klt_ref"]), _pyr(g["klt_cur"]), 160, 120, g["klt_kp1"],
                               g["klt_kp1"].copy())
    assert np.array_equal(kp2.view(np.uint32), g["klt_kp2"].view(np.uint32))
    assert np.array_equal(succ, g["klt_success"])


def test_oracle_pose_2d2d_golden():
    g = golden()
    out = oracle_lib.pose_2d2d(g["p2d_p1"], g["p2d_p2"], g["p2d_K"])
    assert np.array_equal(out["inliers"], g["p2d_inliers"])
    assert np.array_equal(out["stats"], g["p2d_stats"])
    assert np.array_equal(out["R"], g["p2d_R"]) and np.array_equal(out["T"], g["p2d_T"])


def test_oracle_stereo_golden():
    g = golden()
    d, s = oracle_lib.stereo_match(g["st_left"], g["st_right"], g["st_xs"], g["st_ys"], 32)
    assert np.array_equal(d, g["st_disp"]) and np.array_equal(s, g["st_sad"])


def test_oracle_sequence_golden():
    g = golden()
    frames = seq_frames()
    v = oracle_lib.Viso(tuple(g["seq_K"]), W, H, enable_tracking=1)
    for f, img in enumerate(frames):
        v.on_new_frame(img)
        assert v.state == g["seq_states"][f], f
        # stats[15] (keyframe count) postdates the golden files, which hold 0 there
        st = v.stats()
        assert np.array_equal(st[:15], g["seq_stats"][f][:15]), f
    assert np.array_equal(v.poses(), g["seq_poses"])
    assert np.array_equal(v.points(), g["seq_points"])
    assert np.array_equal(v.keyframe_poses(), g["seq_kf_poses"])
    pk, sc, _, ua = v.alignment()
    assert np.array_equal(pk, g["seq_lk_pair"]) and np.array_equal(sc, g["seq_lk_success"])
    assert np.array_equal(ua, g["seq_lk_after"])


def test_factored_sums_vs_golden_v1():
    """The direct pose's per-point sums in the factored form (round 6:
    Jp^T G Jp from six pixel sums, oracle_track.cpp direct_point_partials)
    against golden_v1, frozen while the oracle formed the 28 products per
    pixel: every discrete output equal (states, counts, decisions, LK pairs
    and success flags), fp64 outputs equal to within their last bits (poses
    measured 2.4e-17 rel, map points equal, LK positions 1.6e-17)."""
    with np.load(GOLDEN_V1, allow_pickle=False) as z:
        g1 = {k: z[k] for k in z.files}
    g = golden()
    for k in g1:
        if g1[k].dtype.kind in "iub":
            assert np.array_equal(g[k], g1[k]), k
    assert np.array_equal(g["seq_states"], g1["seq_states"])
    for f in range(len(g1["seq_stats"])):
        for k in (0, 1, 2, 3, 4, 5, 6, 7, 9, 12):  # state, counts and decisions
            assert g["seq_stats"][f][k] == g1["seq_stats"][f][k], (f, k)
    assert _rel(g["seq_stats"], g1["seq_stats"]) < 1e-13
    assert _rel(g["seq_poses"], g1["seq_poses"]) < 1e-15
    assert np.array_equal(g["seq_points"], g1["seq_points"])
    assert np.array_equal(g["seq_lk_pair"], g1["seq_lk_pair"])
    assert np.array_equal(g["seq_lk_success"], g1["seq_lk_success"])
    assert np.max(np.abs(g["seq_lk_after"] - g1["seq_lk_after"])) < 1e-9


# ------------------------------------------------------------------ GPU vs golden
@pytest.mark.gpu
def test_gpu_stages_golden():
    import viso_amd

    g = golden()
    ctx = viso_amd.default_context(160, 120)
    pyr = ctx.pyramid(g["pyr_in"])[0]
    assert np.array_equal(pyr, g["pyr_out"])
    for t in (20, 50):
        xs, ys, sc = ctx.fast(g["fast_in"], t)
        assert np.array_equal(np.stack([xs, ys, sc], 1), g[f"fast_t{t}"]), t
    ref, cur = ctx.pyramid(g["klt_ref"])[0], ctx.pyramid(g["klt_cur"])[0]
    kp2, succ = ctx.klt(ref, cur, 160, 120, g["klt_kp1"], g["klt_kp1"].copy())
    assert np.array_equal(kp2.view(np.uint32), g["klt_kp2"].view(np.uint32))
    assert np.array_equal(succ, g["klt_success"])
    d, s = ctx.stereo_match(g["st_left"], g["st_right"], g["st_xs"], g["st_ys"], 32)
    assert np.array_equal(d, g["st_disp"]) and np.array_equal(s, g["st_sad"])
    ctx = viso_amd.default_context(W, H, K=tuple(g["p2d_K"]))
    out = ctx.pose_2d2d(g["p2d_p1"], g["p2d_p2"])
    assert np.array_equal(out["inliers"], g["p2d_inliers"])
    st = out["stats"]
    assert all(st[k] == g["p2d_stats"][k] for k in (0, 1, 2, 4, 5, 6, 7))
    assert _rel(out["R"], g["p2d_R"]) < 1e-12 and _rel(out["T"], g["p2d_T"]) < 1e-10


@pytest.mark.gpu
def test_gpu_sequence_golden():
    import viso_amd

    g = golden()
    frames = seq_frames()
    v = viso_amd.Viso(*g["seq_K"], width=W, height=H, enable_tracking=1)
    for f, img in enumerate(frames):
        v.OnNewFrame(img)
        assert v.state == g["seq_states"][f], f
        st, gs = v.stats(), g["seq_stats"][f]
        for k in (1, 2, 3, 6, 7, 9, 12):  # counts and decisions: exact
            assert st[k] == gs[k], (f, k, st[k], gs[k])
    assert v.poses.shape == g["seq_poses"].shape
    for i in range(len(g["seq_poses"])):
        assert _rel(v.poses[i], g["seq_poses"][i]) < 1e-10, i
    assert _rel(v.GetPoints(), g["seq_points"]) < 1e-10
    pk, sc, _, ua = v.alignment()
    assert np.array_equal(pk, g["seq_lk_pair"]) and np.array_equal(sc, g["seq_lk_success"])
    assert np.max(np.abs(ua - g["seq_lk_after"])) < 1e-6
