"""Tracking stage: pyramidal KLT (src/viso.cpp:259-391), direct photometric
GN pose (:640-766) and LK alignment (:768-925).

fp64 work with the canonical reduction order on both sides (DESIGN.md
§Numerics): GPU and oracle agree bit for bit on positions and success
flags; poses agree to 1e-12 relative (only libm sin/cos/acos may differ by an
ulp between the device and glibc).
"""
import numpy as np
import pytest

from tests import images, oracle_lib, seqdata

W, H = seqdata.W, seqdata.H


def _fast_kps(img, thresh=50):
    xs, ys, _ = oracle_lib.fast(img, thresh)
    return np.stack([xs, ys], 1).astype(np.float32)


# ------------------------------------------------------------------ CPU oracle sanity
def test_oracle_klt_recovers_integer_shift():
    base = images.smooth(120, 160, seed=2, scale=6)
    shifted = np.roll(np.roll(base, 2, axis=0), 3, axis=1)  # content moves +3 x, +2 y
    p0 = oracle_lib.pyramid(base)
    p1 = oracle_lib.pyramid(shifted)
    kp1 = np.array([[60, 50], [80, 70], [100, 40], [40, 80]], np.float32)
    kp2, succ = oracle_lib.klt(p0, p1, 160, 120, kp1, kp1.copy())
    assert succ.all()
    assert np.allclose(kp2 - kp1, [3, 2], atol=0.05)


def test_oracle_direct_identity_frames_keep_pose():
    d = seqdata.initialised()
    pyr = seqdata.pyramid(d["init_frame"])
    pose = d["kf_poses"][1]
    out = oracle_lib.direct_pose(pyr, pyr, W, H, d["K"], d["points"], pose, pose)
    # identical frames: zero photometric error -> zero update
    assert np.allclose(out, pose, atol=1e-12)


def test_oracle_se3_exp_matches_rodrigues():
    from scipy.spatial.transform import Rotation
    lib = oracle_lib.load()
    xi = np.array([0.1, -0.2, 0.3, 0.05, -0.02, 0.04])
    pose = np.array([1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0], np.float64)
    out = np.zeros(12)
    lib.oracle_se3_exp_left(xi.ctypes.data, pose.ctypes.data, out.ctypes.data)
    R = Rotation.from_rotvec(xi[3:]).as_matrix()
    w = xi[3:]
    th = np.linalg.norm(w)
    Wx = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
    V = np.eye(3) + (1 - np.cos(th)) / th**2 * Wx + (th - np.sin(th)) / th**3 * Wx @ Wx
    assert np.allclose(out[:9].reshape(3, 3), R, atol=1e-14)
    assert np.allclose(out[9:], V @ xi[:3], atol=1e-14)


def test_oracle_lk_align_identity_converges_in_place():
    d = seqdata.initialised()
    pyr = seqdata.pyramid(d["init_frame"])
    kfp = d["kf_poses"]
    pk, sc, ub, ua = oracle_lib.lk_align([seqdata.pyramid(0), pyr], kfp, pyr, kfp[1], W, H,
                                         d["K"], d["points"][:200])
    sel = pk == 1  # aligned against itself: the positions stay put
    assert sel.sum() > 0
    assert np.allclose(ua[sel & (sc == 1)], ub[sel & (sc == 1)], atol=1e-9)


# ------------------------------------------------------------------ GPU parity
@pytest.mark.gpu
@pytest.mark.parametrize("frame", [1, 3, 6])
def test_gpu_klt_bitexact(frame):
    from viso_amd import default_context
    ctx = default_context()
    p0 = seqdata.pyramid(0)
    p1 = seqdata.pyramid(frame)
    kp1 = _fast_kps(seqdata.image(0))
    got_kp, got_s = ctx.klt(p0, p1, W, H, kp1, kp1.copy())
    exp_kp, exp_s = oracle_lib.klt(p0, p1, W, H, kp1, kp1.copy())
    assert np.array_equal(got_s, exp_s)
    assert np.array_equal(got_kp.view(np.uint32), exp_kp.view(np.uint32))
    assert exp_s.mean() > 0.3


@pytest.mark.gpu
def test_gpu_klt_edges():
    from viso_amd import default_context
    ctx = default_context()
    p0 = seqdata.pyramid(0)
    p1 = seqdata.pyramid(2)
    # border points, a flat patch (singular H), far-off initial guesses
    kp1 = np.array([[0, 0], [3, 3], [4.5, 200], [1237, 370], [600, 10], [620.25, 187.75],
                    [100, 100]], np.float32)
    kp2 = kp1.copy()
    kp2[-1] += [300, -90]
    got = ctx.klt(p0, p1, W, H, kp1, kp2)
    exp = oracle_lib.klt(p0, p1, W, H, kp1, kp2)
    assert np.array_equal(got[1], exp[1])
    assert np.array_equal(got[0].view(np.uint32), exp[0].view(np.uint32))
    flat = np.full((64, 64), 100, np.uint8)
    pf = oracle_lib.pyramid(flat)
    k = np.array([[32, 32]], np.float32)
    got = ctx.klt(pf, pf, 64, 64, k, k.copy())
    exp = oracle_lib.klt(pf, pf, 64, 64, k, k.copy())
    assert np.array_equal(got[1], exp[1]) and got[1][0] == 0  # NaN update -> failure


def _rel_frob(a, b):
    return np.linalg.norm(np.asarray(a) - np.asarray(b)) / max(np.linalg.norm(b), 1e-300)


@pytest.mark.gpu
@pytest.mark.parametrize("step", [1, 2])
def test_gpu_direct_pose(step):
    from viso_amd import default_context
    d = seqdata.initialised()
    ctx = default_context(K=d["K"])
    f0 = d["init_frame"]
    last = seqdata.pyramid(f0)
    cur = seqdata.pyramid(f0 + step)
    pose = d["kf_poses"][1]
    got = ctx.direct_pose(last, cur, W, H, d["points"], pose, pose)
    exp = oracle_lib.direct_pose(last, cur, W, H, d["K"], d["points"], pose, pose)
    assert _rel_frob(got, exp) < 1e-12, (got, exp)
    assert not np.allclose(exp, pose)  # the GN step moved the pose


@pytest.mark.gpu
def test_gpu_direct_pose_identical_frames_and_empty():
    from viso_amd import default_context
    d = seqdata.initialised()
    ctx = default_context(K=d["K"])
    pyr = seqdata.pyramid(d["init_frame"])
    pose = d["kf_poses"][1]
    got = ctx.direct_pose(pyr, pyr, W, H, d["points"], pose, pose)
    exp = oracle_lib.direct_pose(pyr, pyr, W, H, d["K"], d["points"], pose, pose)
    assert _rel_frob(got, exp) < 1e-12
    # no map point projects inside -> nGood = 0 -> NaN update -> pose reverted
    far = np.array([[1e3, 1e3, 1.0]])
    got = ctx.direct_pose(pyr, pyr, W, H, far, pose, pose)
    assert np.array_equal(got, oracle_lib.direct_pose(pyr, pyr, W, H, d["K"], far, pose, pose))


@pytest.mark.gpu
def test_gpu_lk_align():
    from viso_amd import default_context
    d = seqdata.initialised()
    ctx = default_context(K=d["K"])
    f0 = d["init_frame"]
    kfs = [seqdata.pyramid(0), seqdata.pyramid(f0)]
    cur = seqdata.pyramid(f0 + 1)
    cur_pose = oracle_lib.direct_pose(seqdata.pyramid(f0), cur, W, H, d["K"], d["points"],
                                      d["kf_poses"][1], d["kf_poses"][1])
    got = ctx.lk_align(kfs, d["kf_poses"], cur, cur_pose, W, H, d["points"])
    exp = oracle_lib.lk_align(kfs, d["kf_poses"], cur, cur_pose, W, H, d["K"], d["points"])
    assert np.array_equal(got[0], exp[0])
    assert np.array_equal(got[1], exp[1])
    assert np.array_equal(got[2], exp[2])
    # aligned positions: bit-exact unless acos differs by an ulp (then 1e-9 px)
    assert np.max(np.abs(got[3] - exp[3])) < 1e-9
    assert exp[1].mean() > 0.5
