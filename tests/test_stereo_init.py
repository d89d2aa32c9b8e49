"""Stereo initialisation (viso_set_stereo, include/viso/viso_c.h): metric
depth from the right image replacing the 2D-2D init of
Viso::PoseEstimation2d2d (src/viso.cpp:178-256) and the map creation of
src/viso.cpp:79-96.  SURVEY.md §8(f) row 1; no reference counterpart, so
parity is HIP path vs the repo's own restatement (oracle/oracle_stereo.cpp
oracle_stereo_points, oracle/oracle_viso.cpp stereo_init) — parity unpinned
vs the reference.

Bars: state, FAST / stereo point counts exact; map points bit-exact (integer
SAD, the same double expressions); poses within 1e-10 relative Frobenius as
for the monocular path (tests/test_pipeline.py).  Size-independent property:
the map is metric, so tracked poses follow the renderer's ground truth
translation directly (no scale alignment)."""
import numpy as np
import pytest

from tests import oracle_lib, seqdata

W, H = seqdata.W, seqdata.H
MAX_DISP = 128


def _rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def _texture(h, w, seed):
    rng = np.random.default_rng(seed)
    # smooth texture (sub-pixel shifts stay meaningful): upsampled noise
    small = rng.integers(0, 256, (h // 4 + 2, w // 4 + 2)).astype(np.float64)
    ys = np.arange(h) / 4.0
    xs = np.arange(w) / 4.0
    y0, x0 = np.floor(ys).astype(int), np.floor(xs).astype(int)
    fy, fx = (ys - y0)[:, None], (xs - x0)[None, :]
    a = small[y0][:, x0]
    b = small[y0][:, x0 + 1]
    c = small[y0 + 1][:, x0]
    d = small[y0 + 1][:, x0 + 1]
    return (a * (1 - fx) * (1 - fy) + b * fx * (1 - fy) + c * (1 - fx) * fy + d * fx * fy)


def _shifted_pair(h, w, disp, seed=3):
    """left(x) = T(x), right(x) = T(x + disp): a fronto-parallel plane at
    disparity `disp` (sub-pixel allowed), both rounded to u8."""
    big = _texture(h, w + 64, seed)
    xs = np.arange(w, dtype=np.float64)
    left = big[:, 32:32 + w]
    src = xs + 32 + disp
    x0 = np.floor(src).astype(int)
    f = src - x0
    right = big[:, x0] * (1 - f) + big[:, x0 + 1] * f
    return (np.clip(np.rint(left), 0, 255).astype(np.uint8),
            np.clip(np.rint(right), 0, 255).astype(np.uint8))


# ------------------------------------------------------------------ CPU: oracle
@pytest.mark.parametrize("disp", [7.0, 12.5, 23.25])
def test_oracle_stereo_points_recover_plane_depth(disp):
    h, w = 64, 200
    left, right = _shifted_pair(h, w, disp)
    ys, xs = np.meshgrid(np.arange(8, h - 8, 6), np.arange(40, w - 8, 6), indexing="ij")
    xs, ys = xs.ravel().astype(np.int32), ys.ravel().astype(np.int32)
    K = (500.0, 500.0, w / 2.0, h / 2.0)
    base = 0.5
    pts = oracle_lib.stereo_points(left, right, xs, ys, 40, 1, K, base)
    assert len(pts) == len(xs)  # every patch is inside and 1 <= d < 40
    z_true = K[0] * base / disp
    # parabola on a V-shaped SAD curve: sub-pixel error under 0.2 px (the
    # known pixel-locking bias of SAD parabolas peaks near quarter offsets)
    dd = K[0] * base / pts[:, 2]
    assert np.abs(np.median(dd) - disp) < 0.2, np.median(dd)
    assert np.abs(dd - disp).max() < 0.35
    # back-projection: X = (x - cx) Z / fx, Y = (y - cy) Z / fy
    assert np.allclose(pts[:, 0], (xs - K[2]) * pts[:, 2] / K[0], rtol=0, atol=1e-12)
    assert np.allclose(pts[:, 1], (ys - K[3]) * pts[:, 2] / K[1], rtol=0, atol=1e-12)
    assert abs(np.median(pts[:, 2]) - z_true) / z_true < 0.02


def test_oracle_stereo_points_edge_cases():
    h, w = 40, 120
    left, right = _shifted_pair(h, w, 5.0)
    K = (400.0, 400.0, 60.0, 20.0)
    # patch outside the image, x - 4 too small for any d range, y at the border
    xs = np.array([3, 4, 5, 6, 116, 117, 60, 60], np.int32)
    ys = np.array([20, 20, 20, 20, 20, 20, 3, 37], np.int32)
    pts = oracle_lib.stereo_points(left, right, xs, ys, 32, 1, K, 0.3)
    # x=3: patch leaves the image; x=4..6: dmax = x - 4 < 2 or d >= dmax;
    # x=117 and y=3/37: patch leaves the image; x=116 is kept
    assert len(pts) == 1
    # min_disp above the true disparity rejects everything
    assert len(oracle_lib.stereo_points(left, right, xs[4:5], ys[4:5], 32, 8, K, 0.3)) == 0
    # empty input
    assert len(oracle_lib.stereo_points(left, right, xs[:0], ys[:0], 32, 1, K, 0.3)) == 0


def _oracle_run(n_frames, **kw):
    seq = seqdata.sequence(0)
    v = oracle_lib.Viso(seq.K, W, H, enable_tracking=1, **kw)
    v.set_stereo(seq.p.baseline, MAX_DISP, 1)
    states, stats = [], []
    for f in range(n_frames):
        v.on_new_stereo(seqdata.image(f), seqdata.image(f, cam=1))
        states.append(v.state)
        stats.append(v.stats())
    return seq, v, states, stats


def test_oracle_stereo_init_is_metric():
    seq, v, states, stats = _oracle_run(8)
    # the first stereo pair initialises: one keyframe, identity pose
    assert states == [1] * 8
    assert stats[0][3] == -2 and stats[0][2] > 1000
    assert len(v.points()) == stats[0][2]
    kf = v.keyframe_poses()
    assert len(kf) == 1 and np.allclose(kf[0], [1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0])
    # metric map: tracked translations follow the renderer's ground truth
    # without any scale alignment
    P = v.poses()
    g0 = seq.pose(0)
    for k, p in enumerate(P):
        gt = seq.pose(k + 1)[9:] - g0[9:]
        assert np.linalg.norm(p[9:] - gt) < 0.1 * np.linalg.norm(gt) + 2e-3, (k, p[9:], gt)


def test_oracle_stereo_disabled_is_the_mono_path():
    seq = seqdata.sequence(0)
    a = oracle_lib.Viso(seq.K, W, H, enable_tracking=1)
    b = oracle_lib.Viso(seq.K, W, H, enable_tracking=1)
    a.set_stereo(0.0, MAX_DISP, 1)
    for f in range(4):
        a.on_new_stereo(seqdata.image(f), seqdata.image(f, cam=1))
        b.on_new_frame(seqdata.image(f))
        assert a.state == b.state
        assert np.array_equal(a.stats(), b.stats())


def test_oracle_too_few_stereo_points_falls_back_to_mono():
    # a right image with no texture: no valid disparity -> the frame goes
    # through the monocular initialisation (re-detect)
    seq = seqdata.sequence(0)
    a = oracle_lib.Viso(seq.K, W, H, enable_tracking=1)
    b = oracle_lib.Viso(seq.K, W, H, enable_tracking=1)
    a.set_stereo(seq.p.baseline, MAX_DISP, 1)
    flat = np.full((H, W), 128, np.uint8)
    a.on_new_stereo(seqdata.image(0), flat)
    b.on_new_frame(seqdata.image(0))
    assert a.state == b.state == 0
    sa, sb = a.stats(), b.stats()
    assert sa[2] <= 50
    assert sa[1] == sb[1] and sa[5] == sb[5]
    k1a, _, _ = a.tracks()
    k1b, _, _ = b.tracks()
    assert np.array_equal(k1a, k1b)


def test_set_stereo_rejects_bad_arguments():
    import viso_amd
    from viso_amd import _lib
    if not _lib.os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built")
    lib = _lib.load()
    assert lib.viso_set_stereo(None, 0.5, 64, 1) == -1


# ------------------------------------------------------------------ GPU vs oracle
@pytest.mark.gpu
def test_gpu_stereo_init_matches_oracle():
    import viso_amd
    n = 8
    seq, ov, states, stats = _oracle_run(n)
    gv = viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=1)
    gv.set_stereo(seq.p.baseline, MAX_DISP, 1)
    for f in range(n):
        gv.process(seqdata.image(f), seqdata.image(f, cam=1))
        gv.synchronize()
        assert gv.state == states[f]
        s = gv.stats()
        assert s[1] == stats[f][1] and s[2] == stats[f][2] and s[3] == stats[f][3], (f, s, stats[f])
        if f == 0:
            assert np.array_equal(gv.GetPoints(), ov.points())
    assert np.array_equal(gv.GetPoints(), ov.points())
    assert len(gv.poses) == len(ov.poses()) == n - 1
    assert _rel(gv.poses, ov.poses()) < 1e-10


@pytest.mark.gpu
def test_gpu_stereo_init_device_ingest_matches_host():
    import torch

    import viso_amd
    seq = seqdata.sequence(0)
    n = 9
    frames = np.stack([seqdata.image(f) for f in range(n)])
    rights = np.stack([seqdata.image(f, cam=1) for f in range(n)])
    ref = viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=1)
    ref.set_stereo(seq.p.baseline, MAX_DISP, 1)
    for f in range(n):
        ref.process(frames[f], rights[f])
    dl = torch.from_numpy(frames).cuda()
    dr = torch.from_numpy(rights).cuda()
    torch.cuda.synchronize()
    bat = viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=1, batch_frames=4)
    bat.set_stereo(seq.p.baseline, MAX_DISP, 1)
    bat.process_device(dl.data_ptr(), dr.data_ptr(), n, W * H)
    bat.synchronize()
    assert bat.state == ref.state == 1
    assert np.array_equal(bat.poses, ref.poses)
    assert np.array_equal(bat.GetPoints(), ref.GetPoints())


@pytest.mark.gpu
def test_gpu_failed_stereo_init_keeps_mono_tracks():
    """A right image with no texture makes every stereo init fail, so each
    frame falls back to the monocular initialisation.  The stereo attempt
    must not disturb the mono state (init_.kp1 of the reference frame and the
    track count): frame by frame the GPU matches the oracle's stats, tracks
    and state through the KLT frames and the 2D-2D map creation."""
    import viso_amd
    seq = seqdata.sequence(0)
    flat = np.full((H, W), 128, np.uint8)
    ov = oracle_lib.Viso(seq.K, W, H, enable_tracking=1)
    ov.set_stereo(seq.p.baseline, MAX_DISP, 1)
    gv = viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=1)
    gv.set_stereo(seq.p.baseline, MAX_DISP, 1)
    states = []
    for f in range(9):
        ov.on_new_stereo(seqdata.image(f), flat)
        gv.process(seqdata.image(f), flat)
        gv.synchronize()
        so, sg = ov.stats(), gv.stats()
        assert gv.state == ov.state, f
        assert [sg[k] for k in (1, 2, 3, 5)] == [so[k] for k in (1, 2, 3, 5)], (f, sg[:6], so[:6])
        if ov.state == 0:
            k1o, k2o, _ = ov.tracks()
            k1g, k2g, _ = gv.tracks()
            assert np.array_equal(k1g, k1o) and np.array_equal(k2g, k2o), f
        states.append(ov.state)
    assert 0 in states and states[-1] == 1  # fallback frames, then the mono map
    assert np.array_equal(gv.GetPoints(), ov.points())
    assert _rel(gv.poses, ov.poses()) < 1e-10


@pytest.mark.gpu
def test_gpu_repeated_frames_take_the_continuation():
    """A frame identical to the last one gives a photometric cost of exactly 0
    at every level: the reference's loop then continues (cost / lastCost is
    0 / 0, src/viso.cpp:751) for 99 more GN iterations.  Both continuation
    paths of the direct-pose kernel run here: in a level launch's prologue
    (levels 3..1) and, under batched ingest, in the next frame's merged L(3)
    (level 0).  GPU == oracle frame by frame, per-frame and batched."""
    import torch

    import viso_amd
    order = [0, 1, 2, 3, 3, 3, 4, 5, 6]
    lefts = np.stack([seqdata.image(f) for f in order])
    rights = np.stack([seqdata.image(f, cam=1) for f in order])
    seq = seqdata.sequence(0)
    ov = oracle_lib.Viso(seq.K, W, H, enable_tracking=1)
    ov.set_stereo(seq.p.baseline, MAX_DISP, 1)
    gv = viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=1)
    gv.set_stereo(seq.p.baseline, MAX_DISP, 1)
    for k in range(len(order)):
        ov.on_new_stereo(lefts[k], rights[k])
        gv.process(lefts[k], rights[k])
        gv.synchronize()
        assert gv.state == ov.state == 1, k
    oP = ov.poses()
    assert len(oP) == len(order) - 1
    # no motion on the repeats (up to the SE3(R, t) -> matrix round trip)
    assert np.allclose(oP[3], oP[2], rtol=0, atol=1e-14) and np.allclose(oP[4], oP[2], rtol=0, atol=1e-14)
    assert _rel(gv.poses, oP) < 1e-10
    dl = torch.from_numpy(lefts).cuda()
    dr = torch.from_numpy(rights).cuda()
    torch.cuda.synchronize()
    bat = viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=1, batch_frames=len(order))
    bat.set_stereo(seq.p.baseline, MAX_DISP, 1)
    bat.process_device(dl.data_ptr(), dr.data_ptr(), len(order), W * H)
    bat.synchronize()
    assert bat.state == 1
    assert np.array_equal(bat.poses, gv.poses)
