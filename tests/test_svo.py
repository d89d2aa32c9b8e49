"""North-star stereo VO (SVO) stages: the CPU spec (oracle/oracle_svo.cpp) pinned
by known answers and by the synthetic renderer's ground truth, then GPU parity
(viso_amd/csrc/svo.hip) against it.  No reference counterpart: "parity
unpinned vs reference" (SURVEY.md §8a)."""
from __future__ import annotations

import numpy as np
import pytest

from tests import images, oracle_lib as ol


def _params(w=1242, h=375, **kw):
    return ol.svo_params(w, h, 718.856, 718.856, 607.19, 185.22, 0.54, **kw)


def _T(p12):
    M = np.eye(4)
    M[:3, :3] = np.asarray(p12[:9]).reshape(3, 3)
    M[:3, 3] = p12[9:]
    return M


# ------------------------------------------------------------------ CPU: spec known answers
def test_responses_known_answers():
    img = np.zeros((20, 20), np.uint8)
    img[10, 10] = 200
    b, c = ol.svo_responses(img)
    assert b[10, 10] == 8 * 200             # centre weight
    assert b[10, 11] == 200 and b[10, 12] == -200  # inner ring +1, outer ring -1
    assert b[10, 13] == 0
    assert c[10, 10] == 0                   # centre row/column weight 0
    assert c[9, 9] == -200 and c[9, 11] == 200  # TL quadrant -1, TR +1 (relative to the pixel)
    assert b[0, 0] == 0 and b[1, 10] == 0   # outside the 5x5 domain
    # checkerboard corner: TL/BR dark, TR/BL bright -> positive corner response
    chk = np.zeros((20, 20), np.uint8)
    chk[:10, 10:] = 100
    chk[10:, :10] = 100
    _, c = ol.svo_responses(chk)
    assert c[10, 10] == 8 * 100
    assert c[10, 10] == c.max()


def test_features_nms_and_order():
    p = _params(64, 48, nms_tau=100, nms_n=2, margin=8)
    img = np.full((48, 64), 50, np.uint8)
    img[20, 30] = 250               # blob max
    img[30, 12] = 0                 # blob min (dark dot on grey)
    img[30, 40] = 250
    img[30, 41] = 250               # a plateau pair: equal responses suppress each other
    f = ol.svo_features(img, p)
    pts = list(zip(f.v.tolist(), f.u.tolist(), f.cls.tolist()))
    assert (20, 30, 0) in pts
    assert (30, 12, 1) in pts
    assert (30, 40, 0) not in pts and (30, 41, 0) not in pts
    assert pts == sorted(pts)       # row-major, then u, then class
    # descriptor of the blob: du at (x-5, y-1) is 0 gradient -> 128
    i = pts.index((20, 30, 0))
    assert f.desc[i, 0] == 128
    # du at (x-1, y-1): right column holds the 250 pixel at weight 1:
    # d = (250 - 50) -> (200 >> 3) + 128 = 153
    assert f.desc[i, 6] == 153


def test_bucketing_keeps_lowest_indices():
    p = _params(200, 100, bucket_width=50, bucket_height=50, bucket_max=2)
    uv8 = np.zeros((6, 8), np.int32)
    uv8[:, 4] = [10, 20, 30, 60, 15, 70]   # u_l2
    uv8[:, 5] = [10, 10, 10, 10, 60, 10]   # v_l2
    keep = ol.svo_bucket(uv8, 200, 100, p)
    assert keep.tolist() == [True, True, False, True, True, True]


def _synthetic_matches(motion, n=300, seed=0, noise=0.0):
    """Points in front of camera t-1 -> integer observations of both pairs."""
    rng = np.random.default_rng(seed)
    fx, fy, cu, cv, b = 718.856, 718.856, 607.19, 185.22, 0.54
    R, t = motion[:9].reshape(3, 3), motion[9:]
    out = []
    while len(out) < n:
        Z = rng.uniform(5, 40)
        u1, v1 = rng.uniform(20, 1220), rng.uniform(20, 355)
        d1 = np.round(fx * b / Z)
        if d1 < 1:
            continue
        u1, v1 = np.round(u1), np.round(v1)
        Zq = fx * b / d1
        P = np.array([(u1 - cu) * Zq / fx, (v1 - cv) * Zq / fy, Zq])
        Q = R @ P + t
        if Q[2] <= 1:
            continue
        uL = fx * Q[0] / Q[2] + cu + rng.normal(0, noise)
        vL = fy * Q[1] / Q[2] + cv + rng.normal(0, noise)
        uR = fx * (Q[0] - b) / Q[2] + cu + rng.normal(0, noise)
        out.append([u1, v1, u1 - d1, v1, np.round(uL), np.round(vL), np.round(uR), np.round(vL)])
    return np.array(out, np.int32)


def test_estimate_recovers_known_motion():
    p = _params()
    a = 0.02
    Rz = np.array([[np.cos(a), -np.sin(a), 0], [np.sin(a), np.cos(a), 0], [0, 0, 1]])
    motion = np.concatenate([Rz.ravel(), [0.1, -0.05, 0.8]])
    uv8 = _synthetic_matches(motion, n=400)
    # 20 % gross outliers
    rng = np.random.default_rng(1)
    bad = rng.choice(len(uv8), 80, replace=False)
    uv8[bad, 4] += rng.integers(20, 60, len(bad))
    m, inl, n = ol.svo_estimate(uv8, 0, p)
    assert n >= 250
    assert not inl[bad].any()
    assert np.abs(m[:9] - motion[:9]).max() < 2e-3
    assert np.abs(m[9:] - motion[9:]).max() < 0.05


def test_estimate_too_few_matches_fails():
    p = _params()
    uv8 = _synthetic_matches(np.array([1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0.5]), n=5)
    m, inl, n = ol.svo_estimate(uv8, 0, p)
    assert n == -1 and not inl.any()
    assert np.array_equal(m, [1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0])


@pytest.fixture(scope="module")
def synth_frames():
    from viso_amd.synth import Sequence
    seq = Sequence(1242, 375, seed=0)
    return seq, [seq.frame(f) for f in range(4)]


def test_sequence_tracks_ground_truth(synth_frames):
    seq, frames = synth_frames
    p = ol.svo_params(1242, 375, *seq.K, seq.p.baseline)
    S = ol.SvoSequence(p)
    for f, (l, r) in enumerate(frames):
        ok = S.process(l, r)
        if f == 0:
            continue
        assert ok
        nl, nr, nm, nb, ni, _ = S.stats
        assert 1500 < nl < 4000 and 1500 < nr < 4000
        assert nb <= nm and ni > 0.6 * nb
        gt = _T(seq.pose(f, 0)) @ np.linalg.inv(_T(seq.pose(f - 1, 0)))
        est = _T(S.motion)
        assert np.abs(gt[:3, :3] - est[:3, :3]).max() < 1e-3
        assert np.abs(gt[:3, 3] - est[:3, 3]).max() < 0.01
    # circular consistency of the last pair's matches: every l2 appears once
    assert len(np.unique(S.matches[:, 4] * 4096 + S.matches[:, 5])) == len(S.matches)


def test_params_layout_and_defaults_match_spec():
    """The library's viso_svo_params / defaults are the spec's (host-only call)."""
    from viso_amd import svo
    assert ctypes_sizeof(svo.SvoParams) == ctypes_sizeof(ol.SvoParams)
    assert [f[0] for f in svo.SvoParams._fields_] == [f[0] for f in ol.SvoParams._fields_]
    a = svo.default_params(1242, 375, 718.856, 718.856, 607.19, 185.22, 0.54)
    b = _params()
    for name, _ in ol.SvoParams._fields_:
        if name != "reserved":
            assert getattr(a, name) == getattr(b, name), name


def ctypes_sizeof(t):
    import ctypes
    return ctypes.sizeof(t)


# ------------------------------------------------------------------ GPU parity
@pytest.fixture(scope="module")
def gpu_vo():
    from viso_amd import svo
    p = svo.default_params(1242, 375, 718.856, 718.856, 607.19, 185.22, 0.54)
    return svo.VisualOdometryStereo(p)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,h,w,tau,n", [
    ("synth", 375, 1242, 700, 5), ("mixed", 375, 1242, 700, 5), ("noise", 120, 160, 300, 2),
    ("blocks", 96, 128, 100, 1), ("synth1080", 1080, 1920, 700, 5), ("smooth", 64, 64, 50, 3),
    # margin 8 < n + 2: responses outside the domain enter the NMS (as -inf)
    ("noise", 150, 300, 200, 7), ("mixed", 200, 700, 300, 8)])
def test_gpu_features_bitexact(kind, h, w, tau, n):
    from viso_amd import svo
    if kind.startswith("synth"):
        from viso_amd.synth import Sequence
        img = Sequence(w, h, seed=3).image(2, 1)
    else:
        img = getattr(images, kind)(h, w, seed=7)
    p = svo.default_params(w, h, 718.856, 718.856, w / 2, h / 2, 0.54, nms_tau=tau, nms_n=n)
    vo = svo.VisualOdometryStereo(p)
    got = vo.features(img)
    exp = ol.svo_features(img, ol.svo_params(w, h, 718.856, 718.856, w / 2, h / 2, 0.54,
                                             nms_tau=tau, nms_n=n))
    assert len(got) == len(exp) > 0
    for a in ("u", "v", "cls", "desc"):
        assert np.array_equal(getattr(got, a), getattr(exp, a)), a


@pytest.mark.gpu
@pytest.mark.parametrize("cap", [700, 1999])
def test_gpu_sequence_truncated_capacity(synth_frames, cap):
    """More candidates than max_features: the first `cap` in row-major order
    are kept (the segment that straddles the cap partly), in the features and
    in the class-band index the matching reads (matches of the whole
    sequence identical to the spec)."""
    from viso_amd import svo
    seq, frames = synth_frames
    p = svo.default_params(1242, 375, *seq.K, seq.p.baseline, max_features=cap)
    q = ol.svo_params(1242, 375, *seq.K, seq.p.baseline, max_features=cap)
    vo = svo.VisualOdometryStereo(p)
    got = vo.features(frames[0][0])
    exp = ol.svo_features(frames[0][0], q)
    assert len(got) == len(exp) == cap
    for a in ("u", "v", "cls", "desc"):
        assert np.array_equal(getattr(got, a), getattr(exp, a)), a
    S = ol.SvoSequence(q)
    for f, (l, r) in enumerate(frames):
        assert vo.process(l, r) == S.process(l, r)
        assert vo.stats().tolist() == S.stats
        if f > 0:
            uv8, inl = vo.getMatches()
            assert np.array_equal(uv8, S.matches) and np.array_equal(inl, S.inliers)


@pytest.mark.gpu
def test_gpu_match_bitexact(gpu_vo, synth_frames):
    seq, frames = synth_frames
    p = _params()
    f4 = [ol.svo_features(frames[0][0], p), ol.svo_features(frames[0][1], p),
          ol.svo_features(frames[1][0], p), ol.svo_features(frames[1][1], p)]
    exp = ol.svo_match(f4, 375, p)
    got = gpu_vo.match(f4)
    assert len(exp) > 500
    assert np.array_equal(got, exp)


@pytest.mark.gpu
@pytest.mark.parametrize("frame", [1, 2, 3])
def test_gpu_estimate_bitexact(gpu_vo, synth_frames, frame):
    seq, frames = synth_frames
    p = _params()
    f4 = [ol.svo_features(frames[frame - 1][0], p), ol.svo_features(frames[frame - 1][1], p),
          ol.svo_features(frames[frame][0], p), ol.svo_features(frames[frame][1], p)]
    uv8 = ol.svo_uv8(f4, ol.svo_match(f4, 375, p))
    sel = uv8[ol.svo_bucket(uv8, 1242, 375, p)]
    m_exp, inl_exp, n_exp = ol.svo_estimate(sel, frame, p)
    m_got, inl_got, n_got = gpu_vo.estimate(sel, frame)
    assert n_got == n_exp > 0
    assert np.array_equal(inl_got, inl_exp)
    assert np.array_equal(m_got, m_exp)  # fp64, same expression order: bit-exact


@pytest.mark.gpu
def test_gpu_estimate_outliers_and_failure(gpu_vo):
    p = _params()
    motion = np.array([1, 0, 0, 0, 1, 0, 0, 0, 1, 0.05, 0, 0.7])
    uv8 = _synthetic_matches(motion, n=300, seed=4)
    uv8[::5, 5] += 30
    for frame in (0, 7):
        m_exp, inl_exp, n_exp = ol.svo_estimate(uv8, frame, p)
        m_got, inl_got, n_got = gpu_vo.estimate(uv8, frame)
        assert n_got == n_exp and np.array_equal(inl_got, inl_exp) and np.array_equal(m_got, m_exp)
    few = uv8[:5]
    m_got, inl_got, n_got = gpu_vo.estimate(few, 0)
    assert n_got == -1 and np.array_equal(m_got, [1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0])


@pytest.mark.gpu
def test_gpu_sequence_matches_oracle(synth_frames):
    from viso_amd import svo
    seq, frames = synth_frames
    p = svo.default_params(1242, 375, *seq.K, seq.p.baseline)
    vo = svo.VisualOdometryStereo(p)
    S = ol.SvoSequence(ol.svo_params(1242, 375, *seq.K, seq.p.baseline))
    for f, (l, r) in enumerate(frames):
        ok = vo.process(l, r)
        ok_exp = S.process(l, r)
        assert ok == ok_exp == (f > 0)
        assert vo.stats().tolist() == S.stats
        if f > 0:
            assert np.array_equal(vo.getMotion()[:3].ravel()[[0, 1, 2, 4, 5, 6, 8, 9, 10]],
                                  S.motion[:9])
            uv8, inl = vo.getMatches()
            assert np.array_equal(uv8, S.matches) and np.array_equal(inl, S.inliers)
    P = vo.poses
    assert len(P) == len(S.poses)
    assert np.allclose(P, np.array(S.poses), rtol=0, atol=1e-9)


@pytest.mark.gpu
def test_gpu_batched_device_path_matches_sequential(synth_frames):
    """viso_svo_process_device (one feature pass + side-by-side motions for a
    batch) gives the per-pair results of process() and of the spec."""
    import torch

    from viso_amd import svo
    seq, frames = synth_frames
    p = svo.default_params(1242, 375, *seq.K, seq.p.baseline)
    L = torch.from_numpy(np.stack([f[0] for f in frames])).cuda()
    R = torch.from_numpy(np.stack([f[1] for f in frames])).cuda()
    vb = svo.VisualOdometryStereo(p)
    vb.process_device(L.data_ptr(), R.data_ptr(), len(frames), 1242 * 375)
    vs = svo.VisualOdometryStereo(p)
    S = ol.SvoSequence(ol.svo_params(1242, 375, *seq.K, seq.p.baseline))
    for l, r in frames:
        vs.process(l, r)
        S.process(l, r)
    assert np.array_equal(vb.poses, vs.poses)
    assert vb.stats().tolist() == vs.stats().tolist() == S.stats
    assert np.array_equal(vb.getMotion(), vs.getMotion())
    ub, ib = vb.getMatches()
    assert np.array_equal(ub, S.matches) and np.array_equal(ib, S.inliers)


@pytest.mark.gpu
def test_gpu_config3_1080p_2048_hypotheses():
    """BASELINE.json configs[2]: synthetic 1920x1080 stereo, ~8k features per
    image, 2048 RANSAC hypotheses — per-pair stats, matches, inlier masks and
    motions identical to the spec, batched device path == per-pair path."""
    import torch

    from viso_amd import svo
    from viso_amd.synth import Sequence
    W, H, n = 1920, 1080, 4
    seq = Sequence(W, H, seed=1000)
    frames = [seq.frame(f) for f in range(n)]
    kw = dict(ransac_iters=2048)
    p = svo.default_params(W, H, *seq.K, seq.p.baseline, **kw)
    vo = svo.VisualOdometryStereo(p)
    S = ol.SvoSequence(ol.svo_params(W, H, *seq.K, seq.p.baseline, **kw))
    for f, (l, r) in enumerate(frames):
        assert vo.process(l, r) == S.process(l, r)
        st = vo.stats().tolist()
        assert st == S.stats
        assert min(st[0], st[1]) > 4000
        if f > 0:
            assert st[5] == 1
            uv8, inl = vo.getMatches()
            assert np.array_equal(uv8, S.matches) and np.array_equal(inl, S.inliers)
    assert np.allclose(vo.poses, np.array(S.poses), rtol=0, atol=1e-9)
    L = torch.from_numpy(np.stack([f[0] for f in frames])).cuda()
    R = torch.from_numpy(np.stack([f[1] for f in frames])).cuda()
    vb = svo.VisualOdometryStereo(p)
    vb.process_device(L.data_ptr(), R.data_ptr(), n, W * H)
    assert np.array_equal(vb.poses, vo.poses)


# ------------------------------------------------------------------ multi-camera rig (configs[4])
@pytest.fixture(scope="module")
def rig_frames():
    from viso_amd.synth import RigSequence
    seq = RigSequence(1242, 375, seed=2000, n_cams=4)
    return seq, [seq.frame(f) for f in range(4)]


def test_rig_spec_recovers_ground_truth(rig_frames):
    seq, frames = rig_frames
    S = ol.SvoRigSequence(ol.svo_params(1242, 375, *seq.K, seq.p.baseline), seq.extrinsics())
    for f, (L, R) in enumerate(frames):
        assert S.process(L, R) == (f > 0)
        if f > 0:
            gt = _T(seq.rig_pose(f)) @ np.linalg.inv(_T(seq.rig_pose(f - 1)))
            M = _T(S.motion)
            assert np.abs(M[:3, :3] - gt[:3, :3]).max() < 1e-3
            assert np.abs(M[:3, 3] - gt[:3, 3]).max() < 5e-3
            assert S.stats[4] > 0.6 * S.stats[3]


def test_rig_identity_extrinsic_is_the_stereo_spec(synth_frames):
    """One camera with the identity extrinsic: the rig estimator performs the
    single-camera arithmetic exactly (multiplications by 1 and additions of 0)."""
    seq, frames = synth_frames
    p = ol.svo_params(1242, 375, *seq.K, seq.p.baseline)
    E = np.array([[1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0]], np.float64)
    A, B = ol.SvoSequence(p), ol.SvoRigSequence(p, E)
    for l, r in frames[:3]:
        assert A.process(l, r) == B.process([l], [r])
        assert A.stats == B.stats
        assert np.array_equal(A.motion, B.motion)


@pytest.mark.gpu
def test_gpu_rig_matches_oracle(rig_frames):
    """configs[4]: 4 stereo cameras per timestep, one shared RANSAC + GN —
    per-timestep stats, matches, cameras, inlier masks and motion identical to
    the spec; batched device path == per-timestep path."""
    import torch

    from viso_amd import svo
    seq, frames = rig_frames
    E = seq.extrinsics()
    p = svo.default_params(1242, 375, *seq.K, seq.p.baseline)
    vo = svo.VisualOdometryStereoRig(p, E)
    S = ol.SvoRigSequence(ol.svo_params(1242, 375, *seq.K, seq.p.baseline), E)
    for f, (L, R) in enumerate(frames):
        assert vo.process(L, R) == S.process(L, R) == (f > 0)
        assert vo.stats().tolist() == S.stats
        if f > 0:
            uv8, inl = vo.getMatches()
            assert np.array_equal(uv8, S.matches) and np.array_equal(inl, S.inliers)
            assert np.array_equal(vo.getMatchCams(), S.cams)
            assert np.array_equal(vo.getMotion()[:3].ravel(), _T(S.motion)[:3].ravel())
    assert np.allclose(vo.poses, np.array(S.poses), rtol=0, atol=1e-9)
    n = len(frames)
    Ls = [torch.from_numpy(np.stack([fr[0][c] for fr in frames])).cuda() for c in range(4)]
    Rs = [torch.from_numpy(np.stack([fr[1][c] for fr in frames])).cuda() for c in range(4)]
    vb = svo.VisualOdometryStereoRig(p, E)
    vb.process_device([t.data_ptr() for t in Ls], [t.data_ptr() for t in Rs], n, 1242 * 375)
    assert np.array_equal(vb.poses, vo.poses)
    assert vb.stats().tolist() == vo.stats().tolist()
