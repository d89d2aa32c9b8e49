"""Multi-camera photometric rig on the reference path (SURVEY.md §8(f) row 3,
BASELINE.json configs[4]; include/viso/viso_rig.h, spec oracle/oracle_rig.cpp).

The reference tracks one camera; the rig runs its per-level photometric
Gauss-Newton (DirectPoseEstimationSingleLayer, src/viso.cpp:661-758) per
camera at E_c T and sums the cameras' H, b (src/viso.cpp:682-729) through
Ad(E_c).  Parity unpinned vs the reference (no rig there): the oracle is the
repo's own restatement, itself pinned by (a) the adjoint identity
E exp(xi) T = exp(Ad(E) xi) E T, (b) a one-camera identity-extrinsic rig
reproducing the single-camera direct pose bit for bit, and (c) the
renderer's ground truth.  GPU bars: faithful precision bit-exact map and
poses <= 1e-10 rel (observed identical); tolerance mode (FAST: fp32 per
pixel, fp16 `last` patch in LDS, LDL^T solve) poses <= 1e-4 rel Frobenius.
"""
import numpy as np
import pytest

from tests import oracle_lib

W, H = 1242, 375
N_CAMS = 4
STEPS = 6  # initialisation + 5 tracking timesteps


def _rel(a, b):
    return np.linalg.norm(a - b, axis=-1) / np.maximum(np.linalg.norm(b, axis=-1), 1e-300)


def _inv(T):
    R = T[:9].reshape(3, 3)
    out = np.zeros(12)
    out[:9] = R.T.reshape(-1)
    out[9:] = -R.T @ T[9:]
    return out


def _mul(A, B):
    RA, RB = A[:9].reshape(3, 3), B[:9].reshape(3, 3)
    out = np.zeros(12)
    out[:9] = (RA @ RB).reshape(-1)
    out[9:] = RA @ B[9:] + A[9:]
    return out


def test_rig_adjoint_moves_cameras_consistently():
    """E exp(xi) T == exp(Ad(E) xi) (E T): the perturbation convention of
    dPixeldXi (translation first) carried through the extrinsic."""
    lib = oracle_lib.load()
    from viso_amd.synth import RigSequence
    E_all = RigSequence(W, H, n_cams=N_CAMS).extrinsics()
    rng = np.random.default_rng(3)
    T = np.zeros(12)  # a random rig pose
    lib.oracle_se3_exp_left(oracle_lib.ptr(rng.normal(0, 0.2, 6)),
                            oracle_lib.ptr(np.array([1.0, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0])), oracle_lib.ptr(T))
    for E in E_all:
        Ad = oracle_lib.rig_adjoint(E)
        xi = rng.normal(0, 0.05, 6)
        left = np.zeros(12)
        lib.oracle_se3_exp_left(oracle_lib.ptr(xi), oracle_lib.ptr(T), oracle_lib.ptr(left))
        lhs = oracle_lib.rig_compose(E, left)
        rhs = np.zeros(12)
        lib.oracle_se3_exp_left(oracle_lib.ptr(Ad @ xi), oracle_lib.ptr(oracle_lib.rig_compose(E, T)),
                                oracle_lib.ptr(rhs))
        assert np.abs(lhs - rhs).max() < 1e-12


def test_rig_one_camera_identity_is_the_direct_pose():
    """A one-camera rig with the identity extrinsic is the single-camera
    direct pose (src/viso.cpp:760-766) bit for bit."""
    from viso_amd.synth import Sequence
    seq = Sequence(W, H, seed=0)
    f0, f1 = seq.image(0, 0), seq.image(1, 0)
    p0, p1 = oracle_lib.pyramid(f0), oracle_lib.pyramid(f1)
    xs, ys, _ = oracle_lib.fast(f0, 50)
    pts = oracle_lib.stereo_points(f0, seq.image(0, 1), xs, ys, 128, 1, seq.K, seq.p.baseline)
    I12 = np.array([1.0, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0])
    pose_rig, _ = oracle_lib.rig_direct([p0], [p1], W, H, seq.K, [pts], I12[None], I12[None], I12)
    pose_one = oracle_lib.direct_pose(p0, p1, W, H, seq.K, pts, I12, I12)
    assert np.array_equal(pose_rig, pose_one)


def _rig_seq():
    from viso_amd.synth import RigSequence
    seq = RigSequence(W, H, seed=0, n_cams=N_CAMS)
    frames = [seq.frame(f) for f in range(STEPS)]
    return seq, frames


@pytest.fixture(scope="module")
def oracle_run():
    seq, frames = _rig_seq()
    r = oracle_lib.Rig(seq.K, W, H, seq.extrinsics(), seq.p.baseline)
    stats = []
    for ls, rs in frames:
        r.process(ls, rs)
        stats.append(r.level_stats())
    return seq, frames, r, stats


def test_rig_oracle_tracks_ground_truth(oracle_run):
    seq, frames, r, _ = oracle_run
    assert r.state == 1
    P = r.poses
    assert len(P) == STEPS - 1
    g0 = seq.rig_pose(0)
    for f in range(1, STEPS):
        rel_gt = _mul(seq.rig_pose(f), _inv(g0))  # world(frame 0 rig) -> rig at f
        assert np.abs(P[f - 1][9:] - rel_gt[9:]).max() < 2e-3, f
        assert np.abs(P[f - 1][:9] - rel_gt[:9]).max() < 2e-3, f


def _gpu_rig(seq, frames, precision, device_ingest):
    import torch

    import viso_amd
    from viso_amd.rig import VisoRig
    g = VisoRig(*seq.K, W, H, seq.extrinsics(), precision=precision)
    g.set_stereo(seq.p.baseline, 128, 1)
    if device_ingest:
        dl = torch.from_numpy(np.stack([im for ls, _ in frames for im in ls])).cuda()
        dr = torch.from_numpy(np.stack([im for _, rs in frames for im in rs])).cuda()
        torch.cuda.synchronize()
        g.process_device(dl.data_ptr(), dr.data_ptr(), len(frames), W * H)
        g.synchronize()
        del dl, dr
    else:
        for ls, rs in frames:
            g.process(ls, rs)
    return g


@pytest.mark.gpu
@pytest.mark.parametrize("device_ingest", [False, True])
def test_gpu_rig_faithful_matches_oracle(oracle_run, device_ingest):
    import viso_amd
    seq, frames, r, stats = oracle_run
    g = _gpu_rig(seq, frames, viso_amd.PRECISION_FAITHFUL, device_ingest)
    assert g.state == r.state == 1
    for c in range(N_CAMS):
        assert np.array_equal(g.points(c), r.points(c)), c
    gP, oP = g.poses, r.poses
    assert gP.shape == oP.shape
    assert _rel(gP, oP).max() <= 1e-10
    gs, os_ = g.level_stats(), stats[-1]
    assert np.array_equal(gs[:, 0], os_[:, 0])  # nGood per level
    np.testing.assert_allclose(gs[:, 2:50], os_[:, 2:50], rtol=1e-9, atol=1e-9)


@pytest.mark.gpu
def test_gpu_rig_fast_within_north_star_bar(oracle_run):
    import viso_amd
    seq, frames, r, _ = oracle_run
    g = _gpu_rig(seq, frames, viso_amd.PRECISION_FAST, True)
    assert g.state == 1
    rel = _rel(g.poses, r.poses)
    assert rel.max() < 1e-4, rel


@pytest.mark.gpu
def test_gpu_rig_rejects_bad_arguments():
    import viso_amd
    from viso_amd.rig import VisoRig
    E = np.tile(np.array([1.0, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0]), (5, 1))
    with pytest.raises(RuntimeError):
        VisoRig(500.0, 500.0, 320.0, 240.0, 640, 480, E)  # 5 > VISO_RIG_MAX_CAMS
    g = VisoRig(500.0, 500.0, 320.0, 240.0, 640, 480, E[:2])
    with pytest.raises(RuntimeError):
        g.set_stereo(-1.0)
    # no stereo set: the rig stays initialising
    img = np.zeros((480, 640), np.uint8)
    g.process([img, img], [img, img])
    assert g.state == viso_amd._lib.STATE_INITIALIZATION
    assert len(g.poses) == 0


@pytest.fixture(scope="module")
def dense_rig_run():
    """Two cameras at FAST threshold 20: > 4096 map points per camera, so a
    camera spans more than 64 tiles of the largest tile size (64 points)."""
    from viso_amd.synth import RigSequence
    seq = RigSequence(W, H, seed=0, n_cams=2)
    frames = [seq.frame(f) for f in range(3)]
    r = oracle_lib.Rig(seq.K, W, H, seq.extrinsics(), seq.p.baseline, fast_thresh=20)
    stats = []
    for ls, rs in frames:
        r.process(ls, rs)
        stats.append(r.level_stats())
    return seq, frames, r, stats


def test_dense_rig_oracle_has_cameras_past_4096_points(dense_rig_run):
    _, _, r, _ = dense_rig_run
    assert r.state == 1
    assert min(len(r.points(c)) for c in range(2)) > 4096


@pytest.mark.gpu
@pytest.mark.parametrize("precision,device_ingest", [("faithful", False), ("faithful", True), ("fast", False)])
def test_gpu_rig_past_4096_points_per_camera(dense_rig_run, precision, device_ingest):
    """Cameras past 4096 points (tiles must stay <= 64 points):
    faithful bit-exact map / nGood and poses <= 1e-10; tolerance mode <= 1e-4.
    With device ingest the timesteps run in one call, so every
    timestep's final solve is merged into the next one's L(3) with cameras of
    more than one reduce wave."""
    import torch

    import viso_amd
    from viso_amd.rig import VisoRig
    seq, frames, r, stats = dense_rig_run
    prec = viso_amd.PRECISION_FAITHFUL if precision == "faithful" else viso_amd.PRECISION_FAST
    g = VisoRig(*seq.K, W, H, seq.extrinsics(), precision=prec, fast_thresh=20)
    g.set_stereo(seq.p.baseline, 128, 1)
    if device_ingest:
        dl = torch.from_numpy(np.stack([im for ls, _ in frames for im in ls])).cuda()
        dr = torch.from_numpy(np.stack([im for _, rs in frames for im in rs])).cuda()
        torch.cuda.synchronize()
        g.process_device(dl.data_ptr(), dr.data_ptr(), len(frames), W * H)
        g.synchronize()
        del dl, dr
    else:
        for ls, rs in frames:
            g.process(ls, rs)
    torch.cuda.synchronize()
    assert g.state == r.state == 1
    for c in range(2):
        assert np.array_equal(g.points(c), r.points(c)), c
    rel = _rel(g.poses, r.poses)
    if precision == "faithful":
        assert rel.max() <= 1e-10, rel
        assert np.array_equal(g.level_stats()[:, 0], stats[-1][:, 0])
    else:
        assert rel.max() < 1e-4, rel
