"""Stereo keyframe insertion (viso_set_keyframes, include/viso/viso_c.h):
map maintenance the reference lacks (the reference's
map is frozen after src/viso.cpp:79-96).  The repo's own spec, restated in
oracle/oracle_viso.cpp: every `interval`-th tracking frame whose level-0
direct-pose nGood is below ngood_permille / 1000 of the map adds its stereo
points (world = R^T (Pc - T)) and becomes a keyframe.  Parity unpinned vs the
reference (no counterpart); GPU vs the oracle: states, counts and inserted
points exact, poses within 1e-10 relative Frobenius (as tests/test_pipeline.py).

Sequence: the synthetic renderer with the camera driving forward
(z = 20 sin(2 pi f / 1000) m, ~0.126 m per frame), so the initial map leaves
the view: without insertion level-0 nGood falls from ~2.3k to ~0.9k over
120 frames."""
import numpy as np
import pytest

from tests import oracle_lib

W, H = 1242, 375
N = 120
INTERVAL, PERMILLE = 10, 500


def _seq():
    from viso_amd.synth import Sequence
    return Sequence(W, H, seed=0, z_amp=20.0, z_period=1000.0)


def _T(p12):
    M = np.eye(4)
    M[:3, :3] = np.asarray(p12[:9]).reshape(3, 3)
    M[:3, 3] = p12[9:]
    return M


def _oracle(seq, n, interval=INTERVAL):
    v = oracle_lib.Viso(seq.K, W, H, enable_tracking=1)
    v.set_stereo(seq.p.baseline, 128, 1)
    if interval:
        v.set_keyframes(interval, PERMILLE)
    stats = []
    for f in range(n):
        v.on_new_stereo(*seq.frame(f))
        stats.append(v.stats())
    return v, np.array(stats)


def test_oracle_keyframe_insertion_keeps_the_map_in_view():
    seq = _seq()
    v, st = _oracle(seq, N)
    inserted = np.nonzero(st[:, 14] > 0)[0]
    assert len(inserted) >= 1
    n_init = len(v.points()) - int(st[:, 14].sum())
    for f in inserted:
        # inserted only on a check frame whose nGood fell below the ratio of
        # the map it was tracked against
        n_map_before = n_init + int(st[:f, 14].sum())
        assert st[f, 9] < PERMILLE / 1000 * n_map_before
    assert st[-1, 15] == 1 + len(inserted)
    assert st[5:, 9].min() > 500
    # metric poses follow the renderer's ground truth (camera centres, metres)
    P = v.poses()
    T0inv = np.linalg.inv(_T(seq.pose(0)))
    err = []
    for k, p in enumerate(P):
        G = _T(seq.pose(k + 1)) @ T0inv
        E = _T(p)
        err.append(np.linalg.norm(-G[:3, :3].T @ G[:3, 3] + E[:3, :3].T @ E[:3, 3]))
    assert max(err) < 0.05, max(err)


def test_oracle_keyframes_off_is_the_frozen_map():
    seq = _seq()
    a, sa = _oracle(seq, 40, interval=0)
    b, sb = _oracle(seq, 40, interval=1000)
    assert np.array_equal(a.poses(), b.poses()) and (sa[:, 14] == 0).all()


@pytest.fixture(scope="module")
def oracle_kf():
    """The oracle's 120 frames with insertion, shared by both GPU variants."""
    return _oracle(_seq(), N)


@pytest.mark.gpu
@pytest.mark.parametrize("batched", [False, True])
def test_gpu_keyframe_insertion_matches_oracle(batched, oracle_kf):
    import torch

    import viso_amd
    seq = _seq()
    ov, ost = oracle_kf
    gv = viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=1, batch_frames=32)
    gv.set_stereo(seq.p.baseline, 128, 1)
    gv.set_keyframes(INTERVAL, PERMILLE)
    if batched:
        frames = [seq.frame(f) for f in range(N)]
        dl = torch.from_numpy(np.stack([f[0] for f in frames])).cuda()
        dr = torch.from_numpy(np.stack([f[1] for f in frames])).cuda()
        torch.cuda.synchronize()
        gv.process_device(dl.data_ptr(), dr.data_ptr(), N, W * H)
        gv.synchronize()
        gs = gv.stats()
        assert gs[15] == ost[-1, 15]
    else:
        for f in range(N):
            gv.process(*seq.frame(f))
            gv.synchronize()
            gs, os_ = gv.stats(), ost[f]
            assert gv.state == os_[0], f
            for k in (1, 6, 7, 9, 14, 15):
                assert gs[k] == os_[k], (f, k, gs[k], os_[k])
    assert ost[:, 14].sum() > 0
    gp, op = gv.GetPoints(), ov.points()
    assert gp.shape == op.shape
    assert np.array_equal(gp[:2465], op[:2465])
    assert np.abs(gp - op).max() <= 1e-9 * np.abs(op).max()
    gP, oP = gv.poses, ov.poses()
    assert gP.shape == oP.shape
    rel = np.linalg.norm(gP - oP, axis=1) / np.linalg.norm(oP, axis=1)
    assert rel.max() < 1e-10, rel.max()
