"""End to end on KITTI-format input: image_0/image_1 PNG pairs + calib.txt on
disk (the layout of the north star's "identical KITTI-format grey pairs",
BASELINE.json configs[0..1]), decoded by the library's own PNG loader
(viso_amd.kitti, include/viso/viso_io.h), then the reference path
(Viso::OnNewFrame, src/viso.cpp:7-145, with the stereo initialisation) and the
north-star stereo VO, each against the CPU oracle on the same decoded pairs.

KITTI itself is absent offline, so the pairs are the synthetic renderer's,
written as 8-bit grey PNGs by PIL at KITTI's native size for sequences 00-02,
1241x376.  That is an odd width and not the bench's
1242x375: every pyramid level, band and strip edge moves.
Bars: as tests/test_pipeline.py and tests/test_svo.py (state and counts
exact, points bit-exact, poses within 1e-10 relative Frobenius; stereo-VO
matches, inliers and motions bit-exact)."""
import os

import numpy as np
import pytest

from tests import oracle_lib

PIL = pytest.importorskip("PIL.Image")

W, H = 1241, 376
N = 8
MAX_DISP = 128


def _rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


@pytest.fixture(scope="module")
def kitti_dir(tmp_path_factory):
    from viso_amd.synth import Sequence
    seq = Sequence(W, H, seed=0)
    root = str(tmp_path_factory.mktemp("kitti") / "sequences" / "00")
    for cam in (0, 1):
        os.makedirs(os.path.join(root, f"image_{cam}"))
        for f in range(N):
            PIL.fromarray(seq.image(f, cam), "L").save(os.path.join(root, f"image_{cam}", f"{f:06d}.png"))
    fx, fy, cx, cy = seq.K
    P0 = [fx, 0, cx, 0, 0, fy, cy, 0, 0, 0, 1, 0]
    P1 = [fx, 0, cx, -fx * seq.p.baseline, 0, fy, cy, 0, 0, 0, 1, 0]
    with open(os.path.join(root, "calib.txt"), "w") as fh:
        for k, P in enumerate((P0, P1, P0, P1)):
            fh.write(f"P{k}: " + " ".join(f"{v:.12e}" for v in P) + "\n")
    return root, seq


def _pairs(root):
    from viso_amd import kitti
    ks = kitti.KittiSequence(root)
    return ks, [ks.frame(f) for f in range(len(ks))]


def test_kitti_native_size_decodes_to_the_rendered_pairs(kitti_dir):
    root, seq = kitti_dir
    ks, pairs = _pairs(root)
    assert (ks.width, ks.height) == (W, H) and len(pairs) == N
    assert np.allclose(ks.K, seq.K, rtol=1e-12) and abs(ks.baseline - seq.p.baseline) < 1e-12
    for f, (l, r) in enumerate(pairs):
        assert np.array_equal(l, seq.image(f, 0)) and np.array_equal(r, seq.image(f, 1))


def test_oracle_kitti_native_size_stereo_init_tracks(kitti_dir):
    root, _ = kitti_dir
    ks, pairs = _pairs(root)
    ov = oracle_lib.Viso(ks.K, W, H, enable_tracking=1)
    ov.set_stereo(ks.baseline, MAX_DISP, 1)
    for l, r in pairs:
        ov.on_new_stereo(l, r)
    assert ov.state == 1 and len(ov.poses()) == N - 1 and len(ov.points()) > 500


@pytest.mark.gpu
def test_gpu_kitti_reference_path_matches_oracle(kitti_dir):
    import viso_amd
    root, _ = kitti_dir
    ks, pairs = _pairs(root)
    gv = viso_amd.Viso(*ks.K, width=W, height=H, enable_tracking=1)
    gv.set_stereo(ks.baseline, MAX_DISP, 1)
    ov = oracle_lib.Viso(ks.K, W, H, enable_tracking=1)
    ov.set_stereo(ks.baseline, MAX_DISP, 1)
    for f, (l, r) in enumerate(pairs):
        gv.process(l, r)
        ov.on_new_stereo(l, r)
        gv.synchronize()
        assert gv.state == ov.state, f
        gs, os_ = gv.stats(), ov.stats()
        assert gs[1] == os_[1] and gs[2] == os_[2] and gs[3] == os_[3], (f, gs, os_)
    assert np.array_equal(gv.GetPoints(), ov.points())
    gP, oP = gv.poses, ov.poses()
    assert gP.shape == oP.shape and len(oP) == N - 1
    assert _rel(gP, oP) < 1e-10


@pytest.mark.gpu
def test_gpu_kitti_stereo_vo_matches_oracle(kitti_dir):
    from viso_amd import svo
    root, _ = kitti_dir
    ks, pairs = _pairs(root)
    vo = svo.VisualOdometryStereo(svo.default_params(W, H, *ks.K, ks.baseline))
    S = oracle_lib.SvoSequence(oracle_lib.svo_params(W, H, *ks.K, ks.baseline))
    for f, (l, r) in enumerate(pairs):
        ok, ok_exp = vo.process(l, r), S.process(l, r)
        assert ok == ok_exp, f
        assert vo.stats().tolist() == S.stats, f
        if f > 0 and ok:
            uv8, inl = vo.getMatches()
            assert np.array_equal(uv8, S.matches) and np.array_equal(inl, S.inliers), f
    assert np.allclose(vo.poses, np.array(S.poses), rtol=0, atol=1e-9)
