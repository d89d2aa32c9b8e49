"""Tolerance mode (viso_params.precision = VISO_PRECISION_FAST): the tracking
stages in fp32 per-pixel arithmetic with fp64 sums (include/viso/viso_c.h),
against the faithful CPU oracle (oracle/, fp64, bit-identical to the
faithful GPU path).

Bars (the north star's): poses within 1e-4 relative Frobenius of the
oracle's, frame by frame, over 200 frames of the bench sequence (stereo
initialised, 1242x375), 80 frames of the monocular bench path and of KITTI's
native 1241x376; the state sequence and the map identical (initialisation is
always faithful); direct-pose nGood within 1% of the oracle's; LK alignment
pairs identical (keyframe choice is fp64) and successes within 1%."""
import numpy as np
import pytest

from tests import oracle_lib

N = 200       # the headline configuration (stereo-initialised 1242x375)
N_OTHER = 80  # the monocular path and KITTI's native size
MAX_DISP = 128


def _rel_rows(a, b):
    return np.linalg.norm(a - b, axis=1) / np.maximum(np.linalg.norm(b, axis=1), 1e-300)


def _run(w, h, stereo, n=N):
    import torch

    import viso_amd
    from viso_amd.synth import Sequence
    seq = Sequence(w, h, seed=0)
    frames = [seq.frame(f) for f in range(n)]
    ov = oracle_lib.Viso(seq.K, w, h, enable_tracking=1)
    gv = viso_amd.Viso(*seq.K, width=w, height=h, enable_tracking=1, batch_frames=50,
                       precision=viso_amd.PRECISION_FAST)
    if stereo:
        ov.set_stereo(seq.p.baseline, MAX_DISP, 1)
        gv.set_stereo(seq.p.baseline, MAX_DISP, 1)
    dl = torch.from_numpy(np.stack([f[0] for f in frames])).cuda()
    dr = torch.from_numpy(np.stack([f[1] for f in frames])).cuda()
    torch.cuda.synchronize()
    gv.process_device(dl.data_ptr(), dr.data_ptr() if stereo else None, n, w * h)
    gv.synchronize()
    ngood_o = []
    for f in range(n):
        if stereo:
            ov.on_new_stereo(*frames[f])
        else:
            ov.on_new_frame(frames[f][0])
        ngood_o.append(ov.stats()[9])
    return gv, ov, ngood_o


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,stereo,n", [(1242, 375, True, N), (1242, 375, False, N_OTHER),
                                         (1241, 376, True, N_OTHER)])
def test_gpu_fast_mode_poses_within_north_star_bar(w, h, stereo, n):
    gv, ov, ngood_o = _run(w, h, stereo, n)
    assert gv.state == ov.state == 1
    assert np.array_equal(gv.GetPoints(), ov.points())  # initialisation is faithful
    gP, oP = gv.poses, ov.poses()
    assert gP.shape == oP.shape and len(oP) >= n - 10
    rel = _rel_rows(gP, oP)
    assert rel.max() < 1e-4, (rel.max(), int(rel.argmax()))
    # the last frame's level-0 statistics and LK alignment
    gs = gv.stats()
    assert abs(gs[9] - ngood_o[-1]) <= 0.01 * ngood_o[-1] + 1
    pk, sc, _, ua = gv.alignment()
    opk, osc, _, oua = ov.alignment()
    assert np.array_equal(pk, opk)
    assert abs(int(sc.sum()) - int(osc.sum())) <= 0.01 * osc.sum() + 1


@pytest.mark.gpu
def test_gpu_fast_mode_default_is_faithful():
    import viso_amd
    p = viso_amd.default_params()
    assert p.precision == viso_amd.PRECISION_FAITHFUL == 0
    with pytest.raises(RuntimeError):
        viso_amd.Viso(500.0, 500.0, 320.0, 240.0, width=640, height=480, precision=7)
