"""The whole per-frame path: FrameHandler::OnNewFrame -> Viso::OnNewFrame
(src/viso.cpp:7-145) on the synthetic KITTI-like sequence, HIP path vs the
oracle frame by frame.

Bars: state, track counts, KLT tracks/success, inlier counts and the map
points' membership are exact; map points and poses within 1e-10 relative
Frobenius (north_star bar: 1e-4; the remaining differences come from device
vs glibc sin/cos/acos in SE3::exp / viewing angles / parallax)."""
import numpy as np
import pytest

from tests import oracle_lib, seqdata

W, H = seqdata.W, seqdata.H


def _rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


# ------------------------------------------------------------------ CPU: oracle sanity
def test_oracle_sequence_initialises_and_tracks():
    d = seqdata.initialised()
    v = d["viso"]
    assert v.state == 1 and len(d["points"]) > 500
    # depth normalisation: mean z of the map = 1 (src/viso.cpp:622-637)
    assert abs(d["points"][:, 2].mean() - 1.0) < 1e-9


def test_oracle_as_shipped_finishes_without_poses():
    seq = seqdata.sequence(0)
    v = oracle_lib.Viso(seq.K, W, H, enable_tracking=0)
    for f in range(d_init_frame() + 3):
        v.on_new_frame(seqdata.image(f))
    # kFinished (src/viso.cpp:97): poses stays empty
    assert v.state == 2 and len(v.poses()) == 0


def d_init_frame():
    return seqdata.initialised()["init_frame"]


def _bg_items(n_frames, n, take=2):
    """track.hip lk_item_kernel's work decomposition, restated: eight heads,
    head x holding points [x seg, (x + 1) seg) of every frame, frames in
    order; dequeues of `take` items; a leftover item published as
    head * per_head + k + 1."""
    seg = (n + 7) // 8
    per_head = n_frames * seg
    seen = []
    for head in range(8):
        last_f = -1
        for k0 in range(0, per_head, take):
            for k in range(k0, min(k0 + take, per_head)):
                f = k // seg
                i = head * seg + (k - f * seg)
                assert f >= last_f  # frames in order within a head
                last_f = f
                e = head * per_head + k + 1  # leftover encoding round trip
                assert ((e - 1) // per_head, (e - 1) % per_head) == (head, k)
                if i < n:
                    seen.append((f, i))
    return seen


@pytest.mark.parametrize("n_frames,n", [(1, 1), (20, 2465), (64, 2465), (3, 7), (5, 8), (2, 5666)])
def test_background_lk_items_cover_every_point_once(n_frames, n):
    """The background LK grid's eight heads cover every (frame, point) of a
    chunk exactly once, with the frames in order within each head, so every
    point's alignment is computed whichever wave (resident or drain) takes it."""
    seen = _bg_items(n_frames, n)
    assert len(seen) == n_frames * n
    assert len(set(seen)) == n_frames * n


def test_oracle_tracking_follows_ground_truth_rotation():
    seq = seqdata.sequence(0)
    v = oracle_lib.Viso(seq.K, W, H, enable_tracking=1)
    n = 16
    for f in range(n):
        v.on_new_frame(seqdata.image(f))
    P = v.poses()
    assert len(P) >= 5
    f_end = n - 1
    # compare the relative rotation between the init keyframe and the last
    # frame with the ground truth (scale-free)
    R_est = P[-1][:9].reshape(3, 3)
    g0 = seq.pose(0)[:9].reshape(3, 3)
    g1 = seq.pose(f_end)[:9].reshape(3, 3)
    R_gt = g1 @ g0.T
    ang = np.degrees(np.arccos(np.clip((np.trace(R_est.T @ R_gt) - 1) / 2, -1, 1)))
    assert ang < 0.5, ang


# ------------------------------------------------------------------ GPU parity
def _run_pair(n_frames, seed=0, enable_tracking=1):
    import viso_amd
    seq = seqdata.sequence(seed)
    K = seq.K
    gv = viso_amd.Viso(*K, width=W, height=H, enable_tracking=enable_tracking)
    ov = oracle_lib.Viso(K, W, H, enable_tracking=enable_tracking)
    return seq, gv, ov


@pytest.mark.gpu
def test_gpu_sequence_parity_frame_by_frame():
    seq, gv, ov = _run_pair(0)
    n_frames = 24
    for f in range(n_frames):
        img = seqdata.image(f)
        gv.OnNewFrame(img)
        ov.on_new_frame(img)
        assert gv.state == ov.state, f
        gs, os_ = gv.stats(), ov.stats()
        assert gs[1] == os_[1], (f, gs, os_)          # tracked points
        assert gs[2] == os_[2], (f, gs, os_)          # nr_inliers
        assert gs[12] == os_[12], (f, gs, os_)        # init on this frame
        if ov.state == 0:
            gk1, gk2, gsu = gv.tracks()
            ok1, ok2, osu = ov.tracks()
            assert np.array_equal(gk1.view(np.uint32), ok1.view(np.uint32)), f
            assert np.array_equal(gk2.view(np.uint32), ok2.view(np.uint32)), f
            assert np.array_equal(gsu, osu), f
        else:
            assert gs[6] == os_[6] and gs[7] == os_[7], (f, gs, os_)  # LK pairs / successes
    gp, op = gv.GetPoints(), ov.points()
    assert gp.shape == op.shape and len(op) > 0
    assert _rel(gp, op) < 1e-10
    gP, oP = gv.poses, ov.poses()
    assert gP.shape == oP.shape and len(oP) > 0
    for i in range(len(oP)):
        assert _rel(gP[i], oP[i]) < 1e-10, (i, gP[i], oP[i])
    pk, sc, ub, ua = gv.alignment()
    opk, osc, oub, oua = ov.alignment()
    assert np.array_equal(pk, opk) and np.array_equal(sc, osc)
    assert np.max(np.abs(ua - oua)) < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["0", "1"])
def test_gpu_init_gate_speculation_paths_agree(mode, monkeypatch):
    """The initialisation's 2D-2D gate read (frame.hip): the H hypotheses
    launched behind the gate before the host reads it (H chain on the context
    stream, E chain on lk_stream) or after it (H chain on lk_stream) — forced
    never (0) / always (1) against the default prediction, which takes both
    paths on this sequence: every frame's counts, the tracks, the map and the
    poses bit for bit."""
    import viso_amd
    seq = seqdata.sequence(0)
    n = d_init_frame() + 3

    def run():
        v = viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=1)
        rows = []
        for f in range(n):
            v.OnNewFrame(seqdata.image(f))
            st = v.stats()
            rows.append((v.state, st[1], st[2], st[3], st[4], st[8], st[12]))
        return rows, v.GetPoints(), v.poses

    ref = run()
    monkeypatch.setenv("VISO_GATE_SPEC", mode)
    got = run()
    assert got[0] == ref[0]
    assert np.array_equal(got[1], ref[1]) and len(ref[1]) > 0
    assert np.array_equal(got[2], ref[2]) and len(ref[2]) > 0


@pytest.mark.gpu
def test_gpu_host_ingest_slot_reuse():
    """Host frames go up on their own stream (frame.hip upload_host): a
    slot's reuse waits for the ingest call that freed it (its epoch event)
    and for its LK batch.  With batch_frames=1 the pool has 10 slots, so
    slots are reused every few frames — the poses, the map and the last LK
    alignment equal a run whose pool never wraps (batch_frames=128), bit for
    bit."""
    import viso_amd
    seq = seqdata.sequence(0)
    n = d_init_frame() + 30

    def run(batch):
        v = viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=1, batch_frames=batch)
        for f in range(n):
            v.OnNewFrame(seqdata.image(f))
        v.synchronize()
        return v.poses, v.GetPoints(), v.alignment()

    ref = run(128)
    got = run(1)
    assert len(ref[0]) >= 25 and np.array_equal(got[0], ref[0])
    assert np.array_equal(got[1], ref[1])
    for a, b in zip(got[2], ref[2]):
        assert np.array_equal(a, b)


_HQ = {}


def _host_queue_oracle(n):
    """The oracle over the bench sequence (stereo init at frame 0, n - 1
    tracking frames): per-frame (nGood, cost, LK pairs, LK successes)."""
    if n not in _HQ:
        from viso_amd.synth import Sequence
        seq = Sequence(1242, 375, seed=0)
        left = [seq.image(f, 0) for f in range(n)]
        right0 = seq.image(0, 1)
        ov = oracle_lib.Viso(seq.K, 1242, 375, enable_tracking=1)
        ov.set_stereo(seq.p.baseline, 128, 1)
        ov.on_new_stereo(left[0], right0)
        log = []
        for f in range(1, n):
            ov.on_new_frame(left[f])
            s = ov.stats()
            log.append((s[9], s[10], s[6], s[7]))
        _HQ[n] = (seq, left, right0, ov.poses(), ov.points(), np.array(log), ov.alignment())
    return _HQ[n]


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", ["16", "3", "0"])
def test_gpu_host_frames_queued_match_oracle(chunk, monkeypatch):
    """The drop-in's calling pattern (FrameSequence::RunOnce -> OnNewFrame,
    include/frame_sequence.h:25-38) in a burst: frame 0's stereo pair, then
    40 viso_process_frame calls with nothing read in between, so tracking
    frames queue and run as chunks of up to VISO_HOST_CHUNK frames (16, the
    default; 3; 0 = the frame-by-frame path).  Poses, the map, the per-frame
    log (level-0 nGood / cost, LK pairs / successes of every frame) and the
    last alignment equal the oracle's."""
    import viso_amd
    monkeypatch.setenv("VISO_HOST_CHUNK", chunk)
    n = 41
    seq, left, right0, oP, op, olog, oal = _host_queue_oracle(n)
    v = viso_amd.Viso(*seq.K, width=1242, height=375, enable_tracking=1)
    v.set_stereo(seq.p.baseline, 128, 1)
    v.set_frame_log(True)
    v.process(left[0], right0)
    for f in range(1, n):
        v.OnNewFrame(left[f])
    v.synchronize()
    gP, glog = v.poses, v.frame_log()
    assert gP.shape == oP.shape == (n - 1, 12)
    assert np.linalg.norm(gP - oP, axis=1).max() <= 1e-10 * np.linalg.norm(oP, axis=1).max()
    assert np.array_equal(v.GetPoints(), op)
    assert np.array_equal(glog[:, [0, 2, 3]], olog[:, [0, 2, 3]])
    assert (np.abs(glog[:, 1] - olog[:, 1]) <= 1e-10 * np.abs(olog[:, 1])).all()
    pk, sc, ub, ua = v.alignment()
    assert np.array_equal(pk, oal[0]) and np.array_equal(sc, oal[1])
    assert np.max(np.abs(ua - oal[3])) < 1e-6
    v.close()


@pytest.mark.gpu
def test_gpu_as_shipped_mode():
    seq, gv, ov = _run_pair(0, enable_tracking=0)
    for f in range(d_init_frame() + 3):
        img = seqdata.image(f)
        gv.OnNewFrame(img)
        ov.on_new_frame(img)
    assert gv.state == ov.state == 2
    assert len(gv.poses) == 0
    assert _rel(gv.GetPoints(), ov.points()) < 1e-10


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [5, 2])
def test_gpu_batched_device_ingest_matches_per_frame(batch):
    """viso_process_frames_device in chunks of `batch` frames equals
    frame-by-frame host ingest; batch 2 makes a 12-slot pool that wraps
    within the 14 frames (slot reuse behind the pyramid's own level-0 copy of
    each chunk's last frame, PyrOwn)."""
    import torch

    import viso_amd
    seq = seqdata.sequence(0)
    n = 14
    frames = np.stack([seqdata.image(f) for f in range(n)])
    rights = np.stack([seqdata.image(f, cam=1) for f in range(n)])
    ref = viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=1)
    for f in range(n):
        ref.OnNewFrame(frames[f])
    dl = torch.from_numpy(frames).cuda()
    dr = torch.from_numpy(rights).cuda()
    torch.cuda.synchronize()
    bat = viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=1, batch_frames=batch)
    bat.process_device(dl.data_ptr(), dr.data_ptr(), n, W * H)
    bat.synchronize()
    assert bat.state == ref.state
    assert np.array_equal(bat.poses, ref.poses)
    assert np.array_equal(bat.GetPoints(), ref.GetPoints())


@pytest.mark.gpu
def test_gpu_stereo_facade_uses_left():
    import viso_amd
    seq = seqdata.sequence(0)
    a = viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=1)
    b = viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=1)
    for f in range(d_init_frame() + 3):
        left, right = seqdata.image(f), seqdata.image(f, cam=1)
        a.process(left, right)
        b.OnNewFrame(left)
    assert np.array_equal(a.poses, b.poses)


# ------------------------------------------------------------------ configs[2] size
W2, H2 = 1920, 1080
# renderer texture scale giving ~8k FAST@50 corners on frame 0 (BASELINE.json
# configs[2]: "~8k features/frame"; 8,215 on frame 0)
BLOCK_1080 = 0.35


@pytest.mark.gpu
def test_gpu_1080p_reference_path_frame_by_frame():
    """BASELINE.json configs[2] on the reference path: Viso::OnNewFrame at
    1920x1080 with ~8k FAST corners, the monocular initialisation (KLT over
    ~8k tracks, E-RANSAC 1000 + H-RANSAC 2000 hypotheses, SelectMotion over
    five candidates, map of ~5.7k points), then tracking (direct pose + LK
    alignment), GPU vs oracle frame by frame with the bars of
    test_gpu_sequence_parity_frame_by_frame."""
    import viso_amd
    from viso_amd.synth import Sequence
    seq = Sequence(W2, H2, seed=0, block_m=BLOCK_1080)
    gv = viso_amd.Viso(*seq.K, width=W2, height=H2, enable_tracking=1)
    ov = oracle_lib.Viso(seq.K, W2, H2, enable_tracking=1)
    states = []
    for f in range(10):
        img = seq.image(f)
        gv.OnNewFrame(img)
        ov.on_new_frame(img)
        assert gv.state == ov.state, f
        gs, os_ = gv.stats(), ov.stats()
        if f == 0:
            assert os_[1] > 7500  # ~8k FAST corners
        for k in (1, 2, 3, 4, 12):  # tracks, inliers, best motion, candidates, init
            assert gs[k] == os_[k], (f, k, gs, os_)
        if ov.state == 0:
            gk1, gk2, gsu = gv.tracks()
            ok1, ok2, osu = ov.tracks()
            assert np.array_equal(gk1.view(np.uint32), ok1.view(np.uint32)), f
            assert np.array_equal(gk2.view(np.uint32), ok2.view(np.uint32)), f
            assert np.array_equal(gsu, osu), f
        else:
            assert gs[6] == os_[6] and gs[7] == os_[7], (f, gs, os_)  # LK pairs / successes
            assert gs[9] == os_[9], (f, gs[9], os_[9])  # direct nGood
        states.append(ov.state)
    assert states.count(1) >= 4
    gp, op = gv.GetPoints(), ov.points()
    assert gp.shape == op.shape and len(op) > 5000
    assert _rel(gp, op) < 1e-10
    gP, oP = gv.poses, ov.poses()
    assert gP.shape == oP.shape and len(oP) >= 4
    for i in range(len(oP)):
        assert _rel(gP[i], oP[i]) < 1e-10, (i, gP[i], oP[i])
    pk, sc, ub, ua = gv.alignment()
    opk, osc, oub, oua = ov.alignment()
    assert np.array_equal(pk, opk) and np.array_equal(sc, osc)
    assert np.max(np.abs(ua - oua)) < 1e-6
