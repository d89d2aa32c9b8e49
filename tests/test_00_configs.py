"""One GPU-vs-oracle test per BASELINE.json GPU config, collected first.

The driver runs ``pytest tests/ -x -q -m gpu``; this file sorts first, so the
four configs are exercised (and recorded) before anything else.  Each test is
bounded to ~20 s of box time.

* configs[1] — the headline's workload exactly: the bench's stereo-
  initialised 1242x375 sequence (seed = rank 0), batched device ingest at the
  driver's --warmup 5 / --steps 20, every pose, the map and the LK alignment
  outputs against the oracle (src/viso.cpp:7-145, 661-925).
* configs[2] — 1920x1080 with ~8k FAST corners: the reference path from frame
  0 (FAST, KLT, E-1000 / H-2000 RANSAC + SelectMotion, map creation,
  src/viso.cpp:14-111) and two tracking frames, frame by frame; plus one
  2048-hypothesis stereo-VO pair against the repo's spec.
* configs[3] — bench.py's N>1 path: two ranks under torch.distributed.run
  (gloo, sharing the box's one GPU) whose gathered pose logs equal the
  oracle's for each rank's own sequence, and the RCCL (nccl) process group at
  one rank gathering the log.
* configs[4] — the 4-camera rig: the photometric rig on the reference path
  (faithful, bit-exact vs oracle/oracle_rig.cpp) and the stereo-VO rig with one
  shared RANSAC + Gauss-Newton (vs oracle/oracle_svo.cpp).
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from tests import oracle_lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STEREO_MAX_DISP = 128  # bench.py


def _rel_rows(a, b):
    return np.linalg.norm(a - b, axis=1) / np.maximum(np.linalg.norm(b, axis=1), 1e-300)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _oracle_stereo_poses(seed, n, W=1242, H=375):
    """The oracle on bench.py's sequence of rank `seed`: stereo init at frame 0,
    then tracking; poses of frames 1..n-1 (one per tracking frame)."""
    from viso_amd.synth import Sequence
    seq = Sequence(W, H, seed=seed)
    ov = oracle_lib.Viso(seq.K, W, H, enable_tracking=1)
    ov.set_stereo(seq.p.baseline, STEREO_MAX_DISP, 1)
    for f in range(n):
        ov.on_new_stereo(seq.image(f, 0), seq.image(f, 1))
    return ov


# ------------------------------------------------------------------ configs[1]
_C1 = dict(W=1242, H=375, warm=5, steps=20)

# bench.py's default line: --warmup 20 (one call; frame 0's stereo pair
# creates the map), then --steps 256 in --batch 128 calls
_C1L = dict(W=1242, H=375, warm=20, steps=256, batch=128)


@pytest.mark.gpu
def test_gpu_config1_200_frames_faithful():
    """configs[1] at (beyond) its stated length, "first 200 stereo pairs": the
    bench's default workload frame for frame — 20 warm-up frames in one call
    (stereo initialisation at frame 0, then 19 tracking frames whose LK
    alignment runs batched after the chain), then 256 tracking frames in two
    128-frame calls, each cut into 64-frame chunks with the chunk-resident
    background LK grid; 276 frames through a pool of 2 x 128 + 8 = 264 slots,
    so slots are reused.  The reference loop (src/viso.cpp:113-138) against
    the oracle, faithful: every pose <= 1e-10 rel (north star: 1e-4), the map
    exact, and per frame (viso_set_frame_log) the level-0 direct-pose nGood
    and cost, LK pairs and LK successes exactly as the oracle's per-frame
    stats; the last frame's alignment exact; the background grid's error word
    clear (synchronize raises it otherwise)."""
    import torch

    import viso_amd
    from viso_amd.shard import sequence_seed
    from viso_amd.synth import Sequence
    W, H, warm, steps, B = _C1L["W"], _C1L["H"], _C1L["warm"], _C1L["steps"], _C1L["batch"]
    n = warm + steps
    seq = Sequence(W, H, seed=sequence_seed(0))
    left = np.stack([seq.image(f, 0) for f in range(n)])
    right = np.stack([seq.image(f, 1) for f in range(warm)])
    # the GPU first (the oracle's 276 frames follow on the host)
    dl, dr = torch.from_numpy(left).cuda(), torch.from_numpy(right).cuda()
    torch.cuda.synchronize()
    fb = W * H
    v = viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=1, batch_frames=B, max_poses=1024)
    v.set_stereo(seq.p.baseline, STEREO_MAX_DISP, 1)
    v.set_frame_log(True)
    assert v.config()["slots"] == 2 * B + 8 < n
    v.process_device(dl.data_ptr(), dr.data_ptr(), warm, fb)
    v.synchronize()
    assert v.state == 1
    f = warm
    while f < n:
        m = min(B, n - f)
        v.process_device(dl.data_ptr() + f * fb, None, m, fb)
        f += m
    v.synchronize()
    gP, gp, glog, gal = v.poses, v.GetPoints(), v.frame_log(), v.alignment()
    assert v.config()["background_lk"] == 1
    v.close()
    # the oracle, frame by frame
    ov = oracle_lib.Viso(seq.K, W, H, enable_tracking=1)
    ov.set_stereo(seq.p.baseline, STEREO_MAX_DISP, 1)
    ov.on_new_stereo(left[0], right[0])
    olog = []
    for f in range(1, n):
        ov.on_new_frame(left[f])
        s = ov.stats()
        olog.append((s[9], s[10], s[6], s[7]))
    olog = np.array(olog)
    assert ov.state == 1
    op, oP = ov.points(), ov.poses()
    assert len(op) > 2000 and np.array_equal(gp, op)
    assert gP.shape == oP.shape == (n - 1, 12)
    assert _rel_rows(gP, oP).max() <= 1e-10
    assert glog.shape == olog.shape == (n - 1, 4)
    assert np.array_equal(glog[:, 0], olog[:, 0]), np.nonzero(glog[:, 0] != olog[:, 0])
    assert np.array_equal(glog[:, 2], olog[:, 2]), np.nonzero(glog[:, 2] != olog[:, 2])
    assert np.array_equal(glog[:, 3], olog[:, 3]), np.nonzero(glog[:, 3] != olog[:, 3])
    assert (np.abs(glog[:, 1] - olog[:, 1]) <= 1e-10 * np.abs(olog[:, 1])).all()
    assert (olog[:, 2] > 0).all()  # every tracking frame aligned points
    pk, sc, ub, ua = gal
    opk, osc, oub, oua = ov.alignment()
    assert np.array_equal(pk, opk) and np.array_equal(sc, osc)
    assert np.max(np.abs(ua - oua)) < 1e-6


def _config1_oracle():
    """The oracle's run of the config-1 workload (cached: the LK-mode variants
    below compare against the same run)."""
    if "oracle" not in _C1:
        from viso_amd.shard import sequence_seed
        from viso_amd.synth import Sequence
        W, H, n = _C1["W"], _C1["H"], _C1["warm"] + _C1["steps"]
        seq = Sequence(W, H, seed=sequence_seed(0))
        left = np.stack([seq.image(f, 0) for f in range(n)])
        right = np.stack([seq.image(f, 1) for f in range(n)])
        ov = oracle_lib.Viso(seq.K, W, H, enable_tracking=1)
        ov.set_stereo(seq.p.baseline, STEREO_MAX_DISP, 1)
        for f in range(n):
            ov.on_new_stereo(left[f], right[f])
        _C1.update(seq=seq, left=left, right=right,
                   oracle=dict(state=ov.state, points=ov.points(), poses=ov.poses(), stats=ov.stats(),
                               alignment=ov.alignment()))
    return _C1["oracle"]


@pytest.mark.gpu
@pytest.mark.parametrize("lk", ["background", "leftovers", "shared-queue", "batched"])
def test_gpu_config1_bench_workload_matches_oracle(lk, monkeypatch):
    """bench.py --warmup 5 --steps 20 on one GPU, as the driver runs it: 5
    warm-up frames (frame 0's stereo pair creates the map), then one 20-frame
    chunk through viso_process_frames_device.  Every pose, the map, the last
    frame's direct-pose nGood and LK alignment against the oracle.  LK
    alignment of the chunk in each of its forms: the chunk-
    resident background grid (the product), the same with the resident waves'
    patience cut to 1 us so the leftover list and the drain carry most items,
    the side stream as a plain stream (VISO_LK_QUEUE=shared), which can put
    the resident grid on the context stream's hardware queue in front of the
    chain it waits for (the round-4 failure, DESIGN.md §5: its waves time
    out, hand their items to the leftover list and leave; the drain runs
    them), and the batched launch after the chain (VISO_LK_BG=0).  A wait
    that ran out sets the grid's error word, which v.synchronize() and the LK
    getters raise, so parity here also means bg_err == 0."""
    import torch

    import viso_amd
    if lk == "leftovers":
        monkeypatch.setenv("VISO_LK_BG_IDLE_US", "1")
    if lk == "batched":
        monkeypatch.setenv("VISO_LK_BG", "0")
    if lk == "shared-queue":
        monkeypatch.setenv("VISO_LK_QUEUE", "shared")
    o = _config1_oracle()
    seq, left, right = _C1["seq"], _C1["left"], _C1["right"]
    W, H, warm, steps = _C1["W"], _C1["H"], _C1["warm"], _C1["steps"]
    n = warm + steps
    dl, dr = torch.from_numpy(left).cuda(), torch.from_numpy(right).cuda()
    torch.cuda.synchronize()
    v = viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=1, batch_frames=128)
    v.set_stereo(seq.p.baseline, STEREO_MAX_DISP, 1)
    fb = W * H
    v.process_device(dl.data_ptr(), dr.data_ptr(), warm, fb)
    v.synchronize()
    assert v.state == 1
    v.process_device(dl.data_ptr() + warm * fb, dr.data_ptr() + warm * fb, steps, fb)
    v.synchronize()
    assert v.state == o["state"] == 1
    gp, op = v.GetPoints(), o["points"]
    assert len(op) > 2000 and np.array_equal(gp, op)
    gP, oP = v.poses, o["poses"]
    assert gP.shape == oP.shape == (n - 1, 12)
    assert _rel_rows(gP, oP).max() <= 1e-10  # north star: 1e-4
    gs, os_ = v.stats(), o["stats"]
    for k in (6, 7, 9):  # LK pairs, LK successes, direct nGood (level 0)
        assert gs[k] == os_[k], (k, gs, os_)
    pk, sc, ub, ua = v.alignment()
    opk, osc, oub, oua = o["alignment"]
    assert np.array_equal(pk, opk) and np.array_equal(sc, osc)
    assert np.max(np.abs(ua - oua)) < 1e-6


@pytest.mark.gpu
def test_gpu_background_lk_error_reaches_host(monkeypatch):
    """A background LK wait that fails sets the grid's error word and its
    pinned host copy from the failing wave itself (no copy behind the chunk):
    v.synchronize() raises it (VISO_ERR_HIP), once — the word is cleared, and
    the next chunk, without the fault, synchronises cleanly with the poses of
    an uninterrupted run.  The fault is injected (VISO_LK_BG_INJECT_FAIL: the
    drain's first wave reports a failed wait)."""
    import torch

    import viso_amd
    from viso_amd._lib import VisoError
    _config1_oracle()  # (the sequence's frames)
    seq, left, right = _C1["seq"], _C1["left"], _C1["right"]
    W, H, warm, steps = _C1["W"], _C1["H"], _C1["warm"], _C1["steps"]
    dl, dr = torch.from_numpy(left).cuda(), torch.from_numpy(right).cuda()
    torch.cuda.synchronize()
    fb = W * H
    half = steps // 2

    def run(inject):
        v = viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=1, batch_frames=128)
        v.set_stereo(seq.p.baseline, STEREO_MAX_DISP, 1)
        v.process_device(dl.data_ptr(), dr.data_ptr(), warm, fb)
        v.synchronize()
        if inject:
            monkeypatch.setenv("VISO_LK_BG_INJECT_FAIL", "1")
        v.process_device(dl.data_ptr() + warm * fb, dr.data_ptr() + warm * fb, half, fb)
        if inject:
            with pytest.raises(VisoError) as e:
                v.synchronize()
            assert e.value.rc == -2  # VISO_ERR_HIP
            monkeypatch.delenv("VISO_LK_BG_INJECT_FAIL")
            v.synchronize()  # reported once
        else:
            v.synchronize()
        f0 = warm + half
        v.process_device(dl.data_ptr() + f0 * fb, dr.data_ptr() + f0 * fb, steps - half, fb)
        v.synchronize()
        return v.poses

    ref = run(False)
    got = run(True)
    assert len(ref) == warm + steps - 1 and np.array_equal(got, ref)


# ------------------------------------------------------------------ configs[2]
@pytest.mark.gpu
def test_gpu_config2_1080p_reference_init_and_tracking():
    """1920x1080, ~8k FAST corners: the reference path from frame 0 through the
    monocular initialisation (the RANSAC frame's inlier mask bit for bit) and
    two tracking frames; one 2048-hypothesis stereo-VO pair vs the spec."""
    from viso_amd import svo
    import viso_amd
    from viso_amd.synth import Sequence
    W, H = 1920, 1080
    seq = Sequence(W, H, seed=0, block_m=0.35)
    gv = viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=1)
    ov = oracle_lib.Viso(seq.K, W, H, enable_tracking=1)
    tracking, ransac_frames, f = 0, 0, 0
    while tracking < 2:
        img = seq.image(f)
        gv.OnNewFrame(img)
        ov.on_new_frame(img)
        assert gv.state == ov.state, f
        gs, os_ = gv.stats(), ov.stats()
        if f == 0:
            assert os_[1] > 7500  # ~8k FAST corners
        for k in (1, 2, 3, 4, 12):  # tracks, inliers, best motion, candidates, init
            assert gs[k] == os_[k], (f, k, gs, os_)
        if f > 0 and (os_[12] or ov.state == 0):
            gk1, gk2, gsu = gv.tracks()
            ok1, ok2, osu = ov.tracks()
            assert np.array_equal(gk2.view(np.uint32), ok2.view(np.uint32)), f
            assert np.array_equal(gsu, osu), f  # init_.success = SelectMotion's inliers
            ransac_frames += int(os_[2] > 0)
        if ov.state == 1 and not os_[12]:
            tracking += 1
            assert gs[9] == os_[9] and gs[6] == os_[6] and gs[7] == os_[7], (f, gs, os_)
        f += 1
        assert f < 12
    assert ransac_frames >= 1
    gp, op = gv.GetPoints(), ov.points()
    assert len(op) > 5000 and gp.shape == op.shape
    assert np.linalg.norm(gp - op) / np.linalg.norm(op) < 1e-10
    assert _rel_rows(gv.poses, ov.poses()).max() < 1e-10
    # configs[2]'s 2048 RANSAC hypotheses on the north-star stereo VO
    kw = dict(ransac_iters=2048)
    p = svo.default_params(W, H, *seq.K, seq.p.baseline, **kw)
    vo = svo.VisualOdometryStereo(p)
    S = oracle_lib.SvoSequence(oracle_lib.svo_params(W, H, *seq.K, seq.p.baseline, **kw))
    for f in range(2):
        left, right = seq.image(f, 0), seq.image(f, 1)
        assert vo.process(left, right) == S.process(left, right)
        assert vo.stats().tolist() == S.stats
    uv8, inl = vo.getMatches()
    assert np.array_equal(uv8, S.matches) and np.array_equal(inl, S.inliers)
    assert np.allclose(vo.poses, np.array(S.poses), rtol=0, atol=1e-9)


# ------------------------------------------------------------------ configs[3]
_BENCH_SMALL = ["--steps", "20", "--warmup", "5", "--no-cpu", "--no-svo", "--no-other", "--rig-steps", "0",
                "--no-init", "--no-config2"]


def _bench_line(r):
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])


@pytest.mark.gpu
def test_gpu_config3_two_ranks_gather_matches_oracle(tmp_path):
    """bench.py's N>1 path launched the way the driver launches it (an
    external torch.distributed.run, 2 ranks; gloo collectives so both ranks
    can share the box's one GPU): each rank tracks its own sequence (seed =
    rank), value = 2 x steps / max-over-ranks time, and the gathered pose log
    of every rank equals the oracle's poses of that rank's sequence."""
    dump = str(tmp_path / "poses.npz")
    env = dict(os.environ, VISO_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--dump-poses", dump] + _BENCH_SMALL
    line = _bench_line(subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=100))
    assert line["n_gpus"] == 2 and line["steps"] == 20 and line["init_frames_timed"] == 0
    assert abs(line["value"] - 2 * 20 / (line["ms_per_step"] * 20 * 1e-3)) / line["value"] < 1e-3
    g = line["pose_gather"]
    assert g["frames_per_rank"] == [20, 20] and g["own_log_exact"]
    assert g["world_size"] == 2 and g["process_group_backend"] == "gloo"
    d = np.load(dump)
    warm = int(d["warm"])
    from viso_amd.shard import sequence_seed
    for r in range(2):
        ov = _oracle_stereo_poses(sequence_seed(r), warm + 20)
        oP = ov.poses()[warm - 1:]
        gP = d[f"rank{r}"]
        assert gP.shape == oP.shape == (20, 12), r
        assert _rel_rows(gP, oP).max() <= 1e-10, r
    assert not np.array_equal(d["rank0"], d["rank1"])


@pytest.mark.gpu
def test_gpu_config3_rccl_process_group_one_rank(tmp_path):
    """The product N>1 path's RCCL leg on the box's one GPU: one rank with
    VISO_DIST_FORCE=1 builds the nccl (= RCCL) process group, takes the
    max-over-ranks time by an RCCL all-reduce and gathers the pose log through
    RCCL (viso_amd/shard.py); the gathered log equals the oracle's."""
    dump = str(tmp_path / "poses.npz")
    env = dict(os.environ, VISO_DIST_FORCE="1", MASTER_ADDR="127.0.0.1")
    env.pop("VISO_DIST_BACKEND", None)
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--dump-poses", dump] + _BENCH_SMALL
    line = _bench_line(subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=100))
    assert line["n_gpus"] == 1 and line["init_frames_timed"] == 0
    g = line["pose_gather"]
    assert g["backend"] == "rccl" and g["process_group_backend"] == "nccl"
    assert g["world_size"] == 1 and g["frames_per_rank"] == [20] and g["own_log_exact"]
    d = np.load(dump)
    ov = _oracle_stereo_poses(0, int(d["warm"]) + 20)
    assert _rel_rows(d["rank0"], ov.poses()[int(d["warm"]) - 1:]).max() <= 1e-10


# ------------------------------------------------------------------ configs[4]
@pytest.mark.gpu
def test_gpu_config4_rig_reference_path_and_stereo_vo():
    """4 synthetic 1242x375 stereo cameras per timestep.  (a) The photometric
    rig on the reference path (per-camera DirectPoseEstimationSingleLayer sums
    through the extrinsics, one shared GN step per level): stereo init, then 2
    tracking timesteps through the batched device path, maps and poses bit for
    bit.  (b) The stereo-VO rig: one shared RANSAC + Gauss-Newton over all
    cameras' matches, stats / matches / inliers / motion identical to the spec."""
    import torch

    import viso_amd
    from viso_amd import svo
    from viso_amd.rig import VisoRig
    from viso_amd.synth import RigSequence
    W, H, nc, steps = 1242, 375, 4, 3
    seq = RigSequence(W, H, seed=2000, n_cams=nc)
    frames = [seq.frame(f) for f in range(steps)]
    E = seq.extrinsics()
    # (a) reference-path rig
    r = oracle_lib.Rig(seq.K, W, H, E, seq.p.baseline, STEREO_MAX_DISP, 1)
    for ls, rs in frames:
        r.process(ls, rs)
    g = VisoRig(*seq.K, W, H, E, precision=viso_amd.PRECISION_FAITHFUL)
    g.set_stereo(seq.p.baseline, STEREO_MAX_DISP, 1)
    dl = torch.from_numpy(np.stack([im for ls, _ in frames for im in ls])).cuda()
    dr = torch.from_numpy(np.stack([im for _, rs in frames for im in rs])).cuda()
    torch.cuda.synchronize()
    g.process_device(dl.data_ptr(), dr.data_ptr(), steps, W * H)
    g.synchronize()
    assert g.state == r.state == 1
    for c in range(nc):
        assert len(r.points(c)) > 500 and np.array_equal(g.points(c), r.points(c)), c
    assert g.poses.shape == r.poses.shape == (steps - 1, 12)
    assert _rel_rows(g.poses, r.poses).max() <= 1e-10
    # (b) stereo-VO rig
    p = svo.default_params(W, H, *seq.K, seq.p.baseline)
    vo = svo.VisualOdometryStereoRig(p, E)
    S = oracle_lib.SvoRigSequence(oracle_lib.svo_params(W, H, *seq.K, seq.p.baseline), E)
    for f, (L, R) in enumerate(frames):
        assert vo.process(L, R) == S.process(L, R) == (f > 0)
        assert vo.stats().tolist() == S.stats
        if f > 0:
            uv8, inl = vo.getMatches()
            assert np.array_equal(uv8, S.matches) and np.array_equal(inl, S.inliers)
            assert np.array_equal(vo.getMatchCams(), S.cams)
    assert np.allclose(vo.poses, np.array(S.poses), rtol=0, atol=1e-9)
