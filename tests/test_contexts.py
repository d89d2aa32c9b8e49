"""The C ABI's context contract on the GPU (include/viso/viso_c.h:11-12,
"distinct contexts may run concurrently") and the pose
log's pinned staging past its first 4,096 entries.

* Two and three contexts in one process, each tracking its own sequence
  (bench.py's sequences of ranks 0, 1, 2) through device-ingest chunks with
  the background LK grid: interleaved from one host thread with no sync
  between the contexts' chunks, and driven from one host thread per context.
  Each context owns a context stream and a CU-masked LK side stream (a
  hardware queue of its own, viso_get_config [1]); every context's poses, map
  and last LK alignment must equal its own oracle run, with the background
  error word clear.
* viso_get_poses past 4,096 poses: the pinned staging grows
  geometrically and the kernels keep mirroring new poses into it; poses read
  after every call equal the log read once at the end by a second context.
"""
from __future__ import annotations

import threading

import numpy as np
import pytest

from tests import oracle_lib

W, H = 1242, 375
STEREO_MAX_DISP = 128
WARM, CHUNK, CHUNKS = 5, 20, 2
_ORACLE: dict = {}


def _seq(r):
    from viso_amd.shard import sequence_seed
    from viso_amd.synth import Sequence
    return Sequence(W, H, seed=sequence_seed(r))


def _frames(r):
    if r not in _ORACLE:
        seq = _seq(r)
        n = WARM + CHUNK * CHUNKS
        left = np.stack([seq.image(f, 0) for f in range(n)])
        right = np.stack([seq.image(f, 1) for f in range(WARM)])
        ov = oracle_lib.Viso(seq.K, W, H, enable_tracking=1)
        ov.set_stereo(seq.p.baseline, STEREO_MAX_DISP, 1)
        ov.on_new_stereo(left[0], right[0])
        for f in range(1, n):
            ov.on_new_frame(left[f])
        _ORACLE[r] = dict(seq=seq, left=left, right=right, poses=ov.poses(), points=ov.points(),
                          alignment=ov.alignment())
    return _ORACLE[r]


class _Run:
    """One context on sequence r: its frames resident in HBM, warmed up."""

    def __init__(self, r):
        import torch

        import viso_amd
        d = _frames(r)
        self.d = d
        self.dl = torch.from_numpy(d["left"]).cuda()
        self.dr = torch.from_numpy(d["right"]).cuda()
        torch.cuda.synchronize()
        seq = d["seq"]
        self.v = viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=1, batch_frames=64)
        self.v.set_stereo(seq.p.baseline, STEREO_MAX_DISP, 1)
        self.v.process_device(self.dl.data_ptr(), self.dr.data_ptr(), WARM, W * H)
        self.v.synchronize()
        assert self.v.state == 1

    def chunk(self, k):
        f0 = WARM + k * CHUNK
        self.v.process_device(self.dl.data_ptr() + f0 * W * H, None, CHUNK, W * H)

    def check(self):
        self.v.synchronize()  # raises the background grid's error word, if set
        o = self.d
        assert np.array_equal(self.v.GetPoints(), o["points"])
        gP, oP = self.v.poses, o["poses"]
        assert gP.shape == oP.shape
        rel = np.linalg.norm(gP - oP, axis=1) / np.linalg.norm(oP, axis=1)
        assert rel.max() <= 1e-10
        pk, sc, ub, ua = self.v.alignment()
        opk, osc, oub, oua = o["alignment"]
        assert np.array_equal(pk, opk) and np.array_equal(sc, osc)
        assert np.max(np.abs(ua - oua)) < 1e-6
        cfg = self.v.config()
        self.v.close()
        return cfg


@pytest.mark.gpu
@pytest.mark.parametrize("n_ctx,threads", [(2, False), (3, False), (3, True)])
def test_gpu_contexts_run_concurrently(n_ctx, threads):
    """n_ctx contexts in one process, device-ingest chunks with the background
    LK grid overlapping on the GPU: interleaved chunk by chunk from one host
    thread (no sync between contexts), or one host thread per context.  Each
    is bit-exact with its own oracle; each context's LK side stream has a
    hardware queue of its own and runs the background mode."""
    runs = [_Run(r) for r in range(n_ctx)]
    if threads:
        errs = []

        def drive(run):
            try:
                for k in range(CHUNKS):
                    run.chunk(k)
                run.v.synchronize()
            except Exception as e:  # pragma: no cover - reported below
                errs.append(e)

        ts = [threading.Thread(target=drive, args=(run,)) for run in runs]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=60)
        assert not any(t.is_alive() for t in ts)
        assert not errs, errs
    else:
        for k in range(CHUNKS):
            for run in runs:
                run.chunk(k)
    cfgs = [run.check() for run in runs]
    for cfg in cfgs:
        assert cfg["background_lk"] == 1 and cfg["lk_queue_dedicated"] == 1, cfgs


@pytest.mark.gpu
def test_gpu_pose_log_past_4096():
    """viso_get_poses read after every call over 4,410 tracking frames (a
    126-frame forward-and-back cycle of the bench sequence, 35 times): the
    pinned staging grows 4096 -> 8192 once, later reads stay on the staged
    path, and every read equals the log read once, at the end, by a second
    context on the same frames (its single read copies the device log)."""
    import torch

    import viso_amd
    d = _frames(0)
    seq = d["seq"]
    fwd = list(range(WARM, WARM + 64))
    cyc = fwd + fwd[-2:0:-1]
    left = np.stack([seq.image(f, 0) for f in range(max(cyc) + 1)])
    frames = torch.from_numpy(np.ascontiguousarray(left[cyc])).cuda()
    dl0, dr0 = torch.from_numpy(d["left"][:WARM]).cuda(), torch.from_numpy(d["right"]).cuda()
    torch.cuda.synchronize()
    reps = 35

    def make():
        v = viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=1, batch_frames=128, max_poses=8192)
        v.set_stereo(seq.p.baseline, STEREO_MAX_DISP, 1)
        v.process_device(dl0.data_ptr(), dr0.data_ptr(), WARM, W * H)
        v.synchronize()
        assert v.state == 1
        return v

    a, b = make(), make()
    reads = []
    for _ in range(reps):
        for v in (a, b):
            v.process_device(frames.data_ptr(), None, len(cyc), W * H)
        a.synchronize()
        reads.append(a.poses)
    b.synchronize()
    ref = b.poses
    assert len(ref) == WARM - 1 + reps * len(cyc) > 4096
    for p in reads:
        assert np.array_equal(p.view(np.uint64), ref[:len(p)].view(np.uint64))
    assert len(reads[-1]) == len(ref)
    a.close()
    b.close()
