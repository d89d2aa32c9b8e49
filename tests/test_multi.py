"""Multi-process path on the CPU (gloo, world_size 2, 127.0.0.1).

The GPU path shards independent sequences one per rank with no data-path
collective; the only exchange is the result gather of the
pose logs (viso_amd/shard.py), which bench.py runs over RCCL.  Here the same
gather runs over gloo: each rank tracks its own synthetic sequence with the
CPU oracle (the per-rank compute stand-in on a GPU-less host), and every rank
checks that the gathered logs are exactly what each rank produced, including
ragged and empty logs.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

WORLD = 2


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _oracle_poses(seed: int, frames: int) -> np.ndarray:
    from tests import oracle_lib, seqdata

    seq = seqdata.sequence(seed)
    ov = oracle_lib.Viso(seq.K, seqdata.W, seqdata.H, enable_tracking=1)
    for f in range(frames):
        ov.on_new_frame(seqdata.image(f, seed))
    return ov.poses()


def _worker(rank: int, port: int, frames: int, q):
    import torch.distributed as dist

    from viso_amd.shard import gather_poses, sequence_seed

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        seed = sequence_seed(rank)
        mine = _oracle_poses(seed, frames)
        got = gather_poses(mine)
        # ragged: rank r contributes r + 3 rows; empty: rank 0 contributes none
        ragged = np.arange((rank + 3) * 12, dtype=np.float64).reshape(-1, 12) + 1000 * rank
        got_ragged = gather_poses(ragged)
        empty = np.zeros((0, 12)) if rank == 0 else np.full((2, 12), float(rank))
        got_empty = gather_poses(empty)
        q.put((rank, mine, got, got_ragged, got_empty))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gather_poses_gloo_world2():
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    frames = 9  # init at frame 5 on the synthetic sequence, then tracking
    procs = [ctx.Process(target=_worker, args=(r, port, frames, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(WORLD):
        rank, mine, got, got_ragged, got_empty = q.get(timeout=280)
        res[rank] = (mine, got, got_ragged, got_empty)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in range(WORLD):
        mine, got, got_ragged, got_empty = res[rank]
        assert len(got) == WORLD
        for r in range(WORLD):
            np.testing.assert_array_equal(got[r], res[r][0])  # bit-exact gather
            assert got_ragged[r].shape == (r + 3, 12)
            np.testing.assert_array_equal(
                got_ragged[r], np.arange((r + 3) * 12, dtype=np.float64).reshape(-1, 12) + 1000 * r)
        assert got_empty[0].shape == (0, 12)
        np.testing.assert_array_equal(got_empty[1], np.full((2, 12), 1.0))
    # the two ranks ran different sequences (seed = rank) and both tracked
    assert len(res[0][0]) > 0 and len(res[1][0]) > 0
    m = min(len(res[0][0]), len(res[1][0]))
    assert not np.array_equal(res[0][0][:m], res[1][0][:m])


def test_sequence_seed_distinct():
    from viso_amd.shard import sequence_seed

    seeds = [sequence_seed(r) for r in range(8)]
    assert len(set(seeds)) == 8


def test_bench_rejects_gpus_world_size_mismatch():
    """An external launcher whose WORLD_SIZE differs from --gpus is an error
    (exit 2) caught before anything touches the GPU, so it runs here."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "1", "--steps", "1"],
                       cwd=root, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "4", "--steps", "1"],
                       cwd=root, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2


def _bench_line(r):
    import json
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])


_BENCH_SMALL = ["--steps", "20", "--warmup", "5", "--no-cpu", "--no-svo", "--no-other", "--rig-steps", "0",
                "--no-init", "--no-config2"]


# The driver-shaped N>1 runs (two gloo ranks on the box's GPU, the RCCL group
# at one rank), each checked against the oracle, are configs[3] in
# tests/test_00_configs.py.


@pytest.mark.gpu
def test_gpu_bench_gpus_flag_launches_ranks(tmp_path):
    """`bench.py --gpus 2` with no external launcher starts its two ranks
    itself (torch.distributed.run as a child, before any GPU call) and prints
    one line with n_gpus 2."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, VISO_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"] + _BENCH_SMALL
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=100)
    line = _bench_line(r)
    assert sum(ln.startswith("{") for ln in r.stdout.splitlines()) == 1
    assert line["n_gpus"] == 2 and line["init_frames_timed"] == 0
    g = line["pose_gather"]
    assert g["world_size"] == 2 and g["frames_per_rank"] == [20, 20] and g["own_log_exact"]
