"""Multi-GPU sharding of independent stereo sequences.

Frames of one sequence are sequentially dependent (``last_frame``,
src/viso.cpp:144), so a sequence never splits across GPUs.  Independent
sequences shard one per rank (BASELINE.json configs[3]: KITTI 00-07 on 8
GPUs) with no data-path collective; the only exchange is the result gather
of every rank's pose log (Tcw, 12 doubles per frame) at the end.

``gather_poses`` works over any initialised ``torch.distributed`` group: RCCL
("nccl") with device tensors on the GPU box, gloo with host tensors in the
CPU tests (tests/test_multi.py).
"""
from __future__ import annotations

import numpy as np


def sequence_seed(rank: int, base: int = 0) -> int:
    """Sequence of rank r: synthetic renderer seed base + r (one sequence per GPU)."""
    return base + rank


def gather_poses(poses: np.ndarray, device=None) -> list[np.ndarray]:
    """All-gather each rank's (n_r, 12) fp64 pose log; returns the list of
    every rank's poses, in rank order, trimmed to each rank's own length.

    Two collectives: a MAX all-reduce of the lengths, then one all-gather of
    the zero-padded (n_max, 13) block (column 12 carries the row-valid flag so
    ranks can be trimmed without a second length exchange)."""
    import torch
    import torch.distributed as dist

    poses = np.ascontiguousarray(poses, dtype=np.float64).reshape(-1, 12)
    world = dist.get_world_size()
    dev = torch.device("cpu") if device is None else torch.device(device)
    n_max = torch.tensor([poses.shape[0]], dtype=torch.int64, device=dev)
    dist.all_reduce(n_max, op=dist.ReduceOp.MAX)
    n = int(n_max.item())
    block = torch.zeros((n, 13), dtype=torch.float64, device=dev)
    if poses.shape[0]:
        block[:poses.shape[0], :12] = torch.from_numpy(poses).to(dev)
        block[:poses.shape[0], 12] = 1.0
    out = [torch.empty_like(block) for _ in range(world)]
    dist.all_gather(out, block)
    res = []
    for t in out:
        a = t.cpu().numpy()
        res.append(a[a[:, 12] > 0.5, :12].copy())
    return res
