"""Shared synthetic-sequence data for the tracking / geometry tests.

Renders the deterministic KITTI-like sequence (viso_amd.synth) and runs the
oracle's whole per-frame path until initialisation, keeping what the stage
tests need (pyramids, FAST tracks, map points, keyframe poses)."""
from __future__ import annotations

import functools

import numpy as np

from tests import oracle_lib

W, H = 1242, 375


@functools.lru_cache(maxsize=4)
def sequence(seed: int = 0, width: int = W, height: int = H):
    from viso_amd.synth import Sequence
    return Sequence(width, height, seed=seed)


@functools.lru_cache(maxsize=64)
def image(frame: int, seed: int = 0, cam: int = 0, width: int = W, height: int = H):
    return sequence(seed, width, height).image(frame, cam)


@functools.lru_cache(maxsize=64)
def pyramid(frame: int, seed: int = 0, cam: int = 0, width: int = W, height: int = H):
    return oracle_lib.pyramid(image(frame, seed, cam, width, height))


@functools.lru_cache(maxsize=4)
def initialised(seed: int = 0, max_frames: int = 12):
    """Runs the oracle until it leaves kInitialization.  Returns a dict with
    the init frame index, map points, keyframe poses and the next frame's
    oracle pose."""
    seq = sequence(seed)
    v = oracle_lib.Viso(seq.K, W, H, enable_tracking=1)
    init_frame = None
    for f in range(max_frames):
        v.on_new_frame(image(f, seed))
        if v.state != 0:
            init_frame = f
            break
    assert init_frame is not None, "synthetic sequence did not initialise"
    return {
        "K": seq.K,
        "init_frame": init_frame,
        "points": v.points(),
        "kf_poses": v.keyframe_poses(),
        "viso": v,
    }
