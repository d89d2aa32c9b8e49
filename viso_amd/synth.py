"""Deterministic synthetic KITTI-like stereo sequence (include/viso/viso_synth.h).

Host-only data source for tests and bench.py (KITTI is not available
offline).  Frames are rendered by C++ in libviso_amd.so.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _lib


class SynthParams(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int32), ("height", ctypes.c_int32),
        ("fx", ctypes.c_double), ("fy", ctypes.c_double),
        ("cx", ctypes.c_double), ("cy", ctypes.c_double),
        ("baseline", ctypes.c_double), ("seed", ctypes.c_uint64),
        ("block_m", ctypes.c_double), ("wall_x", ctypes.c_double),
        ("wall_z", ctypes.c_double), ("ground_y", ctypes.c_double),
        ("pitch0", ctypes.c_double), ("yaw_amp", ctypes.c_double),
        ("yaw_period", ctypes.c_double), ("x_amp", ctypes.c_double),
        ("x_period", ctypes.c_double), ("z_amp", ctypes.c_double),
        ("z_period", ctypes.c_double), ("noise", ctypes.c_int32),
        ("reserved", ctypes.c_int32 * 7),
    ]


def _fns():
    lib = _lib.load()
    lib.viso_synth_default.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    lib.viso_synth_default.restype = None
    lib.viso_synth_pose.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    lib.viso_synth_render.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.c_int]
    lib.viso_synth_rig_extrinsic.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    lib.viso_synth_rig_pose.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_void_p]
    lib.viso_synth_rig_render.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    return lib


class Sequence:
    """Synthetic stereo sequence; ``frame(i)`` -> (left, right) uint8 images."""

    def __init__(self, width: int = 1242, height: int = 375, seed: int = 0, **kw):
        lib = _fns()
        self.p = SynthParams()
        lib.viso_synth_default(ctypes.byref(self.p), width, height)
        self.p.seed = seed
        for k, v in kw.items():
            setattr(self.p, k, v)
        self.width, self.height = width, height
        self.threads = int(os.environ.get("VISO_SYNTH_THREADS", min(16, os.cpu_count() or 1)))

    @property
    def K(self):
        return (self.p.fx, self.p.fy, self.p.cx, self.p.cy)

    def image(self, frame: int, cam: int = 0) -> np.ndarray:
        out = np.empty((self.height, self.width), np.uint8)
        rc = _fns().viso_synth_render(ctypes.byref(self.p), frame, cam, out.ctypes.data,
                                      self.threads)
        if rc != 0:
            raise RuntimeError("viso_synth_render failed")
        return out

    def frame(self, i: int):
        return self.image(i, 0), self.image(i, 1)

    def pose(self, frame: int, cam: int = 0) -> np.ndarray:
        out = np.zeros(12, np.float64)
        _fns().viso_synth_pose(ctypes.byref(self.p), frame, cam, out.ctypes.data)
        return out


class RigSequence(Sequence):
    """The same scene seen by a rig of ``n_cams`` stereo cameras (BASELINE.json
    configs[4]); ``frame(i)`` -> (lefts, rights), one image per camera."""

    def __init__(self, width: int = 1242, height: int = 375, seed: int = 0, n_cams: int = 4, **kw):
        super().__init__(width, height, seed, **kw)
        self.n_cams = n_cams

    def extrinsics(self) -> np.ndarray:
        """(n_cams, 12): rig -> camera c (left), R row-major + t."""
        out = np.zeros((self.n_cams, 12), np.float64)
        for c in range(self.n_cams):
            _fns().viso_synth_rig_extrinsic(c, self.n_cams, out[c].ctypes.data)
        return out

    def cam_image(self, frame: int, cam: int, side: int) -> np.ndarray:
        out = np.empty((self.height, self.width), np.uint8)
        rc = _fns().viso_synth_rig_render(ctypes.byref(self.p), frame, self.n_cams, cam, side,
                                          out.ctypes.data, self.threads)
        if rc != 0:
            raise RuntimeError("viso_synth_rig_render failed")
        return out

    def frame(self, i: int):
        return ([self.cam_image(i, c, 0) for c in range(self.n_cams)],
                [self.cam_image(i, c, 1) for c in range(self.n_cams)])

    def rig_pose(self, frame: int) -> np.ndarray:
        return self.pose(frame, 0)
