"""Multi-camera photometric rig on the reference path (include/viso/viso_rig.h;
SURVEY.md §8(f) row 3, BASELINE.json configs[4]).

``VisoRig`` tracks one rig pose with the reference's direct photometric
Gauss-Newton (src/viso.cpp:661-766) run per camera at the camera's pose
E_c T and the cameras' H, b summed through the rig extrinsics.  The spec is
the repo's own (oracle/oracle_rig.cpp).  No CPU fallback.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .api import default_params


def _p(a):
    return None if a is None else a.ctypes.data


class VisoRig:
    """n_cams (<= 4) stereo cameras with shared intrinsics and rig -> camera
    extrinsics (n_cams x 12: R row-major, t)."""

    def __init__(self, fx, fy, cx, cy, width, height, extrinsics, device: int = 0, **kw):
        self.params = default_params(fx, fy, cx, cy, width, height, **kw)
        self.extrinsics = np.ascontiguousarray(extrinsics, np.float64).reshape(-1, 12)
        self.n_cams = len(self.extrinsics)
        self.width, self.height = width, height
        h = ctypes.c_void_p()
        _lib.call("viso_rig_create", ctypes.byref(self.params), self.n_cams, _p(self.extrinsics), device,
                  ctypes.byref(h))
        self.h = h

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            _lib.load().viso_rig_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stereo(self, baseline: float, max_disp: int = 128, min_disp: int = 1):
        _lib.call("viso_rig_set_stereo", self.h, baseline, max_disp, min_disp)

    def process(self, lefts, rights=None):
        """One timestep from host images (lists of n_cams grey images)."""
        ls = [np.ascontiguousarray(x, np.uint8) for x in lefts]
        P = ctypes.c_void_p * self.n_cams
        dims = (ctypes.c_int32 * 3)(self.width, self.height, self.width)
        if rights is None:
            _lib.call("viso_rig_process", self.h, P(*[_p(x) for x in ls]), None, dims)
        else:
            rs = [np.ascontiguousarray(x, np.uint8) for x in rights]
            _lib.call("viso_rig_process", self.h, P(*[_p(x) for x in ls]), P(*[_p(x) for x in rs]), dims)

    def process_device(self, d_left: int, d_right: int | None, n_steps: int, frame_stride: int):
        """n_steps timesteps in HBM: camera c of step s at base + (s * n_cams + c) * frame_stride."""
        _lib.call("viso_rig_process_device", self.h, d_left, d_right, n_steps, frame_stride)

    def synchronize(self):
        _lib.call("viso_rig_synchronize", self.h)

    @property
    def state(self) -> int:
        s = ctypes.c_int32(0)
        _lib.call("viso_rig_get_state", self.h, ctypes.byref(s))
        return s.value

    @property
    def poses(self) -> np.ndarray:
        n = ctypes.c_size_t(0)
        _lib.call("viso_rig_get_poses", self.h, None, 0, ctypes.byref(n))
        out = np.zeros((max(1, n.value), 12))
        _lib.call("viso_rig_get_poses", self.h, _p(out), n.value, ctypes.byref(n))
        return out[:n.value]

    def points(self, cam: int) -> np.ndarray:
        n = ctypes.c_size_t(0)
        _lib.call("viso_rig_get_points", self.h, cam, None, 0, ctypes.byref(n))
        out = np.zeros((max(1, n.value), 3))
        _lib.call("viso_rig_get_points", self.h, cam, _p(out), n.value, ctypes.byref(n))
        return out[:n.value]

    def level_stats(self) -> np.ndarray:
        out = np.zeros((4, 50))
        _lib.call("viso_rig_get_level_stats", self.h, _p(out))
        return out
