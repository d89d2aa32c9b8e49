"""Host mirror of the reference's classes over the C ABI.

* ``Viso(fx, fy, cx, cy, ...)`` — include/viso.h:11-125: ``OnNewFrame``,
  ``poses``, ``GetPoints()``; plus the north-star ``process(left, right)``.
* ``Keyframe(image)`` — include/keyframe.h:28-46 (pyramid built on device by
  ``OnNewFrame``; ``Pyramids()`` computes it on demand for inspection).
* ``FrameSequence(location, handler)`` — include/frame_sequence.h:11-43:
  ``RunOnce()`` loads ``<location><next_id+1>.png`` and calls
  ``handler.OnNewFrame``.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _lib
from .api import Context, default_params


class Keyframe:
    """A grey frame handed to ``FrameHandler.OnNewFrame``."""

    next_id_ = 0  # Keyframe::next_id_ (src/keyframe.cpp:7)

    def __init__(self, mat: np.ndarray):
        mat = np.ascontiguousarray(mat, dtype=np.uint8)
        if mat.ndim != 2:
            raise ValueError("Keyframe expects a single-channel (grey) image")
        self.mat_ = mat
        self.id_ = Keyframe.next_id_
        Keyframe.next_id_ += 1

    @classmethod
    def GetNextId(cls) -> int:
        return cls.next_id_

    def GetId(self) -> int:
        return self.id_

    def Mat(self) -> np.ndarray:
        return self.mat_


class FrameHandler:
    """FrameSequence::FrameHandler (include/frame_sequence.h:13-16)."""

    def OnNewFrame(self, keyframe: Keyframe) -> None:  # pragma: no cover - interface
        raise NotImplementedError


class Viso(FrameHandler):
    """Viso (include/viso.h:11): one device context per sequence."""

    def __init__(self, fx: float, fy: float, cx: float, cy: float, width: int = 640,
                 height: int = 480, device: int = 0, **params):
        self.params = default_params(fx=fx, fy=fy, cx=cx, cy=cy, width=width, height=height,
                                     **params)
        self.ctx = Context(self.params, device=device)
        self.width, self.height = width, height

    # ----------------------------------------------------------- reference API
    def OnNewFrame(self, cur_frame) -> None:
        img = cur_frame.Mat() if isinstance(cur_frame, Keyframe) else cur_frame
        img = np.ascontiguousarray(img, dtype=np.uint8)
        h, w = img.shape
        _lib.call("viso_process_frame", self.ctx.h, img.ctypes.data, w, h, w)

    @property
    def poses(self) -> np.ndarray:
        """Viso::poses (include/viso.h:54): (n, 3, 4) Tcw."""
        n = ctypes.c_size_t(0)
        _lib.call("viso_get_poses", self.ctx.h, None, 0, ctypes.byref(n))
        out = np.zeros((n.value, 12), np.float64)
        if n.value:
            _lib.call("viso_get_poses", self.ctx.h, out.ctypes.data, n.value, ctypes.byref(n))
        return out

    def GetPoints(self) -> np.ndarray:
        """Viso::GetPoints (include/viso.h:60-67): (n, 3)."""
        n = ctypes.c_size_t(0)
        _lib.call("viso_get_points", self.ctx.h, None, 0, ctypes.byref(n))
        out = np.zeros((n.value, 3), np.float64)
        if n.value:
            _lib.call("viso_get_points", self.ctx.h, out.ctypes.data, n.value, ctypes.byref(n))
        return out

    # ----------------------------------------------------------- north-star API
    def process(self, left: np.ndarray, right: np.ndarray) -> None:
        """A stereo pair through the reference path (viso_process_stereo): the
        left image drives OnNewFrame, the right one the stereo initialisation
        (the north-star VisualOdometryStereo is viso_amd.svo)."""
        left = np.ascontiguousarray(left, dtype=np.uint8)
        right = np.ascontiguousarray(right, dtype=np.uint8)
        h, w = left.shape
        dims = (ctypes.c_int32 * 3)(w, h, w)
        _lib.call("viso_process_stereo", self.ctx.h, left.ctypes.data, right.ctypes.data, dims)

    def set_stereo(self, baseline: float, max_disp: int = 128, min_disp: int = 1) -> None:
        """Stereo initialisation (viso_set_stereo): with baseline > 0 the first
        frame given with its right image creates a metric map at once."""
        _lib.call("viso_set_stereo", self.ctx.h, float(baseline), int(max_disp), int(min_disp))

    def set_keyframes(self, interval: int, ngood_permille: int = 500) -> None:
        """Stereo keyframe insertion (viso_set_keyframes): every `interval`-th
        tracking frame whose level-0 nGood is below ngood_permille / 1000 of
        the map adds its stereo points and becomes a keyframe."""
        _lib.call("viso_set_keyframes", self.ctx.h, int(interval), int(ngood_permille))

    def set_bundle_adjust(self, iterations: int) -> None:
        """Photometric BA (viso_set_bundle_adjust) after every keyframe
        insertion: `iterations` Levenberg-Marquardt steps over the keyframe
        poses and map points (0 = off)."""
        _lib.call("viso_set_bundle_adjust", self.ctx.h, int(iterations))

    def process_device(self, d_left: int, d_right: int | None, n: int, frame_stride: int):
        """Batched ingest of n frames resident in HBM (device pointers)."""
        _lib.call("viso_process_frames_device", self.ctx.h, d_left, d_right, n, frame_stride)

    # ----------------------------------------------------------- inspection
    @property
    def state(self) -> int:
        s = ctypes.c_int32(0)
        _lib.call("viso_get_state", self.ctx.h, ctypes.byref(s))
        return s.value

    def stats(self) -> np.ndarray:
        out = np.zeros(16)
        _lib.call("viso_get_frame_stats", self.ctx.h, out.ctypes.data)
        return out

    def config(self) -> dict:
        """viso_get_config: background LK, dedicated queues, pool size."""
        info = np.zeros(8, np.int32)
        _lib.call("viso_get_config", self.ctx.h, info.ctypes.data)
        return {"background_lk": int(info[0]), "lk_queue_dedicated": int(info[1]),
                "upload_queue_dedicated": int(info[2]), "slots": int(info[3]), "frame_log": int(info[4]),
                "batch_frames": int(info[5]), "tail_copy_bytes": int(info[6]), "tail_zero_ints": int(info[7])}

    def set_frame_log(self, on: bool = True) -> None:
        """Per-frame log (viso_set_frame_log): every tracking frame's level-0
        nGood / cost and LK pair / success counts, kept on the device."""
        _lib.call("viso_set_frame_log", self.ctx.h, 1 if on else 0)

    def frame_log(self) -> np.ndarray:
        """(poses, 4): level-0 nGood, level-0 cost, LK pairs, LK successes per
        tracking frame (row k = pose k); NaN for frames run with the log off."""
        n = ctypes.c_size_t(0)
        _lib.call("viso_get_frame_log", self.ctx.h, None, 0, ctypes.byref(n))
        out = np.zeros((n.value, 4), np.float64)
        if n.value:
            _lib.call("viso_get_frame_log", self.ctx.h, out.ctypes.data, n.value, ctypes.byref(n))
        return out

    def tracks(self):
        """init_.kp1, init_.kp2 (float32 (n,2)) and init_.success."""
        n = ctypes.c_size_t(0)
        _lib.call("viso_get_init_tracks", self.ctx.h, None, None, None, 0, ctypes.byref(n))
        m = n.value
        k1 = np.zeros((m, 2), np.float32)
        k2 = np.zeros((m, 2), np.float32)
        s = np.zeros(m, np.uint8)
        if m:
            _lib.call("viso_get_init_tracks", self.ctx.h, k1.ctypes.data, k2.ctypes.data,
                      s.ctypes.data, m, ctypes.byref(n))
        return k1, k2, s

    def alignment(self):
        """Last LKAlignment (dense per map point)."""
        n = ctypes.c_size_t(0)
        _lib.call("viso_get_alignment", self.ctx.h, None, None, None, None, 0, ctypes.byref(n))
        m = n.value
        pk = np.zeros(m, np.int32)
        sc = np.zeros(m, np.uint8)
        ub = np.zeros((m, 2))
        ua = np.zeros((m, 2))
        if m:
            _lib.call("viso_get_alignment", self.ctx.h, pk.ctypes.data, sc.ctypes.data,
                      ub.ctypes.data, ua.ctypes.data, m, ctypes.byref(n))
        return pk, sc, ub, ua

    def synchronize(self):
        self.ctx.synchronize()

    def close(self):
        self.ctx.close()


class FrameSequence:
    """FrameSequence (include/frame_sequence.h:11-43): reads
    ``<location><Keyframe.GetNextId()+1>.png`` (grey) per RunOnce()."""

    def __init__(self, location: str, handler: FrameHandler):
        self.location_ = location
        self.handler_ = handler

    def RunOnce(self) -> bool:
        path = os.path.join(self.location_, f"{Keyframe.GetNextId() + 1}.png")
        if not os.path.exists(path):
            return False  # the reference silently skips a missing file
        from .kitti import read_png  # cv::imread(path, 0) restated (include/viso/viso_io.h)
        self.handler_.OnNewFrame(Keyframe(read_png(path)))
        return True
