"""Python host mirror of the reference interface over the C ABI.

``Context`` wraps one ``viso_ctx`` (one HIP device + stream).  The stage
functions (``pyramid``, ``fast``, ``klt``, ...) mirror the reference's
functions for the parity tests; ``Viso`` / ``Keyframe`` / ``FrameSequence``
(viso_amd/frontend.py) mirror the reference's classes.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib

_ctx_cache: dict = {}


def _p(a: np.ndarray | None):
    return None if a is None else a.ctypes.data


def pyramid_dims(width: int, height: int):
    dims = np.zeros(8, np.int32)
    total = ctypes.c_size_t(0)
    _lib.call("viso_pyramid_dims", width, height, _p(dims), ctypes.byref(total))
    return [(int(dims[2 * l]), int(dims[2 * l + 1])) for l in range(4)], int(total.value)


def default_params(fx=517.3, fy=516.5, cx=325.1, cy=249.7, width=640, height=480, **kw):
    """Defaults = include/viso.h:20-26 and the intrinsics of src/main.cpp:14-17."""
    p = _lib.viso_params()
    _lib.call("viso_default_params", ctypes.byref(p), fx, fy, cx, cy, width, height)
    for k, v in kw.items():
        if not hasattr(p, k):
            raise AttributeError(k)
        setattr(p, k, v)
    return p


class Context:
    """One viso_ctx: device memory + a HIP stream for one sequence."""

    def __init__(self, params=None, device: int = 0, **kw):
        self.params = params if params is not None else default_params(**kw)
        self.device = device
        h = ctypes.c_void_p()
        _lib.call("viso_create", ctypes.byref(self.params), device, ctypes.byref(h))
        self.h = h

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            _lib.load().viso_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ------------------------------------------------------------ stages
    def pyramid(self, images: np.ndarray) -> np.ndarray:
        """Keyframe pyramid (include/keyframe.h:28-46) of n images (n,h,w) ->
        (n, total_bytes) levels concatenated."""
        images = np.ascontiguousarray(images, dtype=np.uint8)
        if images.ndim == 2:
            images = images[None]
        n, h, w = images.shape
        _, total = pyramid_dims(w, h)
        out = np.zeros((n, total), np.uint8)
        _lib.call("viso_pyramid", self.h, _p(images), n, w, h, _p(out))
        return out

    def fast(self, image: np.ndarray, thresh: int = 50, cap: int = 1 << 20):
        """cv::FAST(img, kps, thresh) + NMS (src/viso.cpp:104): row-major
        (xs, ys, scores)."""
        image = np.ascontiguousarray(image, dtype=np.uint8)
        h, w = image.shape
        xs = np.zeros(cap, np.int32)
        ys = np.zeros(cap, np.int32)
        sc = np.zeros(cap, np.int32)
        n = ctypes.c_size_t(0)
        _lib.call("viso_fast", self.h, _p(image), w, h, thresh, _p(xs), _p(ys), _p(sc), cap,
                  ctypes.byref(n))
        m = min(n.value, cap)
        return xs[:m].copy(), ys[:m].copy(), sc[:m].copy()

    # ------------------------------------------------------------ timing
    def timing_enable(self, on: bool = True):
        _lib.call("viso_timing_enable", self.h, 1 if on else 0)

    def timing(self, kernel: str):
        launches = ctypes.c_int64(0)
        ms = ctypes.c_double(0.0)
        _lib.call("viso_timing_get", self.h, _lib.KERNEL_IDS[kernel], ctypes.byref(launches),
                  ctypes.byref(ms))
        return int(launches.value), float(ms.value)

    def synchronize(self):
        _lib.call("viso_synchronize", self.h)


def default_context(width: int = 640, height: int = 480, device: int = 0) -> Context:
    key = (device,)
    c = _ctx_cache.get(key)
    if c is None:
        c = Context(default_params(width=width, height=height), device=device)
        _ctx_cache[key] = c
    return c
