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

    def klt(self, ref_pyr: np.ndarray, cur_pyr: np.ndarray, width: int, height: int,
            kp1: np.ndarray, kp2: np.ndarray):
        """OpticalFlowMultiLevel(..., inverse=true) (src/viso.cpp:353-391).
        kp1, kp2: (n,2) float32; returns (kp2_out, success)."""
        kp1 = np.ascontiguousarray(kp1, dtype=np.float32)
        kp2 = np.ascontiguousarray(kp2, dtype=np.float32).copy()
        n = kp1.shape[0]
        succ = np.zeros(n, np.uint8)
        _lib.call("viso_klt", self.h, _p(np.ascontiguousarray(ref_pyr)),
                  _p(np.ascontiguousarray(cur_pyr)), width, height, _p(kp1), _p(kp2), _p(succ), n)
        return kp2, succ

    def direct_pose(self, last_pyr, cur_pyr, width, height, points, pose_last, pose_init):
        """DirectPoseEstimationMultiLayer (src/viso.cpp:760-766); poses 12 doubles."""
        pts = np.ascontiguousarray(points, dtype=np.float64).reshape(-1, 3)
        pl = np.ascontiguousarray(pose_last, dtype=np.float64).reshape(12)
        pio = np.ascontiguousarray(pose_init, dtype=np.float64).reshape(12).copy()
        _lib.call("viso_direct_pose", self.h, _p(np.ascontiguousarray(last_pyr)),
                  _p(np.ascontiguousarray(cur_pyr)), width, height, _p(pts), pts.shape[0],
                  _p(pl), _p(pio))
        return pio

    def lk_align(self, kf_pyrs, kf_poses, cur_pyr, cur_pose, width, height, points):
        """LKAlignment (src/viso.cpp:768-843): dense per-map-point outputs
        (pair_kf, success, uv_before (n,2), uv_after (n,2))."""
        kfp = np.ascontiguousarray(np.stack(kf_pyrs) if isinstance(kf_pyrs, (list, tuple))
                                   else kf_pyrs, dtype=np.uint8)
        kposes = np.ascontiguousarray(kf_poses, dtype=np.float64).reshape(-1, 12)
        pts = np.ascontiguousarray(points, dtype=np.float64).reshape(-1, 3)
        n = pts.shape[0]
        pk = np.zeros(n, np.int32)
        sc = np.zeros(n, np.uint8)
        ub = np.zeros((n, 2), np.float64)
        ua = np.zeros((n, 2), np.float64)
        cp = np.ascontiguousarray(cur_pose, dtype=np.float64).reshape(12)
        _lib.call("viso_lk_align", self.h, _p(kfp), _p(kposes), kposes.shape[0],
                  _p(np.ascontiguousarray(cur_pyr)), _p(cp), width, height, _p(pts), n, _p(pk),
                  _p(sc), _p(ub), _p(ua))
        return pk, sc, ub, ua

    def pose_2d2d(self, p1: np.ndarray, p2: np.ndarray, R0=None, T0=None):
        """PoseEstimation2d2d + SelectMotion (src/viso.cpp:178-256, 520-638) on
        normalised (n,3) points.  Returns dict(R, T, inliers, points3d,
        candidates, stats)."""
        p1 = np.ascontiguousarray(p1, dtype=np.float64).reshape(-1, 3)
        p2 = np.ascontiguousarray(p2, dtype=np.float64).reshape(-1, 3)
        n = p1.shape[0]
        R = np.ascontiguousarray(np.eye(3) if R0 is None else R0, dtype=np.float64).reshape(9).copy()
        T = np.ascontiguousarray(np.zeros(3) if T0 is None else T0, dtype=np.float64).reshape(3).copy()
        inl = np.zeros(max(n, 1), np.uint8)
        pts = np.zeros((max(n, 1), 3), np.float64)
        cand = np.zeros((5, 12), np.float64)
        st = np.zeros(8, np.float64)
        _lib.call("viso_pose_2d2d", self.h, _p(p1), _p(p2), n, _p(R), _p(T), _p(inl), _p(pts),
                  _p(cand), _p(st))
        return {"R": R.reshape(3, 3), "T": T, "inliers": inl[:n], "points3d": pts[:n],
                "candidates": cand[:int(st[2])], "stats": st}

    def stereo_match(self, left, right, xs, ys, max_disp: int = 128):
        """North-star stereo SAD stage: (disparity, sad) per left keypoint."""
        left = np.ascontiguousarray(left, dtype=np.uint8)
        right = np.ascontiguousarray(right, dtype=np.uint8)
        h, w = left.shape
        xs = np.ascontiguousarray(xs, dtype=np.int32)
        ys = np.ascontiguousarray(ys, dtype=np.int32)
        n = len(xs)
        d = np.zeros(n, np.int32)
        s = np.zeros(n, np.int32)
        _lib.call("viso_stereo_match", self.h, _p(left), _p(right), w, h, _p(xs), _p(ys), n,
                  max_disp, _p(d), _p(s))
        return d, s

    # ------------------------------------------------------------ timing
    def photometric_ba(self, kf_images, kf_poses, points, host, iterations: int = 5):
        """viso_photometric_ba: the BA of include/bundle_adjuster.h:22-106 on
        host data; returns (poses (k, 12), points (n, 3), report
        (iterations, 4): cost, candidate cost, damping, accepted)."""
        imgs = [np.ascontiguousarray(x, np.uint8) for x in kf_images]
        P = ctypes.c_void_p * len(imgs)
        poses = np.ascontiguousarray(kf_poses, np.float64).reshape(-1, 12).copy()
        pts = np.ascontiguousarray(points, np.float64).reshape(-1, 3).copy()
        hst = np.ascontiguousarray(host, np.int32)
        rep = np.zeros((iterations, 4))
        _lib.call("viso_photometric_ba", self.h, P(*[x.ctypes.data for x in imgs]), len(imgs), _p(poses), _p(pts),
                  _p(hst), len(pts), iterations, _p(rep))
        return poses, pts, rep

    def timing_enable(self, on: bool = True):
        _lib.call("viso_timing_enable", self.h, 1 if on else 0)

    def timing_select(self, kernels=None):
        """Time only the named kernels (None: all)."""
        mask = 0xFFFFFFFF if kernels is None else sum(1 << _lib.KERNEL_IDS[k] for k in kernels)
        _lib.call("viso_timing_select", self.h, mask)

    def timing(self, kernel: str):
        launches = ctypes.c_int64(0)
        ms = ctypes.c_double(0.0)
        _lib.call("viso_timing_get", self.h, _lib.KERNEL_IDS[kernel], ctypes.byref(launches),
                  ctypes.byref(ms))
        return int(launches.value), float(ms.value)

    def synchronize(self):
        _lib.call("viso_synchronize", self.h)


def default_context(width: int = 640, height: int = 480, device: int = 0, K=None) -> Context:
    """A cached context per (device, intrinsics).  The stage functions that
    project points (direct_pose, lk_align, pose_2d2d) use the context's K,
    as the reference's Viso members do (include/viso.h:28-29)."""
    K = tuple(K) if K is not None else (517.3, 516.5, 325.1, 249.7)
    key = (device, K)
    c = _ctx_cache.get(key)
    if c is None or c.h is None:  # absent or closed by a caller
        c = Context(default_params(fx=K[0], fy=K[1], cx=K[2], cy=K[3], width=width,
                                   height=height), device=device)
        _ctx_cache[key] = c
    return c
