"""North-star stereo visual odometry (include/viso/viso_svo.h) — Python mirror.

``VisualOdometryStereo(params).process(left, right)`` and ``Matcher`` keep the
names of the north star's VisualOdometryStereo::process(left, right, dims) /
Matcher API; everything runs in viso_amd/csrc/svo.hip (no CPU fallback).
The stage methods (``features``, ``match``, ``estimate``) exist for the parity
tests against the CPU spec (oracle/oracle_svo.cpp).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib

DESC_BYTES = 32


class SvoParams(ctypes.Structure):
    """viso_svo_params."""
    _fields_ = [
        ("width", ctypes.c_int32), ("height", ctypes.c_int32),
        ("fx", ctypes.c_double), ("fy", ctypes.c_double), ("cu", ctypes.c_double),
        ("cv", ctypes.c_double), ("base", ctypes.c_double),
        ("nms_n", ctypes.c_int32), ("nms_tau", ctypes.c_int32), ("margin", ctypes.c_int32),
        ("disp_max", ctypes.c_int32), ("match_radius", ctypes.c_int32),
        ("bucket_width", ctypes.c_int32), ("bucket_height", ctypes.c_int32),
        ("bucket_max", ctypes.c_int32), ("ransac_iters", ctypes.c_int32),
        ("gn_iters", ctypes.c_int32), ("inlier_threshold", ctypes.c_double),
        ("gn_eps", ctypes.c_double), ("seed", ctypes.c_uint64),
        ("max_features", ctypes.c_int32), ("reserved", ctypes.c_int32 * 7),
    ]


def default_params(width, height, fx, fy, cu, cv, base, **kw) -> SvoParams:
    p = SvoParams()
    _lib.call("viso_svo_default_params", ctypes.byref(p), width, height, fx, fy, cu, cv, base)
    for k, v in kw.items():
        if not hasattr(p, k):
            raise AttributeError(k)
        setattr(p, k, v)
    return p


def _p(a: np.ndarray):
    return a.ctypes.data


class Features:
    """Features of one image: u, v, cls (int32) and desc (n x 32 u8), row-major."""

    def __init__(self, u, v, cls, desc):
        self.u, self.v, self.cls, self.desc = u, v, cls, desc

    def __len__(self):
        return len(self.u)


class VisualOdometryStereo:
    """VisualOdometryStereo(param): one stereo sequence on one GPU."""

    def __init__(self, params: SvoParams, device: int = 0):
        self.params = params
        h = ctypes.c_void_p()
        _lib.call("viso_svo_create", ctypes.byref(params), device, ctypes.byref(h))
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            _lib.call("viso_svo_destroy", self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------- sequence
    def process(self, left: np.ndarray, right: np.ndarray) -> bool:
        """process(left, right, dims): True once a motion was estimated."""
        left = np.ascontiguousarray(left, np.uint8)
        right = np.ascontiguousarray(right, np.uint8)
        h, w = left.shape
        dims = (ctypes.c_int32 * 3)(w, h, w)
        ok = ctypes.c_int32(0)
        _lib.call("viso_svo_process", self.h, _p(left), _p(right), dims, ctypes.byref(ok))
        return bool(ok.value)

    def process_device(self, left_ptr: int, right_ptr: int, n: int, pair_stride: int):
        """n pairs already in HBM (device pointers), no host round trip per pair."""
        _lib.call("viso_svo_process_device", self.h, ctypes.c_void_p(left_ptr),
                  ctypes.c_void_p(right_ptr), n, pair_stride, self.params.width)

    def synchronize(self):
        _lib.call("viso_svo_synchronize", self.h)

    def timing(self, enable: bool = True):
        """HIP-event timing of the batched feature pass -> (ms, pairs) summed
        over the batches since the previous call; then enable / disable."""
        ms = ctypes.c_double(0.0)
        n = ctypes.c_int32(0)
        _lib.call("viso_svo_timing", self.h, int(enable), ctypes.byref(ms), ctypes.byref(n))
        return ms.value, n.value

    def getMotion(self) -> np.ndarray:  # noqa: N802 (north-star name)
        m = np.zeros(12, np.float64)
        _lib.call("viso_svo_get_motion", self.h, _p(m))
        T = np.eye(4)
        T[:3, :3] = m[:9].reshape(3, 3)
        T[:3, 3] = m[9:]
        return T

    def stats(self) -> np.ndarray:
        """[features left, features right, circular matches, bucketed, inliers, ok]."""
        s = np.zeros(6, np.int32)
        _lib.call("viso_svo_get_stats", self.h, _p(s))
        return s

    def getNumberOfMatches(self) -> int:  # noqa: N802
        return int(self.stats()[3])

    def getNumberOfInliers(self) -> int:  # noqa: N802
        return int(self.stats()[4])

    def getMatches(self):  # noqa: N802
        """Bucketed matches of the last pair: (uv8 [n, 8] int32, inlier [n] bool)."""
        n = ctypes.c_size_t(0)
        _lib.call("viso_svo_get_matches", self.h, None, None, 0, ctypes.byref(n))
        uv8 = np.zeros((max(1, n.value), 8), np.int32)
        inl = np.zeros(max(1, n.value), np.uint8)
        _lib.call("viso_svo_get_matches", self.h, _p(uv8), _p(inl), n.value, ctypes.byref(n))
        return uv8[:n.value], inl[:n.value].astype(bool)

    @property
    def poses(self) -> np.ndarray:
        """Accumulated T_wc of the left camera, one 12-vector per processed pair."""
        n = ctypes.c_size_t(0)
        _lib.call("viso_svo_get_poses", self.h, None, 0, ctypes.byref(n))
        out = np.zeros((max(1, n.value), 12), np.float64)
        _lib.call("viso_svo_get_poses", self.h, _p(out), n.value, ctypes.byref(n))
        return out[:n.value]

    # ---------------------------------------------------------------- stages
    def features(self, img: np.ndarray) -> Features:
        img = np.ascontiguousarray(img, np.uint8)
        h, w = img.shape
        cap = self.params.max_features
        u, v, c = (np.zeros(cap, np.int32) for _ in range(3))
        d = np.zeros((cap, DESC_BYTES), np.uint8)
        n = ctypes.c_int32(0)
        _lib.call("viso_svo_features", self.h, _p(img), w, h, _p(u), _p(v), _p(c), _p(d), cap,
                  ctypes.byref(n))
        k = min(n.value, cap)
        return Features(u[:k].copy(), v[:k].copy(), c[:k].copy(), d[:k].copy())

    def match(self, f4) -> np.ndarray:
        """Circular matching of (L1, R1, L2, R2) -> (n, 4) index quads {l1, r1, l2, r2}."""
        arrs = [(np.ascontiguousarray(f.u, np.int32), np.ascontiguousarray(f.v, np.int32),
                 np.ascontiguousarray(f.cls, np.int32), np.ascontiguousarray(f.desc, np.uint8))
                for f in f4]
        P4 = ctypes.c_void_p * 4
        u4 = P4(*[a[0].ctypes.data for a in arrs])
        v4 = P4(*[a[1].ctypes.data for a in arrs])
        c4 = P4(*[a[2].ctypes.data for a in arrs])
        d4 = P4(*[a[3].ctypes.data for a in arrs])
        n4 = (ctypes.c_int32 * 4)(*[len(f) for f in f4])
        cap = max(1, len(f4[2]))
        quad = np.zeros((cap, 4), np.int32)
        n = ctypes.c_int32(0)
        _lib.call("viso_svo_match", self.h, u4, v4, c4, d4, n4, _p(quad), cap, ctypes.byref(n))
        return quad[:n.value].copy()

    def estimate(self, uv8: np.ndarray, frame: int):
        """RANSAC + Gauss-Newton on bucketed matches -> (motion12, inliers, n or -1)."""
        uv8 = np.ascontiguousarray(uv8, np.int32)
        m = np.zeros(12, np.float64)
        inl = np.zeros(max(1, len(uv8)), np.uint8)
        n = ctypes.c_int32(0)
        _lib.call("viso_svo_estimate", self.h, _p(uv8), len(uv8), frame, _p(m), _p(inl),
                  ctypes.byref(n))
        return m, inl[:len(uv8)].astype(bool), n.value


class VisualOdometryStereoRig(VisualOdometryStereo):
    """Multi-camera rig (BASELINE.json configs[4]): ``n_cams`` stereo cameras
    with shared parameters and rig -> camera extrinsics (n_cams x 12); one
    shared RANSAC + Gauss-Newton estimate of the rig motion per timestep."""

    def __init__(self, params: SvoParams, extrinsics: np.ndarray, device: int = 0):
        self.params = params
        self.extrinsics = np.ascontiguousarray(extrinsics, np.float64).reshape(-1, 12)
        self.n_cams = len(self.extrinsics)
        h = ctypes.c_void_p()
        _lib.call("viso_svo_rig_create", ctypes.byref(params), self.n_cams, _p(self.extrinsics), device,
                  ctypes.byref(h))
        self.h = h

    def process(self, lefts, rights) -> bool:
        """One timestep: lists of n_cams left / right images."""
        ls = [np.ascontiguousarray(x, np.uint8) for x in lefts]
        rs = [np.ascontiguousarray(x, np.uint8) for x in rights]
        h, w = ls[0].shape
        P = ctypes.c_void_p * self.n_cams
        dims = (ctypes.c_int32 * 3)(w, h, w)
        ok = ctypes.c_int32(0)
        _lib.call("viso_svo_rig_process", self.h, P(*[_p(x) for x in ls]), P(*[_p(x) for x in rs]), dims,
                  ctypes.byref(ok))
        return bool(ok.value)

    def process_device(self, left_ptrs, right_ptrs, n: int, pair_stride: int):
        """n timesteps in HBM: camera c's pairs at left_ptrs[c] / right_ptrs[c]."""
        P = ctypes.c_void_p * self.n_cams
        _lib.call("viso_svo_rig_process_device", self.h, P(*left_ptrs), P(*right_ptrs), n, pair_stride,
                  self.params.width)

    def getMatchCams(self) -> np.ndarray:  # noqa: N802
        """Camera of each match of getMatches()."""
        n = ctypes.c_size_t(0)
        _lib.call("viso_svo_get_match_cams", self.h, None, 0, ctypes.byref(n))
        out = np.zeros(max(1, n.value), np.uint8)
        _lib.call("viso_svo_get_match_cams", self.h, _p(out), n.value, ctypes.byref(n))
        return out[:n.value]


class Matcher:
    """Matcher facade: pushBack(left, right) twice, matchFeatures(), getMatches()."""

    def __init__(self, params: SvoParams, device: int = 0):
        self.vo = VisualOdometryStereo(params, device)
        self.sets = []

    def pushBack(self, left: np.ndarray, right: np.ndarray):  # noqa: N802
        self.sets = (self.sets + [(self.vo.features(left), self.vo.features(right))])[-2:]

    def matchFeatures(self) -> np.ndarray:  # noqa: N802
        (l1, r1), (l2, r2) = self.sets
        self.f4 = [l1, r1, l2, r2]
        self.quad = self.vo.match(self.f4)
        return self.quad

    def getMatches(self) -> np.ndarray:  # noqa: N802
        out = np.zeros((len(self.quad), 8), np.int32)
        for k in range(4):
            out[:, 2 * k] = self.f4[k].u[self.quad[:, k]]
            out[:, 2 * k + 1] = self.f4[k].v[self.quad[:, k]]
        return out
