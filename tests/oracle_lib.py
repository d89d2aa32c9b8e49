"""TEST INFRASTRUCTURE ONLY — ctypes loader + numpy wrappers for the CPU oracle
(oracle/, see oracle/viso_oracle.h).  Builds oracle/_build/libviso_oracle.so
with make when it is missing or stale."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB = os.path.join(ORACLE_DIR, "_build", "libviso_oracle.so")

_vp = ctypes.c_void_p
_i = ctypes.c_int
_d = ctypes.c_double

SIG = {
    "oracle_pyramid_dims": ([_i, _i, _vp], None),
    "oracle_pyramid_bytes": ([_i, _i], ctypes.c_size_t),
    "oracle_pyr_down": ([_vp, _i, _i, _vp, _i, _i], None),
    "oracle_pyramid": ([_vp, _i, _i, _vp], None),
    "oracle_fast": ([_vp, _i, _i, _i, _vp, _vp, _vp, _i], _i),
    "oracle_fast_score_map": ([_vp, _i, _i, _i, _vp], None),
    "oracle_sample": ([_vp, _i, _i, _d, _d], _d),
    "oracle_gradient": ([_vp, _i, _i, _d, _d, _vp], None),
    "oracle_klt": ([_vp, _vp, _i, _i, _vp, _vp, _vp, _i, _d], None),
    "oracle_direct_pose_level": ([_vp, _vp, _i, _i, _vp, _vp, _i, _vp, _vp, _i, _vp], None),
    "oracle_direct_pose": ([_vp, _vp, _i, _i, _vp, _vp, _i, _vp, _vp], None),
    "oracle_se3_exp_left": ([_vp, _vp, _vp], None),
    "oracle_lk_align": ([_vp, _vp, _i, _vp, _vp, _i, _i, _vp, _vp, _i, _d, _vp, _vp, _vp, _vp],
                        None),
    "oracle_triangulate": ([_vp, _vp, _vp, _vp, _vp], None),
    "oracle_ransac_essential": ([_vp, _vp, _i, _d, _d, _i, ctypes.c_uint64, _vp, _vp, _vp], _i),
    "oracle_ransac_homography": ([_vp, _vp, _i, _d, _d, _i, ctypes.c_uint64, _vp, _vp, _vp], _i),
    "oracle_recover_pose": ([_vp, _vp, _vp, _i, _vp, _vp, _vp], _i),
    "oracle_decompose_homography": ([_vp, _vp, _vp, _vp], _i),
    "oracle_select_motion": ([_vp, _vp, _i, _vp, _vp, _i, _vp, _d, _d, _vp, _vp, _vp, _vp, _vp],
                             _i),
    "oracle_pose_2d2d": ([_vp, _vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp], _i),
    "oracle_default_params": ([_vp, _d, _d, _d, _d, _i, _i], None),
    "oracle_viso_create": ([_vp], _vp),
    "oracle_viso_destroy": ([_vp], None),
    "oracle_viso_on_new_frame": ([_vp, _vp], None),
    "oracle_viso_state": ([_vp], _i),
    "oracle_viso_num_poses": ([_vp], _i),
    "oracle_viso_poses": ([_vp, _vp], None),
    "oracle_viso_num_points": ([_vp], _i),
    "oracle_viso_points": ([_vp, _vp], None),
    "oracle_viso_last_stats": ([_vp, _vp], None),
    "oracle_viso_tracks": ([_vp, _vp, _vp, _vp, _i], _i),
    "oracle_viso_alignment": ([_vp, _vp, _vp, _vp, _vp, _i], _i),
}

_lib = None


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    for f in os.listdir(ORACLE_DIR):
        if f.endswith((".cpp", ".h", ".hpp", "Makefile")):
            if os.path.getmtime(os.path.join(ORACLE_DIR, f)) > t:
                return True
    return False


def build():
    if _stale():
        subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
    return LIB


def load():
    global _lib
    if _lib is None:
        build()
        lib = ctypes.CDLL(LIB)
        for name, (args, res) in SIG.items():
            fn = getattr(lib, name, None)
            if fn is None:
                continue
            fn.argtypes = args
            fn.restype = res
        _lib = lib
    return _lib


def ptr(a: np.ndarray):
    return a.ctypes.data


# ----------------------------------------------------------------- wrappers
def pyramid(img: np.ndarray) -> np.ndarray:
    lib = load()
    h, w = img.shape
    img = np.ascontiguousarray(img, dtype=np.uint8)
    out = np.zeros(lib.oracle_pyramid_bytes(w, h), np.uint8)
    lib.oracle_pyramid(ptr(img), w, h, ptr(out))
    return out


def fast(img: np.ndarray, thresh: int, cap: int = 1 << 20):
    lib = load()
    h, w = img.shape
    img = np.ascontiguousarray(img, dtype=np.uint8)
    xs = np.zeros(cap, np.int32)
    ys = np.zeros(cap, np.int32)
    sc = np.zeros(cap, np.int32)
    n = lib.oracle_fast(ptr(img), w, h, thresh, ptr(xs), ptr(ys), ptr(sc), cap)
    n = min(n, cap)
    return xs[:n].copy(), ys[:n].copy(), sc[:n].copy()
