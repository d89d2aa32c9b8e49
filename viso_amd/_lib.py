"""ctypes binding of the C ABI (include/viso/viso_c.h).

The product path loads ``viso_amd/libviso_amd.so`` (built in-tree by
``viso_amd/build.py``).  There is no CPU fallback: if the library is missing
or a call fails, an exception is raised.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VISO_LIB") or os.path.join(_HERE, "libviso_amd.so")

VISO_OK = 0
ERRORS = {-1: "VISO_ERR_ARG", -2: "VISO_ERR_HIP", -3: "VISO_ERR_CAPACITY",
          -4: "VISO_ERR_STATE", -5: "VISO_ERR_NODEVICE"}

STATE_INITIALIZATION, STATE_RUNNING, STATE_FINISHED = 0, 1, 2
KERNEL_IDS = {"pyramid": 0, "fast": 1, "klt": 2, "ransac": 3, "select": 4, "direct": 5,
              "lkalign": 6, "stereo": 7, "upload": 8}


class VisoError(RuntimeError):
    def __init__(self, fn: str, rc: int):
        super().__init__(f"{fn} failed: {ERRORS.get(rc, rc)}")
        self.rc = rc


class viso_params(ctypes.Structure):
    _fields_ = [
        ("fx", ctypes.c_double), ("fy", ctypes.c_double),
        ("cx", ctypes.c_double), ("cy", ctypes.c_double),
        ("width", ctypes.c_int32), ("height", ctypes.c_int32),
        ("reinitialize_after", ctypes.c_int32), ("fast_thresh", ctypes.c_int32),
        ("projection_error_thresh", ctypes.c_double), ("parallax_thresh", ctypes.c_double),
        ("disparity_squared_thresh", ctypes.c_double),
        ("photometric_error_thresh", ctypes.c_double),
        ("enable_tracking", ctypes.c_int32), ("ransac_e_iters", ctypes.c_int32),
        ("ransac_h_iters", ctypes.c_int32), ("ransac_confidence", ctypes.c_double),
        ("ransac_seed", ctypes.c_uint64), ("max_features", ctypes.c_int32),
        ("max_poses", ctypes.c_int32), ("batch_frames", ctypes.c_int32),
        ("precision", ctypes.c_int32), ("reserved", ctypes.c_int32 * 6),
    ]


_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_sz = ctypes.c_size_t
_d = ctypes.c_double

# name -> argtypes (restype int unless listed in _RESTYPES)
SIGNATURES = {
    "viso_default_params": [_vp, _d, _d, _d, _d, _i32, _i32],
    "viso_create": [_vp, ctypes.c_int, _vp],
    "viso_destroy": [_vp],
    "viso_process_frame": [_vp, _vp, _i32, _i32, _i32],
    "viso_process_stereo": [_vp, _vp, _vp, _vp],
    "viso_process_frames_device": [_vp, _vp, _vp, _i32, _sz],
    "viso_synchronize": [_vp],
    "viso_get_state": [_vp, _vp],
    "viso_get_poses": [_vp, _vp, _sz, _vp],
    "viso_get_points": [_vp, _vp, _sz, _vp],
    "viso_get_init_tracks": [_vp, _vp, _vp, _vp, _sz, _vp],
    "viso_get_alignment": [_vp, _vp, _vp, _vp, _vp, _sz, _vp],
    "viso_get_frame_stats": [_vp, _vp],
    "viso_set_frame_log": [_vp, _i32],
    "viso_get_config": [_vp, _vp],
    "viso_get_frame_log": [_vp, _vp, _sz, _vp],
    "viso_timing_enable": [_vp, _i32],
    "viso_timing_select": [_vp, ctypes.c_uint32],
    "viso_timing_get": [_vp, _i32, _vp, _vp],
    "viso_pyramid_dims": [_i32, _i32, _vp, _vp],
    "viso_pyramid": [_vp, _vp, _i32, _i32, _i32, _vp],
    "viso_fast": [_vp, _vp, _i32, _i32, _i32, _vp, _vp, _vp, _sz, _vp],
    "viso_klt": [_vp, _vp, _vp, _i32, _i32, _vp, _vp, _vp, _i32],
    "viso_direct_pose": [_vp, _vp, _vp, _i32, _i32, _vp, _i32, _vp, _vp],
    "viso_lk_align": [_vp, _vp, _vp, _i32, _vp, _vp, _i32, _i32, _vp, _i32, _vp, _vp, _vp,
                      _vp],
    "viso_pose_2d2d": [_vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp],
    "viso_stereo_match": [_vp, _vp, _vp, _i32, _i32, _vp, _vp, _i32, _i32, _vp, _vp],
    "viso_set_stereo": [_vp, _d, _i32, _i32],
    "viso_set_keyframes": [_vp, _i32, _i32],
    "viso_set_bundle_adjust": [_vp, _i32],
    "viso_photometric_ba": [_vp, _vp, _i32, _vp, _vp, _vp, _i32, _i32, _vp],
    "viso_version": [],
    # north-star stereo VO (include/viso/viso_svo.h)
    "viso_svo_default_params": [_vp, _i32, _i32, _d, _d, _d, _d, _d],
    "viso_svo_create": [_vp, ctypes.c_int, _vp],
    "viso_svo_destroy": [_vp],
    "viso_svo_process": [_vp, _vp, _vp, _vp, _vp],
    "viso_svo_process_device": [_vp, _vp, _vp, _i32, ctypes.c_int64, _i32],
    "viso_svo_synchronize": [_vp],
    "viso_svo_timing": [_vp, _i32, _vp, _vp],
    "viso_svo_get_motion": [_vp, _vp],
    "viso_svo_get_stats": [_vp, _vp],
    "viso_svo_get_poses": [_vp, _vp, _sz, _vp],
    "viso_svo_get_matches": [_vp, _vp, _vp, _sz, _vp],
    "viso_svo_features": [_vp, _vp, _i32, _i32, _vp, _vp, _vp, _vp, _i32, _vp],
    "viso_svo_match": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp],
    "viso_svo_estimate": [_vp, _vp, _i32, ctypes.c_int64, _vp, _vp, _vp],
    "viso_svo_rig_create": [_vp, _i32, _vp, ctypes.c_int, _vp],
    "viso_svo_rig_process": [_vp, _vp, _vp, _vp, _vp],
    "viso_svo_rig_process_device": [_vp, _vp, _vp, _i32, ctypes.c_int64, _i32],
    "viso_svo_get_match_cams": [_vp, _vp, _sz, _vp],
    # multi-camera photometric rig (include/viso/viso_rig.h)
    "viso_rig_create": [_vp, _i32, _vp, ctypes.c_int, _vp],
    "viso_rig_destroy": [_vp],
    "viso_rig_set_stereo": [_vp, _d, _i32, _i32],
    "viso_rig_process": [_vp, _vp, _vp, _vp],
    "viso_rig_process_device": [_vp, _vp, _vp, _i32, _sz],
    "viso_rig_synchronize": [_vp],
    "viso_rig_get_state": [_vp, _vp],
    "viso_rig_get_poses": [_vp, _vp, _sz, _vp],
    "viso_rig_get_points": [_vp, _i32, _vp, _sz, _vp],
    "viso_rig_get_level_stats": [_vp, _vp],
    # frame source (include/viso/viso_io.h)
    "viso_png_info": [ctypes.c_char_p, _vp, _vp],
    "viso_png_read_grey": [ctypes.c_char_p, _vp, _sz, _vp, _vp],
    "viso_png_decode_grey": [_vp, _sz, _vp, _sz, _vp, _vp],
    "viso_kitti_calib": [ctypes.c_char_p, _vp, _vp, _vp, _vp, _vp],
}
_RESTYPES = {"viso_version": ctypes.c_char_p}

_lib = None


def load(path: str | None = None):
    """Load the HIP library (raises if it has not been built)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise ImportError(
            f"viso_amd: {p} not found — build it with `python -m viso_amd.build` "
            "(there is no CPU fallback)")
    # One HIP runtime per process: torch ships its own libamdhip64.so.7.  If
    # torch is importable, load it first so that our NEEDED libamdhip64.so.7
    # binds to the already-loaded copy (soname match); loading ours first
    # would make torch map a second runtime that cannot open the device.
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    lib = ctypes.CDLL(p)
    for name, args in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:  # reported by tests/test_abi.py::test_exports
            continue
        fn.argtypes = args
        fn.restype = _RESTYPES.get(name, ctypes.c_int)
    if path is None:
        _lib = lib
    return lib


def built_hash(lib=None) -> str:
    """The source hash compiled into the library (viso_version's "src:")."""
    v = (lib or load()).viso_version().decode()
    return v.rsplit("src:", 1)[-1] if "src:" in v else ""


def check_source_hash(lib=None) -> str:
    """Raise if the loaded product library was built from other sources than
    the tree's (viso_amd/csrc, include/viso) — a stale prebuilt .so.  Returns
    the hash.  Variant libraries (VISO_LIB) are not checked."""
    from viso_amd import build as vbuild
    want = vbuild.source_hash()
    got = built_hash(lib)
    if os.environ.get("VISO_LIB") or os.environ.get("VISO_VARIANT"):
        return got
    if got != want:
        raise ImportError(f"viso_amd: {LIB_PATH} was built from sources {got!r}, the tree's are {want!r}: "
                          "rebuild with `python -m viso_amd.build`")
    return got


def call(name: str, *args) -> int:
    rc = getattr(load(), name)(*args)
    if rc != VISO_OK:
        raise VisoError(name, rc)
    return rc
