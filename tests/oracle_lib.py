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
    "oracle_set_sum_order": ([_i], None),
    "oracle_get_sum_order": ([], _i),
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
    "oracle_lk_trace": ([_vp, ctypes.c_long], None),
    "oracle_set_reference_copies": ([_i], None),
    "oracle_lk_trace_count": ([], ctypes.c_long),
    "oracle_triangulate": ([_vp, _vp, _vp, _vp, _vp], None),
    "oracle_ransac_essential": ([_vp, _vp, _i, _d, _d, _i, ctypes.c_uint64, _vp, _vp, _vp], _i),
    "oracle_ransac_homography": ([_vp, _vp, _i, _d, _d, _i, ctypes.c_uint64, _vp, _vp, _vp], _i),
    "oracle_recover_pose": ([_vp, _vp, _vp, _i, _vp, _vp, _vp], _i),
    "oracle_decompose_homography": ([_vp, _vp, _vp, _vp], _i),
    "oracle_select_motion": ([_vp, _vp, _i, _vp, _vp, _i, _vp, _d, _d, _vp, _vp, _vp, _vp, _vp],
                             _i),
    "oracle_pose_2d2d": ([_vp, _vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp], _i),
    "oracle_recover_pose": ([_vp, _vp, _vp, _i, _vp, _vp, _vp], _i),
    "oracle_default_params": ([_vp, _d, _d, _d, _d, _i, _i], None),
    "oracle_viso_create": ([_vp], _vp),
    "oracle_photometric_ba": ([_vp, _i, _i, _i, _vp, _vp, _vp, _vp, _i, _i, _vp], _i),
    "oracle_viso_set_bundle_adjust": ([_vp, _i], None),
    "oracle_rig_compose": ([_vp, _vp, _vp], None),
    "oracle_rig_adjoint": ([_vp, _vp], None),
    "oracle_rig_direct": ([_i, _vp, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp], None),
    "oracle_rig_create": ([_i, _i, _i, _vp, _i, _vp, ctypes.c_double, _i, _i], _vp),
    "oracle_rig_destroy": ([_vp], None),
    "oracle_rig_process": ([_vp, _vp, _vp], None),
    "oracle_rig_state": ([_vp], _i),
    "oracle_rig_num_poses": ([_vp], _i),
    "oracle_rig_poses": ([_vp, _vp], None),
    "oracle_rig_num_points": ([_vp, _i], _i),
    "oracle_rig_points": ([_vp, _i, _vp], None),
    "oracle_rig_level_stats": ([_vp, _vp], None),
    "oracle_viso_destroy": ([_vp], None),
    "oracle_viso_on_new_frame": ([_vp, _vp], None),
    "oracle_viso_on_new_stereo": ([_vp, _vp, _vp], None),
    "oracle_viso_set_stereo": ([_vp, _d, _i, _i], None),
    "oracle_viso_set_keyframes": ([_vp, _i, _i], None),
    "oracle_stereo_points": ([_vp, _vp, _i, _i, _vp, _vp, _i, _i, _i, _vp, _d, _vp], _i),
    "oracle_viso_state": ([_vp], _i),
    "oracle_viso_num_poses": ([_vp], _i),
    "oracle_viso_poses": ([_vp, _vp], None),
    "oracle_viso_num_points": ([_vp], _i),
    "oracle_viso_points": ([_vp, _vp], None),
    "oracle_viso_last_stats": ([_vp, _vp], None),
    "oracle_viso_tracks": ([_vp, _vp, _vp, _vp, _i], _i),
    "oracle_viso_alignment": ([_vp, _vp, _vp, _vp, _vp, _i], _i),
    "oracle_viso_keyframe_poses": ([_vp, _vp, _i], _i),
    "oracle_stereo_match": ([_vp, _vp, _i, _i, _vp, _vp, _i, _i, _vp, _vp], None),
    "oracle_svo_default_params": ([_vp, _i, _i, _d, _d, _d, _d, _d], None),
    "oracle_svo_features": ([_vp, _i, _i, _vp, _i, _vp, _vp, _vp, _vp], _i),
    "oracle_svo_responses": ([_vp, _i, _i, _vp, _vp], None),
    "oracle_svo_match": ([_vp, _vp, _vp, _vp, _vp, _i, _vp, _vp, _i], _i),
    "oracle_svo_bucket": ([_vp, _i, _i, _i, _vp, _vp], _i),
    "oracle_svo_estimate": ([_vp, _i, ctypes.c_int64, _vp, _vp, _vp], _i),
    "oracle_svo_rig_estimate": ([_vp, _vp, _i, ctypes.c_int64, _vp, _vp, _vp, _vp], _i),
    "oracle_svo_sad_evals": ([_i], ctypes.c_uint64),
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


def klt(ref_pyr, cur_pyr, w, h, kp1, kp2, thresh=14400.0):
    lib = load()
    kp1 = np.ascontiguousarray(kp1, np.float32)
    kp2 = np.ascontiguousarray(kp2, np.float32).copy()
    n = kp1.shape[0]
    succ = np.zeros(n, np.uint8)
    lib.oracle_klt(ptr(np.ascontiguousarray(ref_pyr)), ptr(np.ascontiguousarray(cur_pyr)), w, h,
                   ptr(kp1), ptr(kp2), ptr(succ), n, thresh)
    return kp2, succ


def direct_pose(last_pyr, cur_pyr, w, h, K, points, pose_last, pose_init):
    lib = load()
    pts = np.ascontiguousarray(points, np.float64).reshape(-1, 3)
    Kd = np.asarray(K, np.float64)
    pl = np.ascontiguousarray(pose_last, np.float64).reshape(12)
    pio = np.ascontiguousarray(pose_init, np.float64).reshape(12).copy()
    lib.oracle_direct_pose(ptr(np.ascontiguousarray(last_pyr)), ptr(np.ascontiguousarray(cur_pyr)),
                           w, h, ptr(Kd), ptr(pts), pts.shape[0], ptr(pl), ptr(pio))
    return pio


def lk_align(kf_pyrs, kf_poses, cur_pyr, cur_pose, w, h, K, points, thresh=14400.0):
    lib = load()
    kfs = [np.ascontiguousarray(k, np.uint8) for k in kf_pyrs]
    arr = (ctypes.c_void_p * len(kfs))(*[k.ctypes.data for k in kfs])
    kposes = np.ascontiguousarray(kf_poses, np.float64).reshape(-1, 12)
    pts = np.ascontiguousarray(points, np.float64).reshape(-1, 3)
    n = pts.shape[0]
    pk = np.zeros(n, np.int32)
    sc = np.zeros(n, np.uint8)
    ub = np.zeros((n, 2))
    ua = np.zeros((n, 2))
    Kd = np.asarray(K, np.float64)
    cp = np.ascontiguousarray(cur_pose, np.float64).reshape(12)
    lib.oracle_lk_align(ctypes.cast(arr, ctypes.c_void_p), ptr(kposes), len(kfs),
                        ptr(np.ascontiguousarray(cur_pyr)), ptr(cp), w, h, ptr(Kd), ptr(pts), n,
                        thresh, ptr(pk), ptr(sc), ptr(ub), ptr(ua))
    return pk, sc, ub, ua


def pose_2d2d(p1, p2, K, w=1242, h=375, R0=None, T0=None, **kw):
    lib = load()
    p1 = np.ascontiguousarray(p1, np.float64).reshape(-1, 3)
    p2 = np.ascontiguousarray(p2, np.float64).reshape(-1, 3)
    n = p1.shape[0]
    prm = params(K, w, h, **kw)
    R = np.ascontiguousarray(np.eye(3) if R0 is None else R0, np.float64).reshape(9).copy()
    T = np.ascontiguousarray(np.zeros(3) if T0 is None else T0, np.float64).reshape(3).copy()
    inl = np.zeros(max(n, 1), np.uint8)
    pts = np.zeros((max(n, 1), 3))
    cand = np.zeros((5, 12))
    st = np.zeros(8)
    Kd = np.asarray(K, np.float64)
    ran = lib.oracle_pose_2d2d(ptr(p1), ptr(p2), n, ptr(Kd), ctypes.byref(prm), ptr(R), ptr(T),
                               ptr(inl), ptr(pts), ptr(cand), ptr(st))
    return {"ran": ran, "R": R.reshape(3, 3), "T": T, "inliers": inl[:n], "points3d": pts[:n],
            "candidates": cand[:int(st[2])], "stats": st}


def stereo_points(left, right, xs, ys, max_disp, min_disp, K, base):
    """Stereo-initialisation points (oracle_stereo_points): (m, 3)."""
    left = np.ascontiguousarray(left, np.uint8)
    right = np.ascontiguousarray(right, np.uint8)
    h, w = left.shape
    xs = np.ascontiguousarray(xs, np.int32)
    ys = np.ascontiguousarray(ys, np.int32)
    n = len(xs)
    pts = np.zeros((n + 1, 3))
    k = np.asarray(K, np.float64)
    m = load().oracle_stereo_points(ptr(left), ptr(right), w, h, ptr(xs), ptr(ys), n, max_disp,
                                    min_disp, ptr(k), float(base), ptr(pts))
    return pts[:m]


def stereo_match(left, right, xs, ys, max_disp):
    lib = load()
    left = np.ascontiguousarray(left, np.uint8)
    right = np.ascontiguousarray(right, np.uint8)
    h, w = left.shape
    xs = np.ascontiguousarray(xs, np.int32)
    ys = np.ascontiguousarray(ys, np.int32)
    n = len(xs)
    d = np.zeros(n, np.int32)
    s = np.zeros(n, np.int32)
    lib.oracle_stereo_match(ptr(left), ptr(right), w, h, ptr(xs), ptr(ys), n, max_disp, ptr(d),
                            ptr(s))
    return d, s


def triangulate(R, T, x1, x2):
    lib = load()
    R = np.ascontiguousarray(R, np.float64).reshape(9)
    T = np.ascontiguousarray(T, np.float64).reshape(3)
    a = np.ascontiguousarray(x1, np.float64).reshape(3)
    b = np.ascontiguousarray(x2, np.float64).reshape(3)
    P = np.zeros(3)
    lib.oracle_triangulate(ptr(R), ptr(T), ptr(a), ptr(b), ptr(P))
    return P


def decompose_homography(H):
    lib = load()
    H = np.ascontiguousarray(H, np.float64).reshape(9)
    Rs = np.zeros((4, 3, 3))
    ts = np.zeros((4, 3))
    ns = np.zeros((4, 3))
    m = lib.oracle_decompose_homography(ptr(H), ptr(Rs), ptr(ts), ptr(ns))
    return Rs[:m], ts[:m], ns[:m]


def ransac(kind, q1, q2, thresh, conf=0.99, iters=1000, seed=0x5eed5eed):
    lib = load()
    q1 = np.ascontiguousarray(q1, np.float64).reshape(-1, 2)
    q2 = np.ascontiguousarray(q2, np.float64).reshape(-1, 2)
    n = q1.shape[0]
    M = np.zeros(9)
    mask = np.zeros(max(n, 1), np.uint8)
    it = ctypes.c_int32(0)
    fn = lib.oracle_ransac_essential if kind == "E" else lib.oracle_ransac_homography
    good = fn(ptr(q1), ptr(q2), n, thresh, conf, iters, seed, ptr(M), ptr(mask), ctypes.byref(it))
    return good, M.reshape(3, 3), mask[:n], it.value


def recover_pose(E, q1, q2, mask):
    lib = load()
    q1 = np.ascontiguousarray(q1, np.float64).reshape(-1, 2)
    q2 = np.ascontiguousarray(q2, np.float64).reshape(-1, 2)
    mask = np.ascontiguousarray(mask, np.uint8).copy()
    E = np.ascontiguousarray(E, np.float64).reshape(9)
    R = np.zeros(9)
    t = np.zeros(3)
    good = lib.oracle_recover_pose(ptr(E), ptr(q1), ptr(q2), q1.shape[0], ptr(mask), ptr(R), ptr(t))
    return good, R.reshape(3, 3), t, mask


class OracleParams(ctypes.Structure):
    _fields_ = [("fx", ctypes.c_double), ("fy", ctypes.c_double), ("cx", ctypes.c_double),
                ("cy", ctypes.c_double), ("width", ctypes.c_int32), ("height", ctypes.c_int32),
                ("reinitialize_after", ctypes.c_int32), ("fast_thresh", ctypes.c_int32),
                ("projection_error_thresh", ctypes.c_double), ("parallax_thresh", ctypes.c_double),
                ("disparity_squared_thresh", ctypes.c_double),
                ("photometric_error_thresh", ctypes.c_double),
                ("enable_tracking", ctypes.c_int32), ("ransac_e_iters", ctypes.c_int32),
                ("ransac_h_iters", ctypes.c_int32), ("ransac_confidence", ctypes.c_double),
                ("ransac_seed", ctypes.c_uint64)]


def params(K, w, h, **kw):
    p = OracleParams()
    load().oracle_default_params(ctypes.byref(p), K[0], K[1], K[2], K[3], w, h)
    for k, v in kw.items():
        setattr(p, k, v)
    return p


class Viso:
    """Oracle of the whole per-frame path (Viso::OnNewFrame)."""

    def __init__(self, K, w, h, **kw):
        self.lib = load()
        self.p = params(K, w, h, **kw)
        self.v = self.lib.oracle_viso_create(ctypes.byref(self.p))
        self.w, self.h = w, h

    def __del__(self):
        try:
            self.lib.oracle_viso_destroy(self.v)
        except Exception:
            pass

    def on_new_frame(self, img):
        img = np.ascontiguousarray(img, np.uint8)
        assert img.shape == (self.h, self.w)
        self.lib.oracle_viso_on_new_frame(self.v, ptr(img))

    def set_stereo(self, baseline, max_disp=128, min_disp=1):
        self.lib.oracle_viso_set_stereo(self.v, float(baseline), int(max_disp), int(min_disp))

    def set_keyframes(self, interval, ngood_permille=500):
        self.lib.oracle_viso_set_keyframes(self.v, int(interval), int(ngood_permille))

    def set_bundle_adjust(self, iterations):
        self.lib.oracle_viso_set_bundle_adjust(self.v, int(iterations))

    def on_new_stereo(self, left, right):
        left = np.ascontiguousarray(left, np.uint8)
        right = np.ascontiguousarray(right, np.uint8)
        assert left.shape == right.shape == (self.h, self.w)
        self.lib.oracle_viso_on_new_stereo(self.v, ptr(left), ptr(right))

    @property
    def state(self):
        return self.lib.oracle_viso_state(self.v)

    def poses(self):
        n = self.lib.oracle_viso_num_poses(self.v)
        out = np.zeros((n, 12))
        if n:
            self.lib.oracle_viso_poses(self.v, ptr(out))
        return out

    def points(self):
        n = self.lib.oracle_viso_num_points(self.v)
        out = np.zeros((n, 3))
        if n:
            self.lib.oracle_viso_points(self.v, ptr(out))
        return out

    def stats(self):
        out = np.zeros(16)
        self.lib.oracle_viso_last_stats(self.v, ptr(out))
        return out

    def tracks(self):
        cap = 1 << 16
        k1 = np.zeros((cap, 2), np.float32)
        k2 = np.zeros((cap, 2), np.float32)
        s = np.zeros(cap, np.uint8)
        n = self.lib.oracle_viso_tracks(self.v, ptr(k1), ptr(k2), ptr(s), cap)
        return k1[:n].copy(), k2[:n].copy(), s[:n].copy()

    def alignment(self):
        cap = 1 << 16
        pk = np.zeros(cap, np.int32)
        s = np.zeros(cap, np.uint8)
        ub = np.zeros((cap, 2))
        ua = np.zeros((cap, 2))
        n = self.lib.oracle_viso_alignment(self.v, ptr(pk), ptr(s), ptr(ub), ptr(ua), cap)
        return pk[:n].copy(), s[:n].copy(), ub[:n].copy(), ua[:n].copy()

    def keyframe_poses(self):
        out = np.zeros((8, 12))
        n = self.lib.oracle_viso_keyframe_poses(self.v, ptr(out), 8)
        return out[:n].copy()


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


# ----------------------------------------------------------------- stereo VO (SVO) spec
class SvoParams(ctypes.Structure):
    """viso_svo_params (include/viso/viso_svo.h)."""
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


def svo_params(w, h, fx, fy, cu, cv, base, **kw) -> SvoParams:
    p = SvoParams()
    load().oracle_svo_default_params(ctypes.byref(p), w, h, fx, fy, cu, cv, base)
    for k, v in kw.items():
        setattr(p, k, v)
    return p


class SvoFeatures:
    """Features of one image: u, v, cls (int32), desc (n x 32 u8)."""

    def __init__(self, u, v, cls, desc):
        self.u, self.v, self.cls, self.desc = u, v, cls, desc

    def __len__(self):
        return len(self.u)


def svo_features(img: np.ndarray, p: SvoParams) -> SvoFeatures:
    lib = load()
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    cap = p.max_features
    u, v, c = (np.zeros(cap, np.int32) for _ in range(3))
    d = np.zeros((cap, 32), np.uint8)
    n = lib.oracle_svo_features(ptr(img), w, h, ctypes.byref(p), cap, ptr(u), ptr(v), ptr(c), ptr(d))
    n = min(n, cap)
    return SvoFeatures(u[:n].copy(), v[:n].copy(), c[:n].copy(), d[:n].copy())


def svo_responses(img: np.ndarray):
    lib = load()
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    b = np.zeros((h, w), np.int32)
    c = np.zeros((h, w), np.int32)
    lib.oracle_svo_responses(ptr(img), w, h, ptr(b), ptr(c))
    return b, c


def svo_match(f4, h: int, p: SvoParams) -> np.ndarray:
    """Circular matches of (L1, R1, L2, R2) -> (n, 4) index quads {l1, r1, l2, r2}."""
    lib = load()
    arrs = [(np.ascontiguousarray(f.u), np.ascontiguousarray(f.v), np.ascontiguousarray(f.cls),
             np.ascontiguousarray(f.desc)) for f in f4]
    P4 = ctypes.c_void_p * 4
    u4 = P4(*[a[0].ctypes.data for a in arrs])
    v4 = P4(*[a[1].ctypes.data for a in arrs])
    c4 = P4(*[a[2].ctypes.data for a in arrs])
    d4 = P4(*[a[3].ctypes.data for a in arrs])
    n4 = np.array([len(f) for f in f4], np.int32)
    cap = max(1, len(f4[2]))
    quad = np.zeros((cap, 4), np.int32)
    n = lib.oracle_svo_match(u4, v4, c4, d4, ptr(n4), h, ctypes.byref(p), ptr(quad), cap)
    return quad[:n].copy()


def svo_uv8(f4, quad: np.ndarray) -> np.ndarray:
    """Index quads -> {u_l1, v_l1, u_r1, v_r1, u_l2, v_l2, u_r2, v_r2} per match."""
    out = np.zeros((len(quad), 8), np.int32)
    for k in range(4):
        out[:, 2 * k] = f4[k].u[quad[:, k]]
        out[:, 2 * k + 1] = f4[k].v[quad[:, k]]
    return out


def svo_bucket(uv8: np.ndarray, w: int, h: int, p: SvoParams) -> np.ndarray:
    lib = load()
    uv8 = np.ascontiguousarray(uv8, np.int32)
    keep = np.zeros(max(1, len(uv8)), np.uint8)
    lib.oracle_svo_bucket(ptr(uv8), len(uv8), w, h, ctypes.byref(p), ptr(keep))
    return keep[:len(uv8)].astype(bool)


def svo_estimate(uv8: np.ndarray, frame: int, p: SvoParams):
    """-> (motion12, inlier mask, n_inliers or -1)."""
    lib = load()
    uv8 = np.ascontiguousarray(uv8, np.int32)
    motion = np.zeros(12, np.float64)
    inl = np.zeros(max(1, len(uv8)), np.uint8)
    n = lib.oracle_svo_estimate(ptr(uv8), len(uv8), frame, ctypes.byref(p), ptr(motion), ptr(inl))
    return motion, inl[:len(uv8)].astype(bool), n


class SvoSequence:
    """The SVO spec end to end on the CPU: features -> circular matching ->
    bucketing -> RANSAC + Gauss-Newton; poses accumulate T_wc = T_wc * Tr^-1."""

    def __init__(self, p: SvoParams):
        self.p = p
        self.prev = None
        self.frame = 0
        self.pose = np.eye(4)
        self.poses = [np.concatenate([self.pose[:3, :3].ravel(), self.pose[:3, 3]])]
        self.motion = None
        self.stats = None

    def process(self, left, right) -> bool:
        fl, fr = svo_features(left, self.p), svo_features(right, self.p)
        ok = False
        self.motion = np.array([1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0], np.float64)
        n_match = n_bucket = n_inl = 0
        if self.prev is not None:
            f4 = [self.prev[0], self.prev[1], fl, fr]
            quad = svo_match(f4, left.shape[0], self.p)
            uv8 = svo_uv8(f4, quad)
            keep = svo_bucket(uv8, left.shape[1], left.shape[0], self.p)
            sel = uv8[keep]
            n_match, n_bucket = len(uv8), len(sel)
            motion, inl, n = svo_estimate(sel, self.frame, self.p)
            self.matches, self.inliers = sel, inl
            if n >= 6:
                ok = True
                n_inl = n
                self.motion = motion
                T = np.eye(4)
                T[:3, :3] = motion[:9].reshape(3, 3)
                T[:3, 3] = motion[9:]
                self.pose = self.pose @ np.linalg.inv(T)
            self.poses.append(np.concatenate([self.pose[:3, :3].ravel(), self.pose[:3, 3]]))
        self.stats = [len(fl), len(fr), n_match, n_bucket, n_inl, int(ok)]
        self.prev = (fl, fr)
        self.frame += 1
        return ok


def svo_rig_estimate(uv8: np.ndarray, cams: np.ndarray, frame: int, p: SvoParams, extr: np.ndarray):
    """Rig motion from the matches of all cameras -> (motion12, inlier mask, n or -1)."""
    lib = load()
    uv8 = np.ascontiguousarray(uv8, np.int32)
    cams = np.ascontiguousarray(cams, np.int32)
    extr = np.ascontiguousarray(extr, np.float64)
    motion = np.zeros(12, np.float64)
    inl = np.zeros(max(1, len(uv8)), np.uint8)
    n = lib.oracle_svo_rig_estimate(ptr(uv8), ptr(cams), len(uv8), frame, ctypes.byref(p), ptr(extr),
                                    ptr(motion), ptr(inl))
    return motion, inl[:len(uv8)].astype(bool), n


class SvoRigSequence:
    """Multi-camera rig (BASELINE.json configs[4]) on the CPU: per camera the
    SVO features, circular matching and bucketing; one RANSAC + Gauss-Newton
    over the matches of all cameras (camera order, then left order) for the
    rig motion; rig poses accumulate T_wr = T_wr * Tr^-1."""

    def __init__(self, p: SvoParams, extr: np.ndarray):
        self.p = p
        self.extr = np.ascontiguousarray(extr, np.float64)
        self.n_cams = len(extr)
        self.prev = None
        self.frame = 0
        self.pose = np.eye(4)
        self.poses = [np.concatenate([self.pose[:3, :3].ravel(), self.pose[:3, 3]])]
        self.motion = None
        self.stats = None

    def process(self, lefts, rights) -> bool:
        feats = [(svo_features(l, self.p), svo_features(r, self.p)) for l, r in zip(lefts, rights)]
        ok = False
        self.motion = np.array([1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0], np.float64)
        n_match = n_bucket = n_inl = 0
        if self.prev is not None:
            sels, cams = [], []
            h, w = lefts[0].shape
            for c in range(self.n_cams):
                f4 = [self.prev[c][0], self.prev[c][1], feats[c][0], feats[c][1]]
                quad = svo_match(f4, h, self.p)
                uv8 = svo_uv8(f4, quad)
                keep = svo_bucket(uv8, w, h, self.p)
                n_match += len(uv8)
                sels.append(uv8[keep])
                cams.append(np.full(int(keep.sum()), c, np.int32))
            sel = np.concatenate(sels).reshape(-1, 8)
            cam = np.concatenate(cams)
            n_bucket = len(sel)
            motion, inl, n = svo_rig_estimate(sel, cam, self.frame, self.p, self.extr)
            self.matches, self.cams, self.inliers = sel, cam, inl
            if n >= 6:
                ok = True
                n_inl = n
                self.motion = motion
                T = np.eye(4)
                T[:3, :3] = motion[:9].reshape(3, 3)
                T[:3, 3] = motion[9:]
                self.pose = self.pose @ np.linalg.inv(T)
            self.poses.append(np.concatenate([self.pose[:3, :3].ravel(), self.pose[:3, 3]]))
        self.stats = [sum(len(f[0]) for f in feats), sum(len(f[1]) for f in feats), n_match, n_bucket,
                      n_inl, int(ok)]
        self.prev = feats
        self.frame += 1
        return ok


# ----------------------------------------------------------------- multi-camera rig
class Rig:
    """oracle/oracle_rig.cpp: the multi-camera photometric rig spec."""

    def __init__(self, K, w, h, extrinsics, baseline, max_disp=128, min_disp=1, fast_thresh=50):
        self.E = np.ascontiguousarray(extrinsics, np.float64).reshape(-1, 12)
        self.n = len(self.E)
        k = np.asarray(K, np.float64)
        self.h = load().oracle_rig_create(self.n, w, h, ptr(k), fast_thresh, ptr(self.E), float(baseline),
                                          max_disp, min_disp)

    def __del__(self):
        try:
            load().oracle_rig_destroy(self.h)
        except Exception:
            pass

    def process(self, lefts, rights=None):
        ls = [np.ascontiguousarray(x, np.uint8) for x in lefts]
        P = ctypes.c_void_p * self.n
        if rights is None:
            load().oracle_rig_process(self.h, P(*[ptr(x) for x in ls]), None)
        else:
            rs = [np.ascontiguousarray(x, np.uint8) for x in rights]
            load().oracle_rig_process(self.h, P(*[ptr(x) for x in ls]), P(*[ptr(x) for x in rs]))

    @property
    def state(self):
        return load().oracle_rig_state(self.h)

    @property
    def poses(self):
        n = load().oracle_rig_num_poses(self.h)
        out = np.zeros((max(n, 1), 12))
        load().oracle_rig_poses(self.h, ptr(out))
        return out[:n]

    def points(self, cam):
        n = load().oracle_rig_num_points(self.h, cam)
        out = np.zeros((max(n, 1), 3))
        load().oracle_rig_points(self.h, cam, ptr(out))
        return out[:n]

    def level_stats(self):
        out = np.zeros((4, 50))
        load().oracle_rig_level_stats(self.h, ptr(out))
        return out


def rig_compose(E, T):
    out = np.zeros(12)
    load().oracle_rig_compose(ptr(np.ascontiguousarray(E, np.float64)), ptr(np.ascontiguousarray(T, np.float64)),
                              ptr(out))
    return out


def rig_adjoint(E):
    out = np.zeros(36)
    load().oracle_rig_adjoint(ptr(np.ascontiguousarray(E, np.float64)), ptr(out))
    return out.reshape(6, 6)


def rig_direct(last_pyrs, cur_pyrs, w, h, K, points, E, cam_last, pose_seed):
    """One rig direct pose (levels 3..0): returns (pose12, stats[4][50])."""
    n = len(last_pyrs)
    P = ctypes.c_void_p * n
    lp = [np.ascontiguousarray(x, np.uint8) for x in last_pyrs]
    cp = [np.ascontiguousarray(x, np.uint8) for x in cur_pyrs]
    pts = [np.ascontiguousarray(x, np.float64).reshape(-1, 3) for x in points]
    npts = np.array([len(x) for x in pts], np.int32)
    k = np.asarray(K, np.float64)
    E = np.ascontiguousarray(E, np.float64).reshape(-1, 12)
    cl = np.ascontiguousarray(cam_last, np.float64).reshape(-1, 12)
    pose = np.ascontiguousarray(pose_seed, np.float64).copy()
    stats = np.zeros((4, 50))
    load().oracle_rig_direct(n, P(*[ptr(x) for x in lp]), P(*[ptr(x) for x in cp]), w, h, ptr(k),
                             P(*[ptr(x) for x in pts]), ptr(npts), ptr(E), ptr(cl), ptr(pose), ptr(stats))
    return pose, stats


# ----------------------------------------------------------------- photometric BA
def photometric_ba(kf_imgs, kf_poses, points, host, K, iterations=5):
    """oracle/oracle_ba.cpp: returns (poses (k, 12), points (n, 3), report
    (iterations, 4): cost, candidate cost, mu, accepted; active edges)."""
    imgs = [np.ascontiguousarray(x, np.uint8) for x in kf_imgs]
    h, w = imgs[0].shape
    P = ctypes.c_void_p * len(imgs)
    poses = np.ascontiguousarray(kf_poses, np.float64).reshape(-1, 12).copy()
    pts = np.ascontiguousarray(points, np.float64).reshape(-1, 3).copy()
    hst = np.ascontiguousarray(host, np.int32)
    rep = np.zeros((max(iterations, 1), 4))
    k = np.asarray(K, np.float64)
    na = load().oracle_photometric_ba(P(*[ptr(x) for x in imgs]), len(imgs), w, h, ptr(k), ptr(poses), ptr(pts),
                                      ptr(hst), len(pts), iterations, ptr(rep))
    return poses, pts, rep[:iterations], na
