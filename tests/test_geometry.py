"""Initialisation geometry: PoseEstimation2d2d (src/viso.cpp:178-256) with the
repo's deterministic RANSAC restatements of cv::findEssentialMat /
cv::findHomography, cv::recoverPose, cv::decomposeHomographyMat, and
SelectMotion / Triangulate (src/viso.cpp:416-431, 520-638).

Parity vs OpenCV itself is unpinned (no OpenCV in the image, no reference
fixtures); the CPU tests pin the oracle with known-answer synthetic
geometry, the GPU tests require the HIP path to reproduce the oracle:
integer outputs (inlier masks, counts, chosen motion, RANSAC iteration
counts) exactly, floating outputs to 1e-12 relative."""
import numpy as np
import pytest

from tests import oracle_lib, seqdata

K_KITTI = (718.856, 718.856, 607.681, 184.715)


def rot(ax, ay, az):
    from scipy.spatial.transform import Rotation
    return Rotation.from_euler("xyz", [ax, ay, az]).as_matrix()


def synth_scene(n=400, seed=0, R=None, t=None, planar=False, outliers=0.0):
    rng = np.random.default_rng(seed)
    R = rot(0.01, 0.03, -0.005) if R is None else R
    t = np.array([0.2, 0.01, 0.05]) if t is None else t
    X = np.stack([rng.uniform(-6, 6, n), rng.uniform(-2, 2, n),
                  np.full(n, 20.0) if planar else rng.uniform(12, 40, n)], 1)
    x1 = X / X[:, 2:]
    Xc = X @ R.T + t
    x2 = Xc / Xc[:, 2:]
    k = int(outliers * n)
    if k:
        x2[:k, :2] += rng.uniform(-0.05, 0.05, (k, 2))
    return x1, x2, R, t, X


# ------------------------------------------------------------------ CPU: oracle pinning
def test_oracle_triangulate_exact():
    x1, x2, R, t, X = synth_scene(20)
    for i in range(20):
        P = oracle_lib.triangulate(R, t, x1[i], x2[i])
        assert np.allclose(P, X[i], rtol=1e-9)


def test_oracle_decompose_homography_recovers_motion():
    R = rot(0.02, -0.05, 0.01)
    t = np.array([0.3, -0.1, 0.2])
    n = np.array([0.0, 0.0, 1.0])
    d = 10.0
    H = R + np.outer(t, n) / d
    Rs, ts, ns = oracle_lib.decompose_homography(H * 3.7)
    assert len(Rs) == 4
    errs = [np.linalg.norm(Ri - R) + np.linalg.norm(ti - t / d) for Ri, ti in zip(Rs, ts)]
    # OpenCV's HomographyDecompInria takes v = 2 * sqrtf(...) in float: ~1e-6
    assert min(errs) < 1e-5
    # pure rotation -> one solution, t = 0
    Rs, ts, _ = oracle_lib.decompose_homography(R)
    assert len(Rs) == 1 and np.allclose(Rs[0], R) and np.allclose(ts[0], 0)


@pytest.mark.parametrize("outliers", [0.0, 0.3])
def test_oracle_ransac_essential_and_recover_pose(outliers):
    # recoverPose drops points farther than 50 x |t| (distanceThresh, unit t):
    # use a baseline that keeps the scene inside that range
    x1, x2, R, t, _ = synth_scene(300, seed=1, outliers=outliers, t=np.array([2.0, 0.1, 0.5]))
    thr = 0.3 / np.hypot(718.856, 718.856)
    good, E, mask, iters = oracle_lib.ransac("E", x1[:, :2], x2[:, :2], thr)
    k = int(outliers * 300)
    assert mask[k:].all() and not mask[:k].any()
    assert good == 300 - k and 0 < iters <= 1000
    g, Rr, tr, m2 = oracle_lib.recover_pose(E, x1[:, :2], x2[:, :2], mask)
    assert np.allclose(Rr, R, atol=1e-9)
    assert np.allclose(tr, t / np.linalg.norm(t), atol=1e-8)


def test_oracle_ransac_homography_planar():
    x1, x2, R, t, _ = synth_scene(200, seed=2, planar=True, outliers=0.2)
    thr = 0.3 / np.hypot(718.856, 718.856)
    good, H, mask, iters = oracle_lib.ransac("H", x1[:, :2], x2[:, :2], thr, iters=2000)
    assert good == 160 and mask[40:].all() and not mask[:40].any()
    Ht = R + np.outer(t, [0, 0, 1.0]) / 20.0
    assert np.allclose(H / H[2, 2], Ht / Ht[2, 2], atol=1e-9)


def test_oracle_pose_2d2d_selects_true_motion():
    # rotation-dominated motion (the reference keeps parallax <= 1 deg: quirk
    # src/viso.cpp:570) with enough disparity for the 225 px^2 gate
    R = rot(0.002, 0.03, 0.001)
    t = np.array([0.05, 0.0, 0.01])
    x1, x2, _, _, X = synth_scene(300, seed=3, R=R, t=t)
    out = oracle_lib.pose_2d2d(x1, x2, K_KITTI)
    assert out["ran"] == 1
    assert out["stats"][0] > 0.9 * 300
    # With rotation-dominated motion the reference's tests are weak: recoverPose's
    # 50*|t| distance cut leaves every E combination empty (ties -> first), and a
    # homography solution within ~0.5 deg passes every SelectMotion test for all
    # points.  Check the chosen rotation is close, not exact.
    ang = np.degrees(np.arccos(np.clip((np.trace(out["R"].T @ R) - 1) / 2, -1, 1)))
    assert ang < 1.0
    # T normalised by the mean depth of the inliers
    zs = out["points3d"][out["inliers"] == 1][:, 2]
    assert abs(zs.mean() - 1.0) < 1e-9


def test_oracle_pose_2d2d_gates():
    x1, x2, _, _, _ = synth_scene(9)
    assert oracle_lib.pose_2d2d(x1, x2, K_KITTI)["ran"] == 0  # N < 10 (src/viso.cpp:184)
    x1, _, _, _, _ = synth_scene(50)
    out = oracle_lib.pose_2d2d(x1, x1, K_KITTI)  # zero disparity (src/viso.cpp:216)
    assert out["ran"] == 0 and out["stats"][3] == 0


# ------------------------------------------------------------------ CPU: the device RANSAC scan
_DBL_MIN = 2.2250738585072014e-308


def _update_num_iters(p, ep, mp, max_iters):
    """cv::RANSACUpdateNumIters as oracle_geom.cpp ransac_update_num_iters."""
    import math
    p = min(max(p, 0.0), 1.0)
    ep = min(max(ep, 0.0), 1.0)
    num = max(1.0 - p, _DBL_MIN)
    den = 1.0 - math.pow(1.0 - ep, mp)
    if den < _DBL_MIN:
        return 0
    num, den = math.log(num), math.log(den)
    return max_iters if (den >= 0 or -num >= max_iters * (-den)) else int(round(num / den))


def _scan_sequential(counts, n, mp, max_iters, conf):
    niters, max_good, best, h = max_iters, 0, -1, 0
    while h < niters:
        c = counts[h]
        if c >= 0 and c > max(max_good, mp - 1):
            max_good, best = c, h
            niters = _update_num_iters(conf, (n - c) / n, mp, niters)
        h += 1
    return best, max_good, h


def _scan_records(counts, n, mp, max_iters, conf):
    """scan_kernel's form (geometry.hip): only the strict prefix-maximum
    records can change the loop state, and niters only shrinks, so the loop
    is the in-order walk over the records until one lies at or past niters;
    the loop variable at exit is max(niters, last record + 1)."""
    import math
    ln_num = math.log(max(1.0 - min(max(conf, 0.0), 1.0), _DBL_MIN))
    run, recs = mp - 1, []
    for h in range(max_iters):
        if counts[h] > run:
            run = counts[h]
            recs.append(h)
    niters, best, max_good, last = max_iters, -1, 0, -1
    for h in recs:
        if h >= niters:
            break
        best, max_good, last = h, counts[h], h
        ep = min(max((n - counts[h]) / n, 0.0), 1.0)
        den = 1.0 - math.pow(1.0 - ep, mp)
        if den < _DBL_MIN:
            niters = 0
            continue
        ld = math.log(den)
        if not (ld >= 0 or -ln_num >= niters * (-ld)):
            niters = int(round(ln_num / ld))
    return best, max_good, max(niters, last + 1)


def test_ransac_scan_record_walk_is_the_sequential_loop():
    rng = np.random.default_rng(1)
    for trial in range(4000):
        n = int(rng.integers(10, 3000))
        mp = int(rng.choice([4, 8]))
        max_iters = int(rng.choice([7, 50, 1000, 2000]))
        mode = trial % 3
        if mode == 0:
            counts = rng.integers(-1, n + 1, max_iters)
        elif mode == 1:
            counts = np.minimum(np.sort(rng.integers(-1, n + 1, max_iters)), n)
        else:
            counts = (rng.random(max_iters) * n * rng.random()).astype(int)
        counts = [int(c) for c in counts]
        assert _scan_sequential(counts, n, mp, max_iters, 0.99) == _scan_records(counts, n, mp, max_iters, 0.99)


def _pairwise(x):
    """The canonical pairwise tree over a power-of-two count of leaves."""
    x = list(x)
    while len(x) > 1:
        x = [x[2 * i] + x[2 * i + 1] for i in range(len(x) // 2)]
    return x[0]


def _normalize_kernel_sum(leaves, threads=1024):
    """normalize_kernel's disparity sum (geometry.hip): P = next pow2 >= n,
    thread t owns C = max(1, P / 1024) consecutive leaves folded by a
    binary-counter stack, the ascending-xor wave tree over 64 threads, then
    the pairwise top over the 16 waves; +0.0 leaves past n."""
    n = len(leaves)
    P = 1
    while P < n:
        P <<= 1
    C = P // threads if P > threads else 1
    per_thread = []
    for t in range(threads):
        stack = []
        for j in range(C):
            i = t * C + j
            x = leaves[i] if i < n else 0.0
            k = j
            while k & 1:
                x = stack.pop() + x
                k >>= 1
            stack.append(x)
        per_thread.append(stack[0])
    waves = []
    for w in range(threads // 64):
        v = per_thread[64 * w:64 * w + 64]
        off = 1
        while off < 64:  # ascending xor butterfly: every lane ends with the tree sum
            v = [v[i] + v[i ^ off] for i in range(64)]
            off <<= 1
        waves.append(v[0])
    return _pairwise(waves)


@pytest.mark.parametrize("n", [1, 10, 255, 256, 700, 1024, 1025, 5000, 8192, 32768])
def test_normalize_disparity_tree_is_the_canonical_tree(n):
    """The 1,024-thread normalisation sums the same pairwise tree over the P
    padded leaves as the oracle's tree_sum (sums of squares: adding +0.0
    leaves and subtrees is exact), so the disparity gate decides alike."""
    rng = np.random.default_rng(n)
    leaves = list(rng.random(n) ** 3 * 1e-3)
    P = 1
    while P < n:
        P <<= 1
    exp = _pairwise(leaves + [0.0] * (P - n))
    assert _normalize_kernel_sum(leaves) == exp


# ------------------------------------------------------------------ GPU parity
def _check_same(got, exp):
    st_g, st_e = got["stats"], exp["stats"]
    # integer decisions: exact
    for k in (0, 1, 2, 4, 5, 6, 7):
        assert st_g[k] == st_e[k], (k, st_g, st_e)
    assert abs(st_g[3] - st_e[3]) <= 1e-12 * max(1.0, abs(st_e[3]))
    assert np.array_equal(got["inliers"], exp["inliers"])
    assert np.allclose(got["R"], exp["R"], rtol=0, atol=1e-12)
    assert np.allclose(got["T"], exp["T"], rtol=1e-12, atol=1e-14)
    assert np.allclose(got["points3d"], exp["points3d"], rtol=1e-11, atol=1e-13)
    assert np.allclose(got["candidates"], exp["candidates"], rtol=1e-11, atol=1e-12)


@pytest.mark.gpu
def test_gpu_pose_2d2d_on_sequence_tracks():
    from viso_amd import default_context
    d = seqdata.initialised()
    k1, k2, _ = d["viso"].tracks()
    K = d["K"]
    Kinv = np.linalg.inv(np.array([[K[0], 0, K[2]], [0, K[1], K[3]], [0, 0, 1]]))
    p1 = np.c_[k1.astype(np.float64), np.ones(len(k1))] @ Kinv.T
    p2 = np.c_[k2.astype(np.float64), np.ones(len(k2))] @ Kinv.T
    ctx = default_context(K=K, width=seqdata.W, height=seqdata.H)
    got = ctx.pose_2d2d(p1, p2)
    exp = oracle_lib.pose_2d2d(p1, p2, K)
    assert exp["ran"] == 1 and exp["stats"][0] > 0
    _check_same(got, exp)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["general", "outliers", "planar", "small"])
def test_gpu_pose_2d2d_synthetic(case):
    from viso_amd import default_context
    R = rot(0.002, 0.03, 0.001)
    t = np.array([0.05, 0.0, 0.01])
    kw = {"general": {}, "outliers": {"outliers": 0.25}, "planar": {"planar": True},
          "small": {"n": 12}}[case]
    x1, x2, _, _, _ = synth_scene(kw.pop("n", 500), seed=7, R=R, t=t, **kw)
    ctx = default_context(K=K_KITTI, width=1242, height=375)
    got = ctx.pose_2d2d(x1, x2)
    exp = oracle_lib.pose_2d2d(x1, x2, K_KITTI)
    _check_same(got, exp)


@pytest.mark.gpu
def test_gpu_pose_2d2d_gates():
    from viso_amd import default_context
    ctx = default_context(K=K_KITTI, width=1242, height=375)
    x1, x2, _, _, _ = synth_scene(9)
    got = ctx.pose_2d2d(x1, x2)
    assert got["stats"][0] == 0 and got["stats"][2] == 0
    x1, _, _, _, _ = synth_scene(50)
    got = ctx.pose_2d2d(x1, x1)
    assert got["stats"][3] == 0 and got["stats"][2] == 0
