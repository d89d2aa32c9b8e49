"""The tree-sum restatement against a literal one (VERDICT r01 "Next" 1a).

The oracle replaces the reference's running sums (H += J J^T, b += -e J,
cost += e^2 at src/viso.cpp:308-310, 727-729, 888-890; the disparity and
mean-depth sums at :199-201, :622-625) by canonical pairwise trees, which the
device reproduces bit for bit.  Here the oracle runs each sequence twice —
tree order and the reference's own running-sum order (oracle_set_sum_order,
tests/drift.py) — over 200 frames of:
  * the bench sequence at 1242x375, monocular (KLT + 2D-2D init + SelectMotion,
    then direct pose + LK alignment);
  * the bench sequence at 1242x375 with the stereo initialisation;
  * KITTI's native 1241x376 (the KITTI-format fixture's renderer output,
    tests/test_kitti_e2e.py decodes its PNGs to these same pairs), stereo.
Bars: every discrete decision identical frame by frame (state, KLT-surviving
tracks = KLT success, SelectMotion inlier masks, direct nGood, LK pairs and
success flags) and poses within the north star's 1e-4 rel-Frobenius.  The
measured drift is recorded in DESIGN.md §2 (tools/literal_drift.py writes
profiles/r02_literal_drift.json)."""
import concurrent.futures as cf

import pytest

from tests import drift

N = 200
CASES = {"mono_1242x375": (1242, 375, False), "stereo_1242x375": (1242, 375, True),
         "stereo_1241x376": (1241, 376, True)}


def run_case(name, n=N):
    from viso_amd.synth import Sequence
    w, h, stereo = CASES[name]
    seq = Sequence(w, h, seed=0)
    frames = [seq.frame(f) for f in range(n)]
    return drift.compare(seq.K, w, h, frames, seq.p.baseline if stereo else 0.0)


@pytest.fixture(scope="module")
def results():
    with cf.ThreadPoolExecutor(len(CASES)) as ex:
        futs = {k: ex.submit(run_case, k) for k in CASES}
        return {k: f.result() for k, f in futs.items()}


@pytest.mark.parametrize("case", list(CASES))
def test_tree_sums_match_literal_running_sums(results, case):
    r = results[case]
    assert r["mismatch"] == [], r["mismatch"][:5]
    assert r["pose_counts"][0] == r["pose_counts"][1] >= N - 10
    # tracking ran on (nearly) every frame and the map stayed in view
    assert min(r["nGood"][-10:]) > 500
    assert r["pose_max_rel_frobenius"] < 1e-4
    # measured: <= 2.6e-14; a regression far above that means
    # the restatement changed, not rounding
    assert r["pose_max_rel_frobenius"] < 1e-10


def test_literal_order_is_not_the_tree_order():
    """The switch really changes the summation order (else the test above
    compares the tree with itself): one DirectPoseEstimationSingleLayer call
    on the bench sequence gives H / b sums that differ in their last bits
    between the two orders, and agree to ~1e-13 relative."""
    import ctypes

    import numpy as np

    from tests import oracle_lib, seqdata
    lib = oracle_lib.load()
    init = seqdata.initialised(0)
    f0 = init["init_frame"]
    last, cur = seqdata.pyramid(f0), seqdata.pyramid(f0 + 1)
    pts = np.ascontiguousarray(init["points"], np.float64)
    K = np.asarray(init["K"], np.float64)
    pose_last = np.ascontiguousarray(init["kf_poses"][-1], np.float64)
    stats = []
    for mode in (0, 1):
        lib.oracle_set_sum_order(mode)
        try:
            pose = pose_last.copy()
            st = np.zeros(50)
            lib.oracle_direct_pose_level(oracle_lib.ptr(last), oracle_lib.ptr(cur), seqdata.W, seqdata.H,
                                         oracle_lib.ptr(K), oracle_lib.ptr(pts), len(pts),
                                         oracle_lib.ptr(pose_last), oracle_lib.ptr(pose), 0,
                                         oracle_lib.ptr(st))
            stats.append(st)
        finally:
            lib.oracle_set_sum_order(0)
    assert lib.oracle_get_sum_order() == 0
    t, l = stats
    assert t[0] == l[0] > 500  # nGood
    Ht, Hl = t[2:38], l[2:38]
    assert not np.array_equal(Ht, Hl)
    assert np.abs(Ht - Hl).max() <= 1e-12 * np.abs(Ht).max()
