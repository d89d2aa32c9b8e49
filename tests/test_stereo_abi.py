"""C ABI surface + the north-star stereo SAD stage.

* every function declared in include/viso/*.h is exported by the HIP
  library (loads without a GPU; no compute calls);
* the stereo stage (no reference counterpart: parity vs the repo's own CPU
  restatement, bit-exact integer SAD / disparities; "parity unpinned vs
  reference")."""
import ctypes
import os
import re

import numpy as np
import pytest

from tests import oracle_lib, seqdata

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    names = set()
    inc = os.path.join(ROOT, "include", "viso")
    for f in os.listdir(inc):
        if not f.endswith(".h"):
            continue
        src = open(os.path.join(inc, f)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"\b(viso_[a-z0-9_]+)\s*\(", src):
            names.add(m.group(1))
    return names


def test_library_exports_every_declared_symbol():
    from viso_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in sorted(_declared()) if not hasattr(lib, n)]
    assert not missing, missing
    assert len(_declared()) >= 25


def test_version_and_host_only_calls():
    from viso_amd import _lib, api
    lib = _lib.load()
    assert b"gfx950" in lib.viso_version()
    dims, total = api.pyramid_dims(1242, 375)
    assert dims == [(1242, 375), (621, 187), (310, 93), (155, 46)]
    assert total == 1242 * 375 + 621 * 187 + 310 * 93 + 155 * 46
    p = api.default_params(718.856, 718.856, 607.19, 185.22, 1242, 375)
    assert p.reinitialize_after == 10 and p.fast_thresh == 50
    assert p.photometric_error_thresh == 14400.0 and p.disparity_squared_thresh == 225.0


def _build_facade(tmp_path):
    import subprocess
    exe = str(tmp_path / "facade_check")
    libdir = os.path.join(ROOT, "viso_amd")
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "facade_check.cpp"), "-L", libdir,
                    "-lviso_amd", f"-Wl,-rpath,{libdir}", "-o", exe], check=True)
    return exe


def test_cpp_facade_compiles_and_links(tmp_path):
    import subprocess
    exe = _build_facade(tmp_path)
    out = subprocess.run([exe], capture_output=True, text=True, check=True)
    assert "facade ok" in out.stdout


@pytest.mark.gpu
def test_gpu_cpp_facade_runs(tmp_path):
    """The C++ facades on the GPU, and the Keyframe accessors
    (include/keyframe.h:50-112) against the oracle: Pyramids() bit-exact,
    GetPixelValue / GetGradient / Project / IsInside / ViewingAngle with the
    reference's expressions."""
    import subprocess
    from viso_amd.synth import Sequence
    exe = _build_facade(tmp_path)
    dump = str(tmp_path / "keyframe.bin")
    out = subprocess.run([exe, "run", dump], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "poses" in out.stdout and "handler:" in out.stdout
    W, H = 1242, 375
    img = Sequence(W, H, seed=0).image(0)
    flat = oracle_lib.pyramid(img)
    raw = open(dump, "rb").read()
    assert np.array_equal(np.frombuffer(raw[:flat.size], np.uint8), flat)
    nb = flat.size
    pyr, off = [], 0
    for lw, lh in [(1242, 375), (621, 187), (310, 93), (155, 46)]:
        pyr.append(flat[off:off + lw * lh].reshape(lh, lw))
        off += lw * lh
    vals = np.frombuffer(raw[nb:], np.float64)

    def px(level, x, y):  # include/keyframe.h:50-57 (taps inside here)
        m = pyr[level].astype(np.float64)
        ix, iy = int(x), int(y)
        xx, yy = x - np.floor(x), y - np.floor(y)
        return ((1 - xx) * (1 - yy) * m[iy, ix] + xx * (1 - yy) * m[iy, ix + 1] + (1 - xx) * yy * m[iy + 1, ix]
                + xx * yy * m[iy + 1, ix + 1])

    xs = [10.25, 100.5, 333.75, 64.0, 140.125]
    ys = [7.5, 40.25, 20.0, 80.75, 30.5]
    k = 0
    for level in range(4):
        for x0, y0 in zip(xs, ys):
            s = 0.5 ** level
            x, y = x0 * s * 2.0, y0 * s * 2.0
            exp = [px(level, x, y), 0.5 * (px(level, x + 1, y) - px(level, x - 1, y)),
                   0.5 * (px(level, x, y + 1) - px(level, x, y - 1))]
            assert np.array_equal(vals[k:k + 3], exp), (level, x, y)
            k += 3
    R = np.array([[0.8, -0.6, 0], [0.6, 0.8, 0], [0, 0, 1]])
    Pc = R @ np.array([1.0, -0.5, 12.0]) + np.array([0.1, -0.2, 0.3])
    for level in range(4):
        s = 0.5 ** level
        u, v = s * (Pc[0] / Pc[2] * 718.856 + 607.19), s * (Pc[1] / Pc[2] * 718.856 + 185.22)
        h, w = pyr[level].shape
        np.testing.assert_allclose(vals[k:k + 2], [u, v], rtol=1e-14)
        assert vals[k + 2] == float(0 <= u < w and 0 <= v < h)
        k += 3
    np.testing.assert_allclose(vals[k], np.arccos(Pc[2] / np.linalg.norm(Pc)), rtol=1e-14)


def test_oracle_stereo_recovers_known_disparity():
    rng = np.random.default_rng(0)
    left = rng.integers(0, 256, (60, 200), dtype=np.uint8)
    right = np.roll(left, -7, axis=1)  # right(x) = left(x + 7): disparity 7
    xs = np.array([50, 100, 150, 3, 197], np.int32)
    ys = np.array([30, 20, 40, 30, 30], np.int32)
    d, s = oracle_lib.stereo_match(left, right, xs, ys, 32)
    assert list(d[:3]) == [7, 7, 7] and list(s[:3]) == [0, 0, 0]
    assert d[3] == -1 and d[4] == -1  # patch leaves the image


@pytest.mark.gpu
@pytest.mark.parametrize("max_disp", [0, 63, 64, 128, 200])
def test_gpu_stereo_bitexact(max_disp):
    from viso_amd import default_context
    left, right = seqdata.image(0), seqdata.image(0, cam=1)
    xs, ys, _ = oracle_lib.fast(left, 50)
    ctx = default_context()
    got = ctx.stereo_match(left, right, xs, ys, max_disp)
    exp = oracle_lib.stereo_match(left, right, xs, ys, max_disp)
    assert np.array_equal(got[0], exp[0]) and np.array_equal(got[1], exp[1])
    if max_disp >= 64:
        # KITTI-like geometry: back-wall points (z ~ 32 m) have d ~ 12 px
        assert np.median(exp[0][exp[0] >= 0]) > 3


def test_library_built_from_this_trees_sources():
    """viso_version() carries the hash of the sources the library was built
    from (viso_amd/build.py source_hash); it must be this tree's, so a stale
    prebuilt library cannot pass for the current code (no GPU call)."""
    from viso_amd import _lib
    from viso_amd import build as vbuild
    lib = _lib.load()
    assert _lib.built_hash(lib) == vbuild.source_hash()
