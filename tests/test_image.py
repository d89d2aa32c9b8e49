"""Image pass: pyramid (cv::pyrDown, include/keyframe.h:28-46) and FAST-9/16 +
NMS (cv::FAST, src/viso.cpp:104).  Integer work: bit-exact everywhere.

CPU tests pin the C++ oracle against the independent numpy restatement
(oracle/numpy_ref.py) and hand-derived known answers; GPU tests compare the
HIP kernels (through the C ABI) with the oracle."""
import numpy as np
import pytest

from oracle import numpy_ref as nr
from tests import images, oracle_lib

SIZES = [(375, 1242), (61, 97), (17, 33), (120, 160), (187, 621), (46, 155), (16, 16)]


# ------------------------------------------------------------------ CPU: the device FAST formulation
_DX = [0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1]
_DY = [3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3]


def _rot16(m, s):
    return ((m >> s) | (m << (16 - s))) & 0xFFFF


def _run9(m):
    a1 = m & _rot16(m, 1)
    a2 = a1 & _rot16(a1, 2)
    a3 = a2 & _rot16(a2, 4)
    return a3 & _rot16(m, 8)


@pytest.mark.parametrize("thresh", [0, 20, 50, 255])
def test_fast_packed_arc_test_matches_oracle_score_map(thresh):
    """fast_tile_kernel's corner test, restated in numpy with its 16-bit
    wrapping arithmetic (image.hip): per circle position k the sign bits of
    (v + t) - C_k and C_k - (v - t) shifted into two 16-bit masks, and a run of
    >= 9 contiguous set bits found by rotate-and-AND (runs of 2, 4, 8, then 9);
    the corners' cornerScore (min / max arcs) then reproduces the oracle's
    score map exactly (OpenCV's scan over 25 circle samples with its
    early-outs is the same predicate)."""
    img = images.mixed(120, 300, seed=3).astype(np.int64)
    h, w = img.shape
    v = img[3:h - 3, 3:w - 3]
    vb, vd = (v + thresh) & 0xFFFF, (v - thresh) & 0xFFFF
    mb = np.zeros_like(v)
    md = np.zeros_like(v)
    circ = [img[3 + _DY[k]:h - 3 + _DY[k], 3 + _DX[k]:w - 3 + _DX[k]] for k in range(16)]
    for k in range(16):
        mb = (mb >> 1) | (((vb - circ[k]) & 0xFFFF) & 0x8000)
        md = (md >> 1) | (((circ[k] - vd) & 0xFFFF) & 0x8000)
    corner = (_run9(mb) | _run9(md)) != 0
    dd = [v - c for c in circ]
    a0 = np.full(v.shape, thresh)
    for k in range(0, 16, 2):
        a = np.minimum(dd[(k + 1) % 16], dd[(k + 2) % 16])
        for j in range(3, 9):
            a = np.minimum(a, dd[(k + j) % 16])
        a0 = np.maximum(a0, np.minimum(a, dd[k]))
        a0 = np.maximum(a0, np.minimum(a, dd[(k + 9) % 16]))
    b0 = -a0
    for k in range(0, 16, 2):
        b = np.maximum(dd[(k + 1) % 16], dd[(k + 2) % 16])
        for j in range(3, 9):
            b = np.maximum(b, dd[(k + j) % 16])
        b0 = np.minimum(b0, np.maximum(b, dd[k]))
        b0 = np.minimum(b0, np.maximum(b, dd[(k + 9) % 16]))
    score = np.where(corner, -b0 - 1, 0).astype(np.uint8)
    lib = oracle_lib.load()
    smap = np.zeros(h * w, np.uint8)
    im8 = np.ascontiguousarray(img.astype(np.uint8))
    lib.oracle_fast_score_map(im8.ctypes.data, w, h, thresh, smap.ctypes.data)
    exp = smap.reshape(h, w)[3:h - 3, 3:w - 3]
    assert np.array_equal(score, exp)


# ------------------------------------------------------------------ CPU: oracle pinning
@pytest.mark.parametrize("h,w", SIZES)
def test_oracle_pyramid_vs_numpy(h, w):
    img = images.mixed(h, w, seed=h * 7 + w)
    got = oracle_lib.pyramid(img)
    exp = np.concatenate([p.ravel() for p in nr.pyramid(img)])
    assert np.array_equal(got, exp)


def test_pyramid_dims_truncate():
    # include/keyframe.h:43 — Size(cols*0.5, rows*0.5) truncates: 375 -> 187
    assert nr.pyr_dims(1242, 375) == [(1242, 375), (621, 187), (310, 93), (155, 46)]
    assert nr.pyr_dims(1920, 1080) == [(1920, 1080), (960, 540), (480, 270), (240, 135)]


def test_pyrdown_known_answer():
    # constant image stays constant; single bright pixel spreads the 5x5 kernel /256
    img = np.full((8, 8), 77, np.uint8)
    assert np.all(nr.pyr_down(img, 4, 4) == 77)
    img = np.zeros((16, 16), np.uint8)
    img[8, 8] = 255
    d = oracle_lib.pyramid(img)[256:256 + 64].reshape(8, 8)
    k = np.array([1, 4, 6, 4, 1])
    # dst(4,4) is centred on src(8,8): 255*36/256 -> (9180+128)>>8 = 36
    assert d[4, 4] == (255 * 36 + 128) >> 8
    # dst(4,5) centred on src(8,10): weight k[0]*k[2]=6 -> (1530+128)>>8 = 6
    assert d[4, 5] == (255 * k[2] * k[0] + 128) >> 8


@pytest.mark.parametrize("kind", ["noise", "blocks", "mixed", "smooth"])
@pytest.mark.parametrize("thresh", [20, 50])
def test_oracle_fast_vs_numpy(kind, thresh):
    h, w = 48, 64
    img = getattr(images, kind)(h, w, seed=3)
    got = oracle_lib.fast(img, thresh)
    exp = nr.fast(img, thresh)
    for g, e in zip(got, exp):
        assert np.array_equal(g, e)


def test_fast_known_answers():
    # a single dark pixel on a bright background is a 16-of-16 "brighter" corner:
    # every circle pixel is 200 brighter -> score = 200 - 1 (cornerScore returns -b0-1)
    img = np.full((16, 16), 230, np.uint8)
    img[8, 8] = 30
    xs, ys, sc = oracle_lib.fast(img, 50)
    assert list(zip(xs, ys, sc)) == [(8, 8, 199)]
    # below threshold -> nothing; exactly at the threshold is not a corner (strict >)
    img[8, 8] = 180
    assert len(oracle_lib.fast(img, 50)[0]) == 0
    # two equal-score corners next to each other: strict-> NMS suppresses both
    img = np.full((16, 20), 230, np.uint8)
    img[8, 8] = 30
    img[8, 9] = 30
    xs, ys, sc = oracle_lib.fast(img, 50)
    assert len(xs) == 0 or not (8 in xs and 9 in xs)
    # corners in rows/cols < 3 or >= size-3 are never reported
    img = np.full((16, 16), 230, np.uint8)
    img[2, 8] = 30
    img[8, 13] = 30
    assert len(oracle_lib.fast(img, 50)[0]) == 0


def test_fast_order_row_major():
    img = images.mixed(120, 160, seed=11)
    xs, ys, _ = oracle_lib.fast(img, 20)
    assert len(xs) > 50
    key = ys.astype(np.int64) * 100000 + xs
    assert np.all(np.diff(key) > 0)


# ------------------------------------------------------------------ GPU parity
@pytest.mark.gpu
# sizes: the bench frame, odd/even widths, strip edges of the 248-column
# waves (dst widths 248k +- 1), levels under 8 columns (scalar form) and
# between 8 and 16 (packed form with both borders in one strip).  Levels 2
# and 3 of images at least 16 columns wide come from the tail launch (bands
# of level-3 rows sized to the chunk: 3 images here, 11 and 133 in the
# batched test); narrower images (15, 8 columns) take per-level launches.
@pytest.mark.parametrize("h,w", [(375, 1242), (61, 97), (1080, 1920), (16, 16), (187, 621),
                                 (8, 8), (9, 17), (20, 15), (50, 497), (30, 993), (12, 994),
                                 (9, 1001), (41, 2047), (33, 31), (18, 64),
                                 (24, 4000), (67, 16), (300, 4096)])
def test_gpu_pyramid_bitexact(h, w):
    from viso_amd import default_context
    ctx = default_context()
    imgs = np.stack([images.mixed(h, w, seed=s) for s in range(3)])
    got = ctx.pyramid(imgs)
    for i in range(3):
        assert np.array_equal(got[i], oracle_lib.pyramid(imgs[i]))


@pytest.mark.gpu
@pytest.mark.parametrize("n,h,w", [(11, 375, 1242), (133, 61, 97), (20, 375, 1242), (32, 187, 621),
                                   (33, 375, 1242)])
def test_gpu_pyramid_batched(n, h, w):
    """Chunks of >= 8 images deal the bands of an image to one XCD (the
    tail launch's block -> (image, band) map, idle blocks past the last
    image); more than kPyrBatch = 128 images split into launches.  Chunks of
    <= 32 images take 4-row level-1 bands, 33 the 8-row ones."""
    from viso_amd import default_context
    ctx = default_context()
    imgs = np.stack([images.mixed(h, w, seed=100 + s) for s in range(n)])
    got = ctx.pyramid(imgs)
    for i in range(n):
        assert np.array_equal(got[i], oracle_lib.pyramid(imgs[i])), i


@pytest.mark.gpu
def test_gpu_pyramid_chunk_sizes_repeated():
    """Back-to-back chunks of different sizes (both level-1 band heights)
    and images stay bit-exact."""
    from viso_amd import default_context
    ctx = default_context()
    for rep, n in enumerate([20, 1, 32, 40, 7, 20]):
        imgs = np.stack([images.mixed(375, 1242, seed=300 + 40 * rep + s) for s in range(n)])
        got = ctx.pyramid(imgs)
        for i in range(n):
            assert np.array_equal(got[i], oracle_lib.pyramid(imgs[i])), (rep, i)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,h,w,thresh", [
    ("mixed", 375, 1242, 50), ("noise", 375, 1242, 50), ("blocks", 120, 160, 20),
    ("mixed", 1080, 1920, 50), ("smooth", 64, 64, 10), ("noise", 16, 16, 50),
    ("mixed", 375, 1242, 0), ("mixed", 375, 1242, 255)])
def test_gpu_fast_bitexact(kind, h, w, thresh):
    from viso_amd import default_context
    ctx = default_context()
    img = getattr(images, kind)(h, w, seed=5)
    got = ctx.fast(img, thresh)
    exp = oracle_lib.fast(img, thresh)
    assert len(got[0]) == len(exp[0])
    for g, e in zip(got, exp):
        assert np.array_equal(g, e)


@pytest.mark.gpu
def test_gpu_fast_empty_and_capacity():
    from viso_amd import default_context
    ctx = default_context()
    flat = np.full((100, 100), 128, np.uint8)
    assert len(ctx.fast(flat, 50)[0]) == 0
    img = images.noise(375, 1242, seed=9)
    full = oracle_lib.fast(img, 20)
    got = ctx.fast(img, 20, cap=100)
    assert np.array_equal(got[0], full[0][:100]) and np.array_equal(got[1], full[1][:100])
