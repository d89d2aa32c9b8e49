"""Host model of the LK engines' window that follows the point
(viso_amd/csrc/track.hip window_follow / sample_win_follow).

A re-placed window is a window of the level's continuous buffer: origin
(x0, y0) = lane 0's (int(x), int(y)) - 7, not clamped to the image, byte
(r, c) = buf[(y0 + r) w + x0 + c] or 0 outside the buffer.  This checks that
every bilinear sample the GPU then takes from the window equals
GetPixelValue's (include/common.h:35-42: int() base, floor() weights, taps
outside the continuous buffer read 0) for patches inside, across and beyond
the image border, and that one re-placement holds the whole 8x8 patch.
"""
import numpy as np

WIN = 24


def _get_pixel(buf, w, h, x, y):
    n = w * h
    base = int(y) * w + int(x)
    def tap(i):
        return float(buf[i]) if 0 <= i < n else 0.0
    d0, d1, d2, d3 = tap(base), tap(base + 1), tap(base + w), tap(base + w + 1)
    xx, yy = x - np.floor(x), y - np.floor(y)
    return (1 - xx) * (1 - yy) * d0 + xx * (1 - yy) * d1 + (1 - xx) * yy * d2 + xx * yy * d3


def _window(buf, w, h, x0, y0):
    n = w * h
    idx = (y0 + np.arange(WIN))[:, None] * w + x0 + np.arange(WIN)[None, :]
    out = np.zeros((WIN, WIN), np.float64)
    ok = (idx >= 0) & (idx < n)
    out[ok] = buf[idx[ok]]
    return out


def _win_sample(win, x0, y0, x, y):
    ix, iy = int(x), int(y)
    r, c = iy - y0, ix - x0
    assert 0 <= r < WIN - 1 and 0 <= c < WIN - 1
    xx, yy = x - np.floor(x), y - np.floor(y)
    return ((1 - xx) * (1 - yy) * win[r, c] + xx * (1 - yy) * win[r, c + 1] + (1 - xx) * yy * win[r + 1, c]
            + xx * yy * win[r + 1, c + 1])


def test_followed_window_reads_getpixelvalue_bytes_at_and_beyond_the_border():
    rng = np.random.default_rng(7)
    w, h = 97, 41
    buf = rng.integers(0, 256, w * h).astype(np.uint8)
    lanes = [((l >> 3) - 4, (l & 7) - 4) for l in range(64)]
    centres = [(rng.uniform(-12, w + 12), rng.uniform(-12, h + 12)) for _ in range(400)]
    centres += [(0.25, 0.5), (-3.75, 2.0), (w - 1.5, h - 0.25), (w + 3.3, -2.2)]
    for cx, cy in centres:
        xs = [cx + px for px, _ in lanes]
        ys = [cy + py for _, py in lanes]
        x0, y0 = int(xs[0]) - 7, int(ys[0]) - 7  # lane 0: px = py = -4
        win = _window(buf, w, h, x0, y0)
        for x, y in zip(xs, ys):
            got = _win_sample(win, x0, y0, x, y)
            assert got == _get_pixel(buf, w, h, x, y), (cx, cy, x, y)
