"""TEST INFRASTRUCTURE ONLY — an independent numpy restatement of the integer
image stages, used to cross-check the C++ oracle (oracle/oracle_image.cpp).

It is written differently on purpose (vectorised, brute force) so that a
transcription error in one restatement shows up as a mismatch:

* ``pyr_down``  — cv::pyrDown (include/keyframe.h:42-43): separable 5-tap
  [1 4 6 4 1] filter via ``np.pad(mode="reflect")`` (== BORDER_REFLECT_101),
  decimation, ``(s + 128) >> 8``; destination size truncated (keyframe.h:43).
* ``fast``      — cv::FAST(img, kps, t) TYPE_9_16 with NMS (src/viso.cpp:104):
  the corner score is found by BRUTE FORCE as the largest threshold t' >= t at
  which the 9-of-16 contiguous-arc test still passes (instead of OpenCV's
  min/max arc recurrence), then strict 3x3 NMS and row-major order.

Only tests/ import this module.
"""
from __future__ import annotations

import numpy as np

CIRCLE = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3),
          (0, -3), (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def pyr_dims(w: int, h: int, levels: int = 4):
    dims = [(w, h)]
    for _ in range(levels - 1):
        w, h = int(w * 0.5), int(h * 0.5)
        dims.append((w, h))
    return dims


def pyr_down(src: np.ndarray, dw: int, dh: int) -> np.ndarray:
    k = np.array([1, 4, 6, 4, 1], dtype=np.int64)
    s = np.pad(src.astype(np.int64), 2, mode="reflect")
    # horizontal then vertical 5-tap filter, evaluated only at even centres
    hs = np.zeros((s.shape[0], dw), dtype=np.int64)
    for j in range(5):
        hs += k[j] * s[:, j: j + 2 * dw: 2][:, :dw]
    out = np.zeros((dh, dw), dtype=np.int64)
    for i in range(5):
        out += k[i] * hs[i: i + 2 * dh: 2][:dh]
    return ((out + 128) >> 8).astype(np.uint8)


def pyramid(img: np.ndarray, levels: int = 4):
    out = [img]
    for _ in range(levels - 1):
        h, w = out[-1].shape
        out.append(pyr_down(out[-1], int(w * 0.5), int(h * 0.5)))
    return out


def _circle_stack(img: np.ndarray) -> np.ndarray:
    h, w = img.shape
    a = img.astype(np.int32)
    st = np.zeros((16, h, w), dtype=np.int32)
    for k, (dx, dy) in enumerate(CIRCLE):
        st[k] = np.roll(np.roll(a, -dy, axis=0), -dx, axis=1)
    return st


def _corner_at(diff: np.ndarray, t: int) -> np.ndarray:
    """diff: (16,h,w) circle - centre.  True where >= 9 contiguous (circular)
    circle pixels are all brighter (> t) or all darker (< -t)."""
    res = np.zeros(diff.shape[1:], dtype=bool)
    for sign in (1, -1):
        good = (sign * diff) > t
        for start in range(16):
            idx = [(start + j) % 16 for j in range(9)]
            res |= np.all(good[idx], axis=0)
    return res


def fast_scores(img: np.ndarray, thresh: int) -> np.ndarray:
    h, w = img.shape
    diff = _circle_stack(img) - img.astype(np.int32)[None]
    valid = np.zeros((h, w), dtype=bool)
    valid[3:h - 3, 3:w - 3] = True
    score = np.zeros((h, w), dtype=np.int32)
    alive = _corner_at(diff, thresh) & valid
    t = thresh
    cur = alive.copy()
    while cur.any() and t < 256:
        score[cur] = t
        t += 1
        cur = cur & _corner_at(diff, t)
    return score


def fast(img: np.ndarray, thresh: int):
    """Returns (xs, ys, scores) in row-major order."""
    s = fast_scores(img, thresh)
    p = np.pad(s, 1)
    c = p[1:-1, 1:-1]
    keep = c > 0
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            if dx == 0 and dy == 0:
                continue
            keep &= c > p[1 + dy: p.shape[0] - 1 + dy, 1 + dx: p.shape[1] - 1 + dx]
    ys, xs = np.nonzero(keep)
    return xs.astype(np.int32), ys.astype(np.int32), c[ys, xs].astype(np.int32)
