"""Deterministic synthetic test images (seeded numpy)."""
from __future__ import annotations

import numpy as np


def noise(h: int, w: int, seed: int = 0) -> np.ndarray:
    return np.random.default_rng(seed).integers(0, 256, (h, w), dtype=np.uint8)


def blocks(h: int, w: int, block: int = 6, seed: int = 0, jitter: int = 6) -> np.ndarray:
    rng = np.random.default_rng(seed)
    b = rng.integers(0, 256, (h // block + 2, w // block + 2))
    img = np.kron(b, np.ones((block, block)))[:h, :w]
    img = img + rng.integers(-jitter, jitter + 1, (h, w))
    return np.clip(img, 0, 255).astype(np.uint8)


def smooth(h: int, w: int, seed: int = 0, scale: int = 8) -> np.ndarray:
    """Bilinearly upsampled value noise (smooth gradients for LK/KLT)."""
    rng = np.random.default_rng(seed)
    gh, gw = h // scale + 3, w // scale + 3
    g = rng.uniform(0, 255, (gh, gw))
    ys = np.arange(h) / scale
    xs = np.arange(w) / scale
    y0 = np.floor(ys).astype(int)
    x0 = np.floor(xs).astype(int)
    fy = (ys - y0)[:, None]
    fx = (xs - x0)[None, :]
    a = g[y0][:, x0]
    b = g[y0][:, x0 + 1]
    c = g[y0 + 1][:, x0]
    d = g[y0 + 1][:, x0 + 1]
    v = (1 - fy) * ((1 - fx) * a + fx * b) + fy * ((1 - fx) * c + fx * d)
    return np.clip(np.rint(v), 0, 255).astype(np.uint8)


def mixed(h: int, w: int, seed: int = 0) -> np.ndarray:
    """Blocks plus smooth shading: many FAST corners with varied scores."""
    a = blocks(h, w, 7, seed).astype(np.int32)
    s = smooth(h, w, seed + 1, 16).astype(np.int32)
    return np.clip((a * 3 + s) // 4, 0, 255).astype(np.uint8)
