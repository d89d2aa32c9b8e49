"""Frame source: PNG -> grey and KITTI odometry sequences (include/viso/viso_io.h).

``read_png`` restates the reference's ``cv::imread(file, 0)``
(include/frame_sequence.h:28-30) in the library's own decoder (zlib +
PNG filters, no OpenCV / PIL).  ``KittiSequence`` reads a KITTI odometry
sequence directory (``image_0/%06d.png``, ``image_1/%06d.png``,
``calib.txt``) — the north star's "KITTI-format grey pairs".
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _lib


def png_info(path: str):
    w, h = ctypes.c_int32(0), ctypes.c_int32(0)
    _lib.call("viso_png_info", os.fsencode(path), ctypes.byref(w), ctypes.byref(h))
    return w.value, h.value


def read_png(path: str) -> np.ndarray:
    """Grey image (h, w) uint8 of a PNG file (cv::imread(path, IMREAD_GRAYSCALE))."""
    w, h = png_info(path)
    out = np.empty((h, w), np.uint8)
    _lib.call("viso_png_read_grey", os.fsencode(path), out.ctypes.data, out.size, None, None)
    return out


def decode_png(data: bytes) -> np.ndarray:
    w, h = ctypes.c_int32(0), ctypes.c_int32(0)
    buf = np.frombuffer(data, np.uint8)
    _lib.call("viso_png_decode_grey", buf.ctypes.data, buf.size, None, 0, ctypes.byref(w), ctypes.byref(h))
    out = np.empty((h.value, w.value), np.uint8)
    _lib.call("viso_png_decode_grey", buf.ctypes.data, buf.size, out.ctypes.data, out.size, None, None)
    return out


def kitti_calib(path: str):
    """calib.txt -> (fx, fy, cx, cy, baseline)."""
    v = [ctypes.c_double(0.0) for _ in range(5)]
    _lib.call("viso_kitti_calib", os.fsencode(path), *[ctypes.byref(x) for x in v])
    return tuple(x.value for x in v)


class KittiSequence:
    """A KITTI odometry sequence directory (e.g. .../sequences/00)."""

    def __init__(self, root: str):
        self.root = root
        self.fx, self.fy, self.cx, self.cy, self.baseline = kitti_calib(os.path.join(root, "calib.txt"))
        names = sorted(f for f in os.listdir(os.path.join(root, "image_0")) if f.endswith(".png"))
        self.n = len(names)
        self.width, self.height = png_info(os.path.join(root, "image_0", names[0])) if names else (0, 0)

    @property
    def K(self):
        return (self.fx, self.fy, self.cx, self.cy)

    def __len__(self):
        return self.n

    def image(self, frame: int, cam: int = 0) -> np.ndarray:
        return read_png(os.path.join(self.root, f"image_{cam}", f"{frame:06d}.png"))

    def frame(self, i: int):
        return self.image(i, 0), self.image(i, 1)
