"""Frame source: PNG -> grey (the reference's cv::imread(file, 0),
include/frame_sequence.h:28-30, restated in viso_amd/csrc/imgio.cpp) and KITTI
odometry sequences (image_0|1/%06d.png + calib.txt).  Host-only code: these
run without a GPU.  Grey PNGs are checked bit-exact against PIL's decoder;
the colour -> grey rule is libpng's png_set_rgb_to_gray(0.299, 0.587)
restated (parity with OpenCV itself unpinned: neither is in the image)."""
import io
import os

import numpy as np
import pytest

PIL = pytest.importorskip("PIL.Image")

from viso_amd import kitti  # noqa: E402


def _png(arr, mode=None, **kw):
    b = io.BytesIO()
    (PIL.fromarray(arr, mode) if mode else PIL.fromarray(arr)).save(b, format="PNG", **kw)
    return b.getvalue()


@pytest.mark.parametrize("h,w", [(1, 1), (7, 13), (375, 1242), (64, 3)])
@pytest.mark.parametrize("optimize", [False, True])
def test_grey8_exact(h, w, optimize):
    rng = np.random.default_rng(h * 1000 + w)
    # noise + smooth ramps: PIL's adaptive filtering picks all five filter types
    img = (rng.integers(0, 256, (h, w)) // 2 + np.add.outer(np.arange(h), np.arange(w)) % 128).astype(np.uint8)
    got = kitti.decode_png(_png(img, "L", optimize=optimize))
    assert got.dtype == np.uint8 and np.array_equal(got, img)


def _png_adam7_grey8(img, filt=(0, 1, 2, 3, 4)):
    """A minimal interlaced (Adam7) 8-bit grey PNG writer (PIL cannot write
    one): every scanline filtered with the next filter type of `filt`."""
    import struct
    import zlib

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)

    def paeth(a, b, c):
        p = a + b - c
        pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
        return a if pa <= pb and pa <= pc else (b if pb <= pc else c)

    h, w = img.shape
    raw, k = bytearray(), 0
    for x0, y0, dx, dy in ((0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2),
                           (0, 1, 1, 2)):
        sub = img[y0::dy, x0::dx]
        if sub.size == 0:
            continue
        prev = np.zeros(sub.shape[1], np.int64)
        for row in sub.astype(np.int64):
            t = filt[k % len(filt)]
            k += 1
            left = np.concatenate([[0], row[:-1]])
            upleft = np.concatenate([[0], prev[:-1]])
            pred = {0: 0 * row, 1: left, 2: prev, 3: (left + prev) // 2,
                    4: np.array([paeth(a, b, c) for a, b, c in zip(left, prev, upleft)])}[t]
            raw += bytes([t]) + bytes(((row - pred) % 256).astype(np.uint8))
            prev = row
    ihdr = struct.pack(">IIBBBBB", w, h, 8, 0, 0, 0, 1)
    return b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", ihdr) + chunk(b"IDAT", zlib.compress(bytes(raw))) + chunk(b"IEND", b"")


@pytest.mark.parametrize("h,w", [(37, 53), (1, 1), (3, 9), (8, 8)])
def test_interlaced_grey_exact(h, w):
    rng = np.random.default_rng(h * w)
    img = rng.integers(0, 256, (h, w), dtype=np.uint8)
    data = _png_adam7_grey8(img)
    assert np.array_equal(np.asarray(PIL.open(io.BytesIO(data))), img)  # the writer is valid
    assert np.array_equal(kitti.decode_png(data), img)


def test_grey16_high_byte_and_low_depths():
    rng = np.random.default_rng(1)
    img16 = rng.integers(0, 65536, (20, 30), dtype=np.uint16)
    got = kitti.decode_png(_png(img16))  # mode I;16
    assert np.array_equal(got, (img16 >> 8).astype(np.uint8))
    bw = rng.integers(0, 2, (9, 17), dtype=np.uint8) * 255
    assert np.array_equal(kitti.decode_png(_png(bw.astype(bool))), bw)  # mode 1: 1-bit grey


def _rgb_to_grey(rgb):
    r, g, b = (rgb[..., k].astype(np.int64) for k in range(3))
    y = (9797 * r + 19234 * g + 3737 * b) >> 15
    return np.where((r == g) & (g == b), r, y).astype(np.uint8)


def test_rgb_rgba_palette_to_grey():
    rng = np.random.default_rng(2)
    rgb = rng.integers(0, 256, (23, 31, 3), dtype=np.uint8)
    rgb[0, :] = rgb[0, :, :1]  # grey pixels pass through unchanged
    exp = _rgb_to_grey(rgb)
    assert np.array_equal(kitti.decode_png(_png(rgb, "RGB")), exp)
    rgba = np.concatenate([rgb, rng.integers(0, 256, (23, 31, 1), dtype=np.uint8)], axis=2)
    assert np.array_equal(kitti.decode_png(_png(rgba, "RGBA")), exp)
    pal = PIL.fromarray(rgb, "RGB").quantize(16)
    b = io.BytesIO()
    pal.save(b, format="PNG")
    assert np.array_equal(kitti.decode_png(b.getvalue()), _rgb_to_grey(np.asarray(pal.convert("RGB"))))


def test_rejects_corrupt():
    from viso_amd._lib import VisoError
    data = bytearray(_png(np.zeros((4, 4), np.uint8), "L"))
    data[40] ^= 0xFF  # inside IDAT: CRC mismatch
    with pytest.raises(VisoError):
        kitti.decode_png(bytes(data))
    with pytest.raises(VisoError):
        kitti.decode_png(b"not a png at all")


def _png_raw(ctype, depth, rows, w, h, extra=()):
    """A minimal non-interlaced PNG (filter 0 on every line) with ancillary
    chunks `extra` = [(type, data, crc_ok)] placed before IDAT."""
    import struct
    import zlib

    def chunk(t, d, ok=True):
        crc = zlib.crc32(t + d) & 0xFFFFFFFF
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", crc if ok else crc ^ 0x5A5A5A5A)

    ihdr = struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, 0)
    raw = b"".join(b"\x00" + r for r in rows)
    body = b"".join(chunk(t, d, ok) for t, d, ok in extra)
    return (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", ihdr) + body + chunk(b"IDAT", zlib.compress(raw)) +
            chunk(b"IEND", b""))


def test_rgb16_ancillary_chunks_and_bad_ancillary_crc():
    """16-bit RGB(A) -> the high byte of each sample (png_set_strip_16), then
    the grey rule; gAMA / tRNS change nothing (imread sets no gamma
    transform, transparency is stripped); an ancillary chunk with a bad CRC
    is skipped (libpng's default), a critical one fails."""
    import struct
    from viso_amd._lib import VisoError
    rng = np.random.default_rng(5)
    h, w = 6, 11
    rgb16 = rng.integers(0, 65536, (h, w, 3), dtype=np.uint16)
    exp = _rgb_to_grey((rgb16 >> 8).astype(np.uint8))
    rows = [rgb16[y].astype(">u2").tobytes() for y in range(h)]
    extra = [(b"gAMA", struct.pack(">I", 45455), True), (b"tRNS", struct.pack(">HHH", 1, 2, 3), True),
             (b"tEXt", b"Comment\x00corrupt", False)]
    assert np.array_equal(kitti.decode_png(_png_raw(2, 16, rows, w, h, extra)), exp)
    rgba16 = np.concatenate([rgb16, rng.integers(0, 65536, (h, w, 1), dtype=np.uint16)], axis=2)
    rows = [rgba16[y].astype(">u2").tobytes() for y in range(h)]
    assert np.array_equal(kitti.decode_png(_png_raw(6, 16, rows, w, h)), exp)
    grey = rng.integers(0, 256, (h, w), dtype=np.uint8)
    ok = _png_raw(0, 8, [grey[y].tobytes() for y in range(h)], w, h, [(b"tRNS", b"\x00\x07", True)])
    assert np.array_equal(kitti.decode_png(ok), grey)
    bad = _png_raw(0, 8, [grey[y].tobytes() for y in range(h)], w, h, [(b"PLTE", b"\x00\x00\x00", False)])
    with pytest.raises(VisoError):
        kitti.decode_png(bad)


def _write_kitti(root, seq, n):
    os.makedirs(os.path.join(root, "image_0"))
    os.makedirs(os.path.join(root, "image_1"))
    for f in range(n):
        l, r = seq.frame(f)
        PIL.fromarray(l, "L").save(os.path.join(root, "image_0", f"{f:06d}.png"))
        PIL.fromarray(r, "L").save(os.path.join(root, "image_1", f"{f:06d}.png"))
    fx, fy, cx, cy = seq.K
    P0 = [fx, 0, cx, 0, 0, fy, cy, 0, 0, 0, 1, 0]
    P1 = [fx, 0, cx, -fx * seq.p.baseline, 0, fy, cy, 0, 0, 0, 1, 0]
    with open(os.path.join(root, "calib.txt"), "w") as fh:
        for k, P in enumerate((P0, P1, P0, P0)):
            fh.write(f"P{k}: " + " ".join(f"{v:.12e}" for v in P) + "\n")
        fh.write("Tr: " + " ".join(["0"] * 12) + "\n")


def test_kitti_sequence_round_trip(tmp_path):
    from viso_amd.synth import Sequence
    seq = Sequence(1242, 375, seed=4)
    root = str(tmp_path / "sequences" / "00")
    _write_kitti(root, seq, 3)
    ks = kitti.KittiSequence(root)
    assert len(ks) == 3 and (ks.width, ks.height) == (1242, 375)
    assert np.allclose(ks.K, seq.K, rtol=1e-12) and abs(ks.baseline - seq.p.baseline) < 1e-12
    for f in range(3):
        l, r = ks.frame(f)
        el, er = seq.frame(f)
        assert np.array_equal(l, el) and np.array_equal(r, er)


def test_frame_sequence_reads_png(tmp_path):
    """FrameSequence::RunOnce (include/frame_sequence.h:25-38): <location><id+1>.png."""
    from viso_amd import frontend

    class Sink(frontend.FrameHandler):
        def __init__(self):
            self.frames = []

        def OnNewFrame(self, kf):
            self.frames.append(kf.mat_)

    img = np.arange(48, dtype=np.uint8).reshape(6, 8)
    nid = frontend.Keyframe.GetNextId()
    PIL.fromarray(img, "L").save(str(tmp_path / f"{nid + 1}.png"))
    sink = Sink()
    fs = frontend.FrameSequence(str(tmp_path), sink)
    assert fs.RunOnce() and np.array_equal(sink.frames[0], img)
    assert not fs.RunOnce()  # the next file does not exist
