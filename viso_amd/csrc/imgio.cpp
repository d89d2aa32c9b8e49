// viso_amd — frame source (host only): PNG -> grey, the restatement of the
// reference's cv::imread("<location><n>.png", 0) (include/frame_sequence.h:
// 28-30), and KITTI calib.txt.  Conversion rules: include/viso/viso_io.h.
// zlib inflates the IDAT stream; scanline filters (None, Sub, Up, Average,
// Paeth) and Adam7 interlacing are undone here.
#include <zlib.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/viso/viso_io.h"

namespace {

uint32_t be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

struct Png {
    uint32_t w = 0, h = 0;
    int depth = 0, ctype = 0, interlace = 0, ch = 0;
    std::vector<uint8_t> idat, plte;
};

// chunk walk: IHDR, PLTE, IDAT (concatenated), IEND.  A CRC error in a
// critical chunk (upper-case first letter) is fatal; an ancillary chunk with
// a bad CRC is skipped, as libpng's default does (png_crc_finish: a benign
// error for ancillary chunks).  Ancillary chunks are not interpreted: gAMA /
// sRGB / iCCP (cv::imread sets no gamma transform) and tRNS (expanded to
// alpha by OpenCV, then stripped for IMREAD_GRAYSCALE) do not change the
// grey bytes.
int parse(const uint8_t* d, size_t n, Png& png) {
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (!d || n < 8 || std::memcmp(d, sig, 8) != 0) return VISO_ERR_ARG;
    size_t o = 8;
    bool ihdr = false, iend = false;
    while (o + 12 <= n && !iend) {
        const uint32_t len = be32(d + o);
        if (len > n - o - 12) return VISO_ERR_ARG;
        const uint8_t* type = d + o + 4;
        const uint8_t* data = d + o + 8;
        const bool critical = (type[0] & 0x20) == 0;
        if (crc32(crc32(0L, Z_NULL, 0), type, len + 4) != be32(data + len)) {
            if (critical) return VISO_ERR_ARG;
            o += (size_t)len + 12;
            continue;
        }
        if (!std::memcmp(type, "IHDR", 4)) {
            if (len != 13) return VISO_ERR_ARG;
            png.w = be32(data);
            png.h = be32(data + 4);
            png.depth = data[8];
            png.ctype = data[9];
            png.interlace = data[12];
            if (data[10] != 0 || data[11] != 0 || png.interlace > 1) return VISO_ERR_ARG;
            ihdr = true;
        } else if (!std::memcmp(type, "PLTE", 4)) {
            png.plte.assign(data, data + len);
        } else if (!std::memcmp(type, "IDAT", 4)) {
            png.idat.insert(png.idat.end(), data, data + len);
        } else if (!std::memcmp(type, "IEND", 4)) {
            iend = true;
        }
        o += (size_t)len + 12;
    }
    if (!ihdr || png.w == 0 || png.h == 0 || png.w > 65535 || png.h > 65535) return VISO_ERR_ARG;
    const int d8 = png.depth;
    switch (png.ctype) {
        case 0: png.ch = 1; if (d8 != 1 && d8 != 2 && d8 != 4 && d8 != 8 && d8 != 16) return VISO_ERR_ARG; break;
        case 2: png.ch = 3; if (d8 != 8 && d8 != 16) return VISO_ERR_ARG; break;
        case 3: png.ch = 1; if (d8 != 1 && d8 != 2 && d8 != 4 && d8 != 8) return VISO_ERR_ARG; break;
        case 4: png.ch = 2; if (d8 != 8 && d8 != 16) return VISO_ERR_ARG; break;
        case 6: png.ch = 4; if (d8 != 8 && d8 != 16) return VISO_ERR_ARG; break;
        default: return VISO_ERR_ARG;
    }
    if (png.ctype == 3 && (png.plte.empty() || png.plte.size() % 3)) return VISO_ERR_ARG;
    return VISO_OK;
}

int paeth(int a, int b, int c) {
    const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    return (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
}

// undo the filter of one scanline in place (prev = previous raw line or null)
bool unfilter(uint8_t* row, const uint8_t* prev, size_t len, int bpp, int type) {
    switch (type) {
        case 0: return true;
        case 1:
            for (size_t i = (size_t)bpp; i < len; ++i) row[i] = (uint8_t)(row[i] + row[i - bpp]);
            return true;
        case 2:
            if (prev)
                for (size_t i = 0; i < len; ++i) row[i] = (uint8_t)(row[i] + prev[i]);
            return true;
        case 3:
            for (size_t i = 0; i < len; ++i) {
                const int a = i >= (size_t)bpp ? row[i - bpp] : 0, b = prev ? prev[i] : 0;
                row[i] = (uint8_t)(row[i] + ((a + b) >> 1));
            }
            return true;
        case 4:
            for (size_t i = 0; i < len; ++i) {
                const int a = i >= (size_t)bpp ? row[i - bpp] : 0, b = prev ? prev[i] : 0;
                const int c = (prev && i >= (size_t)bpp) ? prev[i - bpp] : 0;
                row[i] = (uint8_t)(row[i] + paeth(a, b, c));
            }
            return true;
        default: return false;
    }
}

// libpng 1.6 png_set_rgb_to_gray(png, 1, 0.299, 0.587) without gamma tables
inline uint8_t rgb_to_gray(int r, int g, int b) {
    if (r == g && g == b) return (uint8_t)r;
    return (uint8_t)((9797 * r + 19234 * g + 3737 * b) >> 15);
}

// grey value of pixel i of an unfiltered scanline
inline uint8_t grey_of(const Png& png, const uint8_t* raw, size_t i) {
    const int d = png.depth;
    if (png.ctype == 0 || png.ctype == 3) {
        int v;
        if (d == 16) v = raw[2 * i];  // png_set_strip_16: the high byte
        else if (d == 8) v = raw[i];
        else v = (raw[(i * d) >> 3] >> (8 - d - (int)((i * d) & 7))) & ((1 << d) - 1);
        if (png.ctype == 0) return (uint8_t)(d < 8 ? v * (255 / ((1 << d) - 1)) : v);
        const size_t k = 3 * (size_t)v;
        if (k + 2 >= png.plte.size()) return 0;
        return rgb_to_gray(png.plte[k], png.plte[k + 1], png.plte[k + 2]);
    }
    if (png.ctype == 4) return d == 16 ? raw[4 * i] : raw[2 * i];  // alpha stripped
    if (d == 16) {  // png_set_strip_16: the high byte of every sample
        const uint8_t* p = raw + 2 * (size_t)png.ch * i;
        return rgb_to_gray(p[0], p[2], p[4]);
    }
    const uint8_t* p = raw + (size_t)png.ch * i;  // RGB / RGBA
    return rgb_to_gray(p[0], p[1], p[2]);
}

int decode(const uint8_t* data, size_t size, uint8_t* out, size_t cap, int32_t* width, int32_t* height) {
    Png png;
    const int rc = parse(data, size, png);
    if (rc) return rc;
    if (width) *width = (int32_t)png.w;
    if (height) *height = (int32_t)png.h;
    if (!out) return VISO_OK;
    if (cap < (size_t)png.w * png.h) return VISO_ERR_CAPACITY;
    const int bits = png.depth * png.ch;
    const int bpp = bits >= 8 ? bits / 8 : 1;
    // Adam7 passes (x0, y0, dx, dy); one full pass when not interlaced
    static const int adam7[7][4] = {{0, 0, 8, 8}, {4, 0, 8, 8}, {0, 4, 4, 8}, {2, 0, 4, 4},
                                    {0, 2, 2, 4}, {1, 0, 2, 2}, {0, 1, 1, 2}};
    static const int full[1][4] = {{0, 0, 1, 1}};
    const int (*passes)[4] = png.interlace ? adam7 : full;
    const int np = png.interlace ? 7 : 1;
    size_t total = 0;
    for (int k = 0; k < np; ++k) {
        const size_t pw = (png.w - passes[k][0] + passes[k][2] - 1) / passes[k][2];
        const size_t ph = (png.h - passes[k][1] + passes[k][3] - 1) / passes[k][3];
        if (png.w <= (uint32_t)passes[k][0] || png.h <= (uint32_t)passes[k][1]) continue;
        total += ph * (1 + (pw * bits + 7) / 8);
    }
    std::vector<uint8_t> raw(total);
    z_stream zs;
    std::memset(&zs, 0, sizeof(zs));
    if (inflateInit(&zs) != Z_OK) return VISO_ERR_ARG;
    zs.next_in = const_cast<Bytef*>(png.idat.data());
    zs.avail_in = (uInt)png.idat.size();
    zs.next_out = raw.data();
    zs.avail_out = (uInt)raw.size();
    const int zr = inflate(&zs, Z_FINISH);
    const bool ok = (zr == Z_STREAM_END || zr == Z_OK || zr == Z_BUF_ERROR) && zs.avail_out == 0;
    inflateEnd(&zs);
    if (!ok) return VISO_ERR_ARG;
    size_t o = 0;
    for (int k = 0; k < np; ++k) {
        const int x0 = passes[k][0], y0 = passes[k][1], dx = passes[k][2], dy = passes[k][3];
        if (png.w <= (uint32_t)x0 || png.h <= (uint32_t)y0) continue;
        const size_t pw = (png.w - x0 + dx - 1) / dx, ph = (png.h - y0 + dy - 1) / dy;
        const size_t len = (pw * bits + 7) / 8;
        const uint8_t* prev = nullptr;
        for (size_t r = 0; r < ph; ++r) {
            uint8_t* line = raw.data() + o;
            if (!unfilter(line + 1, prev, len, bpp, line[0])) return VISO_ERR_ARG;
            uint8_t* dst = out + (size_t)(y0 + r * dy) * png.w;
            for (size_t i = 0; i < pw; ++i) dst[x0 + i * dx] = grey_of(png, line + 1, i);
            prev = line + 1;
            o += 1 + len;
        }
    }
    return VISO_OK;
}

bool read_file(const char* path, std::vector<uint8_t>& buf) {
    FILE* f = std::fopen(path, "rb");
    if (!f) return false;
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    if (n < 0) {
        std::fclose(f);
        return false;
    }
    buf.resize((size_t)n);
    const bool ok = std::fread(buf.data(), 1, buf.size(), f) == buf.size();
    std::fclose(f);
    return ok;
}

}  // namespace

extern "C" {

int viso_png_decode_grey(const uint8_t* data, size_t size, uint8_t* out, size_t cap, int32_t* width,
                         int32_t* height) {
    return decode(data, size, out, cap, width, height);
}

int viso_png_read_grey(const char* path, uint8_t* out, size_t cap, int32_t* width, int32_t* height) {
    std::vector<uint8_t> buf;
    if (!path || !read_file(path, buf)) return VISO_ERR_ARG;
    return decode(buf.data(), buf.size(), out, cap, width, height);
}

int viso_png_info(const char* path, int32_t* width, int32_t* height) {
    return viso_png_read_grey(path, nullptr, 0, width, height);
}

int viso_kitti_calib(const char* path, double* fx, double* fy, double* cx, double* cy, double* baseline) {
    std::vector<uint8_t> buf;
    if (!path || !read_file(path, buf)) return VISO_ERR_ARG;
    std::string text(buf.begin(), buf.end());
    double P[2][12];
    bool have[2] = {false, false};
    size_t pos = 0;
    while (pos < text.size()) {
        size_t e = text.find('\n', pos);
        if (e == std::string::npos) e = text.size();
        const std::string line = text.substr(pos, e - pos);
        pos = e + 1;
        for (int k = 0; k < 2; ++k) {
            const std::string tag = "P" + std::to_string(k) + ":";
            if (line.compare(0, tag.size(), tag) != 0) continue;
            const char* s = line.c_str() + tag.size();
            int m = 0;
            for (; m < 12; ++m) {
                char* end = nullptr;
                P[k][m] = std::strtod(s, &end);
                if (end == s) break;
                s = end;
            }
            have[k] = m == 12;
        }
    }
    if (!have[0] || !have[1] || !(P[0][0] > 0) || !(P[1][0] > 0)) return VISO_ERR_ARG;
    if (fx) *fx = P[0][0];
    if (fy) *fy = P[0][5];
    if (cx) *cx = P[0][2];
    if (cy) *cy = P[0][6];
    if (baseline) *baseline = -P[1][3] / P[1][0];
    return VISO_OK;
}

}  // extern "C"
