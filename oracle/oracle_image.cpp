// TEST INFRASTRUCTURE ONLY — oracle image stage: pyramid (cv::pyrDown),
// FAST-9/16 + NMS (cv::FAST), bilinear sampling.  See viso_oracle.h.
#include <algorithm>
#include <cstring>
#include <vector>

#include "oracle_common.hpp"
#include "viso_oracle.h"

using namespace oracle;

namespace {

// cv::borderInterpolate(p, len, BORDER_REFLECT_101)
inline int reflect101(int p, int len) {
    if (len == 1) return 0;
    while (p < 0 || p >= len) {
        if (p < 0)
            p = -p;
        else
            p = 2 * len - p - 2;
    }
    return p;
}

// FAST circle (OpenCV makeOffsets, patternSize 16): (dx, dy)
const int kCircle[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},  {3, 0},  {3, -1},
                            {2, -2}, {1, -3},  {0, -3},  {-1, -3}, {-2, -2}, {-3, -1},
                            {-3, 0}, {-3, 1},  {-2, 2},  {-1, 3}};

// OpenCV FAST_t<16> corner test for one pixel; returns 0 (no corner) or the
// cornerScore<16> value (>= threshold).  The arc test and the score are the
// OpenCV 3.x algorithm (fast.cpp / fast_score.cpp) without its early-outs,
// which do not change results.
int fast_pixel(const uint8_t* img, int w, int x, int y, int thresh) {
    const uint8_t* p = img + (size_t)y * w + x;
    int v = p[0];
    int circ[25];
    for (int k = 0; k < 16; ++k) circ[k] = p[kCircle[k][0] + kCircle[k][1] * w];
    for (int k = 16; k < 25; ++k) circ[k] = circ[k - 16];
    // threshold_tab semantics: 1 = darker (i < -t), 2 = brighter (i > t)
    auto cls = [&](int pix) { int d = pix - v; return d < -thresh ? 1 : (d > thresh ? 2 : 0); };
    int d = cls(circ[0]) | cls(circ[8]);
    if (d == 0) return 0;
    d &= cls(circ[2]) | cls(circ[10]);
    d &= cls(circ[4]) | cls(circ[12]);
    d &= cls(circ[6]) | cls(circ[14]);
    if (d == 0) return 0;
    d &= cls(circ[1]) | cls(circ[9]);
    d &= cls(circ[3]) | cls(circ[11]);
    d &= cls(circ[5]) | cls(circ[13]);
    d &= cls(circ[7]) | cls(circ[15]);
    bool corner = false;
    if (d & 1) {
        int vt = v - thresh, count = 0;
        for (int k = 0; k < 25; ++k) {
            if (circ[k] < vt) {
                if (++count > 8) { corner = true; break; }
            } else
                count = 0;
        }
    }
    if (!corner && (d & 2)) {
        int vt = v + thresh, count = 0;
        for (int k = 0; k < 25; ++k) {
            if (circ[k] > vt) {
                if (++count > 8) { corner = true; break; }
            } else
                count = 0;
        }
    }
    if (!corner) return 0;
    // cornerScore<16>
    int dd[25];
    for (int k = 0; k < 25; ++k) dd[k] = v - circ[k];
    int a0 = thresh;
    for (int k = 0; k < 16; k += 2) {
        int a = std::min(dd[k + 1], dd[k + 2]);
        for (int j = 3; j <= 8; ++j) a = std::min(a, dd[k + j]);
        a0 = std::max(a0, std::min(a, dd[k]));
        a0 = std::max(a0, std::min(a, dd[k + 9]));
    }
    int b0 = -a0;
    for (int k = 0; k < 16; k += 2) {
        int b = std::max(dd[k + 1], dd[k + 2]);
        for (int j = 3; j <= 8; ++j) b = std::max(b, dd[k + j]);
        b0 = std::min(b0, std::max(b, dd[k]));
        b0 = std::min(b0, std::max(b, dd[k + 9]));
    }
    return -b0 - 1;
}

}  // namespace

extern "C" {

void oracle_pyramid_dims(int w, int h, int32_t dims_out[8]) {
    int ws[kLevels], hs[kLevels];
    size_t offs[kLevels];
    pyramid_dims(w, h, ws, hs, offs);
    for (int l = 0; l < kLevels; ++l) {
        dims_out[2 * l] = ws[l];
        dims_out[2 * l + 1] = hs[l];
    }
}

size_t oracle_pyramid_bytes(int w, int h) {
    int ws[kLevels], hs[kLevels];
    size_t offs[kLevels];
    pyramid_dims(w, h, ws, hs, offs);
    return offs[kLevels - 1] + (size_t)ws[kLevels - 1] * hs[kLevels - 1];
}

// cv::pyrDown (imgproc/pyramids.cpp pyrDown_): 5x5 kernel [1 4 6 4 1]^T[1 4 6 4 1],
// BORDER_REFLECT_101 against the SOURCE size, FixPtCast<uchar,8>: (s + 128) >> 8.
void oracle_pyr_down(const uint8_t* src, int sw, int sh, uint8_t* dst, int dw, int dh) {
    static const int wk[5] = {1, 4, 6, 4, 1};
    std::vector<int> row((size_t)dw);
    for (int y = 0; y < dh; ++y) {
        std::fill(row.begin(), row.end(), 0);
        for (int i = 0; i < 5; ++i) {
            int sy = reflect101(2 * y - 2 + i, sh);
            const uint8_t* s = src + (size_t)sy * sw;
            for (int x = 0; x < dw; ++x) {
                int hsum = 0;
                for (int j = 0; j < 5; ++j) hsum += wk[j] * s[reflect101(2 * x - 2 + j, sw)];
                row[(size_t)x] += wk[i] * hsum;
            }
        }
        for (int x = 0; x < dw; ++x) dst[(size_t)y * dw + x] = (uint8_t)((row[(size_t)x] + 128) >> 8);
    }
}

void oracle_pyramid(const uint8_t* img, int w, int h, uint8_t* out) {
    int ws[kLevels], hs[kLevels];
    size_t offs[kLevels];
    pyramid_dims(w, h, ws, hs, offs);
    std::memcpy(out, img, (size_t)w * h);
    for (int l = 1; l < kLevels; ++l)
        oracle_pyr_down(out + offs[l - 1], ws[l - 1], hs[l - 1], out + offs[l], ws[l], hs[l]);
}

void oracle_fast_score_map(const uint8_t* img, int w, int h, int thresh, uint8_t* score) {
    thresh = std::min(std::max(thresh, 0), 255);
    std::memset(score, 0, (size_t)w * h);
    // candidate rows 3 .. h-4, columns 3 .. w-4 (FAST_t: i < rows-3, j < cols-3)
    for (int y = 3; y < h - 3; ++y)
        for (int x = 3; x < w - 3; ++x) score[(size_t)y * w + x] = (uint8_t)fast_pixel(img, w, x, y, thresh);
}

int oracle_fast(const uint8_t* img, int w, int h, int thresh, int32_t* xs, int32_t* ys,
                int32_t* scores, int cap) {
    std::vector<uint8_t> s((size_t)w * h);
    oracle_fast_score_map(img, w, h, thresh, s.data());
    auto at = [&](int x, int y) -> int {
        if (x < 0 || y < 0 || x >= w || y >= h) return 0;
        return s[(size_t)y * w + x];
    };
    int n = 0;
    for (int y = 3; y < h - 3; ++y) {
        for (int x = 3; x < w - 3; ++x) {
            int sc = at(x, y);
            if (sc == 0) continue;
            // strict > against all 8 neighbours (non-corners score 0)
            bool keep = sc > at(x + 1, y) && sc > at(x - 1, y) && sc > at(x - 1, y - 1) &&
                        sc > at(x, y - 1) && sc > at(x + 1, y - 1) && sc > at(x - 1, y + 1) &&
                        sc > at(x, y + 1) && sc > at(x + 1, y + 1);
            if (!keep) continue;
            if (n < cap) {
                xs[n] = x;
                ys[n] = y;
                scores[n] = sc;
            }
            ++n;
        }
    }
    return n;
}

double oracle_sample(const uint8_t* img, int w, int h, double x, double y) {
    return sample(img, w, h, x, y);
}

void oracle_gradient(const uint8_t* img, int w, int h, double x, double y, double out[2]) {
    gradient(img, w, h, x, y, out[0], out[1]);
}

}  // extern "C"
