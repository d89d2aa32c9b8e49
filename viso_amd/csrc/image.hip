// viso_amd — image-pass kernels for gfx950: pyramid (cv::pyrDown restated)
// and FAST-9/16 + NMS (cv::FAST restated).  Integer arithmetic, bit-exact
// against the oracle (oracle/oracle_image.cpp).
//
// Pyramid: one launch per level, batched over every image of a chunk
// (grid.z = image).  A 256-thread workgroup produces a 64x16 output tile: it
// stages the (2*16+3) x (2*64+3) source window in LDS with BORDER_REFLECT_101
// resolved at load time, runs the horizontal 5-tap pass into an int LDS
// buffer, then the vertical pass.  HBM-bound: algorithmic bytes per image =
// level-0 read + levels 1..3 written.
//
// FAST: one workgroup per image row y.  It scores rows y-1, y, y+1 from a
// 9-row LDS window, applies the strict 3x3 NMS to row y and appends the
// surviving corners in ascending x with a ballot/popcount prefix (row-major
// order is then restored across rows by fast_compact, an exclusive prefix
// over per-row counts).
#include <vector>

#include "kernels.hpp"

namespace viso {

namespace {

constexpr int kPyrTileW = 64;
constexpr int kPyrTileH = 16;
constexpr int kPyrInW = 2 * kPyrTileW + 3;  // 131
constexpr int kPyrInH = 2 * kPyrTileH + 3;  // 35

__device__ inline int reflect101(int p, int len) {
    if (len == 1) return 0;
    while (p < 0 || p >= len) p = (p < 0) ? -p : 2 * len - p - 2;
    return p;
}

struct PyrPtrs {
    const uint8_t* src[kPyrBatch];
    uint8_t* dst[kPyrBatch];
};

__global__ __launch_bounds__(256) void pyr_down_kernel(PyrPtrs ptrs, int sw, int sh, int dw,
                                                       int dh) {
    __shared__ uint8_t s_in[kPyrInH][kPyrInW + 1];
    __shared__ int s_h[kPyrInH][kPyrTileW + 1];
    const uint8_t* __restrict__ src = ptrs.src[blockIdx.z];
    uint8_t* __restrict__ dst = ptrs.dst[blockIdx.z];
    const int ox0 = blockIdx.x * kPyrTileW;
    const int oy0 = blockIdx.y * kPyrTileH;
    const int tid = threadIdx.x;
    const int gx0 = 2 * ox0 - 2, gy0 = 2 * oy0 - 2;
    // stage the source window (coalesced byte loads along x)
    for (int idx = tid; idx < kPyrInH * kPyrInW; idx += 256) {
        int r = idx / kPyrInW, c = idx - r * kPyrInW;
        int gy = reflect101(gy0 + r, sh);
        int gx = reflect101(gx0 + c, sw);
        s_in[r][c] = src[(size_t)gy * sw + gx];
    }
    __syncthreads();
    // horizontal 5-tap at even centres
    for (int idx = tid; idx < kPyrInH * kPyrTileW; idx += 256) {
        int r = idx / kPyrTileW, c = idx - r * kPyrTileW;
        const uint8_t* p = &s_in[r][2 * c];
        s_h[r][c] = (int)p[0] + 4 * (int)p[1] + 6 * (int)p[2] + 4 * (int)p[3] + (int)p[4];
    }
    __syncthreads();
    // vertical 5-tap + FixPtCast<uchar,8>
    const int c = tid & 63;
    for (int r = tid >> 6; r < kPyrTileH; r += 4) {
        int ox = ox0 + c, oy = oy0 + r;
        if (ox < dw && oy < dh) {
            int s = s_h[2 * r][c] + 4 * s_h[2 * r + 1][c] + 6 * s_h[2 * r + 2][c] +
                    4 * s_h[2 * r + 3][c] + s_h[2 * r + 4][c];
            dst[(size_t)oy * dw + ox] = (uint8_t)((s + 128) >> 8);
        }
    }
}

// ---------------------------------------------------------------- fused pyramid
// One workgroup owns a level-3 tile of 16x8 and the matching level-2 (32x16)
// and level-1 (64x32) tiles.  It stages the level-0 window that feeds them
// (149 x 85, recursive 5-tap halos) in LDS with 16-byte loads, then runs
// horizontal/vertical passes level by level entirely in LDS.  Every level's
// border uses reflect-101 against that level's own (truncated) size, so
// halo samples are read at reflected coordinates, which always fall inside
// the window.  Integer math: identical to three separate pyrDown passes.
constexpr int kF3W = 16, kF3H = 8;
constexpr int kF2W = 2 * kF3W + 3, kF2H = 2 * kF3H + 3;  // 35 x 19
constexpr int kF1W = 2 * kF2W + 3, kF1H = 2 * kF2H + 3;  // 73 x 41
constexpr int kF0W = 2 * kF1W + 3, kF0H = 2 * kF1H + 3;  // 149 x 85
constexpr int kF0P = 160;                                // LDS pitch of the level-0 window

struct PyrFusedArgs {
    const uint8_t* l0[kPyrBatch];
    uint8_t* slot[kPyrBatch];
    int w[4], h[4];
    unsigned long long off[4];
};

__global__ __launch_bounds__(256) void pyr_fused_kernel(PyrFusedArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t s0[kF0H][kF0P];
    __shared__ short hs0[kF0H][kF1W];
    __shared__ uint8_t s1[kF1H][kF1W + 3];
    __shared__ short hs1[kF1H][kF2W];
    __shared__ uint8_t s2[kF2H][kF2W + 1];
    const uint8_t* __restrict__ src = a.l0[blockIdx.z];
    uint8_t* __restrict__ base = a.slot[blockIdx.z];
    const int tid = threadIdx.x;
    const int X3 = blockIdx.x * kF3W, Y3 = blockIdx.y * kF3H;
    const int ox2 = 2 * X3 - 2, oy2 = 2 * Y3 - 2;
    const int ox1 = 2 * ox2 - 2, oy1 = 2 * oy2 - 2;
    const int ox0 = 2 * ox1 - 2, oy0 = 2 * oy1 - 2;
    const int w0 = a.w[0], h0 = a.h[0], w1 = a.w[1], h1 = a.h[1];
    const int w2 = a.w[2], h2 = a.h[2], w3 = a.w[3], h3 = a.h[3];
    // ---- stage the level-0 window (in-range part), 16-byte aligned chunks
    {
        const int c_lo = max(ox0, 0), c_hi = min(ox0 + kF0W, w0);
        const uintptr_t img_lo = (uintptr_t)src, img_hi = img_lo + (uintptr_t)w0 * h0;
        const int nchunk = (c_hi > c_lo) ? ((c_hi - c_lo) + 15 + 15) / 16 : 0;
        for (int it = tid; it < kF0H * nchunk; it += 256) {
            const int r = it / nchunk, k = it - r * nchunk;
            const int y = oy0 + r;
            if (y < 0 || y >= h0) continue;
            const uintptr_t row = img_lo + (uintptr_t)y * w0;
            const uintptr_t a0 = ((row + c_lo) & ~(uintptr_t)15) + 16 * (uintptr_t)k;
            const uintptr_t lo = row + c_lo, hi = row + c_hi;
            if (a0 >= hi) continue;
            if (a0 >= img_lo && a0 + 16 <= img_hi) {
                const uint4 v = *reinterpret_cast<const uint4*>(a0);
                const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int b = 0; b < 16; ++b) {
                    const uintptr_t ad = a0 + b;
                    if (ad >= lo && ad < hi) s0[r][(int)(ad - row) - ox0] = (uint8_t)(wv[b >> 2] >> (8 * (b & 3)));
                }
            } else {
                for (int b = 0; b < 16; ++b) {
                    const uintptr_t ad = a0 + b;
                    if (ad >= lo && ad < hi) s0[r][(int)(ad - row) - ox0] = *reinterpret_cast<const uint8_t*>(ad);
                }
            }
        }
    }
    __syncthreads();
    // ---- level 1: horizontal pass on every staged row
    for (int it = tid; it < kF0H * kF1W; it += 256) {
        const int r = it / kF1W, c = it - r * kF1W;
        const int y = oy0 + r, x1 = ox1 + c;
        if (y < 0 || y >= h0 || x1 < 0 || x1 >= w1) continue;
        int s = 0;
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const int wgt = j == 2 ? 6 : ((j & 1) ? 4 : 1);
            s += wgt * (int)s0[r][reflect101(2 * x1 - 2 + j, w0) - ox0];
        }
        hs0[r][c] = (short)s;
    }
    __syncthreads();
    uint8_t* d1 = base + a.off[1];
    for (int it = tid; it < kF1H * kF1W; it += 256) {
        const int r = it / kF1W, c = it - r * kF1W;
        const int y1 = oy1 + r, x1 = ox1 + c;
        if (y1 < 0 || y1 >= h1 || x1 < 0 || x1 >= w1) continue;
        int s = 0;
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const int wgt = i == 2 ? 6 : ((i & 1) ? 4 : 1);
            s += wgt * (int)hs0[reflect101(2 * y1 - 2 + i, h0) - oy0][c];
        }
        const uint8_t v = (uint8_t)((s + 128) >> 8);
        s1[r][c] = v;
        if (x1 >= 4 * X3 && x1 < 4 * X3 + 4 * kF3W && y1 >= 4 * Y3 && y1 < 4 * Y3 + 4 * kF3H)
            d1[(size_t)y1 * w1 + x1] = v;
    }
    __syncthreads();
    // ---- level 2
    for (int it = tid; it < kF1H * kF2W; it += 256) {
        const int r = it / kF2W, c = it - r * kF2W;
        const int y1 = oy1 + r, x2 = ox2 + c;
        if (y1 < 0 || y1 >= h1 || x2 < 0 || x2 >= w2) continue;
        int s = 0;
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const int wgt = j == 2 ? 6 : ((j & 1) ? 4 : 1);
            s += wgt * (int)s1[r][reflect101(2 * x2 - 2 + j, w1) - ox1];
        }
        hs1[r][c] = (short)s;
    }
    __syncthreads();
    uint8_t* d2 = base + a.off[2];
    for (int it = tid; it < kF2H * kF2W; it += 256) {
        const int r = it / kF2W, c = it - r * kF2W;
        const int y2 = oy2 + r, x2 = ox2 + c;
        if (y2 < 0 || y2 >= h2 || x2 < 0 || x2 >= w2) continue;
        int s = 0;
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const int wgt = i == 2 ? 6 : ((i & 1) ? 4 : 1);
            s += wgt * (int)hs1[reflect101(2 * y2 - 2 + i, h1) - oy1][c];
        }
        const uint8_t v = (uint8_t)((s + 128) >> 8);
        s2[r][c] = v;
        if (x2 >= 2 * X3 && x2 < 2 * X3 + 2 * kF3W && y2 >= 2 * Y3 && y2 < 2 * Y3 + 2 * kF3H)
            d2[(size_t)y2 * w2 + x2] = v;
    }
    __syncthreads();
    // ---- level 3 (128 outputs, 25 taps each; integer sums are exact)
    uint8_t* d3 = base + a.off[3];
    if (tid < kF3W * kF3H) {
        const int x3 = X3 + (tid & (kF3W - 1)), y3 = Y3 + tid / kF3W;
        if (x3 < w3 && y3 < h3) {
            int s = 0;
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                const int wi = i == 2 ? 6 : ((i & 1) ? 4 : 1);
                const int rr = reflect101(2 * y3 - 2 + i, h2) - oy2;
                int hsum = 0;
#pragma unroll
                for (int j = 0; j < 5; ++j) {
                    const int wj = j == 2 ? 6 : ((j & 1) ? 4 : 1);
                    hsum += wj * (int)s2[rr][reflect101(2 * x3 - 2 + j, w2) - ox2];
                }
                s += wi * hsum;
            }
            d3[(size_t)y3 * w3 + x3] = (uint8_t)((s + 128) >> 8);
        }
    }
}

// ---------------------------------------------------------------- FAST
__constant__ int c_circle_dx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
__constant__ int c_circle_dy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};

// OpenCV FAST_t<16> arc test + cornerScore<16>; returns 0 or the score.
__device__ inline int fast_score(const uint8_t* rows, int rstride, int x, int thresh) {
    // rows points at the centre row of a >= 7 row window
    const int v = rows[x];
    int circ[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) circ[k] = rows[c_circle_dy[k] * rstride + x + c_circle_dx[k]];
    auto cls = [&](int p) { int d = p - v; return d < -thresh ? 1 : (d > thresh ? 2 : 0); };
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
    if (d == 0) return 0;
    bool corner = false;
    if (d & 1) {
        int vt = v - thresh, count = 0;
        for (int k = 0; k < 25; ++k) {
            if (circ[k & 15] < vt) {
                if (++count > 8) { corner = true; break; }
            } else
                count = 0;
        }
    }
    if (!corner && (d & 2)) {
        int vt = v + thresh, count = 0;
        for (int k = 0; k < 25; ++k) {
            if (circ[k & 15] > vt) {
                if (++count > 8) { corner = true; break; }
            } else
                count = 0;
        }
    }
    if (!corner) return 0;
    int dd[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) dd[k] = v - circ[k];
    int a0 = thresh;
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
        int a = min(dd[(k + 1) & 15], dd[(k + 2) & 15]);
#pragma unroll
        for (int j = 3; j <= 8; ++j) a = min(a, dd[(k + j) & 15]);
        a0 = max(a0, min(a, dd[k]));
        a0 = max(a0, min(a, dd[(k + 9) & 15]));
    }
    int b0 = -a0;
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
        int b = max(dd[(k + 1) & 15], dd[(k + 2) & 15]);
#pragma unroll
        for (int j = 3; j <= 8; ++j) b = max(b, dd[(k + j) & 15]);
        b0 = min(b0, max(b, dd[k]));
        b0 = min(b0, max(b, dd[(k + 9) & 15]));
    }
    return -b0 - 1;
}

__global__ __launch_bounds__(256) void fast_rows_kernel(const uint8_t* __restrict__ img, int w,
                                                        int h, int thresh,
                                                        int* __restrict__ row_count,
                                                        int4* __restrict__ row_list,
                                                        int row_cap) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t* s_img = smem;                   // 9 rows (y-4 .. y+4)
    uint8_t* s_sc = smem + 9 * (size_t)w;    // 3 score rows (y-1 .. y+1)
    __shared__ int s_wave[4];
    __shared__ int s_base;
    const int y = blockIdx.x;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    // stage the 9 input rows (rows outside the image are never read)
    for (int r = 0; r < 9; ++r) {
        int gy = y - 4 + r;
        if (gy < 0 || gy >= h) continue;
        const uint8_t* src = img + (size_t)gy * w;
        for (int x = tid; x < w; x += 256) s_img[r * w + x] = src[x];
    }
    __syncthreads();
    // scores of rows y-1, y, y+1 (candidates: rows 3..h-4, cols 3..w-4)
    for (int r = 0; r < 3; ++r) {
        int gy = y - 1 + r;
        bool row_ok = gy >= 3 && gy < h - 3;
        const uint8_t* centre = s_img + (size_t)(r + 3) * w;  // window row of gy
        for (int x = tid; x < w; x += 256) {
            int s = 0;
            if (row_ok && x >= 3 && x < w - 3) s = fast_score(centre, w, x, thresh);
            s_sc[r * w + x] = (uint8_t)s;
        }
    }
    if (tid == 0) s_base = 0;
    __syncthreads();
    // strict 3x3 NMS on row y, ordered append
    for (int x0 = 0; x0 < w; x0 += 256) {
        int x = x0 + tid;
        int sc = 0;
        bool keep = false;
        if (x < w) {
            sc = s_sc[w + x];
            if (sc > 0) {
                auto at = [&](int rr, int xx) -> int {
                    return (xx < 0 || xx >= w) ? 0 : (int)s_sc[rr * w + xx];
                };
                keep = sc > at(1, x + 1) && sc > at(1, x - 1) && sc > at(0, x - 1) &&
                       sc > at(0, x) && sc > at(0, x + 1) && sc > at(2, x - 1) &&
                       sc > at(2, x) && sc > at(2, x + 1);
            }
        }
        unsigned long long m = __ballot(keep);
        int before = __popcll(m & ((1ULL << lane) - 1ULL));
        if (lane == 0) s_wave[wave] = __popcll(m);
        __syncthreads();
        int off = s_base;
        for (int k = 0; k < wave; ++k) off += s_wave[k];
        if (keep) {
            int idx = off + before;
            if (idx < row_cap) row_list[(size_t)y * row_cap + idx] = make_int4(x, y, sc, 0);
        }
        __syncthreads();
        if (tid == 0) s_base += s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
        __syncthreads();
    }
    if (tid == 0) row_count[y] = min(s_base, row_cap);
}

// Exclusive prefix over the per-row counts, then copy (row-major order).
__global__ __launch_bounds__(256) void fast_compact_kernel(const int* __restrict__ row_count,
                                                           const int4* __restrict__ row_list,
                                                           int row_cap, int h, int cap,
                                                           float2* __restrict__ kp_out,
                                                           int4* __restrict__ raw_out,
                                                           int* __restrict__ n_out) {
    __shared__ int s_part[4];
    const int y = blockIdx.x;
    const int tid = threadIdx.x;
    int acc = 0;
    for (int r = tid; r < y; r += 256) acc += row_count[r];
    acc = viso::wave_sum_int(acc);
    if ((tid & 63) == 0) s_part[tid >> 6] = acc;
    __syncthreads();
    const int base = s_part[0] + s_part[1] + s_part[2] + s_part[3];
    const int cnt = row_count[y];
    for (int i = tid; i < cnt; i += 256) {
        int o = base + i;
        if (o < cap) {
            int4 k = row_list[(size_t)y * row_cap + i];
            if (kp_out) kp_out[o] = make_float2((float)k.x, (float)k.y);
            if (raw_out) raw_out[o] = k;
        }
    }
    if (y == h - 1 && tid == 0) *n_out = base + cnt;
}

}  // namespace

void launch_pyramid_frames(const PyrGeom& g, const uint8_t* const* l0, uint8_t* const* slot,
                           int n, hipStream_t stream) {
    auto cdiv = [](int a, int b) { return (a + b - 1) / b; };
    const int tx = std::max(cdiv(g.w[3], kF3W), std::max(cdiv(g.w[2], 2 * kF3W), cdiv(g.w[1], 4 * kF3W)));
    const int ty = std::max(cdiv(g.h[3], kF3H), std::max(cdiv(g.h[2], 2 * kF3H), cdiv(g.h[1], 4 * kF3H)));
    for (int b0 = 0; b0 < n; b0 += kPyrBatch) {
        const int nb = (n - b0) < kPyrBatch ? (n - b0) : kPyrBatch;
        PyrFusedArgs a;
        for (int l = 0; l < kLevels; ++l) {
            a.w[l] = g.w[l];
            a.h[l] = g.h[l];
            a.off[l] = g.off[l];
        }
        for (int i = 0; i < nb; ++i) {
            a.l0[i] = l0[b0 + i];
            a.slot[i] = slot[b0 + i];
        }
        pyr_fused_kernel<<<dim3(tx, ty, nb), 256, 0, stream>>>(a);
    }
}

// Reference (unfused) form: one launch per level; kept for A/B timing.
void launch_pyramid_frames_unfused(const PyrGeom& g, const uint8_t* const* l0,
                                   uint8_t* const* slot, int n, hipStream_t stream) {
    for (int b0 = 0; b0 < n; b0 += kPyrBatch) {
        const int nb = (n - b0) < kPyrBatch ? (n - b0) : kPyrBatch;
        for (int l = 1; l < kLevels; ++l) {
            PyrPtrs p;
            for (int i = 0; i < nb; ++i) {
                p.src[i] = l == 1 ? l0[b0 + i] : slot[b0 + i] + g.off[l - 1];
                p.dst[i] = slot[b0 + i] + g.off[l];
            }
            dim3 grid((g.w[l] + kPyrTileW - 1) / kPyrTileW, (g.h[l] + kPyrTileH - 1) / kPyrTileH, nb);
            pyr_down_kernel<<<grid, 256, 0, stream>>>(p, g.w[l - 1], g.h[l - 1], g.w[l], g.h[l]);
        }
    }
}

void launch_pyramid(const PyrGeom& g, uint8_t* base, int n_images, size_t img_stride,
                    hipStream_t stream) {
    std::vector<const uint8_t*> l0((size_t)n_images);
    std::vector<uint8_t*> slot((size_t)n_images);
    for (int i = 0; i < n_images; ++i) {
        slot[(size_t)i] = base + img_stride * (size_t)i;
        l0[(size_t)i] = slot[(size_t)i];
    }
    launch_pyramid_frames(g, l0.data(), slot.data(), n_images, stream);
}

size_t fast_row_cap(int w) { return (size_t)(w / 2 + 2); }

void launch_fast(const uint8_t* img, int w, int h, int thresh, FastScratch& s, float2* kp_out,
                 int4* raw_out, int cap, int* n_out, hipStream_t stream) {
    int row_cap = (int)fast_row_cap(w);
    size_t smem = 12 * (size_t)w;
    thresh = thresh < 0 ? 0 : (thresh > 255 ? 255 : thresh);
    fast_rows_kernel<<<h, 256, smem, stream>>>(img, w, h, thresh, s.row_count, s.row_list, row_cap);
    fast_compact_kernel<<<h, 256, 0, stream>>>(s.row_count, s.row_list, row_cap, h, cap, kp_out,
                                               raw_out, n_out);
}

}  // namespace viso
