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
