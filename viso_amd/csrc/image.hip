// viso_amd — image-pass kernels for gfx950: pyramid (cv::pyrDown restated)
// and FAST-9/16 + NMS (cv::FAST restated).  Integer arithmetic, bit-exact
// against the oracle (oracle/oracle_image.cpp).
//
// Pyramid (product path): pyr_down_stream_kernel, one launch per level,
// batched over every image of a chunk; register-streaming bands (see below).
// HBM-bound: algorithmic bytes per image = level-0 read + levels 1..3 written
// (DESIGN.md §4).  pyr_fused3_kernel (one launch for all levels, LDS tiles)
// is kept for A/B timing (launch_pyramid_frames_fused).
//
// FAST: one workgroup per image row y.  It scores rows y-1, y, y+1 from a
// 9-row LDS window, applies the strict 3x3 NMS to row y and appends the
// surviving corners in ascending x with a ballot/popcount prefix (row-major
// order is then restored across rows by fast_compact, an exclusive prefix
// over per-row counts).
#include <algorithm>
#include <vector>

#include "kernels.hpp"

namespace viso {

namespace {

__device__ inline int reflect101(int p, int len) {
    if (len == 1) return 0;
    while (p < 0 || p >= len) p = (p < 0) ? -p : 2 * len - p - 2;
    return p;
}

// ---------------------------------------------------------------- fused pyramid (A/B)
// One workgroup owns a level-3 tile of 16x8 and the matching level-2 (32x16)
// and level-1 (64x32) tiles, staging the level-0 window that feeds them
// (149 x 85, recursive 5-tap halos) in LDS and filtering level by level.
constexpr int kF3W = 16, kF3H = 8;
constexpr int kF2W = 2 * kF3W + 3, kF2H = 2 * kF3H + 3;  // 35 x 19
constexpr int kF1W = 2 * kF2W + 3, kF1H = 2 * kF2H + 3;  // 73 x 41
constexpr int kF0W = 2 * kF1W + 3, kF0H = 2 * kF1H + 3;  // 149 x 85

struct PyrFusedArgs {
    const uint8_t* l0[kPyrBatch];
    uint8_t* slot[kPyrBatch];
    int w[4], h[4];
    unsigned long long off[4];
};

// Tile details:
//  * every window (level 0 in LDS as loaded, levels 1 and 2 as computed) is
//    made valid at its out-of-image positions by copying the reflect-101
//    partner (per level, against that level's size) once per border tile, so
//    the filter taps are plain LDS reads at fixed offsets (no per-tap
//    reflection, no bounds tests);
//  * level 0 rows are fetched as aligned 16-byte chunks straight into a raw
//    LDS row (16 bytes of slack either side for the border fill) and read at
//    a per-row byte offset;
//  * the horizontal passes produce two adjacent outputs per thread from 7
//    shared taps.
// Integer sums are exact, so the result equals three separate pyrDown passes.
constexpr int kR0P = 16 + 176 + 16;  // raw level-0 row: slack | chunks | slack

// Barrier for LDS hand-offs only (global loads stay in flight across it).
__device__ inline void lds_barrier_px() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

struct PyrTile {
    const uint8_t* src;
    uint8_t* base;
    int X3, Y3, ox0, oy0, cl, ch;
};

__device__ inline PyrTile pyr_tile(const PyrFusedArgs& a, int t, int tx, int ty) {
    PyrTile T;
    const int per = tx * ty;
    const int z = t / per, rem = t - z * per;
    const int by = rem / tx, bx = rem - by * tx;
    T.src = a.l0[z];
    T.base = a.slot[z];
    T.X3 = bx * kF3W;
    T.Y3 = by * kF3H;
    const int ox2 = 2 * T.X3 - 2, oy2 = 2 * T.Y3 - 2;
    const int ox1 = 2 * ox2 - 2, oy1 = 2 * oy2 - 2;
    T.ox0 = 2 * ox1 - 2;
    T.oy0 = 2 * oy1 - 2;
    T.cl = max(T.ox0, 0);
    T.ch = min(T.ox0 + kF0W, a.w[0]);
    return T;
}

// Level-0 window chunk j of this thread: row r = it / 11, 16-byte chunk k.
// The chunk is addressed as src + off (an offset, not a rebuilt pointer, so
// the load stays a global_load: a flat load would also count in lgkmcnt and
// be drained by the LDS-only barriers).
__device__ inline bool pyr_chunk(const PyrFusedArgs& a, const PyrTile& T, int j, int& r, int& k,
                                 long long& off) {
    const int it = (int)threadIdx.x + 256 * j;
    if (it >= kF0H * 11) return false;
    r = it / 11;
    k = it - r * 11;
    const int ys = reflect101(T.oy0 + r, a.h[0]);
    const long long row = (long long)ys * a.w[0];
    const long long mis = (long long)(((uintptr_t)T.src + (uintptr_t)(row + T.cl)) & 15);
    off = row + T.cl - mis + 16 * (long long)k;
    return off < row + T.ch;
}

__device__ inline void pyr_issue(const PyrFusedArgs& a, const PyrTile& T, uint4 (&v)[4]) {
    const long long n = (long long)a.w[0] * a.h[0];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        int r, k;
        long long off;
        v[j] = make_uint4(0, 0, 0, 0);
        if (!pyr_chunk(a, T, j, r, k, off)) continue;
        if (off >= 0 && off + 16 <= n) {
            v[j] = *reinterpret_cast<const uint4*>(T.src + off);
        } else {  // the image's first / last bytes: no read outside the buffer
            uint32_t wv[4] = {0, 0, 0, 0};
#pragma unroll
            for (int b = 0; b < 16; ++b)
                if (off + b >= 0 && off + b < n) wv[b >> 2] |= (uint32_t)T.src[off + b] << (8 * (b & 3));
            v[j] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
        }
    }
}

// Persistent form of the v2 tile: each workgroup walks tiles t, t + grid,
// ...; the next tile's level-0 chunks are loaded into registers while the
// current tile is filtered (the passes hand off through LDS-only barriers,
// so those loads stay in flight).
__global__ __launch_bounds__(256) void pyr_fused3_kernel(PyrFusedArgs a, int tx, int ty, int total) {
    __shared__ __attribute__((aligned(16))) uint8_t s0[kF0H][kR0P];
    __shared__ int s_base[kF0H];
    __shared__ short hs0[kF0H][kF1W + 1];
    __shared__ uint8_t s1[kF1H][kF1W + 3];
    __shared__ short hs1[kF1H][kF2W + 1];
    __shared__ uint8_t s2[kF2H][kF2W + 1];
    const int tid = threadIdx.x;
    const int w0 = a.w[0], h0 = a.h[0], w1 = a.w[1], h1 = a.h[1];
    const int w2 = a.w[2], h2 = a.h[2], w3 = a.w[3], h3 = a.h[3];
    int t = blockIdx.x;
    if (t >= total) return;
    uint4 v[4];
    PyrTile T = pyr_tile(a, t, tx, ty);
    pyr_issue(a, T, v);
    for (; t < total; t += gridDim.x) {
        const int X3 = T.X3, Y3 = T.Y3;
        const int ox2 = 2 * X3 - 2, oy2 = 2 * Y3 - 2;
        const int ox1 = 2 * ox2 - 2, oy1 = 2 * oy2 - 2;
        const int ox0 = T.ox0, oy0 = T.oy0;
        uint8_t* __restrict__ base = T.base;
        if (tid < kF0H) {
            const int ys = reflect101(oy0 + tid, h0);
            const uintptr_t row = (uintptr_t)T.src + (uintptr_t)ys * w0;
            s_base[tid] = 16 + (int)((row + ox0) - ((row + T.cl) & ~(uintptr_t)15));
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            int r, k;
            long long off;
            if (pyr_chunk(a, T, j, r, k, off)) *reinterpret_cast<uint4*>(&s0[r][16 + 16 * k]) = v[j];
        }
        lds_barrier_px();
        const bool xborder = ox0 < 0 || ox0 + kF0W > w0;
        // prefetch the next tile
        const int tn = t + (int)gridDim.x;
        if (tn < total) {
            T = pyr_tile(a, tn, tx, ty);
            pyr_issue(a, T, v);
        }
        if (xborder) {  // out-of-image columns <- reflect-101 partners (same row)
            for (int it = tid; it < kF0H * kF0W; it += 256) {
                const int r = it / kF0W, c = it - r * kF0W;
                const int x = ox0 + c;
                if (x >= 0 && x < w0) continue;
                const int b = s_base[r];
                s0[r][b + c] = s0[r][b + reflect101(x, w0) - ox0];
            }
            lds_barrier_px();
        }
        // ---- level 1, horizontal: hs0[r][c] for in-image x1 = ox1 + c, two at a time
        const int c1lo = max(0, -ox1), c1hi = min(kF1W, w1 - ox1);
#pragma unroll 4
        for (int it = tid; it < kF0H * 37; it += 256) {
            const int r = it / 37, c = 2 * (it - r * 37);
            if (c >= c1hi || c + 1 < c1lo) continue;
            const uint8_t* p = &s0[r][s_base[r] + 2 * c];
            const int t0 = p[0], t1 = p[1], t2 = p[2], t3 = p[3], t4 = p[4], t5 = p[5], t6 = p[6];
            if (c >= c1lo) hs0[r][c] = (short)(t0 + 4 * t1 + 6 * t2 + 4 * t3 + t4);
            if (c + 1 < c1hi) hs0[r][c + 1] = (short)(t2 + 4 * t3 + 6 * t4 + 4 * t5 + t6);
        }
        lds_barrier_px();
        // ---- level 1, vertical (+ store of the tile's own 64 x 32 core)
        uint8_t* d1 = base + a.off[1];
        const int r1lo = max(0, -oy1), r1hi = min(kF1H, h1 - oy1);
#pragma unroll 4
        for (int it = tid; it < kF1H * kF1W; it += 256) {
            const int r = it / kF1W, c = it - r * kF1W;
            if (r < r1lo || r >= r1hi || c < c1lo || c >= c1hi) continue;
            const int s = hs0[2 * r][c] + 4 * hs0[2 * r + 1][c] + 6 * hs0[2 * r + 2][c] +
                          4 * hs0[2 * r + 3][c] + hs0[2 * r + 4][c];
            const uint8_t o = (uint8_t)((s + 128) >> 8);
            s1[r][c] = o;
            const int x1 = ox1 + c, y1 = oy1 + r;
            if (x1 >= 4 * X3 && x1 < 4 * X3 + 4 * kF3W && y1 >= 4 * Y3 && y1 < 4 * Y3 + 4 * kF3H)
                d1[(size_t)y1 * w1 + x1] = o;
        }
        lds_barrier_px();
        const bool b1 = c1lo > 0 || c1hi < kF1W || r1lo > 0 || r1hi < kF1H;
        if (b1) {
            for (int it = tid; it < kF1H * kF1W; it += 256) {  // columns, in-image rows
                const int r = it / kF1W, c = it - r * kF1W;
                if (r < r1lo || r >= r1hi || (c >= c1lo && c < c1hi)) continue;
                s1[r][c] = s1[r][reflect101(ox1 + c, w1) - ox1];
            }
            lds_barrier_px();
            for (int it = tid; it < kF1H * kF1W; it += 256) {  // whole rows
                const int r = it / kF1W, c = it - r * kF1W;
                if (r >= r1lo && r < r1hi) continue;
                s1[r][c] = s1[reflect101(oy1 + r, h1) - oy1][c];
            }
            lds_barrier_px();
        }
        // ---- level 2, horizontal
        const int c2lo = max(0, -ox2), c2hi = min(kF2W, w2 - ox2);
#pragma unroll 4
        for (int it = tid; it < kF1H * 18; it += 256) {
            const int r = it / 18, c = 2 * (it - r * 18);
            if (c >= c2hi || c + 1 < c2lo) continue;
            const uint8_t* p = &s1[r][2 * c];
            const int t0 = p[0], t1 = p[1], t2 = p[2], t3 = p[3], t4 = p[4];
            if (c >= c2lo) hs1[r][c] = (short)(t0 + 4 * t1 + 6 * t2 + 4 * t3 + t4);
            if (c + 1 < c2hi) {
                const int t5 = p[5], t6 = p[6];
                hs1[r][c + 1] = (short)(t2 + 4 * t3 + 6 * t4 + 4 * t5 + t6);
            }
        }
        lds_barrier_px();
        // ---- level 2, vertical (+ 32 x 16 core)
        uint8_t* d2 = base + a.off[2];
        const int r2lo = max(0, -oy2), r2hi = min(kF2H, h2 - oy2);
#pragma unroll 4
        for (int it = tid; it < kF2H * kF2W; it += 256) {
            const int r = it / kF2W, c = it - r * kF2W;
            if (r < r2lo || r >= r2hi || c < c2lo || c >= c2hi) continue;
            const int s = hs1[2 * r][c] + 4 * hs1[2 * r + 1][c] + 6 * hs1[2 * r + 2][c] +
                          4 * hs1[2 * r + 3][c] + hs1[2 * r + 4][c];
            const uint8_t o = (uint8_t)((s + 128) >> 8);
            s2[r][c] = o;
            const int x2 = ox2 + c, y2 = oy2 + r;
            if (x2 >= 2 * X3 && x2 < 2 * X3 + 2 * kF3W && y2 >= 2 * Y3 && y2 < 2 * Y3 + 2 * kF3H)
                d2[(size_t)y2 * w2 + x2] = o;
        }
        lds_barrier_px();
        const bool b2 = c2lo > 0 || c2hi < kF2W || r2lo > 0 || r2hi < kF2H;
        if (b2) {
            for (int it = tid; it < kF2H * kF2W; it += 256) {
                const int r = it / kF2W, c = it - r * kF2W;
                if (r < r2lo || r >= r2hi || (c >= c2lo && c < c2hi)) continue;
                s2[r][c] = s2[r][reflect101(ox2 + c, w2) - ox2];
            }
            lds_barrier_px();
            for (int it = tid; it < kF2H * kF2W; it += 256) {
                const int r = it / kF2W, c = it - r * kF2W;
                if (r >= r2lo && r < r2hi) continue;
                s2[r][c] = s2[reflect101(oy2 + r, h2) - oy2][c];
            }
            lds_barrier_px();
        }
        // ---- level 3 (16 x 8 outputs, 25 taps each)
        uint8_t* d3 = base + a.off[3];
        if (tid < kF3W * kF3H) {
            const int cx = tid & (kF3W - 1), cy = tid / kF3W;
            const int x3 = X3 + cx, y3 = Y3 + cy;
            if (x3 < w3 && y3 < h3) {
                int s = 0;
    #pragma unroll
                for (int i = 0; i < 5; ++i) {
                    const int wi = i == 2 ? 6 : ((i & 1) ? 4 : 1);
                    const uint8_t* p = &s2[2 * cy + i][2 * cx];
                    s += wi * ((int)p[0] + 4 * (int)p[1] + 6 * (int)p[2] + 4 * (int)p[3] + (int)p[4]);
                }
                d3[(size_t)y3 * w3 + x3] = (uint8_t)((s + 128) >> 8);
            }
        }
        lds_barrier_px();  // the next tile overwrites the windows
    }
}

// ---------------------------------------------------------------- streaming pyrDown
// One launch per level (L0->L1, L1->L2, L2->L3), batched over images.  A wave
// owns a strip of 248 destination columns (4 per lane on lanes 0..61) and a
// band of BH destination rows.  At entry it issues the loads of all 2*BH+3
// source rows of its band (one 8-byte load per lane and row: 512 contiguous
// bytes per wave, enough for the strip's 2*248+3 source columns at any
// alignment), so the band costs one memory round trip; then it walks down the
// band keeping the horizontal 5-tap sums of the last five source rows in
// registers.  Each source row is staged through a 512-byte LDS row so every
// lane can read its 11 taps at offsets with reflect-101 resolved once per
// wave.  Integer sums are exact: the result is cv::pyrDown's.
constexpr int kPsW = 248;   // destination columns per wave
constexpr int kPsRow = 512; // staged source row

struct PyrLevelArgs {
    const uint8_t* src[kPyrBatch];
    uint8_t* dst[kPyrBatch];
    int sw, sh, dw, dh;
    int bands, units;
};

// 8 source bytes at offset off, never reading outside [0, n).
__device__ inline uint2 ps_load(const uint8_t* __restrict__ img, long long off, long long n) {
    if (off >= 0 && off + 8 <= n) return *reinterpret_cast<const uint2*>(img + off);
    uint32_t w[2] = {0, 0};
#pragma unroll
    for (int b = 0; b < 8; ++b)
        if (off + b >= 0 && off + b < n) w[b >> 2] |= (uint32_t)img[off + b] << (8 * (b & 3));
    return make_uint2(w[0], w[1]);
}

template <int BH>
__global__ __launch_bounds__(256) void pyr_down_stream_kernel(PyrLevelArgs a) {
    constexpr int NR = 2 * BH + 3;  // source rows of a band
    __shared__ __attribute__((aligned(16))) uint8_t s_row[4][kPsRow];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int unit = blockIdx.x * 4 + wave;
    if (unit >= a.units) return;  // waves are independent: no block barrier below
    const uint8_t* __restrict__ src = a.src[blockIdx.y];
    uint8_t* __restrict__ dst = a.dst[blockIdx.y];
    const int sw = a.sw, sh = a.sh, dw = a.dw, dh = a.dh;
    // consecutive units = consecutive bands of one strip (shared halo rows)
    const int strip = unit / a.bands, band = unit - strip * a.bands;
    const int X = strip * kPsW, Y = band * BH;
    const int rows = min(BH, dh - Y);
    const long long n = (long long)sw * sh;
    const int cs = max(2 * X - 2, 0);  // first in-image source column of the strip
    // ---- all source rows of the band: one 8-byte load per lane and row
    uint2 v[NR];
    int mis[NR];
#pragma unroll
    for (int i = 0; i < NR; ++i) {
        const long long off = (long long)reflect101(2 * Y - 2 + i, sh) * sw + cs;
        mis[i] = (int)(((uintptr_t)src + (uintptr_t)off) & 7);
        v[i] = ps_load(src, off - mis[i] + 8 * lane, n);
    }
    // per-lane tap offsets (relative to column cs) of source columns
    // 2X + 8*lane - 2 + k, k < 11, reflect-101 against sw; lanes past the
    // level's edge read clamped junk that is never stored
    int P[11];
#pragma unroll
    for (int k = 0; k < 11; ++k)
        P[k] = min(max(reflect101(2 * X + 8 * lane - 2 + k, sw) - cs, 0), kPsRow - 8);
    uint8_t* row_lds = s_row[wave];
    auto hsum = [&](uint2 r, int m, int (&h)[4]) {
        *reinterpret_cast<uint2*>(row_lds + 8 * lane) = r;
        __builtin_amdgcn_wave_barrier();
        int t[11];
#pragma unroll
        for (int k = 0; k < 11; ++k) t[k] = row_lds[P[k] + m];
#pragma unroll
        for (int q = 0; q < 4; ++q)
            h[q] = t[2 * q] + t[2 * q + 4] + 4 * (t[2 * q + 1] + t[2 * q + 3]) + 6 * t[2 * q + 2];
        __builtin_amdgcn_wave_barrier();
    };
    int H[5][4];
#pragma unroll
    for (int i = 0; i < 5; ++i) hsum(v[i], mis[i], H[i]);
#pragma unroll
    for (int j = 0; j < BH; ++j) {
        if (j < rows) {
            const int y = Y + j;
            uint8_t* out = dst + (size_t)y * dw + X + 4 * lane;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int s = H[0][q] + H[4][q] + 4 * (H[1][q] + H[3][q]) + 6 * H[2][q];
                if (lane < kPsW / 4 && X + 4 * lane + q < dw) out[q] = (uint8_t)((s + 128) >> 8);
            }
            if (j + 1 < rows) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    H[0][q] = H[2][q];
                    H[1][q] = H[3][q];
                    H[2][q] = H[4][q];
                }
                hsum(v[5 + 2 * j], mis[5 + 2 * j], H[3]);
                hsum(v[6 + 2 * j], mis[6 + 2 * j], H[4]);
            }
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
            PyrLevelArgs a;
            for (int i = 0; i < nb; ++i) {
                a.src[i] = l == 1 ? l0[b0 + i] : slot[b0 + i] + g.off[l - 1];
                a.dst[i] = slot[b0 + i] + g.off[l];
            }
            a.sw = g.w[l - 1];
            a.sh = g.h[l - 1];
            a.dw = g.w[l];
            a.dh = g.h[l];
            const int bh = l == 1 ? 8 : (l == 2 ? 4 : 2);
            a.bands = (a.dh + bh - 1) / bh;
            a.units = a.bands * ((a.dw + kPsW - 1) / kPsW);
            const dim3 grid((a.units + 3) / 4, nb);
            if (l == 1)
                pyr_down_stream_kernel<8><<<grid, 256, 0, stream>>>(a);
            else if (l == 2)
                pyr_down_stream_kernel<4><<<grid, 256, 0, stream>>>(a);
            else
                pyr_down_stream_kernel<2><<<grid, 256, 0, stream>>>(a);
        }
    }
}

// Fused single-launch form (pyr_fused3_kernel), kept for A/B timing.
void launch_pyramid_frames_fused(const PyrGeom& g, const uint8_t* const* l0, uint8_t* const* slot,
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
        const int total = tx * ty * nb;
        pyr_fused3_kernel<<<std::min(total, 1024), 256, 0, stream>>>(a, tx, ty, total);
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
