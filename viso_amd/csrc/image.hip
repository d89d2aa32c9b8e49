// viso_amd — image-pass kernels for gfx950: pyramid (cv::pyrDown restated)
// and FAST-9/16 + NMS (cv::FAST restated).  Integer arithmetic, bit-exact
// against the oracle (oracle/oracle_image.cpp).
//
// Pyramid: two launches per chunk, batched over every image of it:
// pyr_down_sk_kernel (register-only streaming bands) for level 1, then
// pyr_tail_kernel (levels 2 and 3, one workgroup per band of an image, the
// level-2 halo recomputed in LDS).  pyr_down_stream_kernel (LDS-staged rows)
// covers the levels of images whose level 1 is under 8 columns.  HBM-bound:
// algorithmic bytes per image = level-0 read + levels 1..3 written
// (DESIGN.md §4).
//
// FAST: a tiled scoring / NMS launch and an ordering launch (see the FAST
// section below).
#include <algorithm>
#include <type_traits>
#include <vector>

#include "kernels.hpp"

#ifdef VISO_PROBE
// dev instrumentation: per-wave timeline of the last level-1 launch (start,
// end, HW_ID, XCC_ID) and per-block timeline of the last tail launch
// (start, phase ends, HW_ID | XCC_ID << 32); s_memrealtime, 100 MHz
__device__ unsigned long long g_pyr_tl[8192][5];
#endif

namespace viso {

namespace {

__device__ inline int reflect101(int p, int len) {
    if (len == 1) return 0;
    while (p < 0 || p >= len) p = (p < 0) ? -p : 2 * len - p - 2;
    return p;
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
    // XCD dealing (pyr_down_sk_kernel, xcd_per > 0): the chunk's work list
    // (image-major, 4 units per block) is cut into 8 contiguous runs, block
    // L takes item (L & 7) * xcd_per + (L >> 3), so the bands and strips of
    // an image (which share halo rows and boundary lines) run on one XCD's L2
    int xcd_per, bpi, n_img;
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

// Register-only pyrDown (pyr_down_sk_kernel below; same decomposition and
// exact integer sums as pyr_down_stream_kernel) for source levels at least
// 8 columns wide.  Lane l loads 8 source bytes per row (one unaligned 8-byte
// load) and takes the next lane's first dword by DPP: its 11 taps are bytes
// 0..10 of the 12-byte window (w0, w1, w2).  The horizontal 5-tap sums are
// v_dot4_u32_u8 with weights (1, 4, 6, 4) plus the fifth tap, packed in pairs
// into 16-bit halves, so the vertical sums of two destination columns run as
// one packed op (max 65408 < 2^16).  Reflect-101 at the left/right image
// edges is a per-lane byte permutation of the window, computed once per wave
// (edge waves only).
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ inline u16x2 as_u16x2(uint32_t x) { return __builtin_bit_cast(u16x2, x); }

struct PkEdge {
    uint32_t sel0, sel1, sel2;
};

// horizontal sums for 4 destination columns from their 11 source taps
// (bytes 0..10 of w0, w1, w2)
__device__ inline void pk_hsum3(uint32_t w0, uint32_t w1, uint32_t w2, u16x2 (&h)[2]) {
    constexpr uint32_t K = 0x04060401u;  // taps 0..3 of [1 4 6 4 1]
    const uint32_t a1 = __builtin_amdgcn_alignbyte(w1, w0, 2);  // t2..t5
    const uint32_t a3 = __builtin_amdgcn_alignbyte(w2, w1, 2);  // t6..t9
    const uint32_t h0 = __builtin_amdgcn_udot4(w1, 0x00000001u, __builtin_amdgcn_udot4(w0, K, 0, false), false);
    const uint32_t h1 = __builtin_amdgcn_udot4(w1, 0x00010000u, __builtin_amdgcn_udot4(a1, K, 0, false), false);
    const uint32_t h2 = __builtin_amdgcn_udot4(w2, 0x00000001u, __builtin_amdgcn_udot4(w1, K, 0, false), false);
    const uint32_t h3 = __builtin_amdgcn_udot4(w2, 0x00010000u, __builtin_amdgcn_udot4(a3, K, 0, false), false);
    h[0] = as_u16x2(__builtin_amdgcn_perm(h1, h0, 0x05040100u));
    h[1] = as_u16x2(__builtin_amdgcn_perm(h3, h2, 0x05040100u));
}

// horizontal sums of one source row for the lane's 4 destination columns
template <bool EDGE>
__device__ inline void pk_hsum(uint2 r, const PkEdge& e, u16x2 (&h)[2]) {
    uint32_t w0 = r.x, w1 = r.y;
    // next lane's first dword; lane 63 (which covers the 4 columns left of
    // the strip, see sk_band) wraps to lane 0
    uint32_t w2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r.x, 0x134, 0xf, 0xf, false);
    if (EDGE) {
        const uint32_t e0 = __builtin_amdgcn_perm(w1, w0, e.sel0);
        const uint32_t e1 = __builtin_amdgcn_perm(w1, w0, e.sel1);
        w2 = __builtin_amdgcn_perm(w2, w1, e.sel2);
        w0 = e0;
        w1 = e1;
    }
    pk_hsum3(w0, w1, w2, h);
}

// vertical 5-tap of two destination columns, rounded: (sum + 128) >> 8
__device__ inline u16x2 pk_vsum(u16x2 h0, u16x2 h1, u16x2 h2, u16x2 h3, u16x2 h4) {
    const u16x2 s = (u16x2)6 * h2 + (u16x2)128;
    return ((h0 + h4) + ((u16x2)4 * (h1 + h3) + s)) >> (u16x2)8;
}

// One wave = one strip of 244 destination columns x a band of BH
// destination rows, streamed: a ring of D source rows is kept in flight (one
// 8-byte load per lane and row), each consumed row's slot is refilled with
// the row D below, so HBM reads and the VALU work of the band overlap.
// Wave-uniform work (row pointers, store alignment) is scalar and kept to a
// few SALU ops per row: the scalar unit is shared by the CU's waves and was
// this kernel's first bottleneck.  Bands whose source rows need no
// reflect-101 and no load clamping (INTERIOR) walk running row pointers.
constexpr int kSkW = 244;  // destination columns per wave (lanes 0..60; 61 = right context)
// 8-row bands keep ~7 waves per SIMD in flight (measured in round 1:
// 24/12/6-row bands with a 16-row ring ran 30% slower); a 20-row ring holds
// all 19 source rows of a band, so each wave makes one memory round trip
// (round 2: 13.5 against 14.8 us per 50-image launch with an 8-row ring)
#ifndef VISO_SK_BH1
#define VISO_SK_BH1 8
#endif
constexpr int kSkBH1 = VISO_SK_BH1, kSkRing1 = 2 * kSkBH1 + 4;
// chunks of <= kSkSmallBatch images (under 1.5 waves per SIMD with 8-row
// bands; the launch is latency-bound): 4-row bands, twice the waves and half
// the chain per wave (20 images: 11.2 -> 8.3-8.8 us; 32: 12.2 -> 11.0 us)
constexpr int kSkSmallBatch = 32, kSkBHs = 4, kSkRings = 2 * kSkBHs + 4;

struct SkBand {
    const uint8_t* src;
    uint8_t* dst;
    int sw, sh, dw, n;
    int X, Y, rows, nr, c0, len;
};

template <int D, bool EDGE, bool INTERIOR>
__device__ inline void sk_band(const SkBand& b, const PkEdge& e, int lane) {
    // Lane l < 62 covers destination columns X + 4l .. X + 4l + 3 (lane 61:
    // the next strip's first 4; lane 62 only feeds lane 61's taps), lane 63
    // the 4 columns left of the strip (X > 0): so every aligned dword around
    // the strip's row segment is
    // computed whole by this wave, and neighbouring strips write the bytes
    // they share with identical values.  Only the image's row ends (left of
    // column 0, right of column dw - 1) need partial dwords.
    const int loff = (lane == 63 && b.X > 0) ? -8 : 8 * lane;  // window start - c0
    // ---- source rows: band row i (0 <= i < nr) is image row 2Y - 2 + i; rows
    // past nr repeat row nr - 1 (one real load per call keeps the waitcnt
    // counting exact; the repeats hit the cache)
    const uint8_t* p_next = b.src + (ptrdiff_t)(2 * b.Y - 2) * b.sw + b.c0;  // INTERIOR
    int issued = 0;
    auto row_off = [&](int i) { return reflect101(2 * b.Y - 2 + min(i, b.nr - 1), b.sh) * b.sw + b.c0; };
    auto unsafe_row = [&](int o0) { return o0 - 8 < 0 || o0 + 8 * 64 > b.n; };
    auto issue = [&](int i) -> uint2 {
        unsigned long long q;
        if constexpr (INTERIOR) {
            q = *reinterpret_cast<const __attribute__((address_space(1))) unsigned long long*>(
                reinterpret_cast<uintptr_t>(p_next) + loff);
            if (++issued < b.nr) p_next += b.sw;
        } else {
            const int o0 = row_off(i);
            int oc = o0 + loff;
            if (unsafe_row(o0)) oc = min(max(oc, 0), b.n - 8);
            q = *reinterpret_cast<const __attribute__((address_space(1))) unsigned long long*>(
                reinterpret_cast<uintptr_t>(b.src) + oc);
        }
        return make_uint2((uint32_t)q, (uint32_t)(q >> 32));
    };
    // clamped loads are shifted into place when consumed, not at issue, so
    // no wait is forced on a load still in flight
    auto fix = [&](uint2 r, int i) -> uint2 {
        if constexpr (INTERIOR) {
            return r;
        } else {
            const int o0 = row_off(i);
            if (!unsafe_row(o0)) return r;
            const int o = o0 + loff;
            const int d = max(min(o - min(max(o, 0), b.n - 8), 7), -7);  // lanes past the image: junk
            unsigned long long q = ((unsigned long long)r.y << 32) | r.x;
            q = d >= 0 ? q >> (8 * d) : q << (-8 * d);  // bytes outside [0, n) read as 0
            return make_uint2((uint32_t)q, (uint32_t)(q >> 32));
        }
    };
    // ---- destination rows: lane k < 62 writes the k-th aligned dword from
    // the row segment's start (bytes 4k - ma .. 4k - ma + 3 relative to
    // column X), its low bytes taken from lane k-1 (lane 0: lane 63) by DPP
    // wave_ror:1.  Writable bytes: [wlo, whi) relative to X.
    uint8_t* row_out = b.dst + (ptrdiff_t)b.Y * b.dw + b.X;
    const int wlo_x = b.X > 0 ? 1 : 0;                  // columns left of X exist
    const int whi = b.X + kSkW < b.dw ? kSkW + 4 : b.len;  // columns right of the strip exist
    auto store_row = [&](const u16x2 (&H)[5][2]) {
        const u16x2 o0 = pk_vsum(H[0][0], H[1][0], H[2][0], H[3][0], H[4][0]);
        const u16x2 o1 = pk_vsum(H[0][1], H[1][1], H[2][1], H[3][1], H[4][1]);
        const uint32_t bb = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, o1),
                                                  __builtin_bit_cast(uint32_t, o0), 0x06040200u);
        const int ma = (int)((uintptr_t)row_out & 3);
        const uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)bb, 0x13c, 0xf, 0xf, false);
        const uint32_t word = ma ? __builtin_amdgcn_alignbyte(bb, prev, 4 - ma) : bb;
        const int lo = 4 * lane - ma;
        auto* out = reinterpret_cast<__attribute__((address_space(1))) uint8_t*>(
            reinterpret_cast<uintptr_t>(row_out));
        row_out += b.dw;
        if constexpr (!EDGE) {
            if (lane < 62) *reinterpret_cast<__attribute__((address_space(1))) uint32_t*>(out + lo) = word;
        } else {
            const int wlo = wlo_x ? -ma : 0;
            if (lane < 62 && lo >= wlo && lo + 4 <= whi) {
                *reinterpret_cast<__attribute__((address_space(1))) uint32_t*>(out + lo) = word;
            } else if (lane < 62 && lo + 4 > wlo && lo < whi) {
                // a partial dword at an image row end: 4 byte stores, the
                // bytes outside [wlo, whi) redirected onto an own byte
                const int q0 = max(wlo - lo, 0), q1 = min(whi - lo, 4) - 1;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int qq = min(max(q, q0), q1);
                    out[lo + qq] = (uint8_t)(word >> (8 * qq));
                }
            }
        }
    };
    uint2 ring[D];
#pragma unroll
    for (int i = 0; i < D; ++i) ring[i] = issue(i);
    u16x2 H[5][2];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        pk_hsum<EDGE>(fix(ring[i], i), e, H[i]);
        ring[i] = issue(D + i);
    }
    store_row(H);
    // destination rows j0 .. j0 + D/2 - 1 (j0 = 1 + k D/2) consume source
    // rows k D + 5 .. k D + D + 4, i.e. ring slots 5 .. D-1, 0 .. 4: static
    // after unrolling
    for (int j0 = 1; j0 < b.rows; j0 += D / 2) {
#pragma unroll
        for (int u = 0; u < D / 2; ++u) {
            const int j = j0 + u;
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                H[0][q] = H[2][q];
                H[1][q] = H[3][q];
                H[2][q] = H[4][q];
            }
            pk_hsum<EDGE>(fix(ring[(5 + 2 * u) % D], 2 * j + 3), e, H[3]);
            ring[(5 + 2 * u) % D] = issue(2 * j + 3 + D);
            pk_hsum<EDGE>(fix(ring[(6 + 2 * u) % D], 2 * j + 4), e, H[4]);
            ring[(6 + 2 * u) % D] = issue(2 * j + 4 + D);
            if (j < b.rows) store_row(H);
        }
    }
}

// (the body of pyr_down_sk_kernel for workgroup (bx, by); pyr1_fast_kernel
// runs it for its first workgroups)
template <int BH, int D>
__device__ __forceinline__ void pyr_down_sk_body(const PyrLevelArgs& a, int bx, int by) {
    const int lane = threadIdx.x & 63;
    // everything that depends only on the wave's unit is wave-uniform: keep
    // it in SGPRs (readfirstlane) so the VALU only does the per-lane work
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int img = by, blk = bx;
    if (a.xcd_per > 0) {
        const int w = (bx & 7) * a.xcd_per + (bx >> 3);
        img = w / a.bpi;
        blk = w - img * a.bpi;
        if (img >= a.n_img) return;  // block-uniform (no barrier in this kernel)
    }
    const int unit = blk * 4 + wave;
    if (unit >= a.units) return;
#ifdef VISO_PROBE
    const unsigned long long pr_t0 = __builtin_amdgcn_s_memrealtime();
#endif
    SkBand b;
    b.src = a.src[img];
    b.dst = a.dst[img];
    b.sw = a.sw;
    b.sh = a.sh;
    b.dw = a.dw;
    b.n = a.sw * a.sh;  // levels are < 2^31 bytes (kMaxWidth)
    const int strip = unit / a.bands, band = unit - strip * a.bands;
    b.X = strip * kSkW;
    b.Y = band * BH;
    b.rows = min(BH, a.dh - b.Y);
    b.nr = 2 * b.rows + 3;  // source rows of the band
    b.c0 = 2 * b.X - 2;     // source column of lane 0's window byte 0
    b.len = min(kSkW, a.dw - b.X);  // destination bytes of the wave's row
    // reflect-101 of the window bytes that fall outside [0, sw): byte k of
    // lane l is column c = c0 + loff(l) + k; its value is column r(c), window byte
    // k + r(c) - c.  Lanes whose outputs are never stored keep the identity.
    const bool edge = b.X == 0 || b.c0 + 8 * (kSkW / 4) + 11 >= b.sw;
    PkEdge e{0x03020100u, 0x07060504u, 0x07060504u};
    if (edge) {
#pragma unroll
        for (int k = 0; k < 12; ++k) {
            const int c = b.c0 + ((lane == 63 && b.X > 0) ? -8 : 8 * lane) + k;
            const int rc = reflect101(c, b.sw);
            const int base = k >= 8 ? 4 : 0;  // w2' selects from (w2:w1)
            const int kk = k + rc - c - base;
            if (c != rc && kk >= 0 && kk < 8) {
                const int sh8 = 8 * (k & 3);
                const uint32_t m = ~(0xffu << sh8), val = (uint32_t)kk << sh8;
                if (k < 4) e.sel0 = (e.sel0 & m) | val;
                else if (k < 8) e.sel1 = (e.sel1 & m) | val;
                else e.sel2 = (e.sel2 & m) | val;
            }
        }
    }
    // interior: every band row is an image row and every load is in bounds
    const int r0 = 2 * b.Y - 2, r1 = r0 + b.nr - 1;
    const bool interior = r0 >= 0 && r1 < b.sh && r0 * b.sw + b.c0 >= 0 &&
                          r1 * b.sw + b.c0 + 8 * 64 <= b.n;
    if (interior) {
        if (edge) sk_band<D, true, true>(b, e, lane);
        else sk_band<D, false, true>(b, e, lane);
    } else {
        if (edge) sk_band<D, true, false>(b, e, lane);
        else sk_band<D, false, false>(b, e, lane);
    }
#ifdef VISO_PROBE
    if (lane == 0) {
        const long long w = (long long)img * a.units + unit;
        if (w < 8192) {
            g_pyr_tl[w][0] = pr_t0;
            g_pyr_tl[w][1] = __builtin_amdgcn_s_memrealtime();
            g_pyr_tl[w][2] = __builtin_amdgcn_s_getreg(4 | (31 << 11));
            g_pyr_tl[w][3] = __builtin_amdgcn_s_getreg(20 | (31 << 11));
            g_pyr_tl[w][4] = pr_t0;
        }
    }
#endif
}

template <int BH, int D>
__global__ __launch_bounds__(256) void pyr_down_sk_kernel(PyrLevelArgs a) {
    pyr_down_sk_body<BH, D>(a, (int)blockIdx.x, (int)blockIdx.y);
}

// ---------------------------------------------------------------- pyramid tail
// Levels 2 and 3 of every image of a chunk in ONE launch after the level-1
// launch, no workgroup waiting for another.  A workgroup owns a band of B
// level-3 rows of one image and the 2B level-2 rows above them (the image's
// last band: all remaining rows), and recomputes the level-2 halo rows its
// level-3 rows need:
//   phase 1  level-1 rows [c1a, c1b) from HBM -> LDS (16-byte loads, all in
//            flight at once)
//   phase 2  level-2 rows [c2a, c2b) from the LDS level 1 -> LDS (own rows -> HBM)
//   phase 3  the own level-3 rows from the LDS level 2 -> HBM
// A work item is 4 destination columns x RG destination rows (the register
// ring of sk_band: two new horizontal sums per destination row, v_dot4 +
// packed 16-bit vertical sums).  Staged rows carry reflect-101 pad bytes at
// both ends, so no phase has edge code.  Barriers wait for LDS only (own
// global stores are never re-read).  B is sized so the chunk's bands fill
// the resident workgroup slots once.  Against the per-level launches of
// round 1 the tail replaces two launches (each ~6 us, latency-bound at 50
// images) by one of ~9 us; one launch for all three levels from level 0
// (the level-0 halo staged slice by slice) measured 31 us, VALU-bound on the
// level-1 halo recompute.
constexpr int kPfThreads = 512;
constexpr int kPfRG2 = 2;                 // level-2 rows per work item
constexpr int kPfStage1 = 8;              // 16-byte level-1 loads per thread (max)
constexpr int kPfPad = 16;                // LDS bytes left of a staged row's column 0
#ifndef VISO_PF_SLOTS
#define VISO_PF_SLOTS 512
#endif
constexpr int kPfSlots = VISO_PF_SLOTS;   // resident workgroups the band height is sized for (2 per CU)
constexpr size_t kPfLdsMax = (size_t)160 * 1024 / (kPfSlots / 256);  // the CU's 160 KB LDS over its slots
static_assert(kPfSlots % 256 == 0 && kPfSlots <= 1024, "pyramid tail: 1..4 workgroups per CU");

typedef uint32_t pf_u32x4 __attribute__((ext_vector_type(4)));
constexpr int kPfOwnPer = 4;  // PyrOwn level-0 chunks per thread (16 bytes each)

struct PyrTailArgs {
    uint8_t* slot[kPyrBatch];
    size_t off1, off2, off3;
    int w1, h1, w2, h2, w3, h3;
    int n, nb, band, xcd_map;  // images, bands per image, level-3 rows per band, XCD map
    int s1, s2;                // LDS row strides of staged levels 1 / 2
    int lds1;                  // byte offset of the level-1 rows (level 2 below it)
    // PyrOwn (kernels.hpp) for image own_img: own_len level-0 bytes from
    // own_src into its slot (own_src null: none), its identity pose
    const uint8_t* own_src;
    double* ident_pose;
    int own_img, own_len;
    int* zero;  // PyrOwn::zero, n_zero ints cleared by the grid's threads
    int n_zero;
};

// own rows [o?a, o?b) and computed rows [c?a, c?b) of band b per level
struct PfBand {
    int o2a, o2b, o3a, o3b, c1a, c1b, c2a, c2b;
};

__host__ __device__ inline PfBand pf_band(int b, int nb, int band, int h1, int h2, int h3) {
    PfBand r;
    const bool last = b == nb - 1;
    r.o3a = band * b;
    r.o3b = last ? h3 : r.o3a + band;
    r.o2a = 2 * band * b;
    r.o2b = last ? h2 : r.o2a + 2 * band;
    // destination row y reads source rows 2y-2 .. 2y+2 (reflect-101 at the
    // borders lands within 3 rows of the border, inside the range then)
    r.c2a = min(r.o2a, max(0, 2 * r.o3a - 2));
    r.c2b = max(r.o2b, min(h2, 2 * (r.o3b - 1) + 3));
    r.c1a = max(0, 2 * r.c2a - 2);
    r.c1b = min(h1, 2 * (r.c2b - 1) + 3);
    return r;
}

// workgroup barrier for LDS hand-offs: waits for this wave's LDS traffic only
// (__syncthreads() would also wait for the wave's global stores)
__device__ inline void pf_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// 4 destination bytes (two packed pairs) -> one dword
__device__ inline uint32_t pf_pack(const u16x2 (&H)[5][2]) {
    const u16x2 o0 = pk_vsum(H[0][0], H[1][0], H[2][0], H[3][0], H[4][0]);
    const u16x2 o1 = pk_vsum(H[0][1], H[1][1], H[2][1], H[3][1], H[4][1]);
    return __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, o1), __builtin_bit_cast(uint32_t, o0), 0x06040200u);
}

// destination rows y0 .. y0+cnt-1 (cnt <= RG) of one item: fetch(i, w)
// yields the taps of source row 2*y0 - 2 + i, emit(j, dword) takes row y0 + j
template <int RG, class Fetch, class Emit>
__device__ inline void pf_rows(int cnt, Fetch&& fetch, Emit&& emit) {
    u16x2 H[5][2];
    uint32_t w[3];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        fetch(i, w);
        pk_hsum3(w[0], w[1], w[2], H[i]);
    }
#pragma unroll
    for (int j = 0; j < RG; ++j) {
        if (j < cnt) {
            emit(j, pf_pack(H));
            if (j + 1 < cnt) {
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    H[0][q] = H[2][q];
                    H[1][q] = H[3][q];
                    H[2][q] = H[4][q];
                }
                fetch(5 + 2 * j, w);
                pk_hsum3(w[0], w[1], w[2], H[3]);
                fetch(6 + 2 * j, w);
                pk_hsum3(w[0], w[1], w[2], H[4]);
            }
        }
    }
}

// store the dword of destination columns x .. x+3 of a row of width dw
__device__ inline void pf_store(uint8_t* row, int x, int dw, uint32_t v) {
    if (x + 4 <= dw) {
        *reinterpret_cast<__attribute__((address_space(1))) uint32_t*>(reinterpret_cast<uintptr_t>(row + x)) = v;
    } else {
        for (int q = 0; q < dw - x; ++q) row[x + q] = (uint8_t)(v >> (8 * q));
    }
}

// the taps of staged source row `row` (index into the LDS rows) for
// destination columns 4g .. 4g+3: bytes kPfPad + 8g - 2 .. + 10
__device__ inline void pf_lds_taps(const uint8_t* lds, int stride, int row, int g, uint32_t (&w)[3]) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(lds + (size_t)row * stride + kPfPad - 4 + 8 * g);
    const uint32_t d0 = p[0], d1 = p[1], d2 = p[2], d3 = p[3];
    w[0] = __builtin_amdgcn_alignbyte(d1, d0, 2);
    w[1] = __builtin_amdgcn_alignbyte(d2, d1, 2);
    w[2] = __builtin_amdgcn_alignbyte(d3, d2, 2);
}

// reflect-101 pad bytes (columns -2, -1, w, w+1) of staged rows
__device__ inline void pf_pads(uint8_t* lds, int stride, int rows, int w, int tid) {
    for (int t = tid; t < 4 * rows; t += kPfThreads) {
        const int row = t >> 2, k = t & 3;
        const int c = k < 2 ? k - 2 : w + k - 2;
        uint8_t* base = lds + (size_t)row * stride + kPfPad;
        base[c] = base[reflect101(c, w)];
    }
}

__global__ __launch_bounds__(kPfThreads) void pyr_tail_kernel(PyrTailArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t s_pf[];
    int img, band;
    if (a.xcd_map) {  // blocks are dealt to the 8 XCDs round-robin: all bands of an image on one XCD
        const int q = (int)blockIdx.x >> 3;
        band = q % a.nb;
        img = 8 * (q / a.nb) + ((int)blockIdx.x & 7);
    } else {
        band = (int)blockIdx.x % a.nb;
        img = (int)blockIdx.x / a.nb;
    }
    for (int i = (int)(blockIdx.x * kPfThreads + threadIdx.x); i < a.n_zero; i += (int)(gridDim.x * kPfThreads))
        a.zero[i] = 0;
    if (img >= a.n) return;  // block-uniform, before any barrier
#ifdef VISO_PROBE
    const unsigned long long pr_t0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long pr_t1 = 0, pr_t2 = 0;
#endif
    const PfBand r = pf_band(band, a.nb, a.band, a.h1, a.h2, a.h3);
    const uint8_t* l1 = a.slot[img] + a.off1;
    uint8_t* l2 = a.slot[img] + a.off2;
    uint8_t* l3 = a.slot[img] + a.off3;
    uint8_t* lds1 = s_pf + a.lds1;
    uint8_t* lds2 = s_pf;
    const int tid = (int)threadIdx.x;
    // ---- PyrOwn: the identity pose; the image's bands split its level-0
    // copy in 16-byte chunks (the source possibly unaligned: a caller's frame
    // at f * w * h), at most kPfOwnPer per thread (the launcher's limit),
    // loaded ahead of phase 1's loads and stored behind them, so that the
    // two latencies overlap
    if (img == a.own_img && a.ident_pose && band == 0 && tid < 12)
        a.ident_pose[tid] = (tid == 0 || tid == 4 || tid == 8) ? 1.0 : 0.0;
    const bool own_copy = img == a.own_img && a.own_src;
    const int own_c16 = a.own_len >> 4;
    const int own_lo = own_copy ? (int)((long long)own_c16 * band / a.nb) : 0;
    const int own_hi = own_copy ? (int)((long long)own_c16 * (band + 1) / a.nb) : 0;
    pf_u32x4 oq[kPfOwnPer];
    if (own_copy) {
#pragma unroll
        for (int j = 0; j < kPfOwnPer; ++j) {
            const int k = own_lo + tid + j * kPfThreads;
            if (k < own_hi)
                oq[j] = *reinterpret_cast<const __attribute__((address_space(1))) pf_u32x4*>(
                    reinterpret_cast<uintptr_t>(a.own_src + 16 * (size_t)k));
        }
    }
    // ---- phase 1: level-1 rows [c1a, c1b) from HBM (a chunk past a row end
    // reads into the next row or level 2 of the slot)
    {
        const int C = (a.w1 + 15) >> 4, rows = r.c1b - r.c1a;
        pf_u32x4 q[kPfStage1];
        int off[kPfStage1];
#pragma unroll
        for (int k = 0; k < kPfStage1; ++k) {
            const int t = tid + k * kPfThreads, i = t / C, c = t - i * C;
            off[k] = i < rows ? i * a.s1 + kPfPad + 16 * c : -1;
            if (i < rows)
                q[k] = *reinterpret_cast<const __attribute__((address_space(1))) pf_u32x4*>(
                    reinterpret_cast<uintptr_t>(l1 + (size_t)(r.c1a + i) * a.w1 + 16 * c));
        }
        if (own_copy) {
            uint8_t* dst = a.slot[img];
#pragma unroll
            for (int j = 0; j < kPfOwnPer; ++j) {
                const int k = own_lo + tid + j * kPfThreads;
                if (k < own_hi)
                    *reinterpret_cast<__attribute__((address_space(1))) pf_u32x4*>(
                        reinterpret_cast<uintptr_t>(dst + 16 * (size_t)k)) = oq[j];
            }
            if (band == a.nb - 1)
                for (int i = 16 * own_c16 + tid; i < a.own_len; i += kPfThreads) dst[i] = a.own_src[i];
        }
#pragma unroll
        for (int k = 0; k < kPfStage1; ++k)
            if (off[k] >= 0) *reinterpret_cast<pf_u32x4*>(lds1 + off[k]) = q[k];
        pf_barrier();
#ifdef VISO_PROBE
        pr_t1 = __builtin_amdgcn_s_memrealtime();
#endif
        pf_pads(lds1, a.s1, rows, a.w1, tid);
        pf_barrier();
    }
    // ---- phase 2: level 2
    {
        const int G = (a.w2 + 3) >> 2, rows = r.c2b - r.c2a, nrg = (rows + kPfRG2 - 1) / kPfRG2;
        for (int it = tid; it < nrg * G; it += kPfThreads) {
            const int rg = it / G, g = it - rg * G;
            const int y0 = r.c2a + rg * kPfRG2;
            // source rows 2y0-2 .. 2y0+4 inside level 1: consecutive staged rows
            const bool inner = 2 * y0 - 2 >= 0 && 2 * y0 + 4 < a.h1;
            auto fetch = [&](int i, uint32_t (&w)[3]) {
                const int row = inner ? 2 * y0 - 2 + i : reflect101(2 * y0 - 2 + i, a.h1);
                pf_lds_taps(lds1, a.s1, row - r.c1a, g, w);
            };
            auto emit = [&](int j, uint32_t val) {
                const int y = y0 + j;
                *reinterpret_cast<uint32_t*>(lds2 + (size_t)(y - r.c2a) * a.s2 + kPfPad + 4 * g) = val;
                if (y >= r.o2a && y < r.o2b) pf_store(l2 + (size_t)y * a.w2, 4 * g, a.w2, val);
            };
            pf_rows<kPfRG2>(min(kPfRG2, r.c2b - y0), fetch, emit);
        }
        pf_barrier();
#ifdef VISO_PROBE
        pr_t2 = __builtin_amdgcn_s_memrealtime();
#endif
        pf_pads(lds2, a.s2, rows, a.w2, tid);
        pf_barrier();
    }
    // ---- phase 3: level 3 (own rows only)
    {
        const int G = (a.w3 + 3) >> 2, rows = r.o3b - r.o3a;
        for (int it = tid; it < rows * G; it += kPfThreads) {
            const int y = r.o3a + it / G, g = it % G;
            auto fetch = [&](int i, uint32_t (&w)[3]) {
                pf_lds_taps(lds2, a.s2, reflect101(2 * y - 2 + i, a.h2) - r.c2a, g, w);
            };
            auto emit = [&](int, uint32_t val) { pf_store(l3 + (size_t)y * a.w3, 4 * g, a.w3, val); };
            pf_rows<1>(1, fetch, emit);
        }
    }
#ifdef VISO_PROBE
    // block timeline: start, phase 1 done, phase 2 done, end (100 MHz), HW_ID | XCC_ID << 32
    __syncthreads();
    const int w = img * a.nb + band;
    if (tid == 0 && w < 8192) {
        g_pyr_tl[w][0] = pr_t0;
        g_pyr_tl[w][1] = pr_t1;
        g_pyr_tl[w][2] = pr_t2;
        g_pyr_tl[w][3] = __builtin_amdgcn_s_memrealtime();
        g_pyr_tl[w][4] = (unsigned long long)__builtin_amdgcn_s_getreg(4 | (31 << 11)) |
                         ((unsigned long long)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 32);
    }
#endif
}

// ---------------------------------------------------------------- FAST
// Two launches per image (cv::FAST(img, kp, t) with NMS, src/viso.cpp:104;
// OpenCV 3.x FAST_t<16> + cornerScore<16> restated):
//
// fast_tile_kernel — workgroup = tile of kFtCols output columns x kFtRows
//   output rows.  The tile's pixel rows (+3 circle, +1 NMS halo each side) are
//   staged in LDS once, in two copies offset by two bytes so that every lane's
//   8-byte window starts dword-aligned in one of them.  A lane scores two
//   adjacent pixels at once in packed 16-bit halves: per circle position one
//   v_perm builds the pixel pair, packed subtractions give the brighter /
//   darker sign bits, shifted into two 16-bit arc masks; the 9-contiguous test
//   is three rotate-and-ANDs (runs of 2, 4, 8) and one with the mask rotated
//   by 8 (equivalent to OpenCV's scan over 25 circle samples: a 9-run always
//   covers one of each opposite pair, so its early-outs never change the
//   result).  Corners (~2 % of pixels) are compacted into a per-wave list and
//   scored densely, one lane per corner (cornerScore's min / max arcs).  Then
//   the strict 3x3 NMS over the tile's score rows in LDS; the survivors of each
//   (row, tile) are appended in ascending x by ballot ranks to a slot of
//   kFtCap, with the row's count and the tile's total.
// fast_order_kernel — workgroup = band of kFtRows rows: its offset is the sum
//   of every earlier band's tile totals, an exclusive scan over its (row,
//   tile) counts places each slot, and the keypoints are copied out in
//   row-major, ascending-x order (cv::FAST's order).  The last band writes
//   the total.
// Every pixel is scored once (plus the one-pixel NMS ring of each tile), the
// image is read from L2 once per tile, and no step walks rows serially.
constexpr int kFtCols = 126;                 // output columns of a tile (lanes 0..62, 2 each)
#ifndef VISO_FT_ROWS
#define VISO_FT_ROWS 8
#endif
constexpr int kFtRows = VISO_FT_ROWS;        // output rows of a tile
constexpr int kFtSRows = kFtRows + 2;        // score rows (NMS halo)
constexpr int kFtPRows = kFtRows + 8;        // pixel rows (circle + NMS halo)
constexpr int kFtChunks = 17;                // 8-byte chunks of a staged row (136 bytes)
constexpr int kFtPStride = 8 * kFtChunks;
constexpr int kFtCap = 64;                   // keypoints per (row, tile): strict NMS keeps <= 63
constexpr int kFtList = 192;                 // corner list per wave (scored at >= 64)
constexpr int kFtMaxTx = (kMaxWidth + kFtCols - 1) / kFtCols;

constexpr int kCircleDx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
constexpr int kCircleDy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};

// cornerScore<16> (OpenCV fast_score.cpp) of a corner from dd[k] = v - circle[k]
__device__ inline int fast_corner_score(const int (&dd)[16], int thresh) {
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

// v_perm selector: window bytes m, m + 1 into the low bytes of the two halves
__device__ constexpr uint32_t ft_sel(int m) {
    return (uint32_t)m | (0x0cu << 8) | ((uint32_t)(m + 1) << 16) | (0x0cu << 24);
}

// rotate each 16-bit half right by s (circle positions k + s -> k)
template <int S>
__device__ inline u16x2 ft_rot(u16x2 m) {
    return (m >> (u16x2)S) | (m << (u16x2)(16 - S));
}

// 9 contiguous set bits anywhere on the 16-position circle, per half
__device__ inline u16x2 ft_run9(u16x2 m) {
    const u16x2 a1 = m & ft_rot<1>(m);
    const u16x2 a2 = a1 & ft_rot<2>(a1);
    const u16x2 a3 = a2 & ft_rot<4>(a2);
    return a3 & ft_rot<8>(m);
}

// (the body of fast_tile_kernel for tile (tx, ty); pyr1_fast_kernel runs it
// for its workgroups past the level-1 ones)
__device__ __forceinline__ void fast_tile_body(const uint8_t* __restrict__ img, int w, int h, int thresh, int ntx,
                                               int* __restrict__ cnt, int* __restrict__ tot,
                                               int* __restrict__ lst, const int tx, const int ty) {
    __shared__ __attribute__((aligned(16))) uint8_t s_pa[kFtPRows][kFtPStride];  // pixel index i at i
    __shared__ __attribute__((aligned(16))) uint8_t s_pb[kFtPRows][kFtPStride];  // pixel index i at i - 2
    __shared__ __attribute__((aligned(16))) uint8_t s_sc[kFtSRows][128];
    __shared__ uint16_t s_list[4][kFtList];
    __shared__ int s_tot;
    // output columns [ox, ox + 126), rows [oy, oy + kFtRows); score column j
    // is x = ox - 1 + j, score row r is y = oy - 1 + r; pixel index i is
    // x = ox - 4 + i, pixel row q is y = oy - 4 + q
    const int ox = tx * kFtCols, oy = ty * kFtRows;
    const int t = threadIdx.x, lane = t & 63, wave = wave_id();
    const long long npx = (long long)w * h;
    for (int i = t; i < 2 * kFtPRows * kFtChunks; i += 256) {
        const int cp = i >= kFtPRows * kFtChunks;
        const int k = i - (cp ? kFtPRows * kFtChunks : 0);
        const int q = k / kFtChunks, c = k - q * kFtChunks;
        const int y = oy - 4 + q;
        uint2 v = make_uint2(0u, 0u);
        // bytes outside [0, w) of a row are read but never used by a candidate
        if (y >= 0 && y < h) v = ps_load(img, (long long)y * w + (ox - 4 + 8 * c + 2 * cp), npx);
        *reinterpret_cast<uint2*>((cp ? s_pb[q] : s_pa[q]) + 8 * c) = v;
    }
    for (int i = t; i < kFtSRows * 32; i += 256) reinterpret_cast<uint32_t*>(&s_sc[0][0])[i] = 0u;
    if (t == 0) s_tot = 0;
    __syncthreads();

    // ---- corner test, two pixels (score columns 2l, 2l + 1) per lane
    const uint8_t* win = (lane & 1) ? &s_pb[0][2 * lane - 2] : &s_pa[0][2 * lane];
    const int x_lo = ox - 1 + 2 * lane;
    const bool ok_lo = x_lo >= 3 && x_lo < w - 3, ok_hi = x_lo + 1 >= 3 && x_lo + 1 < w - 3;
    const u16x2 T = (u16x2)(unsigned short)thresh;
    const unsigned long long lt = (1ull << lane) - 1ull;
    int nl = 0;  // wave-uniform list length
    auto score_list = [&](int first, int m) {
        __builtin_amdgcn_wave_barrier();
        if (lane < m) {
            const int e = s_list[wave][first + lane];
            const int r = e >> 8, j = e & 255;
            const uint8_t* cen = &s_pa[r + 3][j + 3];
            const int v = cen[0];
            int dd[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) dd[k] = v - (int)cen[kCircleDy[k] * kFtPStride + kCircleDx[k]];
            s_sc[r][j] = (uint8_t)fast_corner_score(dd, thresh);
        }
        __builtin_amdgcn_wave_barrier();
    };
    for (int r = wave; r < kFtSRows; r += 4) {
        const int y = oy - 1 + r;
        if (y < 3 || y >= h - 3) continue;  // wave-uniform: no candidate row
        uint32_t e0[7], e1[7];
#pragma unroll
        for (int d = 0; d < 7; ++d) {
            const uint32_t* p = reinterpret_cast<const uint32_t*>(win + (r + d) * kFtPStride);
            e0[d] = p[0];
            e1[d] = p[1];
        }
        const u16x2 V = as_u16x2(__builtin_amdgcn_perm(e1[3], e0[3], ft_sel(3)));
        const u16x2 VB = V + T, VD = V - T;  // wrapping; every difference below is within +-510
        u16x2 mb = (u16x2)0, md = (u16x2)0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int d = kCircleDy[k] + 3;
            const u16x2 C = as_u16x2(__builtin_amdgcn_perm(e1[d], e0[d], ft_sel(3 + kCircleDx[k])));
            const u16x2 db = VB - C;  // sign: brighter (C > v + t)
            const u16x2 dk = C - VD;  // sign: darker (C < v - t)
            mb = (mb >> (u16x2)1) | (db & (u16x2)0x8000);
            md = (md >> (u16x2)1) | (dk & (u16x2)0x8000);
        }
        const uint32_t run = __builtin_bit_cast(uint32_t, ft_run9(mb) | ft_run9(md));
        const bool c_lo = ok_lo && (run & 0xffffu) != 0u, c_hi = ok_hi && (run >> 16) != 0u;
        const unsigned long long b_lo = __ballot(c_lo), b_hi = __ballot(c_hi);
        if ((b_lo | b_hi) == 0ull) continue;
        const int n_lo = __popcll(b_lo);
        if (c_lo) s_list[wave][nl + __popcll(b_lo & lt)] = (uint16_t)((r << 8) | (2 * lane));
        if (c_hi) s_list[wave][nl + n_lo + __popcll(b_hi & lt)] = (uint16_t)((r << 8) | (2 * lane + 1));
        nl += n_lo + __popcll(b_hi);
        while (nl >= 64) {
            nl -= 64;
            score_list(nl, 64);
        }
    }
    if (nl > 0) score_list(0, nl);
    __syncthreads();

    // ---- strict 3x3 NMS on output rows 1..kFtRows, columns 2l + 1, 2l + 2
    int wave_total = 0;
    for (int r = 1 + wave; r <= kFtRows; r += 4) {
        const int y = oy + r - 1;
        if (y >= h) break;
        bool k0 = false, k1 = false;
        int s0 = 0, s1 = 0;
        if (lane < 63) {
            int sv[3][4];
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                const uint16_t* p = reinterpret_cast<const uint16_t*>(&s_sc[r - 1 + d][2 * lane]);
                const uint32_t a = p[0], b = p[1];
                sv[d][0] = a & 255;
                sv[d][1] = a >> 8;
                sv[d][2] = b & 255;
                sv[d][3] = b >> 8;
            }
            s0 = sv[1][1];
            s1 = sv[1][2];
            k0 = s0 > 0 && s0 > sv[1][0] && s0 > sv[1][2] && s0 > sv[0][0] && s0 > sv[0][1] && s0 > sv[0][2] &&
                 s0 > sv[2][0] && s0 > sv[2][1] && s0 > sv[2][2];
            k1 = s1 > 0 && s1 > sv[1][1] && s1 > sv[1][3] && s1 > sv[0][1] && s1 > sv[0][2] && s1 > sv[0][3] &&
                 s1 > sv[2][1] && s1 > sv[2][2] && s1 > sv[2][3];
        }
        const unsigned long long b0 = __ballot(k0), b1 = __ballot(k1);
        const int n = __popcll(b0) + __popcll(b1);
        const size_t e = (size_t)y * ntx + tx;
        const int rank = __popcll(b0 & lt) + __popcll(b1 & lt);
        if (k0) lst[e * kFtCap + rank] = (ox + 2 * lane) | (s0 << 16);
        if (k1) lst[e * kFtCap + rank + (k0 ? 1 : 0)] = (ox + 2 * lane + 1) | (s1 << 16);
        if (lane == 0) cnt[e] = n;
        wave_total += n;
    }
    if (lane == 0) atomicAdd(&s_tot, wave_total);
    __syncthreads();
    if (t == 0) tot[(size_t)ty * ntx + tx] = s_tot;
}

__global__ __launch_bounds__(256) void fast_tile_kernel(const uint8_t* __restrict__ img, int w, int h,
                                                        int thresh, int ntx, int* __restrict__ cnt,
                                                        int* __restrict__ tot, int* __restrict__ lst) {
    fast_tile_body(img, w, h, thresh, ntx, cnt, tot, lst, (int)blockIdx.x, (int)blockIdx.y);
}

// A one-image level-1 launch with the image's FAST tiles as extra
// workgroups (FastPre): workgroups [0, n_pyr) are pyr_down_sk_kernel's (its
// XCD-dealt 1-D form: n_pyr = 8 xcd_per), the rest FAST tiles in row-major
// order.  The two share nothing but the launch: level 1 and the tiles both
// only read level 0.
struct FastTileArgs {
    const uint8_t* img;
    int w, h, thresh, ntx;
    int* cnt;
    int* tot;
    int* lst;
};

template <int BH, int D>
__global__ __launch_bounds__(256) void pyr1_fast_kernel(PyrLevelArgs a, int n_pyr, FastTileArgs f) {
    const int b = (int)blockIdx.x;
    if (b < n_pyr) {
        pyr_down_sk_body<BH, D>(a, b, 0);
        return;
    }
    const int t = b - n_pyr;
    fast_tile_body(f.img, f.w, f.h, f.thresh, f.ntx, f.cnt, f.tot, f.lst, t % f.ntx, t / f.ntx);
}

__global__ __launch_bounds__(256) void fast_order_kernel(int h, int ntx, int nty, const int* __restrict__ cnt,
                                                         const int* __restrict__ tot,
                                                         const int* __restrict__ lst, int cap,
                                                         float2* __restrict__ kp_out,
                                                         int4* __restrict__ raw_out, int* __restrict__ n_out,
                                                         float2* __restrict__ kp_copy, int* host_n, int cap_n) {
    __shared__ int s_off[kFtRows * kFtMaxTx + 1];
    __shared__ int s_w[4], s_b[4];
    const int ty = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = wave_id();
    const int oy = ty * kFtRows;
    const int nr = min(kFtRows, h - oy);
    const int E = nr * ntx;  // (row, tile) slots of the band, row-major
    int acc = 0;
    for (int i = t; i < ty * ntx; i += 256) acc += tot[i];
    acc = wave_sum_int(acc);
    constexpr int kPer = (kFtRows * kFtMaxTx + 255) / 256;
    int c[kPer], sum = 0;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int e = kPer * t + k;
        c[k] = e < E ? cnt[(size_t)oy * ntx + e] : 0;
        sum += c[k];
    }
    int incl = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(incl, d);
        if (lane >= d) incl += o;
    }
    if (lane == 63) s_w[wave] = incl;
    if (lane == 0) s_b[wave] = acc;
    __syncthreads();
    int off = incl - sum;
    for (int k = 0; k < wave; ++k) off += s_w[k];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int e = kPer * t + k;
        if (e < E) s_off[e] = off;
        off += c[k];
    }
    const int total = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    const int base = s_b[0] + s_b[1] + s_b[2] + s_b[3];
    if (t == 0) s_off[E] = total;
    __syncthreads();
    for (int i = t; i < total; i += 256) {
        int lo = 0, hi = E;  // largest e with s_off[e] <= i
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (s_off[mid] <= i) lo = mid; else hi = mid;
        }
        const int o = base + i;
        if (o < cap) {
            const int rr = lo / ntx, tx = lo - rr * ntx;
            const int y = oy + rr;
            const int v = lst[((size_t)y * ntx + tx) * kFtCap + (i - s_off[lo])];
            const int x = v & 0xffff, sc = v >> 16;
            if (kp_out) kp_out[o] = make_float2((float)x, (float)y);
            if (kp_copy) kp_copy[o] = make_float2((float)x, (float)y);
            if (raw_out) raw_out[o] = make_int4(x, y, sc, 0);
        }
    }
    if (ty == nty - 1 && t == 0) {
        const int n = cap_n ? min(base + total, cap) : base + total;
        *n_out = n;
        // the pinned host copy: a system-scope store, visible to the host
        // once the launch has completed (FastDetect)
        if (host_n) __hip_atomic_store(host_n, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Tail-launch plan for n images of a geometry; false (level 1 narrower than
// 8 columns) = per-level launches.  The band height starts from the one that
// fills kPfSlots once and shrinks until the staged rows fit the per-thread
// load slots and the LDS budget (B = 2 fits any level 0 up to kMaxWidth).
bool pf_plan(const PyrGeom& g, int n, PyrTailArgs& a, size_t& lds) {
    static_assert(kLevels == 4, "pyramid tail: levels 2..3");
    if (g.w[1] < 8 || g.w[3] < 1 || g.h[3] < 1) return false;
    a.w1 = g.w[1];
    a.h1 = g.h[1];
    a.w2 = g.w[2];
    a.h2 = g.h[2];
    a.w3 = g.w[3];
    a.h3 = g.h[3];
    a.off1 = g.off[1];
    a.off2 = g.off[2];
    a.off3 = g.off[3];
    // a staged row holds its pads, the dword writes of every group of its
    // level and the 16-byte tap reads of every group of the next level
    auto stride = [](int w, int g_self, int g_next) {
        const int s = std::max(kPfPad + w + 2, std::max(kPfPad + 4 * g_self, kPfPad + 8 * g_next + 4));
        return (s + 15) & ~15;
    };
    a.s1 = std::max(stride(a.w1, 0, (a.w2 + 3) / 4), (kPfPad + 16 * ((a.w1 + 15) / 16) + 15) & ~15);
    a.s2 = stride(a.w2, (a.w2 + 3) / 4, (a.w3 + 3) / 4);
    const int nb_target = std::max(1, kPfSlots / std::max(n, 1));
    for (a.band = std::max(2, (g.h[3] + nb_target - 1) / nb_target);; --a.band) {
        a.nb = (g.h[3] + a.band - 1) / a.band;
        int r1 = 0, r2 = 0;
        for (int b = 0; b < a.nb; ++b) {
            const PfBand r = pf_band(b, a.nb, a.band, a.h1, a.h2, a.h3);
            r1 = std::max(r1, r.c1b - r.c1a);
            r2 = std::max(r2, r.c2b - r.c2a);
        }
        a.lds1 = r2 * a.s2;
        lds = (size_t)a.lds1 + (size_t)r1 * a.s1;
        const bool fits = (size_t)r1 * ((a.w1 + 15) / 16) <= (size_t)kPfStage1 * kPfThreads && lds <= kPfLdsMax;
        if (fits) return true;
        if (a.band == 1) return false;
    }
}

// one per-level launch (level l from level l-1) over nb images: the
// register-only streaming form for level 1 at least 8 columns wide, the
// LDS-staged form for the tiny levels of images the tail does not take
void fast_dims(int w, int h, int* ntx, int* nty) {
    *ntx = (w + kFtCols - 1) / kFtCols;
    *nty = (h + kFtRows - 1) / kFtRows;
}

void launch_pyr_level(const PyrGeom& g, int l, const uint8_t* const* l0, uint8_t* const* slot, int nb,
                      hipStream_t stream, FastPre* fp = nullptr) {
    PyrLevelArgs a;
    for (int i = 0; i < nb; ++i) {
        a.src[i] = l == 1 ? l0[i] : slot[i] + g.off[l - 1];
        a.dst[i] = slot[i] + g.off[l];
    }
    a.sw = g.w[l - 1];
    a.sh = g.h[l - 1];
    a.dw = g.w[l];
    a.dh = g.h[l];
    if (l == 1 && a.sw >= 8) {
        const bool small = nb <= kSkSmallBatch;
        const int bh = small ? kSkBHs : kSkBH1;
        a.bands = (a.dh + bh - 1) / bh;
        a.units = a.bands * ((a.dw + kSkW - 1) / kSkW);
        a.bpi = (a.units + 3) / 4;
        a.n_img = nb;
        a.xcd_per = (a.bpi * nb + 7) / 8;
        if (fp && nb == 1 && small) {
            FastTileArgs f{fp->img, fp->w, fp->h, fp->thresh < 0 ? 0 : (fp->thresh > 255 ? 255 : fp->thresh), 0,
                           fp->s.cnt, fp->s.tot, fp->s.lst};
            int nty;
            fast_dims(fp->w, fp->h, &f.ntx, &nty);
            pyr1_fast_kernel<kSkBHs, kSkRings><<<8 * a.xcd_per + f.ntx * nty, 256, 0, stream>>>(a, 8 * a.xcd_per, f);
            fp->done = true;
            return;
        }
        if (small)
            pyr_down_sk_kernel<kSkBHs, kSkRings><<<8 * a.xcd_per, 256, 0, stream>>>(a);
        else
            pyr_down_sk_kernel<kSkBH1, kSkRing1><<<8 * a.xcd_per, 256, 0, stream>>>(a);
        return;
    }
    const int bh = l == 1 ? 8 : (l == 2 ? 4 : 2);
    a.bands = (a.dh + bh - 1) / bh;
    a.units = a.bands * ((a.dw + kPsW - 1) / kPsW);
    a.xcd_per = 0;
    const dim3 grid((a.units + 3) / 4, nb);
    if (l == 1)
        pyr_down_stream_kernel<8><<<grid, 256, 0, stream>>>(a);
    else if (l == 2)
        pyr_down_stream_kernel<4><<<grid, 256, 0, stream>>>(a);
    else
        pyr_down_stream_kernel<2><<<grid, 256, 0, stream>>>(a);
}

}  // namespace

void launch_pyramid_frames(const PyrGeom& g, const uint8_t* const* l0, uint8_t* const* slot,
                           int n, hipStream_t stream, PyrOwn* own) {
    const size_t len0 = (size_t)g.w[0] * g.h[0];
    for (int b0 = 0; b0 < n; b0 += kPyrBatch) {
        const int nb = (n - b0) < kPyrBatch ? (n - b0) : kPyrBatch;
        // this launch's image of `own`, or -1
        const int oi = own && own->img >= b0 && own->img < b0 + nb ? own->img - b0 : -1;
        bool copy = oi >= 0 && l0[b0 + oi] != slot[b0 + oi];
        launch_pyr_level(g, 1, l0 + b0, slot + b0, nb, stream, own && n == 1 ? own->fast : nullptr);
        PyrTailArgs ta;
        size_t lds = 0;
        if (pf_plan(g, nb, ta, lds)) {
            // the copy fits the image's bands' chunk slots (small batches:
            // many bands per image), else it stays the caller's
            copy = copy && (len0 >> 4) <= (size_t)ta.nb * kPfThreads * kPfOwnPer;
            if (oi >= 0) own->copied = copy;
            for (int i = 0; i < nb; ++i) ta.slot[i] = slot[b0 + i];
            ta.n = nb;
            ta.xcd_map = nb >= 8;
            ta.own_img = oi;
            ta.own_src = copy ? l0[b0 + oi] : nullptr;
            ta.own_len = (int)len0;
            ta.ident_pose = oi >= 0 ? own->ident_pose : nullptr;
            const bool last = b0 + nb >= n;  // the words: once, with the last launch
            ta.zero = own && last ? own->zero : nullptr;
            ta.n_zero = own && last && own->zero ? own->n_zero : 0;
            const int grid = ta.xcd_map ? 8 * ta.nb * ((nb + 7) / 8) : ta.nb * nb;
            pyr_tail_kernel<<<grid, kPfThreads, lds, stream>>>(ta);
        } else {
            launch_pyr_level(g, 2, l0 + b0, slot + b0, nb, stream);
            launch_pyr_level(g, 3, l0 + b0, slot + b0, nb, stream);
            if (oi >= 0 && own->ident_pose) {
                const double ident[12] = {1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0};
                launch_set_pose(own->ident_pose, ident, stream);
            }
            if (copy)
                (void)hipMemcpyAsync(slot[b0 + oi], l0[b0 + oi], len0, hipMemcpyDeviceToDevice, stream);
            if (oi >= 0) own->copied = copy;
            if (own && own->zero && b0 + nb >= n)
                (void)hipMemsetAsync(own->zero, 0, sizeof(int) * (size_t)own->n_zero, stream);
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


size_t fast_scratch_bytes(int w, int h) {
    int ntx, nty;
    fast_dims(w, h, &ntx, &nty);
    const size_t slots = (size_t)h * ntx;
    return ((sizeof(int) * (slots + (size_t)nty * ntx) + 255) & ~(size_t)255) + sizeof(int) * slots * kFtCap;
}

FastScratch fast_scratch_at(void* base, int w, int h) {
    int ntx, nty;
    fast_dims(w, h, &ntx, &nty);
    const size_t slots = (size_t)h * ntx;
    FastScratch s;
    s.cnt = (int*)base;
    s.tot = s.cnt + slots;
    s.lst = (int*)((char*)base + ((sizeof(int) * (slots + (size_t)nty * ntx) + 255) & ~(size_t)255));
    return s;
}

void launch_fast(const uint8_t* img, int w, int h, int thresh, FastScratch& s, float2* kp_out,
                 int4* raw_out, int cap, int* n_out, hipStream_t stream, const FastDetect* det, bool tiles_done) {
    int ntx, nty;
    fast_dims(w, h, &ntx, &nty);
    thresh = thresh < 0 ? 0 : (thresh > 255 ? 255 : thresh);
    // (tiles_done: the ingest's level-1 launch ran them, FastPre)
    if (!tiles_done)
        fast_tile_kernel<<<dim3(ntx, nty), 256, 0, stream>>>(img, w, h, thresh, ntx, s.cnt, s.tot, s.lst);
    fast_order_kernel<<<nty, 256, 0, stream>>>(h, ntx, nty, s.cnt, s.tot, s.lst, cap, kp_out, raw_out, n_out,
                                               det ? det->kp_copy : nullptr, det ? det->host_n : nullptr,
                                               det ? 1 : 0);
}

}  // namespace viso

#ifdef VISO_PROBE
extern "C" int viso_debug_pyr_timeline(unsigned long long* out, int n) {
    if (n > 8192) n = 8192;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pyr_tl), sizeof(unsigned long long) * 5 * n) ==
                   hipSuccess ? 0 : -2;
}
#endif
