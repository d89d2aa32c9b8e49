// viso_amd — shared definitions for the gfx950 kernels and the host context.
//
// Numerics contract: fp64 everywhere the reference is
// fp64, operand order as in the reference source, compiled with
// -ffp-contract=off; every sum over patch pixels or points is the canonical
// pairwise tree (xor-butterfly with ascending offsets on a wave64), so the
// device reproduces the CPU oracle bit for bit.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <cstdio>

namespace viso {

constexpr int kLevels = 4;
constexpr int kHalfPatch = 4;    // include/viso.h:25
constexpr int kPatch = 64;       // (2*4)^2 pixels, one per wave64 lane
constexpr int kMaxWidth = 4096;  // FAST row kernel LDS bound

struct PyrGeom {
    int w[kLevels], h[kLevels];
    size_t off[kLevels];
    size_t bytes;  // all levels
    size_t slot;   // bytes per frame slot (bytes rounded up to 256)
};

inline PyrGeom make_geom(int w, int h) {
    PyrGeom g{};
    size_t off = 0;
    for (int l = 0; l < kLevels; ++l) {
        if (l > 0) {
            w = (int)(w * 0.5);  // include/keyframe.h:43 (truncating Size(cols*0.5, rows*0.5))
            h = (int)(h * 0.5);
        }
        g.w[l] = w;
        g.h[l] = h;
        g.off[l] = off;
        off += (size_t)w * (size_t)h;
    }
    g.bytes = off;
    g.slot = (off + 255) & ~(size_t)255;
    return g;
}

// One frame's pyramid as per-level pointers.  Level 0 may live in the
// caller's device buffer (batched ingest) while levels 1..3 live in a frame
// slot of the context; every level is continuous (step == width).
struct FrameDev {
    const uint8_t* l[kLevels];
};

inline FrameDev frame_from_base(const uint8_t* base, const PyrGeom& g) {
    FrameDev f;
    for (int i = 0; i < kLevels; ++i) f.l[i] = base + g.off[i];
    return f;
}

// Pose: R row-major + t (Tcw: Pc = R*Pw + t, include/keyframe.h:84)
struct Pose12 {
    double v[12];
};

__host__ __device__ inline void mat3_vec(const double* R, const double* p, double* o) {
    o[0] = R[0] * p[0] + R[1] * p[1] + R[2] * p[2];
    o[1] = R[3] * p[0] + R[4] * p[1] + R[5] * p[2];
    o[2] = R[6] * p[0] + R[7] * p[1] + R[8] * p[2];
}

// Loads through explicit address spaces.  Image pointers often reach a
// kernel through a run-time-indexed kernel-argument array (a frame of a
// batch, a pyramid level), where the compiler can no longer prove they are
// global and would emit flat loads (which also count in lgkmcnt and get
// drained one by one); LDS windows passed as plain pointers likewise.
__device__ inline uint8_t ld_global_u8(const uint8_t* p, long long i) {
    return ((const __attribute__((address_space(1))) uint8_t*)p)[i];
}
// Byte at a wave-uniform base + a 32-bit unsigned per-lane offset (the
// global_load saddr form: no 64-bit address arithmetic per lane).
__device__ inline uint8_t ld_global_u8_off(const uint8_t* base, uint32_t off) {
    return ((const __attribute__((address_space(1))) uint8_t*)base)[off];
}
// Byte i of a buffer of n bytes, 0 outside it.  The load is unconditional
// (index clamped, value selected): a conditional load compiles to a branch
// with its own s_waitcnt, which serialises a lane's taps.
__device__ inline int ld_u8_or0(const uint8_t* p, long long n, long long i) {
    const bool in = i >= 0 && i < n;
    const int v = ld_global_u8(p, in ? i : 0);
    return in ? v : 0;
}
__device__ inline uint8_t ld_lds_u8(const uint8_t* p, int i) {
    return ((const __attribute__((address_space(3))) uint8_t*)p)[i];
}
__device__ inline void st_lds_u8(uint8_t* p, int i, uint8_t v) {
    ((__attribute__((address_space(3))) uint8_t*)p)[i] = v;
}

// GetPixelValue (include/common.h:35-42): int() base, floor() weights,
// taps outside the continuous level buffer read 0.
__device__ inline double sample_px(const uint8_t* __restrict__ img, int w, int h, double x,
                                   double y) {
    const long long n = (long long)w * (long long)h;
    const bool finite = (x > -1e9 && x < 1e9 && y > -1e9 && y < 1e9);
    long long base = finite ? (long long)(int)y * (long long)w + (long long)(int)x : -(1LL << 40);
    double d0 = (double)ld_u8_or0(img, n, base);
    double d1 = (double)ld_u8_or0(img, n, base + 1);
    double d2 = (double)ld_u8_or0(img, n, base + w);
    double d3 = (double)ld_u8_or0(img, n, base + w + 1);
    double xx = x - floor(x);
    double yy = y - floor(y);
    return double((1 - xx) * (1 - yy) * d0 + xx * (1 - yy) * d1 + (1 - xx) * yy * d2 +
                  xx * yy * d3);
}

__device__ inline void gradient_px(const uint8_t* __restrict__ img, int w, int h, double u,
                                   double v, double& gx, double& gy) {
    gx = 0.5 * (sample_px(img, w, h, u + 1, v) - sample_px(img, w, h, u - 1, v));
    gy = 0.5 * (sample_px(img, w, h, u, v + 1) - sample_px(img, w, h, u, v - 1));
}

// Canonical pairwise tree over the 64 lanes of a wave: ascending xor offsets.
// Every lane ends with the same bits (a + b == b + a in IEEE arithmetic).
__device__ inline double wave_tree_sum(double v) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) v = v + __shfl_xor(v, off, 64);
    return v;
}

// DPP move of both halves of a double (all 64 lanes must be active).  Lanes
// without a source lane read 0 (bound_ctrl), so no "old" value has to be
// materialised first.
template <int CTRL>
__device__ inline double dpp_f64(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffffLL), CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// This thread's wave in the workgroup, visibly wave-uniform to the compiler
// (so values indexed by it stay scalar and branches on them need no EXEC
// bookkeeping).
__device__ inline int wave_id() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }

// A wave-uniform value made visibly uniform to the compiler (exact: every
// lane holds the same bits), so branches on it need no EXEC bookkeeping.
__device__ inline double uniform_f64(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readfirstlane((int)(b & 0xffffffffLL));
    const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ inline double readlane_f64(double v, int lane) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), lane);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// gfx950 v_permlane16_swap / v_permlane32_swap on both halves of a double:
// with both operands = v, lane l receives v[l ^ 16] (v[l ^ 32]) in one of the
// two results and its own row's value in the other.
__device__ inline void permlane16_swap_f64(double a, double b, double& ra, double& rb) {
    const long long x = __double_as_longlong(a), y = __double_as_longlong(b);
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)(x & 0xffffffffLL),
                                                     (unsigned)(y & 0xffffffffLL), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(x >> 32), (unsigned)(y >> 32), false,
                                                     false);
    ra = __longlong_as_double(((long long)hi[0] << 32) | lo[0]);
    rb = __longlong_as_double(((long long)hi[1] << 32) | lo[1]);
}

__device__ inline void permlane32_swap_f64(double a, double b, double& ra, double& rb) {
    const long long x = __double_as_longlong(a), y = __double_as_longlong(b);
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)(x & 0xffffffffLL),
                                                     (unsigned)(y & 0xffffffffLL), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(x >> 32), (unsigned)(y >> 32), false,
                                                     false);
    ra = __longlong_as_double(((long long)hi[0] << 32) | lo[0]);
    rb = __longlong_as_double(((long long)hi[1] << 32) | lo[1]);
}

// The same canonical tree as wave_tree_sum, built from DPP row operations:
// xor-1 and xor-2 by quad_perm; then, because every lane of an aligned 4-
// (8-) group already holds the same partial, row_half_mirror (row_mirror)
// pairs each group with its sibling exactly like xor-4 (xor-8); the last two
// levels pair rows with v_permlane16_swap (row r with r ^ 1) and the wave
// halves with v_permlane32_swap: (r0 + r1) + (r2 + r3).  Every lane ends
// with the sum.  Requires EXEC = all 64 lanes.
__device__ inline double wave_tree_sum_dpp(double v) {
    v = v + dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]  (xor 1)
    v = v + dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]  (xor 2)
    v = v + dpp_f64<0x141>(v);  // row_half_mirror      (xor 4 on uniform quads)
    v = v + dpp_f64<0x140>(v);  // row_mirror           (xor 8 on uniform octets)
    double a, b;
    permlane16_swap_f64(v, v, a, b);  // rows (0,1) and (2,3): a + b = r_even + r_odd
    v = a + b;
    permlane32_swap_f64(v, v, a, b);  // halves: (r0 + r1) + (r2 + r3)
    return a + b;
}

__device__ inline double dsel(bool c, double a, double b) { return c ? a : b; }

// The canonical wave trees of three values at once: reduce-scatter over the
// xor-1 / xor-2 levels (lane class (b1, b0) = (0,0) / (0,1) / (1,0) keeps a /
// b / c, (1,1) a zero), then true xor-4 / xor-8 partners (DPP row_shr /
// row_shl by 4 / 8 + select) and the permlane16 / permlane32 swaps.  Every
// partial sum is the one wave_tree_sum_dpp forms (f64 + is commutative), so
// the results are bit-identical, at about half the instructions of three
// separate trees.  Results read from lanes 0, 1, 2.  Requires EXEC = all lanes.
__device__ inline void wave_tree_sum3(double a, double b, double c, double& ra, double& rb, double& rc) {
    const int lane = threadIdx.x & 63;
    const bool b0 = lane & 1, b1 = lane & 2, b2 = lane & 4, b3 = lane & 8;
    const double p = (b0 ? b : a) + dpp_f64<0xB1>(b0 ? a : b);      // even: a pairs, odd: b pairs
    const double q = (b0 ? 0.0 : c) + dpp_f64<0xB1>(b0 ? c : 0.0);  // even: c pairs, odd: 0
    double v = (b1 ? q : p) + dpp_f64<0x4E>(b1 ? p : q);
    // both DPP moves are evaluated by every lane (a conditional DPP would run
    // under a partial EXEC and read inactive lanes), then selected
    const double r4 = dpp_f64<0x114>(v), l4 = dpp_f64<0x104>(v);  // row_shr / row_shl by 4
    v = v + dsel(b2, r4, l4);                                        // lane ^ 4
    v = v + dpp_f64<0x128>(v);  // lane ^ 8 (row_ror:8 is exactly the xor-8 partner)
    double x, y;
    permlane16_swap_f64(v, v, x, y);
    v = x + y;
    permlane32_swap_f64(v, v, x, y);
    v = x + y;
    ra = readlane_f64(v, 0);
    rb = readlane_f64(v, 1);
    rc = readlane_f64(v, 2);
}

// LK alignment's three per-iteration sums (round 3): the descending-stride
// pairwise tree (pixels p and p + 32 first; oracle tree_sum_desc64).  xor 32
// pairs a (lanes < 32) and b (lanes >= 32) with one v_permlane32_swap and c
// everywhere with another; xor 16 keeps a / b in even rows and c in odd rows;
// then xor 8 / 4 by DPP row_ror (xor 8 exactly; xor 4 because the xor-8
// level leaves lanes l and l ^ 8 equal) and xor 2 / 1 by quad_perm.
// Results read from lanes 0 (a), 32 (b), 16 (c).  Requires EXEC = all lanes.
__device__ inline void wave_tree_sum3_desc(double a, double b, double c, double& ra, double& rb, double& rc) {
    const int lane = threadIdx.x & 63;
    const bool b2 = lane & 4, b3 = lane & 8;
    double x, y;
    permlane32_swap_f64(a, b, x, y);
    const double ab = x + y;
    permlane32_swap_f64(c, c, x, y);
    const double cc = x + y;
    permlane16_swap_f64(ab, cc, x, y);
    double v = x + y;
    v = v + dpp_f64<0x128>(v);  // lane ^ 8: row_ror:8 is exactly the xor-8 partner
    // lane ^ 4: lanes l and l ^ 8 now hold the same sum, so row_ror:4 (lane
    // (l - 4) mod 16, i.e. l ^ 4 or its xor-8 twin) delivers the xor-4 partner's
    v = v + dpp_f64<0x124>(v);
    v = v + dpp_f64<0x4E>(v);                                        // lane ^ 2
    v = v + dpp_f64<0xB1>(v);                                        // lane ^ 1
    ra = readlane_f64(v, 0);
    rb = readlane_f64(v, 32);
    rc = readlane_f64(v, 16);
}

// 28 canonical wave trees at once by reduce-scatter: at butterfly level s
// (partner lane ^ 2^s, ascending) every lane keeps half of its remaining
// values and adds the partner's copy of that half, so each value's partial
// sums follow exactly the ascending-xor tree of wave_tree_sum.  Partners:
// xor 1/2 by DPP quad_perm; xor 4/8 by DPP row_shl/row_shr + select; xor 16
// and xor 32 by v_permlane16_swap / v_permlane32_swap.  On return, lane l (and l^32)
// holds value index 14*b0 + 7*b1 + 4*b2 + 2*b3 + b4 (b = bits of l) when
// 4*b2 + 2*b3 + b4 < 7; the other 4 lane classes hold garbage.

template <int CTRL>
__device__ inline double dpp_or0(double v) {
    return dpp_f64<CTRL>(v);
}

__device__ inline double swizzle_xor16_f64(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_ds_swizzle((int)(b & 0xffffffffLL), 0x401F);
    const int hi = __builtin_amdgcn_ds_swizzle((int)(b >> 32), 0x401F);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ inline double reduce_scatter_28(const double* v, int* value_index) {
    const int lane = threadIdx.x & 63;
    const bool b0 = lane & 1, b1 = lane & 2, b2 = lane & 4, b3 = lane & 8, b4 = lane & 16;
    double a[14];
#pragma unroll
    for (int k = 0; k < 14; ++k) {
        const double send = dsel(b0, v[k], v[14 + k]);
        const double keep = dsel(b0, v[14 + k], v[k]);
        a[k] = keep + dpp_f64<0xB1>(send);
    }
    double c[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        const double send = dsel(b1, a[k], a[7 + k]);
        const double keep = dsel(b1, a[7 + k], a[k]);
        c[k] = keep + dpp_f64<0x4E>(send);
    }
    double d[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const double hi = k < 3 ? c[4 + k] : 0.0;
        const double send = dsel(b2, c[k], hi);
        const double keep = dsel(b2, hi, c[k]);
        const double recv = dsel(b2, dpp_f64<0x114>(send), dpp_f64<0x104>(send));  // row_shr:4 / row_shl:4
        d[k] = keep + recv;
    }
    double e[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const double send = dsel(b3, d[k], d[2 + k]);
        const double keep = dsel(b3, d[2 + k], d[k]);
        const double recv = dpp_f64<0x128>(send);  // row_ror:8 = the xor-8 partner
        e[k] = keep + recv;
    }
    // xor 16: row pairs (0,1), (2,3); even rows keep e[0], odd rows e[1]
    double ra, rb;
    permlane16_swap_f64(e[0], e[1], ra, rb);
    double f = ra + rb;
    // xor 32: the two wave halves
    permlane32_swap_f64(f, f, ra, rb);
    f = ra + rb;
    *value_index = (b0 ? 14 : 0) + (b1 ? 7 : 0) + (b2 ? 4 : 0) + (b3 ? 2 : 0) + (b4 ? 1 : 0);
    const int local = (b2 ? 4 : 0) + (b3 ? 2 : 0) + (b4 ? 1 : 0);
    if (local >= 7) *value_index = -1;
    return f;
}

// The direct pose's 28 patch-pixel sums (round 3): the same reduce-scatter
// with the butterfly levels in DESCENDING xor order (partner lane ^ 32, ^ 16,
// ^ 8, ^ 4, ^ 2, ^ 1), i.e. the pairwise tree that adds pixels p and p + 32
// first (oracle_common.hpp tree_sum_desc64).  The first two levels are then
// v_permlane32_swap / v_permlane16_swap of two values, which leave each lane
// its own and its partner's copy of the half it keeps with no selects: ~3
// instructions per pair instead of ~7.  On return lane l holds value index
// 14*b5 + 7*b4 + 4*b3 + 2*b2 + b1 (b = bits of l) when 4*b3 + 2*b2 + b1 < 7
// and b0 == 0 (lane l ^ 1 holds a copy; *value_index = -1 there and in the
// padded class).
__device__ inline double reduce_scatter_28_desc(const double* v, int* value_index) {
    const int lane = threadIdx.x & 63;
    const bool b0 = lane & 1, b1 = lane & 2, b2 = lane & 4, b3 = lane & 8, b4 = lane & 16, b5 = lane & 32;
    double a[14];
#pragma unroll
    for (int k = 0; k < 14; ++k) {  // xor 32: halves keep k / 14 + k
        double ra, rb;
        permlane32_swap_f64(v[k], v[14 + k], ra, rb);
        a[k] = ra + rb;
    }
    double c[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) {  // xor 16: even / odd rows keep k / 7 + k
        double ra, rb;
        permlane16_swap_f64(a[k], a[7 + k], ra, rb);
        c[k] = ra + rb;
    }
    double d[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // xor 8 (row_shr / row_shl by 8): 7 -> 4 (slot 7 a +0 pad)
        const double hi = k < 3 ? c[4 + k] : 0.0;
        const double send = dsel(b3, c[k], hi);
        const double keep = dsel(b3, hi, c[k]);
        const double recv = dpp_f64<0x128>(send);  // row_ror:8 = the xor-8 partner
        d[k] = keep + recv;
    }
    double e[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {  // xor 4 (row_shr / row_shl by 4)
        const double send = dsel(b2, d[k], d[2 + k]);
        const double keep = dsel(b2, d[2 + k], d[k]);
        const double recv = dsel(b2, dpp_f64<0x114>(send), dpp_f64<0x104>(send));
        e[k] = keep + recv;
    }
    // xor 2 (quad_perm [2,3,0,1])
    const double send = dsel(b1, e[0], e[1]);
    const double keep = dsel(b1, e[1], e[0]);
    double f = keep + dpp_f64<0x4E>(send);
    // xor 1 (quad_perm [1,0,3,2]): both lanes of the pair end with the sum
    f = f + dpp_f64<0xB1>(f);
    const int local = (b3 ? 4 : 0) + (b2 ? 2 : 0) + (b1 ? 1 : 0);
    *value_index = (b0 || local >= 7) ? -1 : (b5 ? 14 : 0) + (b4 ? 7 : 0) + local;
    return f;
}

// ---- fp32 forms (tolerance mode, VISO_PRECISION_FAST)
template <int CTRL>
__device__ inline float dpp_f32(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}

__device__ inline void permlane16_swap_f32(float a, float b, float& ra, float& rb) {
    const auto r = __builtin_amdgcn_permlane16_swap((unsigned)__float_as_int(a), (unsigned)__float_as_int(b),
                                                    false, false);
    ra = __int_as_float((int)r[0]);
    rb = __int_as_float((int)r[1]);
}

__device__ inline void permlane32_swap_f32(float a, float b, float& ra, float& rb) {
    const auto r = __builtin_amdgcn_permlane32_swap((unsigned)__float_as_int(a), (unsigned)__float_as_int(b),
                                                    false, false);
    ra = __int_as_float((int)r[0]);
    rb = __int_as_float((int)r[1]);
}

// reduce_scatter_28 on fp32 values (same butterfly and lane -> index map).
__device__ inline float reduce_scatter_28_f32(const float* v, int* value_index) {
    const int lane = threadIdx.x & 63;
    const bool b0 = lane & 1, b1 = lane & 2, b2 = lane & 4, b3 = lane & 8, b4 = lane & 16;
    float a[14];
#pragma unroll
    for (int k = 0; k < 14; ++k) {
        const float send = b0 ? v[k] : v[14 + k];
        const float keep = b0 ? v[14 + k] : v[k];
        a[k] = keep + dpp_f32<0xB1>(send);
    }
    float c[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        const float send = b1 ? a[k] : a[7 + k];
        const float keep = b1 ? a[7 + k] : a[k];
        c[k] = keep + dpp_f32<0x4E>(send);
    }
    float d[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float hi = k < 3 ? c[4 + k] : 0.0f;
        const float send = b2 ? c[k] : hi;
        const float keep = b2 ? hi : c[k];
        // both DPP moves evaluated by every lane, then selected (a DPP under a
        // partial EXEC would read inactive lanes)
        const float r4 = dpp_f32<0x114>(send), l4 = dpp_f32<0x104>(send);
        const float recv = b2 ? r4 : l4;
        d[k] = keep + recv;
    }
    float e[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const float send = b3 ? d[k] : d[2 + k];
        const float keep = b3 ? d[2 + k] : d[k];
        e[k] = keep + dpp_f32<0x128>(send);  // row_ror:8 = the xor-8 partner
    }
    float ra, rb;
    permlane16_swap_f32(e[0], e[1], ra, rb);
    float f = ra + rb;
    permlane32_swap_f32(f, f, ra, rb);
    f = ra + rb;
    *value_index = (b0 ? 14 : 0) + (b1 ? 7 : 0) + (b2 ? 4 : 0) + (b3 ? 2 : 0) + (b4 ? 1 : 0);
    const int local = (b2 ? 4 : 0) + (b3 ? 2 : 0) + (b4 ? 1 : 0);
    if (local >= 7) *value_index = -1;
    return f;
}

// wave_tree_sum3 on fp32 values (same butterfly; results of lanes 0, 1, 2).
__device__ inline void wave_tree_sum3_f32(float a, float b, float c, float& ra, float& rb, float& rc) {
    const int lane = threadIdx.x & 63;
    const bool b0 = lane & 1, b1 = lane & 2, b2 = lane & 4, b3 = lane & 8;
    const float p = (b0 ? b : a) + dpp_f32<0xB1>(b0 ? a : b);
    const float q = (b0 ? 0.0f : c) + dpp_f32<0xB1>(b0 ? c : 0.0f);
    float v = (b1 ? q : p) + dpp_f32<0x4E>(b1 ? p : q);
    const float r4 = dpp_f32<0x114>(v), l4 = dpp_f32<0x104>(v);
    v = v + (b2 ? r4 : l4);
    v = v + dpp_f32<0x128>(v);  // row_ror:8 = the xor-8 partner
    float x, y;
    permlane16_swap_f32(v, v, x, y);
    v = x + y;
    permlane32_swap_f32(v, v, x, y);
    v = x + y;
    ra = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    rb = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 1));
    rc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 2));
}

// Tolerance-mode form of wave_tree_sum3_desc on fp32 values (LK): same
// butterflies, results from lanes 0, 32, 16; no parity constraint beyond the
// mode's tolerance.  (The same form of reduce_scatter_28 measured no faster
// in the direct point sums: 44.8 vs 44.7 us per frame.)
__device__ inline void wave_tree_sum3_f32_desc(float a, float b, float c, float& ra, float& rb, float& rc) {
    const int lane = threadIdx.x & 63;
    const bool b2 = lane & 4, b3 = lane & 8;
    float x, y;
    permlane32_swap_f32(a, b, x, y);
    const float ab = x + y;
    permlane32_swap_f32(c, c, x, y);
    const float cc = x + y;
    permlane16_swap_f32(ab, cc, x, y);
    float v = x + y;
    v = v + dpp_f32<0x128>(v);  // lane ^ 8 (row_ror:8)
    v = v + dpp_f32<0x124>(v);  // lane ^ 4 (row_ror:4 after the duplicated xor-8 level)
    v = v + dpp_f32<0x4E>(v);
    v = v + dpp_f32<0xB1>(v);
    ra = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    rb = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    rc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
}

// fp32 bilinear with weights (xx, yy) of taps a (x, y), b (x + 1, y),
// c (x, y + 1), d (x + 1, y + 1).
__device__ inline float bilerp_f32(float a, float b, float c, float d, float xx, float yy) {
    const float top = __builtin_fmaf(xx, b - a, a);
    const float bot = __builtin_fmaf(xx, d - c, c);
    return __builtin_fmaf(yy, bot - top, top);
}

__device__ inline int wave_sum_int(int v) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// counter-based RNG of the RANSAC samplers (identical to the oracle's)
__host__ __device__ inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

}  // namespace viso

#define VISO_HIP_CHECK(expr)                                                              \
    do {                                                                                  \
        hipError_t _e = (expr);                                                           \
        if (_e != hipSuccess) {                                                           \
            std::fprintf(stderr, "viso_amd: HIP error %s at %s:%d: %s\n", hipGetErrorName(_e), \
                         __FILE__, __LINE__, #expr);                                      \
            return VISO_ERR_HIP;                                                          \
        }                                                                                 \
    } while (0)
