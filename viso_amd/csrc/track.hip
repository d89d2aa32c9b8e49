// viso_amd — per-point Lucas-Kanade engines for gfx950.
//
//  * klt_kernel: OpticalFlowMultiLevel(ref, cur, kp1, kp2, success,
//    inverse=true) (src/viso.cpp:353-391) with OpticalFlowSingleLevel
//    (:259-350) inside, all four levels in one launch.
//  * lk_align_kernel: LKAlignment + LKAlignmentSingle (src/viso.cpp:768-925):
//    best-viewing-angle keyframe selection, then four levels of <= 100
//    inverse-compositional iterations per pair.
//
// Mapping: one wave64 per point, lane p = one pixel of the 8x8 patch
// (p = (x+4)*8 + (y+4), the reference's x-outer / y-inner order).  Because
// the Jacobian is taken on the reference image (inverse compositional), the
// per-lane template value, gradient and the 2x2 Hessian are computed once per
// level; each GN iteration is one bilinear sample of the current image plus
// three canonical wave-tree sums (b0, b1, cost).  All lanes hold identical
// sums, so the iteration control flow is wave-uniform.  Working set: two
// pyramids (cache-resident); the bound is VALU/latency, not HBM.
#include "device_math.hpp"
#include "kernels.hpp"

#ifdef VISO_PROBE
// [level] iterations summed, [4 + level] calls, [8 + level] window misses
__device__ unsigned long long g_probe_lk[32];
// per item of the background chunk's last frame (row = map point):
// [0] wait start, [1] start (frame ready, pose loaded), [2..5] level 3..0
// iteration start, [6..9] level 3..0 iteration end, [10] end, [11] GN
// iterations L3 | L2 << 16 | L1 << 32 | L0 << 48, [12] HW_ID | XCC << 32 |
// drain << 40 | 1 << 48, [13] window refills, [14] dequeue stamp
constexpr int kProbeItems = 16384;
__device__ unsigned long long g_probe_items[kProbeItems][16];
// per wave of the background grid (rows 0..1023: resident, 1024..: drain):
// [0] start, [1] end, [2] items run, [3] n_left it read
constexpr int kProbeWaves = 8192;
__device__ unsigned long long g_probe_waves[kProbeWaves][4];
#endif

namespace viso {

namespace {

// f.l[level] without indexing a FrameDev at run time (a run-time index into
// a by-value struct makes the compiler copy it per thread into LDS / scratch)
__device__ inline const uint8_t* level_ptr(const FrameDev& f, int level) {
    return level == 0 ? f.l[0] : level == 1 ? f.l[1] : level == 2 ? f.l[2] : f.l[3];
}

struct LkResult {
    double dx, dy;
    bool succ;
    int iters;
};

// Per-wave LDS window of the current image around the patch's starting
// position (inside the image), re-placed by window_follow when the point
// leaves it.  A sample whose four taps lie inside the window reads the same
// bytes from LDS as sample_px would from the buffer; any other sample takes
// sample_px's global path.
constexpr int kWinW = 24, kWinH = 24;

struct Window {
    const uint8_t* lds;  // nullptr: disabled
    int x0, y0;
};

// The window's bytes in flight (issued, not yet in LDS): lane l holds bytes
// l + 64 k of the row-major window.
constexpr int kWinPer = kWinW * kWinH / 64;  // 9
#ifndef VISO_WIN_BYTES
// The window's 24 rows of 24 bytes as 72 unaligned 8-byte loads (row e / 3,
// bytes 8 (e % 3) ..): lanes 0..63 hold chunks 0..63, lanes 0..7 chunks
// 64..71 — two load instructions per window instead of nine byte loads (the
// window sits inside the image, so no byte needs a bounds test).
constexpr int kWinChunks = kWinW * kWinH / 8;  // 72
struct WinRegs {
    uint64_t v[2];
    int x0, y0;
    bool on;
};
#else
struct WinRegs {
    uint8_t v[kWinPer];
    int x0, y0;
    bool on;
};
#endif

// (cx, cy) is the wave's patch centre (the same in every lane): the window's
// placement is taken into SGPRs, so every window test downstream is a
// wave-uniform branch, not an EXEC-mask sequence
__device__ inline WinRegs window_issue(const uint8_t* img, int w, int h, double cx, double cy) {
    WinRegs r;
    r.on = __builtin_amdgcn_readfirstlane(
               !(w < kWinW || h < kWinH || !(cx > -1e6 && cx < 1e6 && cy > -1e6 && cy < 1e6)) ? 1 : 0) != 0;
    r.x0 = r.y0 = 0;
    if (!r.on) return r;
    int x0 = (int)floor(cx) - kWinW / 2 + 1;
    int y0 = (int)floor(cy) - kWinH / 2 + 1;
    x0 = __builtin_amdgcn_readfirstlane(min(max(x0, 0), w - kWinW));
    y0 = __builtin_amdgcn_readfirstlane(min(max(y0, 0), h - kWinH));
    const int lane = threadIdx.x & 63;
    const uint8_t* base = img + ((size_t)y0 * (size_t)w + (size_t)x0);
#ifndef VISO_WIN_BYTES
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int e = lane + 64 * k;
        const int rr = e / 3, c = e - 3 * (e / 3);
        r.v[k] = 0;
        if (e < kWinChunks)
            r.v[k] = *reinterpret_cast<const __attribute__((address_space(1))) uint64_t*>(
                (const __attribute__((address_space(1))) uint8_t*)base + (uint32_t)(rr * w + 8 * c));
    }
#else
    // byte e = lane + 64 k of the row-major window: row e / 24, column e % 24
    // (compile-time per k up to the lane), 32-bit offsets from the window's
    // first byte (a level is far below 2^31 bytes)
#pragma unroll
    for (int k = 0; k < kWinPer; ++k) {
        const int e = lane + 64 * k;
        const int rr = e / kWinW, c = e - rr * kWinW;
        r.v[k] = ld_global_u8_off(base, (uint32_t)(rr * w + c));
    }
#endif
    r.x0 = x0;
    r.y0 = y0;
    return r;
}

__device__ inline Window window_commit(uint8_t* lds, const WinRegs& r) {
    Window win{nullptr, 0, 0};
    if (!r.on) return win;
    const int lane = threadIdx.x & 63;
#ifndef VISO_WIN_BYTES
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int e = lane + 64 * k;
        if (e < kWinChunks)  // chunk e lands at byte 8 e of the row-major window (rows of 24 = 3 chunks)
            *reinterpret_cast<__attribute__((address_space(3))) uint64_t*>(
                (__attribute__((address_space(3))) uint8_t*)lds + 8 * e) = r.v[k];
    }
#else
#pragma unroll
    for (int k = 0; k < kWinPer; ++k) st_lds_u8(lds, lane + 64 * k, r.v[k]);
#endif
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    win.lds = lds;
    win.x0 = r.x0;
    win.y0 = r.y0;
    return win;
}

__device__ inline Window load_window(uint8_t* lds, const uint8_t* img, int w, int h, double cx,
                                     double cy) {
    // all nine loads first, then the LDS stores
    return window_commit(lds, window_issue(img, w, h, cx, cy));
}

// GetPixelValue's bilinear expression on the four taps packed in t (bytes
// d0 | d1 << 8 | d2 << 16 | d3 << 24)
__device__ inline double bilerp_packed(double x, double y, uint32_t t) {
    const double d0 = (double)(t & 0xff), d1 = (double)((t >> 8) & 0xff);
    const double d2 = (double)((t >> 16) & 0xff), d3 = (double)(t >> 24);
    const double xx = x - floor(x);
    const double yy = y - floor(y);
    return double((1 - xx) * (1 - yy) * d0 + xx * (1 - yy) * d1 + (1 - xx) * yy * d2 + xx * yy * d3);
}

// the four window taps of base pixel (ix, iy), packed
__device__ inline uint32_t win_taps(const Window& win, int ix, int iy) {
    const int o = (iy - win.y0) * kWinW + (ix - win.x0);
    return (uint32_t)ld_lds_u8(win.lds, o) | ((uint32_t)ld_lds_u8(win.lds, o + 1) << 8) |
           ((uint32_t)ld_lds_u8(win.lds, o + kWinW) << 16) | ((uint32_t)ld_lds_u8(win.lds, o + kWinW + 1) << 24);
}

// GetPixelValue's bilinear sample with its four taps read from the window
__device__ inline double win_bilinear(const Window& win, double x, double y, int ix, int iy) {
    return bilerp_packed(x, y, win_taps(win, ix, iy));
}

// The GN iterations' window follows the point: once the wave's taps leave
// the window, it is re-placed at the patch's new position and refilled, so
// the following iterations read LDS instead of paying a global round trip
// each.  A re-placed window is a window of the level's continuous buffer, not
// of the image: its origin (x0, y0) is not clamped to the image, and byte
// (r, c) is buffer[(y0 + r) w + x0 + c], 0 outside the buffer — exactly the
// byte sample_px's tap (x0 + c, y0 + r) reads (its row-wrapping and zero
// rules included), so points at or over the image border (the slowest ones:
// up to ~130 GN iterations) are served from LDS too.  Lane 0 holds the
// patch's smallest (ix, iy) (the lanes' integer offsets on a common base).
// Returns false (window unchanged) when some lane's coordinates are not
// finite; the caller then takes its global path.  A wave only overwrites its
// own window, whose earlier reads have all returned (their values fed the
// previous update).
__device__ inline bool window_follow(const uint8_t* __restrict__ img, int w, int h, int ix, int iy, bool ok,
                                    Window& win) {
    if (__builtin_amdgcn_ballot_w64(!ok) != 0) return false;
    // the patch spans <= 9 taps per axis: 7 to spare on each side
    const int x0 = __builtin_amdgcn_readfirstlane(ix) - 7;
    const int y0 = __builtin_amdgcn_readfirstlane(iy) - 7;
    const bool in = (unsigned)(ix - x0) < (unsigned)(kWinW - 1) && (unsigned)(iy - y0) < (unsigned)(kWinH - 1);
    if (__builtin_amdgcn_ballot_w64(in) != ~0ull) return false;
    // the nine loads, then the LDS stores (window_issue / window_commit's
    // forms).  The lane index is made opaque here: its nine window offsets
    // would otherwise be hoisted out of the GN loop and held in registers.
    int lane = threadIdx.x & 63;
    asm volatile("" : "+v"(lane));
    const long long n = (long long)w * (long long)h;
    const long long base = (long long)y0 * (long long)w + (long long)x0;
    uint8_t v[kWinPer];
#pragma unroll
    for (int k = 0; k < kWinPer; ++k) {
        const int e = lane + 64 * k;
        const int rr = e / kWinW, c = e - rr * kWinW;
        v[k] = (uint8_t)ld_u8_or0(img, n, base + (long long)rr * w + c);
    }
    uint8_t* lds = const_cast<uint8_t*>(win.lds);
#pragma unroll
    for (int k = 0; k < kWinPer; ++k) st_lds_u8(lds, lane + 64 * k, v[k]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    win.x0 = x0;
    win.y0 = y0;
    return true;
}

// sample_px with the tap fetch served from the window (re-placed by
// window_follow when the wave leaves it).  The window test is taken for the
// whole wave (one ballot, every lane active: the LK engines' wave-uniform
// control flow).  FINITE: the caller guarantees |x|, |y| < 1e9 (LKAlignment:
// the bounds test passed, so d is within a level of the patch), which
// sample_px's own guard would find true.
template <bool FINITE = false>
__device__ inline double sample_win_follow(const uint8_t* __restrict__ img, int w, int h, double x,
                                           double y, Window& win) {
    if (!win.lds) return sample_px(img, w, h, x, y);  // wave-uniform (window_issue)
    const bool finite = FINITE || (x > -1e9 && x < 1e9 && y > -1e9 && y < 1e9);
    const int ix = finite ? (int)x : 0, iy = finite ? (int)y : 0;
    const bool in = finite && (unsigned)(ix - win.x0) < (unsigned)(kWinW - 1) &&
                    (unsigned)(iy - win.y0) < (unsigned)(kWinH - 1);
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(in) == ~0ull, 1)) return win_bilinear(win, x, y, ix, iy);
    if (window_follow(img, w, h, ix, iy, finite, win)) return win_bilinear(win, x, y, ix, iy);
    return in ? win_bilinear(win, x, y, ix, iy) : sample_px(img, w, h, x, y);
}

// The GN loop's taps of the last window sample, per lane: base pixel (ix,
// iy) and its four bytes.  A converging point's steps are mostly sub-pixel,
// so its base pixels repeat; the taps are buffer bytes (the window mirrors the
// level buffer), so reusing them gives sample_win_follow's value without the
// LDS round trip on the iteration's dependency chain.
struct TapCache {
    int ix, iy;  // INT_MIN: empty
    uint32_t t;
};

template <bool FINITE = false>
__device__ inline double sample_win_cached(const uint8_t* __restrict__ img, int w, int h, double x, double y,
                                           Window& win, TapCache& tc) {
    if (!win.lds) return sample_px(img, w, h, x, y);  // wave-uniform (window_issue)
    const bool finite = FINITE || (x > -1e9 && x < 1e9 && y > -1e9 && y < 1e9);
    const int ix = finite ? (int)x : 0, iy = finite ? (int)y : 0;
#ifndef VISO_LK_NOTAPCACHE
    if (__builtin_amdgcn_ballot_w64(finite && ix == tc.ix && iy == tc.iy) == ~0ull) return bilerp_packed(x, y, tc.t);
#endif
    const bool in = finite && (unsigned)(ix - win.x0) < (unsigned)(kWinW - 1) &&
                    (unsigned)(iy - win.y0) < (unsigned)(kWinH - 1);
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(in) == ~0ull, 1) ||
        window_follow(img, w, h, ix, iy, finite, win)) {
        tc.t = win_taps(win, ix, iy);
        tc.ix = ix;
        tc.iy = iy;
        return bilerp_packed(x, y, tc.t);
    }
    tc.ix = INT_MIN;
    return in ? win_bilinear(win, x, y, ix, iy) : sample_px(img, w, h, x, y);
}

// The per-level template of the inverse-compositional LK: this lane's
// template value I1 and Jacobian (J0, J1) = -grad at ref, and the 2x2 inverse
// of H = sum J J^T (canonical wave trees).  It depends only on the reference
// image and the template position, so LK alignment precomputes it once per
// map (lk_template_kernel) instead of per frame.
struct LkTemplate {
    double I1, J0, J1;
    double i00, i01, i10, i11;
};

// the same in fp32 (tolerance mode)
struct LkTemplateF {
    float I1, J0, J1;
    float ih[4];
};

__device__ inline LkTemplate lk_prepare(const uint8_t* __restrict__ img1, int w1, int h1,
                                        double ref_x, double ref_y) {
    LkTemplate t;
    double gx, gy;
    gradient_px(img1, w1, h1, ref_x, ref_y, gx, gy);
    t.J0 = -gx;
    t.J1 = -gy;
    t.I1 = sample_px(img1, w1, h1, ref_x, ref_y);
    double H00, H01, H11;
    wave_tree_sum3(t.J0 * t.J0, t.J0 * t.J1, t.J1 * t.J1, H00, H01, H11);
    const double H10 = H01;  // J1*J0 == J0*J1 leaf by leaf
    const double invdet = 1.0 / (H00 * H11 - H10 * H01);
    t.i00 = H11 * invdet;
    t.i10 = -H10 * invdet;
    t.i01 = -H01 * invdet;
    t.i11 = H00 * invdet;
    return t;
}

// The GN iterations of one level.
//   cur_x/cur_y: current-image coordinate of this lane's pixel without d;
//   bx/by: coordinate whose +d is bounds-checked (per engine); w1/h1: the
//   size the bounds test uses.
template <int MAXIT, bool KLT_BOUNDS>
__device__ inline LkResult lk_iterate(const LkTemplate& t, int w1, int h1,
                                      const uint8_t* __restrict__ img2, int w2, int h2,
                                      double cur_x, double cur_y, double bx, double by, double dx,
                                      double dy, double thresh, Window win, int boost_at = -1) {
    const double hp = 4.0;
    // the control values are wave-uniform (the sums are read from one lane):
    // said so to the compiler, the loop's branches need no EXEC bookkeeping
    bx = uniform_f64(bx);
    by = uniform_f64(by);
    dx = uniform_f64(dx);
    dy = uniform_f64(dy);
    const double i00 = uniform_f64(t.i00), i01 = uniform_f64(t.i01), i10 = uniform_f64(t.i10),
                 i11 = uniform_f64(t.i11);
    // LKAlignment's bounds test (both corners, 8 comparisons of uniform
    // values) runs lane-parallel: lane l tests coordinate l & 1 (x, y) of
    // corner l & 2 (-hp, +hp), (b + d) + (-+hp) in [0, w or h), the same
    // operations as inside_px on (b + d) -+ hp
    const int lq = threadIdx.x & 3;
    const double b_l = (lq & 1) ? by : bx;
    const double off_l = (lq & 2) ? hp : -hp;
    const double lim_l = (double)((lq & 1) ? h1 : w1);
    double cost = 0, lastCost = 0;
    bool succ = true;
    int iter = 0;
    TapCache tc{INT_MIN, INT_MIN, 0u};
    for (; iter < MAXIT; ++iter) {
        // a point still iterating after boost_at steps (the background grid's
        // last frame, VISO_LK_BOOST): its wave outranks the short points'
        if (iter == boost_at) __builtin_amdgcn_s_setprio(2);
        bool out;
        if (KLT_BOUNDS) {  // src/viso.cpp:286
            out = bx + dx <= hp || bx + dx >= w1 - hp || by + dy <= hp || by + dy >= h1 - hp;
        } else {  // src/viso.cpp:869-873 (ref coords + d, both corners)
            const double q = (b_l + ((lq & 1) ? dy : dx)) + off_l;
            out = __builtin_amdgcn_ballot_w64(!(q >= 0 && q < lim_l)) != 0;
        }
        if (out) {
            succ = false;
            break;
        }
        // (KLT: ten iterations at most, its window path as it was)
        double smp;
        if constexpr (KLT_BOUNDS)
            smp = sample_win_follow<false>(img2, w2, h2, cur_x + dx, cur_y + dy, win);
        else
            smp = sample_win_cached<true>(img2, w2, h2, cur_x + dx, cur_y + dy, win, tc);
        const double e = t.I1 - smp;
        double B0, B1;
        if (KLT_BOUNDS)
            wave_tree_sum3(-t.J0 * e, -t.J1 * e, e * e, B0, B1, cost);
        else  // LK alignment: the descending-stride tree (oracle tree_sum_desc64)
            wave_tree_sum3_desc(-t.J0 * e, -t.J1 * e, e * e, B0, B1, cost);
        const double u0 = i00 * B0 + i01 * B1;
        const double u1 = i10 * B0 + i11 * B1;
        if (isnan(u0)) {
            succ = false;
            break;
        }
        if (iter > 0 && cost > lastCost) break;
        dx += u0;
        dy += u1;
        lastCost = cost;
        succ = !(lastCost > thresh);
    }
    return {dx, dy, succ, iter};
}

// Tolerance mode (VISO_PRECISION_FAST) GN iterations of one LKAlignment
// level: the same control flow (bounds test on ref coords + d, NaN / cost-
// increase stops, success = last accepted cost <= thresh) in fp32.  The
// sub-pixel fraction of (patch origin + d) is shared by the 64 lanes (their
// offsets are integers), so a sample is four window taps and three fmas.
template <int MAXIT>
__device__ inline LkResult lk_iterate_fast(float I1, float J0, float J1, const float* ih, int w1, int h1,
                                           const uint8_t* __restrict__ img2, int w2, int h2, double ox,
                                           double oy, int px, int py, double bx, double by, double thresh,
                                           Window win) {
    const double hp = 4.0;
    double dx = 0.0, dy = 0.0;
    float lastCost = 0.0f;
    bool succ = true;
    int iter = 0;
    const long long n2 = (long long)w2 * h2;
    // the bounds test lane-parallel, as in lk_iterate
    const int lq = threadIdx.x & 3;
    const double b_l = (lq & 1) ? by : bx;
    const double off_l = (lq & 2) ? hp : -hp;
    const double lim_l = (double)((lq & 1) ? h1 : w1);
    for (; iter < MAXIT; ++iter) {
        const double q = (b_l + ((lq & 1) ? dy : dx)) + off_l;
        if (__builtin_amdgcn_ballot_w64(!(q >= 0 && q < lim_l)) != 0) {
            succ = false;
            break;
        }
        const double X = ox + dx, Y = oy + dy;
        const double fX = floor(X), fY = floor(Y);
        const float xx = (float)(X - fX), yy = (float)(Y - fY);
        const int ix = (int)fX + px, iy = (int)fY + py;
        float t0, t1, t2, t3;
        bool in = win.lds && ix >= win.x0 && ix + 1 < win.x0 + kWinW && iy >= win.y0 && iy + 1 < win.y0 + kWinH;
        // (X, Y finite: the bounds test passed)
        if (win.lds && __builtin_amdgcn_ballot_w64(in) != ~0ull && window_follow(img2, w2, h2, ix, iy, true, win))
            in = true;
        if (__builtin_expect(in, 1)) {
            const int o = (iy - win.y0) * kWinW + (ix - win.x0);
            t0 = (float)ld_lds_u8(win.lds, o);
            t1 = (float)ld_lds_u8(win.lds, o + 1);
            t2 = (float)ld_lds_u8(win.lds, o + kWinW);
            t3 = (float)ld_lds_u8(win.lds, o + kWinW + 1);
        } else {
            const long long o = (long long)iy * w2 + ix;
            t0 = (float)ld_u8_or0(img2, n2, o);
            t1 = (float)ld_u8_or0(img2, n2, o + 1);
            t2 = (float)ld_u8_or0(img2, n2, o + w2);
            t3 = (float)ld_u8_or0(img2, n2, o + w2 + 1);
        }
        const float e = I1 - bilerp_f32(t0, t1, t2, t3, xx, yy);
        float B0, B1, cost;
        wave_tree_sum3_f32_desc(-J0 * e, -J1 * e, e * e, B0, B1, cost);
        const float u0 = ih[0] * B0 + ih[1] * B1;
        const float u1 = ih[2] * B0 + ih[3] * B1;
        if (isnan(u0)) {
            succ = false;
            break;
        }
        if (iter > 0 && cost > lastCost) break;
        dx += (double)u0;
        dy += (double)u1;
        lastCost = cost;
        succ = !((double)lastCost > thresh);
    }
    return {dx, dy, succ, iter};
}

__device__ __attribute__((always_inline)) inline void klt_track_body(const FrameDev& ref, const FrameDev& cur, const PyrDev& g,
                                                                     const float2* __restrict__ kp1,
                                                                     float2* __restrict__ kp2,
                                                                     uint8_t* __restrict__ success, int i,
                                                                     double thresh, uint8_t* my_win) {
    const int lane = threadIdx.x & 63;
    const int px = (lane >> 3) - 4, py = (lane & 7) - 4;
    const float2 k1 = kp1[i];
    float2 k2 = kp2[i];
    // kp2[j].pt *= scales[3]  (saturate_cast<float>(x * 0.125))
    k2.x = (float)((double)k2.x * kScale[3]);
    k2.y = (float)((double)k2.y * kScale[3]);
    bool succ = true;
    for (int level = kLevels - 1; level >= 0; --level) {
        const float kx = (float)((double)k1.x * kScale[level]);
        const float ky = (float)((double)k1.y * kScale[level]);
        const double dx0 = (double)(k2.x - kx), dy0 = (double)(k2.y - ky);
        const float fx = kx + (float)px, fy = ky + (float)py;  // float + int
        const int w = g.w[level], h = g.h[level];
        // the current-image window's loads and the template's (reference
        // image) loads are in flight together: one memory round trip per
        // level instead of two
        const WinRegs wr = window_issue(cur.l[level], w, h, (double)kx + dx0, (double)ky + dy0);
        const LkTemplate t = lk_prepare(ref.l[level], w, h, (double)fx, (double)fy);
        const Window win = window_commit(my_win, wr);
        LkResult r = lk_iterate<10, true>(t, w, h, cur.l[level], w, h, (double)fx, (double)fy,
                                          (double)kx, (double)ky, dx0, dy0, thresh, win);
        succ = r.succ;
        k2.x = kx + (float)r.dx;
        k2.y = ky + (float)r.dy;
        if (level != 0) {
            k2.x = (float)((double)k2.x / 0.5);
            k2.y = (float)((double)k2.y / 0.5);
        }
    }
    if (lane == 0) {
        kp2[i] = k2;
        success[i] = succ ? 1 : 0;
    }
}

// n_dev (optional): the track count in device memory (after a re-detection
// frame, whose FAST count the host has not read), capped at n; the grid then
// covers n and waves past the count return at once.  (A grid-stride loop over
// the tracks measured 40 % slower: the loop moved the window state into 16 KB
// of promoted LDS and 110 VGPRs.)
__global__ __launch_bounds__(256) void klt_kernel(FrameDev ref, FrameDev cur, PyrDev g,
                                                  const float2* __restrict__ kp1,
                                                  float2* __restrict__ kp2,
                                                  uint8_t* __restrict__ success, int n,
                                                  double thresh, const int* __restrict__ n_dev) {
    __shared__ __attribute__((aligned(16))) uint8_t s_win[4][kWinW * kWinH];
    const int i = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    if (n_dev) n = min(__builtin_amdgcn_readfirstlane(*n_dev), n);
    if (i >= n) return;  // wave-uniform
    klt_track_body(ref, cur, g, kp1, kp2, success, i, thresh, s_win[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)]);
}


// Keyframe choice of one map point (LKAlignment, src/viso.cpp:774-800):
// the keyframe with the smallest viewing angle (Keyframe::ViewingAngle,
// include/keyframe.h:93-98) among those the point projects into.  It does
// not depend on the current frame.
__device__ inline int lk_choose_kf(const LkAlignArgs& a, const double* P, double& bu, double& bv) {
    const Intrinsics K{a.K[0], a.K[1], a.K[2], a.K[3]};
    const int w0 = a.g.w[0], h0 = a.g.h[0];
    double best_angle = 180.0;
    int kf = -1;
    bu = 0;
    bv = 0;
    const double kPi = 3.14159265358979323846;
    for (int j = 0; j < a.n_kf; ++j) {
        const double* kp = a.kf_poses + 12 * j;
        double ur, vr;
        project_px(kp, K, P, 1.0, ur, vr);
        if (!inside_px(ur, vr, w0, h0)) continue;
        double Pc[3];
        mat3_vec(kp, P, Pc);
        Pc[0] = Pc[0] + kp[9];
        Pc[1] = Pc[1] + kp[10];
        Pc[2] = Pc[2] + kp[11];
        const double nrm = (Pc[0] * Pc[0] + Pc[1] * Pc[1]) + Pc[2] * Pc[2];
        if (nrm > 0) {
            const double sn = sqrt(nrm);
            Pc[0] = Pc[0] / sn;
            Pc[1] = Pc[1] / sn;
            Pc[2] = Pc[2] / sn;
        }
        const double angle = fabs(acos(Pc[2]) / kPi * 180);
        if (angle > 180.0 || angle > best_angle) continue;
        best_angle = angle;
        kf = j;
        bu = ur;
        bv = vr;
    }
    return kf;
}

// Per map point, once per map: the keyframe choice and the four levels'
// templates (lk_prepare) of LK alignment.  tmpl layout: [point][level]
// [I1 | J0 | J1][64 lanes]; tmpl_h: [point][level][i00, i01, i10, i11].
__global__ __launch_bounds__(256) void lk_template_kernel(LkAlignArgs a) {
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= a.n) return;  // wave-uniform
    const int lane = threadIdx.x & 63;
    const int px = (lane >> 3) - 4, py = (lane & 7) - 4;
    const double P[3] = {a.points[3 * i], a.points[3 * i + 1], a.points[3 * i + 2]};
    double bu, bv;
    const int kf = lk_choose_kf(a, P, bu, bv);
    if (lane == 0) {
        a.tmpl_kf[i] = kf;
        a.tmpl_uv[2 * i] = bu;
        a.tmpl_uv[2 * i + 1] = bv;
    }
    if (kf < 0) return;
    const FrameDev refp = a.kf[kf];
    for (int level = kLevels - 1; level >= 0; --level) {
        const double s = kScale[level];
        const int w = a.g.w[level], h = a.g.h[level];
        const LkTemplate t = lk_prepare(refp.l[level], w, h, bu * s + px, bv * s + py);
        if (a.fast) {
            float* d = (float*)a.tmpl + ((size_t)i * kLevels + level) * 192;
            d[lane] = (float)t.I1;
            d[64 + lane] = (float)t.J0;
            d[128 + lane] = (float)t.J1;
            if (lane == 0) {
                float* hh = (float*)a.tmpl_h + ((size_t)i * kLevels + level) * 4;
                hh[0] = (float)t.i00;
                hh[1] = (float)t.i01;
                hh[2] = (float)t.i10;
                hh[3] = (float)t.i11;
            }
            continue;
        }
        double* d = a.tmpl + ((size_t)i * kLevels + level) * 192;
        d[lane] = t.I1;
        d[64 + lane] = t.J0;
        d[128 + lane] = t.J1;
        if (lane == 0) {
            double* hh = a.tmpl_h + ((size_t)i * kLevels + level) * 4;
            hh[0] = t.i00;
            hh[1] = t.i01;
            hh[2] = t.i10;
            hh[3] = t.i11;
        }
    }
}

// LKAlignment over the frames of a batch (blockIdx.y = frame).  Blocks along
// x are point groups; the grid's x extent is a multiple of 8, so a point
// group stays on one XCD for every frame and its templates stay in that
// XCD's L2.
// waves per SIMD the register allocation must allow: faithful 5 (<= 96
// VGPRs, no spills; 6 spills and was 7 % slower), tolerance mode 6 (80 VGPRs,
// no spills: 4 % faster than 5)
#ifndef VISO_LK_MIN_WAVES
#define VISO_LK_MIN_WAVES 5
#endif
#ifndef VISO_LK_MIN_WAVES_FAST
#define VISO_LK_MIN_WAVES_FAST 6
#endif
// One (frame, map point) of LKAlignment: the wave's point i against frame
// `cur` at pose cur_pose (12 doubles), outputs at row offset o.  `ka` is the
// kernel argument in the kernarg segment (run-time indices into its arrays are
// read from there: a run-time index into the by-value struct would copy it per
// thread to scratch).
template <bool FAST>
__device__ __attribute__((always_inline)) inline void lk_point(const LkAlignArgs& a, const LkAlignArgs* ka,
                                                               const FrameDev& cur, const double* cur_pose, int i,
                                                               size_t o, uint8_t* my_win0, uint8_t* my_win1,
                                                               int pr_slot = -1, int boost_at = -1) {
    const int lane = threadIdx.x & 63;
    const int px = (lane >> 3) - 4, py = (lane & 7) - 4;
    const double P[3] = {a.points[3 * i], a.points[3 * i + 1], a.points[3 * i + 2]};
    const Intrinsics K{a.K[0], a.K[1], a.K[2], a.K[3]};
    const int w0 = a.g.w[0], h0 = a.g.h[0];
    int32_t kf = -1;
    uint8_t succ_out = 0;
    double ub[2] = {0.0, 0.0}, ua[2] = {0.0, 0.0};
    double uc, vc;
    project_px(cur_pose, K, P, 1.0, uc, vc);
    if (inside_px(uc, vc, w0, h0)) {  // current_frame->IsInside(Pw, 0)
        double bu, bv;
        if (a.tmpl) {
            kf = a.tmpl_kf[i];
            bu = a.tmpl_uv[2 * i];
            bv = a.tmpl_uv[2 * i + 1];
        } else {
            kf = lk_choose_kf(a, P, bu, bv);
        }
        if (kf >= 0) {
            ub[0] = uc;
            ub[1] = vc;
            double cu = uc, cv = vc;
            const FrameDev& refp = ka->kf[kf];
            bool succ = false;
#ifdef VISO_PROBE
            unsigned long long pr_it[kLevels] = {0, 0, 0, 0}, pr_win = 0, pr_iter = 0, pr_long = 0;
            const unsigned long long pr_t0 = __builtin_amdgcn_s_memrealtime();
#endif
            // level l's window (around the position level l + 1 ended at) and
            // template are loaded when level l + 1 is done
            auto tmpl_load = [&](int level, LkTemplate& t, LkTemplateF& tf) {
                if (FAST) {
                    const float* d = (const float*)a.tmpl + ((size_t)i * kLevels + level) * 192;
                    const float* hh = (const float*)a.tmpl_h + ((size_t)i * kLevels + level) * 4;
                    tf.I1 = d[lane];
                    tf.J0 = d[64 + lane];
                    tf.J1 = d[128 + lane];
                    for (int k = 0; k < 4; ++k) tf.ih[k] = hh[k];
                } else if (a.tmpl) {
                    const double* d = a.tmpl + ((size_t)i * kLevels + level) * 192;
                    const double* hh = a.tmpl_h + ((size_t)i * kLevels + level) * 4;
                    t.I1 = d[lane];
                    t.J0 = d[64 + lane];
                    t.J1 = d[128 + lane];
                    t.i00 = hh[0];
                    t.i01 = hh[1];
                    t.i10 = hh[2];
                    t.i11 = hh[3];
                }
            };
            LkTemplate tn{};
            LkTemplateF tfn{};
            tmpl_load(kLevels - 1, tn, tfn);
            Window win = load_window(my_win0, level_ptr(cur, kLevels - 1), a.g.w[kLevels - 1],
                                     a.g.h[kLevels - 1], cu * kScale[kLevels - 1], cv * kScale[kLevels - 1]);
            for (int level = kLevels - 1; level >= 0; --level) {
                const double s = kScale[level];
                const int w = a.g.w[level], h = a.g.h[level];
                const double cx = cu * s + px, cy = cv * s + py;
                LkTemplate t = tn;
                const LkTemplateF tf = tfn;
                const Window wcur = win;
                // (issuing level l-1's loads before iterating level l was
                // measured slower: the batch is issue-bound, and the extra
                // live registers cost occupancy)
                auto next = [&]() {
                    if (level > 0) {
                        const double s1 = kScale[level - 1];
                        tmpl_load(level - 1, tn, tfn);
#ifdef VISO_PROBE_WIN
                        // (probe) the window's global loads: issue -> data in
                        // registers -> committed to LDS, the slowest level's
                        const unsigned long long pw0 = __builtin_amdgcn_s_memrealtime();
                        const WinRegs wr = window_issue(level_ptr(cur, level - 1), a.g.w[level - 1],
                                                        a.g.h[level - 1], cu * s1, cv * s1);
                        int sum = 0;
#pragma unroll
                        for (int k = 0; k < (int)(sizeof(wr.v) / sizeof(wr.v[0])); ++k) sum += (int)wr.v[k];
                        __builtin_amdgcn_readfirstlane(sum);  // waits for the nine loads
                        asm volatile("" ::"v"(sum));
                        const unsigned long long pw1 = __builtin_amdgcn_s_memrealtime();
                        win = window_commit((level & 1) ? my_win0 : my_win1, wr);
                        const unsigned long long pw2 = __builtin_amdgcn_s_memrealtime();
                        if (pr_slot >= 0 && lane == 0) {
                            const unsigned long long ld = (pw1 - pw0) < 65535 ? (pw1 - pw0) : 65535;
                            const unsigned long long st = (pw2 - pw1) < 65535 ? (pw2 - pw1) : 65535;
                            const unsigned long long old = g_probe_items[pr_slot][15];
                            if (ld > (old & 0xffff))
                                g_probe_items[pr_slot][15] = ld | (st << 16) | ((unsigned long long)(level - 1) << 32) |
                                                             ((pw0 & 0xffffffull) << 40);
                        }
#else
                        win = load_window((level & 1) ? my_win0 : my_win1, level_ptr(cur, level - 1),
                                          a.g.w[level - 1], a.g.h[level - 1], cu * s1, cv * s1);
#endif
                    }
                };
#ifdef VISO_PROBE
                const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
#endif
                if (FAST) {
                    // tolerance mode: fp32 template (lk_template_kernel) and iterations
                    const LkResult r = lk_iterate_fast<100>(tf.I1, tf.J0, tf.J1, tf.ih, w, h, level_ptr(cur, level),
                                                            w, h, cu * s, cv * s, px, py, bu * s, bv * s, a.thresh,
                                                            wcur);
                    succ = r.succ;
                    cu = cu + r.dx / s;
                    cv = cv + r.dy / s;
                    next();
                    continue;
                }
                if (!a.tmpl) t = lk_prepare(level_ptr(refp, level), w, h, bu * s + px, bv * s + py);
#ifdef VISO_PROBE
                const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
#endif
                LkResult r = lk_iterate<100, false>(t, w, h, level_ptr(cur, level), w, h, cx, cy, bu * s,
                                                    bv * s, 0.0, 0.0, a.thresh, wcur, boost_at);
                succ = r.succ;
#ifdef VISO_PROBE
                pr_it[level] += (unsigned long long)r.iters;
                pr_win += t1 - t0;
                const unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
                pr_iter += t2 - t1;
                pr_long += r.iters >= 10 ? 1 : 0;
                if (pr_slot >= 0 && lane == 0) {
                    g_probe_items[pr_slot][2 + (3 - level)] = t1;
                    g_probe_items[pr_slot][6 + (3 - level)] = t2;
                }
#endif
                cu = cu + r.dx / s;  // pair.uv_cur += V2d{dx/s, dy/s}
                cv = cv + r.dy / s;
                next();
            }
#ifdef VISO_PROBE
            if (pr_slot >= 0 && lane == 0)
                g_probe_items[pr_slot][11] = pr_it[3] | (pr_it[2] << 16) | (pr_it[1] << 32) | (pr_it[0] << 48);
#ifndef VISO_PROBE_LIGHT  // (the light probe: plain per-item stores only, no same-address atomics)
            if (lane == 0) {
                for (int l = 0; l < kLevels; ++l) {
                    atomicAdd(&g_probe_lk[l], pr_it[l]);
                    atomicAdd(&g_probe_lk[4 + l], 1ull);
                }
                atomicAdd(&g_probe_lk[8], pr_long);
                atomicAdd(&g_probe_lk[12], pr_win);
                atomicAdd(&g_probe_lk[13], pr_iter);
                const unsigned long long pr_el = __builtin_amdgcn_s_memrealtime() - pr_t0;
                atomicAdd(&g_probe_lk[14], pr_el);
                atomicMax(&g_probe_lk[9], pr_el);  // slowest point (100 MHz ticks)
                atomicMax(&g_probe_lk[10], pr_it[0] + pr_it[1] + pr_it[2] + pr_it[3]);
                if (pr_el >= 2000) atomicAdd(&g_probe_lk[11], 1ull);  // points >= 20 us
                const unsigned long long pr_n = pr_it[0] + pr_it[1] + pr_it[2] + pr_it[3];
                // the slowest point's iterations (24), the most-iterated point's time (25)
                atomicMax(&g_probe_lk[24], (pr_el << 16) | (pr_n < 65535 ? pr_n : 65535));
                atomicMax(&g_probe_lk[25], (pr_n << 40) | (pr_el < (1ull << 40) ? pr_el : (1ull << 40) - 1));
                atomicAdd(&g_probe_lk[15], 1ull);
            }
#endif
#endif
            succ_out = succ ? 1 : 0;
            ua[0] = cu;
            ua[1] = cv;
        }
    }
    if (lane == 0) {
        a.pair_kf[o + i] = kf;
        a.success[o + i] = succ_out;
        a.uv_before[2 * (o + i)] = ub[0];
        a.uv_before[2 * (o + i) + 1] = ub[1];
        a.uv_after[2 * (o + i)] = ua[0];
        a.uv_after[2 * (o + i) + 1] = ua[1];
    }
}

template <bool FAST>
__global__ __launch_bounds__(256, FAST ? VISO_LK_MIN_WAVES_FAST : VISO_LK_MIN_WAVES) void lk_align_kernel(
    LkAlignArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t s_win[4][2][kWinW * kWinH];
    const int i = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    if (i >= a.n) return;
    // frame of the batch (blockIdx.y): its pyramid, pose and output rows
    const LkAlignArgs* ka = (const LkAlignArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    const LkFrame& fr = ka->frames[blockIdx.y];
    const FrameDev cur = fr.cur;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    lk_point<FAST>(a, ka, cur, fr.pose, i, (size_t)blockIdx.y * a.out_stride, s_win[wave][0], s_win[wave][1]);
}

// LK alignment in the background of an ingest chunk (viso_ctx::bg_begin;
// lk_item_kernel):
// one 256-thread workgroup per CU, resident for the whole chunk beside the
// direct pose's workgroups (its LDS request, static + dynamic, caps it at one
// per CU; <= 128 VGPRs: the spare wave slot of each SIMD beside three
// 128-VGPR direct-pose waves).  Each wave takes
// (frame, point) items in frame order from the work heads, waits for the frame's
// pose (the direct pose raises the frame's ready flag after storing it, both
// agent-scope: MI355X_MICROARCH.md's first sc1 hand-off row), and runs that
// point's LKAlignment with the batched kernel's exact per-point code.  Every
// wait is bounded: a resident wave whose item's frame is not ready within
// LkAlignArgs::bg_idle (300 us: ~6 frames of the chain) hands the item to the
// leftover list and leaves (the end-of-
// chunk drain runs the leftovers first, then whatever the heads still hold),
// so a grid that some serialisation of the queues put in the chain's way
// steps aside; the drain's own waits beyond kBgWaitTicks set *bg_err.
// The chunk's drain (launch_lk_drain) is the same kernel without the LDS
// padding, launched after the chunk's last pose: the items the resident grid
// has not reached run beside it on every CU's remaining wave slots.
constexpr unsigned long long kBgWaitTicks = 20000000ull;  // 200 ms of s_memrealtime
#ifndef VISO_LK_BG_TAKE
#define VISO_LK_BG_TAKE 2
#endif
constexpr int kBgTake = VISO_LK_BG_TAKE;  // items per head dequeue (1 or 2)
#ifndef VISO_LK_BOOST
#define VISO_LK_BOOST 12
#endif
// s_sleep quanta (64 cycles) between polls of a frame's ready flag: a
// thousand waiting waves polling one line share the memory system with the
// chain they wait for
#ifndef VISO_LK_BG_POLL
#define VISO_LK_BG_POLL 4
#endif
constexpr int kBgLeftCap = 4096;                           // leftover items (one per resident wave at most)
constexpr int kBgClosed = 1 << 30;                          // bg_left[1]: the drain has read the count
// a background wait that failed: the sticky error word, and its pinned host
// copy (viso_ctx::bg_check reads that after its stream sync)
__device__ inline void bg_fail(const LkAlignArgs& a) {
    atomicOr(a.bg_err, 1);
    if (a.bg_err_host) __hip_atomic_store(a.bg_err_host, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <bool FAST>
__global__ __launch_bounds__(256, 4) void lk_item_kernel(LkAlignArgs a) {
    if (a.n_frames <= 0) return;  // warm_lk_bg
    __shared__ __attribute__((aligned(16))) uint8_t s_win[4][2][kWinW * kWinH];
    __shared__ double s_pose[4][12];  // the wave's current frame pose
    const LkAlignArgs* ka = (const LkAlignArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    int f_loaded = -1;
    // eight work heads, one per XCD (one head saturates near 88 dequeues per
    // us, MI355X_MICROARCH.md "dequeue"): head x holds segment x of every
    // frame's points (points [x seg, (x + 1) seg)), frames in order; a wave
    // drains its own XCD's head, then the others'
    const int seg = (a.n + 7) / 8;
    // A head's item numbers: frames 0 .. n_frames - 2 at one number per
    // point; the last frame (whose pose only the chunk's final solve gives,
    // so its items gate the chunk's end) at two numbers per point, the odd one
    // a dummy, so a two-number dequeue takes ONE of its points and no wave
    // runs two of them back to back.  The last frame starts at an even number.
    const int base = (a.n_frames - 1) * seg;
    const int base_e = base + (base & 1);
    const int per_head = base_e + 2 * seg;
    const int xcc = (int)(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 7);  // HW_REG_XCC_ID
    auto ready = [&](int f) {
        return __builtin_amdgcn_readfirstlane(
                   __hip_atomic_load(a.bg_ready + f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0;
    };
    // The leftover list: bg_left[1] counts the published slots and carries
    // kBgClosed once the drain has read it.  A slot is reserved only by a CAS
    // on an open count, so the count every drain wave reads when it closes
    // the list (atomicOr) is final: no item can land past it.  A resident
    // wave that finds the list closed runs its item itself — the drain starts
    // behind the chunk's last pose, so every ready flag is raised by then.
    // Returns false when the list is closed.
    auto give_back = [&](int head, int k) -> bool {
        int ok = 1;
        if (lane == 0) {
            int c = __hip_atomic_load(a.bg_left + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            for (;;) {
                if (c & kBgClosed) {
                    ok = 0;
                    break;
                }
                if (c >= kBgLeftCap) {  // (one slot per resident wave: unreachable)
                    bg_fail(a);
                    break;
                }
                const int prev = atomicCAS(a.bg_left + 1, c, c + 1);
                if (prev == c) {
                    // publish the item (+1: 0 = not yet written; a drain wave
                    // that read the count may be waiting for it)
                    __hip_atomic_store(a.bg_left + 32 + c, head * per_head + k + 1, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
                c = prev;
            }
        }
        return __builtin_amdgcn_readfirstlane(ok) != 0;
    };
    unsigned long long t_deq = 0;  // (probe) the item's dequeue
    int pr_src = 0;                // (probe) 0 head, 1 leftover list, 2 the dequeue's second item
    // one item: wait for its frame (a resident wave at most a.bg_idle ticks,
    // then the item goes to the leftover list and the wave leaves, unless the
    // list is closed; the drain, and a resident wave whose list is closed, at
    // most kBgWaitTicks, an error), then align the point.  Returns false when
    // the item was handed to the leftover list or its wait failed.
    auto run_item = [&](int head, int k) __attribute__((always_inline)) -> bool {
        int f, i;
        if (k < base) {
            f = k / seg;
            i = head * seg + (k - f * seg);
        } else {
            const int r = k - base_e;
            if (r < 0 || (r & 1)) return true;  // padding / the last frame's dummy numbers
            f = a.n_frames - 1;
            i = head * seg + (r >> 1);
        }
        if (i >= a.n) return true;
        unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        bool must = a.bg_drain != 0;
        while (!ready(f)) {
            const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - t0;
            if (!must && dt > (unsigned long long)a.bg_idle) {
                if (give_back(head, k)) return false;
                must = true;  // the list is closed: every pose is launched
                t0 = __builtin_amdgcn_s_memrealtime();
            }
            if (must && dt > kBgWaitTicks) {
                if (lane == 0) bg_fail(a);
                return false;
            }
            __builtin_amdgcn_s_sleep(VISO_LK_BG_POLL);
        }
        const LkFrame& fr = ka->frames[f];
        if (f != f_loaded) {  // wave-uniform
            if (lane < 12)
                s_pose[wave][lane] = __hip_atomic_load(fr.pose + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            f_loaded = f;
        }
        const FrameDev cur = fr.cur;
#ifdef VISO_PROBE
        const int pr_slot = (f == a.n_frames - 1 && i < kProbeItems) ? i : -1;
        if (pr_slot >= 0 && lane == 0) {
            g_probe_items[pr_slot][0] = t0;
            g_probe_items[pr_slot][1] = __builtin_amdgcn_s_memrealtime();
            g_probe_items[pr_slot][12] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
                                         ((unsigned long long)xcc << 32) | ((unsigned long long)(a.bg_drain ? 1 : 0) << 40) |
                                         (1ull << 48);
            g_probe_items[pr_slot][14] = t_deq;
            g_probe_items[pr_slot][13] = (unsigned long long)pr_src | ((unsigned long long)head << 8);
        }
#else
        const int pr_slot = -1;
#endif
#if defined(VISO_PROBE) && !defined(VISO_PROBE_LIGHT)
        // the chunk's last frame: first ready sighting (16, stored inverted
        // for atomicMax), last completion (17), slowest item (18), items (19),
        // items the drain ran (20), last item start (21)
        const bool pr_last = f == a.n_frames - 1;
        const unsigned long long pr_s = __builtin_amdgcn_s_memrealtime();
        if (pr_last && lane == 0) {
            atomicMax(&g_probe_lk[16], ~pr_s);
            atomicMax(&g_probe_lk[21], pr_s);
        }
#endif
        // the chunk's last frame runs after the chain: its long points take
        // issue priority over the short ones (VISO_LK_BOOST steps, 0 = off)
        const int boost_at = (VISO_LK_BOOST > 0 && f == a.n_frames - 1) ? VISO_LK_BOOST : -1;
        lk_point<FAST>(a, ka, cur, s_pose[wave], i, (size_t)f * a.out_stride, s_win[wave][0], s_win[wave][1],
                       pr_slot, boost_at);
        if (boost_at >= 0) __builtin_amdgcn_s_setprio(0);
#ifdef VISO_PROBE
        if (pr_slot >= 0 && lane == 0) g_probe_items[pr_slot][10] = __builtin_amdgcn_s_memrealtime();
#endif
#if defined(VISO_PROBE) && !defined(VISO_PROBE_LIGHT)
        if (lane == 0) atomicMax(&g_probe_lk[23], __builtin_amdgcn_s_memrealtime());  // any item's end
        if (pr_last && lane == 0) {
            const unsigned long long pr_e = __builtin_amdgcn_s_memrealtime();
            atomicMax(&g_probe_lk[17], pr_e);
            atomicMax(&g_probe_lk[18], pr_e - pr_s);
            atomicAdd(&g_probe_lk[19], 1ull);
            if (a.bg_drain) atomicAdd(&g_probe_lk[20], 1ull);
        }
#endif
        return true;
    };
    // the items resident waves gave back (the drain only), then the heads;
    // one loop, so the per-point code is inlined once
    // the drain's first wave closes the leftover list (the count it reads is
    // final) and publishes that count in bg_left[2] (one word: value and valid
    // bit together); the other drain waves read it there — one atomic instead
    // of one per drain wave (same-address atomics serialise, ~12 ns each:
    // 3,072 of them would cost ~37 us at the chunk's end)
    int n_left = 0;
    if (a.bg_drain) {
        if (blockIdx.x == 0 && wave == 0) {
            if (lane == 0 && a.bg_inject_fail) bg_fail(a);  // (tests: the error path)
            if (lane == 0) {
                n_left = atomicOr(a.bg_left + 1, kBgClosed) & ~kBgClosed;
                __hip_atomic_store(a.bg_left + 2, n_left | kBgClosed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            n_left = __builtin_amdgcn_readfirstlane(n_left);
        } else {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            int v;
            while (!((v = __builtin_amdgcn_readfirstlane(
                          __hip_atomic_load(a.bg_left + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) &
                     kBgClosed)) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > kBgWaitTicks) {
                    if (lane == 0) bg_fail(a);
                    return;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            n_left = v & ~kBgClosed;
        }
        n_left = min(n_left, kBgLeftCap);
    }
    bool left_phase = n_left > 0;
#ifdef VISO_PROBE
    const int pr_w = (a.bg_drain ? 1024 : 0) + (int)blockIdx.x * 4 + wave;
    int pr_items = 0;
    if (lane == 0 && pr_w < kProbeWaves) {
        g_probe_waves[pr_w][0] = __builtin_amdgcn_s_memrealtime();
        g_probe_waves[pr_w][3] = (unsigned long long)n_left;
    }
#endif
#if defined(VISO_PROBE) && !defined(VISO_PROBE_LIGHT)
    if (a.bg_drain && lane == 0) atomicMax(&g_probe_lk[22], ~__builtin_amdgcn_s_memrealtime());  // drain start
#endif
    int h = 0;
    int pend_head = -1, pend_k = 0;  // the second item of the last dequeue
    for (;;) {
        int head = 0, k = 0;
#ifdef VISO_PROBE
        pr_src = pend_head >= 0 ? 2 : left_phase ? 1 : 0;
#endif
        if (pend_head >= 0) {
            head = pend_head;
            k = pend_k;
            pend_head = -1;
        } else if (left_phase) {
            int j = 0;
            if (lane == 0) j = atomicAdd(a.bg_left, 1);
            j = __builtin_amdgcn_readfirstlane(j);
            if (j >= n_left) {
                left_phase = false;
                continue;
            }
            int e = 0;
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            while ((e = __builtin_amdgcn_readfirstlane(
                        __hip_atomic_load(a.bg_left + 32 + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) == 0) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > kBgWaitTicks) {
                    if (lane == 0) bg_fail(a);
                    return;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            head = (e - 1) / per_head;
            k = (e - 1) - head * per_head;
        } else {
            if (h >= 8) {
#ifdef VISO_PROBE
                if (lane == 0 && pr_w < kProbeWaves) {
                    g_probe_waves[pr_w][1] = __builtin_amdgcn_s_memrealtime();
                    g_probe_waves[pr_w][2] = (unsigned long long)pr_items;
                }
#endif
                break;
            }
            head = (xcc + h) & 7;
            // a wave past its own head looks first: an exhausted head costs a
            // load, not an atomic (thousands of waves walking the heads at the
            // chunk's end would otherwise queue behind each other on eight
            // words).  A drain wave at its own head does not: the head holds
            // the last frame's points then, and a look ahead of every
            // dequeue doubled the operations on those eight words.
#ifdef VISO_DRAIN_PEEK_OWN
            if ((h > 0 || a.bg_drain) &&
#else
            if (h > 0 &&
#endif
                __builtin_amdgcn_readfirstlane(__hip_atomic_load(a.bg_next + 32 * head, __ATOMIC_RELAXED,
                                                                 __HIP_MEMORY_SCOPE_AGENT)) >= per_head) {
                ++h;
                continue;
            }
            // two items per dequeue: half the head round trips per item
            if (lane == 0) k = atomicAdd(a.bg_next + 32 * head, kBgTake);
            k = __builtin_amdgcn_readfirstlane(k);
            if (k >= per_head) {
                ++h;
                continue;
            }
            if (kBgTake > 1 && k + 1 < per_head) {
                pend_head = head;
                pend_k = k + 1;
            }
        }
#ifdef VISO_PROBE
        t_deq = __builtin_amdgcn_s_memrealtime();
#endif
        if (!run_item(head, k)) {
            // the second item of the dequeue goes to the list too, or, when
            // the list is closed, is run here
            if (pend_head >= 0 && !give_back(pend_head, pend_k)) (void)run_item(pend_head, pend_k);
            return;
        }
#ifdef VISO_DRAIN_COUNT
        // (dev) items the drain ran: one same-address atomic per item, ~1,500
        // of them queued on one L2 channel in the chunk's tail
        if (a.bg_drain && lane == 0) atomicAdd(a.bg_err + 1, 1);
#endif
#ifdef VISO_PROBE
        ++pr_items;
#endif
    }
}

}  // namespace

void launch_klt(const FrameDev& ref, const FrameDev& cur, const PyrGeom& g, const float2* kp1,
                float2* kp2, uint8_t* success, int n, double thresh, hipStream_t stream) {
    if (n <= 0) return;
    klt_kernel<<<(n + 3) / 4, 256, 0, stream>>>(ref, cur, make_pyrdev(g), kp1, kp2, success, n,
                                                 thresh, nullptr);
}

void launch_klt_dev(const FrameDev& ref, const FrameDev& cur, const PyrGeom& g, const float2* kp1,
                    float2* kp2, uint8_t* success, const int* n_dev, int cap, double thresh, hipStream_t stream) {
    if (cap <= 0) return;
    // one wave per track of the capacity; waves past the device count return
    const int blocks = (cap + 3) / 4;
    klt_kernel<<<blocks, 256, 0, stream>>>(ref, cur, make_pyrdev(g), kp1, kp2, success, cap, thresh, n_dev);
}

void launch_lk_align(const LkAlignArgs& a, hipStream_t stream) {
    if (a.n <= 0 || a.n_frames <= 0) return;
    const int gx = (((a.n + 3) / 4) + 7) / 8 * 8;  // multiple of 8: XCD-stable point groups
    if (a.fast)
        lk_align_kernel<true><<<dim3(gx, a.n_frames), 256, 0, stream>>>(a);
    else
        lk_align_kernel<false><<<dim3(gx, a.n_frames), 256, 0, stream>>>(a);
}

// the background kernel's LDS request: static windows + dynamic = 84 KB, so
// two never share a CU (2 x 84 > 160 KB) while one leaves room for a 12-wave
// direct-pose workgroup (84 + 68 <= 160 KB)
constexpr size_t kBgLdsTotal = 84 * 1024;
// the resident grid's dynamic LDS per precision: its request minus the
// kernel's own static LDS (read from the code object, windows and per-wave
// poses, rather than restated here); the kernels' attributes are raised to
// it once.  (A round-5 variant that prefetched every level's template and
// window into the wave's LDS at item start made the tail 105-126 us instead
// of 81-84: spills at item start and fewer co-resident drain workgroups.)
static size_t lk_bg_dyn_lds(bool fast) {
    // (a function-local static's initialiser runs once, thread-safely:
    // contexts may be created from several host threads)
    struct Dyn {
        size_t v[2] = {0, 0};
        Dyn() {
            const void* k[2] = {(const void*)lk_item_kernel<false>, (const void*)lk_item_kernel<true>};
            for (int j = 0; j < 2; ++j) {
                hipFuncAttributes fa{};
                size_t st = 4 * 2 * kWinW * kWinH;
                if (hipFuncGetAttributes(&fa, k[j]) == hipSuccess) st = fa.sharedSizeBytes;
                v[j] = kBgLdsTotal > st ? kBgLdsTotal - st : 0;
                (void)hipFuncSetAttribute(k[j], hipFuncAttributeMaxDynamicSharedMemorySize, (int)v[j]);
            }
            (void)hipGetLastError();
        }
    };
    static const Dyn dyn;
    return dyn.v[fast ? 1 : 0];
}
void launch_lk_bg(const LkAlignArgs& a, int grid, hipStream_t stream) {
    if (a.n <= 0 || a.bg_items <= 0 || grid <= 0) return;
    const size_t dyn = lk_bg_dyn_lds(a.fast);
    if (a.fast)
        lk_item_kernel<true><<<grid, 256, dyn, stream>>>(a);
    else
        lk_item_kernel<false><<<grid, 256, dyn, stream>>>(a);
}

// The background kernel's one-time costs (its dynamic-LDS attribute, the
// first launch of both precisions) at context init: a one-workgroup launch
// with no frames returns at once.
void warm_lk_bg(hipStream_t stream) {
    (void)lk_bg_dyn_lds(false);
    LkAlignArgs a{};
    a.n_frames = 0;
    lk_item_kernel<true><<<1, 256, 0, stream>>>(a);
    lk_item_kernel<false><<<1, 256, 0, stream>>>(a);
}

void launch_lk_drain(const LkAlignArgs& a, int grid, hipStream_t stream) {
    if (a.n <= 0 || a.bg_items <= 0 || grid <= 0) return;
    if (a.fast)
        lk_item_kernel<true><<<grid, 256, 0, stream>>>(a);
    else
        lk_item_kernel<false><<<grid, 256, 0, stream>>>(a);
}

void launch_lk_template(const LkAlignArgs& a, hipStream_t stream) {
    if (a.n <= 0) return;
    lk_template_kernel<<<(a.n + 3) / 4, 256, 0, stream>>>(a);
}

namespace {
// One workgroup per batch row: the row's pair / success counts (integer
// sums, order-free) into the per-frame log.  Off the product path unless
// the caller enabled the log (viso_set_frame_log).
__global__ __launch_bounds__(256) void lk_count_kernel(const int32_t* __restrict__ pair_kf,
                                                       const uint8_t* __restrict__ success, size_t stride, int n,
                                                       LkCountArgs rows, double* __restrict__ flog) {
    const int idx = rows.idx[blockIdx.x];
    if (idx < 0) return;
    const int32_t* pk = pair_kf + stride * blockIdx.x;
    const uint8_t* sc = success + stride * blockIdx.x;
    int pairs = 0, succ = 0;
    for (int i = threadIdx.x; i < n; i += 256) {
        pairs += pk[i] >= 0;
        succ += sc[i] != 0;
    }
    for (int o = 32; o > 0; o >>= 1) {
        pairs += __shfl_xor(pairs, o);
        succ += __shfl_xor(succ, o);
    }
    __shared__ int s[2][4];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s[0][w] = pairs;
        s[1][w] = succ;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        flog[4 * (size_t)idx + 2] = (double)((s[0][0] + s[0][1]) + (s[0][2] + s[0][3]));
        flog[4 * (size_t)idx + 3] = (double)((s[1][0] + s[1][1]) + (s[1][2] + s[1][3]));
    }
}
}  // namespace

void launch_lk_count(const int32_t* pair_kf, const uint8_t* success, size_t stride, int n, int n_rows,
                     const LkCountArgs& rows, double* flog, hipStream_t stream) {
    if (!flog || n_rows <= 0 || n_rows > kLkBatch) return;
    lk_count_kernel<<<n_rows, 256, 0, stream>>>(pair_kf, success, stride, n < 0 ? 0 : n, rows, flog);
}

}  // namespace viso

#ifdef VISO_PROBE
extern "C" int viso_debug_probe_items(unsigned long long* out, int cap, int reset) {
    const int n = cap < kProbeItems ? cap : kProbeItems;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_probe_items), sizeof(unsigned long long) * 16 * n) != hipSuccess)
        return -2;
    if (reset) {
        void* p = nullptr;
        if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_probe_items)) != hipSuccess) return -2;
        if (hipMemset(p, 0, sizeof(g_probe_items)) != hipSuccess) return -2;
    }
    return n;
}

extern "C" int viso_debug_probe_waves(unsigned long long* out, int cap, int reset) {
    const int n = cap < kProbeWaves ? cap : kProbeWaves;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_probe_waves), sizeof(unsigned long long) * 4 * n) != hipSuccess)
        return -2;
    if (reset) {
        void* p = nullptr;
        if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_probe_waves)) != hipSuccess) return -2;
        if (hipMemset(p, 0, sizeof(g_probe_waves)) != hipSuccess) return -2;
    }
    return n;
}

extern "C" int viso_debug_probe_lk(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_probe_lk), sizeof(unsigned long long) * 32) != hipSuccess)
        return -2;
    if (reset) {
        static unsigned long long zero[32] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_probe_lk), zero, sizeof(zero)) != hipSuccess) return -2;
    }
    return 0;
}
#endif
