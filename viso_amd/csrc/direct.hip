// viso_amd — direct photometric 6-DoF Gauss-Newton pose for gfx950
// (DirectPoseEstimationSingleLayer / MultiLayer + dPixeldXi,
// src/viso.cpp:640-766).
//
// One frame = four launches on one stream in steady state:
//   L(3), L(2), L(1), L(0)   (+ F, the final level-0 solve, which normally
//   runs fused into the next frame's L(3); only the last frame of an ingest
//   call gets a standalone F launch)
// L(l) (one 12-wave workgroup per tile):
//   prologue — every workgroup solves level l+1 from that level's tile
//     partials (written by L(l+1)) and gets T21 for level l.  All workgroups
//     compute the same bits, so no grid-wide hand-off is needed beyond the
//     kernel boundary.  L(3) instead seeds T21 = SE3(R, t) of the last
//     frame's pose (src/viso.cpp:114), or, fused, solves the previous
//     frame's level 0 first.
//     Work that does not depend on T21 is issued first: the tile partial
//     loads of level l+1, and (waves off the solver's SIMD) the tile's map
//     points, their projections into the last frame, the `last` patch taps
//     and a current-image window around the predicted projection.
//   tiles — one wave per map point, lane = patch pixel: J = -grad^T *
//     dPixel/dXi, the 28 sums (21 upper-triangle J J^T, 6 -e J, e^2) by
//     reduce-scatter (the canonical wave tree, common.hpp).  A workgroup owns
//     a tile of T = map_tile(n, 256) = min(64, ceil(n / 256)) consecutive
//     points (247 tiles of 10 at 2,465 points), so there are at most 256
//     tiles; the tile's 28 sums are a tree over its points, stored k-major
//     per level ([28][256]).
// F (one workgroup): solves level 0 and writes the pose (+ pose log).
//
// The solve (one level, replicated in every workgroup): tile t's partials in
// thread t, a canonical tree over the tiles (reduce-scatter per wave, then
// the 4 waves); then on wave 0 alone: Eigen PartialPivLU of H replicated in
// every lane's registers (direct_solve.hpp; the pivot row made wave-uniform),
// the inverse with lane c solving column c, update = H^-1 b,
// SE3::exp(update) * T21 (sin/cos of theta/2 and theta in two lanes at once),
// cost / nGood and the checks of :741-753.  Every element sees the same operations in the same order as the
// sequential oracle, so the result is bit-identical.
// As shipped the loop takes exactly one GN step per level (cost is never
// reset, src/viso.cpp:673); the rare continuation (a level
// whose photometric cost is exactly 0) is executed faithfully by each
// workgroup on its own, re-evaluating every tile into private scratch.
#include <algorithm>
#include <cstring>

#include "device_math.hpp"
#include "direct_solve.hpp"
#include "kernels.hpp"

// Phase probes (build with VISO_VARIANT=probe; tools/probe_direct.py).
// Block 0 keeps s_memrealtime stamps (100 MHz) of its phases in scalar
// registers (every lane of the stamping wave takes the same value) and
// stores them once, with plain stores, at its exit into a ring slot per
// launch; every block's thread 0 raises the launch's exit stamp by a
// non-returning atomic max.  No stamp waits on memory, so the probe does not
// lengthen the phases it measures.  Stamps: 0 entry, 1 wave 0's partials
// reduced, 2 the solver starts (S combined), 3 LU, 4 inverse, 5 update,
// 6 SE3 exp, 7 solve finished, 8 after B2, 9 the last prefetch wave of block
// 0 done (LDS max), 10 block 0's tiles evaluated, 11 block 0 exit; 15 meta =
// (level + 1) | merged << 8 | n_tiles << 16.
#ifdef VISO_PROBE
constexpr int kPRing = 4096;
constexpr int kPSt = 16;
__device__ unsigned long long g_plog[kPRing][kPSt];
__device__ unsigned long long g_pexit[kPRing];
// per-block entry / exit stamps of the last kPRingB launches
constexpr int kPRingB = 512;
__device__ unsigned long long g_pblk[kPRingB][256][4];  // entry, after B2, wave 0's points done, exit
// per block of the last kPRingB launches: [w] wave w's points evaluated
// (w < 16), [15] the last arriver's tile trees stored
__device__ unsigned long long g_pwave[kPRingB][256][16];
#ifdef VISO_PROBE_PT
// (probe) phases of each wave's point in blocks < 32 of the last 128
// launches: entry, quotients, samples, six sums reduced, 28 sums formed
constexpr int kPtRing = 128, kPtBlocks = 32, kPtStamps = 5;
__device__ unsigned long long g_ppt[kPtRing][kPtBlocks][16][kPtStamps];
#define PPT(k)                                                                                       \
    do {                                                                                             \
        if (blockIdx.x < kPtBlocks && (threadIdx.x & 63) == 0)                                       \
            g_ppt[a.probe_seq & (kPtRing - 1)][blockIdx.x][threadIdx.x >> 6][(k)] =                  \
                __builtin_amdgcn_s_memrealtime();                                                    \
    } while (0)
#endif
#define PROBE_DECL()                                \
    __shared__ unsigned long long pst[kPSt];        \
    const unsigned long long probe_t0 = __builtin_amdgcn_s_memrealtime()
// lane 0 of the calling wave (block 0) records stamp k in LDS
#define PST(k)                                                                       \
    do {                                                                             \
        if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) pst[(k)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define PROBE_DECL()
#define PST(k)
#endif
#ifndef VISO_PROBE_PT
#define PPT(k) ((void)0)
#endif

namespace viso {

namespace {

constexpr int kSums = 28;
// waves per workgroup of the direct pose (one map point per wave; 12: three
// 128-VGPR waves per SIMD, so a CU keeps one wave slot per SIMD and LDS for
// the background LK alignment's workgroup, track.hip lk_item_kernel) and of
// the rig (four partial-reduction waves per camera)
#ifndef VISO_DIRECT_WAVES
#define VISO_DIRECT_WAVES 12
#endif
constexpr int kWaves = VISO_DIRECT_WAVES;
constexpr int kThreads = kWaves * 64;
constexpr int kRigWaves = 16;
constexpr int kRigThreads = kRigWaves * 64;
constexpr int kMaxTiles = 256;
constexpr int kMaxTile = kMaxMapPoints / kMaxTiles;  // 64 points

// Points per tile of the canonical map tree (oracle_common.hpp map_tile):
// min(64, max(1, ceil(n / groups))).
inline int map_tile(int n, int groups) {
    int t = (n + groups - 1) / groups;
    return t < 1 ? 1 : (t > kMaxTile ? kMaxTile : t);
}
constexpr int kStats = 50;
constexpr int kStateStride = 8;
// pre_hdr bit 17: a background LK alignment grid shares the CUs (its waves
// run at priority 0): the direct pose's waves run at 1 (the solver at 3)
constexpr int kHdrBg = 1 << 17;

// The two frames of one DirectPoseEstimation call and the `last` pose the
// patches are taken at (Keyframe::Project of last_frame, src/viso.cpp:697).
struct FramePair {
    FrameDev last;
    FrameDev cur;
    const double* pose_last;  // 12 doubles (may point into LDS)
};

// One level of a FramePair (the per-level image pointers resolved once, so no
// local copy of a FrameDev array is ever indexed at run time).
struct LevelPair {
    const uint8_t* last;
    const uint8_t* cur;
    const double* pose_last;
};

__device__ inline LevelPair level_pair(const FramePair& fp, int lv) {
    return LevelPair{fp.last.l[lv], fp.cur.l[lv], fp.pose_last};
}

struct DirectArgs {
    FramePair fp;
    PyrDev g;
    Intrinsics K;
    const double* points;
    int n;
    const double* pose_seed;  // level 3 starts at SE3(R, t) of this pose (12)
    int level;                // tiles of this level; -1: final solve only
    int tile;                 // points per tile (map_tile(n, 256) <= 64); split: the max
    int n_tiles;              // <= 256
    int split;                // tolerance mode: workgroup b owns points
                              // [b n / n_tiles, (b + 1) n / n_tiles) (all CUs busy;
                              // no canonical tree to keep)
    DirectScratch s;
    double* stats;     // [kLevels][kStats] or null
    double* pose_out;  // result pose (12) or null
    double* log;
    int log_index;  // < 0: no log append
    // the log's copy in the context's pinned staging (device address of the
    // host buffer, same index) or null (log_pose)
    double* log_host;
    double* prev_log_host;
    // L(3) fused with the previous frame's final solve (merged != 0): the
    // prologue solves the previous frame's level 0, writes its pose (+ log),
    // and seeds T21 from it (it is this frame's `last` pose)
    int merged;
    int probe_seq;   // probe builds: the launch's ring slot
    FramePair prev;  // the previous frame's pair (its rare continuation)
    double* prev_pose_out;
    double* prev_log;
    int prev_log_index;
    // background LK alignment (track.hip lk_item_kernel): raised (agent scope)
    // once the frame pose (pose_out / prev_pose_out) is stored; may be null
    int* ready;
    int* prev_ready;
    // the per-frame log (viso_set_frame_log; may be null): [log index][4]
    // doubles, the level-0 solve's nGood and cost written here beside the
    // pose log entry (LK pair / success counts by lk_count_kernel)
    double* flog;
};

// The frame pose of a direct-pose launch: 12 agent-scope (sc1) stores by one
// lane, then, when a background LK alignment waits for it, that lane's
// vmcnt(0) and the frame's ready flag (MI355X_MICROARCH.md, first row of the
// sc1 hand-off table).  The plain-launch readers see it either way.
__device__ inline void store_frame_pose(double* dst, const double* pose, int* ready) {
#pragma unroll
    for (int k = 0; k < 12; ++k) __hip_atomic_store(dst + k, pose[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (ready) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(ready, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// A logged pose (one thread), and its copy in the context's pinned staging
// when given: system-scope stores the host reads after its stream sync, so
// viso_synchronize enqueues no copy of the poses (round 5: one copy launch
// at the end of every ingest call).
__device__ inline void log_pose(double* log, double* log_host, int index, const double* pose) {
    if (!log || index < 0) return;
    for (int k = 0; k < 12; ++k) log[12 * (size_t)index + k] = pose[k];
    if (log_host)
        for (int k = 0; k < 12; ++k)
            __hip_atomic_store(log_host + 12 * (size_t)index + k, pose[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// A logged frame's level-0 nGood and cost (the solve's, the values
// viso_get_frame_stats reports as [9] and [10]); one thread, beside log_pose.
__device__ inline void log_frame(double* flog, int index, const SolveLds& L) {
    if (!flog || index < 0) return;
    flog[4 * (size_t)index + 0] = (double)L.ngood;
    flog[4 * (size_t)index + 1] = L.cost;
}

// The map points of workgroup (tile) b: [*first, *first + *cnt).
__device__ inline void tile_range(const DirectArgs& a, int b, int* first, int* cnt) {
    if (a.split) {
        const int f = (int)(((long long)b * a.n) / a.n_tiles);
        *first = f;
        *cnt = (int)(((long long)(b + 1) * a.n) / a.n_tiles) - f;
    } else {
        *first = b * a.tile;
        *cnt = a.tile;  // points past n are skipped (+0.0 leaves)
    }
}

// dPixeldXi (src/viso.cpp:640-658)
__device__ inline void d_pixel_d_xi(const Intrinsics& K, const double* pose, const double* P,
                                    double scale, double* J) {
    double Pc[3];
    mat3_vec(pose, P, Pc);
    Pc[0] = Pc[0] + pose[9];
    Pc[1] = Pc[1] + pose[10];
    Pc[2] = Pc[2] + pose[11];
    const double x = Pc[0], y = Pc[1], z = Pc[2];
    const double fx = K.fx * scale, fy = K.fy * scale;
    const double zz = z * z, xy = x * y;
    J[0] = fx / z;
    J[1] = 0;
    J[2] = -fx * x / zz;
    J[3] = -fx * xy / zz;
    J[4] = fx + fx * x * x / zz;
    J[5] = -fx * y / z;
    J[6] = 0;
    J[7] = fy / z;
    J[8] = -fy * y / zz;
    J[9] = -fy - fy * y * y / zz;
    J[10] = fy * xy / zz;
    J[11] = fy * x / z;
}

// The part of one map point that does not depend on T21: the point, its
// projection into the last frame (src/viso.cpp:697) and the `last` patch
// sample.  sample_px is split in two so the tap loads can be issued early and
// combined after a barrier: ref_issue loads the four tap bytes, ref_finish
// forms the bilinear value with sample_px's exact expression.
struct RefSample {
    double P[3];
    double ur, vr;
    double xx, yy;
    double lval;
    int t0, t1, t2, t3;
    bool ok;
};

__device__ inline void ref_issue(const DirectArgs& a, const LevelPair& fp, int lv, int i,
                                 RefSample& r) {
    const int lane = threadIdx.x & 63;
    const int px = (lane >> 3) - 4, py = (lane & 7) - 4;
    const double scale = kScale[lv];
    const int w = a.g.w[lv], h = a.g.h[lv];
    r.P[0] = a.points[3 * i];
    r.P[1] = a.points[3 * i + 1];
    r.P[2] = a.points[3 * i + 2];
    project_px(fp.pose_last, a.K, r.P, scale, r.ur, r.vr);
    const double hp = 4.0;
    r.ok = inside_px(r.ur - hp, r.vr - hp, w, h) && inside_px(r.ur + hp, r.vr + hp, w, h);
    const double x = r.ur + px, y = r.vr + py;
    const uint8_t* img = fp.last;
    const long long n = (long long)w * (long long)h;
    const long long base = r.ok ? (long long)(int)y * (long long)w + (long long)(int)x : -(1LL << 40);
    r.t0 = ld_u8_or0(img, n, base);
    r.t1 = ld_u8_or0(img, n, base + 1);
    r.t2 = ld_u8_or0(img, n, base + w);
    r.t3 = ld_u8_or0(img, n, base + w + 1);
    r.xx = x - floor(x);
    r.yy = y - floor(y);
}

__device__ inline void ref_finish(RefSample& r) {
    const double d0 = (double)r.t0, d1 = (double)r.t1, d2 = (double)r.t2, d3 = (double)r.t3;
    const double xx = r.xx, yy = r.yy;
    r.lval = r.ok ? double((1 - xx) * (1 - yy) * d0 + xx * (1 - yy) * d1 + (1 - xx) * yy * d2 +
                           xx * yy * d3)
                  : 0.0;
}

// Per-wave LDS window (16 x 16 bytes) of the current image around the
// point's projection under a predicted T21 (the previous level's starting
// pose), loaded while the prologue solves.  A sample whose four taps lie in
// the window (itself inside the image, so no tap wraps a row or leaves the
// buffer) reads the same bytes from LDS; any other takes sample_px's path.
constexpr int kCW = 20;  // window side: +-4..5 px of prediction error still hit
constexpr int kCWBytes = kCW * kCW;
constexpr int kCWLoads = (kCWBytes + 63) / 64;  // bytes per lane

struct CurWin {
    int x0, y0;
    bool on;
    uint8_t b[kCWLoads];  // this lane's bytes e = lane + 64 k of the row-major window
};

__device__ inline void win_issue(const uint8_t* __restrict__ img, int w, int h, double u, double v,
                                 CurWin& c) {
    c.on = w >= kCW && h >= kCW && u > -1e6 && u < 1e6 && v > -1e6 && v < 1e6;
    c.x0 = 0;
    c.y0 = 0;
    if (!c.on) return;
    int x0 = (int)floor(u) - kCW / 2 + 1;
    int y0 = (int)floor(v) - kCW / 2 + 1;
    x0 = min(max(x0, 0), w - kCW);
    y0 = min(max(y0, 0), h - kCW);
    c.x0 = x0;
    c.y0 = y0;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < kCWLoads; ++k) {
        const int e = lane + 64 * k;
        const int r = e / kCW, col = e - r * kCW;
        c.b[k] = ld_global_u8(img, (long long)(y0 + min(r, kCW - 1)) * w + x0 + col);
    }
}

__device__ inline void win_store(uint8_t* lds, const CurWin& c) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < kCWLoads; ++k) {
        const int e = lane + 64 * k;
        if (e < kCWBytes) st_lds_u8(lds, e, c.b[k]);
    }
}

#ifdef VISO_PROBE
// (probe) current-image samples that missed their LDS window, per level
// [0..3]; merged L(3) points whose `last` taps some lane reloaded [4], and
// all merged L(3) points [5].  Counted only in VISO_PROBE_PFB builds: they
// are same-address device atomics (one per missed sample, one or two per
// merged-L(3) point: ~4,900 per merged launch serialised on one L2 channel),
// and in the plain probe build they stretched every merged L(3) launch from
// ~14 to ~34 us — the probe measured itself
#ifdef VISO_PROBE_PFB
#define PFB_ADD(k) atomicAdd(&g_pfb[(k)], 1ull)
#else
#define PFB_ADD(k) ((void)0)
#endif
__device__ unsigned long long g_pfb[8];
#endif

// sample_px with the taps served from the window when all four lie in it
__device__ inline double sample_cw(const uint8_t* __restrict__ img, int w, int h, double x,
                                   double y, const uint8_t* win, const CurWin& c) {
    const bool finite = (x > -1e9 && x < 1e9 && y > -1e9 && y < 1e9);
    if (__builtin_expect(finite && c.on, 1)) {
        const int ix = (int)x, iy = (int)y;
        if (__builtin_expect(ix >= c.x0 && ix + 1 < c.x0 + kCW && iy >= c.y0 && iy + 1 < c.y0 + kCW, 1)) {
            const int o = (iy - c.y0) * kCW + (ix - c.x0);
            const double d0 = (double)ld_lds_u8(win, o), d1 = (double)ld_lds_u8(win, o + 1);
            const double d2 = (double)ld_lds_u8(win, o + kCW), d3 = (double)ld_lds_u8(win, o + kCW + 1);
            const double xx = x - floor(x);
            const double yy = y - floor(y);
            return double((1 - xx) * (1 - yy) * d0 + xx * (1 - yy) * d1 + (1 - xx) * yy * d2 +
                          xx * yy * d3);
        }
        // a sample on the image's last row: its lower taps lie past the
        // level buffer and read 0 (sample_px's rule), the upper two come from
        // the window (clamped to the bottom edge, it holds that row) — the
        // points near the bottom edge, ~10 % of them at level 3, no longer
        // wait for global loads
        if (iy == h - 1 && ix >= c.x0 && ix + 1 < c.x0 + kCW && iy >= c.y0 && iy < c.y0 + kCW) {
            const int o = (iy - c.y0) * kCW + (ix - c.x0);
            const double d0 = (double)ld_lds_u8(win, o), d1 = (double)ld_lds_u8(win, o + 1);
            const double d2 = 0.0, d3 = 0.0;
            const double xx = x - floor(x);
            const double yy = y - floor(y);
            return double((1 - xx) * (1 - yy) * d0 + xx * (1 - yy) * d1 + (1 - xx) * yy * d2 +
                          xx * yy * d3);
        }
    }
#ifdef VISO_PROBE
    PFB_ADD(w >= 1000 ? 0 : w >= 500 ? 1 : w >= 250 ? 2 : 3);
#endif
    return sample_px(img, w, h, x, y);
}

// The twelve quotients of one map point's projection (project_px) and
// dPixel/dXi (d_pixel_d_xi), each with those functions' exact operations,
// one per lane (lane k < 12) so that a single division sequence serves all
// of them; the projection's two go to every lane by readlane (Q), J's ten
// stay in their lanes (the return value; 0 in lanes >= 12).
//   0: x / z, 1: y / z (the projection)        -> Q[0], Q[1]
//   2..11: J[0], J[2], J[3], J[4], J[5], J[7], J[8], J[9], J[10], J[11]
__device__ inline double point_quotients(const Intrinsics& K, const double* pose, const double* P, double scale,
                                         double* Q, double* qt) {
    const int lane = threadIdx.x & 63;
    double Pc[3];
    mat3_vec(pose, P, Pc);
    const double x = Pc[0] + pose[9], y = Pc[1] + pose[10], z = Pc[2] + pose[11];
    const double fx = K.fx * scale, fy = K.fy * scale;
    const double zz = z * z, xy = x * y;
    // numerator = c1 * c2 (c2 = 1.0 where the numerator is a single value:
    // exact), denominator z or zz, per lane:
    //    0: x / z                1: y / z               2: fx / z      (J[0])
    //    3: -fx * x / zz (J[2])  4: -fx * xy / zz (J[3]) 5: fx*x * x / zz (J[4])
    //    6: -fx * y / z  (J[5])  7: fy / z   (J[7])      8: -fy * y / zz (J[8])
    //    9: fy*y * y / zz (J[9]) 10: fy * xy / zz (J[10]) 11: fy * x / z (J[11])
    // The operands come from a per-wave table of the twelve candidate values
    // in LDS, each lane reading its three at fixed per-lane slots (qt given:
    // the tile phase), or by lane-mask selects (26 v_cndmask: the tile phase
    // is VALU-issue-bound, LDS reads are not VALU; -0.6 us per frame,
    // profiles/r05_quotient_table_ab.log).  The twelve results go to every
    // lane by readlane (passing J's ten back through the table measured the
    // same).
    const double fxx = fx * x, fyy = fy * y;
    double c1, c2, den;
    if (qt) {
        // slots: 0 x, 1 y, 2 fx, 3 -fx, 4 fxx, 5 fy, 6 -fy, 7 fyy, 8 1.0, 9 xy, 10 z, 11 zz
        if (lane == 0) {
            double2* t2 = reinterpret_cast<double2*>(qt);
            t2[0] = make_double2(x, y);
            t2[1] = make_double2(fx, -fx);
            t2[2] = make_double2(fxx, fy);
            t2[3] = make_double2(-fy, fyy);
            t2[4] = make_double2(1.0, xy);
            t2[5] = make_double2(z, zz);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // per-lane slots, 4 bits each, lanes 0..11 (lanes >= 12 as lane 11)
        constexpr unsigned long long kC1 = 0x557653433210ULL, kC2 = 0x091181090888ULL,
                                     kDen = 0xABBBAABBBAAAULL;
        const int l = lane < 12 ? lane : 11;
        c1 = qt[(kC1 >> (4 * l)) & 15];
        c2 = qt[(kC2 >> (4 * l)) & 15];
        den = qt[(kDen >> (4 * l)) & 15];
    } else {
        c1 = fy;
        c1 = lane == 0 ? x : c1;
        c1 = lane == 1 ? y : c1;
        c1 = lane == 2 ? fx : c1;
        c1 = (lane == 3 || lane == 4 || lane == 6) ? -fx : c1;
        c1 = lane == 5 ? fxx : c1;
        c1 = lane == 8 ? -fy : c1;
        c1 = lane == 9 ? fyy : c1;
        c2 = 1.0;
        c2 = (lane == 3 || lane == 5 || lane >= 11) ? x : c2;
        c2 = (lane == 4 || lane == 10) ? xy : c2;
        c2 = (lane == 6 || lane == 8 || lane == 9) ? y : c2;
        den = (lane <= 2 || lane == 6 || lane == 7 || lane >= 11) ? z : zz;
    }
    double q = (c1 * c2) / den;
    if (lane == 5) q = fx + q;
    if (lane == 9) q = -fy - q;
    // the projection to every lane; J's ten stay in lanes 2..11 (the factored
    // sums fetch them per lane, direct_point_rs), lanes >= 12 hold J's zeros
    Q[0] = readlane_f64(q, 0);
    Q[1] = readlane_f64(q, 1);
    return lane < 12 ? q : 0.0;
}

// Source lanes of the four J entries lane k needs for sum k of the factored
// form (point_sums_factored): J[a], J[6 + a], J[b], J[6 + b] with (a, b) the
// k-th upper-triangle pair (k < 21) or a = k - 21 (b sums, k < 27).  J[j]
// sits in lane 2 (j = 0), j + 1 (j = 2..5) or j (j = 7..11) of
// point_quotients' result; J[1] = J[6] = 0 read lane 12.  Byte addresses for
// ds_bpermute, packed 8 bits each.  Per wave, once.
__device__ inline unsigned factored_sources() {
    const int k = threadIdx.x & 31;  // (lanes >= 28 unused)
    // per source s, 4 bits per lane: lanes 0-15 in lo[s], 16-27 in hi[s]
    constexpr unsigned long long lo[4] = {0x43333ccccc222222ULL, 0x9888877777ccccccULL, 0x465436543c6543c2ULL,
                                          0x9ba98ba987ba987cULL};
    constexpr unsigned long long hi[4] = {0x26543c265544ULL, 0xcba987cbaa99ULL, 0xccccccc66565ULL,
                                          0x7777777bbabaULL};
    unsigned r = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q)
        r |= (unsigned)((k < 16 ? lo[q] >> (4 * k) : hi[q] >> (4 * (k - 16))) & 15) << (8 * q);
    return r;
}

// The six patch sums of the factored form by reduce-scatter in DESCENDING
// xor order (partner lane ^ 32, ^ 16, ..., ^ 1: the pairwise tree of
// oracle_common.hpp tree_sum_desc64 for each value).  xor 32: the halves keep
// values 0-2 / 3-5 (v_permlane32_swap); xor 16: even rows keep the first,
// odd rows the third of their three, both rows the second (v_permlane16_swap);
// xor 8: lanes with bit 3 clear keep the row's first, the others the second
// (DPP row_ror:8 is the xor-8 partner); then one value per lane: xor 4 by
// row_shr / row_shl 4 + select, xor 2 / 1 by quad_perm.  Lane l ends with
// value 3 * b5 + (b3 ? 1 : b4 ? 2 : 0): value v in lanes 0, 8, 16, 32, 40, 48.
// Requires EXEC = all lanes.
__device__ inline double reduce_scatter_6_desc(const double* v) {
    const int lane = threadIdx.x & 63;
    const bool b2 = lane & 4, b3 = lane & 8;
    double a[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        double ra, rb;
        permlane32_swap_f64(v[k], v[3 + k], ra, rb);
        a[k] = ra + rb;
    }
    double ra, rb;
    permlane16_swap_f64(a[0], a[2], ra, rb);
    const double c0 = ra + rb;
    permlane16_swap_f64(a[1], a[1], ra, rb);
    const double c1 = ra + rb;
    double d = dsel(b3, c1, c0) + dpp_f64<0x128>(dsel(b3, c0, c1));
    const double r4 = dpp_f64<0x114>(d), l4 = dpp_f64<0x104>(d);  // row_shr / row_shl by 4
    d = d + dsel(b2, r4, l4);
    d = d + dpp_f64<0x4E>(d);  // lane ^ 2
    d = d + dpp_f64<0xB1>(d);  // lane ^ 1
    return d;
}

// The 28 sums of one map point (factored form, oracle direct_point_partials):
// returns good; lane k < 28 holds sum k in *out (*idx = k, -1 elsewhere).
// src_lanes: factored_sources() of this lane.
__device__ inline bool direct_point_rs(const DirectArgs& a, const LevelPair& fp, int lv,
                                       const double* cur_pose,
                                       const RefSample& r, const uint8_t* win, const CurWin& cw,
                                       double* out, int* idx, unsigned src_lanes, double* qt = nullptr) {
    const int lane = threadIdx.x & 63;
    const int px = (lane >> 3) - 4, py = (lane & 7) - 4;
    const double scale = kScale[lv];
    const int w = a.g.w[lv], h = a.g.h[lv];
    // project_px and d_pixel_d_xi (bit-identical; divisions lane-parallel)
    PPT(0);
    double Q[2];
    const double jq = point_quotients(a.K, cur_pose, r.P, scale, Q, qt);
    PPT(1);
    const double uc = scale * (Q[0] * a.K.fx + a.K.cx);
    const double vc = scale * (Q[1] * a.K.fy + a.K.cy);
    const double hp = 4.0;
    const bool good = r.ok && inside_px(uc - hp, vc - hp, w, h) && inside_px(uc + hp, vc + hp, w, h);
    if (!good) return false;
    const uint8_t* C = fp.cur;
    const double x = uc + px, y = vc + py;
    double error, g0, g1;
    // Whole patch in the window (wave-uniform, conservative: every lane's
    // samples at x, x +- 1 have int() bases in [floor(uc) - 6, floor(uc) + 5],
    // likewise in y): the five samples read LDS with no per-lane tests;
    // otherwise sample_cw decides per sample.
    const int fu = (int)floor(uc), fv = (int)floor(vc);
    if (__builtin_expect(cw.on && fu - 6 >= cw.x0 && fu + 5 <= cw.x0 + kCW - 2 && fv - 6 >= cw.y0 &&
                             fv + 5 <= cw.y0 + kCW - 2,
                         1)) {
        // uc - 6 .. uc + 6 (and vc's) in one binade: every lane's sample
        // coordinate uc + px + {-1, 0, 1} is then exact, its int() is
        // floor(uc) + px + {-1, 0, 1} (positive: the window test) and its
        // fraction is exactly frac(uc), so all five samples of all lanes share
        // one set of bilinear weights (the same products as the per-sample
        // form) and read 12 distinct taps per lane
        const bool one_binade = (__double_as_longlong(uc - 6.0) >> 52) == (__double_as_longlong(uc + 6.0) >> 52) &&
                                (__double_as_longlong(vc - 6.0) >> 52) == (__double_as_longlong(vc + 6.0) >> 52);
        if (__builtin_expect(one_binade, 1)) {
            const double xx = uc - floor(uc), yy = vc - floor(vc);
            const double w00 = (1 - xx) * (1 - yy), w10 = xx * (1 - yy), w01 = (1 - xx) * yy, w11 = xx * yy;
            // tap (-1, -1) of this lane: every tap below is a non-negative
            // immediate offset from it (one address, twelve ds_read_u8)
            const uint8_t* wb = win + ((fv + py - 1 - cw.y0) * kCW + (fu + px - 1 - cw.x0));
            auto tap = [&](int dx, int dy) { return (double)ld_lds_u8(wb, (dy + 1) * kCW + (dx + 1)); };
            const double tm0 = tap(-1, 0), t00 = tap(0, 0), t10 = tap(1, 0), t20 = tap(2, 0);
            const double tm1 = tap(-1, 1), t01 = tap(0, 1), t11 = tap(1, 1), t21 = tap(2, 1);
            const double t0m = tap(0, -1), t1m = tap(1, -1), t02 = tap(0, 2), t12 = tap(1, 2);
            auto bil = [&](double d0, double d1, double d2, double d3) {
                return double(w00 * d0 + w10 * d1 + w01 * d2 + w11 * d3);
            };
            error = r.lval - bil(t00, t10, t01, t11);
            // GetGradient (include/keyframe.h:57-64)
            g0 = 0.5 * (bil(t10, t20, t11, t21) - bil(tm0, t00, tm1, t01));
            g1 = 0.5 * (bil(t01, t11, t02, t12) - bil(t0m, t1m, t00, t10));
        } else {
            auto smp = [&](double sx, double sy) {
                const int o = ((int)sy - cw.y0) * kCW + ((int)sx - cw.x0);
                const double d0 = (double)ld_lds_u8(win, o), d1 = (double)ld_lds_u8(win, o + 1);
                const double d2 = (double)ld_lds_u8(win, o + kCW), d3 = (double)ld_lds_u8(win, o + kCW + 1);
                const double sxx = sx - floor(sx);
                const double syy = sy - floor(sy);
                return double((1 - sxx) * (1 - syy) * d0 + sxx * (1 - syy) * d1 + (1 - sxx) * syy * d2 +
                              sxx * syy * d3);
            };
            error = r.lval - smp(x, y);
            g0 = 0.5 * (smp(x + 1, y) - smp(x - 1, y));
            g1 = 0.5 * (smp(x, y + 1) - smp(x, y - 1));
        }
    } else {
        error = r.lval - sample_cw(C, w, h, x, y, win, cw);
        g0 = 0.5 * (sample_cw(C, w, h, x + 1, y, win, cw) - sample_cw(C, w, h, x - 1, y, win, cw));
        g1 = 0.5 * (sample_cw(C, w, h, x, y + 1, win, cw) - sample_cw(C, w, h, x, y - 1, win, cw));
    }
    // The factored sums (oracle direct_point_partials): J = -g^T Jp with Jp =
    // dPixel/dXi constant over the patch, so sum_p J J^T = Jp^T G Jp and
    // sum_p -e J = Jp^T (sum_p e g) with G = sum_p g g^T: six pixel sums
    // (descending-xor trees, oracle tree_sum_desc64) instead of 28
    PPT(2);
    const double leaf[6] = {g0 * g0, g0 * g1, g1 * g1, error * g0, error * g1, error * error};
    const double s = reduce_scatter_6_desc(leaf);
    PPT(3);
    // lane k < 28 forms sum k from the six and its four J entries
    const unsigned sa = src_lanes;
    const double p0a = bperm_f64(jq, (int)(sa & 0xff)), p1a = bperm_f64(jq, (int)((sa >> 8) & 0xff));
    const double p0b = bperm_f64(jq, (int)((sa >> 16) & 0xff)), p1b = bperm_f64(jq, (int)(sa >> 24));
    const double S0 = readlane_f64(s, 0), S1 = readlane_f64(s, 8), S2 = readlane_f64(s, 16);
    const double S3 = readlane_f64(s, 32), S4 = readlane_f64(s, 40), S5 = readlane_f64(s, 48);
    double o;
    if (lane < 21)
        o = (S0 * (p0a * p0b) + S1 * (p0a * p1b + p1a * p0b)) + S2 * (p1a * p1b);
    else if (lane < 27)
        o = S3 * p0a + S4 * p1a;
    else
        o = S5;
    *out = o;
    *idx = lane < kSums ? lane : -1;
    PPT(4);
    return true;
}

// ---------------------------------------------------------------- tolerance mode
// VISO_PRECISION_FAST: the point's projection and the good test stay fp64
// (the faithful decisions); then fp32 arithmetic.  The sub-pixel fraction of
// a projection is shared by all 64 patch pixels (their offsets are integers),
// so every lane's five samples (value, x +- 1, y +- 1) come from one 12-tap
// stencil (rows iy-1..iy+2, plus-shaped) with the same weights: from the
// LDS window when it holds the stencil, else from the level buffer
// (out-of-buffer taps 0).  dPixel/dXi, J, the 28 products and the reduce-
// scatter in fp32; the per-point sums are widened to fp64 for the tile and
// map trees.  Returns good; lane l < 32 with *idx >= 0 holds sum *idx.
__device__ inline float tap_f32(const uint8_t* __restrict__ img, long long n, long long i) {
    return (float)ld_u8_or0(img, n, i);
}

__device__ inline bool direct_point_fast(const DirectArgs& a, const LevelPair& fp, int lv, const double* cur_pose,
                                         const double* P, float lval, const uint8_t* win, const CurWin& cw,
                                         float* out, int* idx) {
    const int lane = threadIdx.x & 63;
    const int px = (lane >> 3) - 4, py = (lane & 7) - 4;
    const double scale = kScale[lv];
    const int w = a.g.w[lv], h = a.g.h[lv];
    // project_px's arithmetic, keeping the camera-frame point for dPixel/dXi
    double Pc[3];
    mat3_vec(cur_pose, P, Pc);
    Pc[0] = Pc[0] + cur_pose[9];
    Pc[1] = Pc[1] + cur_pose[10];
    Pc[2] = Pc[2] + cur_pose[11];
    const double uc = scale * ((Pc[0] / Pc[2]) * a.K.fx + a.K.cx);
    const double vc = scale * ((Pc[1] / Pc[2]) * a.K.fy + a.K.cy);
    const double hp = 4.0;
    if (!(inside_px(uc - hp, vc - hp, w, h) && inside_px(uc + hp, vc + hp, w, h))) return false;
    const float x = (float)Pc[0], y = (float)Pc[1], z = (float)Pc[2];
    const float fxs = (float)(a.K.fx * scale), fys = (float)(a.K.fy * scale);
    const float iz = 1.0f / z, iz2 = iz * iz;
    float Jp[12];
    Jp[0] = fxs * iz;
    Jp[1] = 0.0f;
    Jp[2] = -fxs * x * iz2;
    Jp[3] = -fxs * x * y * iz2;
    Jp[4] = fxs + fxs * x * x * iz2;
    Jp[5] = -fxs * y * iz;
    Jp[6] = 0.0f;
    Jp[7] = fys * iz;
    Jp[8] = -fys * y * iz2;
    Jp[9] = -fys - fys * y * y * iz2;
    Jp[10] = fys * x * y * iz2;
    Jp[11] = fys * x * iz;
    const double fu = floor(uc), fv = floor(vc);
    const float xx = (float)(uc - fu), yy = (float)(vc - fv);
    const int ix = (int)fu + px, iy = (int)fv + py;
    float t01, t02, t10, t11, t12, t13, t20, t21, t22, t23, t31, t32;
    if (cw.on && ix - 1 >= cw.x0 && ix + 2 < cw.x0 + kCW && iy - 1 >= cw.y0 && iy + 2 < cw.y0 + kCW) {
        const int o = (iy - cw.y0) * kCW + (ix - cw.x0);
        t01 = (float)ld_lds_u8(win, o - kCW);
        t02 = (float)ld_lds_u8(win, o - kCW + 1);
        t10 = (float)ld_lds_u8(win, o - 1);
        t11 = (float)ld_lds_u8(win, o);
        t12 = (float)ld_lds_u8(win, o + 1);
        t13 = (float)ld_lds_u8(win, o + 2);
        t20 = (float)ld_lds_u8(win, o + kCW - 1);
        t21 = (float)ld_lds_u8(win, o + kCW);
        t22 = (float)ld_lds_u8(win, o + kCW + 1);
        t23 = (float)ld_lds_u8(win, o + kCW + 2);
        t31 = (float)ld_lds_u8(win, o + 2 * kCW);
        t32 = (float)ld_lds_u8(win, o + 2 * kCW + 1);
    } else {
        const uint8_t* C = fp.cur;
        const long long n = (long long)w * h, o = (long long)iy * w + ix;
        t01 = tap_f32(C, n, o - w);
        t02 = tap_f32(C, n, o - w + 1);
        t10 = tap_f32(C, n, o - 1);
        t11 = tap_f32(C, n, o);
        t12 = tap_f32(C, n, o + 1);
        t13 = tap_f32(C, n, o + 2);
        t20 = tap_f32(C, n, o + w - 1);
        t21 = tap_f32(C, n, o + w);
        t22 = tap_f32(C, n, o + w + 1);
        t23 = tap_f32(C, n, o + w + 2);
        t31 = tap_f32(C, n, o + 2 * w);
        t32 = tap_f32(C, n, o + 2 * w + 1);
    }
    const float i0 = bilerp_f32(t11, t12, t21, t22, xx, yy);
    const float g0 = 0.5f * (bilerp_f32(t12, t13, t22, t23, xx, yy) - bilerp_f32(t10, t11, t20, t21, xx, yy));
    const float g1 = 0.5f * (bilerp_f32(t21, t22, t31, t32, xx, yy) - bilerp_f32(t01, t02, t11, t12, xx, yy));
    const float error = lval - i0;
    float J[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) J[k] = -__builtin_fmaf(g0, Jp[k], g1 * Jp[6 + k]);
    float leaf[kSums];
    int e = 0;
#pragma unroll
    for (int rr = 0; rr < 6; ++rr)
#pragma unroll
        for (int c = rr; c < 6; ++c) leaf[e++] = J[rr] * J[c];
#pragma unroll
    for (int k = 0; k < 6; ++k) leaf[21 + k] = -error * J[k];
    leaf[27] = error * error;
    *out = reduce_scatter_28_f32(leaf, idx);
    return true;
}

// The `last` sample of this lane's pixel in tolerance mode: the four taps
// (packed, sample_px's bytes) with the projection's shared fraction.
__device__ inline float fast_lval(uint32_t t, double ur, double vr) {
    const float xx = (float)(ur - floor(ur)), yy = (float)(vr - floor(vr));
    return bilerp_f32((float)(t & 0xff), (float)((t >> 8) & 0xff), (float)((t >> 16) & 0xff), (float)(t >> 24),
                      xx, yy);
}

// Prologue prefetch of a whole tile, in LDS: per point j of the tile its
// world point, its projection into the last frame (ur, vr, the bounds test)
// and the four `last` patch taps of every lane (sample_px's bytes, packed),
// and the 16 x 16 current-image window around its projection under the
// predicted T21.  Issued while wave 0 solves, so after the solve the tiles
// read nothing but LDS (and the rare sample outside its window).
struct PfLds {
    uint32_t taps[kMaxTile][64];
    // tolerance-mode rig: the `last` patch sample of every lane as fp16
    // (computed in the prefetch, off the tile phase's critical path)
    _Float16 lv16[kMaxTile][64];
    uint8_t win[kMaxTile][kCWBytes];
    double P[kMaxTile][3];
    double ur[kMaxTile], vr[kMaxTile];
    int ok[kMaxTile];
    int cw[kMaxTile][3];  // x0, y0, on
};

struct PfPoint {
    RefSample r;
    CurWin c;
};

__device__ inline void pf_issue(const DirectArgs& a, const LevelPair& fp, int lv, int i, const double* pred,
                                bool ref, PfPoint& q) {
    if (ref) {
        ref_issue(a, fp, lv, i, q.r);
    } else {
        q.r.P[0] = a.points[3 * i];
        q.r.P[1] = a.points[3 * i + 1];
        q.r.P[2] = a.points[3 * i + 2];
    }
    double up, vp;
    project_px(pred, a.K, q.r.P, kScale[lv], up, vp);
    win_issue(fp.cur, a.g.w[lv], a.g.h[lv], up, vp, q.c);
}

__device__ inline float fast_lval(uint32_t t, double ur, double vr);

template <bool LV16>
__device__ inline void pf_store(int j, bool ref, const PfPoint& q, PfLds& pf) {
    const int lane = threadIdx.x & 63;
    if (ref)
        pf.taps[j][lane] = (uint32_t)q.r.t0 | ((uint32_t)q.r.t1 << 8) | ((uint32_t)q.r.t2 << 16) |
                           ((uint32_t)q.r.t3 << 24);
    if (LV16) pf.lv16[j][lane] = (_Float16)(q.r.ok ? fast_lval(pf.taps[j][lane], q.r.ur, q.r.vr) : 0.0f);
    if (q.c.on) win_store(pf.win[j], q.c);
    if (lane == 0) {
        pf.P[j][0] = q.r.P[0];
        pf.P[j][1] = q.r.P[1];
        pf.P[j][2] = q.r.P[2];
        pf.ur[j] = ref ? q.r.ur : 0.0;
        pf.vr[j] = ref ? q.r.vr : 0.0;
        pf.ok[j] = (ref && q.r.ok) ? 1 : 0;
        pf.cw[j][0] = q.c.x0;
        pf.cw[j][1] = q.c.y0;
        pf.cw[j][2] = q.c.on ? 1 : 0;
    }
}

// Points j = first, first + stride, ... of tile b, two at a time (the loads
// of both in flight together).  `pose_last` is the pose of the `last`
// projection: the `last` frame's own, or in a merged L(3) (whose `last` pose
// is solved in this launch) a prediction, checked per lane in the tile phase.
template <bool LV16 = false>
__device__ void prefetch_tile(const DirectArgs& a, int lv, int b, const double* pred, const double* pose_last,
                              bool ref, int first, int stride, PfLds& pf, const FramePair* fpair = nullptr) {
    LevelPair fp = level_pair(fpair ? *fpair : a.fp, lv);
    fp.pose_last = pose_last;
    int p0, T;
    tile_range(a, b, &p0, &T);
    for (int j = first; j < T; j += 2 * stride) {
        const int j2 = j + stride;
        const int i0 = p0 + j, i1 = p0 + j2;
        const bool v0 = i0 < a.n, v1 = j2 < T && i1 < a.n;
        PfPoint q0{}, q1{};
        if (v0) pf_issue(a, fp, lv, i0, pred, ref, q0);
        if (v1) pf_issue(a, fp, lv, i1, pred, ref, q1);
        if (v0) pf_store<LV16>(j, ref, q0, pf);
        if (v1) pf_store<LV16>(j2, ref, q1, pf);
    }
}

// The RefSample of prefetched point j: sample_px's expression on the
// prefetched taps, with ref_issue's weights.
__device__ inline void pf_ref(const PfLds& pf, int j, RefSample& r) {
    const int lane = threadIdx.x & 63;
    const int px = (lane >> 3) - 4, py = (lane & 7) - 4;
    r.P[0] = pf.P[j][0];
    r.P[1] = pf.P[j][1];
    r.P[2] = pf.P[j][2];
    r.ur = pf.ur[j];
    r.vr = pf.vr[j];
    r.ok = pf.ok[j] != 0;
    const uint32_t t = pf.taps[j][lane];
    r.t0 = (int)(t & 0xff);
    r.t1 = (int)((t >> 8) & 0xff);
    r.t2 = (int)((t >> 16) & 0xff);
    r.t3 = (int)(t >> 24);
    const double x = r.ur + px, y = r.vr + py;
    r.xx = x - floor(x);
    r.yy = y - floor(y);
    ref_finish(r);
}

// The `last` sample of prefetched point j in a merged L(3): the projection
// under the solved `last` pose (ref_issue's arithmetic); the taps prefetched
// under the predicted pose are used where a lane's base pixel is the same,
// any other lane loads its four taps now (ref_issue's loads).
__device__ inline void merged_ref(const DirectArgs& a, const LevelPair& fp, int lv, const PfLds& pf, int j,
                                  RefSample& r) {
    const int lane = threadIdx.x & 63;
    const int px = (lane >> 3) - 4, py = (lane & 7) - 4;
    const int w = a.g.w[lv], h = a.g.h[lv];
    r.P[0] = pf.P[j][0];
    r.P[1] = pf.P[j][1];
    r.P[2] = pf.P[j][2];
    project_px(fp.pose_last, a.K, r.P, kScale[lv], r.ur, r.vr);
    const double hp = 4.0;
    r.ok = inside_px(r.ur - hp, r.vr - hp, w, h) && inside_px(r.ur + hp, r.vr + hp, w, h);
    const double x = r.ur + px, y = r.vr + py;
    r.xx = x - floor(x);
    r.yy = y - floor(y);
    r.t0 = r.t1 = r.t2 = r.t3 = 0;
    if (!r.ok) return;
    const long long base = (long long)(int)y * (long long)w + (long long)(int)x;
    const double xp = pf.ur[j] + px, yp = pf.vr[j] + py;
    const long long bp = pf.ok[j] ? (long long)(int)yp * (long long)w + (long long)(int)xp : -(1LL << 40);
#ifdef VISO_PROBE_PFB
    {
        const unsigned long long rl = __ballot(base != bp);
        if (lane == 0) {
            PFB_ADD(5);
            if (rl) PFB_ADD(4);
        }
    }
#endif
    if (__builtin_expect(base == bp, 1)) {
        const uint32_t t = pf.taps[j][lane];
        r.t0 = (int)(t & 0xff);
        r.t1 = (int)((t >> 8) & 0xff);
        r.t2 = (int)((t >> 16) & 0xff);
        r.t3 = (int)(t >> 24);
    } else {
        const uint8_t* img = fp.last;
        const long long n = (long long)w * (long long)h;
        r.t0 = ld_u8_or0(img, n, base);
        r.t1 = ld_u8_or0(img, n, base + 1);
        r.t2 = ld_u8_or0(img, n, base + w);
        r.t3 = ld_u8_or0(img, n, base + w + 1);
    }
}

// Tile b of level lv from the prologue's prefetch (the tile phase of
// direct_level_kernel; direct_tile's arithmetic and tree; FAST: the
// tolerance-mode point sums).
// Tiles of <= 16 points (maps up to 4,096 points) end without a block
// barrier: each wave that evaluated points adds itself to an LDS arrival
// count after its sums are in LDS, and the wave that arrives last forms the
// tile's 28 trees (lane k: tree over the 16 point slots, zeros past T, then
// the two +0 levels of the 64-lane tree, the same operations as
// wave_tree_sum_dpp on T slots) and stores them; the other waves are done.
// `last_arriver` = false (the continuation, which reuses s_pts in a loop)
// keeps the block-barrier form.
constexpr unsigned kSrcHere = 0xffffffffu;  // direct_tile_pf: factored_sources() computed there

template <bool FAST, bool LV16 = false, int W = kWaves>
__device__ void direct_tile_pf(const DirectArgs& a, const LevelPair& fp, int lv, const double* cur_pose, int b,
                               const PfLds& pf, bool merged, double* part, int* good, double* s_pts,
                               int* s_good, int* s_cnt = nullptr, double* s_qt = nullptr,
                               unsigned src_in = kSrcHere) {
    const int wave = wave_id(), lane = threadIdx.x & 63;
    int first, T;
    tile_range(a, b, &first, &T);
    int good_cnt = 0;
    const unsigned src_lanes = FAST ? 0u : src_in != kSrcHere ? src_in : factored_sources();
    for (int local = wave; local < T; local += W) {
        const int i = first + local;
        double f = 0.0;
        int idx = -1;
        bool ok = false;
        if (i < a.n) {
            RefSample r;
            if (merged) {
                merged_ref(a, fp, lv, pf, local, r);
                if (!FAST) ref_finish(r);
            } else if (!FAST) {
                pf_ref(pf, local, r);
            } else {
                r.P[0] = pf.P[local][0];
                r.P[1] = pf.P[local][1];
                r.P[2] = pf.P[local][2];
                r.ur = pf.ur[local];
                r.vr = pf.vr[local];
                r.ok = pf.ok[local] != 0;
                const uint32_t t = pf.taps[local][lane];
                r.t0 = (int)(t & 0xff);
                r.t1 = (int)((t >> 8) & 0xff);
                r.t2 = (int)((t >> 16) & 0xff);
                r.t3 = (int)(t >> 24);
            }
            CurWin cw;
            cw.x0 = pf.cw[local][0];
            cw.y0 = pf.cw[local][1];
            cw.on = pf.cw[local][2] != 0;
            if (FAST) {
                float ff = 0.0f;
                if (r.ok) {
                    const uint32_t t = (uint32_t)r.t0 | ((uint32_t)r.t1 << 8) | ((uint32_t)r.t2 << 16) |
                                       ((uint32_t)r.t3 << 24);
                    const float lval = (LV16 && !merged) ? (float)pf.lv16[local][lane] : fast_lval(t, r.ur, r.vr);
                    ok = direct_point_fast(a, fp, lv, cur_pose, r.P, lval, pf.win[local], cw, &ff, &idx);
                }
                f = (double)ff;
            } else {
                ok = direct_point_rs(a, fp, lv, cur_pose, r, pf.win[local], cw, &f, &idx, src_lanes,
                                     s_qt ? s_qt + 12 * wave : nullptr);
            }
        }
        if (!ok) {
            if (lane < kSums) s_pts[local * kSums + lane] = 0.0;
        } else if ((!FAST || lane < 32) && idx >= 0) {  // faithful: reduce_scatter_28_desc's map
            s_pts[local * kSums + idx] = f;
        }
        good_cnt += ok ? 1 : 0;
    }
    if (lane == 0 && good_cnt) atomicAdd(s_good, good_cnt);
#ifdef VISO_PROBE
    if (threadIdx.x == 0 && blockIdx.x < 256) g_pblk[a.probe_seq & (kPRingB - 1)][blockIdx.x][2] = __builtin_amdgcn_s_memrealtime();
    if (lane == 0 && blockIdx.x < 256 && wave < 15)
        g_pwave[a.probe_seq & (kPRingB - 1)][blockIdx.x][wave] = __builtin_amdgcn_s_memrealtime();
#endif
    if (s_cnt && T <= 16) {
        const int nw = T < W ? T : W;  // waves that evaluated points
        if (wave >= nw) return;
        int prev = 0;
        if (lane == 0)
            prev = __hip_atomic_fetch_add(s_cnt, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
        prev = __builtin_amdgcn_readfirstlane(prev);
        if (prev != nw - 1) return;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if (lane < kSums) {
            double v[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) v[j] = j < T ? s_pts[j * kSums + lane] : 0.0;
#pragma unroll
            for (int st = 1; st < 16; st <<= 1)
#pragma unroll
                for (int j = 0; j < 16; j += 2 * st) v[j] = v[j] + v[j + st];
            double r = v[0] + 0.0;  // lanes 16..31 (+0)
            r = r + 0.0;            // the other half wave (+0)
            part[(size_t)lane * kMaxTiles + b] = r;  // k-major: [28][256]
        }
        if (lane == 0) good[b] = __hip_atomic_load(s_good, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#ifdef VISO_PROBE
        if (lane == 0 && blockIdx.x < 256)
            g_pwave[a.probe_seq & (kPRingB - 1)][blockIdx.x][15] = __builtin_amdgcn_s_memrealtime();
#endif
        return;
    }
    __syncthreads();
    for (int k = wave; k < kSums; k += W) {
        const double v = lane < T ? s_pts[lane * kSums + k] : 0.0;
        const double r = wave_tree_sum_dpp(v);
        if (lane == 0) part[(size_t)k * kMaxTiles + b] = r;  // k-major: [28][256]
    }
    if (threadIdx.x == 0) good[b] = *s_good;
    __syncthreads();
}

__device__ inline void state_to_pose(const double* st, double* pose) {
    double q[4] = {st[0], st[1], st[2], st[3]};
    quat_to_matrix(q, pose);
    pose[9] = st[4];
    pose[10] = st[5];
    pose[11] = st[6];
}

// ---------------------------------------------------------------- solve

// Thread t < 256 loads tile t's partials (zeros beyond n_tiles).  The
// partials of a level are stored k-major ([28][256]: sum k of tile t at
// k * 256 + t), so each of a wave's 28 loads is one coalesced 512-byte run
// (4 cache lines) rather than 64 lines strided by a tile record.
__device__ inline void load_partials(const double* __restrict__ part, const int* __restrict__ good,
                                     int n_tiles, double* v, int& gg) {
    const int t = threadIdx.x;
    if (t < n_tiles) {
#pragma unroll
        for (int k = 0; k < kSums; ++k) v[k] = part[(size_t)k * kMaxTiles + t];
        gg = good[t];
    } else {
#pragma unroll
        for (int k = 0; k < kSums; ++k) v[k] = 0.0;
        gg = 0;
    }
}

// Canonical tree over <= 256 tiles (thread t holds tile t) -> L.S, L.ngood.
__device__ inline void reduce_partials(const double* v, int gg, SolveLds& L) {
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    if (t < 256) {
        int idx;
        const double f = reduce_scatter_28(v, &idx);
        if (lane < 32 && idx >= 0) L.red[wave][idx] = f;
        const int g = wave_sum_int(gg);
        if (lane == 0) L.g[wave] = g;
    }
    __syncthreads();
    if (t < kSums) L.S[t] = (L.red[0][t] + L.red[1][t]) + (L.red[2][t] + L.red[3][t]);
    if (t == 0) L.ngood = (L.g[0] + L.g[1]) + (L.g[2] + L.g[3]);
    __syncthreads();
}

// Barrier for LDS hand-offs only: waits for this wave's LDS operations, not
// for its global loads, so loads issued before it stay in flight (a
// __syncthreads() also drains vmcnt).
__device__ inline void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// GN iterations 1.. of level lv (the faithful continuation, rare): every
// workgroup re-evaluates all tiles of level lv of frame pair fpair itself at
// the new T21, into its own scratch, and solves again.  The tiles go through
// the tile phase's own prefetch + evaluation (all waves prefetch, then
// evaluate), so this rare path adds no register pressure to the kernel.
template <bool FAST>
__device__ void solve_continue(const DirectArgs& a, const FramePair& fpair, int lv, SolveLds& L,
                               double* stats, double* s_pose, double* s_pts, int* s_good, PfLds& pf) {
    const int t = threadIdx.x, wave = t >> 6;
    double* part = a.s.cont_part + (size_t)blockIdx.x * kMaxTiles * kSums;
    int* good = a.s.cont_good + (size_t)blockIdx.x * kMaxTiles;
    const LevelPair fp = level_pair(fpair, lv);
    for (int iter = 1; iter < 100 && L.cont; ++iter) {
        if (t == 0) state_to_pose(L.state, s_pose);
        __syncthreads();
        double pose[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) pose[k] = s_pose[k];
        for (int b = 0; b < a.n_tiles; ++b) {
            if (t == 0) *s_good = 0;
            prefetch_tile(a, lv, b, pose, fpair.pose_last, true, wave, kWaves, pf, &fpair);
            __syncthreads();
            direct_tile_pf<FAST>(a, fp, lv, pose, b, pf, false, part, good, s_pts, s_good);
        }
        __threadfence_block();
        __syncthreads();
        double v[kSums];
        int gg = 0;
        if (t < 256) load_partials(part, good, a.n_tiles, v, gg);
        reduce_partials(v, gg, L);
        if (wave == 0) {
            if (FAST)
                solve_wave0_ldlt(L, iter, stats);
            else
                solve_wave0(L, iter, stats);
        }
        __syncthreads();
    }
}

// Issue the T21-independent loads of map point i: the `last` patch taps and
// the current-image window around its projection under the predicted T21
// (the pose level sl was evaluated at, or the seed).  In a merged L(3) the
// `last` pose is solved in the same launch, so its taps are issued again
// after the solve; the early ones (projected with the stale pose, bounds-
// checked) are discarded.
__device__ inline void prefetch_point(const DirectArgs& a, int lv, int i, bool solve, int sl,
                                      RefSample& r, CurWin& cw) {
    ref_issue(a, level_pair(a.fp, lv), lv, i, r);
    double pred[12];
    if (!solve) {
        for (int k = 0; k < 12; ++k) pred[k] = a.pose_seed[k];
    } else {
        double sp[7];
        for (int k = 0; k < 7; ++k) sp[k] = a.s.state[sl * kStateStride + k];
        state_to_pose(sp, pred);
    }
    double up, vp;
    project_px(pred, a.K, r.P, kScale[lv], up, vp);
    win_issue(a.fp.cur.l[lv], a.g.w[lv], a.g.h[lv], up, vp, cw);
}

// After the solve of level sl: in a merged L(3), the solved T21 is the
// previous frame's pose -> written out (block 0), kept in LDS as this
// frame's `last` pose, and the seed SE3(R, t) of it becomes T21.  Then the
// pose the tiles are evaluated at.  One thread.
__device__ inline void after_solve(const DirectArgs& a, bool merged, SolveLds& L, double* s_last,
                                   double* s_pose) {
    if (merged) {
        state_to_pose(L.state, s_last);
        if (blockIdx.x == 0) {
            for (int k = 0; k < 7; ++k) a.s.state[kLevels * kStateStride + k] = L.state[k];
            if (a.prev_pose_out) store_frame_pose(a.prev_pose_out, s_last, a.prev_ready);
            log_pose(a.prev_log, a.prev_log_host, a.prev_log_index, s_last);
            log_frame(a.flog, a.prev_log_index, L);
        }
        // Sophus::SE3d(R, t) of last_frame (src/viso.cpp:114)
        double q[4];
        quat_from_matrix(s_last, q);
        for (int k = 0; k < 4; ++k) L.state[k] = q[k];
        L.state[4] = s_last[9];
        L.state[5] = s_last[10];
        L.state[6] = s_last[11];
    }
    state_to_pose(L.state, s_pose);
}

// L(level) and F (level = -1).
//   Wave 0 is the solver: it reduces its quarter of the tile partials of the
//   solved level, waits on an LDS arrival count for waves 1-3 (the other
//   quarters) and thread 256 (the T21 that level was evaluated at), then
//   solves.  No block barrier sits in front of the solve, so the other waves'
//   prefetches (their map point, `last` patch taps and current-image window;
//   wave 4 also prefetches wave 0's point) stay off its path.  B2 (block
//   barrier) hands the new pose to every wave; then the tiles.
// The three leading arguments repeat what the prologue's first loads need
// (the partials of the level it solves, their nGood counts, n_tiles | solve
// << 16): scalar arguments ahead of the by-value struct are preloaded into
// SGPRs at wave launch (-amdgpu-kernarg-preload-count, viso_amd/build.py), so
// the partial loads issue without waiting for a kernel-argument load.
template <bool FAST>
// (at most 128 VGPRs: four waves per SIMD, the fourth the background's)
__global__ __launch_bounds__(kThreads, 4) void direct_level_kernel(const double* __restrict__ pre_part,
                                                                 const int* __restrict__ pre_good, int pre_hdr,
                                                                 DirectArgs a) {
    PROBE_DECL();
    // the chain's waves outrank co-resident LK alignment waves (the
    // background grid, or a host-frame call's LK batch on the side stream)
    __builtin_amdgcn_s_setprio(1);
    __shared__ SolveLds L;
    __shared__ double s_pose[12];
    __shared__ double s_last[12];  // merged L(3): this frame's `last` pose
    __shared__ double s_pts[kMaxTile * kSums];
    __shared__ int s_good;
    __shared__ int s_cnt;  // waves done with their points (last-arriver tile tree)
    __shared__ int s_arrive;
    __shared__ PfLds s_pf;
#ifndef VISO_NO_QT
    // the quotient operand tables of the tile phase (point_quotients)
    __shared__ __attribute__((aligned(16))) double s_qt[FAST ? 2 : kWaves * 12];
    double* const qt = FAST ? nullptr : s_qt;
#else
    double* const qt = nullptr;
#endif
    const int lv = a.level;
    const bool merged = a.merged && lv == kLevels - 1;
    const int prev = lv + 1;
    const bool solve = prev < kLevels || merged;
    const int sl = merged ? 0 : prev;  // level solved in the prologue
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    const bool tiles = lv >= 0 && (int)blockIdx.x < a.n_tiles;
    // ---- the loads that need no LDS are issued first, so they are in flight
    // while the workgroup's waves arrive at the first barrier: the partials
    // of level sl (waves 0-3) and the T21 that level was evaluated at (thread
    // 256; every prefetch wave for its prediction)
    double v[kSums];
    int gg = 0;
    if (((pre_hdr >> 16) & 1) && t < 256) load_partials(pre_part, pre_good, pre_hdr & 0xffff, v, gg);
    const bool pf_wave = !solve || (wave & 3) != 0;
    double st[7];
    if (t == 256 || (solve && tiles && pf_wave)) {
        if (!solve) {
            // Sophus::SE3d(R, t): R -> quaternion
            quat_from_matrix(a.pose_seed, st);
            st[4] = a.pose_seed[9];
            st[5] = a.pose_seed[10];
            st[6] = a.pose_seed[11];
        } else {
#pragma unroll
            for (int k = 0; k < 7; ++k) st[k] = a.s.state[sl * kStateStride + k];
        }
    }
    if (t == 0) {
        s_arrive = 0;
        s_good = 0;
        s_cnt = 0;
#ifdef VISO_PROBE
        for (int k = 0; k < kPSt; ++k) pst[k] = 0;
        pst[0] = probe_t0;
        if (blockIdx.x < 256) g_pblk[a.probe_seq & (kPRingB - 1)][blockIdx.x][0] = probe_t0;
#endif
    }
    lds_barrier();  // the LDS words above; the global loads stay in flight

    if (t == 256) {
        for (int k = 0; k < 7; ++k) {
            L.state[k] = st[k];
            L.best[k] = st[k];
        }
        L.cost = 0.0;
        L.last_cost = 0.0;
        L.cont = 0;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        atomicAdd(&s_arrive, 1);
    }
    if (solve && t < 256) {
        int idx;
        const double f = reduce_scatter_28(v, &idx);
        if (lane < 32 && idx >= 0) L.red[wave][idx] = f;
        const int g = wave_sum_int(gg);
        if (lane == 0) L.g[wave] = g;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) atomicAdd(&s_arrive, 1);
    }
    if (wave == 0) PST(1);

    // ---- prefetch of the whole tile (every wave but the solver): the pose
    // the windows are predicted at is the seed (unsolved L(3)) or the T21
    // level sl was evaluated at
    const bool solver = solve && wave == 0;
    // the solver's SIMD (waves 0, 4, 8, 12: wave w runs on SIMD w % 4) is
    // left to the solver; its waves join the prefetch only when there is no
    // solve
    if (tiles && pf_wave) {
        double pred[12];
        if (!solve) {
            for (int k = 0; k < 12; ++k) pred[k] = a.pose_seed[k];
        } else {
            state_to_pose(st, pred);  // loaded above
        }
        const int first = solve ? wave - (wave >> 2) - 1 : wave;
        const int stride = solve ? kWaves - kWaves / 4 : kWaves;
        // merged: the `last` pose is this launch's solve of the previous
        // frame's level 0, predicted by the T21 that level was evaluated at
        prefetch_tile(a, lv, blockIdx.x, pred, merged ? pred : a.fp.pose_last, true, first, stride, s_pf);
#ifdef VISO_PROBE
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        if (blockIdx.x == 0 && lane == 0) atomicMax(&pst[9], __builtin_amdgcn_s_memrealtime());
#endif
    }

    // ---- the solve (wave 0)
    if (solver) {
        __builtin_amdgcn_s_setprio(3);
        while (__hip_atomic_load(&s_arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < 5)
            __builtin_amdgcn_s_sleep(1);
        // canonical tree, last level: (w0 + w1) + (w2 + w3)
        if (lane < kSums) L.S[lane] = (L.red[0][lane] + L.red[1][lane]) + (L.red[2][lane] + L.red[3][lane]);
        if (lane == 0) L.ngood = (L.g[0] + L.g[1]) + (L.g[2] + L.g[3]);
        PST(2);
        double* stp = (a.stats && blockIdx.x == 0) ? a.stats + (size_t)kStats * sl : nullptr;
#ifdef VISO_PROBE
        unsigned long long stamps[5] = {probe_t0, probe_t0, probe_t0, probe_t0, probe_t0};
        if (FAST)
            solve_wave0_ldlt(L, 0, stp, stamps);
        else
            solve_wave0(L, 0, stp, stamps);
        if (blockIdx.x == 0 && lane == 0)
            for (int k = 0; k < 4; ++k) pst[3 + k] = stamps[k];
        if (blockIdx.x == 0 && lane == 0) pst[12] = stamps[4];
#else
        if (FAST)
            solve_wave0_ldlt(L, 0, stp);
        else
            solve_wave0(L, 0, stp);
#endif
        PST(7);
        __builtin_amdgcn_s_setprio(1);
    }
    if (!solve && wave == 0 && lane == 0) {
        // seeded level: no solve, T21 is the seed (thread 256 wrote it)
        while (__hip_atomic_load(&s_arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < 1)
            __builtin_amdgcn_s_sleep(1);
    }
    if (wave == 0 && lane == 0 && !L.cont) after_solve(a, merged, L, s_last, s_pose);
    // the factored sums' per-lane J sources (direct_point_rs), ahead of B2
    const unsigned src_lanes = FAST ? 0u : factored_sources();
    __syncthreads();  // B2
    if (__builtin_expect(solve && L.cont, 0)) {
        // the continuation needs every thread; it leaves s_good dirty
        double* stp = (a.stats && blockIdx.x == 0) ? a.stats + (size_t)kStats * sl : nullptr;
        solve_continue<FAST>(a, merged ? a.prev : a.fp, sl, L, stp, s_pose, s_pts, &s_good, s_pf);
        if (t == 0) {
            after_solve(a, merged, L, s_last, s_pose);
            s_good = 0;
        }
        __syncthreads();
        // the continuation used the prefetch buffer: this tile's again, at
        // the solved pose (and, merged, the solved `last` pose)
        if (tiles) {
            double pose[12];
#pragma unroll
            for (int k = 0; k < 12; ++k) pose[k] = s_pose[k];
            prefetch_tile(a, lv, blockIdx.x, pose, merged ? s_last : a.fp.pose_last, true, wave, kWaves, s_pf);
        }
        __syncthreads();
    }
    if (wave == 0) PST(8);
#ifdef VISO_PROBE
    if (t == 0 && blockIdx.x < 256) g_pblk[a.probe_seq & (kPRingB - 1)][blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
#endif
    const int out = lv >= 0 ? lv : kLevels;
    if (blockIdx.x == 0 && t == 0 && !merged) {
        for (int k = 0; k < 7; ++k) a.s.state[out * kStateStride + k] = L.state[k];
        if (lv < 0 && a.pose_out) {
            store_frame_pose(a.pose_out, s_pose, a.ready);
            log_pose(a.log, a.log_host, a.log_index, s_pose);
            log_frame(a.flog, a.log_index, L);
        }
    }
    if (blockIdx.x == 0 && t == 0 && merged)
        for (int k = 0; k < 7; ++k) a.s.state[lv * kStateStride + k] = L.state[k];
    if (tiles) {
        LevelPair fp = level_pair(a.fp, lv);
        // merged: the `last` pose was solved above, its patch taps are read now
        if (merged) fp.pose_last = s_last;
        double pose[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) pose[k] = s_pose[k];
        direct_tile_pf<FAST>(a, fp, lv, pose, blockIdx.x, s_pf, merged, a.s.part + (size_t)lv * kMaxTiles * kSums,
                       a.s.good + lv * kMaxTiles, s_pts, &s_good, &s_cnt, qt, src_lanes);
    }
#ifdef VISO_PROBE
    // block 0 exit: its stamps to the launch's ring slot.  The exit stamp is
    // taken behind a block barrier, so it is the block's last wave (the
    // last-arriver tile trees finish after wave 0's points)
    __syncthreads();
    const unsigned long long t_exit = __builtin_amdgcn_s_memrealtime();
    const int slot = a.probe_seq & (kPRing - 1);
    // (no same-address atomic here: 247 serialised atomics per launch ran for
    // ~2 us after the last stamp and were counted as launch boundary; the
    // launch's exit is the maximum of the per-block stamps, host side)
    if (t == 0 && blockIdx.x < 256) g_pblk[a.probe_seq & (kPRingB - 1)][blockIdx.x][3] = t_exit;
    if (blockIdx.x == 0 && t == 0) {
        pst[11] = t_exit;
        pst[15] = (unsigned long long)(lv + 1) | ((unsigned long long)merged << 8) |
                  ((unsigned long long)a.n_tiles << 16);
        for (int k = 0; k < kPSt; ++k) g_plog[slot][k] = pst[k];
    }
#endif
}

// ================================================================ rig
// Multi-camera photometric rig (the repo's own spec,
// oracle/oracle_rig.cpp): one Gauss-Newton step of the rig pose T (world ->
// rig) per level.  Camera c sees the world at T_c = E_c T (E_c: rig ->
// camera); its 28 sums are DirectPoseEstimationSingleLayer's
// (src/viso.cpp:682-729) at T_c, reduced by the canonical tree over its own
// points; a rig perturbation xi moves camera c by Ad(E_c) xi, so
//   H = sum_c Ad_c^T H_c Ad_c,  b = sum_c Ad_c^T b_c,  cost = sum_c cost_c
// (cameras ascending), then the direct pose's solve and T <- exp(update) T
// (unchanged when the update is NaN).  Launches per timestep: L(3..0), the
// final solve merged into the next timestep's L(3) within an ingest call
// (F at the call's end); the tiles of all cameras in one grid (workgroup =
// one tile of one camera), the prologue of L(l) solving level l+1 from
// every camera's tile partials.  Tiles: one size T = map_tile(rig total,
// 256) for every camera, so the cameras share the 256 workgroups in
// proportion to their points; up to 256 per camera (T <= 64 points covers
// kMaxMapPoints); a camera's partials are reduced by 1, 2 or 4 waves (64
// tiles each) and the waves' sums folded as the canonical tree's top levels.
constexpr int kRigTiles = kMaxTiles;  // also the k-major partial stride of direct_tile_pf

// waves reducing a camera of n_tiles tiles (the canonical tree over 64 q tiles)
__device__ __host__ inline int rig_reduce_waves(int n_tiles) { return n_tiles <= 64 ? 1 : n_tiles <= 128 ? 2 : 4; }

struct RigCamArgs {
    DirectArgs d;       // the camera's pyramids (fp: last, cur; fp.pose_last =
                        // its `last` pose E_c T_last), points, tiling, and
                        // tile partials s.part / s.good ([kLevels][kRigTiles])
    const double* Ad;   // 36, row-major Ad(E_c)
    double E[12];       // rig -> camera (R row-major, t)
};

struct RigArgs {
    RigCamArgs cam[kMaxRigCams];
    int n_cams;
    int tile_off[kMaxRigCams + 1];  // camera c owns workgroups [tile_off[c], tile_off[c + 1])
    int level;                      // tiles of this level; -1: F
    double* state;                  // [kLevels + 1][kStateStride]: T each level was evaluated at
    const double* seed;             // L(3): the last rig pose (12)
    double* stats;                  // [kLevels][kStats] or null
    double* pose_out;               // F: rig pose (12)
    double* log;
    int log_index;
    double* cam_last;               // F: n_cams x 12, E_c T (next frame's `last` poses)
    // L(3) fused with the previous timestep's F (merged != 0): the prologue
    // solves the previous timestep's level 0, writes its pose / log / cam_last
    // (block 0), seeds T with SE3(R, t) of it, and takes each camera's `last`
    // pose E_c T_prev from it
    int merged;
    double* prev_pose_out;
    double* prev_log;
    int prev_log_index;
};

// Tc = E T (R row-major + t): Rc = Re R, tc = Re t + te
__device__ inline void rig_compose(const double* E, const double* T, double* out) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
        for (int j = 0; j < 3; ++j)
            out[3 * i + j] = (E[3 * i] * T[j] + E[3 * i + 1] * T[3 + j]) + E[3 * i + 2] * T[6 + j];
        out[9 + i] = ((E[3 * i] * T[9] + E[3 * i + 1] * T[10]) + E[3 * i + 2] * T[11]) + E[9 + i];
    }
}

// (unrolled with unconditional kernarg reads: the loads issue together
// instead of one dependent round trip per camera)
__device__ inline int rig_camera(const RigArgs& ra, int b) {
    int c = 0;
#pragma unroll
    for (int k = 1; k < kMaxRigCams; ++k) {
        const int off = ra.tile_off[k];
        if (k < ra.n_cams && b >= off) c = k;
    }
    return c;
}

// Camera c's contribution to the rig's 28 sums, by the camera's leader
// reduce wave once its q_c waves' sums are in red[0..q_c): first S_c = the
// top of the camera's canonical tree over its waves (r0; r0 + r1; (r0 + r1) +
// (r2 + r3)) into red[0]; then M = H_c Ad (lane l < 36: M[l / 6][l % 6])
// and lane e < 21 (upper-triangle entry (i, j) of Ad^T M), 21 + i
// ((Ad^T b_c)_i) or 27 (cost_c) into con.  The cameras' leaders run
// concurrently; wave 0 folds their contributions in ascending camera order
// (rig_fold).  Ad: row-major Ad(E_c), staged in LDS.
__device__ inline void rig_contrib(int q, double (*red)[kSums], const double* Ad, double* sM, double* con) {
    const int lane = threadIdx.x & 63;
    if (q > 1 && lane < kSums) {
        const double v = q == 2 ? red[0][lane] + red[1][lane]
                                : (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
        red[0][lane] = v;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const double* S = red[0];
    if (lane < 36) {
        const int i = lane / 6, j = lane - 6 * (lane / 6);
        double m = 0.0;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const int a = i < k ? i : k, bb = i < k ? k : i;
            const double h = S[a * 6 - (a * (a - 1)) / 2 + (bb - a)];
            m = k == 0 ? h * Ad[j] : m + h * Ad[6 * k + j];
        }
        sM[lane] = m;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // (i, j) of upper entry e, row-major over i <= j
    int ei = 0, ej = 0;
    {
        int e = lane < 21 ? lane : 0, r = 0;
        while (e >= 6 - r) {
            e -= 6 - r;
            ++r;
        }
        ei = r;
        ej = r + e;
    }
    double v = 0.0;
    if (lane < 21) {
#pragma unroll
        for (int k = 0; k < 6; ++k) v = k == 0 ? Ad[ei] * sM[ej] : v + Ad[6 * k + ei] * sM[6 * k + ej];
    } else if (lane < 27) {
        const int i = lane - 21;
#pragma unroll
        for (int k = 0; k < 6; ++k) v = k == 0 ? Ad[i] * S[21] : v + Ad[6 * k + i] * S[21 + k];
    } else if (lane == 27) {
        v = S[27];
    }
    if (lane < kSums) con[lane] = v;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// Wave 0, every camera's contribution in: the rig's 28 sums (cameras
// ascending) into L.S and nGood into L.ngood
__device__ inline void rig_fold(const RigArgs& ra, const double (*con)[kSums], const int (*g)[4], SolveLds& L) {
    const int lane = threadIdx.x & 63;
    int ng = 0;
    for (int c = 0; c < ra.n_cams; ++c) {
        const int q = rig_reduce_waves(ra.cam[c].d.n_tiles);
        for (int j = 0; j < q; ++j) ng += g[c][j];
    }
    if (lane < kSums) {
        double acc = con[0][lane];
        for (int c = 1; c < ra.n_cams; ++c) acc = acc + con[c][lane];
        L.S[lane] = acc;
    }
    if (lane == 0) L.ngood = ng;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// bytes of one camera's scratch (rig_scratch_bytes): tile partials
// [kLevels][28][256] f64, then nGood counts [kLevels][256]
constexpr size_t kRigPartBytes = (size_t)kLevels * kRigTiles * kSums * 8;
constexpr size_t kRigScratchBytes = kRigPartBytes + (size_t)kLevels * kRigTiles * 4;

// The leading arguments repeat what the reduce waves' first loads need, so
// they arrive in SGPRs at wave launch (-amdgpu-kernarg-preload-count; the
// direct pose's prologue does the same): every camera's scratch and Ad(E_c)
// at fixed strides from two bases, pre_hdr = (level + 1) | n_cams << 8 |
// 1 << 16 when the cameras' scratch / Ad are laid out that way (rig.cpp;
// else the by-value arguments are read), and the cameras' tile counts in
// 16-bit halves of pre_t01 / pre_t23.
template <bool FAST, bool MERGED>
__global__ __launch_bounds__(kRigThreads) void rig_level_kernel(const char* __restrict__ pre_scratch,
                                                                const double* __restrict__ pre_ad, int pre_hdr,
                                                                int pre_t01, int pre_t23, RigArgs ra) {
    __shared__ SolveLds L;
    __shared__ double s_red[kMaxRigCams][4][kSums];
    __shared__ int s_g[kMaxRigCams][4];
    __shared__ double s_M[kMaxRigCams][36];
    __shared__ double s_Ad[kMaxRigCams][36];
    __shared__ double s_con[kMaxRigCams][kSums];
    __shared__ int s_camarr[kMaxRigCams];
    __shared__ double s_pose[12];
    __shared__ double s_last[12];  // merged L(3): this workgroup's camera `last` pose E_c T_prev
    __shared__ double s_pts[kMaxTile * kSums];
    __shared__ int s_good;
    __shared__ int s_cnt;
    __shared__ int s_arrive;
    __shared__ PfLds s_pf;

    PROBE_DECL();
    // wave-uniform in SGPRs: ra.cam[wave / 4] is then read with scalar loads
    const int t = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63;
    // ---- every camera's tile partials of level sl (wave w: camera w % 4,
    // tiles 64 (w / 4) .. +63 of it, when the camera has that many waves:
    // the cameras' leaders 0..3 sit on different SIMDs, so their reductions
    // and transforms run side by side),
    // issued first (before the workgroup's own camera is looked up and
    // before the first LDS barrier, which waits for LDS traffic only)
    static_assert(kRigWaves >= 4 * kMaxRigCams, "four reduce waves per camera");
    const int rc = wave & 3, rq = wave >> 2;
    // the kernel arguments this wave's loads need, read unconditionally
    // (cam[rc] exists for every rc < kMaxRigCams) so the scalar loads issue
    // together: one argument round trip before the partial loads
    int rc_tiles, n_cams, lv_arg;
    const double* rc_part;
    const int* rc_good;
    const double* rc_ad;
    if (pre_hdr & (1 << 16)) {
        // preloaded: no kernel-argument load in front of the partial loads
        lv_arg = (pre_hdr & 0xff) - 1;
        n_cams = (pre_hdr >> 8) & 0xff;
        rc_tiles = ((rc < 2 ? pre_t01 : pre_t23) >> (16 * (rc & 1))) & 0xffff;
        const char* sc = pre_scratch + (size_t)rc * kRigScratchBytes;
        rc_part = (const double*)sc;
        rc_good = (const int*)(sc + kRigPartBytes);
        rc_ad = pre_ad + 36 * rc;
    } else {
        rc_tiles = ra.cam[rc].d.n_tiles;
        rc_part = ra.cam[rc].d.s.part;
        rc_good = ra.cam[rc].d.s.good;
        rc_ad = ra.cam[rc].Ad;
        n_cams = ra.n_cams;
        lv_arg = ra.level;
        // (the empty asm takes every argument at once and hands the level on:
        // nothing derived from it is scheduled between the scalar loads)
        asm volatile("" : "+s"(lv_arg) : "s"(rc_tiles), "s"(rc_part), "s"(rc_good), "s"(rc_ad));
    }
    const int lv = lv_arg;
    const bool merged = MERGED;  // launched for L(3) only
    const bool solve = lv < kLevels - 1 || merged;  // an unmerged L(3) is seeded
    const int sl = merged ? 0 : lv + 1;              // level solved in the prologue (F: 0)
    const int q_rc = rc < n_cams ? rig_reduce_waves(rc_tiles) : 0;
    const bool rwave = solve && rq < q_rc;
    double v[kSums];
    int gg = 0;
    double ad = 0.0;  // the leader stages Ad(E_c) (its load overlaps the partials')
    if (rwave) {
        const int tl = 64 * rq + lane;
        if (rq == 0 && lane < 36) ad = rc_ad[lane];
        if (tl < rc_tiles) {
            const double* src = rc_part + (size_t)sl * kRigTiles * kSums;  // k-major [28][256]
#pragma unroll
            for (int k = 0; k < kSums; ++k) v[k] = src[(size_t)k * kRigTiles + tl];
            gg = rc_good[sl * kRigTiles + tl];
        } else {
#pragma unroll
            for (int k = 0; k < kSums; ++k) v[k] = 0.0;
        }
    }
    const int c = rig_camera(ra, blockIdx.x);
    const int bt = (int)blockIdx.x - ra.tile_off[c];
    const DirectArgs& a = ra.cam[c].d;
    const bool tiles = lv >= 0 && bt < a.n_tiles;
    if (t == 0) {
        s_arrive = 0;
        s_good = 0;
        s_cnt = 0;
#ifdef VISO_PROBE
        for (int k = 0; k < kPSt; ++k) pst[k] = 0;
        pst[0] = probe_t0;
        if (blockIdx.x < 256) g_pblk[a.probe_seq & (kPRingB - 1)][blockIdx.x][0] = probe_t0;
#endif
    }
    if (t < kMaxRigCams) s_camarr[t] = 0;
    lds_barrier();
#ifdef VISO_PROBE
    if (rwave && wave == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        PST(3);
    }
#endif
    if (rwave) {
        int idx;
        const double f = reduce_scatter_28(v, &idx);
        if (lane < 32 && idx >= 0) s_red[rc][rq][idx] = f;
        const int g = wave_sum_int(gg);
        if (lane == 0) s_g[rc][rq] = g;
        if (rq == 0 && lane < 36) s_Ad[rc][lane] = ad;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (rq > 0) {
            if (lane == 0) atomicAdd(&s_camarr[rc], 1);
        } else {
            // the camera's other waves, then its contribution
            while (__hip_atomic_load(&s_camarr[rc], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < q_rc - 1)
                __builtin_amdgcn_s_sleep(1);
            rig_contrib(q_rc, s_red[rc], s_Ad[rc], s_M[rc], s_con[rc]);
            if (wave == 0) PST(4);
            if (lane == 0) atomicAdd(&s_arrive, 1);
        }
    }
    // ---- the T this level starts from (thread 192: wave 3 is camera 3's
    // leader reduce wave, so for a 4-camera rig this write waits behind that
    // camera's reduction; wave 0 needs both before it solves, so only the
    // order, not the result, depends on it)
    if (t == 192) {
        double st[7];
        if (!solve) {
            quat_from_matrix(ra.seed, st);
            st[4] = ra.seed[9];
            st[5] = ra.seed[10];
            st[6] = ra.seed[11];
        } else {
            for (int k = 0; k < 7; ++k) st[k] = ra.state[sl * kStateStride + k];
        }
        for (int k = 0; k < 7; ++k) {
            L.state[k] = st[k];
            L.best[k] = st[k];
        }
        L.cost = 0.0;
        L.last_cost = 0.0;
        L.cont = 0;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        atomicAdd(&s_arrive, 1);
    }
    // ---- prefetch of this workgroup's tile at the predicted camera pose (a
    // merged L(3) also predicts its `last` pose: E_c times the T the previous
    // level 0 was evaluated at; the tile phase re-checks every lane's taps)
    const bool pf_wave = !solve || (wave & 3) != 0;
    if (tiles && pf_wave) {
        double T[12], pred[12];
        if (!solve) {
            for (int k = 0; k < 12; ++k) T[k] = ra.seed[k];
        } else {
            double sp[7];
            for (int k = 0; k < 7; ++k) sp[k] = ra.state[sl * kStateStride + k];
            state_to_pose(sp, T);
        }
        rig_compose(ra.cam[c].E, T, pred);
        const int first = solve ? wave - (wave >> 2) - 1 : wave;
        const int stride = solve ? kRigWaves - kRigWaves / 4 : kRigWaves;
        prefetch_tile<FAST>(a, lv, bt, pred, merged ? pred : a.fp.pose_last, true, first, stride, s_pf);
    }
    // ---- the solve (wave 0)
    if (wave == 0) {
        const int need = 1 + (solve ? ra.n_cams : 0);  // the start T, each camera's contribution
        while (__hip_atomic_load(&s_arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < need)
            __builtin_amdgcn_s_sleep(1);
        PST(1);
        if (solve) {
            __builtin_amdgcn_s_setprio(3);
            rig_fold(ra, s_con, s_g, L);
            PST(2);
            double* stp = (ra.stats && blockIdx.x == 0) ? ra.stats + (size_t)kStats * sl : nullptr;
            if (FAST)
                solve_wave0_ldlt(L, 0, stp);
            else
                solve_wave0(L, 0, stp);
            __builtin_amdgcn_s_setprio(0);
        }
        if (lane == 0) {
            // one step per level: L.cont (the reference's cost == 0
            // continuation) is not part of the rig spec
            double T[12];
            state_to_pose(L.state, T);
            const bool fin = lv < 0 || merged;  // the solve just done finished a timestep
            if (fin && blockIdx.x == 0) {
                double* po = merged ? ra.prev_pose_out : ra.pose_out;
                double* lg = merged ? ra.prev_log : ra.log;
                const int li = merged ? ra.prev_log_index : ra.log_index;
                for (int k = 0; k < 7; ++k) ra.state[kLevels * kStateStride + k] = L.state[k];
                if (po)
                    for (int k = 0; k < 12; ++k) po[k] = T[k];
                if (lg && li >= 0)
                    for (int k = 0; k < 12; ++k) lg[12 * (size_t)li + k] = T[k];
                for (int cc = 0; cc < ra.n_cams; ++cc) {
                    double Tc[12];
                    rig_compose(ra.cam[cc].E, T, Tc);
                    for (int k = 0; k < 12; ++k) ra.cam_last[12 * cc + k] = Tc[k];
                }
            }
            if (merged) {
                // this camera's `last` pose, and SE3(R, t) of the previous
                // timestep's pose as this timestep's seed (src/viso.cpp:114)
                rig_compose(ra.cam[c].E, T, s_last);
                double q[4];
                quat_from_matrix(T, q);
                for (int k = 0; k < 4; ++k) L.state[k] = q[k];
                L.state[4] = T[9];
                L.state[5] = T[10];
                L.state[6] = T[11];
                state_to_pose(L.state, T);
            }
            rig_compose(ra.cam[c].E, T, s_pose);
            if (blockIdx.x == 0 && lv >= 0)
                for (int k = 0; k < 7; ++k) ra.state[lv * kStateStride + k] = L.state[k];
        }
        PST(7);
    }
    __syncthreads();  // B2
    if (wave == 0) PST(8);
#ifdef VISO_PROBE
    if (t == 0 && blockIdx.x < 256) g_pblk[a.probe_seq & (kPRingB - 1)][blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
#endif
    if (tiles) {
        LevelPair fp = level_pair(a.fp, lv);
        if (merged) fp.pose_last = s_last;
        double pose[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) pose[k] = s_pose[k];
        direct_tile_pf<FAST, FAST, kRigWaves>(a, fp, lv, pose, bt, s_pf, merged,
                                              a.s.part + (size_t)lv * kRigTiles * kSums, a.s.good + lv * kRigTiles,
                                              s_pts, &s_good, &s_cnt);  // (the operand table measured no gain here)
    }
#ifdef VISO_PROBE
    const unsigned long long t_exit = __builtin_amdgcn_s_memrealtime();
    const int slot = a.probe_seq & (kPRing - 1);
    // (no same-address atomic here: 247 serialised atomics per launch ran for
    // ~2 us after the last stamp and were counted as launch boundary; the
    // launch's exit is the maximum of the per-block stamps, host side)
    if (t == 0 && blockIdx.x < 256) g_pblk[a.probe_seq & (kPRingB - 1)][blockIdx.x][3] = t_exit;
    if (blockIdx.x == 0 && t == 0) {
        pst[11] = t_exit;
        pst[15] = (unsigned long long)(lv + 1) | ((unsigned long long)merged << 8) |
                  ((unsigned long long)a.n_tiles << 16);
        for (int k = 0; k < kPSt; ++k) g_plog[slot][k] = pst[k];
    }
#endif
}
static_assert(sizeof(RigArgs) <= 4096, "rig kernel arguments exceed 4 KB");

struct Pose12v {
    double v[12];
};

__global__ void set_pose_kernel(double* dst, Pose12v p) {
    if (threadIdx.x < 12) dst[threadIdx.x] = p.v[threadIdx.x];
}

// Map creation (src/viso.cpp:79-96) in one launch: the current frame's pose
// (by value), the map points (the 2D-2D result's inlier points), and the two
// keyframe poses (the reference frame's, read on the device, and the new one).
__global__ void map_create_kernel(double* __restrict__ cur_pose, Pose12v p, const double* __restrict__ pts_src,
                                  double* __restrict__ pts_dst, int n_dbl, const double* __restrict__ ref_pose,
                                  double* __restrict__ kf_poses) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    for (int i = t; i < n_dbl; i += gridDim.x * blockDim.x) pts_dst[i] = pts_src[i];
    if (blockIdx.x == 0 && threadIdx.x < 12) {
        cur_pose[threadIdx.x] = p.v[threadIdx.x];
        kf_poses[threadIdx.x] = ref_pose[threadIdx.x];
        kf_poses[12 + threadIdx.x] = p.v[threadIdx.x];
    }
}

}  // namespace

void launch_map_create(double* cur_pose, const double pose[12], const double* pts_src, double* pts_dst, int n_pts,
                       const double* ref_pose, double* kf_poses, hipStream_t stream) {
    Pose12v p;
    for (int k = 0; k < 12; ++k) p.v[k] = pose[k];
    const int n_dbl = 3 * n_pts;
    const int blocks = std::max(1, std::min((n_dbl + 255) / 256, 64));
    map_create_kernel<<<blocks, 256, 0, stream>>>(cur_pose, p, pts_src, pts_dst, n_dbl, ref_pose, kf_poses);
}

void launch_set_pose(double* dst, const double src[12], hipStream_t stream) {
    Pose12v p;
    for (int k = 0; k < 12; ++k) p.v[k] = src[k];
    set_pose_kernel<<<1, 64, 0, stream>>>(dst, p);
}

size_t direct_scratch_bytes() {
    return (size_t)kLevels * kMaxTiles * kSums * 8 + (size_t)kLevels * kMaxTiles * 4 +
           (size_t)(kLevels + 1) * kStateStride * 8 + (size_t)kMaxTiles * kMaxTiles * kSums * 8 +
           (size_t)kMaxTiles * kMaxTiles * 4 + 5 * 256;
}

DirectScratch direct_scratch_at(void* base) {
    auto align = [](size_t o) { return (o + 255) & ~(size_t)255; };
    char* b = (char*)base;
    size_t o = 0;
    DirectScratch s;
    s.part = (double*)(b + o);
    o = align(o + (size_t)kLevels * kMaxTiles * kSums * 8);
    s.good = (int*)(b + o);
    o = align(o + (size_t)kLevels * kMaxTiles * 4);
    s.state = (double*)(b + o);
    o = align(o + (size_t)(kLevels + 1) * kStateStride * 8);
    s.cont_part = (double*)(b + o);
    o = align(o + (size_t)kMaxTiles * kMaxTiles * kSums * 8);
    s.cont_good = (int*)(b + o);
    return s;
}

namespace {
// probe builds: ring slot of the next direct-pose launch (0 otherwise)
#ifdef VISO_PROBE
static unsigned g_probe_host_seq = 0;
int next_probe_seq() { return (int)(g_probe_host_seq++); }
#else
int next_probe_seq() { return 0; }
#endif

DirectArgs direct_args(const FrameDev& last_pyr, const FrameDev& cur_pyr, const PyrGeom& g,
                       const double K[4], const double* points, int n, const double* pose_last12,
                       const double* pose_seed12, const DirectScratch& s, double* stats, bool split) {
    DirectArgs a{};
    a.fp.last = last_pyr;
    a.fp.cur = cur_pyr;
    a.fp.pose_last = pose_last12;
    a.g = make_pyrdev(g);
    a.K = Intrinsics{K[0], K[1], K[2], K[3]};
    a.points = points;
    a.n = n;
    a.pose_seed = pose_seed12;
    // the canonical map tree's tiles (oracle_common.hpp map_tree_sum, groups
    // = 256): one workgroup per tile, <= 256 tiles of <= 64 points
    a.tile = map_tile(n, kMaxTiles);
    a.n_tiles = (n + a.tile - 1) / a.tile;
    if (split && n > 0) {
        a.split = 1;
        a.n_tiles = n < kMaxTiles ? n : kMaxTiles;
        a.tile = (n + a.n_tiles - 1) / a.n_tiles;
    }
    a.s = s;
    a.stats = stats;
    a.log_index = -1;
    a.prev_log_index = -1;
    return a;
}
}  // namespace

bool direct_fits_background() { return kThreads <= 768; }

void launch_direct_levels(const FrameDev& last_pyr, const FrameDev& cur_pyr, const PyrGeom& g,
                          const double K[4], const double* points, int n,
                          const double* pose_last12, const double* pose_seed12,
                          const DirectScratch& s, double* stats, const DirectPrev* merge,
                          hipStream_t stream, int precision, bool bg) {
    DirectArgs a = direct_args(last_pyr, cur_pyr, g, K, points, n, pose_last12, pose_seed12, s,
                               stats, precision == VISO_PRECISION_FAST);
    if (merge) {
        a.merged = 1;
        a.prev.last = merge->last;
        a.prev.cur = merge->cur;
        a.prev.pose_last = merge->pose_last12;
        a.prev_pose_out = merge->pose_out;
        a.prev_log = merge->log;
        a.prev_log_index = merge->log ? merge->log_index : -1;
        a.prev_log_host = merge->log ? merge->log_host : nullptr;
        a.prev_ready = merge->ready;
        a.flog = merge->log ? merge->flog : nullptr;
    }
    const int grid = a.n_tiles > 0 ? a.n_tiles : 1;
    for (int level = kLevels - 1; level >= 0; --level) {
        a.level = level;
        a.probe_seq = next_probe_seq();
        const bool merged = a.merged && level == kLevels - 1;
        const bool solve = level + 1 < kLevels || merged;
        const int sl = merged ? 0 : level + 1;
        const double* pp = solve ? a.s.part + (size_t)sl * kMaxTiles * kSums : nullptr;
        const int* pg = solve ? a.s.good + sl * kMaxTiles : nullptr;
        const int hdr = a.n_tiles | (solve ? 1 << 16 : 0) | (bg ? kHdrBg : 0);
        if (precision == VISO_PRECISION_FAST)
            direct_level_kernel<true><<<grid, kThreads, 0, stream>>>(pp, pg, hdr, a);
        else
            direct_level_kernel<false><<<grid, kThreads, 0, stream>>>(pp, pg, hdr, a);
        a.merged = 0;
    }
}

void launch_direct_final(const FrameDev& last_pyr, const FrameDev& cur_pyr, const PyrGeom& g,
                         const double K[4], const double* points, int n,
                         const double* pose_last12, const DirectScratch& s, double* stats,
                         double* pose_out, double* log, int log_index, hipStream_t stream, int precision,
                         int* ready, double* log_host, double* flog) {
    DirectArgs a = direct_args(last_pyr, cur_pyr, g, K, points, n, pose_last12, pose_last12, s,
                               stats, precision == VISO_PRECISION_FAST);
    a.pose_out = pose_out;
    a.ready = ready;
    a.log = log;
    a.log_index = log ? log_index : -1;
    a.log_host = log ? log_host : nullptr;
    a.flog = log ? flog : nullptr;
    a.level = -1;
    a.probe_seq = next_probe_seq();
    // F solves level 0
    const int hdr = a.n_tiles | (1 << 16) | (ready ? kHdrBg : 0);
    if (precision == VISO_PRECISION_FAST)
        direct_level_kernel<true><<<1, kThreads, 0, stream>>>(a.s.part, a.s.good, hdr, a);
    else
        direct_level_kernel<false><<<1, kThreads, 0, stream>>>(a.s.part, a.s.good, hdr, a);
}

// A rig camera of n points in tiles of T points (T shared by the cameras,
// map_tile of the rig's total; oracle_rig.cpp); tolerance mode (split) evens
// the points over the same number of tiles
static int rig_tiling(int n, int T, bool split, int* tile, int* n_tiles) {
    if (n < 0 || n > kMaxMapPoints) return -1;
    *tile = T;
    *n_tiles = (n + T - 1) / T;
    if (split && n > 0) *tile = (n + *n_tiles - 1) / *n_tiles;
    // the prefetch and tile tree hold at most kMaxTile points per workgroup
    return (*tile <= kMaxTile && *n_tiles <= kRigTiles) ? 0 : -1;
}

size_t rig_scratch_bytes() { return kRigScratchBytes; }

int launch_rig_direct(const RigCamDev* cams, int n_cams, const PyrGeom& g, const double K[4], double* state,
                      const double* seed12, double* stats, double* pose_out, double* log, int log_index,
                      double* cam_last, hipStream_t stream, int precision, int merge_prev, int prev_log_index,
                      int levels, int final_solve) {
    if (n_cams < 1 || n_cams > kMaxRigCams) return -1;
    const bool fast = precision == VISO_PRECISION_FAST;
    RigArgs ra{};
    ra.n_cams = n_cams;
    // tiles of one size for every camera (map_tile of the rig's total map):
    // the cameras' tiles fill the 256 workgroups in proportion to their points
    int n_total = 0;
    for (int c = 0; c < n_cams; ++c) n_total += cams[c].n > 0 ? cams[c].n : 0;
    const int T = map_tile(n_total, kMaxTiles);
    int off = 0;
    for (int c = 0; c < n_cams; ++c) {
        const RigCamDev& cd = cams[c];
        DirectArgs& a = ra.cam[c].d;
        a.fp.last = cd.last;
        a.fp.cur = cd.cur;
        a.fp.pose_last = cd.pose_last12;
        a.g = make_pyrdev(g);
        a.K = Intrinsics{K[0], K[1], K[2], K[3]};
        a.points = cd.points;
        a.n = cd.n;
        if (rig_tiling(cd.n, T, fast, &a.tile, &a.n_tiles) != 0) return -1;
        a.split = fast && cd.n > 0 ? 1 : 0;
        a.s.part = (double*)cd.scratch;
        a.s.good = (int*)((char*)cd.scratch + (size_t)kLevels * kRigTiles * kSums * 8);
        a.log_index = -1;
        a.prev_log_index = -1;
        ra.cam[c].Ad = cd.Ad;
        for (int k = 0; k < 12; ++k) ra.cam[c].E[k] = cd.E[k];
        ra.tile_off[c] = off;
        off += a.n_tiles;
    }
    ra.tile_off[n_cams] = off;
    ra.state = state;
    ra.seed = seed12;
    ra.stats = stats;
    ra.log_index = -1;
    ra.cam_last = cam_last;
    ra.prev_log_index = -1;
    const int grid = off > 0 ? off : 1;
    // the preloaded prologue arguments (rig_level_kernel): valid when every
    // camera's scratch and Ad(E_c) sit at fixed strides from camera 0's
#ifndef VISO_RIG_PRELOAD
#define VISO_RIG_PRELOAD 1
#endif
    bool pre_ok = VISO_RIG_PRELOAD != 0;
    int tl[kMaxRigCams] = {0, 0, 0, 0};
    for (int c = 0; c < n_cams; ++c) {
        pre_ok = pre_ok && (const char*)cams[c].scratch == (const char*)cams[0].scratch + kRigScratchBytes * c &&
                 cams[c].Ad == cams[0].Ad + 36 * c;
        tl[c] = ra.cam[c].d.n_tiles;
    }
    const int t01 = (tl[0] & 0xffff) | (tl[1] << 16), t23 = (tl[2] & 0xffff) | (tl[3] << 16);
    for (int level = levels ? kLevels - 1 : -1; level >= -1; --level) {
        ra.level = level;
#ifdef VISO_PROBE
        {
            const int seq = next_probe_seq();
            for (int c = 0; c < n_cams; ++c) ra.cam[c].d.probe_seq = seq;
        }
#endif
        ra.merged = 0;
        if (level == kLevels - 1 && merge_prev) {
            ra.merged = 1;
            ra.prev_pose_out = pose_out;
            ra.prev_log = log;
            ra.prev_log_index = log ? prev_log_index : -1;
        }
        if (level < 0) {
            if (!final_solve) break;
            ra.pose_out = pose_out;
            ra.log = log;
            ra.log_index = log ? log_index : -1;
        }
        const int gl = level < 0 ? 1 : grid;
        const int hdr = ((level + 1) & 0xff) | (n_cams << 8) | (pre_ok ? 1 << 16 : 0);
        const char* psc = (const char*)cams[0].scratch;
        const double* pad = cams[0].Ad;
        if (ra.merged) {
            if (fast)
                rig_level_kernel<true, true><<<gl, kRigThreads, 0, stream>>>(psc, pad, hdr, t01, t23, ra);
            else
                rig_level_kernel<false, true><<<gl, kRigThreads, 0, stream>>>(psc, pad, hdr, t01, t23, ra);
        } else if (fast) {
            rig_level_kernel<true, false><<<gl, kRigThreads, 0, stream>>>(psc, pad, hdr, t01, t23, ra);
        } else {
            rig_level_kernel<false, false><<<gl, kRigThreads, 0, stream>>>(psc, pad, hdr, t01, t23, ra);
        }
    }
    return 0;
}

void launch_direct_pose(const FrameDev& last_pyr, const FrameDev& cur_pyr, const PyrGeom& g,
                        const double K[4], const double* points, int n,
                        const double* pose_last12, const double* pose_seed12,
                        const DirectScratch& s, double* stats, double* pose_out, double* log,
                        int log_index, hipStream_t stream, int precision) {
    launch_direct_levels(last_pyr, cur_pyr, g, K, points, n, pose_last12, pose_seed12, s, stats,
                         nullptr, stream, precision);
    launch_direct_final(last_pyr, cur_pyr, g, K, points, n, pose_last12, s, stats, pose_out, log,
                        log_index, stream, precision);
}

}  // namespace viso

#ifdef VISO_PROBE
// The direct-pose probe ring: *n_launches = launches since the last reset;
// log (cap x 16 stamps) and exits (cap) in launch order for the last
// min(cap, n, 4096) launches.
extern "C" int viso_debug_probe_ring(unsigned long long* log, unsigned long long* exits, int cap, int* n_launches,
                                     int reset) {
    using namespace viso;
    static unsigned long long hlog[kPRing][kPSt], hexit[kPRing];
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    if (hipMemcpyFromSymbol(hlog, HIP_SYMBOL(g_plog), sizeof(hlog)) != hipSuccess) return -2;
    if (hipMemcpyFromSymbol(hexit, HIP_SYMBOL(g_pexit), sizeof(hexit)) != hipSuccess) return -2;
    const int n = (int)g_probe_host_seq;
    const int m = std::min(std::min(cap, n), kPRing);
    for (int i = 0; i < m; ++i) {
        const int s = (n - m + i) & (kPRing - 1);
        for (int k = 0; k < kPSt; ++k) log[(size_t)i * kPSt + k] = hlog[s][k];
        exits[i] = hexit[s];
    }
    // launch exits: the maximum of the per-block exit stamps (kept for the
    // last kPRingB launches)
    {
        static unsigned long long hb[kPRingB][256][4];
        if (hipMemcpyFromSymbol(hb, HIP_SYMBOL(g_pblk), sizeof(hb)) != hipSuccess) return -2;
        for (int i = std::max(0, m - kPRingB); i < m; ++i) {
            const int sb = (n - m + i) & (kPRingB - 1);
            unsigned long long mx = 0;
            for (int b = 0; b < 256; ++b) mx = std::max(mx, hb[sb][b][3]);
            exits[i] = mx;
        }
    }
    *n_launches = n;
    if (reset) {
        static unsigned long long z3[kPRingB][256][4] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_pblk), z3, sizeof(z3)) != hipSuccess) return -2;
        static unsigned long long z1[kPRing][kPSt] = {}, z2[kPRing] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_plog), z1, sizeof(z1)) != hipSuccess) return -2;
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_pexit), z2, sizeof(z2)) != hipSuccess) return -2;
        g_probe_host_seq = 0;
    }
    return 0;
}

#ifdef VISO_PROBE_PT
// (probe) per-point phase stamps (g_ppt) of the last min(cap, n, 128)
// launches, in launch order: out[i][b < 32][wave < 16][5]
extern "C" int viso_debug_probe_points(unsigned long long* out, int cap) {
    using namespace viso;
    static unsigned long long h[kPtRing][kPtBlocks][16][kPtStamps];
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_ppt), sizeof(h)) != hipSuccess) return -2;
    const int n = (int)g_probe_host_seq;
    const int m = std::min(std::min(cap, n), kPtRing);
    for (int i = 0; i < m; ++i) {
        const int s = (n - m + i) & (kPtRing - 1);
        std::memcpy(out + (size_t)i * kPtBlocks * 16 * kPtStamps, &h[s][0][0][0], sizeof(h[s]));
    }
    return m;
}
#endif

// (probe) window misses per level since the last reset: out[8] (g_pfb)
extern "C" int viso_debug_probe_window_misses(unsigned long long* out, int reset) {
    using namespace viso;
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pfb), 8 * sizeof(unsigned long long)) != hipSuccess) return -2;
    if (reset) {
        static const unsigned long long z[8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_pfb), z, sizeof(z)) != hipSuccess) return -2;
    }
    return 0;
}

// Per-block, per-wave tile stamps (g_pwave) of the last min(cap, n, 512)
// launches, in launch order: out[i][b][16].
extern "C" int viso_debug_probe_waves_direct(unsigned long long* out, int cap) {
    using namespace viso;
    static unsigned long long h[kPRingB][256][16];
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_pwave), sizeof(h)) != hipSuccess) return -2;
    const int n = (int)g_probe_host_seq;
    const int m = std::min(std::min(cap, n), kPRingB);
    for (int i = 0; i < m; ++i) {
        const int s = (n - m + i) & (kPRingB - 1);
        for (int b = 0; b < 256; ++b)
            for (int k = 0; k < 16; ++k) out[((size_t)i * 256 + b) * 16 + k] = h[s][b][k];
    }
    return m;
}

// Per-block stamps of the last min(cap, n, 512) launches, in launch order:
// out[i][b][0..3] = entry, after B2, wave 0's points evaluated, exit.
extern "C" int viso_debug_probe_blocks(unsigned long long* out, int cap) {
    using namespace viso;
    static unsigned long long h[kPRingB][256][4];
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_pblk), sizeof(h)) != hipSuccess) return -2;
    const int n = (int)g_probe_host_seq;
    const int m = std::min(std::min(cap, n), kPRingB);
    for (int i = 0; i < m; ++i) {
        const int s = (n - m + i) & (kPRingB - 1);
        for (int b = 0; b < 256; ++b)
            for (int k = 0; k < 4; ++k) out[((size_t)i * 256 + b) * 4 + k] = h[s][b][k];
    }
    return m;
}
#endif
