// viso_amd — north-star stereo visual odometry (SVO) on gfx950.
//
// Spec: include/viso/viso_svo.h + DESIGN.md §10; CPU restatement (the parity
// checker): oracle/oracle_svo.cpp.  No reference counterpart.
//
// Per stereo pair (all on one HIP stream, no host round trip):
//   svo_detect_kernel    thread per column of a 256-column tile: image rows
//                        staged in LDS, 5x5 blob / checkerboard responses
//                        from a register row window, strict (2n+1)^2 NMS of
//                        the four classes as packed 16-bit max/min, per-(row,
//                        tile, wave) candidate lists in (x, class) order
//   svo_scan_kernel      row-major prefix over the lists -> u, v, class
//   svo_describe_kernel  16 lanes per feature: Sobel du/dv at the 16 sample
//                        offsets -> 32-byte descriptor
//   svo_circle_kernel    wave per current-left feature: four best-SAD
//                        searches (v_sad_u8, wave argmin on (sad, index))
//                        left_t -> right_t -> right_t-1 -> left_t-1 -> left_t
//   svo_bucket_kernel    wave per bucket: first bucket_max matches of the
//                        bucket in left order (ballot ranks)
//   svo_select_kernel    one workgroup: compaction of the kept matches
//   svo_obs_kernel       the selected matches' 3-D points / observations
//   svo_hyp_kernel       thread per RANSAC hypothesis: 3-point Gauss-Newton
//   svo_count_kernel     hypotheses x matches inlier counts (ballot/popc)
//   svo_refine_kernel    one workgroup: best hypothesis, Gauss-Newton over
//                        its inliers (28 canonical tree sums per iteration),
//                        inlier flags, motion, pose accumulation
// Integer stages are exact; the pose math is fp64 with +,-,*,/ only in the
// oracle's expression order (-ffp-contract=off), so results are bit-identical.
#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/viso/viso_svo.h"
#include "common.hpp"
#include "staging.hpp"
#include "trace.hpp"

namespace viso {
namespace {

constexpr int kMaxNms = 8;      // nms_n bound (detect kernel instances)
constexpr int kDesc = VISO_SVO_DESC_BYTES;

__constant__ int c_p16[16][2] = {{-5, -1}, {-5, 1}, {-3, -3}, {-3, 3}, {-1, -5}, {-1, 5},
                                 {-1, -1}, {-1, 1}, {1, -1},  {1, 1},  {1, -5},  {1, 5},
                                 {3, -3},  {3, 3},  {5, -1},  {5, 1}};

struct SvoDev {  // kernel view of the parameters
    int w, h, nms_n, tau, margin, disp_max, radius, bw, bh, bmax, iters, gn_iters, cap, nband, ow, ncam, sw;
    float inv_ow, inv_sw;  // 1 / ow, 1 / sw (division-free band_of)
    double fx, fy, cu, cv, base, th2, eps;
    uint64_t seed;
};

// one feature set (an image's features), SoA in device memory
struct FeatDev {
    int* u;
    int* v;
    int* c;
    uint8_t* d;    // [cap][32]
    int* row0;     // [h + 1]: first feature index of each row; row0[h] = n
    // class-band index: the features of class k in column band b, rows in
    // ascending order; list kb = k * nband + b, brow0[kb * (h + 1) + y] = first
    // position of row y
    int* bidx;     // [cap] feature index
    int* buc;      // [cap] u | v << 15 | class << 30 of that feature
    uint8_t* bd;   // [cap][32] its descriptor
    int* bpos;     // [cap] position of feature i in the index
    int* brow0;    // [4 nband][h + 1]
    int* bcnt;     // [4 nband][h] scratch
    int* n;        // [1]
    int* cnt;      // [h][tiles][4] per (row, tile, wave) segment: candidate counts of the
                   // four classes, 8 bits each
    int* list;     // [h][tiles][4][seg_cap] packed x | cls << 16
};

constexpr int kMaxCams = VISO_SVO_MAX_CAMS;

// the images of a batch of timesteps, nc cameras each: image z = timestep
// z / (2 nc), camera (z / 2) % nc, side z & 1 (left, right)
struct ImgSrc {
    const uint8_t* left[kMaxCams];
    const uint8_t* right[kMaxCams];
    long long pair_stride;  // bytes between consecutive timesteps
    __device__ const uint8_t* at(int z, int nc) const {
        const int cam = (z >> 1) % nc;
        return ((z & 1) ? right[cam] : left[cam]) + (long long)(z / (2 * nc)) * pair_stride;
    }
};

// per-batch estimation buffers: pair b of a batch (sequence frame frame0 + b)
// owns slot b of every array
struct PairArgs {
    const FeatDev* sets;
    int ring;
    long long frame0;
    int ncam;            // cameras per timestep (1: one stereo camera; > 1: rig)
    int cap, mcap;       // features per image, bucketed matches per timestep (all cameras)
    int4* circ;          // [P][cap]      {l1, r1, r2, -}
    int4* rec8;          // [P][2 cap]    {u_l1, v_l1, u_r1, v_r1}, {u_l2, v_l2, u_r2, v_r2}
    uint8_t* keep;       // [P][cap]
    int* uv8;            // [P][mcap * 8]
    uint8_t* mcam;       // [P][mcap] camera of each selected match
    double* obs;         // [P][mcap][kObs] each selected match's Obs (svo_obs_kernel)
    uint8_t* hok;        // [P][iters] hypothesis solved (svo_hyp_kernel)
    const double* extr;  // [ncam][12] rig -> camera extrinsics (rig only)
    int* n_sel;          // [P]
    int* counts;         // [P][iters]
    double* models;      // [P][iters * 12]
    uint8_t* sel;        // [P][mcap]
    uint8_t* inl;        // [P][mcap]
    double* motion;      // [P][12]
    int* stats;          // [P][8]
};

__device__ inline FeatDev set_frame(const PairArgs& a, long long frame, int cam, int side) {
    return a.sets[2 * ((int)(frame % a.ring) * a.ncam + cam) + side];
}

// ---------------------------------------------------------------- detect
// Thread per response column.  A workgroup stages the image rows of a tile
// (4 x (64 - 2n) output columns x kDTH output rows, plus halos) in LDS once
// (coalesced dword loads); each wave then owns a 64-column strip (its 64 - 2n
// output columns and n halo columns either side) and walks it down the rows
// on its own, with no workgroup barrier in the row loop: horizontal tap sums
// of a new image row from two LDS dwords (dot4), the 5x5 blob / checkerboard
// responses from a 5-row register window
//   B = 7 I + 2 S3x3 - S5x5,   C = g(y-2) + g(y-1) - g(y+1) - g(y+2),
//   g = (I(x+1) + I(x+2)) - (I(x-2) + I(x-1)),
// packed as (B, C) 16-bit pairs, so the four classes' strict NMS runs as
// packed max (B max, C max) and packed min (B min, C min) ops: horizontal
// neighbour extrema over +-n columns through the wave's LDS row buffer,
// vertical ones from a (2n+1)-row register window.  Features of an output row
// are emitted per (row, tile, wave) segment in (x, class) order by ballot
// ranks, with per-class counts.  Responses outside the domain [2, w-3] x
// [2, h-3] only matter when margin < n + 2 (DOM): then they enter the NMS as
// -inf / +inf.
constexpr int kDW = 256;                  // response columns per workgroup
constexpr int kDTH = 64;                  // output rows per tile
constexpr int kImgDw = (kDW + 4) / 4;     // LDS dwords per staged image row (260 bytes)

typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ inline s16x2 pk_max(s16x2 a, s16x2 b) { return __builtin_elementwise_max(a, b); }
__device__ inline s16x2 pk_min(s16x2 a, s16x2 b) { return __builtin_elementwise_min(a, b); }
__device__ inline uint32_t pk_bits(s16x2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ inline s16x2 pk_of(uint32_t v) { return __builtin_bit_cast(s16x2, v); }
__device__ inline int mbcnt64(unsigned long long b) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
}

// image z of a batch = pair z / 2 (left, right); its feature set lives in the
// ring slot of that pair
__device__ inline FeatDev set_of(const FeatDev* sets, int ring, int nc, int pair0, int z) {
    return sets[2 * (((pair0 + z / (2 * nc)) % ring) * nc + (z >> 1) % nc) + (z & 1)];
}

// The 1-D grid is dealt so that all tiles of one image share one XCD (block
// b runs on XCD b % 8, round-robin; speed only): the halo rows and columns
// that neighbouring tiles both stage are then fetched into one L2, not into
// several.  Block b: xcd = b % 8, q = b / 8, tile q % (tiles_x * tiles_y) of
// image 8 (q / (tiles_x * tiles_y)) + xcd.
template <int R, bool DOM>
__global__ __launch_bounds__(256) void svo_detect_kernel(ImgSrc src, SvoDev p,
                                                         const FeatDev* __restrict__ sets, int ring,
                                                         int pair0, int seg_cap, int tiles_x, int tiles_y,
                                                         int n_img) {
    const int xcd = blockIdx.x & 7, q = blockIdx.x >> 3, tpi = tiles_x * tiles_y;
    const int image = 8 * (q / tpi) + xcd, tile = q % tpi;
    if (image >= n_img) return;
    const int bx_ = tile % tiles_x, by_ = tile / tiles_x;
    constexpr int SW = 64 - 2 * R;    // output columns per wave strip
    constexpr int OW = 4 * SW;        // output columns per tile
    constexpr int RR = kDTH + 2 * R;  // response rows
    constexpr int IR = RR + 4;        // image rows
    constexpr int NV = 2 * R + 1;
    __shared__ uint32_t s_img[IR * kImgDw];
    __shared__ uint32_t s_rx[4][64 + 2 * R];                   // per wave: P (max view)
    __shared__ uint32_t s_rn[DOM ? 4 : 1][DOM ? 64 + 2 * R : 1];  // P (min view, DOM only)
    const uint8_t* __restrict__ img = src.at(image, p.ncam);
    const FeatDev F = set_of(sets, ring, p.ncam, pair0, image);
    const int w = p.w, h = p.h;
    const int x0 = bx_ * OW, y0 = by_ * kDTH;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // ---- stage image rows y0-R-2 .. y0+kDTH+R+1, columns x0-R-2 .. x0-R+257
    // (the tile uses OW + 2R + 4 <= 260 of them):
    // every load is issued unconditionally (clamped into the image buffer) before
    // the first LDS store, then shifted into place / zeroed where it was clamped
    {
        constexpr int NI = IR * kImgDw, NL = (NI + kDW - 1) / kDW;
        const long long n = (long long)w * h;
        const int gx0 = x0 - R - 2, gy0 = y0 - R - 2;
        uint32_t v[NL];
#pragma unroll
        for (int q = 0; q < NL; ++q) {
            const int i = tid + q * kDW;
            const int r = i / kImgDw, k = i - r * kImgDw;
            const long long o = (long long)(gy0 + r) * w + gx0 + 4 * k;
            const long long oc = min(max(o, 0LL), n - 4);
            v[q] = *reinterpret_cast<const __attribute__((address_space(1))) uint32_t*>(
                reinterpret_cast<uintptr_t>(img) + oc);
        }
#pragma unroll
        for (int q = 0; q < NL; ++q) {
            const int i = tid + q * kDW;
            if (q == NL - 1 && i >= NI) break;
            const int r = i / kImgDw, k = i - r * kImgDw;
            const int gy = gy0 + r;
            const long long o = (long long)gy * w + gx0 + 4 * k;
            const long long d = o - min(max(o, 0LL), n - 4);
            uint32_t x = v[q];
            if (gy < 0 || gy >= h || d <= -4 || d >= 4) x = 0;
            else if (d < 0) x <<= (uint32_t)(-8 * d);
            else if (d > 0) x >>= (uint32_t)(8 * d);
            s_img[i] = x;
        }
    }
    __syncthreads();
    const int col = wave * SW + lane;  // this thread's response column, tile-relative (x0 - R + col)
    const int x = x0 - R + col;
    const bool xin = lane >= R && lane < 64 - R && x >= p.margin && x < w - p.margin;
    const int tau = p.tau;
    const int sh = 8 * (col & 3);
    const uint32_t* srow = s_img + (col >> 2);
    uint32_t* bx = s_rx[wave];
    const int tiles = tiles_x;
    // Row rings of length L (image row i lives in slot i % L): the row loop is
    // unrolled L times, so every ring index is a compile-time constant and no
    // register moves are needed.  Vertical strict-neighbour extrema through a
    // sliding window of R rows built from power-of-two levels (M2, M4, M8):
    //   U(c) = max HI(c-R .. c-1) = W(c-1),  D(c) = max HI(c+1 .. c+R) = W(c+R),
    //   W(i) = max(M_K(i), M_K(i-R+K)), K = largest power of two <= R.
    constexpr int L = R + 2 > 5 ? R + 2 : 5;
    constexpr int K = R >= 8 ? 8 : (R >= 4 ? 4 : (R >= 2 ? 2 : 1));
    int H5[L], H3[L], G[L], Cc[L];
    s16x2 HX[L], HN[L], X2[L], N2[L], X4[L], N4[L], X8[L], N8[L], WX[L], WN[L], DP[L], DX[L], DN[L];
    for (int i0 = 0; i0 < IR; i0 += L) {
#pragma unroll
        for (int u = 0; u < L; ++u) {
            const int i = i0 + u;
            if (i >= IR) goto done;
            auto S = [&](int k) { return (u - k + 4 * L) % L; };  // slot of row i - k
            // taps a0..a4 = image columns x-2 .. x+2 of image row i
            const uint32_t lo = srow[i * kImgDw], hi = srow[i * kImgDw + 1];
            const uint32_t win = __builtin_amdgcn_alignbyte(hi, lo, col & 3);  // a0..a3
            const int a4 = (int)((hi >> sh) & 0xffu);
            H5[S(0)] = (int)__builtin_amdgcn_udot4(win, 0x01010101u, 0u, false) + a4;
            H3[S(0)] = (int)__builtin_amdgcn_udot4(win, 0x01010100u, 0u, false);
            G[S(0)] = ((int)(win >> 24) + a4) - (int)__builtin_amdgcn_udot4(win, 0x00000101u, 0u, false);
            Cc[S(0)] = (int)((win >> 16) & 0xffu);
            if (i < 4) continue;
            const int j = i - 4;  // response row: y = y0 - R + j (centre image row i - 2)
            const int B = (7 * Cc[S(2)] + 2 * ((H3[S(3)] + H3[S(2)]) + H3[S(1)])) -
                          ((((H5[S(4)] + H5[S(3)]) + H5[S(2)]) + H5[S(1)]) + H5[S(0)]);
            const int C = (G[S(4)] + G[S(3)]) - (G[S(1)] + G[S(0)]);
            const s16x2 P = {(short)B, (short)C};
            s16x2 PX = P, PN = P;
            if (DOM) {
                const int y = y0 - R + j;
                if (x < 2 || x >= w - 2 || y < 2 || y >= h - 2) {
                    PX = s16x2{-32768, -32768};
                    PN = s16x2{32767, 32767};
                }
            }
            // the wave's row buffer: LDS ops of one wave complete in order, so the
            // fences only keep the compiler from moving them across each other
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            bx[lane + R] = pk_bits(PX);
            if (DOM) s_rn[wave][lane + R] = pk_bits(PN);
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            s16x2 EX = s16x2{-32768, -32768}, EN = s16x2{32767, 32767};
#pragma unroll
            for (int d = 1; d <= R; ++d) {
                const s16x2 l = pk_of(bx[lane + R - d]), r = pk_of(bx[lane + R + d]);
                EX = pk_max(EX, pk_max(l, r));
                if (DOM) {
                    const uint32_t* bn = s_rn[wave];
                    EN = pk_min(EN, pk_min(pk_of(bn[lane + R - d]), pk_of(bn[lane + R + d])));
                } else {
                    EN = pk_min(EN, pk_min(l, r));
                }
            }
            DP[S(0)] = P;
            DX[S(0)] = EX;
            DN[S(0)] = EN;
            HX[S(0)] = pk_max(EX, PX);
            HN[S(0)] = pk_min(EN, PN);
            s16x2 MX = HX[S(0)], MN = HN[S(0)], MXo = HX[S(R - K)], MNo = HN[S(R - K)];
            if (K >= 2) {
                X2[S(0)] = pk_max(HX[S(0)], HX[S(1)]);
                N2[S(0)] = pk_min(HN[S(0)], HN[S(1)]);
                MX = X2[S(0)], MN = N2[S(0)], MXo = X2[S(R - K)], MNo = N2[S(R - K)];
            }
            if (K >= 4) {
                X4[S(0)] = pk_max(X2[S(0)], X2[S(2)]);
                N4[S(0)] = pk_min(N2[S(0)], N2[S(2)]);
                MX = X4[S(0)], MN = N4[S(0)], MXo = X4[S(R - K)], MNo = N4[S(R - K)];
            }
            if (K >= 8) {
                X8[S(0)] = pk_max(X4[S(0)], X4[S(4)]);
                N8[S(0)] = pk_min(N4[S(0)], N4[S(4)]);
                MX = X8[S(0)], MN = N8[S(0)], MXo = X8[S(R - K)], MNo = N8[S(R - K)];
            }
            WX[S(0)] = R == K ? MX : pk_max(MX, MXo);
            WN[S(0)] = R == K ? MN : pk_min(MN, MNo);
            if (j < 2 * R) continue;
            const int yc = y0 + j - 2 * R;  // centre (output) row = response row j - R
            if (yc >= h) goto done;         // uniform: no later row of the tile is in the image
            const s16x2 NX = pk_max(pk_max(WX[S(R + 1)], WX[S(0)]), DX[S(R)]);
            const s16x2 NN = pk_min(pk_min(WN[S(R + 1)], WN[S(0)]), DN[S(R)]);
            int flags = 0;
            if (xin && yc >= p.margin && yc < h - p.margin) {
                const int b = DP[S(R)].x, c = DP[S(R)].y;
                flags = (b > tau && b > NX.x ? 1 : 0) | (-b > tau && b < NN.x ? 2 : 0) |
                        (c > tau && c > NX.y ? 4 : 0) | (-c > tau && c < NN.y ? 8 : 0);
            }
            const unsigned long long q0 = __ballot(flags & 1), q1 = __ballot(flags & 2),
                                     q2 = __ballot(flags & 4), q3 = __ballot(flags & 8);
            const size_t seg = ((size_t)yc * tiles + bx_) * 4 + wave;
            if (q0 | q1 | q2 | q3) {
                int pos = (mbcnt64(q0) + mbcnt64(q1)) + (mbcnt64(q2) + mbcnt64(q3));
                int* list = F.list + seg * seg_cap;
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (flags & (1 << k)) {
                        if (pos < seg_cap) list[pos] = x | (k << 16);
                        ++pos;
                    }
            }
            // per-class counts (strict NMS: <= ceil(64 / (n + 1)) <= 32 per class)
            if (lane == 0)
                F.cnt[seg] = __popcll(q0) | (__popcll(q1) << 8) | (__popcll(q2) << 16) | (__popcll(q3) << 24);
        }
    }
done:;
}

// exclusive block prefix (1024 threads): wave scans by shuffles + wave totals
__device__ inline int block_excl_scan(int v, int* s_w, int& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
    }
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    int base = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int t = s_w[k];
        base += k < wave ? t : 0;
        tot += t;
    }
    __syncthreads();
    total = tot;
    return base + incl - v;
}

__device__ inline int bytesum(int c) { return (c & 0xff) + ((c >> 8) & 0xff) + ((c >> 16) & 0xff) + ((c >> 24) & 0xff); }
__device__ inline int pack_uvc(int u, int v, int c) { return u | (v << 15) | (c << 30); }

// Per image, one workgroup of 1024 threads, every phase parallel over rows,
// (column, row-chunk) items or segments:
//   1. row totals and each segment's offset within its row (thread per row);
//   2. exclusive scan of the row totals -> row starts; segment offsets made
//      absolute; row0 / n (capped at the feature capacity);
//   3. class-band index: column kb = class k x band (segment column s), rows
//      ascending; the kept (row-major index < cap) class-k counts summed per
//      (column, chunk of CR rows), one exclusive scan over the items in
//      (column, chunk) order = the index order, then brow0 row by row;
//   4. thread per segment: the features' u, v, class at their row-major index
//      and their index entries (rank among the segment's class-k entries).
constexpr int kScanItems = 8192;

__global__ __launch_bounds__(1024) void svo_scan_kernel(SvoDev p, const FeatDev* __restrict__ sets, int ring,
                                                        int pair0, int segs, int seg_cap) {
    const FeatDev F = set_of(sets, ring, p.ncam, pair0, blockIdx.x);
    __shared__ int s_w[16];
    __shared__ int s_total;
    __shared__ int s_item[kScanItems];
    const int h = p.h, tid = threadIdx.x, cap = p.cap;
    int* off = F.bcnt;                      // [h][segs] offset of each segment
    int* rs = F.bcnt + (size_t)h * segs;    // [h] row starts (uncapped)
    // ---- 1
    for (int y = tid; y < h; y += 1024) {
        const int* c = F.cnt + (size_t)y * segs;
        int* o = off + (size_t)y * segs;
        int acc = 0;
#pragma unroll 8
        for (int s = 0; s < segs; ++s) {
            o[s] = acc;
            acc += bytesum(c[s]);
        }
        rs[y] = acc;
    }
    __syncthreads();
    // ---- 2
    {
        const int per = (h + 1023) / 1024, b = min(tid * per, h), e = min(b + per, h);
        int sum = 0;
        for (int y = b; y < e; ++y) sum += rs[y];
        int total;
        int acc = block_excl_scan(sum, s_w, total);
        for (int y = b; y < e; ++y) {
            const int t = rs[y];
            rs[y] = acc;
            F.row0[y] = min(acc, cap);
            acc += t;
        }
        if (tid == 0) {
            F.row0[h] = min(total, cap);
            *F.n = min(total, cap);
            s_total = total;
        }
    }
    __syncthreads();
    for (int y = tid; y < h; y += 1024) {
        int* o = off + (size_t)y * segs;
        const int r = rs[y];
#pragma unroll 8
        for (int s = 0; s < segs; ++s) o[s] += r;
    }
    __syncthreads();
    // ---- 3
    const bool full = s_total <= cap;  // nothing truncated: every count is kept
    auto kept = [&](int y, int s, int k) {
        const size_t i = (size_t)y * segs + s;
        const int c4 = F.cnt[i];
        if (full) return (c4 >> (8 * k)) & 0xff;
        const int c = bytesum(c4), lim = min(c, max(cap - off[i], 0));
        if (lim == c) return (c4 >> (8 * k)) & 0xff;
        const int* list = F.list + i * seg_cap;
        int r = 0;
        for (int q = 0; q < lim; ++q) r += (list[q] >> 16) == k ? 1 : 0;
        return r;
    };
    const int ncol = 4 * segs;
    int cr = 32;
    while ((long long)ncol * ((h + cr - 1) / cr) > kScanItems) cr *= 2;
    const int nch = (h + cr - 1) / cr, items = ncol * nch;
    for (int it = tid; it < items; it += 1024) {
        const int col = it / nch, ch = it - col * nch, k = col / segs, s = col - k * segs;
        const int y0 = ch * cr, y1 = min(y0 + cr, h);
        int sum = 0;
#pragma unroll 8
        for (int y = y0; y < y1; ++y) sum += kept(y, s, k);
        s_item[it] = sum;
    }
    __syncthreads();
    {
        const int per = (items + 1023) / 1024, b = min(tid * per, items), e = min(b + per, items);
        int sum = 0;
        for (int it = b; it < e; ++it) sum += s_item[it];
        int total;
        int acc = block_excl_scan(sum, s_w, total);
        for (int it = b; it < e; ++it) {
            const int t = s_item[it];
            s_item[it] = acc;
            acc += t;
        }
    }
    __syncthreads();
    for (int it = tid; it < items; it += 1024) {
        const int col = it / nch, ch = it - col * nch, k = col / segs, s = col - k * segs;
        const int y0 = ch * cr, y1 = min(y0 + cr, h);
        int* b0 = F.brow0 + (size_t)col * (h + 1);
        int acc = s_item[it];
#pragma unroll 8
        for (int y = y0; y < y1; ++y) {
            b0[y] = acc;
            acc += kept(y, s, k);
        }
        if (y1 == h) b0[h] = acc;
    }
    __syncthreads();
    // ---- 4
    const int n = h * segs;
    for (int i = tid; i < n; i += 1024) {
        const int c4 = F.cnt[i];
        if (!c4) continue;
        const int y = i / segs, s = i - y * segs;
        const int c = bytesum(c4), o0 = off[i], lim = min(c, max(cap - o0, 0));
        const int* list = F.list + (size_t)i * seg_cap;
        int rank[4] = {0, 0, 0, 0};
        for (int q = 0; q < c; ++q) {
            const int o = o0 + q;
            if (o >= cap) break;
            const int ent = list[q], k = ent >> 16, u = ent & 0xffff;
            F.u[o] = u;
            F.v[o] = y;
            F.c[o] = k;
            if (q < lim) {
                const int pos = F.brow0[(size_t)(k * segs + s) * (h + 1) + y] + rank[k]++;
                F.bidx[pos] = o;
                F.buc[pos] = pack_uvc(u, y, k);
                F.bpos[o] = pos;
            }
        }
    }
}

// The same scan with the per-segment tables in LDS (images whose h x segs
// candidate counts fit kScanLds ints: 1242x375 has 9,000): the counts are
// read from HBM once, coalesced, and every prefix walk runs in LDS.  The
// class-band index is built column by column, one wave per column: a wave
// scan over 64 rows at a time gives each row's brow0, stored coalesced.
// Same outputs as svo_scan_kernel, bit for bit (integer work).
constexpr int kScanLds = 12288;

__global__ __launch_bounds__(1024) void svo_scan_lds_kernel(SvoDev p, const FeatDev* __restrict__ sets, int ring,
                                                            int pair0, int segs, int seg_cap) {
    const FeatDev F = set_of(sets, ring, p.ncam, pair0, blockIdx.x);
    extern __shared__ int s_dyn[];
    __shared__ int s_w[16];
    __shared__ int s_total;
    const int h = p.h, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, cap = p.cap;
    const int n = h * segs, ncol = 4 * segs;
    int* s_cnt = s_dyn;          // [h][segs] candidate counts (4 classes, 8 bits each)
    int* s_off = s_cnt + n;      // [h][segs] first feature index of the segment
    int* s_rs = s_off + n;       // [h] row starts
    int* s_col = s_rs + h;       // [4 segs] first index position of each class-band column
    for (int i = tid; i < n; i += 1024) s_cnt[i] = F.cnt[i];
    __syncthreads();
    // ---- 1: offsets within the row, row totals
    for (int y = tid; y < h; y += 1024) {
        int acc = 0;
        for (int s = 0; s < segs; ++s) {
            s_off[y * segs + s] = acc;
            acc += bytesum(s_cnt[y * segs + s]);
        }
        s_rs[y] = acc;
    }
    __syncthreads();
    // ---- 2: row starts
    {
        const int per = (h + 1023) / 1024, b = min(tid * per, h), e = min(b + per, h);
        int sum = 0;
        for (int y = b; y < e; ++y) sum += s_rs[y];
        int total;
        int acc = block_excl_scan(sum, s_w, total);
        for (int y = b; y < e; ++y) {
            const int t = s_rs[y];
            s_rs[y] = acc;
            acc += t;
        }
        if (tid == 0) {
            F.row0[h] = min(total, cap);
            *F.n = min(total, cap);
            s_total = total;
        }
    }
    __syncthreads();
    for (int y = tid; y < h; y += 1024) F.row0[y] = min(s_rs[y], cap);
    for (int i = tid; i < n; i += 1024) s_off[i] += s_rs[i / segs];
    __syncthreads();
    // ---- 3: class-band index (column kb = class k x band s, rows ascending)
    const bool full = s_total <= cap;
    auto kept = [&](int y, int s, int k) {
        const int i = y * segs + s;
        const int c4 = s_cnt[i];
        if (full) return (c4 >> (8 * k)) & 0xff;
        const int c = bytesum(c4), lim = min(c, max(cap - s_off[i], 0));
        if (lim == c) return (c4 >> (8 * k)) & 0xff;
        const int* list = F.list + (size_t)i * seg_cap;
        int r = 0;
        for (int q = 0; q < lim; ++q) r += (list[q] >> 16) == k ? 1 : 0;
        return r;
    };
    for (int col = wave; col < ncol; col += 16) {  // column totals
        const int k = col / segs, s = col - k * segs;
        int t = 0;
        for (int y = lane; y < h; y += 64) t += kept(y, s, k);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
        if (lane == 0) s_col[col] = t;
    }
    __syncthreads();
    {
        const int v = tid < ncol ? s_col[tid] : 0;
        int total;
        const int e = block_excl_scan(v, s_w, total);
        if (tid < ncol) s_col[tid] = e;
    }
    __syncthreads();
    for (int col = wave; col < ncol; col += 16) {
        const int k = col / segs, s = col - k * segs;
        int* b0 = F.brow0 + (size_t)col * (h + 1);
        int base = s_col[col];
        for (int y0 = 0; y0 < h; y0 += 64) {
            const int y = y0 + lane;
            const int v = y < h ? kept(y, s, k) : 0;
            int incl = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int t = __shfl_up(incl, o, 64);
                if (lane >= o) incl += t;
            }
            if (y < h) b0[y] = base + incl - v;
            base += __shfl(incl, 63, 64);
        }
        if (lane == 0) b0[h] = base;
    }
    __syncthreads();
    // ---- 4: thread per stored feature o (row-major index < cap): its segment
    // is the last one starting at or before o (binary search over the LDS
    // offsets), its class rank among the segment's earlier entries gives its
    // index position; u / v / class / bpos stores are coalesced
    const int nf = min(s_total, cap);
    for (int o = tid; o < nf; o += 1024) {
        int lo = 0, hi = n - 1;  // s_off[lo] <= o < s_off[hi + 1]
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (s_off[mid] <= o) lo = mid;
            else hi = mid - 1;
        }
        const int i = lo, y = i / segs, s = i - y * segs, q = o - s_off[i];
        const int* list = F.list + (size_t)i * seg_cap;
        const int ent = list[q], k = ent >> 16, u = ent & 0xffff;
        int rank = 0;
        for (int r = 0; r < q; ++r) rank += (list[r] >> 16) == k ? 1 : 0;
        F.u[o] = u;
        F.v[o] = y;
        F.c[o] = k;
        const int pos = F.brow0[(size_t)(k * segs + s) * (h + 1) + y] + rank;
        F.bidx[pos] = o;
        F.buc[pos] = pack_uvc(u, y, k);
        F.bpos[o] = pos;
    }
}

__device__ inline int sobel_q(const uint8_t* I, int w, int x, int y, bool du) {
    auto px = [&](int dx, int dy) { return (int)I[(size_t)(y + dy) * w + x + dx]; };
    const int d = du ? (px(1, -1) + 2 * px(1, 0) + px(1, 1)) - (px(-1, -1) + 2 * px(-1, 0) + px(-1, 1))
                     : (px(-1, 1) + 2 * px(0, 1) + px(1, 1)) - (px(-1, -1) + 2 * px(0, -1) + px(1, -1));
    return (d >> 3) + 128;
}

// 16 lanes per feature (lane j: sample offset j): the 32-byte descriptor.
// kDescWg workgroups per image, grid-stride over its features; the 1-D grid
// is dealt so that all of an image's workgroups share one XCD (blocks are
// dealt round-robin over the 8 XCDs: block b runs on XCD b % 8; speed only):
// every image row is then fetched into one L2, not into all eight.
constexpr int kDescWg = 16;

__global__ __launch_bounds__(256) void svo_describe_kernel(ImgSrc src, SvoDev p,
                                                           const FeatDev* __restrict__ sets, int ring,
                                                           int pair0, int n_img) {
    const int xcd = blockIdx.x & 7, q = blockIdx.x >> 3;
    const int wg = q % kDescWg, image = 8 * (q / kDescWg) + xcd;
    if (image >= n_img) return;
    const uint8_t* __restrict__ img = src.at(image, p.ncam);
    const FeatDev F = set_of(sets, ring, p.ncam, pair0, image);
    const int n = *F.n;
    const int j = threadIdx.x & 15;
    for (int o = wg * 16 + (threadIdx.x >> 4); o < n; o += kDescWg * 16) {
        const int sx = F.u[o] + c_p16[j][0], sy = F.v[o] + c_p16[j][1];
        const uint8_t du = (uint8_t)sobel_q(img, p.w, sx, sy, true), dv = (uint8_t)sobel_q(img, p.w, sx, sy, false);
        const size_t bp = (size_t)F.bpos[o] * kDesc;
        F.d[(size_t)o * kDesc + j] = du;
        F.d[(size_t)o * kDesc + 16 + j] = dv;
        F.bd[bp + j] = du;
        F.bd[bp + 16 + j] = dv;
    }
}

// Column-band index of a feature set (one workgroup of 1024 threads per
// set): per (band, row) counts by a thread per row, a band-major exclusive
// scan, then each row's features placed in index order.  The matching
// searches then visit only the bands their column window overlaps.
// Bands are the detect kernel's (tile, wave) column segments (wave w of tile
// t: output columns t*ow + w*(64 - 2n) .. + 63 - 2n), so the feature pass
// emits the band-major order directly (svo_scan_kernel); this kernel builds
// the same index for feature sets uploaded by viso_svo_match.
// floor(a / b) for 0 <= a < 2^24 from a float reciprocal, corrected to exact
__device__ inline int div_floor(int a, int b, float inv_b) {
    int q = (int)((float)a * inv_b);
    q -= q * b > a ? 1 : 0;
    q += (q + 1) * b <= a ? 1 : 0;
    return q;
}

__device__ inline int band_of(int u, const SvoDev& p) {
    const int t = div_floor(u, p.ow, p.inv_ow);
    return min(max(4 * t + div_floor(u - t * p.ow, p.sw, p.inv_sw), 0), p.nband - 1);
}

__global__ __launch_bounds__(1024) void svo_index_kernel(SvoDev p, const FeatDev* __restrict__ sets, int ring,
                                                         int pair0) {
    const FeatDev F = set_of(sets, ring, p.ncam, pair0, blockIdx.x);
    __shared__ int s_w[16];
    const int h = p.h, nk = 4 * p.nband, tid = threadIdx.x;
    auto kb_of = [&](int i) { return F.c[i] * p.nband + band_of(F.u[i], p); };
    for (int y = tid; y < h; y += 1024) {
        for (int kb = 0; kb < nk; ++kb) F.bcnt[kb * h + y] = 0;
        const int e = F.row0[y + 1];
        for (int i = F.row0[y]; i < e; ++i) ++F.bcnt[kb_of(i) * h + y];
    }
    __syncthreads();
    const int n = nk * h;
    const int per = (n + 1023) / 1024;
    const int b0 = min(tid * per, n), e0 = min(b0 + per, n);
    int sum = 0;
    for (int i = b0; i < e0; ++i) sum += F.bcnt[i];
    int total;
    int acc = block_excl_scan(sum, s_w, total);
    for (int i = b0; i < e0; ++i) {
        const int kb = i / h, y = i - kb * h;
        F.brow0[kb * (h + 1) + y] = acc;
        acc += F.bcnt[i];
        if (y == h - 1) F.brow0[kb * (h + 1) + h] = acc;
    }
    __syncthreads();
    for (int y = tid; y < h; y += 1024) {
        const int r0 = F.row0[y], e = F.row0[y + 1];
        for (int i = r0; i < e; ++i) {
            const int kb = kb_of(i);
            int rank = 0;
            for (int k = r0; k < i; ++k) rank += kb_of(k) == kb ? 1 : 0;
            const int pos = F.brow0[kb * (h + 1) + y] + rank;
            F.bidx[pos] = i;
            F.buc[pos] = pack_uvc(F.u[i], y, F.c[i]);
            F.bpos[i] = pos;
            for (int q = 0; q < kDesc; ++q) F.bd[(size_t)pos * kDesc + q] = F.d[(size_t)i * kDesc + q];
        }
    }
}

// ---------------------------------------------------------------- matching
__device__ inline int sad32(const uint4 a0, const uint4 a1, const uint4 b0, const uint4 b1) {
    unsigned s = 0;
    s = __builtin_amdgcn_sad_u8(a0.x, b0.x, s);
    s = __builtin_amdgcn_sad_u8(a0.y, b0.y, s);
    s = __builtin_amdgcn_sad_u8(a0.z, b0.z, s);
    s = __builtin_amdgcn_sad_u8(a0.w, b0.w, s);
    s = __builtin_amdgcn_sad_u8(a1.x, b1.x, s);
    s = __builtin_amdgcn_sad_u8(a1.y, b1.y, s);
    s = __builtin_amdgcn_sad_u8(a1.z, b1.z, s);
    s = __builtin_amdgcn_sad_u8(a1.w, b1.w, s);
    return (int)s;
}

// wave minimum by DPP butterflies (quad_perm xor 1 / xor 2, then half-row /
// row mirrors on the already uniform groups) and the gfx950 permlane16/32
// swaps: every lane ends with the minimum.  All 64 lanes must be active.
__device__ inline unsigned wave_min_u32(unsigned v) {
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false));
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false));
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false));
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false));
    const auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    v = min((unsigned)a[0], (unsigned)a[1]);
    const auto b = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return min((unsigned)b[0], (unsigned)b[1]);
}

constexpr int kMaxQB = 8;  // column bands a search window may span (svo_check)

// The best candidate of a search: feature index j (-1: none), its u, v and
// descriptor (so the next search of the circle needs no extra loads).
struct Cand {
    int j, u, v;
    uint4 d0, d1;
};

// best candidate in `S` for the query (u, v, class c, desc): rows [v - dv,
// v + dv], u - du_hi <= u' <= u - du_lo; min SAD, ties -> lowest index.  The
// class-c lists of the column bands the window overlaps give one contiguous
// position range each (lanes 0..nq-1 load the bounds, a wave scan
// concatenates them); every candidate's packed (u, v, class), index and
// descriptor are loaded together, 128 candidates per step; the winner's data
// is reloaded by scalar loads.  Wave-uniform arguments and result.
__device__ Cand best_match(const FeatDev& S, const SvoDev& p, int u, int v, int c, uint4 q0, uint4 q1,
                           int du_lo, int du_hi, int dv) {
    Cand r;
    r.j = -1;
    r.u = r.v = 0;
    r.d0 = r.d1 = make_uint4(0, 0, 0, 0);
    const int lane = threadIdx.x & 63, h = p.h;
    u = __builtin_amdgcn_readfirstlane(u);
    v = __builtin_amdgcn_readfirstlane(v);
    c = __builtin_amdgcn_readfirstlane(c);
    const int va = max(v - dv, 0), vb = min(v + dv, h - 1);
    const int ua = u - du_hi, ub = u - du_lo;
    if (ub < 0) return r;
    const int ba = band_of(max(ua, 0), p), bq = band_of(ub, p);
    const int nq = bq - ba + 1;  // <= kMaxQB: windows up to ~7 bands (disp_max 255 spans <= 6)
    int s = 0, len = 0;
    if (lane < min(nq, kMaxQB)) {
        const int* rw = S.brow0 + (size_t)(c * p.nband + ba + lane) * (h + 1);
        s = rw[va];
        len = rw[vb + 1] - s;
    }
    // band l covers candidate slots [E[l], E[l + 1]) at positions k + O[l]
    // (scalars; bands past nq have len = 0)
    int E[kMaxQB], O[kMaxQB], total = 0;
#pragma unroll
    for (int l = 0; l < kMaxQB; ++l) {
        const int sl = __builtin_amdgcn_readlane(s, l), ll = __builtin_amdgcn_readlane(len, l);
        E[l] = total;
        O[l] = sl - total;
        total += ll;
    }
    unsigned best = 0xffffffffu;
    // candidate slot k of the concatenated ranges -> its index position
    auto pos_of = [&](int k) {
        int ps = k + O[0];
#pragma unroll
        for (int l = 1; l < kMaxQB; ++l) {
            if (l >= nq) break;
            ps = k >= E[l] ? k + O[l] : ps;
        }
        return ps;
    };
    auto consider = [&](int e, int j, uint4 d0, uint4 d1) {
        const int dd = u - (e & 0x7fff);
        if (dd < du_lo || dd > du_hi) return;
        best = min(best, ((unsigned)sad32(q0, q1, d0, d1) << 15) | (unsigned)j);
    };
    for (int k0 = 0; k0 < total; k0 += 128) {
        // two candidates per lane, all loads issued before the first use;
        // lanes past the end load nothing
        const int ka = k0 + lane, kb = ka + 64;
        const bool two = k0 + 64 < total;  // wave-uniform
        int ea = 0, eb = 0, ja = 0, jb = 0;
        uint4 a0 = make_uint4(0, 0, 0, 0), a1 = a0, b0 = a0, b1 = a0;
        if (ka < total) {
            const int ps = pos_of(ka);
            ea = S.buc[ps];
            ja = S.bidx[ps];
            const uint4* da = reinterpret_cast<const uint4*>(S.bd + (size_t)ps * kDesc);
            a0 = da[0];
            a1 = da[1];
        }
        if (two && kb < total) {
            const int ps = pos_of(kb);
            eb = S.buc[ps];
            jb = S.bidx[ps];
            const uint4* db = reinterpret_cast<const uint4*>(S.bd + (size_t)ps * kDesc);
            b0 = db[0];
            b1 = db[1];
        }
        if (ka < total) consider(ea, ja, a0, a1);
        if (two && kb < total) consider(eb, jb, b0, b1);
    }
    const unsigned wbest = (unsigned)__builtin_amdgcn_readfirstlane((int)wave_min_u32(best));
    if (wbest == 0xffffffffu) return r;
    // the winner's coordinates and descriptor: uniform (scalar) loads
    const int j = (int)(wbest & 0x7fffu);
    r.j = j;
    r.u = S.u[j];
    r.v = S.v[j];
    const uint4* dj = reinterpret_cast<const uint4*>(S.d + (size_t)j * kDesc);
    r.d0 = dj[0];
    r.d1 = dj[1];
    return r;
}

// Workgroup -> (slot, chunk) so that consecutive (timestep, camera) slots
// share an XCD: blocks b and b + 8 are dealt to the same XCD (MI355X guide,
// workgroup dispatch), so block b serves slot (b % 8) * per + j, chunk c with
// b / 8 = j * chunks + c.  A slot's four feature sets (and the next slot's
// previous pair) then stay in one XCD's L2.  Returns false for padding blocks.
__device__ inline bool xcd_slot(int nq, int chunks, int& slot, int& chunk) {
    const int per = (nq + 7) >> 3;
    const int b = blockIdx.x, s = b >> 3;
    const int j = s / chunks;
    chunk = s - j * chunks;
    slot = (b & 7) * per + j;
    return j < per && slot < nq;
}

// wave per current-left feature of (timestep, camera) slot q (b0 * ncam +
// the block's slot); circ[i2] = {l1, r1, r2, -} and rec8[i2] = {u_l1, v_l1,
// u_r1, v_r1, u_l2, v_l2, u_r2, v_r2}, or circ[i2].x = rec8[i2].x = -1.  The
// four searches chain through the winners' coordinates and descriptors.
__global__ __launch_bounds__(256) void svo_circle_kernel(SvoDev p, PairArgs pa, int b0, int nq, int chunks) {
    int qr, chunk;
    if (!xcd_slot(nq, chunks, qr, chunk)) return;
    const int q = b0 * pa.ncam + qr;
    const int pb = q / pa.ncam, cam = q - pb * pa.ncam;
    const long long fr = pa.frame0 + pb;
    const FeatDev L1 = set_frame(pa, fr - 1, cam, 0), R1 = set_frame(pa, fr - 1, cam, 1),
                  L2 = set_frame(pa, fr, cam, 0), R2 = set_frame(pa, fr, cam, 1);
    int4* __restrict__ out = pa.circ + (size_t)q * pa.cap;
    int4* __restrict__ rec8 = pa.rec8 + (size_t)q * 2 * pa.cap;
    uint8_t* __restrict__ keep = pa.keep + (size_t)q * pa.cap;
    const int n2 = *L2.n;
    const int D = p.disp_max, Rr = p.radius;
    const int lane = threadIdx.x & 63;
    for (int i2 = chunk * 4 + (threadIdx.x >> 6); i2 < n2; i2 += chunks * 4) {
        const int c = L2.c[i2], u2 = L2.u[i2], v2 = L2.v[i2];
        const uint4* dq = reinterpret_cast<const uint4*>(L2.d + (size_t)i2 * kDesc);
        const uint4 a = dq[0], b = dq[1];
        int4 res = make_int4(-1, -1, -1, 0);
        int4 ra = make_int4(-1, 0, 0, 0), rb = make_int4(0, 0, 0, 0);
        const Cand r2 = best_match(R2, p, u2, v2, c, a, b, 0, D, 1);  // left_t -> right_t
        if (r2.j >= 0) {
            const Cand r1 = best_match(R1, p, r2.u, r2.v, c, r2.d0, r2.d1, -Rr, Rr, Rr);  // -> right_t-1
            if (r1.j >= 0) {
                const Cand l1 = best_match(L1, p, r1.u, r1.v, c, r1.d0, r1.d1, -D, 0, 1);  // -> left_t-1
                if (l1.j >= 0) {
                    const Cand i2b = best_match(L2, p, l1.u, l1.v, c, l1.d0, l1.d1, -Rr, Rr, Rr);  // -> left_t
                    if (i2b.j == i2 && l1.u - r1.u >= 1 && u2 - r2.u >= 1) {
                        res = make_int4(l1.j, r1.j, r2.j, 0);
                        ra = make_int4(l1.u, l1.v, r1.u, r1.v);
                        rb = make_int4(u2, v2, r2.u, r2.v);
                    }
                }
            }
        }
        if (lane == 0) out[i2] = res;
        if (lane == 2) keep[i2] = 0;
        if (lane == 1) {
            rec8[2 * (size_t)i2] = ra;
            rec8[2 * (size_t)i2 + 1] = rb;
        }
    }
}

// ---------------------------------------------------------------- pose math
// (oracle_svo.cpp: make_obs, transform, residual_rows, match_sums, solve6,
// apply_update, is_inlier — same expressions, same order)
struct Obs {
    double X, Y, Z, uL, vL, uR, vR;
    const double* E;  // rig: extrinsic of the match's camera (rig -> camera), else null
    double Xr[3];     // rig: the point in the rig frame t-1
};

__device__ inline Obs make_obs(const int* m, const SvoDev& p) {
    Obs o;
    const double d = (double)(m[0] - m[2]);
    o.Z = (p.fx * p.base) / d;
    o.X = (((double)m[0] - p.cu) * o.Z) / p.fx;
    o.Y = (((double)m[1] - p.cv) * o.Z) / p.fy;
    o.uL = (double)m[4];
    o.vL = (double)m[5];
    o.uR = (double)m[6];
    o.vR = (double)m[7];
    o.E = nullptr;
    return o;
}

// match m of a timestep's selection; rig (ncam > 1): with its camera's
// extrinsic E and the rig-frame point Xr = Re^T (X - te) (oracle make_obs_rig)
__device__ inline Obs obs_at(const int* uv8, const uint8_t* mcam, int m, const PairArgs& pa, const SvoDev& p) {
    Obs o = make_obs(uv8 + 8 * (size_t)m, p);
    o.Xr[0] = o.Xr[1] = o.Xr[2] = 0.0;
    if (pa.ncam > 1) {
        const double* E = pa.extr + 12 * (int)mcam[m];
        o.E = E;
        const double d0 = o.X - E[9], d1 = o.Y - E[10], d2 = o.Z - E[11];
#pragma unroll
        for (int k = 0; k < 3; ++k) o.Xr[k] = ((E[k] * d0 + E[3 + k] * d1) + E[6 + k] * d2);
    }
    return o;
}

// Obs of the selected matches, computed once per timestep (svo_obs_kernel):
// X, Y, Z, uL, vL, uR, vR, camera, Xr[3]
constexpr int kObs = 12;

__device__ inline void obs_store(double* O, const Obs& o, int cam) {
    const double v[kObs] = {o.X, o.Y, o.Z, o.uL, o.vL, o.uR, o.vR, (double)cam, o.Xr[0], o.Xr[1], o.Xr[2], 0.0};
#pragma unroll
    for (int k = 0; k < kObs; ++k) O[k] = v[k];
}

__device__ inline Obs obs_load(const double* __restrict__ O, const PairArgs& pa) {
    Obs o;
    const double2* q = reinterpret_cast<const double2*>(O);
    const double2 a = q[0], b = q[1], c = q[2], d = q[3], e = q[4];
    o.X = a.x;
    o.Y = a.y;
    o.Z = b.x;
    o.uL = b.y;
    o.vL = c.x;
    o.uR = c.y;
    o.vR = d.x;
    o.E = pa.ncam > 1 ? pa.extr + 12 * (int)d.y : nullptr;
    o.Xr[0] = e.x;
    o.Xr[1] = e.y;
    o.Xr[2] = O[10];
    return o;
}

// rig: Q = R Xr + t (rig frame t), P = Re Q + te (camera frame t)
__device__ inline void rig_point(const double* R, const double* t, const Obs& o, double* Q, double* P) {
    Q[0] = ((R[0] * o.Xr[0] + R[1] * o.Xr[1]) + R[2] * o.Xr[2]) + t[0];
    Q[1] = ((R[3] * o.Xr[0] + R[4] * o.Xr[1]) + R[5] * o.Xr[2]) + t[1];
    Q[2] = ((R[6] * o.Xr[0] + R[7] * o.Xr[1]) + R[8] * o.Xr[2]) + t[2];
    const double* E = o.E;
    P[0] = ((E[0] * Q[0] + E[1] * Q[1]) + E[2] * Q[2]) + E[9];
    P[1] = ((E[3] * Q[0] + E[4] * Q[1]) + E[5] * Q[2]) + E[10];
    P[2] = ((E[6] * Q[0] + E[7] * Q[1]) + E[8] * Q[2]) + E[11];
}

__device__ inline void transform(const double* R, const double* t, const Obs& o, double* P) {
    P[0] = ((R[0] * o.X + R[1] * o.Y) + R[2] * o.Z) + t[0];
    P[1] = ((R[3] * o.X + R[4] * o.Y) + R[5] * o.Z) + t[1];
    P[2] = ((R[6] * o.X + R[7] * o.Y) + R[8] * o.Z) + t[2];
}

__device__ inline void residual_rows(const double* P, const Obs& o, const SvoDev& p, double* e,
                                     double (*J)[6]) {
    const double iz = 1.0 / P[2];
    const double iz2 = iz * iz;
    const double xr = P[0] - p.base;
    const double pu = ((p.fx * P[0]) * iz) + p.cu;
    const double pv = ((p.fy * P[1]) * iz) + p.cv;
    const double pr = ((p.fx * xr) * iz) + p.cu;
    e[0] = o.uL - pu;
    e[1] = o.vL - pv;
    e[2] = o.uR - pr;
    e[3] = o.vR - pv;
    const double g[4][3] = {{p.fx * iz, 0.0, -(p.fx * P[0]) * iz2},
                            {0.0, p.fy * iz, -(p.fy * P[1]) * iz2},
                            {p.fx * iz, 0.0, -(p.fx * xr) * iz2},
                            {0.0, p.fy * iz, -(p.fy * P[1]) * iz2}};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const double gx = g[r][0], gy = g[r][1], gz = g[r][2];
        J[r][0] = gz * P[1] - gy * P[2];
        J[r][1] = gx * P[2] - gz * P[0];
        J[r][2] = gy * P[0] - gx * P[1];
        J[r][3] = gx;
        J[r][4] = gy;
        J[r][5] = gz;
    }
}

// rig: residuals from P; gradients taken to the rig frame (g' = Re^T g), J = [Q x g', g']
__device__ inline void residual_rows_rig(const double* P, const double* Q, const Obs& o, const SvoDev& p,
                                         double* e, double (*J)[6]) {
    const double iz = 1.0 / P[2];
    const double iz2 = iz * iz;
    const double xr = P[0] - p.base;
    const double pu = ((p.fx * P[0]) * iz) + p.cu;
    const double pv = ((p.fy * P[1]) * iz) + p.cv;
    const double pr = ((p.fx * xr) * iz) + p.cu;
    e[0] = o.uL - pu;
    e[1] = o.vL - pv;
    e[2] = o.uR - pr;
    e[3] = o.vR - pv;
    const double g[4][3] = {{p.fx * iz, 0.0, -(p.fx * P[0]) * iz2},
                            {0.0, p.fy * iz, -(p.fy * P[1]) * iz2},
                            {p.fx * iz, 0.0, -(p.fx * xr) * iz2},
                            {0.0, p.fy * iz, -(p.fy * P[1]) * iz2}};
    const double* E = o.E;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const double gx = (E[0] * g[r][0] + E[3] * g[r][1]) + E[6] * g[r][2];
        const double gy = (E[1] * g[r][0] + E[4] * g[r][1]) + E[7] * g[r][2];
        const double gz = (E[2] * g[r][0] + E[5] * g[r][1]) + E[8] * g[r][2];
        J[r][0] = gz * Q[1] - gy * Q[2];
        J[r][1] = gx * Q[2] - gz * Q[0];
        J[r][2] = gy * Q[0] - gx * Q[1];
        J[r][3] = gx;
        J[r][4] = gy;
        J[r][5] = gz;
    }
}

__device__ inline void match_sums(const double* e, const double (*J)[6], double* s) {
    int k = 0;
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int b = a; b < 6; ++b, ++k)
            s[k] = ((J[0][a] * J[0][b] + J[1][a] * J[1][b]) + J[2][a] * J[2][b]) + J[3][a] * J[3][b];
#pragma unroll
    for (int a = 0; a < 6; ++a, ++k) s[k] = ((J[0][a] * e[0] + J[1][a] * e[1]) + J[2][a] * e[2]) + J[3][a] * e[3];
    s[27] = ((e[0] * e[0] + e[1] * e[1]) + e[2] * e[2]) + e[3] * e[3];
}

// the 28 sums of match o under (R, t); zeros if !sel
__device__ inline void match_leaf(const double* R, const double* t, const Obs& o, const SvoDev& p,
                                  bool sel, double* s) {
    if (!sel) {
#pragma unroll
        for (int k = 0; k < 28; ++k) s[k] = 0.0;
        return;
    }
    double P[3], e[4], J[4][6];
    if (o.E) {
        double Q[3];
        rig_point(R, t, o, Q, P);
        residual_rows_rig(P, Q, o, p, e, J);
    } else {
        transform(R, t, o, P);
        residual_rows(P, o, p, e, J);
    }
    match_sums(e, J, s);
}

// A x = g by LDL^T, no pivoting (oracle_svo.cpp solve6: same operations,
// same order); fully unrolled, register-resident.
__device__ inline bool solve6(const double* S, double* x) {
    double A[6][6], g[6], L[6][6], D[6], inv[6];
    {
        int k = 0;
#pragma unroll
        for (int a = 0; a < 6; ++a)
#pragma unroll
            for (int b = a; b < 6; ++b, ++k) A[a][b] = A[b][a] = S[k];
    }
#pragma unroll
    for (int a = 0; a < 6; ++a) g[a] = S[21 + a];
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        double d = A[j][j];
#pragma unroll
        for (int q = 0; q < j; ++q) d = d - (L[j][q] * L[j][q]) * D[q];
        ok = ok && d > 1e-12;
        D[j] = d;
        inv[j] = 1.0 / d;
#pragma unroll
        for (int i = j + 1; i < 6; ++i) {
            double s = A[i][j];
#pragma unroll
            for (int q = 0; q < j; ++q) s = s - (L[i][q] * L[j][q]) * D[q];
            L[i][j] = s * inv[j];
        }
    }
    if (!ok) return false;
    double z[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        double s = g[i];
#pragma unroll
        for (int q = 0; q < i; ++q) s = s - L[i][q] * z[q];
        z[i] = s;
    }
#pragma unroll
    for (int i = 5; i >= 0; --i) {
        double s = z[i] * inv[i];
#pragma unroll
        for (int q = i + 1; q < 6; ++q) s = s - L[q][i] * x[q];
        x[i] = s;
    }
    return true;
}

__device__ inline void mat3_mul_s(const double* A, const double* B, double* C) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            C[3 * i + j] = (A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j]) + A[3 * i + 2] * B[6 + j];
}

__device__ inline void apply_update(const double* x, double* R, double* t) {
    const double w2 = (x[0] * x[0] + x[1] * x[1]) + x[2] * x[2];
    const double c = 1.0 / (1.0 + 0.25 * w2);
    const double W[9] = {0.0, -x[2], x[1], x[2], 0.0, -x[0], -x[1], x[0], 0.0};
    double W2[9], Q[9], Rn[9], tn[3];
    mat3_mul_s(W, W, W2);
    for (int i = 0; i < 9; ++i) Q[i] = ((i % 4 == 0) ? 1.0 : 0.0) + c * (W[i] + 0.5 * W2[i]);
    mat3_mul_s(Q, R, Rn);
    for (int i = 0; i < 3; ++i) tn[i] = ((Q[3 * i] * t[0] + Q[3 * i + 1] * t[1]) + Q[3 * i + 2] * t[2]) + x[3 + i];
    for (int i = 0; i < 9; ++i) R[i] = Rn[i];
    for (int i = 0; i < 3; ++i) t[i] = tn[i];
}

// the residuals of residual_rows alone (same expressions)
__device__ inline void residuals(const double* P, const Obs& o, const SvoDev& p, double* e) {
    const double iz = 1.0 / P[2];
    const double xr = P[0] - p.base;
    const double pu = ((p.fx * P[0]) * iz) + p.cu;
    const double pv = ((p.fy * P[1]) * iz) + p.cv;
    const double pr = ((p.fx * xr) * iz) + p.cu;
    e[0] = o.uL - pu;
    e[1] = o.vL - pv;
    e[2] = o.uR - pr;
    e[3] = o.vR - pv;
}

__device__ inline bool is_inlier(const double* R, const double* t, const Obs& o, const SvoDev& p) {
    double P[3], e[4];
    if (o.E) {
        double Q[3];
        rig_point(R, t, o, Q, P);
    } else {
        transform(R, t, o, P);
    }
    if (!(P[2] > 0.0)) return false;
    residuals(P, o, p, e);
    const double d2 = ((e[0] * e[0] + e[1] * e[1]) + e[2] * e[2]) + e[3] * e[3];
    return d2 < p.th2;
}

__device__ inline double shfl_xor_f64(double v, int m) {
    const long long b = __double_as_longlong(v);
    const int lo = __shfl_xor((int)(b & 0xffffffffLL), m, 64);
    const int hi = __shfl_xor((int)(b >> 32), m, 64);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// canonical pairwise tree over aligned groups of 2^levels lanes (every lane
// of a group ends with the group's sum): the levels of wave_tree_sum_dpp
__device__ inline double lane_tree(double v, int levels) {
    if (levels >= 1) v = v + dpp_f64<0xB1>(v);   // xor 1
    if (levels >= 2) v = v + dpp_f64<0x4E>(v);   // xor 2
    if (levels >= 3) v = v + dpp_f64<0x141>(v);  // xor 4 (uniform quads)
    if (levels >= 4) v = v + dpp_f64<0x140>(v);  // xor 8 (uniform octets)
    if (levels >= 5) {
        double a, b;
        permlane16_swap_f64(v, v, a, b);
        v = a + b;
    }
    if (levels >= 6) {
        double a, b;
        permlane32_swap_f64(v, v, a, b);
        v = a + b;
    }
    return v;
}

// ---------------------------------------------------------------- selection
// ---- selection: bucketing (wave per bucket) and compaction
constexpr int kMaxBuckets = 4096;

// Bucketing: wave per bucket.  The bucket's candidates are the current-left
// features of its band of rows (a contiguous index range, features being
// row-major); lanes test 64 at a time (circular match present, column in the
// bucket), a ballot ranks them in index order, the first bucket_max are kept.
__global__ __launch_bounds__(256) void svo_bucket_kernel(SvoDev p, PairArgs pa, int b0) {
    const int q = b0 * pa.ncam + blockIdx.y;  // (timestep, camera) slot
    const int pb = q / pa.ncam, cam = q - pb * pa.ncam;
    const FeatDev L2 = set_frame(pa, pa.frame0 + pb, cam, 0);
    const int4* __restrict__ rec8 = pa.rec8 + (size_t)q * 2 * pa.cap;
    uint8_t* __restrict__ keep = pa.keep + (size_t)q * pa.cap;
    const int lane = threadIdx.x & 63;
    const int nbx = (p.w + p.bw - 1) / p.bw, nby = (p.h + p.bh - 1) / p.bh;
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= nbx * nby) return;
    const int br = b / nbx, bc = b - br * nbx;
    const int i0 = L2.row0[br * p.bh], i1 = L2.row0[min((br + 1) * p.bh, p.h)];
    int kept = 0;
    for (int j0 = i0; j0 < i1 && kept < p.bmax; j0 += 64) {
        const int j = j0 + lane;
        bool mem = false;
        if (j < i1) {
            const int4 a = rec8[2 * (size_t)j];
            mem = a.x >= 0 && L2.u[j] / p.bw == bc;
        }
        const unsigned long long bal = __ballot(mem);
        const int rank = kept + __popcll(bal & ((1ull << lane) - 1ull));
        if (mem && rank < p.bmax) keep[j] = 1;
        kept += __popcll(bal);
    }
}

// Compaction of the kept matches of timestep b0 + blockIdx.x, camera by
// camera, each in left order -> uv8 (+ the camera of each match in mcam);
// stats[2] = circular matches, stats[3] = bucketed (all cameras).
__global__ __launch_bounds__(1024) void svo_select_kernel(SvoDev p, PairArgs pa, int b0) {
    const int pb = b0 + blockIdx.x;
    int* __restrict__ uv8 = pa.uv8 + (size_t)pb * pa.mcap * 8;
    uint8_t* __restrict__ mcam = pa.mcam + (size_t)pb * pa.mcap;
    int* __restrict__ n_sel = pa.n_sel + pb;
    int* __restrict__ stats = pa.stats + (size_t)pb * 8;
    __shared__ int s_w[16];
    const int tid = threadIdx.x;
    int base = 0, m_all = 0;
    for (int cam = 0; cam < pa.ncam; ++cam) {
        const size_t q = (size_t)pb * pa.ncam + cam;
        const FeatDev L2 = set_frame(pa, pa.frame0 + pb, cam, 0);
        const int4* __restrict__ rec8 = pa.rec8 + q * 2 * pa.cap;
        const uint8_t* __restrict__ keep = pa.keep + q * pa.cap;
        const int n2 = *L2.n;
        for (int c0 = 0; c0 < n2; c0 += 1024) {
            const int i2 = c0 + tid;
            int4 a = make_int4(-1, 0, 0, 0), bq = make_int4(0, 0, 0, 0);
            int k = 0;
            if (i2 < n2) {
                a = rec8[2 * (size_t)i2];
                bq = rec8[2 * (size_t)i2 + 1];
                k = keep[i2];
            }
            const int f = a.x >= 0 ? 1 : 0;
            int tot, totf;
            block_excl_scan(f, s_w, totf);
            const int o = block_excl_scan(k, s_w, tot);
            if (k) {
                int4* r = reinterpret_cast<int4*>(uv8 + 8 * (size_t)(base + o));
                r[0] = a;
                r[1] = bq;
                mcam[base + o] = (uint8_t)cam;
            }
            base += tot;
            m_all += totf;
        }
    }
    if (tid == 0) {
        *n_sel = base;
        stats[2] = m_all;
        stats[3] = base;
    }
}

// ---------------------------------------------------------------- RANSAC
__device__ inline bool sample3(uint64_t seed, int h, int M, int* idx) {
    int got = 0;
    for (int k = 0; k < 16 && got < 3; ++k) {
        const int r = (int)(mix64(seed + (uint64_t)h * 16u + (uint64_t)k) % (uint64_t)M);
        bool dup = false;
        for (int j = 0; j < got; ++j) dup = dup || idx[j] == r;
        if (!dup) idx[got++] = r;
    }
    return got == 3;
}

// Obs of every selected match of timestep b0 + blockIdx.y (thread per match)
__global__ __launch_bounds__(256) void svo_obs_kernel(SvoDev p, PairArgs pa, int b0) {
    const int pb = b0 + blockIdx.y;
    const int M = pa.n_sel[pb];
    const int* __restrict__ uv8 = pa.uv8 + (size_t)pb * pa.mcap * 8;
    const uint8_t* __restrict__ mcam = pa.mcam + (size_t)pb * pa.mcap;
    double* __restrict__ O = pa.obs + (size_t)pb * pa.mcap * kObs;
    for (int m = blockIdx.x * 256 + threadIdx.x; m < M; m += gridDim.x * 256)
        obs_store(O + (size_t)m * kObs, obs_at(uv8, mcam, m, pa, p), pa.ncam > 1 ? (int)mcam[m] : 0);
}

// Thread per hypothesis: its 3-match sample, Gauss-Newton from the identity
// (sums over the sample as the 3-leaf canonical tree (s0 + s1) + (s2 + 0)),
// models[h] = R(9) t(3) (identity if the sample or a solve failed), hok[h].
__global__ __launch_bounds__(64) void svo_hyp_kernel(SvoDev p, PairArgs pa, int b0) {
    const int pb = b0 + blockIdx.y;
    const int hyp = blockIdx.x * 64 + threadIdx.x;
    if (hyp >= p.iters) return;
    const int M = pa.n_sel[pb];
    const double* __restrict__ O = pa.obs + (size_t)pb * pa.mcap * kObs;
    double* __restrict__ model = pa.models + ((size_t)pb * p.iters + hyp) * 12;
    double R[9] = {1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0}, t[3] = {0.0, 0.0, 0.0};
    int idx[3];
    bool ok = M >= 6 && sample3(mix64(p.seed ^ (uint64_t)(pa.frame0 + pb)), hyp, M, idx);
    if (ok) {
        const Obs o0 = obs_load(O + (size_t)idx[0] * kObs, pa), o1 = obs_load(O + (size_t)idx[1] * kObs, pa),
                  o2 = obs_load(O + (size_t)idx[2] * kObs, pa);
        for (int it = 0; it < p.gn_iters; ++it) {
            double S[28], l[28], x[6];
            match_leaf(R, t, o0, p, true, S);
            match_leaf(R, t, o1, p, true, l);
#pragma unroll
            for (int k = 0; k < 28; ++k) S[k] = S[k] + l[k];
            match_leaf(R, t, o2, p, true, l);
#pragma unroll
            for (int k = 0; k < 28; ++k) S[k] = S[k] + (l[k] + 0.0);
            if (!solve6(S, x)) {
                ok = false;
                break;
            }
            apply_update(x, R, t);
            double mx = 0.0;
            for (int k = 0; k < 6; ++k) mx = fmax(mx, fabs(x[k]));
            if (mx < p.eps) break;
        }
    }
    for (int i = 0; i < 12; ++i) model[i] = ok ? (i < 9 ? R[i] : t[i - 9]) : ((i % 4 == 0 && i < 9) ? 1.0 : 0.0);
    pa.hok[(size_t)pb * p.iters + hyp] = ok ? 1 : 0;
}

// Inlier counts: a workgroup scores kHypBlock hypotheses of one timestep
// against all its matches (each match's Obs loaded once for all of them),
// ballot + popcount per wave, wave totals summed in LDS.
constexpr int kHypBlock = 8;

__global__ __launch_bounds__(256) void svo_count_kernel(SvoDev p, PairArgs pa, int b0) {
    const int pb = b0 + blockIdx.y;
    const int h0 = blockIdx.x * kHypBlock;
    const int M = pa.n_sel[pb];
    const double* __restrict__ O = pa.obs + (size_t)pb * pa.mcap * kObs;
    __shared__ double s_mod[kHypBlock][12];
    __shared__ int s_ok[kHypBlock];
    __shared__ int s_cnt[4][kHypBlock];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < kHypBlock * 12) {
        const int hh = tid / 12, i = tid - hh * 12;
        s_mod[hh][i] = h0 + hh < p.iters ? pa.models[((size_t)pb * p.iters + h0 + hh) * 12 + i] : 0.0;
    }
    if (tid < kHypBlock) s_ok[tid] = h0 + tid < p.iters ? pa.hok[(size_t)pb * p.iters + h0 + tid] : 0;
    __syncthreads();
    int cnt[kHypBlock];
#pragma unroll
    for (int hh = 0; hh < kHypBlock; ++hh) cnt[hh] = 0;
    for (int m0 = 0; m0 < M; m0 += 256) {
        const int m = m0 + tid;
        Obs o;
        if (m < M) o = obs_load(O + (size_t)m * kObs, pa);
#pragma unroll
        for (int hh = 0; hh < kHypBlock; ++hh) {
            if (!s_ok[hh]) continue;
            const bool in = m < M && is_inlier(s_mod[hh], s_mod[hh] + 9, o, p);
            cnt[hh] += __popcll(__ballot(in));
        }
    }
    if (lane == 0)
#pragma unroll
        for (int hh = 0; hh < kHypBlock; ++hh) s_cnt[wave][hh] = cnt[hh];
    __syncthreads();
    if (tid < kHypBlock && h0 + tid < p.iters)
        pa.counts[(size_t)pb * p.iters + h0 + tid] = (s_cnt[0][tid] + s_cnt[1][tid]) + (s_cnt[2][tid] + s_cnt[3][tid]);
}

// ---------------------------------------------------------------- refine
// One workgroup: best hypothesis (max count, lowest index), Gauss-Newton over
// its inliers (sums: canonical tree over all M leaves, unselected = 0), final
// inlier flags, motion, pose update T_wc <- T_wc * Tr^-1, stats.
constexpr int kMaxChunks = 128;  // 64-leaf chunks: M <= 8192 (bucket count x bucket_max)

constexpr int kRefineThreads = 256;  // 4 waves: up to 256 VGPRs per lane (fp64 leaves + 28 sums)

__global__ __launch_bounds__(kRefineThreads) void svo_refine_kernel(SvoDev p, PairArgs pa, int b0) {
    const int pb = b0 + blockIdx.x;
    const double* __restrict__ O = pa.obs + (size_t)pb * pa.mcap * kObs;
    const int* __restrict__ n_sel = pa.n_sel + pb;
    const int* __restrict__ counts = pa.counts + (size_t)pb * p.iters;
    const double* __restrict__ models = pa.models + (size_t)pb * p.iters * 12;
    uint8_t* __restrict__ sel = pa.sel + (size_t)pb * pa.mcap;
    uint8_t* __restrict__ inl = pa.inl + (size_t)pb * pa.mcap;
    double* __restrict__ motion = pa.motion + (size_t)pb * 12;
    int* __restrict__ stats = pa.stats + (size_t)pb * 8;
    __shared__ double s_chunk[kMaxChunks][28];
    __shared__ double s_st[12];
    __shared__ int s_best, s_ok, s_conv, s_cnt;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int M = *n_sel;
    if (wave == 0) {
        // argmax (max count, lowest hypothesis) as a wave min of
        // (-count, h) packed into 64 bits
        unsigned long long key = ~0ull;
        for (int h = lane; h < p.iters; h += 64)
            key = min(key, ((unsigned long long)(0x7fffffff - counts[h]) << 32) | (unsigned)h);
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned long long t = ((unsigned long long)(unsigned)__shfl_xor((int)(key >> 32), o, 64) << 32) |
                                         (unsigned)__shfl_xor((int)(key & 0xffffffffu), o, 64);
            key = min(key, t);
        }
        if (lane == 0) {
            const int bc = 0x7fffffff - (int)(key >> 32), bh = (int)(key & 0xffffffffu);
            s_best = (M >= 6 && bc >= 6) ? bh : -1;
            s_ok = s_best >= 0 ? 1 : 0;
            s_cnt = 0;
        }
    }
    __syncthreads();
    const int best = s_best;
    if (tid < 12) s_st[tid] = best >= 0 ? models[(size_t)best * 12 + tid] : ((tid % 4 == 0 && tid < 9) ? 1.0 : 0.0);
    __syncthreads();
    if (best >= 0) {
        double R[9], t[3];
        for (int i = 0; i < 9; ++i) R[i] = s_st[i];
        for (int i = 0; i < 3; ++i) t[i] = s_st[9 + i];
        for (int m = tid; m < M; m += kRefineThreads)
            sel[m] = is_inlier(R, t, obs_load(O + (size_t)m * kObs, pa), p) ? 1 : 0;
        __syncthreads();
        int P2 = 1;
        while (P2 < M) P2 <<= 1;
        const int nch = (P2 + 63) / 64;               // chunks of 64 leaves (P2 >= 64) or 1
        const int lv_in = P2 >= 64 ? 6 : __builtin_ctz(P2);
        int lv_out = 0;
        while ((1 << lv_out) < nch) ++lv_out;
        for (int it = 0; it < p.gn_iters; ++it) {
            for (int i = 0; i < 9; ++i) R[i] = s_st[i];
            for (int i = 0; i < 3; ++i) t[i] = s_st[9 + i];
            for (int ch = wave; ch < nch; ch += kRefineThreads / 64) {
                const int m = ch * 64 + lane;
                double s[28];
                if (m < M) match_leaf(R, t, obs_load(O + (size_t)m * kObs, pa), p, sel[m] != 0, s);
                else
                    for (int k = 0; k < 28; ++k) s[k] = 0.0;
                if (lv_in == 6) {
                    int vi;
                    const double r = reduce_scatter_28(s, &vi);
                    if (vi >= 0 && lane < 32) s_chunk[ch][vi] = r;
                } else {
#pragma unroll
                    for (int k = 0; k < 28; ++k) {
                        const double r = lane_tree(s[k], lv_in);
                        if (lane == 0) s_chunk[ch][k] = r;
                    }
                }
            }
            __syncthreads();
            if (wave == 0) {
                // pairwise tree over the chunk sums (padded to 2^lv_out with zeros)
                double S[28];
#pragma unroll
                for (int k = 0; k < 28; ++k) {
                    // nch is a power of two; more than 64 chunks (128): each lane
                    // first sums its aligned pair of chunks, then the 64 pair sums
                    const double v = lv_out <= 6 ? (lane < nch ? s_chunk[lane][k] : 0.0)
                                                 : s_chunk[2 * lane][k] + s_chunk[2 * lane + 1][k];
                    S[k] = lane_tree(v, lv_out <= 6 ? lv_out : 6);
                }
                if (lane == 0) {
                    double x[6];
                    if (!solve6(S, x)) {
                        s_ok = 0;
                        s_conv = 1;
                    } else {
                        apply_update(x, R, t);
                        for (int i = 0; i < 9; ++i) s_st[i] = R[i];
                        for (int i = 0; i < 3; ++i) s_st[9 + i] = t[i];
                        double mx = 0.0;
                        for (int k = 0; k < 6; ++k) mx = fmax(mx, fabs(x[k]));
                        s_conv = mx < p.eps ? 1 : 0;
                    }
                }
            }
            __syncthreads();
            if (s_conv) break;
            __syncthreads();
        }
        if (!s_ok && tid < 12) s_st[tid] = models[(size_t)best * 12 + tid];  // keep the hypothesis
        __syncthreads();
        for (int i = 0; i < 9; ++i) R[i] = s_st[i];
        for (int i = 0; i < 3; ++i) t[i] = s_st[9 + i];
        int c = 0;
        for (int m = tid; m < M; m += kRefineThreads) {
            const bool in = is_inlier(R, t, obs_load(O + (size_t)m * kObs, pa), p);
            inl[m] = in ? 1 : 0;
            c += in ? 1 : 0;
        }
        atomicAdd(&s_cnt, c);
        __syncthreads();
    } else {
        for (int m = tid; m < M; m += kRefineThreads) inl[m] = 0;
    }
    __syncthreads();
    if (tid == 0) {
        const bool ok = best >= 0 && s_cnt >= 6;
        double T[12];
        for (int i = 0; i < 12; ++i) T[i] = ok ? s_st[i] : ((i % 4 == 0 && i < 9) ? 1.0 : 0.0);
        for (int i = 0; i < 12; ++i) motion[i] = T[i];
        stats[4] = ok ? s_cnt : 0;
        stats[5] = ok ? 1 : 0;
    }
}

// Tail of a batch (one wave): feature counts, each pair's Tr^-1 = [R^T,
// -R^T t] lane-parallel, then the camera poses T_wc <- T_wc * Tr^-1 composed
// in pair order by lane 0 and written back lane-parallel.
constexpr int kPoseThreads = 128;  // >= timesteps per batch

__global__ __launch_bounds__(kPoseThreads) void svo_pose_kernel(PairArgs pa, int nb, double* __restrict__ pose,
                                                      double* __restrict__ pose_log, long long max_poses) {
    __shared__ double s_inv[kPoseThreads][12];
    __shared__ double s_pose[kPoseThreads][12];
    __shared__ int s_ok[kPoseThreads];
    const int b = threadIdx.x;
    if (b < nb) {
        const long long fr = pa.frame0 + b;
        int* st = pa.stats + (size_t)b * 8;
        int nl = 0, nr = 0;
        for (int cam = 0; cam < pa.ncam; ++cam) {
            nl += *set_frame(pa, fr, cam, 0).n;
            nr += *set_frame(pa, fr, cam, 1).n;
        }
        st[0] = nl;
        st[1] = nr;
        int ok = 0;
        if (fr == 0) {
            for (int i = 2; i < 8; ++i) st[i] = 0;
            ok = -1;  // pose := identity
        } else if (st[5]) {
            const double* T = pa.motion + (size_t)b * 12;
            double Ri[9];
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) Ri[3 * i + j] = T[3 * j + i];
            for (int i = 0; i < 9; ++i) s_inv[b][i] = Ri[i];
            for (int i = 0; i < 3; ++i)
                s_inv[b][9 + i] = -((Ri[3 * i] * T[9] + Ri[3 * i + 1] * T[10]) + Ri[3 * i + 2] * T[11]);
            ok = 1;
        }
        s_ok[b] = ok;
    }
    __syncthreads();
    if (b == 0) {
        double P[12];
        for (int i = 0; i < 12; ++i) P[i] = pose[i];
        for (int k = 0; k < nb; ++k) {
            if (s_ok[k] < 0) {
                for (int i = 0; i < 12; ++i) P[i] = (i % 4 == 0 && i < 9) ? 1.0 : 0.0;
            } else if (s_ok[k] > 0) {
                const double* Ri = s_inv[k];
                const double* ti = s_inv[k] + 9;
                double Rn[9], tn[3];
                mat3_mul_s(P, Ri, Rn);
                for (int i = 0; i < 3; ++i) tn[i] = ((P[3 * i] * ti[0] + P[3 * i + 1] * ti[1]) + P[3 * i + 2] * ti[2]) + P[9 + i];
                for (int i = 0; i < 9; ++i) P[i] = Rn[i];
                for (int i = 0; i < 3; ++i) P[9 + i] = tn[i];
            }
            for (int i = 0; i < 12; ++i) s_pose[k][i] = P[i];
        }
        for (int i = 0; i < 12; ++i) pose[i] = P[i];
    }
    __syncthreads();
    for (int q = b; q < nb * 12; q += kPoseThreads) {
        const int k = q / 12, i = q - k * 12;
        const long long fr = pa.frame0 + k;
        if (fr < max_poses) pose_log[12 * fr + i] = s_pose[k][i];
        else if (k == nb - 1) pose_log[12 * (max_poses - 1) + i] = s_pose[k][i];
    }
}

// RANSAC + refinement of timesteps b0 .. b0 + np - 1 (selection in pa)
void launch_ransac(const SvoDev& d, const PairArgs& pa, int b0, int np, hipStream_t st) {
    svo_obs_kernel<<<dim3((pa.mcap + 255) / 256, np), 256, 0, st>>>(d, pa, b0);
    svo_hyp_kernel<<<dim3((d.iters + 63) / 64, np), 64, 0, st>>>(d, pa, b0);
    svo_count_kernel<<<dim3((d.iters + kHypBlock - 1) / kHypBlock, np), 256, 0, st>>>(d, pa, b0);
    svo_refine_kernel<<<np, kRefineThreads, 0, st>>>(d, pa, b0);
}

template <int R>
void launch_detect_r(bool dom, dim3 g, hipStream_t st, const ImgSrc& imgs, const SvoDev& d,
                     const FeatDev* sets, int ring, int pair0, int seg_cap) {
    // g = (tiles_x, tiles_y, images) -> the XCD-dealt 1-D grid
    const int tpi = (int)(g.x * g.y), ni = (int)g.z;
    const dim3 g1(8 * tpi * ((ni + 7) / 8));
    if (dom)
        svo_detect_kernel<R, true><<<g1, kDW, 0, st>>>(imgs, d, sets, ring, pair0, seg_cap, g.x, g.y, ni);
    else
        svo_detect_kernel<R, false><<<g1, kDW, 0, st>>>(imgs, d, sets, ring, pair0, seg_cap, g.x, g.y, ni);
}

void launch_detect(int R, bool dom, dim3 g, hipStream_t st, const ImgSrc& imgs, const SvoDev& d,
                   const FeatDev* sets, int ring, int pair0, int seg_cap) {
    switch (R) {
        case 1: launch_detect_r<1>(dom, g, st, imgs, d, sets, ring, pair0, seg_cap); break;
        case 2: launch_detect_r<2>(dom, g, st, imgs, d, sets, ring, pair0, seg_cap); break;
        case 3: launch_detect_r<3>(dom, g, st, imgs, d, sets, ring, pair0, seg_cap); break;
        case 4: launch_detect_r<4>(dom, g, st, imgs, d, sets, ring, pair0, seg_cap); break;
        case 5: launch_detect_r<5>(dom, g, st, imgs, d, sets, ring, pair0, seg_cap); break;
        case 6: launch_detect_r<6>(dom, g, st, imgs, d, sets, ring, pair0, seg_cap); break;
        case 7: launch_detect_r<7>(dom, g, st, imgs, d, sets, ring, pair0, seg_cap); break;
        default: launch_detect_r<8>(dom, g, st, imgs, d, sets, ring, pair0, seg_cap); break;
    }
}

}  // namespace
}  // namespace viso

// ====================================================================== context
using namespace viso;

struct viso_svo {
    static constexpr int kMaxPairBatch = 128;  // camera pairs per batch (feature pass + estimation)
    viso::HostStage stage;  // pinned staging of host pairs (viso_svo_rig_process)
    viso_svo_params p{};
    int ncam = 1;           // stereo cameras per timestep (> 1: rig, BASELINE.json configs[4])
    int tb = kMaxPairBatch; // timesteps per batch: kMaxPairBatch / ncam
    int ring = kMaxPairBatch + 1;  // feature-set ring (timesteps): a batch + the previous timestep
    std::vector<double> extr;      // [ncam][12] rig -> camera (rig only)
    int device = 0;
    hipStream_t stream = nullptr;
    int tiles = 0;          // detect tiles per row (256 - 2 nms_n output columns each)
    int seg_cap = 0;        // candidates per (row, tile, wave) segment
    size_t frame = 0;       // timesteps processed; timestep k uses ring slot k % ring
    int last_b = -1;        // batch slot of the last processed timestep
    std::vector<FeatDev> sets;        // [ring][ncam][left, right]
    FeatDev* d_sets = nullptr;
    PairArgs pa{};                    // per-pair estimation buffers of a batch
    std::vector<void*> allocs;
    uint8_t* img = nullptr;           // host-path upload buffer (ncam x (left, right))
    double* pose = nullptr;
    double* pose_log = nullptr;       // [max_poses][12]
    size_t max_poses = 0;
    // HIP-event timing of the batched feature passes while enabled: an event
    // pair per batch, read (and summed) only when timing is queried
    std::vector<hipEvent_t> tev;
    int tev_n = 0;
    int timed_pairs = 0;
    bool timed = false;

    SvoDev dev() const {
        SvoDev d;
        d.w = p.width;
        d.h = p.height;
        d.nms_n = p.nms_n;
        d.tau = p.nms_tau;
        d.margin = p.margin;
        d.disp_max = p.disp_max;
        d.radius = p.match_radius;
        d.bw = p.bucket_width;
        d.bh = p.bucket_height;
        d.bmax = p.bucket_max;
        d.iters = p.ransac_iters;
        d.gn_iters = p.gn_iters;
        d.cap = p.max_features;
        d.ncam = ncam;
        d.sw = 64 - 2 * p.nms_n;
        d.ow = 4 * d.sw;
        d.inv_ow = 1.0f / (float)d.ow;
        d.inv_sw = 1.0f / (float)d.sw;
        d.nband = 4 * ((p.width + d.ow - 1) / d.ow);
        d.fx = p.fx;
        d.fy = p.fy;
        d.cu = p.cu;
        d.cv = p.cv;
        d.base = p.base;
        d.th2 = p.inlier_threshold * p.inlier_threshold;
        d.eps = p.gn_eps;
        d.seed = p.seed;
        return d;
    }
    // device buffers are carved from one zeroed arena (256-byte aligned
    // slices): alloc() records the slice, place() makes the one allocation
    std::vector<std::pair<void**, size_t>> pending;
    template <class T>
    int alloc(T*& ptr, size_t n) {
        ptr = nullptr;
        pending.emplace_back(reinterpret_cast<void**>(&ptr), (n * sizeof(T) + 255) & ~(size_t)255);
        return VISO_OK;
    }
    int place() {
        size_t total = 0;
        for (const auto& q : pending) total += std::max<size_t>(q.second, 256);
        void* base = nullptr;
        VISO_HIP_CHECK(hipMalloc(&base, total));
        allocs.push_back(base);
        VISO_HIP_CHECK(hipMemset(base, 0, total));
        size_t o = 0;
        for (const auto& q : pending) {
            *q.first = static_cast<char*>(base) + o;
            o += std::max<size_t>(q.second, 256);
        }
        pending.clear();
        return VISO_OK;
    }
    int init() {
        const int w = p.width, h = p.height, cap = p.max_features;
        tiles = (w + 4 * (64 - 2 * p.nms_n) - 1) / (4 * (64 - 2 * p.nms_n));
        // strict NMS of radius n: same-class maxima of a row are > n apart, so
        // a wave's 64 columns hold at most ceil(64 / (n + 1)) per class
        seg_cap = 4 * ((64 + p.nms_n) / (p.nms_n + 1));
        tb = kMaxPairBatch / ncam;
        ring = tb + 1;
        sets.assign((size_t)2 * ring * ncam, FeatDev{});
        for (FeatDev& f : sets)
            if (alloc(f.u, cap) || alloc(f.v, cap) || alloc(f.c, cap) || alloc(f.d, (size_t)cap * kDesc) ||
                alloc(f.row0, (size_t)h + 1) || alloc(f.n, 1) || alloc(f.cnt, (size_t)h * tiles * 4) ||
                alloc(f.list, (size_t)h * tiles * 4 * seg_cap) || alloc(f.bidx, cap) || alloc(f.buc, cap) ||
                alloc(f.bd, (size_t)cap * kDesc) || alloc(f.bpos, cap) ||
                alloc(f.brow0, (size_t)4 * nband() * (h + 1)) || alloc(f.bcnt, (size_t)4 * nband() * h))
                return VISO_ERR_HIP;
        const int nbk = ((w + p.bucket_width - 1) / p.bucket_width) * ((h + p.bucket_height - 1) / p.bucket_height);
        const int P = kMaxPairBatch, it = std::max(1, p.ransac_iters);
        pa.ring = ring;
        pa.ncam = ncam;
        pa.cap = cap;
        pa.mcap = ncam * std::min(cap, nbk * p.bucket_max);  // per timestep, all cameras
        max_poses = 65536;
        double* d_extr = nullptr;
        if (alloc(d_sets, sets.size()) || alloc(img, 2 * (size_t)ncam * w * h) ||
            alloc(pa.mcam, (size_t)P * pa.mcap) || alloc(d_extr, (size_t)12 * ncam) ||
            alloc(pa.obs, (size_t)P * pa.mcap * kObs) || alloc(pa.hok, (size_t)P * it) ||
            alloc(pa.circ, (size_t)P * cap) || alloc(pa.rec8, (size_t)P * 2 * cap) || alloc(pa.keep, (size_t)P * cap) ||
            alloc(pa.uv8, (size_t)P * pa.mcap * 8) || alloc(pa.n_sel, P) || alloc(pa.counts, (size_t)P * it) ||
            alloc(pa.models, (size_t)P * it * 12) || alloc(pa.sel, (size_t)P * pa.mcap) ||
            alloc(pa.inl, (size_t)P * pa.mcap) || alloc(pa.motion, (size_t)P * 12) || alloc(pa.stats, (size_t)P * 8) ||
            alloc(pose, 12) || alloc(pose_log, max_poses * 12))
            return VISO_ERR_HIP;
        if (place()) return VISO_ERR_HIP;
        pa.sets = d_sets;
        pa.extr = d_extr;
        if (!extr.empty())
            VISO_HIP_CHECK(hipMemcpy(d_extr, extr.data(), extr.size() * sizeof(double), hipMemcpyHostToDevice));
        VISO_HIP_CHECK(hipMemcpy(d_sets, sets.data(), sets.size() * sizeof(FeatDev), hipMemcpyHostToDevice));
        return VISO_OK;
    }
    void release() {
        stage.release();
        for (void* q : allocs) (void)hipFree(q);
        allocs.clear();
        for (hipEvent_t& e : tev)
            if (e) (void)hipEventDestroy(e);
        tev.clear();
        if (stream) (void)hipStreamDestroy(stream);
        stream = nullptr;
    }
    FeatDev& set_at(size_t pair, int side) { return sets[2 * ((pair % ring) * ncam) + side]; }  // camera 0
    int nband() const { return 4 * tiles; }

    // features of timesteps frame .. frame + nb - 1 (all cameras)
    int detect(const ImgSrc& imgs, int nb) {
        const SvoDev d = dev();
        const int pair0 = (int)(frame % ring);
        const int ni = 2 * nb * ncam;  // images
        const dim3 g(tiles, (p.height + kDTH - 1) / kDTH, ni);
        if (timed) {
            while ((int)tev.size() < 2 * (tev_n + 1)) {
                hipEvent_t e;
                VISO_HIP_CHECK(hipEventCreate(&e));
                tev.push_back(e);
            }
            VISO_HIP_CHECK(hipEventRecord(tev[2 * tev_n], stream));
        }
        // responses outside [2, w-3] x [2, h-3] reach the NMS only if margin < n + 2
        const bool dom = p.margin < p.nms_n + 2;
        launch_detect(p.nms_n, dom, g, stream, imgs, d, d_sets, ring, pair0, seg_cap);
        const int segs = 4 * tiles;
        if ((long long)p.height * segs <= kScanLds)
            svo_scan_lds_kernel<<<ni, 1024, (size_t)(2 * p.height * segs + p.height + 4 * segs) * sizeof(int), stream>>>(
                d, d_sets, ring, pair0, segs, seg_cap);
        else
            svo_scan_kernel<<<ni, 1024, 0, stream>>>(d, d_sets, ring, pair0, segs, seg_cap);
        svo_describe_kernel<<<8 * kDescWg * ((ni + 7) / 8), 256, 0, stream>>>(imgs, d, d_sets, ring, pair0, ni);
        if (timed) {
            VISO_HIP_CHECK(hipEventRecord(tev[2 * tev_n + 1], stream));
            ++tev_n;
            timed_pairs += nb * ncam;
        }
        VISO_HIP_CHECK(hipGetLastError());
        return VISO_OK;
    }
    // motion estimation of batch slots [b0, b0 + np) (pairs frame0 + b): every
    // pair needs only its own and the previous pair's features, so the pairs
    // of a batch run side by side in each launch
    int estimate(long long frame0, int b0, int np) {
        if (np <= 0) return VISO_OK;
        const SvoDev d = dev();
        pa.frame0 = frame0;
        const int nbk = ((p.width + p.bucket_width - 1) / p.bucket_width) *
                        ((p.height + p.bucket_height - 1) / p.bucket_height);
        const int nq = np * ncam;  // (timestep, camera) slots
        const int chunks = std::max(32, 2048 / nq);
        svo_circle_kernel<<<8 * ((nq + 7) / 8) * chunks, 256, 0, stream>>>(d, pa, b0, nq, chunks);
        svo_bucket_kernel<<<dim3((nbk + 3) / 4, nq), 256, 0, stream>>>(d, pa, b0);
        svo_select_kernel<<<np, 1024, 0, stream>>>(d, pa, b0);
        launch_ransac(d, pa, b0, np, stream);
        VISO_HIP_CHECK(hipGetLastError());
        return VISO_OK;
    }
    // a batch of nb <= tb timesteps: features, motions, poses
    int batch(const ImgSrc& imgs, int nb) {
        RoctxRange range("svo:batch");
        int rc = detect(imgs, nb);
        if (rc) return rc;
        const int b0 = frame == 0 ? 1 : 0;
        rc = estimate((long long)frame, b0, nb - b0);
        if (rc) return rc;
        pa.frame0 = (long long)frame;
        svo_pose_kernel<<<1, kPoseThreads, 0, stream>>>(pa, nb, pose, pose_log, (long long)max_poses);
        VISO_HIP_CHECK(hipGetLastError());
        frame += nb;
        last_b = nb - 1;
        return VISO_OK;
    }
};

namespace {
int svo_check(const viso_svo_params* p, int ncam) {
    if (!p || p->width < 32 || p->height < 32 || p->width > 32767 || p->height > 32767 || p->nms_n < 1 ||
        p->nms_n > kMaxNms || p->margin < 8 || p->max_features < 1 || p->max_features > 32768 ||
        p->bucket_width < 1 || p->bucket_height < 1 || p->ransac_iters < 1 || p->gn_iters < 1 ||
        p->disp_max < 0 || p->match_radius < 0 || !(p->base > 0) || !(p->fx > 0) || !(p->fy > 0))
        return VISO_ERR_ARG;
    const int nbx = (p->width + p->bucket_width - 1) / p->bucket_width;
    const int nby = (p->height + p->bucket_height - 1) / p->bucket_height;
    if ((long long)nbx * nby > kMaxBuckets) return VISO_ERR_ARG;
    if ((long long)ncam * nbx * nby * p->bucket_max > 64LL * kMaxChunks) return VISO_ERR_ARG;  // M bound
    // a search window spans at most ceil(width / band width) + 1 <= kMaxQB column bands
    const long long win = std::max((long long)p->disp_max + 1, 2LL * p->match_radius + 1);
    if (win > (long long)(kMaxQB - 1) * (64 - 2 * p->nms_n)) return VISO_ERR_ARG;
    return VISO_OK;
}
}  // namespace

extern "C" {

int viso_svo_default_params(viso_svo_params* p, int32_t width, int32_t height, double fx, double fy,
                            double cu, double cv, double base) {
    if (!p) return VISO_ERR_ARG;
    std::memset(p, 0, sizeof(*p));
    p->width = width;
    p->height = height;
    p->fx = fx;
    p->fy = fy;
    p->cu = cu;
    p->cv = cv;
    p->base = base;
    p->nms_n = 5;
    p->nms_tau = 700;
    p->margin = 8;
    p->disp_max = 255;
    p->match_radius = 96;
    p->bucket_width = 50;
    p->bucket_height = 50;
    p->bucket_max = 4;
    p->ransac_iters = 200;
    p->gn_iters = 20;
    p->inlier_threshold = 2.0;
    p->gn_eps = 1e-6;
    p->seed = 0x5EED5EEDull;
    p->max_features = 16384;
    return VISO_OK;
}

int viso_svo_create(const viso_svo_params* p, int device, viso_svo** out) {
    return viso_svo_rig_create(p, 1, nullptr, device, out);
}

int viso_svo_rig_create(const viso_svo_params* p, int32_t n_cams, const double* extrinsics, int device,
                        viso_svo** out) {
    if (!out) return VISO_ERR_ARG;
    *out = nullptr;
    if (n_cams < 1 || n_cams > VISO_SVO_MAX_CAMS || (n_cams > 1 && !extrinsics) || svo_check(p, n_cams))
        return VISO_ERR_ARG;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return VISO_ERR_NODEVICE;
    VISO_HIP_CHECK(hipSetDevice(device));
    viso_svo* s = new (std::nothrow) viso_svo();
    if (!s) return VISO_ERR_ARG;
    s->p = *p;
    s->device = device;
    s->ncam = n_cams;
    if (n_cams > 1) s->extr.assign(extrinsics, extrinsics + 12 * n_cams);
    if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess || s->init() != VISO_OK) {
        s->release();
        delete s;
        return VISO_ERR_HIP;
    }
    *out = s;
    return VISO_OK;
}

int viso_svo_destroy(viso_svo* s) {
    if (!s) return VISO_ERR_ARG;
    (void)hipSetDevice(s->device);
    (void)hipStreamSynchronize(s->stream);
    s->release();
    delete s;
    return VISO_OK;
}

int viso_svo_synchronize(viso_svo* s) {
    if (!s) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(s->device));
    VISO_HIP_CHECK(hipStreamSynchronize(s->stream));
    return VISO_OK;
}

int viso_svo_rig_process(viso_svo* s, const uint8_t* const* lefts, const uint8_t* const* rights,
                         const int32_t dims[3], int32_t* ok) {
    if (!s || !lefts || !rights || !dims) return VISO_ERR_ARG;
    const int w = dims[0], h = dims[1], stride = dims[2];
    if (w != s->p.width || h != s->p.height || stride < w) return VISO_ERR_ARG;
    for (int c = 0; c < s->ncam; ++c)
        if (!lefts[c] || !rights[c]) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(s->device));
    ImgSrc src{};
    for (int c = 0; c < s->ncam; ++c) {
        uint8_t* dl = s->img + (size_t)(2 * c) * w * h;
        uint8_t* dr = dl + (size_t)w * h;
        // pinned staging (staging.hpp; a pageable hipMemcpy2DAsync measured
        // 3.25 ms per 1242x375 image)
        VISO_HIP_CHECK(s->stage.upload(dl, lefts[c], w, h, stride, s->stream));
        VISO_HIP_CHECK(s->stage.upload(dr, rights[c], w, h, stride, s->stream));
        src.left[c] = dl;
        src.right[c] = dr;
    }
    int rc = s->batch(src, 1);
    if (rc) return rc;
    VISO_HIP_CHECK(hipStreamSynchronize(s->stream));
    if (ok) {
        int st[8];
        VISO_HIP_CHECK(hipMemcpy(st, s->pa.stats + 8 * s->last_b, sizeof(st), hipMemcpyDeviceToHost));
        *ok = st[5];
    }
    return VISO_OK;
}

int viso_svo_process(viso_svo* s, const uint8_t* left, const uint8_t* right, const int32_t dims[3],
                     int32_t* ok) {
    if (!s || s->ncam != 1) return VISO_ERR_ARG;
    return viso_svo_rig_process(s, &left, &right, dims, ok);
}

int viso_svo_rig_process_device(viso_svo* s, const uint8_t* const* lefts, const uint8_t* const* rights, int32_t n,
                                int64_t pair_stride, int32_t stride) {
    if (!s || !lefts || !rights || n < 0 || stride != s->p.width) return VISO_ERR_ARG;
    for (int c = 0; c < s->ncam; ++c)
        if (!lefts[c] || !rights[c]) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(s->device));
    // batches of up to tb timesteps (kMaxPairBatch camera pairs), queued back
    // to back on the stream (image addresses are computed in the kernels: no
    // per-batch host data, no host synchronisation)
    for (int i0 = 0; i0 < n; i0 += s->tb) {
        const int nb = std::min(n - i0, s->tb);
        ImgSrc src{};
        for (int c = 0; c < s->ncam; ++c) {
            src.left[c] = lefts[c] + (long long)i0 * pair_stride;
            src.right[c] = rights[c] + (long long)i0 * pair_stride;
        }
        src.pair_stride = (long long)pair_stride;
        const int rc = s->batch(src, nb);
        if (rc) return rc;
    }
    return VISO_OK;
}

int viso_svo_process_device(viso_svo* s, const uint8_t* left, const uint8_t* right, int32_t n,
                            int64_t pair_stride, int32_t stride) {
    if (!s || s->ncam != 1) return VISO_ERR_ARG;
    return viso_svo_rig_process_device(s, &left, &right, n, pair_stride, stride);
}

int viso_svo_timing(viso_svo* s, int32_t enable, double* feature_pass_ms, int32_t* pairs) {
    if (!s) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(s->device));
    double ms = 0.0;
    if (s->tev_n > 0) {
        VISO_HIP_CHECK(hipStreamSynchronize(s->stream));
        for (int k = 0; k < s->tev_n; ++k) {
            float m = 0.f;
            VISO_HIP_CHECK(hipEventElapsedTime(&m, s->tev[2 * k], s->tev[2 * k + 1]));
            ms += m;
        }
    }
    if (feature_pass_ms) *feature_pass_ms = ms;
    if (pairs) *pairs = s->timed_pairs;
    s->tev_n = 0;
    s->timed_pairs = 0;
    s->timed = enable != 0;
    return VISO_OK;
}

int viso_svo_get_motion(viso_svo* s, double* motion12) {
    if (!s || !motion12) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(s->device));
    VISO_HIP_CHECK(hipStreamSynchronize(s->stream));
    if (s->frame < 2) {
        for (int i = 0; i < 12; ++i) motion12[i] = (i % 4 == 0 && i < 9) ? 1.0 : 0.0;
        return VISO_OK;
    }
    VISO_HIP_CHECK(hipMemcpy(motion12, s->pa.motion + 12 * s->last_b, 12 * sizeof(double), hipMemcpyDeviceToHost));
    return VISO_OK;
}

int viso_svo_get_stats(viso_svo* s, int32_t* stats6) {
    if (!s || !stats6) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(s->device));
    VISO_HIP_CHECK(hipStreamSynchronize(s->stream));
    if (s->last_b < 0) {
        for (int i = 0; i < 6; ++i) stats6[i] = 0;
        return VISO_OK;
    }
    VISO_HIP_CHECK(hipMemcpy(stats6, s->pa.stats + 8 * s->last_b, 6 * sizeof(int32_t), hipMemcpyDeviceToHost));
    return VISO_OK;
}

int viso_svo_get_poses(viso_svo* s, double* poses12, size_t cap, size_t* n) {
    if (!s || !n) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(s->device));
    VISO_HIP_CHECK(hipStreamSynchronize(s->stream));
    const size_t m = std::min(s->frame, s->max_poses);
    *n = m;
    if (poses12 && cap)
        VISO_HIP_CHECK(hipMemcpy(poses12, s->pose_log, std::min(m, cap) * 12 * sizeof(double),
                                 hipMemcpyDeviceToHost));
    return VISO_OK;
}

int viso_svo_get_matches(viso_svo* s, int32_t* uv8, uint8_t* inlier, size_t cap, size_t* n) {
    if (!s || !n) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(s->device));
    VISO_HIP_CHECK(hipStreamSynchronize(s->stream));
    int m = 0;
    const int b = s->last_b;
    if (s->frame >= 2) VISO_HIP_CHECK(hipMemcpy(&m, s->pa.n_sel + b, sizeof(int), hipMemcpyDeviceToHost));
    *n = (size_t)m;
    const size_t k = std::min((size_t)m, cap);
    if (uv8 && k)
        VISO_HIP_CHECK(hipMemcpy(uv8, s->pa.uv8 + (size_t)b * s->pa.mcap * 8, k * 8 * sizeof(int32_t),
                                 hipMemcpyDeviceToHost));
    if (inlier && k)
        VISO_HIP_CHECK(hipMemcpy(inlier, s->pa.inl + (size_t)b * s->pa.mcap, k, hipMemcpyDeviceToHost));
    return VISO_OK;
}

int viso_svo_get_match_cams(viso_svo* s, uint8_t* cams, size_t cap, size_t* n) {
    if (!s || !n) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(s->device));
    VISO_HIP_CHECK(hipStreamSynchronize(s->stream));
    int m = 0;
    const int b = s->last_b;
    if (s->frame >= 2) VISO_HIP_CHECK(hipMemcpy(&m, s->pa.n_sel + b, sizeof(int), hipMemcpyDeviceToHost));
    *n = (size_t)m;
    const size_t k = std::min((size_t)m, cap);
    if (cams && k)
        VISO_HIP_CHECK(hipMemcpy(cams, s->pa.mcam + (size_t)b * s->pa.mcap, k, hipMemcpyDeviceToHost));
    return VISO_OK;
}

int viso_svo_features(viso_svo* s, const uint8_t* img, int32_t width, int32_t height, int32_t* u,
                      int32_t* v, int32_t* cls, uint8_t* desc, int32_t cap, int32_t* n) {
    if (!s || !img || !n || width != s->p.width || height != s->p.height || s->ncam != 1) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(s->device));
    const size_t bytes = (size_t)width * height;
    VISO_HIP_CHECK(hipMemcpyAsync(s->img, img, bytes, hipMemcpyHostToDevice, s->stream));
    ImgSrc src{};
    src.left[0] = src.right[0] = s->img;
    int rc = s->detect(src, 1);  // into the slot of pair `frame` (not advanced)
    if (rc) return rc;
    VISO_HIP_CHECK(hipStreamSynchronize(s->stream));
    const FeatDev F = s->set_at(s->frame, 0);
    int m = 0;
    VISO_HIP_CHECK(hipMemcpy(&m, F.n, sizeof(int), hipMemcpyDeviceToHost));
    *n = m;
    const int k = std::min(m, cap);
    if (k > 0) {
        if (u) VISO_HIP_CHECK(hipMemcpy(u, F.u, k * sizeof(int), hipMemcpyDeviceToHost));
        if (v) VISO_HIP_CHECK(hipMemcpy(v, F.v, k * sizeof(int), hipMemcpyDeviceToHost));
        if (cls) VISO_HIP_CHECK(hipMemcpy(cls, F.c, k * sizeof(int), hipMemcpyDeviceToHost));
        if (desc) VISO_HIP_CHECK(hipMemcpy(desc, F.d, (size_t)k * kDesc, hipMemcpyDeviceToHost));
    }
    return VISO_OK;
}

int viso_svo_match(viso_svo* s, const int32_t* const* u4, const int32_t* const* v4,
                   const int32_t* const* cls4, const uint8_t* const* desc4, const int32_t n4[4],
                   int32_t* quad, int32_t cap, int32_t* n) {
    if (!s || !u4 || !v4 || !cls4 || !desc4 || !n4 || !n || s->ncam != 1) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(s->device));
    const int h = s->p.height;
    // the four sets go to the slots of pairs frame + 1 (previous) and
    // frame + 2 (current): pair `frame`'s slot (the sequence's last pair) is kept
    const size_t p1 = s->frame + 1, p2 = s->frame + 2;
    FeatDev* F4[4] = {&s->set_at(p1, 0), &s->set_at(p1, 1), &s->set_at(p2, 0), &s->set_at(p2, 1)};
    for (int k = 0; k < 4; ++k) {
        const int m = n4[k];
        if (m < 0 || m > s->p.max_features) return VISO_ERR_ARG;
        for (int i = 1; i < m; ++i)
            if (v4[k][i] < v4[k][i - 1]) return VISO_ERR_ARG;  // row-major order required
        FeatDev& F = *F4[k];
        std::vector<int> row0((size_t)h + 1, m);
        for (int i = m - 1; i >= 0; --i) {
            if (v4[k][i] < 0 || v4[k][i] >= h || u4[k][i] < 0 || u4[k][i] >= s->p.width) return VISO_ERR_ARG;
            row0[(size_t)v4[k][i]] = i;
        }
        for (int y = h - 1; y >= 0; --y) row0[(size_t)y] = std::min(row0[(size_t)y], row0[(size_t)y + 1]);
        if (m > 0) {
            VISO_HIP_CHECK(hipMemcpy(F.u, u4[k], m * sizeof(int), hipMemcpyHostToDevice));
            VISO_HIP_CHECK(hipMemcpy(F.v, v4[k], m * sizeof(int), hipMemcpyHostToDevice));
            VISO_HIP_CHECK(hipMemcpy(F.c, cls4[k], m * sizeof(int), hipMemcpyHostToDevice));
            VISO_HIP_CHECK(hipMemcpy(F.d, desc4[k], (size_t)m * kDesc, hipMemcpyHostToDevice));
        }
        VISO_HIP_CHECK(hipMemcpy(F.row0, row0.data(), row0.size() * sizeof(int), hipMemcpyHostToDevice));
        VISO_HIP_CHECK(hipMemcpy(F.n, &m, sizeof(int), hipMemcpyHostToDevice));
    }
    const SvoDev d = s->dev();
    svo_index_kernel<<<4, 1024, 0, s->stream>>>(d, s->d_sets, s->ring, (int)(p1 % s->ring));
    PairArgs pa = s->pa;
    pa.frame0 = (long long)p2;  // slot 0 = pair p2 (previous: p1)
    svo_circle_kernel<<<8 * 1024, 256, 0, s->stream>>>(d, pa, 0, 1, 1024);
    VISO_HIP_CHECK(hipGetLastError());
    VISO_HIP_CHECK(hipStreamSynchronize(s->stream));
    std::vector<int4> res((size_t)std::max(1, n4[2]));
    if (n4[2] > 0)
        VISO_HIP_CHECK(hipMemcpy(res.data(), s->pa.circ, (size_t)n4[2] * sizeof(int4), hipMemcpyDeviceToHost));
    int m = 0;
    for (int i2 = 0; i2 < n4[2]; ++i2)
        if (res[(size_t)i2].x >= 0) {
            if (m < cap && quad) {
                quad[4 * m + 0] = res[(size_t)i2].x;
                quad[4 * m + 1] = res[(size_t)i2].y;
                quad[4 * m + 2] = i2;
                quad[4 * m + 3] = res[(size_t)i2].z;
            }
            ++m;
        }
    *n = m;
    return VISO_OK;
}

int viso_svo_estimate(viso_svo* s, const int32_t* uv8, int32_t n, int64_t frame, double* motion12,
                      uint8_t* inlier, int32_t* n_inliers) {
    if (!s || (!uv8 && n > 0) || n < 0 || n > s->p.max_features || !motion12 || s->ncam != 1) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(s->device));
    if (n > s->pa.mcap) return VISO_ERR_CAPACITY;
    if (n > 0) VISO_HIP_CHECK(hipMemcpy(s->pa.uv8, uv8, (size_t)n * 8 * sizeof(int), hipMemcpyHostToDevice));
    VISO_HIP_CHECK(hipMemcpy(s->pa.n_sel, &n, sizeof(int), hipMemcpyHostToDevice));
    const SvoDev d = s->dev();
    PairArgs pa = s->pa;
    pa.frame0 = frame;  // slot 0: the sampler stream of `frame`
    launch_ransac(d, pa, 0, 1, s->stream);
    VISO_HIP_CHECK(hipGetLastError());
    VISO_HIP_CHECK(hipStreamSynchronize(s->stream));
    VISO_HIP_CHECK(hipMemcpy(motion12, s->pa.motion, 12 * sizeof(double), hipMemcpyDeviceToHost));
    if (inlier && n > 0) VISO_HIP_CHECK(hipMemcpy(inlier, s->pa.inl, n, hipMemcpyDeviceToHost));
    int st[8];
    VISO_HIP_CHECK(hipMemcpy(st, s->pa.stats, sizeof(st), hipMemcpyDeviceToHost));
    if (n_inliers) *n_inliers = st[5] ? st[4] : -1;
    return VISO_OK;
}

}  // extern "C"
