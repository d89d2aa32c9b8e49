// viso_amd — 2D-2D initialisation geometry for gfx950:
// Viso::PoseEstimation2d2d (src/viso.cpp:178-256) with the repo's
// deterministic RANSAC for E and H (stand-ins for cv::findEssentialMat /
// cv::findHomography, see oracle_geom.cpp), cv::recoverPose and
// cv::decomposeHomographyMat restated, then Viso::SelectMotion (:520-638).
//
// Parallel structure:
//  * hypothesis kernels: one lane per RANSAC hypothesis (minimal solver);
//  * scoring kernels: one workgroup per hypothesis, points strided over the
//    256 lanes, inliers counted with __ballot/__popcll per wave;
//  * scan kernel: one lane replays OpenCV's sequential loop
//    (RANSACUpdateNumIters) over the per-hypothesis counts — identical to a
//    sequential RANSAC whose i-th sample is hypothesis i;
//  * select-motion: one lane per (candidate, point) triangulation + tests,
//    one workgroup for the strict-max choice and the mean-depth tree.
#include <cfloat>
#include <climits>

#include "device_math.hpp"
#include "geometry.hpp"
#include "linalg.hpp"

namespace viso {

namespace {

__device__ inline uint64_t sample_hash(uint64_t seed, int h, int t, int k, int a) {
    uint64_t z = seed + 0x632BE59BD9B4E019ULL * (uint64_t)(h + 1) +
                 0x9E3779B97F4A7C15ULL * (uint64_t)(t + 1) +
                 0xD1B54A32D192ED03ULL * (uint64_t)(k * 64 + a + 1);
    return mix64(z);
}

template <int M>
__device__ inline void draw_subset(uint64_t seed, int h, int t, int n, int* idx) {
    for (int k = 0; k < M; ++k) {
        int chosen = -1;
        for (int a = 0; a < 64 && chosen < 0; ++a) {
            const int c = (int)(sample_hash(seed, h, t, k, a) % (uint64_t)n);
            bool dup = false;
            for (int j = 0; j < k; ++j) dup |= (idx[j] == c);
            if (!dup) chosen = c;
        }
        if (chosen < 0) {
            for (int c = 0; c < n && chosen < 0; ++c) {
                bool dup = false;
                for (int j = 0; j < k; ++j) dup |= (idx[j] == c);
                if (!dup) chosen = c;
            }
        }
        idx[k] = chosen;
    }
}

// draw_subset<M> on one wave (every lane gets the same idx): the 64 attempts
// of a sample are hashed by the 64 lanes at once and the first attempt that
// is not a duplicate wins, as in the sequential loop; if all 64 are
// duplicates, the first free index in 0..n-1, as there.
template <int M>
__device__ inline void draw_subset_wave(uint64_t seed, int h, int t, int n, int* idx) {
    const int lane = threadIdx.x & 63;
    for (int k = 0; k < M; ++k) {
        const int cand = (int)(sample_hash(seed, h, t, k, lane) % (uint64_t)n);
        bool dup = false;
        for (int j = 0; j < k; ++j) dup |= (idx[j] == cand);
        unsigned long long ok = __ballot(!dup);
        int chosen = -1;
        if (ok) {
            chosen = __builtin_amdgcn_readlane(cand, __ffsll((long long)ok) - 1);
        } else {
            for (int c0 = 0; c0 < n && chosen < 0; c0 += 64) {
                const int c = c0 + lane;
                bool d2 = c >= n;
                for (int j = 0; j < k; ++j) d2 |= (idx[j] == c);
                ok = __ballot(!d2);
                if (ok) chosen = __builtin_amdgcn_readlane(c, __ffsll((long long)ok) - 1);
            }
        }
        idx[k] = chosen;
    }
}

// the uniform array entry v[i] at a per-lane index i < M (a select chain:
// no scratch)
template <int M>
__device__ inline int pick_uniform(const int* v, int i) {
    int r = v[0];
#pragma unroll
    for (int k = 1; k < M; ++k)
        if (i == k) r = v[k];
    return r;
}

// the control block into a.host_ctl (GeoArgs) by the block's first threads,
// after a barrier that follows the block's last ctl write: system-scope
// stores, visible to the host once the launch has completed
__device__ inline void ctl_mirror(const GeoArgs& a) {
    if (!a.host_ctl) return;
    constexpr int kWords = (int)(sizeof(GeoCtl) / 8);
    const uint64_t* src = reinterpret_cast<const uint64_t*>(a.ctl);
    uint64_t* dst = reinterpret_cast<uint64_t*>(a.host_ctl);
    for (int k = threadIdx.x; k < kWords; k += blockDim.x)
        __hip_atomic_store(dst + k, src[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---------------------------------------------------------------- normalise
// p = K_inv * (x, y, 1) (src/viso.cpp:45-48); q = float-rounded (cv::Point2f,
// :204-205); disparity = canonical tree of |p2 - p1|^2 (:199-211).
// One 1,024-thread workgroup: thread t owns the C = P / 1024 consecutive
// points [t C, t C + C) of the padded count P (C <= 64: max_features <=
// 65536), normalises them, and folds their leaves into its subtree in
// registers (binary-counter stack with compile-time slots); then the wave
// trees and the 16 waves' pairwise top.  The same pairwise tree over the P
// padded leaves as block_tree_sum (+0.0 leaves past n, and past P up to
// 1,024 leaves: adding +0.0 to a sum of squares is exact).
constexpr int kNormThreads = 1024;
constexpr int kNormMaxC = 64;

// With ci.success (launch_compact_gate) the same workgroup first erases the
// failed tracks (src/viso.cpp:23-40, order kept): thread t owns the
// ceil(n / 1024) consecutive tracks [t C, t C + C), counts its survivors, one
// block-wide exclusive scan places them, and each thread copies its own in
// order into ci.out1 / ci.out2 (= a.kp1 / a.kp2); the count goes to
// ci.n_out (= a.n_dev) and, through LDS, to the normalisation below.
// ci.n < 0: the input count is *ci.n_out's value capped at -n (a
// re-detection frame's FAST count the host has not read).
__global__ __launch_bounds__(kNormThreads) void normalize_kernel(GeoArgs a, CompactIn ci) {
    __shared__ double s_w[kNormThreads / 64];
    __shared__ int s_c[kNormThreads / 64];
    __shared__ int s_n;
    if (ci.success) {
        int m = ci.n;
        if (m < 0) m = min(*ci.n_out, -m);
        const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
        const int Cc = (m + kNormThreads - 1) / kNormThreads;
        const int lo = min(t * Cc, m), hi = min(lo + Cc, m);
        int cnt = 0;
        for (int i = lo; i < hi; ++i) cnt += ci.success[i] != 0;
        int incl = cnt;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int o = __shfl_up(incl, d);
            if (lane >= d) incl += o;
        }
        if (lane == 63) s_c[wave] = incl;
        __syncthreads();  // (also: every thread has read *ci.n_out)
        int off = incl - cnt;
        for (int k = 0; k < wave; ++k) off += s_c[k];
        for (int i = lo; i < hi; ++i)
            if (ci.success[i]) {
                ci.out1[off] = ci.in1[i];
                ci.out2[off] = ci.in2[i];
                ++off;
            }
        if (t == kNormThreads - 1) {
            *ci.n_out = off;
            s_n = off;
        }
        __syncthreads();  // the compacted tracks (global, this workgroup's) and their count
    }
    const int n = ci.success ? s_n : *a.n_dev;
    const double* Ki = a.Kinv;
    int P = 1;
    while (P < n) P <<= 1;
    const int C = P > kNormThreads ? P / kNormThreads : 1;
    const int t = threadIdx.x;
    double stack[7];  // log2(kNormMaxC) + 1 slots
#pragma unroll
    for (int j = 0; j < kNormMaxC; ++j) {
        if (j >= C) break;
        const int i = t * C + j;
        double leaf = 0.0;
        if (i < n) {
            double p1[3], p2[3];
            if (a.p1_in) {
                for (int r = 0; r < 3; ++r) {
                    p1[r] = a.p1_in[3 * i + r];
                    p2[r] = a.p2_in[3 * i + r];
                }
            } else {
                const float2 k1 = a.kp1[i], k2 = a.kp2[i];
                const double u1[3] = {(double)k1.x, (double)k1.y, 1};
                const double u2[3] = {(double)k2.x, (double)k2.y, 1};
                for (int r = 0; r < 3; ++r) {
                    p1[r] = Ki[3 * r] * u1[0] + Ki[3 * r + 1] * u1[1] + Ki[3 * r + 2] * u1[2];
                    p2[r] = Ki[3 * r] * u2[0] + Ki[3 * r + 1] * u2[1] + Ki[3 * r + 2] * u2[2];
                }
            }
            for (int r = 0; r < 3; ++r) {
                a.p1[3 * i + r] = p1[r];
                a.p2[3 * i + r] = p2[r];
            }
            a.q1[2 * i] = (double)(float)p1[0];
            a.q1[2 * i + 1] = (double)(float)p1[1];
            a.q2[2 * i] = (double)(float)p2[0];
            a.q2[2 * i + 1] = (double)(float)p2[1];
            const double dx = p2[0] - p1[0];
            const double dy = p2[1] - p1[1];
            leaf = dx * dx + dy * dy;
        }
        // binary counter: leaf j closes the subtrees of its trailing one bits
        int sp = __builtin_popcount(j);
#pragma unroll
        for (int k = j; k & 1; k >>= 1) leaf = stack[--sp] + leaf;
        stack[sp] = leaf;
    }
    double v = wave_tree_sum(stack[0]);
    if ((t & 63) == 0) s_w[t >> 6] = v;
    __syncthreads();
    if (t == 0) {
        double l1[8], l2[4];
        for (int k = 0; k < 8; ++k) l1[k] = s_w[2 * k] + s_w[2 * k + 1];
        for (int k = 0; k < 4; ++k) l2[k] = l1[2 * k] + l1[2 * k + 1];
        double d = (l2[0] + l2[1]) + (l2[2] + l2[3]);
        const double f = (a.K[0] + a.K[1]) / 2;
        if (d != 0) {
            d /= n;
            d *= f * f;
        }
        GeoCtl* c = a.ctl;
        c->n = n;
        c->disparity = d;
        c->gate = (n >= 10 && !(d < a.disparity_thresh)) ? 1 : 0;
        c->n_cand = 0;
        c->e_ncand = c->h_ncand = 0;
        c->e_count = c->h_count = 0;
        c->e_best = c->h_best = -1;
        c->e_iters = c->h_iters = 0;
        c->nr_inliers = 0;
        c->best_motion = -1;
    }
    __syncthreads();
    ctl_mirror(a);
}

// ---------------------------------------------------------------- E RANSAC
__device__ inline bool essential_from_8(const double* q1, const double* q2, const int* idx,
                                        double* E) {
    double A[72];
    for (int r = 0; r < 8; ++r) {
        const double x1 = q1[2 * idx[r]], y1 = q1[2 * idx[r] + 1];
        const double x2 = q2[2 * idx[r]], y2 = q2[2 * idx[r] + 1];
        double* row = A + 9 * r;
        row[0] = x2 * x1;
        row[1] = x2 * y1;
        row[2] = x2;
        row[3] = y2 * x1;
        row[4] = y2 * y1;
        row[5] = y2;
        row[6] = x1;
        row[7] = y1;
        row[8] = 1.0;
    }
    double e[9];
    if (!null_vector_8x9(A, e)) return false;
    double U[9], s[3], V[9];
    svd3(e, U, s, V);
    if (!(s[1] > 0)) return false;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) E[3 * i + j] = U[3 * i + 0] * V[3 * j + 0] + U[3 * i + 1] * V[3 * j + 1];
    return true;
}

__device__ inline float sampson_err(const double* E, double x1, double y1, double x2, double y2) {
    const double ex0 = E[0] * x1 + E[1] * y1 + E[2];
    const double ex1 = E[3] * x1 + E[4] * y1 + E[5];
    const double ex2 = E[6] * x1 + E[7] * y1 + E[8];
    const double et0 = E[0] * x2 + E[3] * y2 + E[6];
    const double et1 = E[1] * x2 + E[4] * y2 + E[7];
    const double x2tEx1 = x2 * ex0 + y2 * ex1 + ex2;
    const double aa = ex0 * ex0, b = ex1 * ex1, c = et0 * et0, d = et1 * et1;
    return (float)(x2tEx1 * x2tEx1 / (aa + b + c + d));
}

// One wave per hypothesis (4 per workgroup, so the 1000 hypotheses spread
// over 250 workgroups): the 8-point subset drawn lane-parallel, lane l
// builds elements l and 64 + l of the 8x9 system, the null vector by the
// wave's complete-pivot elimination (null_vector_8x9_wave: each element sees
// the sequential routine's operations), then svd3 and the (1, 1, 0)
// projection on every lane (uniform), exactly as essential_from_8.
__global__ __launch_bounds__(256) void e_hyp_kernel(GeoArgs a) {
    __shared__ double s_m[4][72];
    const int wave = wave_id(), lane = threadIdx.x & 63;
    const int h = blockIdx.x * 4 + wave;
    if (h >= a.e_iters) return;
    const GeoCtl* c = a.ctl;
    if (!c->gate) return;
    const int n = c->n;
    int idx[8];
    if (n == 8) {
        for (int k = 0; k < 8; ++k) idx[k] = k;
    } else {
        draw_subset_wave<8>(a.seed, h, 0, n, idx);
    }
    auto elem = [&](int i) -> double {
        const int r = i / 9, col = i - 9 * (i / 9);
        const int p = pick_uniform<8>(idx, r);
        const double x1 = a.q1[2 * p], y1 = a.q1[2 * p + 1];
        const double x2 = a.q2[2 * p], y2 = a.q2[2 * p + 1];
        switch (col) {
            case 0: return x2 * x1;
            case 1: return x2 * y1;
            case 2: return x2;
            case 3: return y2 * x1;
            case 4: return y2 * y1;
            case 5: return y2;
            case 6: return x1;
            case 7: return y1;
            default: return 1.0;
        }
    };
    double A[2] = {elem(lane), lane < 8 ? elem(64 + lane) : 0.0};
    double e[9];
    bool ok = null_vector_8x9_wave(A, s_m[wave], e);
    double E[9];
    if (ok) {
        double U[9], sv[3], V[9];
        svd3(e, U, sv, V);
        ok = sv[1] > 0;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) E[3 * i + j] = U[3 * i + 0] * V[3 * j + 0] + U[3 * i + 1] * V[3 * j + 1];
    }
    if (lane == 0) {
        if (ok)
            for (int k = 0; k < 9; ++k) a.e_models[9 * (size_t)h + k] = E[k];
        a.e_valid[h] = ok ? 1 : 0;
    }
}

// ---------------------------------------------------------------- H RANSAC
__device__ inline bool subset_ok_h(const double* p1, const double* p2, const int* idx) {
    const int tt[4][3] = {{0, 1, 2}, {1, 2, 3}, {0, 2, 3}, {0, 1, 3}};
    const float eps = FLT_EPSILON;
    for (int img = 0; img < 2; ++img) {
        const double* p = img == 0 ? p1 : p2;
        for (int q = 0; q < 4; ++q) {
            const int* t = tt[q];
            const double dx1 = p[2 * idx[t[1]]] - p[2 * idx[t[0]]], dy1 = p[2 * idx[t[1]] + 1] - p[2 * idx[t[0]] + 1];
            const double dx2 = p[2 * idx[t[2]]] - p[2 * idx[t[0]]], dy2 = p[2 * idx[t[2]] + 1] - p[2 * idx[t[0]] + 1];
            if (fabs(dx2 * dy1 - dy2 * dx1) <= eps * (fabs(dx1) + fabs(dy1) + fabs(dx2) + fabs(dy2)))
                return false;
        }
    }
    int negative = 0;
    for (int q = 0; q < 4; ++q) {
        const int* t = tt[q];
        double A[9], B[9];
        for (int r = 0; r < 3; ++r) {
            A[3 * r] = p1[2 * idx[t[r]]];
            A[3 * r + 1] = p1[2 * idx[t[r]] + 1];
            A[3 * r + 2] = 1.0;
            B[3 * r] = p2[2 * idx[t[r]]];
            B[3 * r + 1] = p2[2 * idx[t[r]] + 1];
            B[3 * r + 2] = 1.0;
        }
        negative += det3(A) * det3(B) < 0;
    }
    return negative == 0 || negative == 4;
}

__device__ inline void h_rows(double x1, double y1, double x2, double y2, double* ra, double* rb) {
    ra[0] = x1;
    ra[1] = y1;
    ra[2] = 1.0;
    ra[3] = 0.0;
    ra[4] = 0.0;
    ra[5] = 0.0;
    ra[6] = -x2 * x1;
    ra[7] = -x2 * y1;
    ra[8] = -x2;
    rb[0] = 0.0;
    rb[1] = 0.0;
    rb[2] = 0.0;
    rb[3] = x1;
    rb[4] = y1;
    rb[5] = 1.0;
    rb[6] = -y2 * x1;
    rb[7] = -y2 * y1;
    rb[8] = -y2;
}

__device__ inline float transfer_err(const double* H, double x1, double y1, double x2, double y2) {
    const double w = H[6] * x1 + H[7] * y1 + H[8];
    const double px = (H[0] * x1 + H[1] * y1 + H[2]) / w;
    const double py = (H[3] * x1 + H[4] * y1 + H[5]) / w;
    const double dx = px - x2, dy = py - y2;
    return (float)(dx * dx + dy * dy);
}

// One wave per hypothesis: the up to 100 sampling tries of the sequential
// loop run 64 at a time, one per lane (a try's subset depends only on its
// index), the first try whose subset passes checkSubset wins; then the 8x9
// DLT system (two rows per point, h_rows) and the wave's null vector.
__global__ __launch_bounds__(256) void h_hyp_kernel(GeoArgs a) {
    __shared__ double s_m[4][72];
    const int wave = wave_id(), lane = threadIdx.x & 63;
    const int h = blockIdx.x * 4 + wave;
    if (h >= a.h_iters) return;
    const GeoCtl* c = a.ctl;
    if (!c->gate) return;
    const int n = c->n;
    int idx[4] = {0, 1, 2, 3};
    bool ok = false;
    if (n == 4) {
        ok = subset_ok_h(a.q1, a.q2, idx);
    } else {
        for (int t0 = 0; t0 < 100 && !ok; t0 += 64) {
            const int t = t0 + lane;
            int my[4] = {0, 0, 0, 0};
            bool good = false;
            if (t < 100) {
                draw_subset<4>(a.seed ^ 0x4848484848484848ULL, h, t, n, my);
                good = subset_ok_h(a.q1, a.q2, my);
            }
            const unsigned long long b = __ballot(good);
            if (b) {
                const int L = __ffsll((long long)b) - 1;
                for (int k = 0; k < 4; ++k) idx[k] = __builtin_amdgcn_readlane(my[k], L);
                ok = true;
            }
        }
    }
    if (!ok) {
        if (lane == 0) a.h_valid[h] = 0;
        return;
    }
    auto elem = [&](int i) -> double {
        const int r = i / 9, col = i - 9 * (i / 9);
        const int p = pick_uniform<4>(idx, r >> 1);
        const double x1 = a.q1[2 * p], y1 = a.q1[2 * p + 1];
        const double x2 = a.q2[2 * p], y2 = a.q2[2 * p + 1];
        double ra[9], rb[9];
        h_rows(x1, y1, x2, y2, ra, rb);
        double v = 0.0;
#pragma unroll
        for (int k = 0; k < 9; ++k)
            if (col == k) v = (r & 1) ? rb[k] : ra[k];
        return v;
    };
    double A[2] = {elem(lane), lane < 8 ? elem(64 + lane) : 0.0};
    double e[9];
    const bool nv = null_vector_8x9_wave(A, s_m[wave], e);
    if (lane == 0) {
        if (nv)
            for (int k = 0; k < 9; ++k) a.h_models[9 * (size_t)h + k] = e[k];
        a.h_valid[h] = nv ? 1 : 0;
    }
}

// ---------------------------------------------------------------- scoring
template <bool IS_E>
__global__ __launch_bounds__(256) void score_kernel(GeoArgs a) {
    __shared__ int s_cnt;
    const int h = blockIdx.x;
    const GeoCtl* c = a.ctl;
    int* counts = IS_E ? a.e_counts : a.h_counts;
    const uint8_t* valid = IS_E ? a.e_valid : a.h_valid;
    if (!c->gate) return;
    if (!valid[h]) {
        if (threadIdx.x == 0) counts[h] = -1;
        return;
    }
    const double* M = (IS_E ? a.e_models : a.h_models) + 9 * (size_t)h;
    double m[9];
    for (int k = 0; k < 9; ++k) m[k] = M[k];
    const float t2 = a.t2;
    const int n = c->n;
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    int cnt = 0;
    for (int i0 = 0; i0 < n; i0 += 256) {
        const int i = i0 + threadIdx.x;
        bool in = false;
        if (i < n) {
            const double x1 = a.q1[2 * i], y1 = a.q1[2 * i + 1], x2 = a.q2[2 * i], y2 = a.q2[2 * i + 1];
            in = (IS_E ? sampson_err(m, x1, y1, x2, y2) : transfer_err(m, x1, y1, x2, y2)) <= t2;
        }
        cnt += __popcll(__ballot(in));
    }
    if ((threadIdx.x & 63) == 0) atomicAdd(&s_cnt, cnt);
    __syncthreads();
    if (threadIdx.x == 0) counts[h] = s_cnt;
}

// cv::RANSACUpdateNumIters
__device__ inline int update_num_iters(double p, double ep, int modelPoints, int maxIters) {
    p = fmax(p, 0.);
    p = fmin(p, 1.);
    ep = fmax(ep, 0.);
    ep = fmin(ep, 1.);
    double num = fmax(1. - p, DBL_MIN);
    double denom = 1. - pow(1. - ep, (double)modelPoints);
    if (denom < DBL_MIN) return 0;
    num = log(num);
    denom = log(denom);
    return denom >= 0 || -num >= maxIters * (-denom) ? maxIters : (int)rint(num / denom);
}

// OpenCV's sequential RANSAC loop over the precomputed counts, without
// walking them one by one: a hypothesis changes the loop state only where
// its count beats max(modelPoints - 1, every earlier count) (a strict prefix
// maximum, "record"), and the loop's bound niters only shrinks, so the loop
// is the walk over the records in order until one lies at or past niters.
// The counts are scanned in segments of 2048 (8 per thread: a block max-scan
// finds the records, an exclusive sum scan places them in LDS), the
// records' RANSACUpdateNumIters logs are computed lane-parallel, and thread 0
// applies the cheap part of each update in order.  Same state sequence as
// the sequential loop; then the winner's inlier mask (all lanes).
constexpr int kScanSeg = 2048;
constexpr int kScanPer = kScanSeg / 256;

__device__ inline int block_excl_scan_max(int v, int* s_w, int* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(incl, d);
        if (lane >= d) incl = max(incl, o);
    }
    const int excl_w = __shfl_up(incl, 1);
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    int pre = INT_MIN;
    for (int k = 0; k < wave; ++k) pre = max(pre, s_w[k]);
    *total = max(max(s_w[0], s_w[1]), max(s_w[2], s_w[3]));
    __syncthreads();
    return lane == 0 ? pre : max(pre, excl_w);
}

__device__ inline int block_excl_scan_sum(int v, int* s_w, int* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(incl, d);
        if (lane >= d) incl += o;
    }
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    int pre = 0;
    for (int k = 0; k < wave; ++k) pre += s_w[k];
    *total = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    __syncthreads();
    return pre + incl - v;
}

template <bool IS_E>
__global__ __launch_bounds__(256) void scan_kernel(GeoArgs a) {
    __shared__ int s_w[4];
    __shared__ int s_rec[kScanSeg];
    __shared__ double s_ln[kScanSeg];  // log(denom) of each record's update (or +inf: returns 0)
    __shared__ int s_q[kScanSeg];      // rint(num / denom)
    __shared__ int s_state[4];         // niters, best, maxGood, last
    __shared__ int s_done;
    GeoCtl* c = a.ctl;
    if (!c->gate) return;
    const int n = c->n;
    const int modelPoints = IS_E ? 8 : 4;
    const int maxIters = IS_E ? a.e_iters : a.h_iters;
    const int* counts = IS_E ? a.e_counts : a.h_counts;
    const bool enough = n >= modelPoints && (!IS_E || n >= 8);
    const int t = threadIdx.x;
    // log(1 - p), the update's numerator (p = confidence, clamped)
    const double p = fmin(fmax(a.confidence, 0.), 1.);
    const double ln_num = log(fmax(1. - p, DBL_MIN));
    if (t == 0) {
        s_state[0] = maxIters;
        s_state[1] = -1;
        s_state[2] = 0;
        s_state[3] = -1;
        s_done = enough ? 0 : 1;
    }
    __syncthreads();
    int run_base = modelPoints - 1;  // max(modelPoints - 1, counts before the segment)
    for (int seg = 0; seg < maxIters && !s_done; seg += kScanSeg) {
        const int lo = seg + kScanPer * t, hi = min(lo + kScanPer, maxIters);
        int cc[kScanPer], m = INT_MIN;
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) {
            cc[k] = lo + k < hi ? counts[lo + k] : -1;
            m = max(m, cc[k]);
        }
        int seg_max;
        const int pre = max(run_base, block_excl_scan_max(m, s_w, &seg_max));
        int run = pre, nrec = 0;
#pragma unroll
        for (int k = 0; k < kScanPer; ++k)
            if (cc[k] > run) {
                run = cc[k];
                ++nrec;
            }
        int n_total;
        int pos = block_excl_scan_sum(nrec, s_w, &n_total);
        run = pre;
#pragma unroll
        for (int k = 0; k < kScanPer; ++k)
            if (cc[k] > run) {
                run = cc[k];
                // cv::RANSACUpdateNumIters(p, (n - count) / n, modelPoints, .): the
                // part that does not depend on the current niters
                const double ep = fmin(fmax((double)(n - cc[k]) / n, 0.), 1.);
                const double denom = 1. - pow(1. - ep, (double)modelPoints);
                const double ln_den = denom < DBL_MIN ? INFINITY : log(denom);
                s_rec[pos] = lo + k;
                s_ln[pos] = ln_den;
                s_q[pos] = denom < DBL_MIN ? 0 : (int)rint(ln_num / ln_den);
                ++pos;
            }
        __syncthreads();
        if (t == 0) {
            int niters = s_state[0], best = s_state[1], maxGood = s_state[2], last = s_state[3];
            for (int i = 0; i < n_total; ++i) {
                const int h = s_rec[i];
                if (h >= niters) {
                    s_done = 1;
                    break;
                }
                best = h;
                maxGood = counts[h];
                last = h;
                const double ld = s_ln[i];
                if (ld == INFINITY)
                    niters = 0;  // denom < DBL_MIN
                else if (!(ld >= 0 || -ln_num >= niters * (-ld)))
                    niters = s_q[i];
            }
            s_state[0] = niters;
            s_state[1] = best;
            s_state[2] = maxGood;
            s_state[3] = last;
        }
        run_base = max(run_base, seg_max);
        __syncthreads();
    }
    const int best = s_state[1];
    if (t == 0) {
        // the loop variable at exit: the first h >= niters after the last record
        const int h_exit = max(s_state[0], s_state[3] + 1);
        if (IS_E) {
            c->e_count = best >= 0 ? s_state[2] : 0;
            c->e_best = best;
            c->e_iters = enough ? h_exit : 0;
        } else {
            c->h_count = best >= 0 ? s_state[2] : 0;
            c->h_best = best;
            c->h_iters = enough ? h_exit : 0;
        }
    }
    if (best < 0) return;
    const double* M = (IS_E ? a.e_models : a.h_models) + 9 * (size_t)best;
    uint8_t* mask = IS_E ? a.e_mask : a.h_mask;
    for (int i = t; i < n; i += 256) {
        const double x1 = a.q1[2 * i], y1 = a.q1[2 * i + 1], x2 = a.q2[2 * i], y2 = a.q2[2 * i + 1];
        mask[i] = (IS_E ? sampson_err(M, x1, y1, x2, y2) : transfer_err(M, x1, y1, x2, y2)) <= a.t2;
    }
}

// ---------------------------------------------------------------- recoverPose
// cv::recoverPose(E, ...) in three launches: the decomposition (one
// thread), the cheirality test of every point under the four motions (one
// thread per point over the whole grid; integer counts, so the atomic adds
// are order-free and exact), and the pick.
__global__ __launch_bounds__(64) void recover_setup_kernel(GeoArgs a) {
    GeoCtl* c = a.ctl;
    if (!c->gate || c->e_best < 0) return;
    if (threadIdx.x < 4) a.rp_good[threadIdx.x] = 0;
    if (threadIdx.x != 0) return;
    const double* E = a.e_models + 9 * (size_t)c->e_best;
    double U[9], s[3], V[9];
    svd3(E, U, s, V);
    if (det3(U) < 0)
        for (int k = 0; k < 9; ++k) U[k] = -U[k];
    double Vt[9];
    transpose3(V, Vt);
    if (det3(Vt) < 0)
        for (int k = 0; k < 9; ++k) Vt[k] = -Vt[k];
    const double W[9] = {0, 1, 0, -1, 0, 0, 0, 0, 1};
    double Wt[9], UW[9];
    transpose3(W, Wt);
    matmul3(U, W, UW);
    matmul3(UW, Vt, a.rp);
    matmul3(U, Wt, UW);
    matmul3(UW, Vt, a.rp + 9);
    a.rp[18] = U[2] * 1.0;
    a.rp[19] = U[5] * 1.0;
    a.rp[20] = U[8] * 1.0;
}

__global__ __launch_bounds__(256) void recover_count_kernel(GeoArgs a) {
    const GeoCtl* c = a.ctl;
    if (!c->gate || c->e_best < 0) return;
    const int n = c->n;
    // thread = (point, motion): lane l holds motion l & 3 of point l >> 2
    const int g = blockIdx.x * 256 + threadIdx.x;
    if ((int)blockIdx.x * 64 >= n) return;  // workgroup-uniform
    const int i = g >> 2, m = g & 3;
    bool ok = false;
    if (i < n) {
        const double sg = m < 2 ? 1.0 : -1.0;
        const double* R = a.rp + 9 * (m & 1);
        const double* s_t = a.rp + 18;
        const double x1 = a.q1[2 * i], y1 = a.q1[2 * i + 1], x2 = a.q2[2 * i], y2 = a.q2[2 * i + 1];
        const double tt[3] = {sg * s_t[0], sg * s_t[1], sg * s_t[2]};
        double X[4];
        triangulate_h(R, tt, x1, y1, x2, y2, X);
        ok = X[2] * X[3] > 0;
        const double Q[3] = {X[0] / X[3], X[1] / X[3], X[2] / X[3]};
        ok = (Q[2] < 50.0) && ok;
        const double z2 = R[6] * Q[0] + R[7] * Q[1] + R[8] * Q[2] + tt[2] * 1.0;
        ok = (z2 > 0) && ok;
        ok = (z2 < 50.0) && ok;
        ok = ok && a.e_mask[i];
    }
    // per motion: the lanes l with l & 3 == m
    const unsigned long long b = __ballot(ok);
    const unsigned long long sel = 0x1111111111111111ULL;
    if ((threadIdx.x & 63) < 4) {
        const int cnt = __popcll(b & (sel << (threadIdx.x & 3)));
        if (cnt) atomicAdd(&a.rp_good[threadIdx.x & 3], cnt);
    }
}

__global__ __launch_bounds__(64) void recover_pick_kernel(GeoArgs a) {
    GeoCtl* c = a.ctl;
    if (!c->gate || c->e_best < 0 || threadIdx.x != 0) return;
    int G[4];
    for (int m = 0; m < 4; ++m) G[m] = a.rp_good[m];
    int pick;
    if (G[0] >= G[1] && G[0] >= G[2] && G[0] >= G[3])
        pick = 0;
    else if (G[1] >= G[0] && G[1] >= G[2] && G[1] >= G[3])
        pick = 1;
    else if (G[2] >= G[0] && G[2] >= G[1] && G[2] >= G[3])
        pick = 2;
    else
        pick = 3;
    double* cand = c->cand[0];  // the E path's slot
    for (int k = 0; k < 9; ++k) cand[k] = a.rp[9 * (pick & 1) + k];
    for (int k = 0; k < 3; ++k) cand[9 + k] = pick >= 2 ? -a.rp[18 + k] : a.rp[18 + k];
    c->e_ncand = 1;
}

// ---------------------------------------------------------------- H refine moments
// The least-squares DLT refinement's 9 x 9 moment matrix M = sum_i (ra ra^T +
// rb rb^T) over the winner's inliers: the 45 upper-triangle leaves of every
// point in one pass (thread per point), then the 45 canonical trees in
// parallel (workgroup per entry), each exactly block_tree_sum's.
__global__ __launch_bounds__(256) void h_moment_leaves_kernel(GeoArgs a) {
    const GeoCtl* c = a.ctl;
    if (!c->gate || c->h_best < 0 || c->h_count < 4) return;
    const int n = c->n;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    double ra[9], rb[9];
    h_rows(a.q1[2 * i], a.q1[2 * i + 1], a.q2[2 * i], a.q2[2 * i + 1], ra, rb);
    const bool in = a.h_mask[i] != 0;
    int k = 0;
    for (int r = 0; r < 9; ++r)
        for (int col = r; col < 9; ++col, ++k)
            a.hm[(size_t)k * a.cap + i] = in ? ra[r] * ra[col] + rb[r] * rb[col] : 0.0;
}

__global__ __launch_bounds__(256) void h_moment_sums_kernel(GeoArgs a) {
    __shared__ double s_red[4];
    const GeoCtl* c = a.ctl;
    if (!c->gate || c->h_best < 0 || c->h_count < 4) return;
    const int n = c->n;
    const int k = blockIdx.x;  // upper-triangle entry, row-major
    int r = 0, e = k;
    while (e >= 9 - r) {
        e -= 9 - r;
        ++r;
    }
    const int col = r + e;
    const double* leaf = a.hm + (size_t)k * a.cap;
    const double s = block_tree_sum(n, [&](int i) { return leaf[i]; }, s_red);
    if (threadIdx.x == 0) {
        a.hM[9 * r + col] = s;
        a.hM[9 * col + r] = s;
    }
}

// ---------------------------------------------------------------- H refine + decompose
// LDS hand-off between the lanes of one wave
__device__ inline void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The eigenvector of the smallest eigenvalue of the symmetric 9 x 9 moment
// matrix (the least-squares DLT refinement of the winning homography) by a
// round-robin (parallel-ordered) cyclic Jacobi on one wave: per round each
// (pair, index) lane forms its pair's rotation from the round's A, rotates
// the column pairs of A and V, then the row pairs of A (two LDS hand-offs per
// round; round 4 formed the rotations in lanes 0-4 and passed them on: three).  Restated step for step by oracle_linalg.hpp jacobi_eigen_rr
// (sweep test, stop rule, descending selection sort).  All lanes return it.
__device__ void smallest_eigvec9_rr(const double* __restrict__ Min, double* out) {
    constexpr int N = 9, M = 10, R = 9, P = 5;
    __shared__ double sA[81], sV[81];
    const int lane = threadIdx.x & 63;
    for (int k = lane; k < 81; k += 64) {
        sA[k] = Min[k];
        sV[k] = (k % (N + 1) == 0) ? 1.0 : 0.0;
    }
    wave_lds_sync();
    for (int sweep = 0; sweep < 50; ++sweep) {
        // every lane forms the same sums (the oracle's order)
        double off = 0, diag = 0;
        for (int p = 0; p < N; ++p) {
            diag = diag + sA[N * p + p] * sA[N * p + p];
            for (int q = p + 1; q < N; ++q) off = off + sA[N * p + q] * sA[N * p + q];
        }
        off = uniform_f64(off);
        diag = uniform_f64(diag);
        if (off <= 1e-30 * diag || off == 0.0) break;
        for (int r = 0; r < R; ++r) {
            // lane (i, k) < 45: pair i's rotation, formed in the lane itself
            // from the round's A (the same operations in all nine lanes of
            // the pair: no hand-off through LDS), then its rotation of the
            // column pairs (p, q) of A and of V at row k, then of A's row
            // pairs at column k; (p, q) from the circle method: arr[0] = 0,
            // arr[j] = 1 + (j - 1 + r) mod 9, pair i = (arr[i], arr[9 - i])
            const int i = lane / N, k = lane - N * (lane / N);
            const bool own = lane < P * N;
            const int a0 = i == 0 ? 0 : 1 + (i - 1 + r) % (M - 1);
            const int b0 = 1 + (M - 1 - i - 1 + r) % (M - 1);
            const int p = a0 < b0 ? a0 : b0, q0 = a0 < b0 ? b0 : a0;
            const int q = q0 < N ? q0 : p;  // the idle pair (q0 = 9) loads in bounds, stores nothing
            double c = 0.0, sn = 0.0;
            bool act = false;
            if (own) {
                const double apq = sA[N * p + q];
                act = q0 < N && apq != 0.0;
                if (act) {
                    const double theta = (sA[N * q + q] - sA[N * p + p]) / (2.0 * apq);
                    const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                    c = 1.0 / sqrt(t * t + 1.0);
                    sn = t * c;
                }
            }
            double akp = 0, akq = 0, vkp = 0, vkq = 0;
            if (own) {
                akp = sA[N * k + p];
                akq = sA[N * k + q];
                vkp = sV[N * k + p];
                vkq = sV[N * k + q];
            }
            // every lane of the wave has read the round's A before any lane writes
            wave_lds_sync();
            if (own && act) {
                sA[N * k + p] = c * akp - sn * akq;
                sA[N * k + q] = sn * akp + c * akq;
                sV[N * k + p] = c * vkp - sn * vkq;
                sV[N * k + q] = sn * vkp + c * vkq;
            }
            wave_lds_sync();
            // row pairs of A
            if (own) {
                const double apk = sA[N * p + k], aqk = sA[N * q + k];
                if (act) {
                    sA[N * p + k] = c * apk - sn * aqk;
                    sA[N * q + k] = sn * apk + c * aqk;
                }
            }
            wave_lds_sync();
        }
    }
    // descending selection sort of the diagonal (first maximum first); the
    // last position's column
    int idx[N];
    double d[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        idx[i] = i;
        d[i] = sA[N * i + i];
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {
        int m = i;
#pragma unroll
        for (int j = i + 1; j < N; ++j)
            if (d[idx[j]] > d[idx[m]]) m = j;
        const int tmp = idx[i];
        idx[i] = idx[m];
        idx[m] = tmp;
    }
    const int last = idx[N - 1];
    for (int k = 0; k < N; ++k) out[k] = sV[N * k + last];
}

__global__ __launch_bounds__(64) void h_refine_decompose_kernel(GeoArgs a) {
    GeoCtl* c = a.ctl;
    if (!c->gate || c->h_best < 0) return;
    const int good = c->h_count;
    double H[9];
    const double* Hb = a.h_models + 9 * (size_t)c->h_best;
    for (int k = 0; k < 9; ++k) H[k] = Hb[k];
    if (good >= 4) smallest_eigvec9_rr(a.hM, H);  // the whole wave
    if (threadIdx.x != 0) return;
    if (fabs(H[8]) > 1e-12) {
        const double d = H[8];
        for (int k = 0; k < 9; ++k) H[k] = H[k] / d;
    }
    for (int k = 0; k < 9; ++k) c->H[k] = H[k];
    // cv::decomposeHomographyMat(H, I) — HomographyDecompInria
    double U[9], s[3], V[9];
    svd3(H, U, s, V);
    double Hn[9];
    const double inv = 1.0 / s[1];
    for (int k = 0; k < 9; ++k) Hn[k] = H[k] * inv;
    double Ht[9], S[9];
    transpose3(Hn, Ht);
    matmul3(Ht, Hn, S);
    S[0] -= 1.0;
    S[4] -= 1.0;
    S[8] -= 1.0;
    double mx = 0;
    for (int k = 0; k < 9; ++k) mx = fmax(mx, fabs(S[k]));
    if (mx < 0.001) {
        double* cand = c->cand[1];  // the H path's slots start at 1
        for (int k = 0; k < 9; ++k) cand[k] = Hn[k];
        cand[9] = cand[10] = cand[11] = 0;
        c->h_ncand = 1;
        return;
    }
    auto minor = [&](int row, int col) {
        const int x1 = col == 0 ? 1 : 0, x2 = col == 2 ? 1 : 2;
        const int y1 = row == 0 ? 1 : 0, y2 = row == 2 ? 1 : 2;
        return S[3 * y1 + x2] * S[3 * y2 + x1] - S[3 * y1 + x1] * S[3 * y2 + x2];
    };
    auto signd = [](double x) { return x >= 0 ? 1 : -1; };
    const double M00 = minor(0, 0), M11 = minor(1, 1), M22 = minor(2, 2);
    const double rtM00 = sqrt(M00), rtM11 = sqrt(M11), rtM22 = sqrt(M22);
    const double M01 = minor(0, 1), M12 = minor(1, 2), M02 = minor(0, 2);
    const int e12 = signd(M12), e02 = signd(M02), e01 = signd(M01);
    const double nS00 = fabs(S[0]), nS11 = fabs(S[4]), nS22 = fabs(S[8]);
    int indx = 0;
    if (nS00 < nS11) {
        indx = 1;
        if (nS11 < nS22) indx = 2;
    } else {
        if (nS00 < nS22) indx = 2;
    }
    double npa[3], npb[3];
    if (indx == 0) {
        npa[0] = S[0], npb[0] = S[0];
        npa[1] = S[1] + rtM22, npb[1] = S[1] - rtM22;
        npa[2] = S[2] + e12 * rtM11, npb[2] = S[2] - e12 * rtM11;
    } else if (indx == 1) {
        npa[0] = S[1] + rtM22, npb[0] = S[1] - rtM22;
        npa[1] = S[4], npb[1] = S[4];
        npa[2] = S[5] - e02 * rtM00, npb[2] = S[5] + e02 * rtM00;
    } else {
        npa[0] = S[2] + e01 * rtM11, npb[0] = S[2] - e01 * rtM11;
        npa[1] = S[5] + rtM00, npb[1] = S[5] - rtM00;
        npa[2] = S[8], npb[2] = S[8];
    }
    const double traceS = S[0] + S[4] + S[8];
    const double v = 2.0 * (double)sqrtf((float)(1 + traceS - M00 - M11 - M22));
    const double ESii = signd(S[3 * indx + indx]);
    const double r = sqrt(2 + traceS + v);
    const double n_t = sqrt(2 + traceS - v);
    const double na_n = sqrt((npa[0] * npa[0] + npa[1] * npa[1]) + npa[2] * npa[2]);
    const double nb_n = sqrt((npb[0] * npb[0] + npb[1] * npb[1]) + npb[2] * npb[2]);
    double na[3], nb[3];
    for (int k = 0; k < 3; ++k) {
        na[k] = npa[k] / na_n;
        nb[k] = npb[k] / nb_n;
    }
    const double half_nt = 0.5 * n_t;
    const double esii_t_r = ESii * r;
    double ta_star[3], tb_star[3];
    for (int k = 0; k < 3; ++k) {
        ta_star[k] = half_nt * (esii_t_r * nb[k] - n_t * na[k]);
        tb_star[k] = half_nt * (esii_t_r * na[k] - n_t * nb[k]);
    }
    auto rmat = [&](const double* tstar, const double* nn, double* R) {
        double Mx[9];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) Mx[3 * i + j] = (i == j ? 1.0 : 0.0) - (2 / v) * tstar[i] * nn[j];
        matmul3(Hn, Mx, R);
        if (det3(R) < 0)
            for (int k = 0; k < 9; ++k) R[k] = -R[k];
    };
    double Ra[9], Rb[9], ta[3], tb[3];
    rmat(ta_star, na, Ra);
    mat3_vec(Ra, ta_star, ta);
    rmat(tb_star, nb, Rb);
    mat3_vec(Rb, tb_star, tb);
    const double* Rs[4] = {Ra, Ra, Rb, Rb};
    const double* ts[4] = {ta, ta, tb, tb};
    const double sg[4] = {1, -1, 1, -1};
    for (int m = 0; m < 4; ++m) {
        double* cand = c->cand[1 + m];
        for (int k = 0; k < 9; ++k) cand[k] = Rs[m][k];
        for (int k = 0; k < 3; ++k) cand[9 + k] = sg[m] > 0 ? ts[m][k] : -ts[m][k];
    }
    c->h_ncand = 4;
}

// candidate mi of SelectMotion (the reference's order: recoverPose's, then
// decomposeHomographyMat's) -> its slot
__device__ inline int cand_slot(const GeoCtl* c, int mi) { return mi < c->e_ncand ? 0 : 1 + (mi - c->e_ncand); }

// ---------------------------------------------------------------- SelectMotion
__global__ __launch_bounds__(256) void select_points_kernel(GeoArgs a) {
    const GeoCtl* c = a.ctl;
    if (!c->gate) return;
    const int n = c->n, m = c->e_ncand + c->h_ncand;
    const int gid = blockIdx.x * 256 + threadIdx.x;
    const int mi = gid / a.cap, i = gid - mi * a.cap;
    if (mi >= m || i >= n) return;
    const double kPi = 3.14159265358979323846;
    const double* R = c->cand[cand_slot(c, mi)];
    const double* T = c->cand[cand_slot(c, mi)] + 9;
    uint8_t* inl = a.sel_in + (size_t)mi * a.cap;
    double* pts = a.sel_pts + (size_t)mi * a.cap * 3;
    inl[i] = 0;
    pts[3 * i] = pts[3 * i + 1] = pts[3 * i + 2] = 0.0;
    double O2[3];
    for (int r = 0; r < 3; ++r) O2[r] = (-R[3 * r]) * T[0] + (-R[3 * r + 1]) * T[1] + (-R[3 * r + 2]) * T[2];
    const double x1 = a.p1[3 * i], y1 = a.p1[3 * i + 1], x2 = a.p2[3 * i], y2 = a.p2[3 * i + 1];
    double X[4];
    triangulate_h(R, T, x1, y1, x2, y2, X);
    const double P1[3] = {X[0] / X[3], X[1] / X[3], X[2] / X[3]};
    if (P1[2] < 0) return;
    const double n2[3] = {P1[0] - O2[0], P1[1] - O2[1], P1[2] - O2[2]};
    const double d1 = sqrt((P1[0] * P1[0] + P1[1] * P1[1]) + P1[2] * P1[2]);
    const double d2 = sqrt((n2[0] * n2[0] + n2[1] * n2[1]) + n2[2] * n2[2]);
    double parallax = (P1[0] * n2[0] + P1[1] * n2[1]) + P1[2] * n2[2];
    parallax /= (d1 * d2);
    parallax = acos(parallax) * 180 / kPi;
    if (parallax > a.parallax_thresh) return;
    double dx = (P1[0] / P1[2] - x1) * a.K[0];
    double dy = (P1[1] / P1[2] - y1) * a.K[1];
    if (sqrt(dx * dx + dy * dy) > a.proj_thresh) return;
    double P2[3];
    mat3_vec(R, P1, P2);
    P2[0] = P2[0] + T[0];
    P2[1] = P2[1] + T[1];
    P2[2] = P2[2] + T[2];
    if (P2[2] < 0) return;
    dx = (P2[0] / P2[2] - x2) * a.K[0];
    dy = (P2[1] / P2[2] - y2) * a.K[1];
    if (sqrt(dx * dx + dy * dy) > a.proj_thresh) return;
    inl[i] = 1;
    pts[3 * i] = P1[0];
    pts[3 * i + 1] = P1[1];
    pts[3 * i + 2] = P1[2];
}

// SelectMotion's reduction and output in one single-workgroup launch
// (src/viso.cpp:596-638): the candidates' inlier counts in one pass over the
// flags (integers: any order), the first maximum, the mean depth of the
// best candidate's points (block_tree_sum, the oracle's tree), then the
// normalised inlier points in index order: thread t owns the contiguous
// flags [t per, (t + 1) per), so one exclusive scan of the per-thread counts
// places every point (round 4: one launch per step and three block barriers
// per 256 flags, 31 us for ~2,000 tracks).  1,024 threads: each thread's
// serial share of flags, depth leaves and outputs (dependent global loads,
// one latency each) is a quarter of a 256-thread block's.
constexpr int kSelThreads = 1024;
constexpr int kSelWaves = kSelThreads / 64;

__global__ __launch_bounds__(kSelThreads) void select_finish_kernel(GeoArgs a) {
    __shared__ double s_red[kSelWaves];
    __shared__ int s_cnt[kSelWaves][kMaxCandidates];
    __shared__ int s_wave[kSelWaves];
    __shared__ int s_best, s_bestn;
    GeoCtl* c = a.ctl;
    if (!c->gate) return;
    const int n = c->n, m = c->e_ncand + c->h_ncand;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    int cnt[kMaxCandidates];
#pragma unroll
    for (int k = 0; k < kMaxCandidates; ++k) cnt[k] = 0;
    for (int i = t; i < n; i += kSelThreads)
#pragma unroll
        for (int k = 0; k < kMaxCandidates; ++k)
            if (k < m) cnt[k] += a.sel_in[(size_t)k * a.cap + i];
#pragma unroll
    for (int k = 0; k < kMaxCandidates; ++k) {
        const int w = wave_sum_int(cnt[k]);
        if (lane == 0) s_cnt[wave][k] = w;
    }
    __syncthreads();
    if (t == 0) {
        int best = -1, bestn = 0;
        for (int k = 0; k < m; ++k) {
            int tot = 0;
            for (int w = 0; w < kSelWaves; ++w) tot += s_cnt[w][k];
            if (tot > bestn) {  // strict: the first maximum wins (src/viso.cpp:605)
                bestn = tot;
                best = k;
            }
        }
        s_best = best;
        s_bestn = bestn;
    }
    __syncthreads();
    const int best = s_best, nr = s_bestn;
    double mean = 0.0;
    if (best >= 0) {
        const uint8_t* inl = a.sel_in + (size_t)best * a.cap;
        const double* pts = a.sel_pts + (size_t)best * a.cap * 3;
        // (both loads issued together: the depth's load does not wait for
        // the flag's)
        mean = block_tree_sum<kSelThreads>(n, [&](int i) {
            const double z = pts[3 * i + 2];
            return inl[i] ? z : 0.0;
        }, s_red);
    }
    // every thread derives the ctl values it needs from the same operations
    const bool nonzero = mean != 0;
    const double md = nonzero ? mean / nr : mean;
    if (t == 0) {
        c->n_cand = m;
        c->nr_inliers = nr;
        c->best_motion = best;
        if (best >= 0) {
            for (int k = 0; k < 9; ++k) c->R[k] = c->cand[cand_slot(c, best)][k];
            for (int k = 0; k < 3; ++k) c->T[k] = c->cand[cand_slot(c, best)][9 + k];
        }
        c->mean_depth = md;
        c->mean_nonzero = nonzero ? 1 : 0;
        if (nonzero)
            for (int k = 0; k < 3; ++k) c->T[k] = c->T[k] / md;
    }
    __syncthreads();
    ctl_mirror(a);
    // output: flags, and the inlier points in order
    const int per = (n + kSelThreads - 1) / kSelThreads;
    const int i0 = min(t * per, n), i1 = min(i0 + per, n);
    const uint8_t* inl = a.sel_in + (size_t)(best >= 0 ? best : 0) * a.cap;
    int own = 0;
    for (int i = i0; i < i1; ++i) own += (best >= 0 && inl[i]) ? 1 : 0;
    // exclusive scan of `own` over the block
    int incl = own;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(incl, off, 64);
        if (lane >= off) incl += y;
    }
    if (lane == 63) s_wave[wave] = incl;
    __syncthreads();
    int off = incl - own;
    for (int k = 0; k < wave; ++k) off += s_wave[k];
    const double* pts = a.sel_pts + (size_t)(best >= 0 ? best : 0) * a.cap * 3;
    for (int i = i0; i < i1; ++i) {
        const bool in = best >= 0 && inl[i] != 0;
        a.inliers[i] = in ? 1 : 0;
        if (in) {
            const double* P = pts + 3 * (size_t)i;
            double* o = a.points_out + 3 * (size_t)off;
            if (nonzero) {
                o[0] = P[0] / md;
                o[1] = P[1] / md;
                o[2] = P[2] / md;
            } else {
                o[0] = P[0];
                o[1] = P[1];
                o[2] = P[2];
            }
            ++off;
        }
    }
}

}  // namespace

void launch_pose_2d2d_gate(const GeoArgs& a, hipStream_t stream) {
    normalize_kernel<<<1, kNormThreads, 0, stream>>>(a, CompactIn{});
}

void launch_compact_gate(const CompactIn& ci, const GeoArgs& a, hipStream_t stream) {
    normalize_kernel<<<1, kNormThreads, 0, stream>>>(a, ci);
}

void launch_pose_2d2d_spec(const GeoArgs& a, hipStream_t stream) {
    if (a.h_iters > 0) h_hyp_kernel<<<(a.h_iters + 3) / 4, 256, 0, stream>>>(a);
}

hipStream_t launch_pose_2d2d_body(const GeoArgs& a, hipStream_t stream, hipStream_t hs, hipEvent_t e_done,
                                  hipEvent_t join, bool h_spec) {
    const bool split = hs && e_done && join && a.h_iters > 0 && a.e_iters > 0;
    // the H chain (the longer one) on `stream` behind its speculative first
    // launch (h_spec) and the E chain on hs, or the H chain on hs
    const hipStream_t sh = h_spec ? stream : (split ? hs : stream);
    const hipStream_t se = h_spec ? (split ? hs : stream) : stream;
    // the two chains interleaved launch by launch so that neither waits for
    // the other's host-side enqueue
    for (int step = 0; step < 6; ++step) {
        if (a.h_iters > 0) {
            switch (step) {
                case 0: if (!h_spec) h_hyp_kernel<<<(a.h_iters + 3) / 4, 256, 0, sh>>>(a); break;
                case 1: score_kernel<false><<<a.h_iters, 256, 0, sh>>>(a); break;
                case 2: scan_kernel<false><<<1, 256, 0, sh>>>(a); break;
                case 3: h_moment_leaves_kernel<<<(a.cap + 255) / 256, 256, 0, sh>>>(a); break;
                case 4: h_moment_sums_kernel<<<45, 256, 0, sh>>>(a); break;
                default: h_refine_decompose_kernel<<<1, 64, 0, sh>>>(a); break;
            }
        }
        if (a.e_iters > 0) {
            switch (step) {
                case 0: e_hyp_kernel<<<(a.e_iters + 3) / 4, 256, 0, se>>>(a); break;
                case 1: score_kernel<true><<<a.e_iters, 256, 0, se>>>(a); break;
                case 2: scan_kernel<true><<<1, 256, 0, se>>>(a); break;
                case 3: recover_setup_kernel<<<1, 64, 0, se>>>(a); break;
                case 4: recover_count_kernel<<<(4 * a.cap + 255) / 256, 256, 0, se>>>(a); break;
                default: recover_pick_kernel<<<1, 64, 0, se>>>(a); break;
            }
        }
    }
    // SelectMotion behind the H chain, once the E chain's event has passed
    if (split) {
        (void)hipEventRecord(e_done, se);
        (void)hipStreamWaitEvent(sh, e_done, 0);
    }
    const int total = 5 * a.cap;
    select_points_kernel<<<(total + 255) / 256, 256, 0, sh>>>(a);
    select_finish_kernel<<<1, kSelThreads, 0, sh>>>(a);
    if (split && sh != stream) {
        (void)hipEventRecord(join, sh);
        (void)hipStreamWaitEvent(stream, join, 0);
    }
    return sh;
}

void launch_pose_2d2d(const GeoArgs& a, hipStream_t stream, Timing* timing) {
    launch_pose_2d2d_gate(a, stream);
    launch_pose_2d2d_body(a, stream);
    (void)timing;
}

}  // namespace viso
