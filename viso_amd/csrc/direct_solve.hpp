// viso_amd — the serial 6x6 Gauss-Newton step of one direct-pose level on
// one wave (DirectPoseEstimationSingleLayer, src/viso.cpp:731-753): H, b from
// the 28 canonical sums -> Eigen PartialPivLU inverse -> update = H^-1 b ->
// Sophus SE3::exp(update) * T21 -> the loop decision.  Shared by
// direct_level_kernel (direct.hip) and the solve micro-benchmark
// (tools/ubench/solve_bench.hip).
#pragma once

#include "common.hpp"
#include "device_math.hpp"


namespace viso {

constexpr int kSolveSums = 28;
constexpr int kSolveStateStride = 8;

struct SolveLds {
    double red[4][kSolveSums];
    double S[kSolveSums];
    int g[4];
    int ngood;
    double state[kSolveStateStride], best[kSolveStateStride];
    double cost, last_cost;
    int cont;
};

// phase stamps (probe builds): s_memrealtime after LU / inverse / update /
// exp, kept in registers (the caller records them)
#define SPROBE(k)                                                   \
    do {                                                            \
        if (stamps) stamps[(k)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)

// The rest of one GN step after `update` (src/viso.cpp:735-753): SE3::exp,
// T21 = exp(update) * T21, cost /= nGood and the loop decision; stats of
// block 0.  `h`: this lane's H element (lane < 36, row-major) for stats.
__device__ __attribute__((always_inline)) inline void solve_finish(SolveLds& L, const double* update, double h, int iter, double* stats,
                                    unsigned long long* stamps) {
    const int lane = threadIdx.x & 63;
    const bool in = lane < 36;
    // the loop decision (src/viso.cpp:739-753) does not depend on the new
    // T21: its operands are read and evaluated first, off the exp chain
    const int ngood = L.ngood;
    double cost = L.cost + L.S[27];
    cost /= ngood;
    const double lastCost = L.last_cost;
    const bool nan_update = isnan(update[0]);
    const bool cost_up = iter > 0 && cost > lastCost;
    const bool converged = (1 - cost / (double)lastCost) < 0.005;
    SE3d T21;
#pragma unroll
    for (int k = 0; k < 4; ++k) T21.q[k] = L.state[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) T21.t[k] = L.state[4 + k];
    // ---- SE3::exp(update) (Sophus), sin/cos of theta/2 and theta in lanes 0/1
    SE3d E;
    {
        const double eps = 1e-10;
        const double* w = update + 3;
        const double theta_sq = (w[0] * w[0] + w[1] * w[1]) + w[2] * w[2];
        const double theta = sqrt(theta_sq);
        const double half_theta = 0.5 * theta;
        double sn, cs;
        sincos((lane & 1) ? theta : half_theta, &sn, &cs);
        const double s_half = readlane_f64(sn, 0), c_half = readlane_f64(cs, 0);
        const double s_th = readlane_f64(sn, 1), c_th = readlane_f64(cs, 1);
        double imag, real;
        if (theta < eps) {
            const double theta_po4 = theta_sq * theta_sq;
            imag = 0.5 - (1.0 / 48.0) * theta_sq + (1.0 / 3840.0) * theta_po4;
            real = 1.0 - 0.5 * theta_sq + (1.0 / 384.0) * theta_po4;
        } else {
            imag = s_half / theta;
            real = c_half;
        }
        E.q[0] = imag * w[0];
        E.q[1] = imag * w[1];
        E.q[2] = imag * w[2];
        E.q[3] = real;
        double V[9];
        if (theta < eps) {
            quat_to_matrix(E.q, V);
        } else {
            const double O[9] = {0.0, -w[2], w[1], w[2], 0.0, -w[0], -w[1], w[0], 0.0};
            double O2[9];
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 3; ++j)
                    O2[3 * i + j] = (O[3 * i + 0] * O[0 + j] + O[3 * i + 1] * O[3 + j]) + O[3 * i + 2] * O[6 + j];
            const double th2 = theta * theta;
            const double c1 = (1.0 - c_th) / th2;
            const double c2 = (theta - s_th) / (th2 * theta);
#pragma unroll
            for (int i = 0; i < 9; ++i) {
                const double id = (i % 4 == 0) ? 1.0 : 0.0;
                V[i] = (id + c1 * O[i]) + c2 * O2[i];
            }
        }
        mat3_vec(V, update, E.t);
    }
    SPROBE(3);
    T21 = se3_mul(E, T21);
    if (stats) {
        if (in) stats[2 + lane] = h;
        if (lane == 0) {
            stats[0] = ngood;
            stats[1] = cost;
            for (int k = 0; k < 6; ++k) stats[38 + k] = L.S[21 + k];
            for (int k = 0; k < 6; ++k) stats[44 + k] = update[k];
        }
    }
    if (lane == 0) {
        int cont = 1;
        if (nan_update) {
            for (int k = 0; k < 7; ++k) L.state[k] = L.best[k];
            cont = 0;
        } else {
            for (int k = 0; k < 4; ++k) L.state[k] = T21.q[k];
            for (int k = 0; k < 3; ++k) L.state[4 + k] = T21.t[k];
            if (cost_up) {
                for (int k = 0; k < 7; ++k) L.state[k] = L.best[k];
                cont = 0;
            } else if (converged) {
                cont = 0;
            } else {
                for (int k = 0; k < 7; ++k) L.best[k] = L.state[k];
                L.last_cost = cost;
            }
        }
        L.cost = cost;
        L.cont = cont;
    }
}



__device__ __attribute__((always_inline)) inline void solve_after_lu(SolveLds& L, const double* A, const int* tr,
                                                                      double h, int iter, double* stats,
                                                                      unsigned long long* stamps);

// One GN step of one level on wave 0 (all 64 lanes): L.S -> update, the new
// L.state and the loop decision L.cont (src/viso.cpp:731-753), with the LU
// replicated in every lane's registers (the
// product's solve: solve_wave0 below).
__device__ __attribute__((always_inline)) inline void solve_wave0_rep(SolveLds& L, int iter, double* stats,
                                   unsigned long long* stamps = nullptr) {
    const int lane = threadIdx.x & 63;
    const int row = lane / 6, col = lane - 6 * (lane / 6);
    const bool in = lane < 36;
    // H (symmetric) from the 21 upper-triangle sums, one element per lane
    const int r0 = row < col ? row : col, c0 = row < col ? col : row;
    const double h = in ? L.S[r0 * 6 - (r0 * (r0 - 1)) / 2 + (c0 - r0)] : 0.0;
    // ---- Eigen PartialPivLU (first maximal |pivot| wins), replicated in the
    // registers of every lane: no cross-lane traffic on the serial chain; the
    // pivot row is wave-uniform, so a row swap is a scalar branch + moves.
    double A[36];
    int tr[6];
#ifdef VISO_LU_TWICE
    // probe experiment: the LU runs twice (the same instructions), the first
    // pass's end stamped in stamps[4] -- a second pass faster than the first
    // means the first waited on instruction fetch
#pragma clang loop unroll(disable)
    for (int rep = 0; rep < 2; ++rep) {
#endif
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int c = 0; c < 6; ++c) {
            const int r1 = r < c ? r : c, c1 = r < c ? c : r;
            A[6 * r + c] = L.S[r1 * 6 - (r1 * (r1 - 1)) / 2 + (c1 - r1)];
        }
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        int p = k;
        double best = fabs(A[7 * k]);
#pragma unroll
        for (int i = k + 1; i < 6; ++i) {
            const double s = fabs(A[6 * i + k]);
            if (s > best) {
                best = s;
                p = i;
            }
        }
        p = __builtin_amdgcn_readfirstlane(p);
        tr[k] = p;
        if (__builtin_amdgcn_readfirstlane(best != 0.0 ? 1 : 0)) {
#pragma unroll
            for (int i = k + 1; i < 6; ++i) {
                if (p == i) {
#pragma unroll
                    for (int c = 0; c < 6; ++c) {
                        const double tmp = A[6 * k + c];
                        A[6 * k + c] = A[6 * i + c];
                        A[6 * i + c] = tmp;
                    }
                }
            }
            const double piv = A[7 * k];
#pragma unroll
            for (int i = k + 1; i < 6; ++i) A[6 * i + k] = A[6 * i + k] / piv;
        }
#pragma unroll
        for (int i = k + 1; i < 6; ++i)
#pragma unroll
            for (int c = k + 1; c < 6; ++c) A[6 * i + c] = A[6 * i + c] - A[6 * i + k] * A[6 * k + c];
    }
#ifdef VISO_LU_TWICE
    if (rep == 0) {
        asm volatile("" ::"v"(A[35]), "v"(A[0]));
        if (stamps) stamps[4] = __builtin_amdgcn_s_memrealtime();
    }
    }
#endif
    SPROBE(0);
    solve_after_lu(L, A, tr, h, iter, stats, stamps);
}

// The rest of the faithful step after the LU factors (A, unit L below the
// diagonal, U on and above, replicated in every lane) and the row
// transpositions tr: the inverse, update = H^-1 b, solve_finish.
__device__ __attribute__((always_inline)) inline void solve_after_lu(SolveLds& L, const double* A, const int* tr,
                                                                      double h, int iter, double* stats,
                                                                      unsigned long long* stamps) {
    const int lane = threadIdx.x & 63;
    // ---- inverse: lane c < 6 solves column c of X = P * I by forward (unit
    // L) and backward (U) substitution
    const int cc = lane < 6 ? lane : 0;
    int pos = cc;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        if (pos == k) pos = tr[k];
        else if (pos == tr[k]) pos = k;
    }
    double x[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) x[r] = (r == pos) ? 1.0 : 0.0;
#pragma unroll
    for (int j = 0; j < 6; ++j)
#pragma unroll
        for (int i = j + 1; i < 6; ++i) x[i] = x[i] - A[6 * i + j] * x[j];
#pragma unroll
    for (int j = 5; j >= 0; --j) {
        x[j] = x[j] / A[7 * j];
#pragma unroll
        for (int i = 0; i < j; ++i) x[i] = x[i] - A[6 * i + j] * x[j];
    }
    SPROBE(1);
    // ---- update = H^-1 * b (row-wise, ascending columns); H^-1[r][c] is
    // lane c's x[r]: transposed through LDS (L.red is free once L.S is
    // formed), lane r < 6 forms row r's dot product, then every lane reads
    // the six results (the same products and sums as a per-row loop over
    // readlanes, a quarter of the instructions)
    double update[6];
    {
        double* Tt = &L.red[0][0];
        if (lane < 6) {
#pragma unroll
            for (int r = 0; r < 6; ++r) Tt[6 * r + lane] = x[r];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        double s = 0.0;
        if (lane < 6) {
            const double* row = Tt + 6 * lane;
            s = row[0] * L.S[21];
#pragma unroll
            for (int c = 1; c < 6; ++c) s = s + row[c] * L.S[21 + c];
        }
#pragma unroll
        for (int r = 0; r < 6; ++r) update[r] = readlane_f64(s, r);
    }
    SPROBE(2);
    solve_finish(L, update, h, iter, stats, stamps);
}


// Lane-per-element PartialPivLU : lane 6 r + c < 36 holds
// A[r][c]; per step the pivot column is read by readlane (uniform, first
// maximal |pivot| wins as in Eigen), the row swap and the rank-1 update's
// operands move by ds_bpermute, the division and update are one element per
// lane with the replicated form's operations.  The factors then go through
// LDS into every lane's registers for solve_after_lu (same inverse / update /
// finish): the result bits equal solve_wave0_rep's (solve_bench checks the
// hash).  Per step one division and one update per lane instead of up to
// five divisions and 25 updates in every lane: 2.84 against 3.13 us per solve
// alone (profiles/r05_solve_bench.log), but 0.1 us per level SLOWER inside
// direct_level_kernel, where the other waves' prefetch shares the LDS pipe
// with its ds_bpermute hops (profiles/r05_solve_ab.log): not the product's
// (build with -DVISO_SOLVE_LANE to use it).
__device__ inline double bperm_f64(double v, int src) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_ds_bpermute(src * 4, (int)(b & 0xffffffffLL));
    const int hi = __builtin_amdgcn_ds_bpermute(src * 4, (int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __attribute__((always_inline)) inline void solve_wave0_lane(SolveLds& L, int iter, double* stats,
                                                                        unsigned long long* stamps = nullptr) {
    const int lane = threadIdx.x & 63;
    const int r = lane / 6, c = lane - 6 * (lane / 6);
    const bool in = lane < 36;
    const int r0 = r < c ? r : c, c0 = r < c ? c : r;
    const double h = in ? L.S[r0 * 6 - (r0 * (r0 - 1)) / 2 + (c0 - r0)] : 0.0;
    double a = h;
    int tr[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        int p = k;
        double best = fabs(readlane_f64(a, 7 * k));
#pragma unroll
        for (int i = k + 1; i < 6; ++i) {
            const double s = fabs(readlane_f64(a, 6 * i + k));
            if (s > best) {
                best = s;
                p = i;
            }
        }
        p = __builtin_amdgcn_readfirstlane(p);
        tr[k] = p;
        if (__builtin_amdgcn_readfirstlane(best != 0.0 ? 1 : 0)) {
            if (p != k) a = bperm_f64(a, r == k ? 6 * p + c : (r == p ? 6 * k + c : lane));
            const double piv = readlane_f64(a, 7 * k);
            if (in && r > k && c == k) a = a / piv;
        }
        if (k < 5) {
            const double lk = bperm_f64(a, 6 * r + k), kc = bperm_f64(a, 6 * k + c);
            if (in && r > k && c > k) a = a - lk * kc;
        }
    }
    double* T = &L.red[0][0];
    if (in) T[lane] = a;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    double A[36];
#pragma unroll
    for (int i = 0; i < 36; ++i) A[i] = T[i];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    SPROBE(0);
    solve_after_lu(L, A, tr, h, iter, stats, stamps);
}


__device__ __attribute__((always_inline)) inline void solve_wave0(SolveLds& L, int iter, double* stats,
                                                                   unsigned long long* stamps = nullptr) {
#ifdef VISO_SOLVE_LANE
    solve_wave0_lane(L, iter, stats, stamps);
#else
    solve_wave0_rep(L, iter, stats, stamps);
#endif
}

// Tolerance mode (VISO_PRECISION_FAST): update = H^-1 b by an LDL^T
// factorisation of the (symmetric positive semi-definite) H and two
// triangular solves, replicated in every lane (no pivoting, no explicit
// inverse: ~1/4 of the faithful PartialPivLU chain).  A non-positive or
// non-finite pivot gives a NaN update, which reverts the level as the
// reference's isnan(update[0]) test does.  Then solve_finish as faithful.
__device__ __attribute__((always_inline)) inline void solve_wave0_ldlt(SolveLds& L, int iter, double* stats,
                                        unsigned long long* stamps = nullptr) {
    const int lane = threadIdx.x & 63;
    const int row = lane / 6, col = lane - 6 * (lane / 6);
    const bool in = lane < 36;
    const int r0 = row < col ? row : col, c0 = row < col ? col : row;
    const double h = in ? L.S[r0 * 6 - (r0 * (r0 - 1)) / 2 + (c0 - r0)] : 0.0;
    double A[21];  // lower triangle, row-major: A[i(i+1)/2 + j], j <= i
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) A[i * (i + 1) / 2 + j] = L.S[j * 6 - (j * (j - 1)) / 2 + (i - j)];
    double b[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) b[k] = L.S[21 + k];
    double Dinv[6];
    bool bad = false;
    // A = L D L^T in place: A[i][j] (j < i) <- L_ij, A[i][i] <- D_i
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        double d = A[k * (k + 1) / 2 + k];
#pragma unroll
        for (int j = 0; j < k; ++j) {
            const double lkj = A[k * (k + 1) / 2 + j];
            d = __builtin_fma(-lkj * lkj, A[j * (j + 1) / 2 + j], d);
        }
        bad = bad || !(d > 0.0) || !(d < 1e300);
        const double di = 1.0 / d;
        Dinv[k] = di;
        A[k * (k + 1) / 2 + k] = d;
#pragma unroll
        for (int i = k + 1; i < 6; ++i) {
            double s = A[i * (i + 1) / 2 + k];
#pragma unroll
            for (int j = 0; j < k; ++j)
                s = __builtin_fma(-A[i * (i + 1) / 2 + j] * A[j * (j + 1) / 2 + j], A[k * (k + 1) / 2 + j], s);
            A[i * (i + 1) / 2 + k] = s * di;
        }
    }
    SPROBE(0);
    // L y = b, z = D^-1 y, L^T x = z
    double y[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        double s = b[i];
#pragma unroll
        for (int j = 0; j < i; ++j) s = __builtin_fma(-A[i * (i + 1) / 2 + j], y[j], s);
        y[i] = s;
    }
    double update[6];
#pragma unroll
    for (int i = 5; i >= 0; --i) {
        double s = y[i] * Dinv[i];
#pragma unroll
        for (int j = i + 1; j < 6; ++j) s = __builtin_fma(-A[j * (j + 1) / 2 + i], update[j], s);
        update[i] = s;
    }
    if (bad)
#pragma unroll
        for (int k = 0; k < 6; ++k) update[k] = __builtin_nan("");
    SPROBE(1);
    SPROBE(2);
    solve_finish(L, update, h, iter, stats, stamps);
}

}  // namespace viso
