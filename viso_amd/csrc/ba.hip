// viso_amd — photometric bundle adjustment on gfx950 (SURVEY.md §8(f) row 4;
// the BA that include/bundle_adjuster.h:22-106 sketches with g2o).  Spec and
// CPU restatement: oracle/oracle_ba.cpp (header) — every sum here follows its
// order, so GPU == oracle up to libm (sin/cos/sqrt of SE3::exp).
//
// Per Levenberg-Marquardt iteration (all on one stream, no host sync):
//   linearise   wave per map point; 4 edges at a time, 16 lanes per edge
//               (lane = patch pixel): residual and analytic Jacobians, the 55
//               per-edge sums by a 16-lane xor tree; V, bp, cost folded over
//               the point's edges (target keyframe ascending)
//   [it 0] mu0  1e-5 max diag of the Hessian (camera diagonal trees + point max)
//   vinv        thread per point: (V + mu I)^-1
//   reduce      workgroup per entry of the reduced camera system S, g and the
//               camera gradient bc: the canonical tree over the points
//   solve       one wave: LDL^T of S + mu I (lane per row), substitutions
//   points      thread per point: dp = Vinv (bp - W dc), candidate X', its
//               part of the predicted decrease; candidate poses exp(dc) T
//   cost        wave per point: the candidate's 16-pixel costs
//   decide      one workgroup: costs / predicted decrease -> rho, accept,
//               mu / nu update (g2o OptimizationAlgorithmLevenberg)
//   commit      thread per point: accepted candidates become the estimate
// The edge set (every tap inside both images) is fixed at the first
// linearisation point, as the sketch's setLevel(1) at its first evaluation.
#include "context.hpp"
#include "device_math.hpp"
#include "linalg.hpp"

namespace viso {

namespace {

constexpr int kPx = 16;
constexpr int kEs = 55;  // Hpp 6, Hpc 18, Hcc 21, bp 3, bc 6, cost 1

struct BaDev {
    const uint8_t* img[kMaxKeyframes];  // level-0 images
    int n_kf, n, w, h, m;               // m = 6 (n_kf - 1)
    double K[4];
    double* poses;    // n_kf x 12 (in/out)
    double* poses_c;  // candidates
    double* poses0;   // the poses at the start of the call: every edge's host
                      // (source) pose stays fixed there (the sketch's binary
                      // edge, bundle_adjuster.h:58-100; g2o never moves the
                      // Keyframe's own R_, T_ that srcFrame->Project reads)
    double* pts;      // n x 3 (in/out)
    double* pts_c;
    const int* host;
    uint8_t* active;  // [n][kMaxKeyframes]
    double* E;        // [kMaxKeyframes][kEs][n]
    double* V;        // [6][n]
    double* bp;       // [3][n]
    double* Vinv;     // [9][n]
    double* pcost;    // [n] cost of the current estimate
    double* pcost_c;  // [n] of the candidate
    double* pred;     // [n] points' part of the predicted decrease
    double* S;        // m x m
    double* g;        // m
    double* bc;       // m
    double* udiag;    // m
    double* dc;       // m
    double* ctl;      // [0] mu, [1] nu, [2] accept, [3] vmax
    double* report;   // [iterations][4]
};

__device__ inline void ba_target_uv(const double* T, const double* K, const double* X, double* uv, double* Pc) {
    mat3_vec(T, X, Pc);
    Pc[0] = Pc[0] + T[9];
    Pc[1] = Pc[1] + T[10];
    Pc[2] = Pc[2] + T[11];
    const double k0 = (K[0] * Pc[0] + 0.0 * Pc[1]) + K[2] * Pc[2];
    const double k1 = (0.0 * Pc[0] + K[1] * Pc[1]) + K[3] * Pc[2];
    uv[0] = k0 / Pc[2];
    uv[1] = k1 / Pc[2];
}

__device__ inline void ba_source_uv(const double* T, const double* K, const double* X, double* uv, double* Pc) {
    mat3_vec(T, X, Pc);
    Pc[0] = Pc[0] + T[9];
    Pc[1] = Pc[1] + T[10];
    Pc[2] = Pc[2] + T[11];
    const double x = Pc[0] / Pc[2], y = Pc[1] / Pc[2];
    uv[0] = 1.0 * (x * K[0] + K[2]);
    uv[1] = 1.0 * (y * K[1] + K[3]);
}

__device__ inline void ba_dproj_dX(const double* K, const double* Pc, const double* R, double* D) {
    const double x = Pc[0], y = Pc[1], z = Pc[2], zz = z * z;
    const double a0 = K[0] / z, a2 = -K[0] * x / zz;
    const double b1 = K[1] / z, b2 = -K[1] * y / zz;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        D[c] = a0 * R[c] + a2 * R[6 + c];
        D[3 + c] = b1 * R[3 + c] + b2 * R[6 + c];
    }
}

__device__ inline void ba_dpixel_dxi(const double* K, const double* Pc, double* J) {
    const double x = Pc[0], y = Pc[1], z = Pc[2];
    const double fx = K[0], fy = K[1];
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

__device__ inline void ba_taps(double u, double v, int p, double* fu, double* fv) {
    const int i = (p & 3) - 2, j = (p >> 2) - 2;
    *fu = (double)(float)(u + (double)i);
    *fv = (double)(float)(v + (double)j);
}

// pairwise tree over the 16 lanes of each quarter wave (xor 1, 2, 4, 8)
__device__ inline double tree16(double v) {
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) v = v + __shfl_xor(v, off, 64);
    return v;
}

// ---------------------------------------------------------------- edge set
__global__ __launch_bounds__(256) void ba_active_kernel(BaDev a) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (g < 12 * a.n_kf) a.poses0[g] = a.poses[g];
    const int i = g / kMaxKeyframes, k = g - kMaxKeyframes * (g / kMaxKeyframes);
    if (i >= a.n) return;
    uint8_t on = 0;
    const int hst = a.host[i];
    if (k < a.n_kf && k != hst) {
        const double* X = a.pts + 3 * (size_t)i;
        double us[2], ut[2], Pc[3];
        ba_source_uv(a.poses + 12 * hst, a.K, X, us, Pc);
        ba_target_uv(a.poses + 12 * k, a.K, X, ut, Pc);
        on = 1;
        for (int p = 0; p < kPx; ++p) {
            double u1, v1, u2, v2;
            ba_taps(ut[0], ut[1], p, &u1, &v1);
            ba_taps(us[0], us[1], p, &u2, &v2);
            if (!inside_px(u1, v1, a.w, a.h) || !inside_px(u2, v2, a.w, a.h)) on = 0;
        }
    }
    a.active[(size_t)i * kMaxKeyframes + k] = on;
}

// ---------------------------------------------------------------- linearise / cost
// Wave per point; lanes 16 e + p: pixel p of the point's edge 4 q + e.
// LINEARISE: the 55 sums per edge to E, V / bp / pcost folded; else the
// candidate's cost to pcost_c.
template <bool LINEARISE>
__global__ __launch_bounds__(256) void ba_edges_kernel(BaDev a) {
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= a.n) return;  // wave-uniform
    const int lane = threadIdx.x & 63, e = lane >> 4, p = lane & 15;
    const int hst = a.host[i];
    const double* poses = LINEARISE ? a.poses : a.poses_c;
    const double* X = (LINEARISE ? a.pts : a.pts_c) + 3 * (size_t)i;
    double V[6] = {0, 0, 0, 0, 0, 0}, bp[3] = {0, 0, 0}, cost = 0.0;
    bool first = true;
    for (int q = 0; q < (a.n_kf + 3) / 4; ++q) {
        const int k = 4 * q + e;
        const bool on = k < a.n_kf && a.active[(size_t)i * kMaxKeyframes + k] != 0;
        double sums[kEs];
        {
            const int kk = on ? k : hst;  // a valid pose for inactive lanes
            double us[2], ut[2], Ps[3], Pt[3];
            ba_source_uv(a.poses0 + 12 * hst, a.K, X, us, Ps);
            ba_target_uv(poses + 12 * kk, a.K, X, ut, Pt);
            double u1, v1, u2, v2;
            ba_taps(ut[0], ut[1], p, &u1, &v1);
            ba_taps(us[0], us[1], p, &u2, &v2);
            const uint8_t* Si = a.img[hst];
            const uint8_t* Ti = a.img[kk];
            const double r = sample_px(Si, a.w, a.h, u2, v2) - sample_px(Ti, a.w, a.h, u1, v1);
            if (LINEARISE) {
                double Ds[6], Dt[6], Jx[12];
                ba_dproj_dX(a.K, Ps, a.poses0 + 12 * hst, Ds);
                ba_dproj_dX(a.K, Pt, poses + 12 * kk, Dt);
                ba_dpixel_dxi(a.K, Pt, Jx);
                double gsx, gsy, gtx, gty;
                gradient_px(Si, a.w, a.h, u2, v2, gsx, gsy);
                gradient_px(Ti, a.w, a.h, u1, v1, gtx, gty);
                double Jp[3], Jc[6];
#pragma unroll
                for (int c = 0; c < 3; ++c) Jp[c] = (gsx * Ds[c] + gsy * Ds[3 + c]) - (gtx * Dt[c] + gty * Dt[3 + c]);
#pragma unroll
                for (int c = 0; c < 6; ++c) Jc[c] = -gtx * Jx[c] + -gty * Jx[6 + c];
                int s = 0;
#pragma unroll
                for (int x = 0; x < 3; ++x)
#pragma unroll
                    for (int y = x; y < 3; ++y) sums[s++] = Jp[x] * Jp[y];
#pragma unroll
                for (int x = 0; x < 3; ++x)
#pragma unroll
                    for (int y = 0; y < 6; ++y) sums[s++] = Jp[x] * Jc[y];
#pragma unroll
                for (int x = 0; x < 6; ++x)
#pragma unroll
                    for (int y = x; y < 6; ++y) sums[s++] = Jc[x] * Jc[y];
#pragma unroll
                for (int x = 0; x < 3; ++x) sums[s++] = -Jp[x] * r;
#pragma unroll
                for (int x = 0; x < 6; ++x) sums[s++] = -Jc[x] * r;
                sums[s++] = r * r;
#pragma unroll
                for (int s2 = 0; s2 < kEs; ++s2) sums[s2] = tree16(sums[s2]);
            } else {
                sums[kEs - 1] = tree16(r * r);
            }
        }
        if (LINEARISE && p == 0 && k < a.n_kf) {
#pragma unroll
            for (int s2 = 0; s2 < kEs; ++s2)
                a.E[((size_t)k * kEs + s2) * a.n + i] = on ? sums[s2] : 0.0;
        }
        // fold the point's edges in keyframe order (every lane, uniform)
        for (int ee = 0; ee < 4; ++ee) {
            const int k2 = 4 * q + ee;
            const bool on2 = k2 < a.n_kf && a.active[(size_t)i * kMaxKeyframes + k2] != 0;
            double c2 = __shfl(sums[kEs - 1], 16 * ee, 64);
            if (LINEARISE) {
                double v6[6], b3[3];
#pragma unroll
                for (int s2 = 0; s2 < 6; ++s2) v6[s2] = __shfl(sums[s2], 16 * ee, 64);
#pragma unroll
                for (int s2 = 0; s2 < 3; ++s2) b3[s2] = __shfl(sums[45 + s2], 16 * ee, 64);
                if (on2) {
#pragma unroll
                    for (int s2 = 0; s2 < 6; ++s2) V[s2] = first ? v6[s2] : V[s2] + v6[s2];
#pragma unroll
                    for (int s2 = 0; s2 < 3; ++s2) bp[s2] = first ? b3[s2] : bp[s2] + b3[s2];
                }
            }
            if (on2) {
                cost = first ? c2 : cost + c2;
                first = false;
            }
        }
    }
    if (lane == 0) {
        if (LINEARISE) {
#pragma unroll
            for (int s2 = 0; s2 < 6; ++s2) a.V[(size_t)s2 * a.n + i] = V[s2];
#pragma unroll
            for (int s2 = 0; s2 < 3; ++s2) a.bp[(size_t)s2 * a.n + i] = bp[s2];
            a.pcost[i] = cost;
        } else {
            a.pcost_c[i] = cost;
        }
    }
}

// ---------------------------------------------------------------- mu0
// workgroup per camera-diagonal entry (sum over points), plus the points'
// diagonal maximum in the last workgroup
__global__ __launch_bounds__(256) void ba_udiag_kernel(BaDev a) {
    __shared__ double s_red[4];
    __shared__ double s_mx[256];
    const int b = blockIdx.x;
    if (b < a.m) {
        const int cam = b / 6 + 1, r = b - 6 * (b / 6);
        const int ur = r * 6 - (r * (r - 1)) / 2;
        const double* leaf = a.E + ((size_t)cam * kEs + 24 + ur) * a.n;
        const double s = block_tree_sum(a.n, [&](int i) { return leaf[i]; }, s_red);
        if (threadIdx.x == 0) a.udiag[b] = s;
    } else {
        double mx = 0.0;
        for (int i = threadIdx.x; i < a.n; i += 256) {
            mx = fmax(mx, a.V[i]);
            mx = fmax(mx, a.V[(size_t)3 * a.n + i]);
            mx = fmax(mx, a.V[(size_t)5 * a.n + i]);
        }
        s_mx[threadIdx.x] = mx;
        __syncthreads();
        if (threadIdx.x == 0) {
            double m2 = 0.0;
            for (int t = 0; t < 256; ++t) m2 = fmax(m2, s_mx[t]);
            a.ctl[3] = m2;
        }
    }
}

__global__ void ba_mu0_kernel(BaDev a) {
    if (threadIdx.x != 0) return;
    double mx = 0.0;
    for (int j = 0; j < a.m; ++j) mx = fmax(mx, a.udiag[j]);
    mx = fmax(mx, a.ctl[3]);
    a.ctl[0] = 1e-5 * mx;
    a.ctl[1] = 2.0;
}

// ---------------------------------------------------------------- Schur
__global__ __launch_bounds__(256) void ba_vinv_kernel(BaDev a) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.n) return;
    const double mu = a.ctl[0];
    const double v0 = a.V[i], v1 = a.V[(size_t)a.n + i], v2 = a.V[(size_t)2 * a.n + i],
                 v3 = a.V[(size_t)3 * a.n + i], v4 = a.V[(size_t)4 * a.n + i], v5 = a.V[(size_t)5 * a.n + i];
    const double A = v0 + mu, B = v1, C = v2, D = v3 + mu, E = v4, F = v5 + mu;
    const double c00 = D * F - E * E, c01 = C * E - B * F, c02 = B * E - C * D;
    const double det = (A * c00 + B * c01) + C * c02;
    const double id = 1.0 / det;
    double inv[9];
    inv[0] = c00 * id;
    inv[1] = c01 * id;
    inv[2] = c02 * id;
    inv[3] = c01 * id;
    inv[4] = (A * F - C * C) * id;
    inv[5] = (B * C - A * E) * id;
    inv[6] = c02 * id;
    inv[7] = (B * C - A * E) * id;
    inv[8] = (A * D - B * B) * id;
#pragma unroll
    for (int k = 0; k < 9; ++k) a.Vinv[(size_t)k * a.n + i] = inv[k];
}

__device__ inline double ba_W(const BaDev& a, int i, int cam, int t, int c) {
    return a.E[((size_t)cam * kEs + 6 + 6 * t + c) * a.n + i];
}

__device__ inline double ba_Y(const BaDev& a, int i, int cam, int r, int s) {
    return (ba_W(a, i, cam, 0, r) * a.Vinv[(size_t)s * a.n + i] + ba_W(a, i, cam, 1, r) * a.Vinv[(size_t)(3 + s) * a.n + i]) +
           ba_W(a, i, cam, 2, r) * a.Vinv[(size_t)(6 + s) * a.n + i];
}

// workgroup b: S upper entry (A <= B) for b < m(m+1)/2, then g (m), then bc (m)
__global__ __launch_bounds__(256) void ba_reduce_kernel(BaDev a) {
    __shared__ double s_red[4];
    const int m = a.m, nS = m * (m + 1) / 2;
    int b = blockIdx.x;
    if (b < nS) {
        int A = 0, e = b;
        while (e >= m - A) {
            e -= m - A;
            ++A;
        }
        const int B = A + e;
        const int ca = A / 6 + 1, r = A - 6 * (A / 6), cb = B / 6 + 1, c = B - 6 * (B / 6);
        const int lo = r < c ? r : c, hi = r < c ? c : r;
        const int uidx = 24 + lo * 6 - (lo * (lo - 1)) / 2 + (hi - lo);
        const double s = block_tree_sum(a.n, [&](int i) {
            const double term = (ba_Y(a, i, ca, r, 0) * ba_W(a, i, cb, 0, c) + ba_Y(a, i, ca, r, 1) * ba_W(a, i, cb, 1, c)) +
                                ba_Y(a, i, ca, r, 2) * ba_W(a, i, cb, 2, c);
            const double u = ca == cb ? a.E[((size_t)ca * kEs + uidx) * a.n + i] : 0.0;
            return u - term;
        }, s_red);
        if (threadIdx.x == 0) {
            a.S[(size_t)A * m + B] = s;
            a.S[(size_t)B * m + A] = s;
        }
        return;
    }
    b -= nS;
    if (b < m) {
        const int ca = b / 6 + 1, r = b - 6 * (b / 6);
        const double s = block_tree_sum(a.n, [&](int i) {
            const double bci = a.E[((size_t)ca * kEs + 48 + r) * a.n + i];
            return bci - ((ba_Y(a, i, ca, r, 0) * a.bp[i] + ba_Y(a, i, ca, r, 1) * a.bp[(size_t)a.n + i]) +
                          ba_Y(a, i, ca, r, 2) * a.bp[(size_t)2 * a.n + i]);
        }, s_red);
        if (threadIdx.x == 0) a.g[b] = s;
        return;
    }
    b -= m;
    if (b < m) {
        const int ca = b / 6 + 1, r = b - 6 * (b / 6);
        const double* leaf = a.E + ((size_t)ca * kEs + 48 + r) * a.n;
        const double s = block_tree_sum(a.n, [&](int i) { return leaf[i]; }, s_red);
        if (threadIdx.x == 0) a.bc[b] = s;
    }
}

// ---------------------------------------------------------------- solve
// one wave: LDL^T of S + mu I (lane i computes row i of L), then the
// substitutions on lane 0 (the oracle's loop order throughout)
constexpr int kBaMaxM = 6 * (kMaxKeyframes - 1);

__global__ __launch_bounds__(64) void ba_solve_kernel(BaDev a) {
    __shared__ double L[kBaMaxM][kBaMaxM];
    __shared__ double D[kBaMaxM];
    __shared__ double y[kBaMaxM];
    const int m = a.m, lane = threadIdx.x;
    const double mu = a.ctl[0];
    for (int k = 0; k < m; ++k) {
        double d = a.S[(size_t)k * m + k] + mu;
        for (int j = 0; j < k; ++j) d = d - (L[k][j] * L[k][j]) * D[j];
        if (lane == 0) D[k] = d;
        if (lane > k && lane < m) {
            double s = a.S[(size_t)lane * m + k];
            for (int j = 0; j < k; ++j) s = s - (L[lane][j] * L[k][j]) * D[j];
            L[lane][k] = s / d;
        }
        __syncthreads();
    }
    if (lane == 0) {
        for (int i = 0; i < m; ++i) {
            double s = a.g[i];
            for (int j = 0; j < i; ++j) s = s - L[i][j] * y[j];
            y[i] = s;
        }
        for (int i = m - 1; i >= 0; --i) {
            double s = y[i] / D[i];
            for (int j = i + 1; j < m; ++j) s = s - L[j][i] * a.dc[j];
            a.dc[i] = s;
        }
    }
}

// ---------------------------------------------------------------- update
__global__ __launch_bounds__(256) void ba_points_kernel(BaDev a) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    const double mu = a.ctl[0];
    if (blockIdx.x == 0 && threadIdx.x < a.n_kf) {
        const int k = threadIdx.x;
        double* out = a.poses_c + 12 * k;
        const double* T = a.poses + 12 * k;
        if (k == 0) {
            for (int q = 0; q < 12; ++q) out[q] = T[q];
        } else {
            SE3d t0;
            quat_from_matrix(T, t0.q);
            t0.t[0] = T[9];
            t0.t[1] = T[10];
            t0.t[2] = T[11];
            const SE3d s = se3_mul(se3_exp(a.dc + 6 * (k - 1)), t0);
            quat_to_matrix(s.q, out);
            out[9] = s.t[0];
            out[10] = s.t[1];
            out[11] = s.t[2];
        }
    }
    if (i >= a.n) return;
    const int nf = a.n_kf - 1;
    double q[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) {
        double s = a.bp[(size_t)t * a.n + i];
        for (int c0 = 0; c0 < nf; ++c0) {
            double wd = ba_W(a, i, c0 + 1, t, 0) * a.dc[6 * c0];
            for (int c = 1; c < 6; ++c) wd = wd + ba_W(a, i, c0 + 1, t, c) * a.dc[6 * c0 + c];
            s = s - wd;
        }
        q[t] = s;
    }
    double dp[3];
#pragma unroll
    for (int s = 0; s < 3; ++s)
        dp[s] = (a.Vinv[(size_t)(3 * s) * a.n + i] * q[0] + a.Vinv[(size_t)(3 * s + 1) * a.n + i] * q[1]) +
                a.Vinv[(size_t)(3 * s + 2) * a.n + i] * q[2];
#pragma unroll
    for (int s = 0; s < 3; ++s) a.pts_c[3 * (size_t)i + s] = a.pts[3 * (size_t)i + s] + dp[s];
    const double b0 = a.bp[i], b1 = a.bp[(size_t)a.n + i], b2 = a.bp[(size_t)2 * a.n + i];
    a.pred[i] = (dp[0] * (mu * dp[0] + b0) + dp[1] * (mu * dp[1] + b1)) + dp[2] * (mu * dp[2] + b2);
}

__global__ __launch_bounds__(256) void ba_decide_kernel(BaDev a, int it) {
    __shared__ double s_red[4];
    const double cost_cur = block_tree_sum(a.n, [&](int i) { return a.pcost[i]; }, s_red);
    const double cost_new = block_tree_sum(a.n, [&](int i) { return a.pcost_c[i]; }, s_red);
    const double pred_pts = block_tree_sum(a.n, [&](int i) { return a.pred[i]; }, s_red);
    if (threadIdx.x != 0) return;
    const double mu = a.ctl[0], nu = a.ctl[1];
    double pred_c = 0.0;
    for (int A = 0; A < a.m; ++A) pred_c = pred_c + a.dc[A] * (mu * a.dc[A] + a.bc[A]);
    const double pred = 0.5 * (pred_c + pred_pts);
    const double rho = pred > 0 ? (0.5 * (cost_cur - cost_new)) / pred : -1.0;
    const bool accept = rho > 0;
    if (a.report) {
        a.report[4 * it] = cost_cur;
        a.report[4 * it + 1] = cost_new;
        a.report[4 * it + 2] = mu;
        a.report[4 * it + 3] = accept ? 1.0 : 0.0;
    }
    if (accept) {
        const double t = 2.0 * rho - 1.0;
        a.ctl[0] = mu * fmax(1.0 / 3.0, 1.0 - (t * t) * t);
        a.ctl[1] = 2.0;
    } else {
        a.ctl[0] = mu * nu;
        a.ctl[1] = 2.0 * nu;
    }
    a.ctl[2] = accept ? 1.0 : 0.0;
}

__global__ __launch_bounds__(256) void ba_commit_kernel(BaDev a) {
    if (a.ctl[2] == 0.0) return;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x < 12 * a.n_kf) a.poses[threadIdx.x] = a.poses_c[threadIdx.x];
    if (i < a.n)
        for (int s = 0; s < 3; ++s) a.pts[3 * (size_t)i + s] = a.pts_c[3 * (size_t)i + s];
}

}  // namespace

size_t ba_scratch_bytes(int n) {
    const size_t N = (size_t)(n > 0 ? n : 1);
    return 256 * 40 + N * (kMaxKeyframes + 8 * (kMaxKeyframes * kEs + 6 + 3 + 9 + 3 + 3)) +
           8 * (size_t)kBaMaxM * kBaMaxM + 8 * 8 * kBaMaxM + 8 * 64 + 2 * 8 * 12 * kMaxKeyframes + 256;
}

int launch_photometric_ba(const uint8_t* const* kf_l0, int n_kf, int w, int h, const double K[4], double* poses,
                          double* pts, const int* host, int n, int iterations, void* scratch, double* report,
                          hipStream_t stream) {
    if (n_kf < 2 || n_kf > kMaxKeyframes || n < 1 || iterations < 1) return -1;
    BaDev a{};
    for (int k = 0; k < n_kf; ++k) a.img[k] = kf_l0[k];
    a.n_kf = n_kf;
    a.n = n;
    a.w = w;
    a.h = h;
    a.m = 6 * (n_kf - 1);
    for (int k = 0; k < 4; ++k) a.K[k] = K[k];
    a.poses = poses;
    a.pts = pts;
    a.host = host;
    char* b = (char*)scratch;
    auto take = [&](size_t bytes) {
        char* p = b;
        b += (bytes + 255) & ~(size_t)255;
        return (void*)p;
    };
    const size_t N = (size_t)n;
    a.active = (uint8_t*)take(N * kMaxKeyframes);
    a.E = (double*)take(8 * N * kMaxKeyframes * kEs);
    a.V = (double*)take(8 * N * 6);
    a.bp = (double*)take(8 * N * 3);
    a.Vinv = (double*)take(8 * N * 9);
    a.pcost = (double*)take(8 * N);
    a.pcost_c = (double*)take(8 * N);
    a.pred = (double*)take(8 * N);
    a.pts_c = (double*)take(8 * N * 3);
    a.S = (double*)take(8 * (size_t)kBaMaxM * kBaMaxM);
    a.g = (double*)take(8 * kBaMaxM);
    a.bc = (double*)take(8 * kBaMaxM);
    a.udiag = (double*)take(8 * kBaMaxM);
    a.dc = (double*)take(8 * kBaMaxM);
    a.ctl = (double*)take(8 * 8);
    a.poses_c = (double*)take(8 * 12 * kMaxKeyframes);
    a.poses0 = (double*)take(8 * 12 * kMaxKeyframes);
    a.report = report;
    const int gp = (n + 255) / 256, gw = (n + 3) / 4;
    ba_active_kernel<<<(n * kMaxKeyframes + 255) / 256, 256, 0, stream>>>(a);
    for (int it = 0; it < iterations; ++it) {
        ba_edges_kernel<true><<<gw, 256, 0, stream>>>(a);
        if (it == 0) {
            ba_udiag_kernel<<<a.m + 1, 256, 0, stream>>>(a);
            ba_mu0_kernel<<<1, 64, 0, stream>>>(a);
        }
        ba_vinv_kernel<<<gp, 256, 0, stream>>>(a);
        ba_reduce_kernel<<<a.m * (a.m + 1) / 2 + 2 * a.m, 256, 0, stream>>>(a);
        ba_solve_kernel<<<1, 64, 0, stream>>>(a);
        ba_points_kernel<<<gp, 256, 0, stream>>>(a);
        ba_edges_kernel<false><<<gw, 256, 0, stream>>>(a);
        ba_decide_kernel<<<1, 256, 0, stream>>>(a, it);
        ba_commit_kernel<<<gp, 256, 0, stream>>>(a);
    }
    return 0;
}

}  // namespace viso
