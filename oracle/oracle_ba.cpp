// TEST INFRASTRUCTURE ONLY (see viso_oracle.h) — photometric bundle
// adjustment: the repo's own spec for the BA that the reference sketches in
// include/bundle_adjuster.h:22-106 (g2o, never compiled there; SURVEY.md
// §8(f) row 4).  GPU counterpart: viso_amd/csrc/ba.hip.
//
// Variables: keyframe poses T_k (Tcw; keyframe 0 fixed: the gauge) and map
// points X_i (world).  Point i was created by its host keyframe h(i).
// Edge (i, t), t != h(i) (EdgeDirectProjection, bundle_adjuster.h:58-100):
//   target uv = K (R_t X + t_t) / z (the sketch's K * (R p + t), then / z),
//   source uv = Keyframe::Project(T_h, X);
//   16 residuals, j = -2..1 (outer), i = -2..1 (inner):
//     u1 = (float)(target_u + i), v1 = (float)(target_v + j), u2, v2 likewise
//     r = GetPixelValue(src, u2, v2) - GetPixelValue(tgt, u1, v1);
//   the edge is active when every tap is inside both images at the initial
//   estimate (the sketch's setLevel(1) otherwise); the active set is fixed
//   for the call, later evaluations read 0 outside the level buffer.
// Jacobians (analytic; g2o would differentiate numerically): with g =
// GetGradient at the tap, Jpi(Pc) = [[fx/z, 0, -fx x/z^2], [0, fy/z, -fy y/z^2]],
//   dr/dX = g_s Jpi(T_h X) R_h - g_t Jpi(T_t X) R_t,
//   dr/dxi_t = -g_t dPixeldXi(T_t X)  (src/viso.cpp:640-658; T_t <- exp(xi) T_t,
//   VertexPose::oplusImpl, bundle_adjuster.h:48-53).  The host pose is fixed
//   in the edge, as in the sketch's binary edge: the source projection reads
//   T_h as it was when the call started (srcFrame->Project uses the
//   Keyframe's own R_, T_, which g2o never updates), in the linearisation and
//   in the candidate cost alike.
// Solver: Levenberg-Marquardt as g2o's OptimizationAlgorithmLevenberg
// (bundle_adjuster.h:111-115) with the points marginalised (Schur
// complement, setMarginalized(true)):
//   per edge the 16-pixel sums (pairwise tree) of Hpp, Hpc (= W), Hcc (= U),
//   bp = -sum Jp r, bc = -sum Jc r, cost = sum r^2; per point V = sum over its
//   edges (target keyframe ascending), bp likewise;
//   mu0 = 1e-5 max(diag H); Vinv = (V + mu I)^-1 (cofactors);
//   S_ab = [a == b] sum_i U_ia - sum_i W_ia^T Vinv_i W_ib,
//   g_a = sum_i bc_ia - sum_i W_ia^T Vinv_i bp_i   (sums over points: the
//   canonical tree), (S + mu I) dc = g by LDL^T, dp_i = Vinv_i (bp_i - sum_a
//   W_ia dc_a); candidate T_a' = exp(dc_a) T_a, X_i' = X_i + dp_i;
//   rho = (F - F') / (0.5 (dc.(mu dc + bc) + sum_i dp_i.(mu dp_i + bp_i))),
//   F = 0.5 sum r^2; rho > 0: accept, mu *= max(1/3, 1 - (2 rho - 1)^3),
//   nu = 2; else mu *= nu, nu *= 2.  A fixed number of iterations.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "oracle_common.hpp"
#include "oracle_se3.hpp"
#include "viso_oracle.h"

using namespace oracle;

namespace {

constexpr int kBaPx = 16;
constexpr int kBaEdgeSums = 55;  // Hpp 6, Hpc 18, Hcc 21, bp 3, bc 6, cost 1

struct BaProblem {
    int w, h, n_kf, n;
    double K[4];
    const uint8_t* const* img;
    const int32_t* host;
};

// target projection as the sketch: K * Pc, then / z
inline void target_uv(const double* T, const double K[4], const double* X, double* uv, double* Pc) {
    mat3_vec(T, X, Pc);
    Pc[0] = Pc[0] + T[9];
    Pc[1] = Pc[1] + T[10];
    Pc[2] = Pc[2] + T[11];
    const double k0 = (K[0] * Pc[0] + 0.0 * Pc[1]) + K[2] * Pc[2];
    const double k1 = (0.0 * Pc[0] + K[1] * Pc[1]) + K[3] * Pc[2];
    uv[0] = k0 / Pc[2];
    uv[1] = k1 / Pc[2];
}

// Keyframe::Project at level 0, keeping the camera point
inline void source_uv(const double* T, const double K[4], const double* X, double* uv, double* Pc) {
    mat3_vec(T, X, Pc);
    Pc[0] = Pc[0] + T[9];
    Pc[1] = Pc[1] + T[10];
    Pc[2] = Pc[2] + T[11];
    const double x = Pc[0] / Pc[2], y = Pc[1] / Pc[2];
    uv[0] = 1.0 * (x * K[0] + K[2]);
    uv[1] = 1.0 * (y * K[1] + K[3]);
}

// d(u, v)/dX = Jpi(Pc) R (2 x 3, row-major)
inline void dproj_dX(const double K[4], const double* Pc, const double* R, double* D) {
    const double x = Pc[0], y = Pc[1], z = Pc[2], zz = z * z;
    const double a0 = K[0] / z, a2 = -K[0] * x / zz;
    const double b1 = K[1] / z, b2 = -K[1] * y / zz;
    for (int c = 0; c < 3; ++c) {
        D[c] = a0 * R[c] + a2 * R[6 + c];
        D[3 + c] = b1 * R[3 + c] + b2 * R[6 + c];
    }
}

// the 2x6 dPixeldXi at level 0 (src/viso.cpp:640-658)
inline void dpixel_dxi(const double K[4], const double* Pc, double* J) {
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

inline double tree16(const double* v) {
    double t[16];
    for (int k = 0; k < 16; ++k) t[k] = v[k];
    for (int s = 1; s < 16; s <<= 1)
        for (int k = 0; k < 16; k += 2 * s) t[k] = t[k] + t[k + s];
    return t[0];
}

// pixel (j, i) -> residual index (j + 2) * 4 + (i + 2)
inline void taps(double u, double v, int p, float* fu, float* fv) {
    const int i = (p & 3) - 2, j = (p >> 2) - 2;
    *fu = (float)(u + (double)i);
    *fv = (float)(v + (double)j);
}

bool edge_active(const BaProblem& P, const double* poses, const double* X, int host, int tgt) {
    double us[2], ut[2], Pc[3];
    source_uv(poses + 12 * host, P.K, X, us, Pc);  // at the call's start: host0 == poses
    target_uv(poses + 12 * tgt, P.K, X, ut, Pc);
    for (int p = 0; p < kBaPx; ++p) {
        float u1, v1, u2, v2;
        taps(ut[0], ut[1], p, &u1, &v1);
        taps(us[0], us[1], p, &u2, &v2);
        if (!is_inside(u1, v1, P.w, P.h) || !is_inside(u2, v2, P.w, P.h)) return false;
    }
    return true;
}

// the 55 sums of edge (X, host, tgt) at the given estimates (host0: the
// fixed host poses)
void edge_sums(const BaProblem& P, const double* host0, const double* poses, const double* X, int host, int tgt,
               double* out) {
    double us[2], ut[2], Ps[3], Pt[3];
    source_uv(host0 + 12 * host, P.K, X, us, Ps);
    target_uv(poses + 12 * tgt, P.K, X, ut, Pt);
    double Ds[6], Dt[6], Jx[12];
    dproj_dX(P.K, Ps, host0 + 12 * host, Ds);
    dproj_dX(P.K, Pt, poses + 12 * tgt, Dt);
    dpixel_dxi(P.K, Pt, Jx);
    double leaf[kBaEdgeSums][kBaPx];
    const uint8_t* S = P.img[host];
    const uint8_t* T = P.img[tgt];
    for (int p = 0; p < kBaPx; ++p) {
        float u1, v1, u2, v2;
        taps(ut[0], ut[1], p, &u1, &v1);
        taps(us[0], us[1], p, &u2, &v2);
        const double r = sample(S, P.w, P.h, u2, v2) - sample(T, P.w, P.h, u1, v1);
        double gsx, gsy, gtx, gty;
        gradient(S, P.w, P.h, u2, v2, gsx, gsy);
        gradient(T, P.w, P.h, u1, v1, gtx, gty);
        double Jp[3], Jc[6];
        for (int c = 0; c < 3; ++c) Jp[c] = (gsx * Ds[c] + gsy * Ds[3 + c]) - (gtx * Dt[c] + gty * Dt[3 + c]);
        for (int c = 0; c < 6; ++c) Jc[c] = -gtx * Jx[c] + -gty * Jx[6 + c];
        int e = 0;
        for (int a = 0; a < 3; ++a)
            for (int b = a; b < 3; ++b) leaf[e++][p] = Jp[a] * Jp[b];
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 6; ++b) leaf[e++][p] = Jp[a] * Jc[b];
        for (int a = 0; a < 6; ++a)
            for (int b = a; b < 6; ++b) leaf[e++][p] = Jc[a] * Jc[b];
        for (int a = 0; a < 3; ++a) leaf[e++][p] = -Jp[a] * r;
        for (int a = 0; a < 6; ++a) leaf[e++][p] = -Jc[a] * r;
        leaf[e++][p] = r * r;
    }
    for (int k = 0; k < kBaEdgeSums; ++k) out[k] = tree16(leaf[k]);
}

double edge_cost(const BaProblem& P, const double* host0, const double* poses, const double* X, int host, int tgt) {
    double us[2], ut[2], Pc[3];
    source_uv(host0 + 12 * host, P.K, X, us, Pc);
    target_uv(poses + 12 * tgt, P.K, X, ut, Pc);
    double leaf[kBaPx];
    for (int p = 0; p < kBaPx; ++p) {
        float u1, v1, u2, v2;
        taps(ut[0], ut[1], p, &u1, &v1);
        taps(us[0], us[1], p, &u2, &v2);
        const double r = sample(P.img[host], P.w, P.h, u2, v2) - sample(P.img[tgt], P.w, P.h, u1, v1);
        leaf[p] = r * r;
    }
    return tree16(leaf);
}

// (V + mu I)^-1 of a symmetric 3x3 given by its upper triangle (cofactors)
void inv3_sym(const double* v6, double mu, double* inv) {
    const double a = v6[0] + mu, b = v6[1], c = v6[2], d = v6[3] + mu, e = v6[4], f = v6[5] + mu;
    const double c00 = d * f - e * e, c01 = c * e - b * f, c02 = b * e - c * d;
    const double det = (a * c00 + b * c01) + c * c02;
    const double id = 1.0 / det;
    inv[0] = c00 * id;
    inv[1] = c01 * id;
    inv[2] = c02 * id;
    inv[3] = c01 * id;
    inv[4] = (a * f - c * c) * id;
    inv[5] = (b * c - a * e) * id;
    inv[6] = c02 * id;
    inv[7] = (b * c - a * e) * id;
    inv[8] = (a * d - b * b) * id;
}

}  // namespace

extern "C" {

// Photometric BA (spec above).  kf_img: n_kf level-0 images (w x h);
// kf_poses: n_kf x 12 (in/out; keyframe 0 fixed); points: n x 3 (in/out);
// host: n keyframe indices; report (may be null): per iteration [cost before,
// cost of the candidate, mu, accepted] (cost = sum r^2 over the active edges);
// returns the number of active edges.
int oracle_photometric_ba(const uint8_t* const* kf_img, int n_kf, int w, int h, const double K[4], double* kf_poses,
                          double* points, const int32_t* host, int n, int iterations, double* report) {
    BaProblem P{w, h, n_kf, n, {K[0], K[1], K[2], K[3]}, kf_img, host};
    const int nf = n_kf - 1;  // free cameras 1..n_kf-1
    const int m = 6 * nf;
    if (nf < 1 || n < 1) return 0;
    std::vector<uint8_t> active((size_t)n * n_kf, 0);
    int n_active = 0;
    for (int i = 0; i < n; ++i)
        for (int k = 0; k < n_kf; ++k)
            if (k != host[i] && edge_active(P, kf_poses, points + 3 * i, host[i], k)) {
                active[(size_t)i * n_kf + k] = 1;
                ++n_active;
            }
    double mu = -1.0, nu = 2.0;
    std::vector<double> E((size_t)n * n_kf * kBaEdgeSums), V((size_t)n * 6), bp((size_t)n * 3), leaf((size_t)n);
    std::vector<double> poses_c((size_t)12 * n_kf), pts_c((size_t)3 * n);
    const std::vector<double> host0(kf_poses, kf_poses + (size_t)12 * n_kf);
    for (int it = 0; it < iterations; ++it) {
        // linearise
        double cost_cur_pts_dummy = 0;
        (void)cost_cur_pts_dummy;
        std::vector<double> pcost((size_t)n, 0.0);
        for (int i = 0; i < n; ++i) {
            bool first = true;
            for (int k = 0; k < n_kf; ++k) {
                double* e = &E[((size_t)i * n_kf + k) * kBaEdgeSums];
                if (!active[(size_t)i * n_kf + k]) {
                    for (int q = 0; q < kBaEdgeSums; ++q) e[q] = 0.0;
                    continue;
                }
                edge_sums(P, host0.data(), kf_poses, points + 3 * i, host[i], k, e);
                for (int q = 0; q < 6; ++q) V[6 * (size_t)i + q] = first ? e[q] : V[6 * (size_t)i + q] + e[q];
                for (int q = 0; q < 3; ++q) bp[3 * (size_t)i + q] = first ? e[45 + q] : bp[3 * (size_t)i + q] + e[45 + q];
                pcost[(size_t)i] = first ? e[54] : pcost[(size_t)i] + e[54];
                first = false;
            }
            if (first) {
                for (int q = 0; q < 6; ++q) V[6 * (size_t)i + q] = 0.0;
                for (int q = 0; q < 3; ++q) bp[3 * (size_t)i + q] = 0.0;
            }
        }
        const double cost_cur = tree_sum(pcost.data(), n);
        if (mu < 0) {
            // mu0 = 1e-5 max diag of the full Hessian
            double mx = 0.0;
            for (int a = 0; a < nf; ++a)
                for (int r = 0; r < 6; ++r) {
                    const int ur = r * 6 - (r * (r - 1)) / 2;  // upper index of (r, r)
                    for (int i = 0; i < n; ++i) leaf[(size_t)i] = E[((size_t)i * n_kf + a + 1) * kBaEdgeSums + 24 + ur];
                    mx = std::max(mx, tree_sum(leaf.data(), n));
                }
            for (int i = 0; i < n; ++i) {
                mx = std::max(mx, V[6 * (size_t)i]);
                mx = std::max(mx, V[6 * (size_t)i + 3]);
                mx = std::max(mx, V[6 * (size_t)i + 5]);
            }
            mu = 1e-5 * mx;
        }
        // reduced camera system
        std::vector<double> Vinv((size_t)n * 9);
        for (int i = 0; i < n; ++i) inv3_sym(&V[6 * (size_t)i], mu, &Vinv[9 * (size_t)i]);
        auto W = [&](int i, int a, int t, int c) {  // Hpc of edge (i, camera a + 1): row t, column c
            return E[((size_t)i * n_kf + a + 1) * kBaEdgeSums + 6 + 6 * t + c];
        };
        auto U = [&](int i, int a, int r, int c) {
            const int lo = std::min(r, c), hi = std::max(r, c);
            return E[((size_t)i * n_kf + a + 1) * kBaEdgeSums + 24 + lo * 6 - (lo * (lo - 1)) / 2 + (hi - lo)];
        };
        auto Y = [&](int i, int a, int r, int s) {
            const double* Vi = &Vinv[9 * (size_t)i];
            return (W(i, a, 0, r) * Vi[s] + W(i, a, 1, r) * Vi[3 + s]) + W(i, a, 2, r) * Vi[6 + s];
        };
        std::vector<double> S((size_t)m * m), g((size_t)m), bc((size_t)m);
        for (int A = 0; A < m; ++A)
            for (int B = A; B < m; ++B) {
                const int a = A / 6, r = A % 6, b = B / 6, c = B % 6;
                for (int i = 0; i < n; ++i) {
                    const double term = (Y(i, a, r, 0) * W(i, b, 0, c) + Y(i, a, r, 1) * W(i, b, 1, c)) +
                                        Y(i, a, r, 2) * W(i, b, 2, c);
                    leaf[(size_t)i] = (a == b ? U(i, a, r, c) : 0.0) - term;
                }
                S[(size_t)A * m + B] = S[(size_t)B * m + A] = tree_sum(leaf.data(), n);
            }
        for (int A = 0; A < m; ++A) {
            const int a = A / 6, r = A % 6;
            for (int i = 0; i < n; ++i) {
                const double* b3 = &bp[3 * (size_t)i];
                const double bci = E[((size_t)i * n_kf + a + 1) * kBaEdgeSums + 48 + r];
                leaf[(size_t)i] = bci - ((Y(i, a, r, 0) * b3[0] + Y(i, a, r, 1) * b3[1]) + Y(i, a, r, 2) * b3[2]);
            }
            g[(size_t)A] = tree_sum(leaf.data(), n);
            for (int i = 0; i < n; ++i) leaf[(size_t)i] = E[((size_t)i * n_kf + a + 1) * kBaEdgeSums + 48 + r];
            bc[(size_t)A] = tree_sum(leaf.data(), n);
        }
        // (S + mu I) dc = g by LDL^T
        std::vector<double> L((size_t)m * m, 0.0), D((size_t)m), dc((size_t)m), y((size_t)m);
        for (int k = 0; k < m; ++k) {
            double d = S[(size_t)k * m + k] + mu;
            for (int j = 0; j < k; ++j) d = d - (L[(size_t)k * m + j] * L[(size_t)k * m + j]) * D[(size_t)j];
            D[(size_t)k] = d;
            for (int i = k + 1; i < m; ++i) {
                double s = S[(size_t)i * m + k];
                for (int j = 0; j < k; ++j) s = s - (L[(size_t)i * m + j] * L[(size_t)k * m + j]) * D[(size_t)j];
                L[(size_t)i * m + k] = s / d;
            }
        }
        for (int i = 0; i < m; ++i) {
            double s = g[(size_t)i];
            for (int j = 0; j < i; ++j) s = s - L[(size_t)i * m + j] * y[(size_t)j];
            y[(size_t)i] = s;
        }
        for (int i = m - 1; i >= 0; --i) {
            double s = y[(size_t)i] / D[(size_t)i];
            for (int j = i + 1; j < m; ++j) s = s - L[(size_t)j * m + i] * dc[(size_t)j];
            dc[(size_t)i] = s;
        }
        // points, candidate estimates, predicted decrease
        std::vector<double> pred_pts((size_t)n);
        for (int i = 0; i < n; ++i) {
            double q[3];
            for (int t = 0; t < 3; ++t) {
                double s = bp[3 * (size_t)i + t];
                for (int a = 0; a < nf; ++a) {
                    double wd = W(i, a, t, 0) * dc[(size_t)6 * a];
                    for (int c = 1; c < 6; ++c) wd = wd + W(i, a, t, c) * dc[(size_t)6 * a + c];
                    s = s - wd;
                }
                q[t] = s;
            }
            const double* Vi = &Vinv[9 * (size_t)i];
            double dp[3];
            for (int s = 0; s < 3; ++s) dp[s] = (Vi[3 * s] * q[0] + Vi[3 * s + 1] * q[1]) + Vi[3 * s + 2] * q[2];
            for (int s = 0; s < 3; ++s) pts_c[3 * (size_t)i + s] = points[3 * (size_t)i + s] + dp[s];
            const double* b3 = &bp[3 * (size_t)i];
            pred_pts[(size_t)i] = ((dp[0] * (mu * dp[0] + b3[0]) + dp[1] * (mu * dp[1] + b3[1])) +
                                   dp[2] * (mu * dp[2] + b3[2]));
        }
        double pred_c = 0.0;
        for (int A = 0; A < m; ++A) pred_c = pred_c + dc[(size_t)A] * (mu * dc[(size_t)A] + bc[(size_t)A]);
        const double pred = 0.5 * (pred_c + tree_sum(pred_pts.data(), n));
        std::memcpy(poses_c.data(), kf_poses, sizeof(double) * 12 * n_kf);
        for (int a = 0; a < nf; ++a) {
            const double* T = kf_poses + 12 * (a + 1);
            SE3 s = se3_mul(se3_exp(&dc[(size_t)6 * a]), se3_from_Rt(T, T + 9));
            quat_to_matrix(s.q, &poses_c[(size_t)12 * (a + 1)]);
            for (int k = 0; k < 3; ++k) poses_c[(size_t)12 * (a + 1) + 9 + k] = s.t[k];
        }
        // candidate cost
        for (int i = 0; i < n; ++i) {
            double c = 0.0;
            bool first = true;
            for (int k = 0; k < n_kf; ++k) {
                if (!active[(size_t)i * n_kf + k]) continue;
                const double e = edge_cost(P, host0.data(), poses_c.data(), &pts_c[3 * (size_t)i], host[i], k);
                c = first ? e : c + e;
                first = false;
            }
            pcost[(size_t)i] = c;
        }
        const double cost_new = tree_sum(pcost.data(), n);
        const double rho = pred > 0 ? (0.5 * (cost_cur - cost_new)) / pred : -1.0;
        const bool accept = rho > 0;
        if (report) {
            report[4 * it] = cost_cur;
            report[4 * it + 1] = cost_new;
            report[4 * it + 2] = mu;
            report[4 * it + 3] = accept ? 1.0 : 0.0;
        }
        if (accept) {
            std::memcpy(kf_poses, poses_c.data(), sizeof(double) * 12 * n_kf);
            std::memcpy(points, pts_c.data(), sizeof(double) * 3 * n);
            const double t = 2.0 * rho - 1.0;
            mu = mu * std::max(1.0 / 3.0, 1.0 - (t * t) * t);
            nu = 2.0;
        } else {
            mu = mu * nu;
            nu = 2.0 * nu;
        }
    }
    return n_active;
}

}  // extern "C"
