// TEST INFRASTRUCTURE ONLY — CPU restatement of the repo's north-star stereo
// visual odometry spec (SVO; include/viso/viso_svo.h), the
// checker of viso_amd/csrc/svo.hip.  The reference has no stereo path
// ("North_star stages with NO reference counterpart"), so this
// file IS the spec: "parity unpinned vs reference".  It is pinned instead by
// known answers (tests/test_svo.py: single-blob / checkerboard responses,
// hand-computed descriptors) and by recovering the synthetic renderer's
// ground-truth motion.
//
// Numerics: integers for filters, NMS, descriptors, SAD and matching (exact);
// fp64 for the pose with +,-,*,/ only (no transcendental functions: the
// rotation update is the Cayley map), every expression in the order written
// here, compiled with -ffp-contract=off, and every sum over matches the
// canonical pairwise tree (oracle_common.hpp tree_sum), so the GPU result is
// bit-identical.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../include/viso/viso_svo.h"
#include "oracle_common.hpp"

namespace {

using oracle::mix64;
using oracle::tree_sum;

struct Feat {
    int u, v, c;
    uint8_t d[VISO_SVO_DESC_BYTES];
};

// 5x5 blob mask: outer ring -1, inner ring +1, centre +8 (sums to 0).
int blob5(const uint8_t* I, int w, int x, int y) {
    int s = 0;
    for (int dy = -2; dy <= 2; ++dy)
        for (int dx = -2; dx <= 2; ++dx) {
            const int a = I[(size_t)(y + dy) * w + x + dx];
            const int r = std::max(std::abs(dx), std::abs(dy));
            s += r == 2 ? -a : (r == 1 ? a : 8 * a);
        }
    return s;
}

// 5x5 checkerboard corner mask: quadrants TL/BR -1, TR/BL +1, centre row
// and column 0 (sums to 0).
int corner5(const uint8_t* I, int w, int x, int y) {
    int s = 0;
    for (int dy = -2; dy <= 2; ++dy)
        for (int dx = -2; dx <= 2; ++dx) {
            if (dx == 0 || dy == 0) continue;
            const int a = I[(size_t)(y + dy) * w + x + dx];
            s += ((dx < 0) == (dy < 0)) ? -a : a;
        }
    return s;
}

// 3x3 Sobel, quantised to u8: (d >> 3) + 128 (arithmetic shift; |d| <= 1020).
uint8_t sobel_du(const uint8_t* I, int w, int x, int y) {
    auto p = [&](int dx, int dy) { return (int)I[(size_t)(y + dy) * w + x + dx]; };
    const int d = (p(1, -1) + 2 * p(1, 0) + p(1, 1)) - (p(-1, -1) + 2 * p(-1, 0) + p(-1, 1));
    return (uint8_t)((d >> 3) + 128);
}
uint8_t sobel_dv(const uint8_t* I, int w, int x, int y) {
    auto p = [&](int dx, int dy) { return (int)I[(size_t)(y + dy) * w + x + dx]; };
    const int d = (p(-1, 1) + 2 * p(0, 1) + p(1, 1)) - (p(-1, -1) + 2 * p(0, -1) + p(1, -1));
    return (uint8_t)((d >> 3) + 128);
}

// descriptor sample offsets (dx, dy): bytes 0..15 = du, 16..31 = dv
const int kP16[16][2] = {{-5, -1}, {-5, 1}, {-3, -3}, {-3, 3}, {-1, -5}, {-1, 5}, {-1, -1}, {-1, 1},
                         {1, -1},  {1, 1},  {1, -5},  {1, 5},  {3, -3},  {3, 3},  {5, -1},  {5, 1}};

std::vector<Feat> features(const uint8_t* I, int w, int h, const viso_svo_params& p) {
    std::vector<int> B((size_t)w * h, 0), C((size_t)w * h, 0);
    for (int y = 2; y < h - 2; ++y)
        for (int x = 2; x < w - 2; ++x) {
            B[(size_t)y * w + x] = blob5(I, w, x, y);
            C[(size_t)y * w + x] = corner5(I, w, x, y);
        }
    auto resp = [&](int k, int x, int y) {
        const int b = k < 2 ? B[(size_t)y * w + x] : C[(size_t)y * w + x];
        return (k & 1) ? -b : b;
    };
    const int n = p.nms_n, m = p.margin;
    std::vector<Feat> out;
    for (int y = m; y < h - m; ++y)
        for (int x = m; x < w - m; ++x)
            for (int k = 0; k < 4; ++k) {
                const int r = resp(k, x, y);
                if (r <= p.nms_tau) continue;
                bool mx = true;
                for (int dy = -n; dy <= n && mx; ++dy)
                    for (int dx = -n; dx <= n; ++dx) {
                        if (dx == 0 && dy == 0) continue;
                        const int qx = x + dx, qy = y + dy;
                        if (qx < 2 || qx >= w - 2 || qy < 2 || qy >= h - 2) continue;
                        if (resp(k, qx, qy) >= r) {
                            mx = false;
                            break;
                        }
                    }
                if (!mx) continue;
                Feat f;
                f.u = x;
                f.v = y;
                f.c = k;
                for (int j = 0; j < 16; ++j) {
                    f.d[j] = sobel_du(I, w, x + kP16[j][0], y + kP16[j][1]);
                    f.d[16 + j] = sobel_dv(I, w, x + kP16[j][0], y + kP16[j][1]);
                }
                out.push_back(f);
            }
    return out;
}

int sad32(const uint8_t* a, const uint8_t* b) {
    int s = 0;
    for (int i = 0; i < VISO_SVO_DESC_BYTES; ++i) s += std::abs((int)a[i] - (int)b[i]);
    return s;
}

struct FeatSet {
    const int32_t *u, *v, *c;
    const uint8_t* d;
    int n;
    std::vector<int> row0;  // first feature index of each row (size h + 1)
    void index(int h) {
        row0.assign((size_t)h + 2, n);
        for (int i = n - 1; i >= 0; --i) row0[(size_t)v[i]] = i;
        for (int y = h; y >= 0; --y) row0[(size_t)y] = std::min(row0[(size_t)y], row0[(size_t)y + 1]);
    }
};

// candidates whose SAD the spec evaluates (the matching pass's algorithmic
// work: 32 byte differences each; oracle_svo_sad_evals, for the bench's
// VALU-fraction figure of svo_circle_kernel)
unsigned long long g_sad_evals = 0;

// best candidate of `dst` for a query (u, v, class, descriptor): rows
// [v - dv, v + dv], u - du_hi <= u' <= u - du_lo; min SAD, ties -> lowest index
int best_match(const FeatSet& dst, int h, int u, int v, int c, const uint8_t* d, int du_lo,
               int du_hi, int dv) {
    int best = -1, best_sad = INT_MAX;
    for (int y = std::max(v - dv, 0); y <= std::min(v + dv, h - 1); ++y)
        for (int j = dst.row0[(size_t)y]; j < dst.row0[(size_t)y + 1]; ++j) {
            if (dst.c[j] != c) continue;
            const int dd = u - dst.u[j];
            if (dd < du_lo || dd > du_hi) continue;
            const int s = sad32(d, dst.d + (size_t)j * VISO_SVO_DESC_BYTES);
            ++g_sad_evals;
            if (s < best_sad || (s == best_sad && j < best)) {
                best_sad = s;
                best = j;
            }
        }
    return best;
}

// ---------------------------------------------------------------- pose
struct Obs {
    double X, Y, Z;         // point in camera t-1
    double uL, vL, uR, vR;  // observations in the current pair
    const double* E;        // rig: extrinsic of the match's camera (rig -> camera), else null
    double Xr[3];           // rig: the point in the rig frame t-1, E^-1 (X, Y, Z)
};

Obs make_obs(const int32_t* m, const viso_svo_params& p) {
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
    o.Xr[0] = o.Xr[1] = o.Xr[2] = 0.0;
    return o;
}

// Multi-camera rig (BASELINE.json configs[4]): camera c sees the rig frame
// through its extrinsic E_c = (Re, te), P_c = Re P_rig + te (12 doubles, Re
// row-major).  The motion (R, t) is the rig's; a match of camera c predicts
// Q = R Xr + t (rig frame t), P = Re Q + te (camera c, t).
Obs make_obs_rig(const int32_t* m, const double* E, const viso_svo_params& p) {
    Obs o = make_obs(m, p);
    o.E = E;
    const double d0 = o.X - E[9], d1 = o.Y - E[10], d2 = o.Z - E[11];
    for (int k = 0; k < 3; ++k) o.Xr[k] = ((E[k] * d0 + E[3 + k] * d1) + E[6 + k] * d2);
    return o;
}

void transform(const double* R, const double* t, const Obs& o, double* P) {
    P[0] = ((R[0] * o.X + R[1] * o.Y) + R[2] * o.Z) + t[0];
    P[1] = ((R[3] * o.X + R[4] * o.Y) + R[5] * o.Z) + t[1];
    P[2] = ((R[6] * o.X + R[7] * o.Y) + R[8] * o.Z) + t[2];
}

// the 4 residuals (uL, vL, uR, vR) and their Jacobian rows w.r.t. the left
// perturbation (dw, dt): P' -> P' + dw x P' + dt
void residual_rows(const double* P, const Obs& o, const viso_svo_params& p, double e[4], double J[4][6]) {
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

// rig form of transform + residual_rows: Q = R Xr + t, P = Re Q + te; the
// residual gradients g (w.r.t. P) are taken to the rig frame, g' = Re^T g,
// and J = [Q x g', g'] (left perturbation of the rig motion)
void rig_point(const double* R, const double* t, const Obs& o, double* Q, double* P) {
    Q[0] = ((R[0] * o.Xr[0] + R[1] * o.Xr[1]) + R[2] * o.Xr[2]) + t[0];
    Q[1] = ((R[3] * o.Xr[0] + R[4] * o.Xr[1]) + R[5] * o.Xr[2]) + t[1];
    Q[2] = ((R[6] * o.Xr[0] + R[7] * o.Xr[1]) + R[8] * o.Xr[2]) + t[2];
    const double* E = o.E;
    P[0] = ((E[0] * Q[0] + E[1] * Q[1]) + E[2] * Q[2]) + E[9];
    P[1] = ((E[3] * Q[0] + E[4] * Q[1]) + E[5] * Q[2]) + E[10];
    P[2] = ((E[6] * Q[0] + E[7] * Q[1]) + E[8] * Q[2]) + E[11];
}

void residual_rows_rig(const double* P, const double* Q, const Obs& o, const viso_svo_params& p, double e[4],
                       double J[4][6]) {
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

// residuals + Jacobian of one match under (R, t), mono or rig; P = camera point
void match_rows(const double* R, const double* t, const Obs& o, const viso_svo_params& p, double* P, double e[4],
                double J[4][6]) {
    if (o.E) {
        double Q[3];
        rig_point(R, t, o, Q, P);
        residual_rows_rig(P, Q, o, p, e, J);
    } else {
        transform(R, t, o, P);
        residual_rows(P, o, p, e, J);
    }
}

// the 28 per-match sums (21 upper-triangle J^T J row-major, 6 J^T e, e^T e),
// each ((row0 + row1) + row2) + row3
void match_sums(const double e[4], const double J[4][6], double* s28) {
    int k = 0;
    for (int a = 0; a < 6; ++a)
        for (int b = a; b < 6; ++b, ++k)
            s28[k] = ((J[0][a] * J[0][b] + J[1][a] * J[1][b]) + J[2][a] * J[2][b]) + J[3][a] * J[3][b];
    for (int a = 0; a < 6; ++a, ++k) s28[k] = ((J[0][a] * e[0] + J[1][a] * e[1]) + J[2][a] * e[2]) + J[3][a] * e[3];
    s28[27] = ((e[0] * e[0] + e[1] * e[1]) + e[2] * e[2]) + e[3] * e[3];
}

// A x = g by LDL^T (A = J^T J is symmetric positive definite unless the
// samples are degenerate): no pivoting, one division per column; fails if a
// pivot D_j is not > 1e-12.  Every sum runs in ascending k.
bool solve6(const double* S, double* x) {
    double A[6][6], g[6], L[6][6] = {}, D[6], inv[6];
    int k = 0;
    for (int a = 0; a < 6; ++a)
        for (int b = a; b < 6; ++b, ++k) A[a][b] = A[b][a] = S[k];
    for (int a = 0; a < 6; ++a) g[a] = S[21 + a];
    for (int j = 0; j < 6; ++j) {
        double d = A[j][j];
        for (int q = 0; q < j; ++q) d = d - (L[j][q] * L[j][q]) * D[q];
        if (!(d > 1e-12)) return false;
        D[j] = d;
        inv[j] = 1.0 / d;
        for (int i = j + 1; i < 6; ++i) {
            double s = A[i][j];
            for (int q = 0; q < j; ++q) s = s - (L[i][q] * L[j][q]) * D[q];
            L[i][j] = s * inv[j];
        }
    }
    double z[6];
    for (int i = 0; i < 6; ++i) {
        double s = g[i];
        for (int q = 0; q < i; ++q) s = s - L[i][q] * z[q];
        z[i] = s;
    }
    for (int i = 5; i >= 0; --i) {
        double s = z[i] * inv[i];
        for (int q = i + 1; q < 6; ++q) s = s - L[q][i] * x[q];
        x[i] = s;
    }
    return true;
}

void mat3_mul(const double* A, const double* B, double* C) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            C[3 * i + j] = (A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j]) + A[3 * i + 2] * B[6 + j];
}

// R <- Q R, t <- Q t + dt with Q = Cayley(dw) = I + c (W + W^2 / 2),
// c = 1 / (1 + |dw|^2 / 4), W = [dw]x
void apply_update(const double* x, double* R, double* t) {
    const double w2 = (x[0] * x[0] + x[1] * x[1]) + x[2] * x[2];
    const double c = 1.0 / (1.0 + 0.25 * w2);
    const double W[9] = {0.0, -x[2], x[1], x[2], 0.0, -x[0], -x[1], x[0], 0.0};
    double W2[9], Q[9], Rn[9];
    mat3_mul(W, W, W2);
    for (int i = 0; i < 9; ++i) Q[i] = ((i % 4 == 0) ? 1.0 : 0.0) + c * (W[i] + 0.5 * W2[i]);
    mat3_mul(Q, R, Rn);
    double tn[3];
    for (int i = 0; i < 3; ++i) tn[i] = ((Q[3 * i] * t[0] + Q[3 * i + 1] * t[1]) + Q[3 * i + 2] * t[2]) + x[3 + i];
    std::memcpy(R, Rn, sizeof(Rn));
    std::memcpy(t, tn, sizeof(tn));
}

// Gauss-Newton over the selected matches (sel[i] != 0); sums are trees over
// all n leaves (unselected = 0).  Returns false if a system is singular.
bool gauss_newton(const std::vector<Obs>& obs, const std::vector<uint8_t>& sel,
                  const viso_svo_params& p, double* R, double* t) {
    const int n = (int)obs.size();
    std::vector<double> leaf((size_t)n * 28);
    std::vector<double> col((size_t)n);
    for (int it = 0; it < p.gn_iters; ++it) {
        for (int i = 0; i < n; ++i) {
            double* s = &leaf[(size_t)i * 28];
            if (!sel[(size_t)i]) {
                for (int k = 0; k < 28; ++k) s[k] = 0.0;
                continue;
            }
            double P[3], e[4], J[4][6];
            match_rows(R, t, obs[(size_t)i], p, P, e, J);
            match_sums(e, J, s);
        }
        double S[28], x[6];
        for (int k = 0; k < 28; ++k) {
            for (int i = 0; i < n; ++i) col[(size_t)i] = leaf[(size_t)i * 28 + k];
            S[k] = tree_sum(col.data(), n);
        }
        if (!solve6(S, x)) return false;
        apply_update(x, R, t);
        double mx = 0.0;
        for (int k = 0; k < 6; ++k) mx = std::max(mx, std::fabs(x[k]));
        if (mx < p.gn_eps) break;
    }
    return true;
}

bool is_inlier(const double* R, const double* t, const Obs& o, const viso_svo_params& p) {
    double P[3], e[4], J[4][6];
    if (o.E) {
        double Q[3];
        rig_point(R, t, o, Q, P);
        if (!(P[2] > 0.0)) return false;
        residual_rows_rig(P, Q, o, p, e, J);
    } else {
        transform(R, t, o, P);
        if (!(P[2] > 0.0)) return false;
        residual_rows(P, o, p, e, J);
    }
    const double d2 = ((e[0] * e[0] + e[1] * e[1]) + e[2] * e[2]) + e[3] * e[3];
    return d2 < p.inlier_threshold * p.inlier_threshold;
}

const double kI3[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};

// the 3 distinct sample indices of hypothesis h (false if 16 draws do not give 3)
bool sample3(uint64_t seed, int h, int M, int* idx) {
    int got = 0;
    for (int k = 0; k < 16 && got < 3; ++k) {
        const int r = (int)(mix64(seed + (uint64_t)h * 16u + (uint64_t)k) % (uint64_t)M);
        bool dup = false;
        for (int j = 0; j < got; ++j) dup = dup || idx[j] == r;
        if (!dup) idx[got++] = r;
    }
    return got == 3;
}

// cams / extr: the rig form (match i seen by camera cams[i], extrinsics
// extr[12 c ..]); null for one stereo camera
int estimate(const int32_t* uv8, int M, int64_t frame, const viso_svo_params& p, double* motion,
             uint8_t* inlier, const int32_t* cams = nullptr, const double* extr = nullptr) {
    for (int i = 0; i < 12; ++i) motion[i] = (i < 9) ? kI3[i] : 0.0;
    for (int i = 0; i < M; ++i) inlier[i] = 0;
    if (M < 6) return -1;
    std::vector<Obs> obs((size_t)M);
    for (int i = 0; i < M; ++i)
        obs[(size_t)i] = cams ? make_obs_rig(uv8 + 8 * i, extr + 12 * cams[i], p) : make_obs(uv8 + 8 * i, p);
    const uint64_t seed = mix64(p.seed ^ (uint64_t)frame);
    int best_h = -1, best_cnt = -1;
    double bR[9], bt[3];
    std::vector<uint8_t> sel((size_t)M);
    for (int h = 0; h < p.ransac_iters; ++h) {
        int idx[3];
        int cnt = 0;
        double R[9], t[3] = {0, 0, 0};
        std::memcpy(R, kI3, sizeof(R));
        if (sample3(seed, h, M, idx)) {
            // the three samples, in draw order, as a 3-leaf tree: (s0 + s1) + (s2 + 0)
            const std::vector<Obs> obs3 = {obs[(size_t)idx[0]], obs[(size_t)idx[1]], obs[(size_t)idx[2]]};
            const std::vector<uint8_t> sel3 = {1, 1, 1};
            if (gauss_newton(obs3, sel3, p, R, t))
                for (int i = 0; i < M; ++i) cnt += is_inlier(R, t, obs[(size_t)i], p) ? 1 : 0;
        }
        if (cnt > best_cnt) {
            best_cnt = cnt;
            best_h = h;
            std::memcpy(bR, R, sizeof(bR));
            std::memcpy(bt, t, sizeof(bt));
        }
    }
    if (best_h < 0 || best_cnt < 6) return -1;
    for (int i = 0; i < M; ++i) sel[(size_t)i] = is_inlier(bR, bt, obs[(size_t)i], p) ? 1 : 0;
    double R[9], t[3];
    std::memcpy(R, bR, sizeof(R));
    std::memcpy(t, bt, sizeof(t));
    if (!gauss_newton(obs, sel, p, R, t)) {  // keep the best hypothesis
        std::memcpy(R, bR, sizeof(R));
        std::memcpy(t, bt, sizeof(t));
    }
    int n_inl = 0;
    for (int i = 0; i < M; ++i) {
        inlier[i] = is_inlier(R, t, obs[(size_t)i], p) ? 1 : 0;
        n_inl += inlier[i];
    }
    if (n_inl < 6) {
        for (int i = 0; i < M; ++i) inlier[i] = 0;
        return -1;  // motion stays the identity
    }
    for (int i = 0; i < 9; ++i) motion[i] = R[i];
    for (int i = 0; i < 3; ++i) motion[9 + i] = t[i];
    return n_inl;
}

}  // namespace

extern "C" {

int oracle_svo_features(const uint8_t* img, int w, int h, const viso_svo_params* p, int cap,
                        int32_t* u, int32_t* v, int32_t* cls, uint8_t* desc) {
    const std::vector<Feat> f = features(img, w, h, *p);
    const int n = (int)f.size();
    for (int i = 0; i < n && i < cap; ++i) {
        u[i] = f[(size_t)i].u;
        v[i] = f[(size_t)i].v;
        cls[i] = f[(size_t)i].c;
        std::memcpy(desc + (size_t)i * VISO_SVO_DESC_BYTES, f[(size_t)i].d, VISO_SVO_DESC_BYTES);
    }
    return n;
}

// Response maps (tests): blob / corner at every pixel (0 outside the domain).
void oracle_svo_responses(const uint8_t* img, int w, int h, int32_t* blob, int32_t* corner) {
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            const bool in = x >= 2 && x < w - 2 && y >= 2 && y < h - 2;
            blob[(size_t)y * w + x] = in ? blob5(img, w, x, y) : 0;
            corner[(size_t)y * w + x] = in ? corner5(img, w, x, y) : 0;
        }
}

// Circular matching; quad = {l1, r1, l2, r2} per match in ascending l2.
int oracle_svo_match(const int32_t* const* u4, const int32_t* const* v4, const int32_t* const* c4,
                     const uint8_t* const* d4, const int32_t* n4, int h, const viso_svo_params* p,
                     int32_t* quad, int cap) {
    FeatSet S[4];
    for (int k = 0; k < 4; ++k) {
        S[k].u = u4[k];
        S[k].v = v4[k];
        S[k].c = c4[k];
        S[k].d = d4[k];
        S[k].n = n4[k];
        S[k].index(h);
    }
    const FeatSet &L1 = S[0], &R1 = S[1], &L2 = S[2], &R2 = S[3];
    const int D = p->disp_max, Rr = p->match_radius;
    int n = 0;
    auto desc = [](const FeatSet& s, int i) { return s.d + (size_t)i * VISO_SVO_DESC_BYTES; };
    for (int i2 = 0; i2 < L2.n; ++i2) {
        const int c = L2.c[i2];
        // left_t -> right_t: u_r = u_l - d, 0 <= d <= D
        const int r2 = best_match(R2, h, L2.u[i2], L2.v[i2], c, desc(L2, i2), 0, D, 1);
        if (r2 < 0) continue;
        // right_t -> right_t-1
        const int r1 = best_match(R1, h, R2.u[r2], R2.v[r2], c, desc(R2, r2), -Rr, Rr, Rr);
        if (r1 < 0) continue;
        // right_t-1 -> left_t-1: u_l = u_r + d  (u_r - u_l in [-D, 0])
        const int l1 = best_match(L1, h, R1.u[r1], R1.v[r1], c, desc(R1, r1), -D, 0, 1);
        if (l1 < 0) continue;
        // left_t-1 -> left_t
        const int i2b = best_match(L2, h, L1.u[l1], L1.v[l1], c, desc(L1, l1), -Rr, Rr, Rr);
        if (i2b != i2) continue;
        if (L1.u[l1] - R1.u[r1] < 1 || L2.u[i2] - R2.u[r2] < 1) continue;
        if (n < cap) {
            quad[4 * n + 0] = l1;
            quad[4 * n + 1] = r1;
            quad[4 * n + 2] = i2;
            quad[4 * n + 3] = r2;
        }
        ++n;
    }
    return n;
}

// Bucketing of matches given as uv8 (ascending l2): keep[i] = 1 for the first
// bucket_max matches of each (u_l2 / bw, v_l2 / bh) bucket.
int oracle_svo_bucket(const int32_t* uv8, int n, int w, int h, const viso_svo_params* p,
                      uint8_t* keep) {
    const int bx = (w + p->bucket_width - 1) / p->bucket_width;
    const int by = (h + p->bucket_height - 1) / p->bucket_height;
    std::vector<int> cnt((size_t)bx * by, 0);
    int kept = 0;
    for (int i = 0; i < n; ++i) {
        const int b = (uv8[8 * i + 5] / p->bucket_height) * bx + uv8[8 * i + 4] / p->bucket_width;
        keep[i] = cnt[(size_t)b] < p->bucket_max ? 1 : 0;
        cnt[(size_t)b] += 1;
        kept += keep[i];
    }
    return kept;
}

int oracle_svo_estimate(const int32_t* uv8, int n, int64_t frame, const viso_svo_params* p,
                        double* motion12, uint8_t* inlier) {
    return estimate(uv8, n, frame, *p, motion12, inlier);
}

// Rig motion from the matches of all cameras (camera of match i: cams[i]).
int oracle_svo_rig_estimate(const int32_t* uv8, const int32_t* cams, int n, int64_t frame,
                            const viso_svo_params* p, const double* extr, double* motion12, uint8_t* inlier) {
    return estimate(uv8, n, frame, *p, motion12, inlier, cams, extr);
}

// SAD evaluations of the matching so far (reset: zero the count after reading).
unsigned long long oracle_svo_sad_evals(int reset) {
    const unsigned long long n = g_sad_evals;
    if (reset) g_sad_evals = 0;
    return n;
}

}  // extern "C"

// Spec defaults (the library's viso_svo_default_params returns the same).
extern "C" void oracle_svo_default_params(viso_svo_params* p, int w, int h, double fx, double fy,
                                          double cu, double cv, double base) {
    std::memset(p, 0, sizeof(*p));
    p->width = w;
    p->height = h;
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
}
