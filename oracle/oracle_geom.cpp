// TEST INFRASTRUCTURE ONLY — oracle geometry stage: Viso::Triangulate
// (src/viso.cpp:416-431), Viso::SelectMotion (:520-638),
// Viso::PoseEstimation2d2d (:178-256) and the repo's deterministic
// restatement of the OpenCV calls it makes (findEssentialMat, recoverPose,
// findHomography, decomposeHomographyMat).
//
// RANSAC spec (parity vs OpenCV unpinned):
//  * hypothesis h draws its minimal sample from a counter-based hash
//    (seed, h, try, k, attempt) -> index, so every hypothesis is independent
//    of the others and the device scores all of them in parallel;
//  * E: 8-point null vector (complete-pivot Gauss-Jordan) + projection onto
//    the essential manifold (singular values (1,1,0)); Sampson error
//    (OpenCV EMEstimatorCallback::computeError); 1000 hypotheses max;
//  * H: 4-point DLT null vector; OpenCV's checkSubset (collinearity +
//    orientation consistency); forward transfer error; 2000 max; the winner
//    is refined by a least-squares DLT over its inliers (stand-in for
//    OpenCV's LM refine);
//  * OpenCV's sequential loop (RANSACPointSetRegistrator::run with
//    RANSACUpdateNumIters) is reproduced exactly by scanning the
//    per-hypothesis inlier counts in order.
#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include "oracle_common.hpp"
#include "oracle_linalg.hpp"
#include "viso_oracle.h"

using namespace oracle;

namespace oracle {

// cv::RANSACUpdateNumIters (calib3d/src/ptsetreg.cpp)
int ransac_update_num_iters(double p, double ep, int modelPoints, int maxIters) {
    p = std::max(p, 0.);
    p = std::min(p, 1.);
    ep = std::max(ep, 0.);
    ep = std::min(ep, 1.);
    double num = std::max(1. - p, DBL_MIN);
    double denom = 1. - std::pow(1. - ep, modelPoints);
    if (denom < DBL_MIN) return 0;
    num = std::log(num);
    denom = std::log(denom);
    return denom >= 0 || -num >= maxIters * (-denom) ? maxIters : (int)std::rint(num / denom);
}

inline uint64_t sample_hash(uint64_t seed, int h, int t, int k, int a) {
    uint64_t z = seed + 0x632BE59BD9B4E019ULL * (uint64_t)(h + 1) +
                 0x9E3779B97F4A7C15ULL * (uint64_t)(t + 1) +
                 0xD1B54A32D192ED03ULL * (uint64_t)(k * 64 + a + 1);
    return mix64(z);
}

// distinct indices for minimal subset (hypothesis h, try t)
void draw_subset(uint64_t seed, int h, int t, int n, int m, int* idx) {
    for (int k = 0; k < m; ++k) {
        int chosen = -1;
        for (int a = 0; a < 64 && chosen < 0; ++a) {
            int c = (int)(sample_hash(seed, h, t, k, a) % (uint64_t)n);
            bool dup = false;
            for (int j = 0; j < k; ++j) dup |= (idx[j] == c);
            if (!dup) chosen = c;
        }
        if (chosen < 0) {  // smallest unused index
            for (int c = 0; c < n && chosen < 0; ++c) {
                bool dup = false;
                for (int j = 0; j < k; ++j) dup |= (idx[j] == c);
                if (!dup) chosen = c;
            }
        }
        idx[k] = chosen;
    }
}

// ---- essential matrix
bool essential_from_8(const double* p1, const double* p2, const int* idx, double* E) {
    double A[72];
    for (int r = 0; r < 8; ++r) {
        const double x1 = p1[2 * idx[r]], y1 = p1[2 * idx[r] + 1];
        const double x2 = p2[2 * idx[r]], y2 = p2[2 * idx[r] + 1];
        double* a = A + 9 * r;
        a[0] = x2 * x1;
        a[1] = x2 * y1;
        a[2] = x2;
        a[3] = y2 * x1;
        a[4] = y2 * y1;
        a[5] = y2;
        a[6] = x1;
        a[7] = y1;
        a[8] = 1.0;
    }
    double e[9];
    if (!null_vector_8x9(A, e)) return false;
    double U[9], s[3], V[9];
    svd3(e, U, s, V);
    if (!(s[1] > 0)) return false;
    // E' = u0 v0^T + u1 v1^T  (singular values (1, 1, 0))
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) E[3 * i + j] = U[3 * i + 0] * V[3 * j + 0] + U[3 * i + 1] * V[3 * j + 1];
    return true;
}

inline float sampson_err(const double* E, double x1, double y1, double x2, double y2) {
    const double ex0 = E[0] * x1 + E[1] * y1 + E[2];
    const double ex1 = E[3] * x1 + E[4] * y1 + E[5];
    const double ex2 = E[6] * x1 + E[7] * y1 + E[8];
    const double et0 = E[0] * x2 + E[3] * y2 + E[6];
    const double et1 = E[1] * x2 + E[4] * y2 + E[7];
    const double x2tEx1 = x2 * ex0 + y2 * ex1 + ex2;
    const double a = ex0 * ex0, b = ex1 * ex1, c = et0 * et0, d = et1 * et1;
    return (float)(x2tEx1 * x2tEx1 / (a + b + c + d));
}

// ---- homography
bool subset_ok_h(const double* p1, const double* p2, const int* idx) {
    static const int tt[4][3] = {{0, 1, 2}, {1, 2, 3}, {0, 2, 3}, {0, 1, 3}};
    const float eps = FLT_EPSILON;
    for (int img = 0; img < 2; ++img) {
        const double* p = img == 0 ? p1 : p2;
        for (int a = 0; a < 4; ++a) {
            const int* t = tt[a];
            double dx1 = p[2 * idx[t[1]]] - p[2 * idx[t[0]]], dy1 = p[2 * idx[t[1]] + 1] - p[2 * idx[t[0]] + 1];
            double dx2 = p[2 * idx[t[2]]] - p[2 * idx[t[0]]], dy2 = p[2 * idx[t[2]] + 1] - p[2 * idx[t[0]] + 1];
            if (std::fabs(dx2 * dy1 - dy2 * dx1) <=
                eps * (std::fabs(dx1) + std::fabs(dy1) + std::fabs(dx2) + std::fabs(dy2)))
                return false;
        }
    }
    int negative = 0;
    for (int a = 0; a < 4; ++a) {
        const int* t = tt[a];
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

void h_rows(double x1, double y1, double x2, double y2, double* a, double* b) {
    a[0] = x1;
    a[1] = y1;
    a[2] = 1.0;
    a[3] = 0.0;
    a[4] = 0.0;
    a[5] = 0.0;
    a[6] = -x2 * x1;
    a[7] = -x2 * y1;
    a[8] = -x2;
    b[0] = 0.0;
    b[1] = 0.0;
    b[2] = 0.0;
    b[3] = x1;
    b[4] = y1;
    b[5] = 1.0;
    b[6] = -y2 * x1;
    b[7] = -y2 * y1;
    b[8] = -y2;
}

bool homography_from_4(const double* p1, const double* p2, const int* idx, double* H) {
    double A[72];
    for (int r = 0; r < 4; ++r)
        h_rows(p1[2 * idx[r]], p1[2 * idx[r] + 1], p2[2 * idx[r]], p2[2 * idx[r] + 1], A + 18 * r,
               A + 18 * r + 9);
    return null_vector_8x9(A, H);
}

inline float transfer_err(const double* H, double x1, double y1, double x2, double y2) {
    const double w = H[6] * x1 + H[7] * y1 + H[8];
    const double px = (H[0] * x1 + H[1] * y1 + H[2]) / w;
    const double py = (H[3] * x1 + H[4] * y1 + H[5]) / w;
    const double dx = px - x2, dy = py - y2;
    return (float)(dx * dx + dy * dy);
}

int scan_hypotheses(const std::vector<int>& counts, int n, int modelPoints, double conf,
                    int maxIters, int* best_out, int* iters_out) {
    int niters = maxIters, maxGood = 0, best = -1, h = 0;
    for (h = 0; h < niters; ++h) {
        const int c = counts[(size_t)h];
        if (c < 0) continue;
        if (c > std::max(maxGood, modelPoints - 1)) {
            maxGood = c;
            best = h;
            niters = ransac_update_num_iters(conf, (double)(n - c) / n, modelPoints, niters);
        }
    }
    *best_out = best;
    *iters_out = h;
    return maxGood;
}

// Viso::Triangulate (src/viso.cpp:416-431) with P1 = [I|0], P2 = [R|T];
// returns the homogeneous null vector (before the division by V(3,3)).
void triangulate_h(const double* R, const double* T, double x1, double y1, double x2, double y2,
                   double* X) {
    double P2[12] = {R[0], R[1], R[2], T[0], R[3], R[4], R[5], T[1], R[6], R[7], R[8], T[2]};
    double A[16];
    // Pi1 = [I | 0]: rows (1,0,0,0), (0,1,0,0), (0,0,1,0)
    const double P1[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    for (int j = 0; j < 4; ++j) {
        A[j] = x1 * P1[8 + j] - P1[j];
        A[4 + j] = y1 * P1[8 + j] - P1[4 + j];
        A[8 + j] = x2 * P2[8 + j] - P2[j];
        A[12 + j] = y2 * P2[8 + j] - P2[4 + j];
    }
    null_vector_jacobi<4>(A, X);
}

}  // namespace oracle

extern "C" {

void oracle_triangulate(const double R[9], const double T[3], const double x1[3],
                        const double x2[3], double P[3]) {
    double X[4];
    triangulate_h(R, T, x1[0], x1[1], x2[0], x2[1], X);
    P[0] = X[0] / X[3];
    P[1] = X[1] / X[3];
    P[2] = X[2] / X[3];
}

int oracle_ransac_essential(const double* p1, const double* p2, int n, double thresh,
                            double confidence, int max_iters, uint64_t seed, double E_out[9],
                            uint8_t* mask_out, int32_t* iters_out) {
    if (iters_out) *iters_out = 0;
    if (n < 8) return 0;
    const float t2 = (float)(thresh * thresh);
    std::vector<int> counts((size_t)max_iters, -1);
    std::vector<double> models((size_t)max_iters * 9);
    for (int h = 0; h < max_iters; ++h) {
        int idx[8];
        if (n == 8)
            for (int k = 0; k < 8; ++k) idx[k] = k;
        else
            draw_subset(seed, h, 0, n, 8, idx);
        double* E = &models[(size_t)h * 9];
        if (!essential_from_8(p1, p2, idx, E)) continue;
        int c = 0;
        for (int i = 0; i < n; ++i)
            c += sampson_err(E, p1[2 * i], p1[2 * i + 1], p2[2 * i], p2[2 * i + 1]) <= t2;
        counts[(size_t)h] = c;
    }
    int best, iters;
    int good = scan_hypotheses(counts, n, 8, confidence, max_iters, &best, &iters);
    if (iters_out) *iters_out = iters;
    if (best < 0) return 0;
    const double* E = &models[(size_t)best * 9];
    for (int k = 0; k < 9; ++k) E_out[k] = E[k];
    if (mask_out)
        for (int i = 0; i < n; ++i)
            mask_out[i] = sampson_err(E, p1[2 * i], p1[2 * i + 1], p2[2 * i], p2[2 * i + 1]) <= t2;
    return good;
}

int oracle_ransac_homography(const double* p1, const double* p2, int n, double thresh,
                             double confidence, int max_iters, uint64_t seed, double H_out[9],
                             uint8_t* mask_out, int32_t* iters_out) {
    if (iters_out) *iters_out = 0;
    if (n < 4) return 0;
    const float t2 = (float)(thresh * thresh);
    std::vector<int> counts((size_t)max_iters, -1);
    std::vector<double> models((size_t)max_iters * 9);
    for (int h = 0; h < max_iters; ++h) {
        int idx[4];
        bool ok = false;
        for (int t = 0; t < 100 && !ok; ++t) {
            if (n == 4)
                for (int k = 0; k < 4; ++k) idx[k] = k;
            else
                draw_subset(seed ^ 0x4848484848484848ULL, h, t, n, 4, idx);
            ok = subset_ok_h(p1, p2, idx);
            if (n == 4) break;
        }
        if (!ok) continue;
        double* H = &models[(size_t)h * 9];
        if (!homography_from_4(p1, p2, idx, H)) continue;
        int c = 0;
        for (int i = 0; i < n; ++i)
            c += transfer_err(H, p1[2 * i], p1[2 * i + 1], p2[2 * i], p2[2 * i + 1]) <= t2;
        counts[(size_t)h] = c;
    }
    int best, iters;
    int good = scan_hypotheses(counts, n, 4, confidence, max_iters, &best, &iters);
    if (iters_out) *iters_out = iters;
    if (best < 0) return 0;
    const double* Hb = &models[(size_t)best * 9];
    std::vector<uint8_t> mask((size_t)n);
    for (int i = 0; i < n; ++i)
        mask[(size_t)i] = transfer_err(Hb, p1[2 * i], p1[2 * i + 1], p2[2 * i], p2[2 * i + 1]) <= t2;
    // least-squares DLT refine over the inliers: smallest eigenvector of
    // sum_i (a_i a_i^T + b_i b_i^T), 45 tree sums over the point index.
    double H[9];
    for (int k = 0; k < 9; ++k) H[k] = Hb[k];
    if (good >= 4) {
        std::vector<double> leaf((size_t)n);
        double M[81];
        int idx = 0;
        for (int r = 0; r < 9; ++r)
            for (int c = r; c < 9; ++c) {
                for (int i = 0; i < n; ++i) {
                    double a[9], b[9];
                    h_rows(p1[2 * i], p1[2 * i + 1], p2[2 * i], p2[2 * i + 1], a, b);
                    leaf[(size_t)i] = mask[(size_t)i] ? a[r] * a[c] + b[r] * b[c] : 0.0;
                }
                double s = tree_sum(leaf.data(), n);
                M[9 * r + c] = s;
                M[9 * c + r] = s;
                ++idx;
            }
        double ev[9], V[81];
        jacobi_eigen_rr<9>(M, ev, V);  // the device's parallel (round-robin) ordering
        for (int k = 0; k < 9; ++k) H[k] = V[9 * k + 8];
    }
    if (std::fabs(H[8]) > 1e-12) {
        const double d = H[8];
        for (int k = 0; k < 9; ++k) H[k] = H[k] / d;
    }
    for (int k = 0; k < 9; ++k) H_out[k] = H[k];
    if (mask_out)
        for (int i = 0; i < n; ++i) mask_out[i] = mask[(size_t)i];
    return good;
}

int oracle_recover_pose(const double E[9], const double* p1, const double* p2, int n,
                        uint8_t* mask, double R_out[9], double t_out[3]) {
    // decomposeEssentialMat
    double U[9], s[3], V[9];
    svd3(E, U, s, V);
    if (det3(U) < 0)
        for (int k = 0; k < 9; ++k) U[k] = -U[k];
    double Vt[9];
    transpose3(V, Vt);
    if (det3(Vt) < 0)
        for (int k = 0; k < 9; ++k) Vt[k] = -Vt[k];
    const double W[9] = {0, 1, 0, -1, 0, 0, 0, 0, 1};
    double Wt[9], UW[9], R1[9], R2[9];
    transpose3(W, Wt);
    matmul3(U, W, UW);
    matmul3(UW, Vt, R1);
    matmul3(U, Wt, UW);
    matmul3(UW, Vt, R2);
    const double t[3] = {U[2] * 1.0, U[5] * 1.0, U[8] * 1.0};
    const double dist = 50.0;
    const double* Rs[4] = {R1, R2, R1, R2};
    const double sg[4] = {1, 1, -1, -1};
    int good[4];
    std::vector<uint8_t> masks((size_t)4 * n);
    for (int m = 0; m < 4; ++m) {
        const double tt[3] = {sg[m] * t[0], sg[m] * t[1], sg[m] * t[2]};
        int g = 0;
        for (int i = 0; i < n; ++i) {
            double X[4];
            triangulate_h(Rs[m], tt, p1[2 * i], p1[2 * i + 1], p2[2 * i], p2[2 * i + 1], X);
            bool ok = X[2] * X[3] > 0;
            double Q[3] = {X[0] / X[3], X[1] / X[3], X[2] / X[3]};
            ok = (Q[2] < dist) && ok;
            double z2 = Rs[m][6] * Q[0] + Rs[m][7] * Q[1] + Rs[m][8] * Q[2] + tt[2] * 1.0;
            ok = (z2 > 0) && ok;
            ok = (z2 < dist) && ok;
            if (mask) ok = ok && mask[i];
            masks[(size_t)m * n + i] = ok;
            g += ok;
        }
        good[m] = g;
    }
    int pick;
    if (good[0] >= good[1] && good[0] >= good[2] && good[0] >= good[3])
        pick = 0;
    else if (good[1] >= good[0] && good[1] >= good[2] && good[1] >= good[3])
        pick = 1;
    else if (good[2] >= good[0] && good[2] >= good[1] && good[2] >= good[3])
        pick = 2;
    else
        pick = 3;
    for (int k = 0; k < 9; ++k) R_out[k] = Rs[pick][k];
    for (int k = 0; k < 3; ++k) t_out[k] = pick >= 2 ? -t[k] : t[k];
    if (mask)
        for (int i = 0; i < n; ++i) mask[i] = masks[(size_t)pick * n + i];
    return good[pick];
}

// cv::decomposeHomographyMat(H, K = I) — HomographyDecompInria
int oracle_decompose_homography(const double Hin[9], double* Rs, double* ts, double* ns) {
    double U[9], s[3], V[9];
    svd3(Hin, U, s, V);
    double Hn[9];
    const double inv = 1.0 / s[1];
    for (int k = 0; k < 9; ++k) Hn[k] = Hin[k] * inv;
    double Ht[9], S[9];
    transpose3(Hn, Ht);
    matmul3(Ht, Hn, S);
    S[0] -= 1.0;
    S[4] -= 1.0;
    S[8] -= 1.0;
    double mx = 0;
    for (int k = 0; k < 9; ++k) mx = std::max(mx, std::fabs(S[k]));
    if (mx < 0.001) {
        for (int k = 0; k < 9; ++k) Rs[k] = Hn[k];
        ts[0] = ts[1] = ts[2] = 0;
        ns[0] = ns[1] = ns[2] = 0;
        return 1;
    }
    auto minor = [&](int row, int col) {
        int x1 = col == 0 ? 1 : 0, x2 = col == 2 ? 1 : 2;
        int y1 = row == 0 ? 1 : 0, y2 = row == 2 ? 1 : 2;
        return S[3 * y1 + x2] * S[3 * y2 + x1] - S[3 * y1 + x1] * S[3 * y2 + x2];
    };
    auto signd = [](double x) { return x >= 0 ? 1 : -1; };
    const double M00 = minor(0, 0), M11 = minor(1, 1), M22 = minor(2, 2);
    const double rtM00 = std::sqrt(M00), rtM11 = std::sqrt(M11), rtM22 = std::sqrt(M22);
    const double M01 = minor(0, 1), M12 = minor(1, 2), M02 = minor(0, 2);
    const int e12 = signd(M12), e02 = signd(M02), e01 = signd(M01);
    const double nS00 = std::fabs(S[0]), nS11 = std::fabs(S[4]), nS22 = std::fabs(S[8]);
    int indx = 0;
    if (nS00 < nS11) {
        indx = 1;
        if (nS11 < nS22) indx = 2;
    } else {
        if (nS00 < nS22) indx = 2;
    }
    double npa[3], npb[3];
    switch (indx) {
        case 0:
            npa[0] = S[0], npb[0] = S[0];
            npa[1] = S[1] + rtM22, npb[1] = S[1] - rtM22;
            npa[2] = S[2] + e12 * rtM11, npb[2] = S[2] - e12 * rtM11;
            break;
        case 1:
            npa[0] = S[1] + rtM22, npb[0] = S[1] - rtM22;
            npa[1] = S[4], npb[1] = S[4];
            npa[2] = S[5] - e02 * rtM00, npb[2] = S[5] + e02 * rtM00;
            break;
        default:
            npa[0] = S[2] + e01 * rtM11, npb[0] = S[2] - e01 * rtM11;
            npa[1] = S[5] + rtM00, npb[1] = S[5] - rtM00;
            npa[2] = S[8], npb[2] = S[8];
            break;
    }
    const double traceS = S[0] + S[4] + S[8];
    const double v = 2.0 * (double)sqrtf((float)(1 + traceS - M00 - M11 - M22));
    const double ESii = signd(S[3 * indx + indx]);
    const double r_2 = 2 + traceS + v;
    const double nt_2 = 2 + traceS - v;
    const double r = std::sqrt(r_2);
    const double n_t = std::sqrt(nt_2);
    const double na_n = std::sqrt((npa[0] * npa[0] + npa[1] * npa[1]) + npa[2] * npa[2]);
    const double nb_n = std::sqrt((npb[0] * npb[0] + npb[1] * npb[1]) + npb[2] * npb[2]);
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
    auto rmat = [&](const double* tstar, const double* n, double* R) {
        double M[9];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) M[3 * i + j] = (i == j ? 1.0 : 0.0) - (2 / v) * tstar[i] * n[j];
        matmul3(Hn, M, R);
        if (det3(R) < 0)
            for (int k = 0; k < 9; ++k) R[k] = -R[k];
    };
    double Ra[9], Rb[9], ta[3], tb[3];
    rmat(ta_star, na, Ra);
    mat3_vec(Ra, ta_star, ta);
    rmat(tb_star, nb, Rb);
    mat3_vec(Rb, tb_star, tb);
    for (int k = 0; k < 9; ++k) {
        Rs[k] = Ra[k];
        Rs[9 + k] = Ra[k];
        Rs[18 + k] = Rb[k];
        Rs[27 + k] = Rb[k];
    }
    for (int k = 0; k < 3; ++k) {
        ts[k] = ta[k];
        ts[3 + k] = -ta[k];
        ts[6 + k] = tb[k];
        ts[9 + k] = -tb[k];
        ns[k] = na[k];
        ns[3 + k] = -na[k];
        ns[6 + k] = nb[k];
        ns[9 + k] = -nb[k];
    }
    return 4;
}

int oracle_select_motion(const double* p1, const double* p2, int n, const double* Rs,
                         const double* Ts, int m, const double K[4], double proj_thresh,
                         double parallax_thresh, int32_t* best_out, double R_out[9],
                         double T_out[3], uint8_t* inliers, double* points3d) {
    const double kPi = 3.14159265358979323846;  // CV_PI
    int best_nr = 0, best_motion = -1;
    std::vector<uint8_t> cur_in((size_t)n), best_in((size_t)n, 0);
    std::vector<double> cur_pts((size_t)3 * n), best_pts((size_t)3 * n, 0.0);
    for (int mi = 0; mi < m; ++mi) {
        const double* R = Rs + 9 * mi;
        const double* T = Ts + 3 * mi;
        // O2 = -R * T (src/viso.cpp:543)
        double O2[3];
        for (int i = 0; i < 3; ++i) O2[i] = (-R[3 * i]) * T[0] + (-R[3 * i + 1]) * T[1] + (-R[3 * i + 2]) * T[2];
        int cnt = 0;
        for (int i = 0; i < n; ++i) {
            cur_in[(size_t)i] = 0;
            cur_pts[(size_t)3 * i] = cur_pts[(size_t)3 * i + 1] = cur_pts[(size_t)3 * i + 2] = 0.0;
            const double x1 = p1[3 * i], y1 = p1[3 * i + 1], x2 = p2[3 * i], y2 = p2[3 * i + 1];
            double X[4];
            triangulate_h(R, T, x1, y1, x2, y2, X);
            double P1[3] = {X[0] / X[3], X[1] / X[3], X[2] / X[3]};
            if (P1[2] < 0) continue;
            double n2[3] = {P1[0] - O2[0], P1[1] - O2[1], P1[2] - O2[2]};
            double d1 = std::sqrt((P1[0] * P1[0] + P1[1] * P1[1]) + P1[2] * P1[2]);
            double d2 = std::sqrt((n2[0] * n2[0] + n2[1] * n2[1]) + n2[2] * n2[2]);
            double parallax = (P1[0] * n2[0] + P1[1] * n2[1]) + P1[2] * n2[2];
            parallax /= (d1 * d2);
            parallax = std::acos(parallax) * 180 / kPi;
            if (parallax > parallax_thresh) continue;
            double pj[2] = {P1[0] / P1[2], P1[1] / P1[2]};
            double dx = (pj[0] - x1) * K[0];
            double dy = (pj[1] - y1) * K[1];
            if (std::sqrt(dx * dx + dy * dy) > proj_thresh) continue;
            double P2[3];
            mat3_vec(R, P1, P2);
            P2[0] = P2[0] + T[0];
            P2[1] = P2[1] + T[1];
            P2[2] = P2[2] + T[2];
            if (P2[2] < 0) continue;
            double q[2] = {P2[0] / P2[2], P2[1] / P2[2]};
            dx = (q[0] - x2) * K[0];
            dy = (q[1] - y2) * K[1];
            if (std::sqrt(dx * dx + dy * dy) > proj_thresh) continue;
            cur_in[(size_t)i] = 1;
            cur_pts[(size_t)3 * i] = P1[0];
            cur_pts[(size_t)3 * i + 1] = P1[1];
            cur_pts[(size_t)3 * i + 2] = P1[2];
            ++cnt;
        }
        if (cnt > best_nr) {
            best_nr = cnt;
            best_motion = mi;
            best_in = cur_in;
            best_pts = cur_pts;
        }
    }
    if (best_out) *best_out = best_motion;
    if (best_motion != -1) {
        for (int k = 0; k < 9; ++k) R_out[k] = Rs[9 * best_motion + k];
        for (int k = 0; k < 3; ++k) T_out[k] = Ts[3 * best_motion + k];
    }
    // depth normalisation (src/viso.cpp:622-637): tree sum of the inliers' z
    std::vector<double> leaf((size_t)n);
    for (int i = 0; i < n; ++i) leaf[(size_t)i] = best_in[(size_t)i] ? best_pts[(size_t)3 * i + 2] : 0.0;
    double mean_depth = acc_sum(leaf.data(), n);
    if (mean_depth != 0) {
        mean_depth /= best_nr;
        for (int i = 0; i < n; ++i)
            if (best_in[(size_t)i])
                for (int k = 0; k < 3; ++k) best_pts[(size_t)3 * i + k] = best_pts[(size_t)3 * i + k] / mean_depth;
        for (int k = 0; k < 3; ++k) T_out[k] = T_out[k] / mean_depth;
    }
    for (int i = 0; i < n; ++i) {
        inliers[i] = best_in[(size_t)i];
        for (int k = 0; k < 3; ++k) points3d[3 * i + k] = best_pts[(size_t)3 * i + k];
    }
    return best_nr;
}

// Viso::PoseEstimation2d2d (src/viso.cpp:178-256) + SelectMotion.
// p1, p2: n x 3 normalised (z = 1).  stats = {nr_inliers, best_motion,
// n_candidates, disparity_sq, e_inliers, h_inliers, e_iters, h_iters}.
// Returns 0 if an early return happened (R, T, inliers untouched), 1 otherwise.
int oracle_pose_2d2d(const double* p1, const double* p2, int n, const double K[4],
                     const oracle_params* prm, double R[9], double T[3], uint8_t* inliers,
                     double* points3d, double* candidates, double stats[8]) {
    for (int k = 0; k < 8; ++k) stats[k] = 0;
    if (n < 10) return 0;
    const double thresh = prm->projection_error_thresh / std::sqrt(K[0] * K[0] + K[1] * K[1]);
    const double f = (K[0] + K[1]) / 2;
    std::vector<double> leaf((size_t)n), q1((size_t)2 * n), q2((size_t)2 * n);
    for (int i = 0; i < n; ++i) {
        double dx = p2[3 * i] - p1[3 * i];
        double dy = p2[3 * i + 1] - p1[3 * i + 1];
        leaf[(size_t)i] = dx * dx + dy * dy;
        q1[(size_t)2 * i] = (double)(float)p1[3 * i];
        q1[(size_t)2 * i + 1] = (double)(float)p1[3 * i + 1];
        q2[(size_t)2 * i] = (double)(float)p2[3 * i];
        q2[(size_t)2 * i + 1] = (double)(float)p2[3 * i + 1];
    }
    double disparity_squared = acc_sum(leaf.data(), n);
    if (disparity_squared != 0) {
        disparity_squared /= n;
        disparity_squared *= f * f;
    }
    stats[3] = disparity_squared;
    if (disparity_squared < prm->disparity_squared_thresh) return 0;
    std::vector<double> Rs, Ts;
    double E[9];
    std::vector<uint8_t> emask((size_t)n);
    int32_t eit = 0, hit = 0;
    int ein = oracle_ransac_essential(q1.data(), q2.data(), n, thresh, prm->ransac_confidence,
                                      prm->ransac_e_iters, prm->ransac_seed, E, emask.data(), &eit);
    stats[4] = ein;
    stats[6] = eit;
    if (ein > 0) {
        double Re[9], te[3];
        oracle_recover_pose(E, q1.data(), q2.data(), n, emask.data(), Re, te);
        Rs.insert(Rs.end(), Re, Re + 9);
        Ts.insert(Ts.end(), te, te + 3);
    }
    double H[9];
    int hin = oracle_ransac_homography(q1.data(), q2.data(), n, thresh, prm->ransac_confidence,
                                       prm->ransac_h_iters, prm->ransac_seed, H, nullptr, &hit);
    stats[5] = hin;
    stats[7] = hit;
    if (hin > 0) {
        double hR[36], hT[12], hN[12];
        int ns = oracle_decompose_homography(H, hR, hT, hN);
        for (int s = 0; s < ns; ++s) {
            Rs.insert(Rs.end(), hR + 9 * s, hR + 9 * s + 9);
            Ts.insert(Ts.end(), hT + 3 * s, hT + 3 * s + 3);
        }
    }
    const int m = (int)Ts.size() / 3;
    stats[2] = m;
    if (candidates)
        for (int c = 0; c < m; ++c) {
            for (int k = 0; k < 9; ++k) candidates[12 * c + k] = Rs[(size_t)9 * c + k];
            for (int k = 0; k < 3; ++k) candidates[12 * c + 9 + k] = Ts[(size_t)3 * c + k];
        }
    int32_t best = -1;
    int nr = oracle_select_motion(p1, p2, n, Rs.data(), Ts.data(), m, K,
                                  prm->projection_error_thresh, prm->parallax_thresh, &best, R, T,
                                  inliers, points3d);
    stats[0] = nr;
    stats[1] = best;
    return 1;
}

}  // extern "C"
