// TEST INFRASTRUCTURE ONLY — oracle tracking stage: pyramidal inverse-
// compositional KLT (OpticalFlowSingle/MultiLevel, src/viso.cpp:259-391),
// direct photometric 6-DoF Gauss-Newton (DirectPoseEstimationSingle/
// MultiLayer + dPixeldXi, src/viso.cpp:640-766) and LK feature alignment
// (LKAlignment / LKAlignmentSingle, src/viso.cpp:768-925).  See viso_oracle.h
// for the spec decisions (tree sums, zero taps).
#include <cmath>
#include <cstring>
#include <vector>

#include "oracle_common.hpp"
#include "oracle_se3.hpp"
#include "viso_oracle.h"

using namespace oracle;

namespace oracle {

// ------------------------------------------------------------------ KLT
// OpticalFlowSingleLevel(img1, img2, kp1, kp2, success, inverse=true) with
// have_initial = true (kp2 non-empty, src/viso.cpp:267).
void klt_single_level(const uint8_t* img1, const uint8_t* img2, int cols, int rows,
                      const float* kp1, float* kp2, uint8_t* success, int n, double thresh) {
    const double hp = 4.0;  // half_patch_size (double, include/viso.h:25)
    double hxx[64], hxy[64], hyx[64], hyy[64], b0[64], b1[64], cc[64];
    for (int i = 0; i < n; ++i) {
        const float kx = kp1[2 * i], ky = kp1[2 * i + 1];
        double dx = (double)(kp2[2 * i] - kx);  // float - float (src/viso.cpp:273)
        double dy = (double)(kp2[2 * i + 1] - ky);
        double cost = 0, lastCost = 0;
        bool succ = true;
        for (int iter = 0; iter < 10; ++iter) {
            cost = 0;
            if ((double)kx + dx <= hp || (double)kx + dx >= cols - hp || (double)ky + dy <= hp ||
                (double)ky + dy >= rows - hp) {
                succ = false;
                break;
            }
            for (int x = -4; x < 4; ++x)
                for (int y = -4; y < 4; ++y) {
                    const int p = (x + 4) * 8 + (y + 4);
                    const float fx = kx + (float)x;  // float + int (src/viso.cpp:302)
                    const float fy = ky + (float)y;
                    double gx, gy;
                    gradient(img1, cols, rows, (double)fx, (double)fy, gx, gy);
                    const double J0 = -gx, J1 = -gy;
                    const double error = sample(img1, cols, rows, (double)fx, (double)fy) -
                                         sample(img2, cols, rows, (double)fx + dx, (double)fy + dy);
                    hxx[p] = J0 * J0;
                    hxy[p] = J0 * J1;
                    hyx[p] = J1 * J0;
                    hyy[p] = J1 * J1;
                    b0[p] = -J0 * error;
                    b1[p] = -J1 * error;
                    cc[p] = error * error;
                }
            const double H00 = acc_sum(hxx, 64), H01 = acc_sum(hxy, 64), H10 = acc_sum(hyx, 64),
                         H11 = acc_sum(hyy, 64);
            const double B0 = acc_sum(b0, 64), B1 = acc_sum(b1, 64);
            cost = acc_sum(cc, 64);
            // Eigen 2x2 inverse (compute_inverse_size2_helper)
            const double invdet = 1.0 / (H00 * H11 - H10 * H01);
            const double i00 = H11 * invdet, i10 = -H10 * invdet, i01 = -H01 * invdet,
                         i11 = H00 * invdet;
            const double u0 = i00 * B0 + i01 * B1;
            const double u1 = i10 * B0 + i11 * B1;
            if (std::isnan(u0)) {
                succ = false;
                break;
            }
            if (iter > 0 && cost > lastCost) break;
            dx += u0;
            dy += u1;
            lastCost = cost;
            succ = !(lastCost > thresh);
        }
        success[i] = succ ? 1 : 0;
        kp2[2 * i] = kx + (float)dx;  // cv::Point2f + cv::Point2f (src/viso.cpp:343)
        kp2[2 * i + 1] = ky + (float)dy;
    }
}

// ------------------------------------------------------------------ direct pose
// dPixeldXi (src/viso.cpp:640-658)
void d_pixel_d_xi(const double K[4], const double* R, const double* T, const double* P,
                  double scale, double J[12]) {
    double Pc[3];
    mat3_vec(R, P, Pc);
    Pc[0] = Pc[0] + T[0];
    Pc[1] = Pc[1] + T[1];
    Pc[2] = Pc[2] + T[2];
    const double x = Pc[0], y = Pc[1], z = Pc[2];
    const double fx = K[0] * scale, fy = K[1] * scale;
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

// Per-map-point partial sums of one DirectPoseEstimationSingleLayer
// iteration (28 = 21 upper-triangle H + 6 b + 1 cost).  Returns false if the
// point is not "good" (:704-715).
// Canonical (tree) form, factored (round 6): the reference's per-pixel
// J = -J_img_pixel^T J_pixel_xi (:725) has J_pixel_xi computed once per point
// (:718), so over the patch
//   sum_p J J^T  = Jp^T G Jp,  G = sum_p g g^T  (g = J_img_pixel)
//   sum_p -e J   = Jp^T (sum_p e g)
// i.e. six pixel sums (g0 g0, g0 g1, g1 g1, e g0, e g1, e e; each the
// descending pairwise tree tree_sum_desc64, the device's reduce_scatter_6_desc)
// and then, per H entry (a, b), (G00 (Jp0a Jp0b) + G01 (Jp0a Jp1b + Jp1a Jp0b))
// + G11 (Jp1a Jp1b), per b entry (e g0) Jp0a + (e g1) Jp1a, and the cost
// sum e e — the same real-number sums as the reference's, rounded
// differently; tests/test_literal_drift.py bounds what that does to the
// poses against the literal form below.
// With `running` (literal order) the pixel terms are instead formed per pixel
// and added straight into the level's running sums, x outer / y inner, as
// H += J J^T, b += -error J, cost += error^2 do at src/viso.cpp:722-729.
bool direct_point_partials(const PyrView& last, const PyrView& cur, const Pose& last_pose,
                           const Pose& cur_pose, const double K[4], const double* P, int level,
                           double out[28], double* running = nullptr) {
    const int w = last.w[level], h = last.h[level];
    double u_ref, v_ref, u_cur, v_cur;
    project(last_pose, K, P, level, u_ref, v_ref);
    project(cur_pose, K, P, level, u_cur, v_cur);
    const double hp = 4.0;
    bool good = is_inside(u_ref - hp, v_ref - hp, w, h) && is_inside(u_ref + hp, v_ref + hp, w, h) &&
                is_inside(u_cur - hp, v_cur - hp, cur.w[level], cur.h[level]) &&
                is_inside(u_cur + hp, v_cur + hp, cur.w[level], cur.h[level]);
    if (!good) return false;
    double Jpx[12];
    d_pixel_d_xi(K, cur_pose.R, cur_pose.t, P, kScales[level], Jpx);
    static thread_local double leaf[6][64];
    const uint8_t* L = last.level(level);
    const uint8_t* C = cur.level(level);
    for (int x = -4; x < 4; ++x)
        for (int y = -4; y < 4; ++y) {
            const int p = (x + 4) * 8 + (y + 4);
            const double error = sample(L, w, h, u_ref + x, v_ref + y) -
                                 sample(C, cur.w[level], cur.h[level], u_cur + x, v_cur + y);
            double g0, g1;
            gradient(C, cur.w[level], cur.h[level], u_cur + x, v_cur + y, g0, g1);
            if (running) {
                double J[6];
                for (int k = 0; k < 6; ++k) J[k] = -g0 * Jpx[k] + -g1 * Jpx[6 + k];
                int idx = 0;
                for (int a = 0; a < 6; ++a)
                    for (int b = a; b < 6; ++b) {
                        running[idx] = running[idx] + J[a] * J[b];
                        ++idx;
                    }
                for (int k = 0; k < 6; ++k) running[21 + k] = running[21 + k] + -error * J[k];
                running[27] = running[27] + error * error;
                continue;
            }
            leaf[0][p] = g0 * g0;
            leaf[1][p] = g0 * g1;
            leaf[2][p] = g1 * g1;
            leaf[3][p] = error * g0;
            leaf[4][p] = error * g1;
            leaf[5][p] = error * error;
        }
    if (running) return true;
    double G[6];
    for (int k = 0; k < 6; ++k) G[k] = tree_sum_desc64(leaf[k]);  // device reduce_scatter_6_desc
    const double* J0 = Jpx;      // dPixel/dXi row 0 (u)
    const double* J1 = Jpx + 6;  // row 1 (v)
    int idx = 0;
    for (int a = 0; a < 6; ++a)
        for (int b = a; b < 6; ++b)
            out[idx++] = (G[0] * (J0[a] * J0[b]) + G[1] * (J0[a] * J1[b] + J1[a] * J0[b])) + G[2] * (J1[a] * J1[b]);
    for (int a = 0; a < 6; ++a) out[21 + a] = G[3] * J0[a] + G[4] * J1[a];
    out[27] = G[5];
    return true;
}

}  // namespace oracle

namespace {

inline Pose pose_from12(const double* p) {
    Pose r;
    for (int i = 0; i < 9; ++i) r.R[i] = p[i];
    for (int i = 0; i < 3; ++i) r.t[i] = p[9 + i];
    return r;
}

inline Pose pose_from_se3(const SE3& s) {
    Pose r;
    quat_to_matrix(s.q, r.R);
    for (int i = 0; i < 3; ++i) r.t[i] = s.t[i];
    return r;
}

// DirectPoseEstimationSingleLayer (src/viso.cpp:661-758), literal control flow
// (cost declared outside the loop and never reset, src/viso.cpp:673).
void direct_single_layer(const PyrView& last, const PyrView& cur, const double K[4],
                         const double* points, int n, const Pose& last_pose, SE3& T21, int level,
                         double* stats) {
    const double delta_thresh = 0.005;
    double cost = 0, lastCost = 0;
    int nGood = 0;
    SE3 best = T21;
    std::vector<double> part((size_t)n * 28);
    std::vector<double> leaf((size_t)n);
    for (int iter = 0; iter < 100; ++iter) {
        nGood = 0;
        Pose cur_pose = pose_from_se3(T21);
        double S[28];
        if (sum_literal()) {
            // M6d H = M6d::Zero(); V6d b = V6d::Zero(); running over points
            // ascending, then the patch (src/viso.cpp:682-729); the cost's
            // running sum continues across iterations (never reset, :673)
            for (int k = 0; k < 28; ++k) S[k] = 0.0;
            S[27] = cost;
            for (int i = 0; (ref_points_cond(n), i < n); ++i) {
                ref_points_at(n, i);
                if (direct_point_partials(last, cur, last_pose, cur_pose, K, points + 3 * i, level,
                                          nullptr, S))
                    ++nGood;
            }
        } else {
            for (int i = 0; (ref_points_cond(n), i < n); ++i) {
                ref_points_at(n, i);
                double* o = &part[(size_t)i * 28];
                if (direct_point_partials(last, cur, last_pose, cur_pose, K, points + 3 * i, level, o))
                    ++nGood;
                else
                    for (int k = 0; k < 28; ++k) o[k] = 0.0;
            }
            for (int k = 0; k < 28; ++k) {
                for (int i = 0; i < n; ++i) leaf[(size_t)i] = part[(size_t)i * 28 + k];
                S[k] = map_tree_sum(leaf.data(), n, 256);  // one tile per workgroup
            }
        }
        double H[36], b[6];
        int idx = 0;
        for (int a = 0; a < 6; ++a)
            for (int c = a; c < 6; ++c) {
                H[6 * a + c] = S[idx];
                H[6 * c + a] = S[idx];
                ++idx;
            }
        for (int k = 0; k < 6; ++k) b[k] = S[21 + k];
        cost = sum_literal() ? S[27] : cost + S[27];
        double inv[36], update[6];
        inverse6(H, inv);
        for (int r = 0; r < 6; ++r) {
            double s = inv[6 * r] * b[0];
            for (int c = 1; c < 6; ++c) s = s + inv[6 * r + c] * b[c];
            update[r] = s;
        }
        T21 = se3_mul(se3_exp(update), T21);
        cost /= nGood;
        if (stats) {
            stats[0] = nGood;
            stats[1] = cost;
            for (int k = 0; k < 36; ++k) stats[2 + k] = H[k];
            for (int k = 0; k < 6; ++k) stats[38 + k] = b[k];
            for (int k = 0; k < 6; ++k) stats[44 + k] = update[k];
        }
        if (std::isnan(update[0])) {
            T21 = best;
            break;
        }
        if (iter > 0 && cost > lastCost) {
            T21 = best;
            break;
        }
        if ((1 - cost / (double)lastCost) < delta_thresh) break;
        best = T21;
        lastCost = cost;
    }
}

// Optional per-iteration trace of LKAlignment (analysis tooling only,
// tools/lk_trace.py): rows of (point, level, iter, X, Y, cost) where (X, Y)
// is the patch origin's current-image coordinate the iteration samples at.
struct LkTrace {
    double* buf = nullptr;
    long cap = 0, n = 0;
    int point = -1;
};
LkTrace& lk_trace() {
    static LkTrace t;
    return t;
}

// LKAlignmentSingle for one pair at one level (src/viso.cpp:855-918)
void lk_pair_level(const PyrView& ref, const PyrView& cur, int level, const double uv_ref[2],
                   double uv_cur[2], bool& succ_out, double thresh) {
    const double s = kScales[level];
    const double hp = 4.0;
    const int rw = ref.w[level], rh = ref.h[level];
    const uint8_t* R = ref.level(level);
    const uint8_t* C = cur.level(level);
    double dx = 0, dy = 0;
    double cost = 0, lastCost = 0;
    bool succ = true;
    double hxx[64], hxy[64], hyx[64], hyy[64], b0[64], b1[64], cc[64];
    for (int iter = 0; iter < 100; ++iter) {
        cost = 0;
        if (!is_inside(uv_ref[0] * s + dx - hp, uv_ref[1] * s + dy - hp, rw, rh) ||
            !is_inside(uv_ref[0] * s + dx + hp, uv_ref[1] * s + dy + hp, rw, rh)) {
            succ = false;
            break;
        }
        for (int x = -4; x < 4; ++x)
            for (int y = -4; y < 4; ++y) {
                const int p = (x + 4) * 8 + (y + 4);
                double gx, gy;
                gradient(R, rw, rh, uv_ref[0] * s + x, uv_ref[1] * s + y, gx, gy);
                const double J0 = -gx, J1 = -gy;
                const double error =
                    sample(R, rw, rh, uv_ref[0] * s + x, uv_ref[1] * s + y) -
                    sample(C, cur.w[level], cur.h[level], uv_cur[0] * s + x + dx, uv_cur[1] * s + y + dy);
                hxx[p] = J0 * J0;
                hxy[p] = J0 * J1;
                hyx[p] = J1 * J0;
                hyy[p] = J1 * J1;
                b0[p] = -J0 * error;
                b1[p] = -J1 * error;
                cc[p] = error * error;
            }
        const double H00 = acc_sum(hxx, 64), H01 = acc_sum(hxy, 64), H10 = acc_sum(hyx, 64),
                     H11 = acc_sum(hyy, 64);
        // the per-iteration sums by the descending-stride tree (device
        // wave_tree_sum3_desc); H keeps the ascending tree (device lk_prepare)
        const double B0 = acc_sum_desc64(b0), B1 = acc_sum_desc64(b1);
        cost = acc_sum_desc64(cc);
        if (lk_trace().buf && lk_trace().n < lk_trace().cap) {
            double* r = lk_trace().buf + 6 * lk_trace().n++;
            r[0] = lk_trace().point;
            r[1] = level;
            r[2] = iter;
            r[3] = uv_cur[0] * s + dx;
            r[4] = uv_cur[1] * s + dy;
            r[5] = cost;
        }
        const double invdet = 1.0 / (H00 * H11 - H10 * H01);
        const double i00 = H11 * invdet, i10 = -H10 * invdet, i01 = -H01 * invdet, i11 = H00 * invdet;
        const double u0 = i00 * B0 + i01 * B1;
        const double u1 = i10 * B0 + i11 * B1;
        if (std::isnan(u0)) {
            succ = false;
            break;
        }
        if (iter > 0 && cost > lastCost) break;
        dx += u0;
        dy += u1;
        lastCost = cost;
        succ = !(lastCost > thresh);
    }
    succ_out = succ;
    uv_cur[0] = uv_cur[0] + dx / s;  // pair.uv_cur += V2d{dx/s, dy/s} (src/viso.cpp:917)
    uv_cur[1] = uv_cur[1] + dy / s;
}

}  // namespace

namespace oracle {
void direct_layer(const uint8_t* last_pyr, const uint8_t* cur_pyr, int w, int h, const double* K,
                  const double* points, int n, const double* pose_last12, SE3& T21, int level,
                  double* stats) {
    PyrView L = make_view(last_pyr, w, h), C = make_view(cur_pyr, w, h);
    direct_single_layer(L, C, K, points, n, pose_from12(pose_last12), T21, level, stats);
}
}  // namespace oracle

extern "C" {

void oracle_set_sum_order(int literal) { sum_literal() = literal ? 1 : 0; }
int oracle_get_sum_order(void) { return sum_literal(); }

void oracle_klt(const uint8_t* ref_pyr, const uint8_t* cur_pyr, int w, int h, const float* kp1,
                float* kp2, uint8_t* success, int n, double photometric_thresh) {
    PyrView R = make_view(ref_pyr, w, h), C = make_view(cur_pyr, w, h);
    // kp2[j].pt *= scales[3]  (cv::Point2f *= double -> saturate_cast<float>(x * b))
    for (int j = 0; j < n; ++j) {
        kp2[2 * j] = (float)((double)kp2[2 * j] * kScales[3]);
        kp2[2 * j + 1] = (float)((double)kp2[2 * j + 1] * kScales[3]);
    }
    std::vector<float> kp1s((size_t)2 * n);
    for (int level = kLevels - 1; level >= 0; --level) {
        for (int j = 0; j < 2 * n; ++j) kp1s[(size_t)j] = (float)((double)kp1[j] * kScales[level]);
        klt_single_level(R.level(level), C.level(level), R.w[level], R.h[level], kp1s.data(), kp2,
                         success, n, photometric_thresh);
        if (level != 0)
            for (int j = 0; j < 2 * n; ++j) kp2[j] = (float)((double)kp2[j] / 0.5);
    }
}

void oracle_set_reference_copies(int on) { ref_copies().on = on != 0; }

void oracle_lk_trace(double* buf, long cap) {
    lk_trace().buf = buf;
    lk_trace().cap = cap;
    lk_trace().n = 0;
}
long oracle_lk_trace_count(void) { return lk_trace().n; }

void oracle_se3_exp_left(const double xi[6], const double pose_in[12], double pose_out[12]) {
    SE3 a = se3_from_Rt(pose_in, pose_in + 9);
    SE3 r = se3_mul(se3_exp(xi), a);
    Pose p = pose_from_se3(r);
    for (int i = 0; i < 9; ++i) pose_out[i] = p.R[i];
    for (int i = 0; i < 3; ++i) pose_out[9 + i] = p.t[i];
}

void oracle_direct_pose_level(const uint8_t* last_pyr, const uint8_t* cur_pyr, int w, int h,
                              const double K[4], const double* points, int n_points,
                              const double pose_last[12], double pose_io[12], int level,
                              double* stats_out) {
    PyrView L = make_view(last_pyr, w, h), C = make_view(cur_pyr, w, h);
    SE3 T21 = se3_from_Rt(pose_io, pose_io + 9);
    direct_single_layer(L, C, K, points, n_points, pose_from12(pose_last), T21, level, stats_out);
    Pose p = pose_from_se3(T21);
    for (int i = 0; i < 9; ++i) pose_io[i] = p.R[i];
    for (int i = 0; i < 3; ++i) pose_io[9 + i] = p.t[i];
}

void oracle_direct_pose(const uint8_t* last_pyr, const uint8_t* cur_pyr, int w, int h,
                        const double K[4], const double* points, int n_points,
                        const double pose_last[12], double pose_io[12]) {
    PyrView L = make_view(last_pyr, w, h), C = make_view(cur_pyr, w, h);
    // Sophus::SE3d X(last_frame->GetR(), last_frame->GetT()) (src/viso.cpp:114)
    SE3 T21 = se3_from_Rt(pose_io, pose_io + 9);
    for (int level = 3; level >= 0; --level)
        direct_single_layer(L, C, K, points, n_points, pose_from12(pose_last), T21, level, nullptr);
    Pose p = pose_from_se3(T21);
    for (int i = 0; i < 9; ++i) pose_io[i] = p.R[i];
    for (int i = 0; i < 3; ++i) pose_io[9 + i] = p.t[i];
}

void oracle_lk_align(const uint8_t* const* kf_pyrs, const double* kf_poses, int n_kf,
                     const uint8_t* cur_pyr, const double cur_pose[12], int w, int h,
                     const double K[4], const double* points, int n_points,
                     double photometric_thresh, int32_t* pair_kf, uint8_t* success,
                     double* uv_before, double* uv_after) {
    PyrView C = make_view(cur_pyr, w, h);
    Pose cp = pose_from12(cur_pose);
    const double max_angle = 180.0;
    const double kPi = 3.14159265358979323846;  // CV_PI
    for (int i = 0; (ref_points_cond(n_points), i < n_points); ++i) {
        ref_points_at(n_points, i);
        const double* Pw = points + 3 * i;
        pair_kf[i] = -1;
        success[i] = 0;
        uv_before[2 * i] = uv_before[2 * i + 1] = 0.0;
        uv_after[2 * i] = uv_after[2 * i + 1] = 0.0;
        double uc, vc;
        project(cp, K, Pw, 0, uc, vc);
        if (!is_inside(uc, vc, w, h)) continue;  // current_frame->IsInside(Pw, 0)
        ref_keyframes(n_kf);                     // auto keyframes = map_.Keyframes()
        double best_angle = 180.0;
        int best = -1;
        double best_uv[2] = {0, 0};
        for (int j = 0; j < n_kf; ++j) {
            Pose kp = pose_from12(kf_poses + 12 * j);
            double ur, vr;
            project(kp, K, Pw, 0, ur, vr);
            if (!is_inside(ur, vr, w, h)) continue;
            // Keyframe::ViewingAngle (include/keyframe.h:93-98)
            double Pc[3];
            mat3_vec(kp.R, Pw, Pc);
            Pc[0] = Pc[0] + kp.t[0];
            Pc[1] = Pc[1] + kp.t[1];
            Pc[2] = Pc[2] + kp.t[2];
            double nrm = (Pc[0] * Pc[0] + Pc[1] * Pc[1]) + Pc[2] * Pc[2];
            if (nrm > 0) {
                double s = std::sqrt(nrm);
                Pc[0] = Pc[0] / s;
                Pc[1] = Pc[1] / s;
                Pc[2] = Pc[2] / s;
            }
            double angle = std::fabs(std::acos(Pc[2]) / kPi * 180);
            if (angle > max_angle || angle > best_angle) continue;
            best_angle = angle;
            best = j;
            best_uv[0] = ur;
            best_uv[1] = vr;
        }
        if (best == -1) continue;
        pair_kf[i] = best;
        double uvc[2] = {uc, vc};
        uv_before[2 * i] = uc;
        uv_before[2 * i + 1] = vc;
        PyrView R = make_view(kf_pyrs[best], w, h);
        lk_trace().point = i;
        bool succ = false;
        for (int level = kLevels - 1; level >= 0; --level)
            lk_pair_level(R, C, level, best_uv, uvc, succ, photometric_thresh);
        success[i] = succ ? 1 : 0;
        uv_after[2 * i] = uvc[0];
        uv_after[2 * i + 1] = uvc[1];
    }
}

}  // extern "C"
