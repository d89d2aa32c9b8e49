// TEST INFRASTRUCTURE ONLY (see viso_oracle.h) — the multi-camera photometric
// rig: the repo's own spec for SURVEY.md §8(f) row 3 ("sum per-camera H, b
// from DirectPoseEstimationSingleLayer (src/viso.cpp:682-729) through rig
// extrinsics"); the reference has a single camera, so parity is GPU vs this
// restatement (viso_amd/csrc/direct.hip rig_level_kernel).
//
// Spec.  Rig pose T: world -> rig; camera c sees the world at T_c = E_c T
// (E_c = (Re, te): rig -> camera).  Map points live in the world frame (the
// rig frame of the initialising timestep).  Per tracking timestep, for level
// l = 3..0, ONE Gauss-Newton step (the reference's effective behaviour: its
// cost is never reset, src/viso.cpp:673, so the loop stops after the first
// step; the cost == 0 continuation is not part of the rig spec):
//   * camera c: the 28 sums of DirectPoseEstimationSingleLayer at T_c
//     (pixel trees, then the canonical tree over the camera's points), its
//     `last` patch at E_c T_last;
//   * H = sum_c Ad_c^T H_c Ad_c, b = sum_c Ad_c^T b_c, cost = sum_c cost_c,
//     nGood = sum_c nGood_c, cameras ascending (left fold), with
//     Ad(E) = [[Re, [te]x Re], [0, Re]] for xi = (upsilon, omega) (Sophus
//     SE3::Adj, the ordering of dPixeldXi, src/viso.cpp:640-658): a rig
//     perturbation exp(xi) T moves camera c by exp(Ad_c xi);
//     M = H_c Ad_c (k ascending), entry (i, j) = sum_k Ad_c[k][i] M[k][j];
//   * update = H^-1 b (Eigen PartialPivLU inverse, as the direct pose),
//     T = exp(update) * T unless update[0] is NaN.
// Initialisation: the first timestep with right images gives every camera
// FAST + stereo points (oracle_stereo_points, the single-camera stereo
// init), taken to the world frame X = Re^T (X_c - te); more than 50 points
// in all start tracking at T = I.  The first tracking timestep seeds T from
// the identity, later ones from the last rig pose (SE3(R, t), as
// src/viso.cpp:114).
#include <cmath>
#include <cstring>
#include <memory>
#include <vector>

#include "oracle_common.hpp"
#include "oracle_linalg.hpp"
#include "oracle_se3.hpp"
#include "viso_oracle.h"

namespace oracle {
bool direct_point_partials(const PyrView& last, const PyrView& cur, const Pose& last_pose,
                           const Pose& cur_pose, const double K[4], const double* P, int level,
                           double out[28], double* running);
}

using namespace oracle;

extern "C" {

// Tc = E T: Rc = Re R, tc = Re t + te (the device's rig_compose)
void oracle_rig_compose(const double E[12], const double T[12], double out[12]) {
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j)
            out[3 * i + j] = (E[3 * i] * T[j] + E[3 * i + 1] * T[3 + j]) + E[3 * i + 2] * T[6 + j];
        out[9 + i] = ((E[3 * i] * T[9] + E[3 * i + 1] * T[10]) + E[3 * i + 2] * T[11]) + E[9 + i];
    }
}

// Ad(E) row-major 6x6: [[Re, S Re], [0, Re]], S = [te]x, (S Re)[i][j] =
// (S[i][0] Re[0][j] + S[i][1] Re[1][j]) + S[i][2] Re[2][j]
void oracle_rig_adjoint(const double E[12], double Ad[36]) {
    const double* R = E;
    const double tx = E[9], ty = E[10], tz = E[11];
    const double S[9] = {0.0, -tz, ty, tz, 0.0, -tx, -ty, tx, 0.0};
    for (int k = 0; k < 36; ++k) Ad[k] = 0.0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            Ad[6 * i + j] = R[3 * i + j];
            Ad[6 * (i + 3) + (j + 3)] = R[3 * i + j];
            Ad[6 * i + (j + 3)] = (S[3 * i] * R[j] + S[3 * i + 1] * R[3 + j]) + S[3 * i + 2] * R[6 + j];
        }
}

}  // extern "C"

namespace {

Pose pose_of12(const double* p) {
    Pose r;
    for (int i = 0; i < 9; ++i) r.R[i] = p[i];
    for (int i = 0; i < 3; ++i) r.t[i] = p[9 + i];
    return r;
}

void pose12_of_se3(const SE3& s, double* out) {
    quat_to_matrix(s.q, out);
    for (int i = 0; i < 3; ++i) out[9 + i] = s.t[i];
}

// Camera c's 28 canonical sums at cur_pose (the two-level map tree over its
// points in tiles of `tile` points: the device's workgroup tiles); returns
// nGood
int camera_sums(const PyrView& last, const PyrView& cur, const double K[4], const double* points, int n,
                const Pose& last_pose, const Pose& cur_pose, int level, int tile, double S[28]) {
    std::vector<double> part((size_t)n * 28), leaf((size_t)n);
    int good = 0;
    for (int i = 0; i < n; ++i) {
        double* o = &part[(size_t)i * 28];
        if (direct_point_partials(last, cur, last_pose, cur_pose, K, points + 3 * i, level, o, nullptr))
            ++good;
        else
            for (int k = 0; k < 28; ++k) o[k] = 0.0;
    }
    for (int k = 0; k < 28; ++k) {
        for (int i = 0; i < n; ++i) leaf[(size_t)i] = part[(size_t)i * 28 + k];
        S[k] = map_tree_sum_tiles(leaf.data(), n, tile);
    }
    return good;
}

// Ad^T H_c Ad (21 upper entries), Ad^T b_c, cost_c: the device's rig_combine
void transform_sums(const double Ad[36], const double S[28], double out[28]) {
    double H[36], M[36];
    int idx = 0;
    for (int a = 0; a < 6; ++a)
        for (int c = a; c < 6; ++c) {
            H[6 * a + c] = S[idx];
            H[6 * c + a] = S[idx];
            ++idx;
        }
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) {
            double m = H[6 * i] * Ad[j];
            for (int k = 1; k < 6; ++k) m = m + H[6 * i + k] * Ad[6 * k + j];
            M[6 * i + j] = m;
        }
    idx = 0;
    for (int i = 0; i < 6; ++i)
        for (int j = i; j < 6; ++j) {
            double v = Ad[i] * M[j];
            for (int k = 1; k < 6; ++k) v = v + Ad[6 * k + i] * M[6 * k + j];
            out[idx++] = v;
        }
    for (int i = 0; i < 6; ++i) {
        double v = Ad[i] * S[21];
        for (int k = 1; k < 6; ++k) v = v + Ad[6 * k + i] * S[21 + k];
        out[21 + i] = v;
    }
    out[27] = S[27];
}

}  // namespace

extern "C" {

// One rig direct pose (levels 3..0) of one timestep: pose_io = the seed rig
// pose in, the result out (12).  pyramids: n_cams continuous pyramids each;
// points[c] (n_points[c] x 3, world); cam_last: n_cams x 12 `last` poses;
// stats (may be null): [4][50] per level as the direct pose's.
void oracle_rig_direct(int n_cams, const uint8_t* const* last_pyrs, const uint8_t* const* cur_pyrs, int w,
                       int h, const double K[4], const double* const* points, const int* n_points,
                       const double* extrinsics, const double* cam_last, double pose_io[12], double* stats) {
    std::vector<PyrView> L, C;
    std::vector<std::vector<double>> Ad((size_t)n_cams, std::vector<double>(36));
    for (int c = 0; c < n_cams; ++c) {
        L.push_back(make_view(last_pyrs[c], w, h));
        C.push_back(make_view(cur_pyrs[c], w, h));
        oracle_rig_adjoint(extrinsics + 12 * c, Ad[(size_t)c].data());
    }
    SE3 T = se3_from_Rt(pose_io, pose_io + 9);
    // one tile size for every camera, from the rig's total map: the cameras'
    // tiles then fill the device's 256 workgroups in proportion to their
    // points (a one-camera rig tiles exactly as the direct pose)
    int n_total = 0;
    for (int c = 0; c < n_cams; ++c) n_total += n_points[c];
    const int tile = map_tile(n_total, 256);
    for (int level = 3; level >= 0; --level) {
        double T12[12];
        pose12_of_se3(T, T12);
        double acc[28] = {0};
        int ngood = 0;
        for (int c = 0; c < n_cams; ++c) {
            double Tc[12];
            oracle_rig_compose(extrinsics + 12 * c, T12, Tc);
            double S[28], V[28];
            ngood += camera_sums(L[(size_t)c], C[(size_t)c], K, points[c], n_points[c],
                                 pose_of12(cam_last + 12 * c), pose_of12(Tc), level, tile, S);
            transform_sums(Ad[(size_t)c].data(), S, V);
            for (int k = 0; k < 28; ++k) acc[k] = c == 0 ? V[k] : acc[k] + V[k];
        }
        double H[36], b[6];
        int idx = 0;
        for (int a = 0; a < 6; ++a)
            for (int c = a; c < 6; ++c) {
                H[6 * a + c] = acc[idx];
                H[6 * c + a] = acc[idx];
                ++idx;
            }
        for (int k = 0; k < 6; ++k) b[k] = acc[21 + k];
        double inv[36], update[6];
        inverse6(H, inv);
        for (int r = 0; r < 6; ++r) {
            double s = inv[6 * r] * b[0];
            for (int c = 1; c < 6; ++c) s = s + inv[6 * r + c] * b[c];
            update[r] = s;
        }
        if (stats) {
            double* st = stats + 50 * level;
            st[0] = ngood;
            st[1] = acc[27] / ngood;
            for (int k = 0; k < 36; ++k) st[2 + k] = H[k];
            for (int k = 0; k < 6; ++k) st[38 + k] = b[k];
            for (int k = 0; k < 6; ++k) st[44 + k] = update[k];
        }
        if (!std::isnan(update[0])) T = se3_mul(se3_exp(update), T);
    }
    pose12_of_se3(T, pose_io);
}

}  // extern "C"

// ---------------------------------------------------------------- rig sequence
struct oracle_rig {
    int n = 0, w = 0, h = 0;
    double K[4] = {0};
    int fast_thresh = 50;
    double base = 0.0;
    int max_disp = 128, min_disp = 1;
    std::vector<double> E;                       // n x 12
    std::vector<std::vector<uint8_t>> last_pyr;  // per camera
    std::vector<std::vector<double>> points;     // per camera, world
    std::vector<double> cam_last;                // n x 12
    double T_last[12] = {1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0};
    int state = 0;  // 0 initialising, 1 running
    std::vector<double> poses;
    double stats[200] = {0};
};

extern "C" {

oracle_rig* oracle_rig_create(int n_cams, int w, int h, const double K[4], int fast_thresh, const double* extrinsics,
                              double baseline, int max_disp, int min_disp) {
    if (n_cams < 1) return nullptr;
    auto* r = new oracle_rig;
    r->n = n_cams;
    r->w = w;
    r->h = h;
    for (int k = 0; k < 4; ++k) r->K[k] = K[k];
    r->fast_thresh = fast_thresh;
    r->E.assign(extrinsics, extrinsics + 12 * (size_t)n_cams);
    r->base = baseline;
    r->max_disp = max_disp;
    r->min_disp = min_disp;
    r->last_pyr.resize((size_t)n_cams);
    r->points.resize((size_t)n_cams);
    r->cam_last.assign(12 * (size_t)n_cams, 0.0);
    return r;
}

void oracle_rig_destroy(oracle_rig* r) { delete r; }

// One timestep: lefts[c], rights[c] (rights may be null while tracking)
void oracle_rig_process(oracle_rig* r, const uint8_t* const* lefts, const uint8_t* const* rights) {
    const int w = r->w, h = r->h;
    std::vector<std::vector<uint8_t>> cur((size_t)r->n);
    for (int c = 0; c < r->n; ++c) {
        cur[(size_t)c].resize(oracle_pyramid_bytes(w, h));
        oracle_pyramid(lefts[c], w, h, cur[(size_t)c].data());
    }
    if (r->state == 0) {
        if (rights) {
            int total = 0;
            std::vector<std::vector<double>> pts((size_t)r->n);
            for (int c = 0; c < r->n; ++c) {
                std::vector<int32_t> xs((size_t)w * h / 4 + 16), ys(xs.size()), sc(xs.size());
                const int nf = oracle_fast(cur[(size_t)c].data(), w, h, r->fast_thresh, xs.data(), ys.data(),
                                           sc.data(), (int)xs.size());
                std::vector<double> p((size_t)3 * nf + 3);
                const int m = oracle_stereo_points(cur[(size_t)c].data(), rights[c], w, h, xs.data(), ys.data(), nf,
                                                   r->max_disp, r->min_disp, r->K, r->base, p.data());
                // camera -> world (the rig frame at T = I): X = Re^T (X_c - te)
                const double* E = &r->E[12 * (size_t)c];
                pts[(size_t)c].resize((size_t)3 * m);
                for (int i = 0; i < m; ++i) {
                    const double d0 = p[3 * (size_t)i] - E[9], d1 = p[3 * (size_t)i + 1] - E[10],
                                 d2 = p[3 * (size_t)i + 2] - E[11];
                    for (int k = 0; k < 3; ++k)
                        pts[(size_t)c][3 * (size_t)i + k] = (E[k] * d0 + E[3 + k] * d1) + E[6 + k] * d2;
                }
                total += m;
            }
            if (total > 50) {
                r->points = pts;
                r->state = 1;
                const double I[12] = {1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0};
                std::memcpy(r->T_last, I, sizeof(I));
                for (int c = 0; c < r->n; ++c) oracle_rig_compose(&r->E[12 * (size_t)c], I, &r->cam_last[12 * (size_t)c]);
            }
        }
    } else {
        std::vector<const uint8_t*> lp((size_t)r->n), cp((size_t)r->n);
        std::vector<const double*> pp((size_t)r->n);
        std::vector<int> np((size_t)r->n);
        for (int c = 0; c < r->n; ++c) {
            lp[(size_t)c] = r->last_pyr[(size_t)c].data();
            cp[(size_t)c] = cur[(size_t)c].data();
            pp[(size_t)c] = r->points[(size_t)c].data();
            np[(size_t)c] = (int)(r->points[(size_t)c].size() / 3);
        }
        double pose[12];
        std::memcpy(pose, r->T_last, sizeof(pose));
        oracle_rig_direct(r->n, lp.data(), cp.data(), w, h, r->K, pp.data(), np.data(), r->E.data(),
                          r->cam_last.data(), pose, r->stats);
        std::memcpy(r->T_last, pose, sizeof(pose));
        for (int c = 0; c < r->n; ++c) oracle_rig_compose(&r->E[12 * (size_t)c], pose, &r->cam_last[12 * (size_t)c]);
        r->poses.insert(r->poses.end(), pose, pose + 12);
    }
    for (int c = 0; c < r->n; ++c) r->last_pyr[(size_t)c] = std::move(cur[(size_t)c]);
}

int oracle_rig_state(const oracle_rig* r) { return r->state; }
int oracle_rig_num_poses(const oracle_rig* r) { return (int)(r->poses.size() / 12); }
void oracle_rig_poses(const oracle_rig* r, double* out12) {
    std::memcpy(out12, r->poses.data(), sizeof(double) * r->poses.size());
}
int oracle_rig_num_points(const oracle_rig* r, int cam) { return (int)(r->points[(size_t)cam].size() / 3); }
void oracle_rig_points(const oracle_rig* r, int cam, double* out3) {
    std::memcpy(out3, r->points[(size_t)cam].data(), sizeof(double) * r->points[(size_t)cam].size());
}
void oracle_rig_level_stats(const oracle_rig* r, double* out200) { std::memcpy(out200, r->stats, sizeof(r->stats)); }

}  // extern "C"
