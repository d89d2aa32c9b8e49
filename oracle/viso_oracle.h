// TEST INFRASTRUCTURE ONLY — the CPU oracle for the viso_amd hot path.
//
// A single-threaded C++ restatement of the reference's per-frame path
// (Seasandwpy/viso, `Viso::OnNewFrame`, src/viso.cpp:7-145) and of the
// third-party operations it calls (OpenCV 3.x pyrDown / FAST / RANSAC
// geometry, Eigen inverse / JacobiSVD, Sophus SE3::exp).  Only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and
// only as the checker.  The product (viso_amd/) never links or calls it.
//
// PARITY STATUS: "parity unpinned" vs the reference.  The reference ships no
// tests, fixtures or golden vectors, and cannot be built here (OpenCV 3,
// Eigen3, Sophus and Pangolin are absent).  The
// integer stages are cross-checked by an independent numpy restatement
// (oracle/numpy_ref.py) and by hand-derived known answers (tests/).
//
// Spec decisions that make GPU-vs-oracle parity exact:
//  * every float expression follows the reference's operand order and is
//    compiled with -ffp-contract=off (no FMA contraction on either side);
//  * every sum over patch pixels is the canonical pairwise tree over the
//    index range padded to a power of two (leaf i+1 added to leaf i, then
//    pairs of pairs, ...), not the reference's running sum; a sum over map
//    points (direct pose, rig) is two-level: pairwise trees over tiles of
//    T = min(64, ceil(n / groups)) consecutive points, then the pairwise tree
//    over the tile sums (oracle_common.hpp map_tree_sum); skipped items are
//    +0.0 leaves;
//  * out-of-buffer bilinear taps read 0 (the reference reads past the
//    cv::Mat; include/common.h:35-41 — UB there).
#ifndef VISO_ORACLE_H
#define VISO_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// ---------------------------------------------------------------- summation order
// 0 (default): canonical pairwise tree sums (the device's order, above).
// 1: "literal" — the reference's running sums in its loop order (KLT, direct
// pose, LK alignment, disparity, mean depth).  Per calling thread; used to
// measure the drift of the tree substitution (tests/test_literal_drift.py).
void oracle_set_sum_order(int literal);
int oracle_get_sum_order(void);

// ---------------------------------------------------------------- images
// Level sizes: w_l = (int)(w_{l-1} * 0.5), h likewise (include/keyframe.h:42-43).
void oracle_pyramid_dims(int w, int h, int32_t dims_out[8]);
// Total bytes of the 4-level continuous pyramid (levels concatenated).
size_t oracle_pyramid_bytes(int w, int h);
// cv::pyrDown(src, dst, Size(dw, dh)) with BORDER_REFLECT_101 (keyframe.h:42).
void oracle_pyr_down(const uint8_t* src, int sw, int sh, uint8_t* dst, int dw, int dh);
// Keyframe::Keyframe pyramid (keyframe.h:28-46): out receives levels 0..3.
void oracle_pyramid(const uint8_t* img, int w, int h, uint8_t* out);
// cv::FAST(img, kps, thresh) TYPE_9_16 + 3x3 NMS (src/viso.cpp:104).  Writes
// row-major keypoints (x, y, score).  Returns the keypoint count (may exceed
// cap; only cap are written).
int oracle_fast(const uint8_t* img, int w, int h, int thresh, int32_t* xs, int32_t* ys,
                int32_t* scores, int cap);
// FAST score map before NMS (0 where not a corner) — diagnostic.
void oracle_fast_score_map(const uint8_t* img, int w, int h, int thresh, uint8_t* score);
// GetPixelValue (include/common.h:35-42) on a continuous u8 buffer.
double oracle_sample(const uint8_t* img, int w, int h, double x, double y);
void oracle_gradient(const uint8_t* img, int w, int h, double x, double y, double out[2]);

// ---------------------------------------------------------------- tracking
// OpticalFlowMultiLevel(..., inverse=true) (src/viso.cpp:353-391 and
// OpticalFlowSingleLevel :259-350).  kp1/kp2 are float (cv::Point2f) x,y
// interleaved; kp2 is the initial guess and is updated in place.
void oracle_klt(const uint8_t* ref_pyr, const uint8_t* cur_pyr, int w, int h,
                const float* kp1, float* kp2, uint8_t* success, int n, double photometric_thresh);

// One DirectPoseEstimationSingleLayer call (src/viso.cpp:661-758), faithful
// semantics.  pose_last/pose_io: 12 doubles = R row-major (9) + t (3).
// pose_io is the SE3 T21 (input seed, output estimate).  stats_out (may be
// NULL): [nGood, cost, H(36), b(6), update(6)].
void oracle_direct_pose_level(const uint8_t* last_pyr, const uint8_t* cur_pyr, int w, int h,
                              const double K[4], const double* points, int n_points,
                              const double pose_last[12], double pose_io[12], int level,
                              double* stats_out);
// DirectPoseEstimationMultiLayer (src/viso.cpp:760-766): levels 3..0.
void oracle_direct_pose(const uint8_t* last_pyr, const uint8_t* cur_pyr, int w, int h,
                        const double K[4], const double* points, int n_points,
                        const double pose_last[12], double pose_io[12]);
// Sophus::SE3d::exp(xi) * T (src/viso.cpp:737).  xi = [upsilon; omega].
void oracle_se3_exp_left(const double xi[6], const double pose_in[12], double pose_out[12]);

// LKAlignment (src/viso.cpp:768-843) against n_kf keyframes (pyramids +
// poses).  Per map point outputs (dense, index = map point):
//   pair_kf[i]   : chosen keyframe index or -1 (no pair)
//   success[i]   : level-0 success of the pair (0 when no pair)
//   uv_before[2i], uv_after[2i] : projection into cur / aligned position.
// The reference's by-value Map::GetPoints() / Keyframes() copies inside the
// direct-pose and LKAlignment loops (src/viso.cpp:688,690,774,776,787),
// reproduced on a mirror of the map for the copies-included CPU baseline
// (timing only; results unchanged).  Off by default.
void oracle_set_reference_copies(int on);
// Analysis tooling: record LKAlignment's iterations into buf (6 doubles per
// row: point, level, iter, X, Y, cost; at most cap rows); buf NULL disables.
void oracle_lk_trace(double* buf, long cap);
long oracle_lk_trace_count(void);
void oracle_lk_align(const uint8_t* const* kf_pyrs, const double* kf_poses, int n_kf,
                     const uint8_t* cur_pyr, const double cur_pose[12], int w, int h,
                     const double K[4], const double* points, int n_points,
                     double photometric_thresh, int32_t* pair_kf, uint8_t* success,
                     double* uv_before, double* uv_after);

// ---------------------------------------------------------------- geometry
// Viso::Triangulate (src/viso.cpp:416-431): P1 = [I|0], P2 = [R|T].
void oracle_triangulate(const double R[9], const double T[3], const double x1[3],
                        const double x2[3], double P[3]);

// RANSAC estimators (the repo's deterministic restatement of
// cv::findEssentialMat / cv::findHomography).
// p1,p2: n x 2 doubles (float-rounded normalised coordinates).
// Returns the number of inliers of the best model (0 => no model).
int oracle_ransac_essential(const double* p1, const double* p2, int n, double thresh,
                            double confidence, int max_iters, uint64_t seed, double E_out[9],
                            uint8_t* mask_out, int32_t* iters_out);
int oracle_ransac_homography(const double* p1, const double* p2, int n, double thresh,
                             double confidence, int max_iters, uint64_t seed, double H_out[9],
                             uint8_t* mask_out, int32_t* iters_out);
// cv::recoverPose(E, p1, p2, R, t, 1.0, (0,0), mask) restated; mask in/out.
int oracle_recover_pose(const double E[9], const double* p1, const double* p2, int n,
                        uint8_t* mask, double R_out[9], double t_out[3]);
// cv::decomposeHomographyMat(H, I, ...) restated (INRIA method).  Returns the
// number of solutions (1 or 4); Rs: 9 per solution, ts, ns: 3 per solution.
int oracle_decompose_homography(const double H[9], double* Rs, double* ts, double* ns);

// Viso::SelectMotion (src/viso.cpp:520-638).  Rs: m x 9, Ts: m x 3.
// Outputs: best motion index (-1 none), R_out/T_out (T normalised by mean
// depth), inliers (n), points3d (n x 3, zero rows for outliers; the
// reference's compacted list is points3d[inliers]).  Returns nr_inliers.
int oracle_select_motion(const double* p1, const double* p2, int n, const double* Rs,
                         const double* Ts, int m, const double K[4], double proj_thresh,
                         double parallax_thresh, int32_t* best_out, double R_out[9],
                         double T_out[3], uint8_t* inliers, double* points3d);

// North-star stereo SAD stage (no reference counterpart; the repo's own spec,
// viso_amd/csrc/stereo.hip): 8x8 SAD along the row, d = 0..max_disp while
// x - d - 4 >= 0, smallest SAD wins, ties -> smallest d; -1 when the left
// patch leaves the image.
void oracle_stereo_match(const uint8_t* L, const uint8_t* R, int w, int h, const int32_t* xs,
                         const int32_t* ys, int n, int max_disp, int32_t* disp, int32_t* best_sad);

// Stereo initialisation points (the repo's own spec, see oracle_stereo.cpp):
// camera-frame points of the keypoints with a valid sub-pixel disparity, in
// keypoint order; returns their count (pts: n x 3 capacity).
int oracle_stereo_points(const uint8_t* L, const uint8_t* R, int w, int h, const int32_t* xs,
                         const int32_t* ys, int n, int max_disp, int min_disp, const double K[4],
                         double base, double* pts);

// ---------------------------------------------------------------- full path
struct oracle_params;
// Viso::PoseEstimation2d2d (src/viso.cpp:178-256) + SelectMotion on n x 3
// normalised points.  stats = {nr_inliers, best_motion, n_candidates,
// disparity_sq, e_inliers, h_inliers, e_iters, h_iters}; candidates <= 5 x 12.
// Returns 0 on an early return (R, T, inliers untouched), else 1.
int oracle_pose_2d2d(const double* p1, const double* p2, int n, const double K[4],
                     const struct oracle_params* prm, double R[9], double T[3], uint8_t* inliers,
                     double* points3d, double* candidates, double stats[8]);

typedef struct oracle_viso oracle_viso;
typedef struct oracle_params {
    double fx, fy, cx, cy;
    int32_t width, height;
    int32_t reinitialize_after;
    int32_t fast_thresh;
    double projection_error_thresh;
    double parallax_thresh;
    double disparity_squared_thresh;
    double photometric_error_thresh;
    int32_t enable_tracking;  // 0: as shipped (kFinished), 1: kRunning
    int32_t ransac_e_iters;
    int32_t ransac_h_iters;
    double ransac_confidence;
    uint64_t ransac_seed;
} oracle_params;

void oracle_default_params(oracle_params* p, double fx, double fy, double cx, double cy, int w,
                           int h);
oracle_viso* oracle_viso_create(const oracle_params* p);
void oracle_viso_destroy(oracle_viso* v);
// FrameHandler::OnNewFrame equivalent (level-0 grey image, continuous rows).
void oracle_viso_on_new_frame(oracle_viso* v, const uint8_t* img);
// Stereo initialisation (viso_set_stereo): baseline > 0 enables it.
void oracle_viso_set_stereo(oracle_viso* v, double baseline, int max_disp, int min_disp);
// VisualOdometryStereo::process(left, right): while initialising with stereo
// enabled, a frame whose left FAST corners give > 50 stereo points creates the
// map from them (one keyframe, identity pose, metric scale); otherwise, and
// in every other state, the left image goes through OnNewFrame.
void oracle_viso_on_new_stereo(oracle_viso* v, const uint8_t* left, const uint8_t* right);
// Stereo keyframe insertion (viso_set_keyframes; the repo's own map
// maintenance, no reference counterpart): with stereo enabled, after every
// `interval`-th tracking frame whose level-0 nGood is below
// ngood_permille / 1000 of the map size, the frame's stereo points (world =
// R^T (Pc - T)) are appended to the map and the frame becomes a keyframe (at
// most 8 keyframes, 16384 points).  interval 0 = off (default).
void oracle_viso_set_keyframes(oracle_viso* v, int interval, int ngood_permille);
// Photometric BA (oracle_photometric_ba) over every keyframe and the map after
// each keyframe insertion, `iterations` LM iterations (0 = off, default); the
// refined keyframe poses replace the keyframes' (keyframe 0 fixed).
void oracle_viso_set_bundle_adjust(oracle_viso* v, int iterations);
int oracle_viso_state(const oracle_viso* v);
int oracle_viso_num_poses(const oracle_viso* v);
void oracle_viso_poses(const oracle_viso* v, double* out12);
int oracle_viso_num_points(const oracle_viso* v);
void oracle_viso_points(const oracle_viso* v, double* out3);
// Per-frame diagnostics of the last frame: [state, n_tracked, nr_inliers,
// best_motion, n_candidates, frame_cnt, n_alignment, n_align_success,
// disparity_sq (as int bits? no: see oracle), ...]
void oracle_viso_last_stats(const oracle_viso* v, double* out16);
// Current init tracks (kp1, kp2 float x,y) and success flags.
int oracle_viso_tracks(const oracle_viso* v, float* kp1, float* kp2, uint8_t* success, int cap);
// Map keyframe poses (12 doubles each); returns the keyframe count.
int oracle_viso_keyframe_poses(const oracle_viso* v, double* out12, int cap);
// Last LK alignment outputs (dense over map points).
int oracle_viso_alignment(const oracle_viso* v, int32_t* pair_kf, uint8_t* success,
                          double* uv_before, double* uv_after, int cap);

// ---------------------------------------------------------------- multi-camera rig
// The repo's own spec for SURVEY.md §8(f) row 3 (oracle_rig.cpp header):
// rig pose T (world -> rig), camera c at E_c T (extrinsics: n x 12 rig ->
// camera, R row-major + t), per level one Gauss-Newton step whose H, b are
// the cameras' DirectPoseEstimationSingleLayer sums through Ad(E_c).
void oracle_rig_compose(const double E[12], const double T[12], double out[12]);
void oracle_rig_adjoint(const double E[12], double Ad[36]);
void oracle_rig_direct(int n_cams, const uint8_t* const* last_pyrs, const uint8_t* const* cur_pyrs, int w,
                       int h, const double K[4], const double* const* points, const int* n_points,
                       const double* extrinsics, const double* cam_last, double pose_io[12], double* stats);
typedef struct oracle_rig oracle_rig;
oracle_rig* oracle_rig_create(int n_cams, int w, int h, const double K[4], int fast_thresh, const double* extrinsics,
                              double baseline, int max_disp, int min_disp);
void oracle_rig_destroy(oracle_rig* r);
// one timestep (rights: n images, or null while tracking)
void oracle_rig_process(oracle_rig* r, const uint8_t* const* lefts, const uint8_t* const* rights);
int oracle_rig_state(const oracle_rig* r);
int oracle_rig_num_poses(const oracle_rig* r);
void oracle_rig_poses(const oracle_rig* r, double* out12);
int oracle_rig_num_points(const oracle_rig* r, int cam);
void oracle_rig_points(const oracle_rig* r, int cam, double* out3);
// [4 levels][50]: nGood, cost / nGood, H (36), b (6), update (6) of the last step
void oracle_rig_level_stats(const oracle_rig* r, double* out200);

// ---------------------------------------------------------------- photometric BA
// The repo's own spec of include/bundle_adjuster.h:22-106 (oracle_ba.cpp
// header): keyframe poses (keyframe 0 fixed) and map points, 16-residual 4x4
// patch edges point -> every non-host keyframe, Levenberg-Marquardt with the
// points marginalised.  Returns the number of active edges.
int oracle_photometric_ba(const uint8_t* const* kf_img, int n_kf, int w, int h, const double K[4], double* kf_poses,
                          double* points, const int32_t* host, int n, int iterations, double* report);

#ifdef __cplusplus
}
#endif
#endif
