/* viso_amd — north-star stereo visual odometry (SVO), C ABI.
 *
 * The north star names a stereo path the reference does not contain
 * ("North_star stages with NO reference counterpart"): blob /
 * checkerboard-corner features with non-maximum suppression, SAD descriptors
 * on Sobel responses, circular stereo + temporal matching, bucketing, and
 * RANSAC + Gauss-Newton minimisation of the stereo reprojection error, behind
 * VisualOdometryStereo::process(left, right, dims) / Matcher.  The spec is
 * this repo's own and its CPU restatement is oracle/oracle_svo.cpp;
 * parity is GPU vs that restatement ("parity unpinned vs reference").
 *
 * Conventions as in viso_c.h: int return codes (VISO_OK / VISO_ERR_*), the
 * caller owns host buffers, a context is bound to one HIP device and one
 * stream and is not thread-safe.
 */
#ifndef VISO_SVO_H
#define VISO_SVO_H

#include <stddef.h>
#include <stdint.h>

#include "viso_c.h"

#ifdef __cplusplus
extern "C" {
#endif

/* feature classes (the four NMS maps) */
#define VISO_SVO_BLOB_MAX 0
#define VISO_SVO_BLOB_MIN 1
#define VISO_SVO_CORNER_MAX 2
#define VISO_SVO_CORNER_MIN 3
#define VISO_SVO_DESC_BYTES 32
#define VISO_SVO_MAX_CAMS 8      /* stereo cameras of a rig */

typedef struct viso_svo_params {
    int32_t width, height;       /* rectified grey pair size (continuous rows) */
    double fx, fy, cu, cv;       /* left camera intrinsics (right: same, shifted by base) */
    double base;                 /* stereo baseline [m] */
    int32_t nms_n;               /* NMS window radius: (2n+1)^2 window (5) */
    int32_t nms_tau;             /* response threshold of all four classes (700) */
    int32_t margin;              /* features only at margin <= u < w-margin, same for v (8) */
    int32_t disp_max;            /* stereo search: 0 <= u_left - u_right <= disp_max (255) */
    int32_t match_radius;        /* temporal search: |du|, |dv| <= radius (96) */
    int32_t bucket_width;        /* bucketing grid over the current left image (50) */
    int32_t bucket_height;       /* (50) */
    int32_t bucket_max;          /* matches kept per bucket, lowest left index first (4) */
    int32_t ransac_iters;        /* hypotheses (200) */
    int32_t gn_iters;            /* Gauss-Newton iterations cap (20) */
    double inlier_threshold;     /* stereo reprojection error [px] (2.0) */
    double gn_eps;               /* convergence: max |update| below this (1e-6) */
    uint64_t seed;               /* RANSAC sampler seed (mixed with the frame index) */
    int32_t max_features;        /* per-image feature capacity (16384) */
    int32_t reserved[7];
} viso_svo_params;

typedef struct viso_svo viso_svo;

int viso_svo_default_params(viso_svo_params* p, int32_t width, int32_t height, double fx,
                            double fy, double cu, double cv, double base);

/* VisualOdometryStereo(param) on HIP device `device`. */
int viso_svo_create(const viso_svo_params* p, int device, viso_svo** out);
int viso_svo_destroy(viso_svo* s);

/* VisualOdometryStereo::process(left, right, dims): dims = {width, height,
 * stride}.  Uploads the pair, extracts features of both images, and from the
 * second call on matches against the previous pair and estimates the motion.
 * *ok (may be NULL) = 1 if a motion was estimated (>= 6 inliers). */
int viso_svo_process(viso_svo* s, const uint8_t* left, const uint8_t* right,
                     const int32_t dims[3], int32_t* ok);

/* The same for n pairs already in HBM (device pointers, `stride` bytes per
 * row, consecutive pairs `pair_stride` bytes apart); no host round trip per
 * pair: motions and poses accumulate on the device. */
int viso_svo_process_device(viso_svo* s, const uint8_t* left, const uint8_t* right, int32_t n,
                            int64_t pair_stride, int32_t stride);
int viso_svo_synchronize(viso_svo* s);
/* HIP-event timing of the batched feature pass (detect + scan + describe of
 * the pairs of each batch): returns the time summed over the batches since
 * the previous call and their pair count (waits for the stream if any batch
 * was timed), then enables (enable != 0) or disables timing. */
int viso_svo_timing(viso_svo* s, int32_t enable, double* feature_pass_ms, int32_t* pairs);

/* Last motion Tr (camera t-1 -> camera t: P_t = R P_{t-1} + t), 12 doubles
 * (R row-major, t).  getMotion(). */
int viso_svo_get_motion(viso_svo* s, double* motion12);
/* counts of the last processed pair: [features left, features right,
 * circular matches, bucketed matches, inliers, ok] */
int viso_svo_get_stats(viso_svo* s, int32_t* stats6);
/* Accumulated camera poses (T_wc of the left camera, 12 doubles each; pose 0
 * = identity at the first pair): one per processed pair. */
int viso_svo_get_poses(viso_svo* s, double* poses12, size_t cap, size_t* n);
/* Matcher::getMatches(): the bucketed matches of the last pair:
 * per match {u_l1, v_l1, u_r1, v_r1, u_l2, v_l2, u_r2, v_r2} and its
 * inlier flag. */
int viso_svo_get_matches(viso_svo* s, int32_t* uv8, uint8_t* inlier, size_t cap, size_t* n);

/* ---- multi-camera rig (BASELINE.json configs[4]) -----------------------
 * n_cams rigidly mounted stereo cameras with identical parameters p;
 * extrinsics (n_cams x 12 doubles, R row-major + t) map the rig frame to
 * camera c's left camera: P_c = R P_rig + t.  Per timestep every camera's
 * pair runs the stereo path (features, circular matching, bucketing); one
 * RANSAC + Gauss-Newton estimates the rig motion from the matches of all
 * cameras (camera order, then left order), residuals taken through each
 * match's extrinsic.  get_motion / get_poses then report the rig's motion and
 * poses, get_stats sums over the cameras.  viso_svo_create is this with
 * n_cams = 1 (no extrinsic); the stage entry points below need n_cams = 1. */
int viso_svo_rig_create(const viso_svo_params* p, int32_t n_cams, const double* extrinsics, int device,
                        viso_svo** out);
/* one timestep: lefts[c], rights[c] = host images of camera c */
int viso_svo_rig_process(viso_svo* s, const uint8_t* const* lefts, const uint8_t* const* rights,
                         const int32_t dims[3], int32_t* ok);
/* n timesteps already in HBM: camera c's pairs at lefts[c] / rights[c]
 * (device pointers), consecutive timesteps pair_stride bytes apart */
int viso_svo_rig_process_device(viso_svo* s, const uint8_t* const* lefts, const uint8_t* const* rights,
                                int32_t n, int64_t pair_stride, int32_t stride);
/* camera of each match returned by viso_svo_get_matches */
int viso_svo_get_match_cams(viso_svo* s, uint8_t* cams, size_t cap, size_t* n);

/* ---- stage entry points (parity tests) ---------------------------------
 * Features of one image: row-major (v, then u, then class); n <= cap. */
int viso_svo_features(viso_svo* s, const uint8_t* img, int32_t width, int32_t height,
                      int32_t* u, int32_t* v, int32_t* cls, uint8_t* desc, int32_t cap,
                      int32_t* n);

/* Circular matching of four feature sets (previous left/right, current
 * left/right; arrays as produced by viso_svo_features).  Output: index
 * quadruples {l1, r1, l2, r2} in ascending l2 order, before bucketing. */
int viso_svo_match(viso_svo* s, const int32_t* const* u4, const int32_t* const* v4,
                   const int32_t* const* cls4, const uint8_t* const* desc4, const int32_t n4[4],
                   int32_t* quad, int32_t cap, int32_t* n);

/* Bucketing + RANSAC + Gauss-Newton on matches given as {u_l1, v_l1, u_r1,
 * v_r1, u_l2, v_l2, u_r2, v_r2} (already bucketed).  frame selects the
 * sampler stream.  Output: motion (12), inlier flags, *n_inliers. */
int viso_svo_estimate(viso_svo* s, const int32_t* uv8, int32_t n, int64_t frame, double* motion12,
                      uint8_t* inlier, int32_t* n_inliers);

#ifdef __cplusplus
}
#endif

#endif /* VISO_SVO_H */
