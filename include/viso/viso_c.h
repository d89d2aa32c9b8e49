/* viso_amd — MI355X-native (gfx950) visual-odometry hot path, C ABI.
 *
 * This is the drop-in boundary for the reference's per-frame path
 * (Seasandwpy/viso).  Each entry point names the reference interface it
 * replaces (file:line under the reference tree).  Conventions:
 *   - every function returns int: VISO_OK (0) or a negative VISO_ERR_*;
 *     nothing throws across this boundary;
 *   - the caller owns host buffers; inputs are consumed (uploaded) before a
 *     call returns unless the name says "_device" (then the pointers are HIP
 *     device pointers that must stay valid until viso_synchronize());
 *   - a viso_ctx is bound to one HIP device and one HIP stream; it is not
 *     thread-safe; distinct contexts may run concurrently;
 *   - no C++ or torch types cross this boundary.
 */
#ifndef VISO_C_H
#define VISO_C_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VISO_OK 0
#define VISO_ERR_ARG (-1)
#define VISO_ERR_HIP (-2)
#define VISO_ERR_CAPACITY (-3)
#define VISO_ERR_STATE (-4)
#define VISO_ERR_NODEVICE (-5)

/* include/viso.h:13-17 */
#define VISO_STATE_INITIALIZATION 0
#define VISO_STATE_RUNNING 1
#define VISO_STATE_FINISHED 2

/* Constructor arguments Viso(fx, fy, cx, cy) (include/viso.h:47) plus the
 * reference's hard-coded constants (include/viso.h:20-26) and the switches
 * the reference does not have. */
typedef struct viso_params {
    double fx, fy, cx, cy;            /* include/viso.h:47-50 */
    int32_t width, height;            /* level-0 frame size (continuous rows) */
    int32_t reinitialize_after;       /* 10     include/viso.h:20 */
    int32_t fast_thresh;              /* 50     include/viso.h:21 */
    double projection_error_thresh;   /* 0.3    include/viso.h:22 */
    double parallax_thresh;           /* 1 deg  include/viso.h:23 */
    double disparity_squared_thresh;  /* 225    include/viso.h:24 */
    double photometric_error_thresh;  /* 14400  include/viso.h:26 */
    int32_t enable_tracking;          /* 0: as shipped (kFinished after init,
                                         src/viso.cpp:97); 1: kRunning */
    int32_t ransac_e_iters;           /* 1000 (OpenCV findEssentialMat default) */
    int32_t ransac_h_iters;           /* 2000 (src/viso.cpp:240) */
    double ransac_confidence;         /* 0.99 (src/viso.cpp:222,240) */
    uint64_t ransac_seed;             /* counter-RNG seed of the samplers */
    int32_t max_features;             /* capacity of FAST / KLT arrays (1..65536) */
    int32_t max_poses;                /* capacity of the pose log */
    int32_t batch_frames;             /* frames per viso_process_frames_device
                                         chunk (frame-slot pool size) */
    int32_t precision;                /* VISO_PRECISION_FAITHFUL (default) or
                                         VISO_PRECISION_FAST (tracking stages) */
    int32_t reserved[6];
} viso_params;

/* viso_params.precision.
 * FAITHFUL: fp64 wherever the reference is fp64, results bit-identical to
 *   the oracle (canonical tree sums, Eigen PartialPivLU inverse).
 * FAST: tolerance mode for the tracking stages (direct pose, LK alignment):
 *   fp32 per-pixel sampling / Jacobians / products with fp64 per-point and
 *   per-map sums, an LDL^T solve of the 6x6 normal equations; validated
 *   against the oracle at the north star's 1e-4 rel-Frobenius pose bar
 *   (tests/test_fast_mode.py).  Initialisation stages are always faithful. */
#define VISO_PRECISION_FAITHFUL 0
#define VISO_PRECISION_FAST 1

typedef struct viso_ctx viso_ctx;

/* Defaults = the reference's constants (include/viso.h:20-26). */
int viso_default_params(viso_params* p, double fx, double fy, double cx, double cy,
                        int32_t width, int32_t height);

/* Viso::Viso(fx,fy,cx,cy) (include/viso.h:47-52) on HIP device `device`. */
int viso_create(const viso_params* p, int device, viso_ctx** out);
int viso_destroy(viso_ctx* ctx);

/* FrameSequence::FrameHandler::OnNewFrame(Keyframe::Ptr)
 * (include/frame_sequence.h:13-16, implemented by Viso::OnNewFrame,
 * src/viso.cpp:7-145).  `grey`: width x height u8 rows, `stride` bytes apart
 * (copied before the call returns).  Builds the 4-level pyramid (Keyframe
 * ctor, include/keyframe.h:28-46).  Asynchronous: while tracking, the
 * frame's last pose step and its LK alignment may still be queued when the
 * call returns; every other call on the context (getters,
 * viso_synchronize, setters, stage calls, device ingest) launches them
 * first, so results read through the API are always complete.  An error of
 * that deferred work (frame k's final solve or LK batch) is returned by the
 * call that launches it — the next call on the context — not by frame k's. */
int viso_process_frame(viso_ctx* ctx, const uint8_t* grey, int32_t width, int32_t height,
                       int32_t stride);

/* North-star facade VisualOdometryStereo::process(left, right, dims):
 * dims = {width, height, stride}.  The left image drives the reference path;
 * the right image (level 0 only, no pyramid) feeds the stereo initialisation
 * and stereo keyframe insertion (viso_set_stereo).  (No reference
 * counterpart: the reference is monocular) */
int viso_process_stereo(viso_ctx* ctx, const uint8_t* left, const uint8_t* right,
                        const int32_t dims[3]);

/* Batched ingest of n consecutive frames already resident in HBM (device
 * pointers, frame f at d_left + f * frame_stride, rows continuous).  Builds
 * all left pyramids of the chunk in one batched launch, then runs OnNewFrame
 * per frame in order.  d_right may be NULL (mono).
 * Buffer contract: the frames are read in place, asynchronously, on the
 * context stream.  Their producer must have completed before the call (the
 * caller synchronises its own stream), and the buffers must stay valid and
 * unmodified until viso_synchronize(ctx) returns.  Frames the context retains
 * (reference / last / keyframes) are copied into its own pool before that. */
int viso_process_frames_device(viso_ctx* ctx, const uint8_t* d_left, const uint8_t* d_right,
                               int32_t n, size_t frame_stride);

/* Wait for all queued work of the context. */
int viso_synchronize(viso_ctx* ctx);

/* State (include/viso.h:44) */
int viso_get_state(viso_ctx* ctx, int32_t* state);
/* Viso::poses (include/viso.h:54): Tcw per tracked frame, 12 doubles each
 * (R row-major, t); the first min(cap, count, max_poses) are copied (one
 * device round trip).  *n receives the total count, which is host state: with
 * Tcw12 NULL or cap 0 the call does not touch the device. */
int viso_get_poses(viso_ctx* ctx, double* Tcw12, size_t cap, size_t* n);
/* Viso::GetPoints() (include/viso.h:60-67): map points, 3 doubles each. */
int viso_get_points(viso_ctx* ctx, double* xyz, size_t cap, size_t* n);
/* Initialisation tracks: init_.kp1 / init_.kp2 (float x,y) and
 * init_.success (include/viso.h:33-41). */
int viso_get_init_tracks(viso_ctx* ctx, float* kp1, float* kp2, uint8_t* success, size_t cap,
                         size_t* n);
/* Last LKAlignment outputs (src/viso.cpp:768-843), dense over map points:
 * pair_kf (-1 = no pair), success, uv_before, uv_after (2 doubles each). */
int viso_get_alignment(viso_ctx* ctx, int32_t* pair_kf, uint8_t* success, double* uv_before,
                       double* uv_after, size_t cap, size_t* n);
/* Per-frame statistics of the last processed frame (16 doubles):
 * [0] state, [1] tracked points, [2] nr_inliers, [3] best motion,
 * [4] candidates, [5] init frame_cnt, [6] alignment pairs,
 * [7] alignment successes, [8] disparity_squared, [9] direct-pose nGood
 * (level 0), [10] direct-pose cost (level 0), [11] frames processed,
 * [12] init succeeded on this frame, [13..15] reserved. */
int viso_get_frame_stats(viso_ctx* ctx, double stats[16]);
/* Per-frame log (structured per-frame statistics, every tracking frame
 * rather than the last one; no reference counterpart — the reference prints
 * nGood / cost per level, src/viso.cpp:755-757).  enable != 0 allocates
 * max_poses rows of 4 doubles on the device: for the tracking frame with
 * pose index k (the k-th entry of viso_get_poses), row k = {level-0 nGood,
 * level-0 cost (as viso_get_frame_stats [9], [10]), LK alignment pairs,
 * LK alignment successes (as [6], [7])}, written by the kernels themselves
 * (the direct pose's logging thread; one counting launch per LK batch);
 * rows of frames processed while it was off read NaN.  enable = 0 frees it. */
int viso_set_frame_log(viso_ctx* ctx, int32_t enable);
/* The context's execution resources (no reference counterpart), 8 ints:
 * [0] LK alignment of device-ingest chunks in the background of the direct
 *     chain (1) or batched after it (0: VISO_LK_BG=0, serialised kernels, or
 *     no side queue of its own could be made),
 * [1] the LK side stream has a hardware queue of its own (CU-masked stream),
 * [2] the host-upload stream likewise (-1: not created yet, it is made by the
 *     first host frame),
 * [3] frame slots in the pool, [4] per-frame log on, [5] batch_frames,
 * [6] level-0 bytes the last ingest's pyramid tail launch copied into the
 *     pool beside levels 2-3 (its last frame, kept as last_frame: 0 or
 *     width x height), [7] background-LK words (int32) it cleared.
 * See INTEGRATION.md §4 for the queue budget. */
int viso_get_config(viso_ctx* ctx, int32_t info[8]);
/* The first min(cap, poses) rows (4 doubles each) of the per-frame log; *n =
 * the pose count.  VISO_ERR_STATE when the log is off. */
int viso_get_frame_log(viso_ctx* ctx, double* rows, size_t cap, size_t* n);

/* Kernel timing (HIP events on the context stream) for roofline accounting.
 * kernel ids: see VISO_KERNEL_*.  When enabled, every launch of the kernel
 * is bracketed by events; viso_timing_get returns the launch count and the
 * summed milliseconds. */
#define VISO_KERNEL_PYRAMID 0
#define VISO_KERNEL_FAST 1
#define VISO_KERNEL_KLT 2
#define VISO_KERNEL_RANSAC 3
#define VISO_KERNEL_SELECT 4
#define VISO_KERNEL_DIRECT 5
#define VISO_KERNEL_LKALIGN 6
#define VISO_KERNEL_STEREO 7
#define VISO_KERNEL_UPLOAD 8 /* host -> device copy of a frame (viso_process_frame / _stereo) */
#define VISO_KERNEL_COUNT 9
/* (timing_get first launches what host-frame calls left pending, as the
 * getters do; an error of a frame's deferred work — its final solve or LK
 * batch — is returned by the next call on the context that launches it) */
int viso_timing_enable(viso_ctx* ctx, int32_t enable);
/* Restrict timing to the kernels whose bit (1 << VISO_KERNEL_*) is set
 * (default: all).  Each timed region records two events on its stream. */
int viso_timing_select(viso_ctx* ctx, uint32_t kernel_mask);
int viso_timing_get(viso_ctx* ctx, int32_t kernel, int64_t* launches, double* total_ms);

/* ------------------------------------------------------------------------
 * Stage-level entry points (host buffers in/out; synchronous).  Used by the
 * parity tests; each runs the same device kernels as the frame path.
 * ---------------------------------------------------------------------- */

/* Sizes of the 4 pyramid levels: dims[2l] = w_l, dims[2l+1] = h_l;
 * w_l = (int)(w_{l-1} * 0.5) (include/keyframe.h:42-43). */
int viso_pyramid_dims(int32_t width, int32_t height, int32_t dims[8], size_t* total_bytes);

/* Keyframe::Keyframe pyramid (include/keyframe.h:28-46) for n images at once:
 * in: n * w * h bytes; out: n * total_bytes (levels concatenated). */
int viso_pyramid(viso_ctx* ctx, const uint8_t* images, int32_t n, int32_t width, int32_t height,
                 uint8_t* out);

/* cv::FAST(img, kps, thresh) with NMS (src/viso.cpp:104): row-major
 * keypoints; *n = total count (only cap written). */
int viso_fast(viso_ctx* ctx, const uint8_t* image, int32_t width, int32_t height, int32_t thresh,
              int32_t* xs, int32_t* ys, int32_t* scores, size_t cap, size_t* n);

/* OpticalFlowMultiLevel(ref, cur, kp1, kp2, success, inverse=true)
 * (src/viso.cpp:353-391): pyramids as produced by viso_pyramid. */
int viso_klt(viso_ctx* ctx, const uint8_t* ref_pyr, const uint8_t* cur_pyr, int32_t width,
             int32_t height, const float* kp1, float* kp2, uint8_t* success, int32_t n);

/* DirectPoseEstimationMultiLayer (src/viso.cpp:760-766, one GN step per
 * level as shipped).  poses: 12 doubles (R row-major, t). */
int viso_direct_pose(viso_ctx* ctx, const uint8_t* last_pyr, const uint8_t* cur_pyr,
                     int32_t width, int32_t height, const double* points, int32_t n_points,
                     const double pose_last[12], double pose_io[12]);

/* LKAlignment (src/viso.cpp:768-843) against n_kf keyframes. */
int viso_lk_align(viso_ctx* ctx, const uint8_t* kf_pyrs, const double* kf_poses, int32_t n_kf,
                  const uint8_t* cur_pyr, const double cur_pose[12], int32_t width,
                  int32_t height, const double* points, int32_t n_points, int32_t* pair_kf,
                  uint8_t* success, double* uv_before, double* uv_after);

/* Viso::PoseEstimation2d2d (src/viso.cpp:178-256) followed by SelectMotion
 * (src/viso.cpp:520-638) on normalised coordinates p1, p2 (n x 3 doubles,
 * z = 1).  Outputs: R, T (T normalised by mean depth), inliers (n),
 * points3d (n x 3; rows of outliers are zero), candidates (<= 5 x 12),
 * stats = {nr_inliers, best_motion, n_candidates, disparity_sq,
 *          e_inliers, h_inliers, e_iters, h_iters}. */
int viso_pose_2d2d(viso_ctx* ctx, const double* p1, const double* p2, int32_t n, double R[9],
                   double T[3], uint8_t* inliers, double* points3d, double* candidates,
                   double stats[8]);

/* North-star stereo stage: for each left keypoint (x, y integer pixels) find
 * the right-image column by 8x8 SAD along the same row, disparities
 * 0..max_disp (winner = smallest SAD, ties -> smallest disparity).  Outputs
 * disparity (-1 = invalid) and best SAD.  No reference counterpart. */
int viso_stereo_match(viso_ctx* ctx, const uint8_t* left, const uint8_t* right, int32_t width,
                      int32_t height, const int32_t* xs, const int32_t* ys, int32_t n,
                      int32_t max_disp, int32_t* disparity, int32_t* sad);

/* Stereo initialisation (north star: metric depth from the right image
 * replacing the 2D-2D init of Viso::PoseEstimation2d2d, src/viso.cpp:178-256
 * and the map creation of src/viso.cpp:79-96; the repo's own spec, restated in
 * oracle/oracle_stereo.cpp).  baseline > 0 enables it (metres; 0 disables):
 * while initialising, a frame given with its right image (viso_process_stereo
 * or viso_process_frames_device with d_right) runs FAST on the left image,
 * the SAD disparity of every corner (as viso_stereo_match, d in
 * 0..min(max_disp, x - 4)), keeps corners with min_disp <= d < that upper end,
 * refines d by the parabola through SAD(d-1), SAD(d), SAD(d+1) and
 * back-projects Z = fx * baseline / d.  More than 50 such points create the
 * map at once (the frame is the only keyframe, at R = I, T = 0; points in its
 * camera frame; metric scale; stats[3] = -2); otherwise the frame goes
 * through the monocular initialisation.  VISO_ERR_ARG unless
 * 1 <= min_disp < max_disp when enabled. */
int viso_set_stereo(viso_ctx* ctx, double baseline, int32_t max_disp, int32_t min_disp);

/* Stereo keyframe insertion (map maintenance the
 * reference lacks: its map is frozen after src/viso.cpp:79-96; the repo's own
 * spec, restated in oracle/oracle_viso.cpp).  With stereo enabled and
 * interval > 0: after every interval-th tracking frame whose level-0 direct-
 * pose nGood is below ngood_permille / 1000 of the map size, the frame's
 * stereo points (as viso_set_stereo, in world coordinates R^T (Pc - T) with
 * its pose) are appended to the map, the frame becomes a keyframe (LK
 * alignment may pair points with it) and stats[14] = points added;
 * stats[15] = keyframes.  At most 8 keyframes and 16384 map points.  Each
 * check is one host synchronisation.  interval 0 (default) = off, the
 * reference's frozen map. */
int viso_set_keyframes(viso_ctx* ctx, int32_t interval, int32_t ngood_permille);

/* Photometric bundle adjustment (the repo's own spec of the BA that
 * include/bundle_adjuster.h:22-106 sketches with g2o, SURVEY.md §8(f) row 4;
 * oracle/oracle_ba.cpp): after every stereo keyframe insertion, `iterations`
 * Levenberg-Marquardt steps refine every keyframe pose but the first and
 * every map point over 16-residual 4x4 patch edges (each point against every
 * keyframe but its host), points marginalised (Schur complement).
 * 0 = off (default). */
int viso_set_bundle_adjust(viso_ctx* ctx, int32_t iterations);
/* Stage entry (parity tests): the same BA on host data.  kf_images: n_kf
 * (2..8) level-0 images of the context's size; kf_poses: n_kf x 12 (in/out;
 * keyframe 0 fixed); points: n x 3 world (in/out), 1 <= n <= 16384; host: n
 * keyframe indices (an edge's host pose stays at its value from the start of
 * the call); report (may be NULL): iterations x 4 (cost, candidate cost,
 * damping, accepted).  src: bundle_adjuster.h:58-100 (EdgeDirectProjection).
 * VISO_ERR_ARG on any out-of-range argument. */
int viso_photometric_ba(viso_ctx* ctx, const uint8_t* const* kf_images, int32_t n_kf, double* kf_poses,
                        double* points, const int32_t* host, int32_t n, int32_t iterations, double* report);

/* Library build/version string, "viso_amd 0.1 gfx950 (HIP) src:<hash>": the
 * hash of the sources and flags it was built from (viso_amd/build.py
 * source_hash), so a stale prebuilt library can be detected. */
const char* viso_version(void);

#ifdef __cplusplus
}
#endif
#endif /* VISO_C_H */
