/* viso_amd — multi-camera photometric rig on the reference path, C ABI.
 *
 * SURVEY.md §8(f) row 3 / BASELINE.json configs[4]: n <= 4 stereo cameras
 * rigidly mounted on one body, tracked by ONE direct (photometric) pose.
 * The reference has a single camera; its per-level Gauss-Newton
 * (DirectPoseEstimationSingleLayer, src/viso.cpp:661-758) is run per camera
 * at the camera's pose E_c T, and the cameras' H, b (src/viso.cpp:682-729)
 * are summed through the rig extrinsics:
 *   H = sum_c Ad(E_c)^T H_c Ad(E_c),  b = sum_c Ad(E_c)^T b_c,
 * one step per level (levels 3..0), T <- exp(H^-1 b) T.  Initialisation is
 * the stereo initialisation of viso_set_stereo per camera (metric map per
 * camera, in the rig frame of the first timestep).  The spec is this repo's
 * own (oracle/oracle_rig.cpp); parity is GPU vs that restatement: bit-exact
 * for the map, poses <= 1e-10 rel in FAITHFUL precision, <= 1e-4 rel
 * Frobenius in FAST (fp32 per pixel, the `last` patch kept as fp16 in LDS).
 *
 * Conventions as in viso_c.h: int return codes, caller-owned host buffers,
 * one HIP device and stream per rig, not thread-safe.  Device image buffers
 * passed to viso_rig_process_device must stay valid and unmodified until
 * viso_rig_synchronize (or any getter) returns.
 */
#ifndef VISO_RIG_H
#define VISO_RIG_H

#include <stddef.h>
#include <stdint.h>

#include "viso_c.h"

#ifdef __cplusplus
extern "C" {
#endif

#define VISO_RIG_MAX_CAMS 4

typedef struct viso_rig viso_rig;

/* p: the single-camera parameters (intrinsics and image size shared by all
 * cameras; fast_thresh, precision, max_poses are used).  extrinsics: n_cams x
 * 12 doubles, rig -> camera c (left camera): R row-major, then t, so that
 * X_c = R X_rig + t. */
int viso_rig_create(const viso_params* p, int32_t n_cams, const double* extrinsics, int device,
                    viso_rig** out);
int viso_rig_destroy(viso_rig* rig);
/* metric stereo initialisation (viso_set_stereo's parameters); required:
 * the rig initialises from the first timestep with right images */
int viso_rig_set_stereo(viso_rig* rig, double baseline, int32_t max_disp, int32_t min_disp);
/* One timestep from host images: lefts[c] / rights[c] (rights may be null
 * once tracking), dims = {width, height, stride}. */
int viso_rig_process(viso_rig* rig, const uint8_t* const* lefts, const uint8_t* const* rights,
                     const int32_t dims[3]);
/* n_steps timesteps already in device memory: camera c of step s at
 * d_left + (s * n_cams + c) * frame_stride (d_right likewise, may be null). */
int viso_rig_process_device(viso_rig* rig, const uint8_t* d_left, const uint8_t* d_right, int32_t n_steps,
                            size_t frame_stride);
int viso_rig_synchronize(viso_rig* rig);
int viso_rig_get_state(viso_rig* rig, int32_t* state);
/* rig poses (world -> rig, 12 doubles: R row-major, t), one per tracking
 * timestep */
int viso_rig_get_poses(viso_rig* rig, double* T12, size_t cap, size_t* n);
/* camera c's map points (world frame) */
int viso_rig_get_points(viso_rig* rig, int32_t cam, double* xyz, size_t cap, size_t* n);
/* the last timestep's per-level stats, [4][50]: nGood, cost / nGood, H (36),
 * b (6), update (6) (the direct pose's layout) */
int viso_rig_get_level_stats(viso_rig* rig, double out[200]);

#ifdef __cplusplus
}
#endif
#endif
