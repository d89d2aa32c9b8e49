/* viso_amd — synthetic stereo sequence source (host only).
 *
 * KITTI odometry data is not available offline, so the tests and bench.py
 * render a deterministic KITTI-like sequence (seq-00 intrinsics, 0.54 m
 * baseline) with this renderer.  No reference counterpart (the reference
 * reads rgb/<n>.png through FrameSequence, include/frame_sequence.h:25-38). */
#ifndef VISO_SYNTH_H
#define VISO_SYNTH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct viso_synth_params {
    int32_t width, height;
    double fx, fy, cx, cy;
    double baseline;   /* right camera offset along +x (m) */
    uint64_t seed;
    double block_m;    /* texture block size (m) */
    double wall_x;     /* side walls at x = +-wall_x */
    double wall_z;     /* back wall at z = wall_z */
    double ground_y;   /* ground plane y (camera y points down) */
    double pitch0;     /* camera pitch-up (rad) */
    double yaw_amp, yaw_period;
    double x_amp, x_period;
    double z_amp, z_period;
    int32_t noise;     /* +- grey-level hashed pixel noise */
    int32_t reserved[7];
} viso_synth_params;

void viso_synth_default(viso_synth_params* p, int width, int height);
/* Ground-truth Tcw of frame `frame`, camera 0 (left) / 1 (right):
 * 12 doubles, R row-major + t. */
int viso_synth_pose(const viso_synth_params* p, int frame, int cam, double* Rt12);
/* Render one grey frame (width x height, continuous rows). */
int viso_synth_render(const viso_synth_params* p, int frame, int cam, uint8_t* out, int threads);

/* Multi-camera rig (BASELINE.json configs[4]): n_cams stereo cameras fixed on
 * the trajectory of viso_synth_pose(frame, 0) (the rig frame), camera c yawed
 * by (c - (n-1)/2) * 20 deg and offset (c - (n-1)/2) * 0.35 m along the rig x
 * axis.  Extrinsic E_c: rig -> camera c (left), 12 doubles (R row-major, t). */
int viso_synth_rig_extrinsic(int cam, int n_cams, double* E12);
int viso_synth_rig_pose(const viso_synth_params* p, int frame, int n_cams, int cam, int side, double* Rt12);
int viso_synth_rig_render(const viso_synth_params* p, int frame, int n_cams, int cam, int side, uint8_t* out,
                          int threads);

#ifdef __cplusplus
}
#endif
#endif
