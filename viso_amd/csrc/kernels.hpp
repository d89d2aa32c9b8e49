// viso_amd — host-side launcher declarations (one translation unit per stage).
#pragma once

#include "../../include/viso/viso_c.h"
#include "common.hpp"

namespace viso {

// ---------------------------------------------------------------- image pass
// Builds levels 1..3 of n_images pyramids; image i's level-0 bytes live at
// base + i*img_stride (levels follow, PyrGeom offsets).
void launch_pyramid(const PyrGeom& g, uint8_t* base, int n_images, size_t img_stride,
                    hipStream_t stream);
// Batched pyramid over frames whose level 0 is at l0[i] and whose levels
// 1..3 go to slot[i] + g.off[l] (n <= kPyrBatch per launch; more are split).
constexpr int kPyrBatch = 128;
// Two launches: level 1 (streaming bands), levels 2-3 (pyr_tail_kernel).
// own (optional): for frame img, its level 0 copied from l0[img] into
// slot[img] (when they differ and the batch is small enough: copied says
// whether it was) and, when ident_pose is set, the identity pose written
// there — done by the tail launch (a frame-by-frame caller's copy and pose
// launches folded into it).
// zero (optional): n_zero ints cleared by the same launch (the chunk's
// background-LK words, bg_begin).
// FAST device scratch (image.hip): per (row, tile) keypoint counts and
// slots, per-tile totals; carved from fast_scratch_bytes(w, h) bytes.
struct FastScratch {
    int* cnt = nullptr;  // [h][tiles across]
    int* tot = nullptr;  // [bands][tiles across]
    int* lst = nullptr;  // [h][tiles across][64]
};

// A one-image ingest whose frame starts with FAST (the initialisation's
// detection frame): the FAST tiles of `img` (the frame's level 0) run as
// extra workgroups of the level-1 launch (pyr1_fast_kernel) instead of a
// launch of their own behind the pyramid; done = they were launched, so the
// frame's launch_fast only orders them (tiles_done).
struct FastPre {
    const uint8_t* img = nullptr;
    int w = 0, h = 0, thresh = 0;
    FastScratch s;
    bool done = false;
};

struct PyrOwn {
    int img;
    double* ident_pose;
    bool copied;
    int* zero = nullptr;
    int n_zero = 0;
    FastPre* fast = nullptr;
};
void launch_pyramid_frames(const PyrGeom& g, const uint8_t* const* l0, uint8_t* const* slot,
                           int n, hipStream_t stream, PyrOwn* own = nullptr);
size_t fast_scratch_bytes(int w, int h);
FastScratch fast_scratch_at(void* base, int w, int h);
// FAST + NMS on a level-0 image; writes up to cap keypoints (float2 and/or
// raw int4 {x, y, score, 0}) and the total count to *n_out (device).
// det (a re-detection frame, src/viso.cpp:100-108): the count is stored
// capped at cap, the keypoints also go to kp_copy (kp2 = kp1) and the capped
// count also to host_n (pinned host memory, device-mapped; may be null).
struct FastDetect {
    float2* kp_copy;
    int* host_n;
};
void launch_fast(const uint8_t* img, int w, int h, int thresh, FastScratch& s, float2* kp_out,
                 int4* raw_out, int cap, int* n_out, hipStream_t stream, const FastDetect* det = nullptr,
                 bool tiles_done = false);

// ---------------------------------------------------------------- tracking
// OpticalFlowMultiLevel(inverse=true): kp2 in/out, success out (level 0).
void launch_klt(const FrameDev& ref, const FrameDev& cur, const PyrGeom& g, const float2* kp1,
                float2* kp2, uint8_t* success, int n, double thresh, hipStream_t stream);
// the same with the track count in device memory (*n_dev, capped at cap)
void launch_klt_dev(const FrameDev& ref, const FrameDev& cur, const PyrGeom& g, const float2* kp1,
                    float2* kp2, uint8_t* success, const int* n_dev, int cap, double thresh, hipStream_t stream);

constexpr int kMaxKeyframes = 8;
// One frame of a batched LKAlignment launch: its pyramid and pose (device).
struct LkFrame {
    FrameDev cur;
    const double* pose;  // 12 doubles
};
constexpr int kLkBatch = 64;  // frames per launch (kernel arguments stay < 4 KB)
struct LkAlignArgs {
    FrameDev kf[kMaxKeyframes];
    const double* kf_poses;  // n_kf x 12 (device)
    int n_kf;
    int n_frames;            // <= kLkBatch
    LkFrame frames[kLkBatch];
    const double* points;    // n x 3
    int n;
    double K[4];
    double thresh;
    struct {
        int w[4], h[4];
        unsigned long long off[4];
    } g;
    // outputs of frame f at f * out_stride (elements)
    size_t out_stride;
    int32_t* pair_kf;
    uint8_t* success;
    double* uv_before;  // 2 per point
    double* uv_after;
    // per-map templates (lk_template_kernel); tmpl == nullptr: computed inline
    double* tmpl = nullptr;    // [n][4 levels][3][64]
    double* tmpl_h = nullptr;  // [n][4][4]
    int32_t* tmpl_kf = nullptr;
    double* tmpl_uv = nullptr;  // [n][2]
    // tolerance mode (VISO_PRECISION_FAST): tmpl / tmpl_h hold floats, same
    // layout; the iterations run in fp32 (lk_align_kernel<true>)
    int fast = 0;
    // background mode (launch_lk_bg): items = frames x n, taken from eight
    // heads bg_next[32 x] (one per XCD, each a segment of every frame's points,
    // frames in order); frame f's pose is valid once bg_ready[f] != 0
    int* bg_ready = nullptr;
    int* bg_next = nullptr;
    int* bg_err = nullptr;
    // the error word's pinned host copy (device address): set with bg_err[0]
    // by the (rare) failing wave, so the end of a chunk copies nothing back
    int* bg_err_host = nullptr;
    int bg_inject_fail = 0;  // tests (VISO_LK_BG_INJECT_FAIL): the drain reports a failed wait
    int bg_items = 0;
    // leftovers: [0] drain cursor, [1] count, [32 ..] items (head * per_head + k)
    int* bg_left = nullptr;
    int bg_drain = 0;  // this launch is the end-of-chunk drain
    // a resident wave's longest wait for its item's frame before handing the
    // item to the drain (s_memrealtime ticks, 100 MHz)
    unsigned int bg_idle = 30000;
};
void launch_lk_align(const LkAlignArgs& a, hipStream_t stream);
// LK alignment of an ingest chunk's frames beside its direct-pose chain: grid
// workgroups (one per CU) resident for the chunk (track.hip lk_item_kernel)
void launch_lk_bg(const LkAlignArgs& a, int grid, hipStream_t stream);
// the items of a background launch it has not taken yet, at full occupancy
// (after the chunk's last pose): grid workgroups pull from the same counter
void launch_lk_drain(const LkAlignArgs& a, int grid, hipStream_t stream);
// the background kernel's attribute and first launches (context init)
void warm_lk_bg(hipStream_t stream);
// Keyframe choice + per-level templates of every map point (once per map).
void launch_lk_template(const LkAlignArgs& a, hipStream_t stream);
// The per-frame log's LK columns (viso_set_frame_log): for batch row f with
// log index idx[f] >= 0, flog[4 idx + 2] = points paired with a keyframe
// (pair_kf >= 0), flog[4 idx + 3] = successes, over the row's n points.
struct LkCountArgs {
    int idx[kLkBatch];
};
void launch_lk_count(const int32_t* pair_kf, const uint8_t* success, size_t stride, int n, int n_rows,
                     const LkCountArgs& rows, double* flog, hipStream_t stream);

// ---------------------------------------------------------------- stereo (north star)
// stereo initialisation (stereo.hip): per keypoint flag / camera point, then
// the kept points compacted in keypoint order into out (<= cap), *count kept
struct StereoCam {
    double fx, fy, cx, cy, base;
};
void launch_stereo_points(const uint8_t* left, const uint8_t* right, int w, int h, const float2* kp,
                          int n, int max_disp, int min_disp, const StereoCam& cam, int* flag,
                          double* pts, double* out, int cap, int* count, hipStream_t stream);
// pts (n x 3, device) <- R^T (pts - T) with the Tcw pose (12 doubles, device)
void launch_points_to_world(double* pts, int n, const double* pose12, hipStream_t stream);
void launch_stereo_sad(const uint8_t* left, const uint8_t* right, int w, int h, const int* xs,
                       const int* ys, int n, int max_disp, int* disp, int* sad,
                       hipStream_t stream);

// ---------------------------------------------------------------- direct pose
constexpr int kMaxMapPoints = 16384;
// Device scratch of the direct pose (carved from one buffer of
// direct_scratch_bytes() by direct_scratch_at).
struct DirectScratch {
    double* part = nullptr;       // [kLevels][256 tiles][28] tile partial sums
    int* good = nullptr;          // [kLevels][256]
    double* state = nullptr;      // [kLevels + 1][8] T21 per level (+ result)
    double* cont_part = nullptr;  // [256 workgroups][256][28] continuation scratch
    int* cont_good = nullptr;     // [256 workgroups][256]
};
size_t direct_scratch_bytes();
DirectScratch direct_scratch_at(void* base);
// DirectPoseEstimationMultiLayer (src/viso.cpp:760-766): levels 3..0, each a
// faithful DirectPoseEstimationSingleLayer (:661-758), starting from
// T21 = SE3(R, t) of pose_seed12 (src/viso.cpp:114); the patch reference is
// `last` at pose_last12.  Five launches: the tiles of level l run in a launch
// whose prologue solves level l+1 from its tile partials; a final one-
// workgroup launch solves level 0.
// stats (device, may be null): per level [nGood, cost, H(36), b(6), update(6)].
// pose_out (device, may be null) receives R, t of the result, also stored at
// log[12*log_index] when log is non-null.
void launch_direct_pose(const FrameDev& last, const FrameDev& cur, const PyrGeom& g,
                        const double K[4], const double* points, int n,
                        const double* pose_last12, const double* pose_seed12,
                        const DirectScratch& s, double* stats, double* pose_out, double* log,
                        int log_index, hipStream_t stream, int precision = VISO_PRECISION_FAITHFUL);
// The same call split for the frame pipeline: L(3..0) of this frame, then F
// later.  With `merge`, L(3) also runs the previous frame's pending F (its
// level-0 solve; the solved pose is this frame's `last` pose and seed, so
// pose_last12 / pose_seed12 are read only by L(2..0), after L(3) wrote them
// to merge->pose_out).
struct DirectPrev {
    FrameDev last, cur;         // the previous frame's pair (rare continuation)
    const double* pose_last12;  // its `last` pose
    double* pose_out;           // its pose (= this frame's pose_last12)
    double* log;
    int log_index;
    int* ready = nullptr;  // background LK alignment's flag for that pose (or null)
    double* log_host = nullptr;  // the log's pinned host copy (device address), same index
    double* flog = nullptr;      // the per-frame log (viso_set_frame_log), same index, or null
};
// true when a direct-pose workgroup leaves its CU room for the background LK
// alignment's (12 waves of 128 VGPRs + <= 76 KB LDS beside 4 waves + 84 KB)
bool direct_fits_background();
void launch_direct_levels(const FrameDev& last, const FrameDev& cur, const PyrGeom& g,
                          const double K[4], const double* points, int n,
                          const double* pose_last12, const double* pose_seed12,
                          const DirectScratch& s, double* stats, const DirectPrev* merge,
                          hipStream_t stream, int precision = VISO_PRECISION_FAITHFUL, bool bg = false);
void launch_direct_final(const FrameDev& last, const FrameDev& cur, const PyrGeom& g,
                         const double K[4], const double* points, int n,
                         const double* pose_last12, const DirectScratch& s, double* stats,
                         double* pose_out, double* log, int log_index, hipStream_t stream,
                         int precision = VISO_PRECISION_FAITHFUL, int* ready = nullptr,
                         double* log_host = nullptr, double* flog = nullptr);
// ---------------------------------------------------------------- rig direct pose
// Multi-camera photometric rig (the repo's own spec;
// oracle/oracle_rig.cpp): levels 3..0 of one rig Gauss-Newton step each over
// every camera's map points, camera c at E_c T, per-camera 28 sums combined
// through Ad(E_c); then F writes the rig pose (+ log) and each camera's next
// `last` pose E_c T.  5 launches.
constexpr int kMaxRigCams = 4;
struct RigCamDev {
    FrameDev last, cur;          // the camera's pyramids
    const double* points;        // its map points (world), n x 3
    int n;
    const double* pose_last12;   // its `last` pose (device, E_c T_last)
    double E[12];                // rig -> camera
    const double* Ad;            // device, 36
    void* scratch;               // rig_scratch_bytes()
};
size_t rig_scratch_bytes();
// state: [kLevels + 1][8] device; seed12: last rig pose (device); stats:
// [kLevels][50] or null; cam_last: n_cams x 12 device.  Returns -1 on a bad
// camera count.
// One rig timestep's direct pose: levels (L(3..0), when `levels`) and the
// final level-0 solve F (when `final_solve`); merge_prev: L(3) first solves
// the previous timestep's level 0 (its F, deferred) and logs it at
// prev_log_index.  An F alone (levels = 0, final_solve = 1) flushes a
// deferred one.
int launch_rig_direct(const RigCamDev* cams, int n_cams, const PyrGeom& g, const double K[4], double* state,
                      const double* seed12, double* stats, double* pose_out, double* log, int log_index,
                      double* cam_last, hipStream_t stream, int precision, int merge_prev = 0,
                      int prev_log_index = -1, int levels = 1, int final_solve = 1);
// ---------------------------------------------------------------- photometric BA
// The BA include/bundle_adjuster.h:22-106 sketches (SURVEY.md §8(f) row 4;
// spec oracle/oracle_ba.cpp): keyframe poses (n_kf x 12 device, keyframe 0
// fixed) and map points (n x 3 device) refined in place by `iterations`
// Levenberg-Marquardt steps over 16-residual 4x4 patch edges point -> every
// non-host keyframe (host: n device ints).  kf_l0: the keyframes' level-0
// images (device).  report (device, may be null): [iterations][4] cost,
// candidate cost, mu, accepted.  scratch: ba_scratch_bytes(n).  Returns -1
// on bad sizes.
size_t ba_scratch_bytes(int n);
int launch_photometric_ba(const uint8_t* const* kf_l0, int n_kf, int w, int h, const double K[4], double* poses,
                          double* pts, const int* host, int n, int iterations, void* scratch, double* report,
                          hipStream_t stream);
// dst (12 doubles, device) <- src (host values, passed by value)
void launch_set_pose(double* dst, const double src[12], hipStream_t stream);
// map creation: cur_pose <- pose, pts_dst <- pts_src (n_pts x 3), kf_poses[0]
// <- *ref_pose, kf_poses[1] <- pose (one launch)
void launch_map_create(double* cur_pose, const double pose[12], const double* pts_src, double* pts_dst, int n_pts,
                       const double* ref_pose, double* kf_poses, hipStream_t stream);

}  // namespace viso
