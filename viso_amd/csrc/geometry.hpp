// viso_amd — device state and launcher of the 2D-2D initialisation geometry
// (PoseEstimation2d2d + SelectMotion, src/viso.cpp:178-256, 520-638).
#pragma once

#include "common.hpp"

namespace viso {

struct Timing;

constexpr int kMaxCandidates = 5;

// Device-resident result block of one PoseEstimation2d2d call (read back by
// the host once per initialisation frame).
struct GeoCtl {
    int n;
    int gate;  // N >= 10 and disparity >= threshold (src/viso.cpp:184, 216)
    double disparity;
    int e_count, e_best, e_iters;
    int h_count, h_best, h_iters;
    int n_cand;
    // candidate slots: [0] recoverPose's (E path, e_ncand = 0 or 1), [1..4]
    // decomposeHomographyMat's (H path, h_ncand of them) — fixed slots, so
    // the two paths can run concurrently; SelectMotion walks them in the
    // reference's order (E first, then H; src/viso.cpp:236-244)
    int e_ncand, h_ncand;
    double cand[kMaxCandidates][12];
    double H[9];
    int nr_inliers, best_motion;
    double R[9], T[3];
    double mean_depth;
    int mean_nonzero;
    int pad;
};

static_assert(sizeof(GeoCtl) % 8 == 0, "GeoCtl is mirrored in 8-byte words");

struct GeoArgs {
    const int* n_dev;  // tracked point count (device)
    const float2* kp1;
    const float2* kp2;
    const double* p1_in;  // optional normalised inputs (n x 3) instead of kp1/kp2
    const double* p2_in;
    double Kinv[9];
    double K[4];
    double* p1;  // cap x 3
    double* p2;
    double* q1;  // cap x 2 (float-rounded)
    double* q2;
    GeoCtl* ctl;
    // optional: the control block mirrored into pinned host memory (device
    // address) by the gate and by SelectMotion's last launch, for the host
    // to read after its stream sync without a copy launch
    GeoCtl* host_ctl;
    double disparity_thresh;
    double proj_thresh;
    double parallax_thresh;
    double confidence;
    float t2;  // (float)(thresh^2), thresh = 0.3 / sqrt(fx^2 + fy^2)
    uint64_t seed;
    int e_iters, h_iters;
    double* e_models;
    uint8_t* e_valid;
    int* e_counts;
    uint8_t* e_mask;
    double* h_models;
    uint8_t* h_valid;
    int* h_counts;
    uint8_t* h_mask;
    int cap;
    uint8_t* sel_in;   // kMaxCandidates x cap
    double* sel_pts;   // kMaxCandidates x cap x 3
    uint8_t* inliers;  // cap (best motion's inlier flags)
    double* points_out;  // cap x 3 (normalised inlier points, compacted)
    // recoverPose: the two rotations and t of E's decomposition (2 x 9 + 3)
    // and the four motions' cheirality counts
    double* rp = nullptr;
    int* rp_good = nullptr;
    // homography refinement: the 45 upper-triangle moment leaves per point
    // ([45][cap]) and their canonical tree sums (9 x 9, symmetric)
    double* hm = nullptr;
    double* hM = nullptr;
};

void launch_pose_2d2d(const GeoArgs& a, hipStream_t stream, Timing* timing);
// The same in two parts: the normalisation and the gates of
// src/viso.cpp:184, 216 (GeoCtl n / disparity / gate), then the RANSACs,
// recoverPose / decomposition and SelectMotion.  Every kernel of the body
// returns at once when the gate is closed; a caller that has read the gate
// on the host may skip the body.
void launch_pose_2d2d_gate(const GeoArgs& a, hipStream_t stream);
// The erase of failed tracks (src/viso.cpp:23-40) and the gate in one
// launch: in1 / in2 [0, n) with success -> out1 / out2 (which must be a.kp1 /
// a.kp2), the count -> *n_out (which must be a.n_dev); n < 0: the count is
// *n_out's input value capped at -n.
struct CompactIn {
    const float2* in1 = nullptr;
    const float2* in2 = nullptr;
    const uint8_t* success = nullptr;
    int n = 0;
    float2* out1 = nullptr;
    float2* out2 = nullptr;
    int* n_out = nullptr;
};
void launch_compact_gate(const CompactIn& ci, const GeoArgs& a, hipStream_t stream);
// The H chain's first launch (the hypotheses), enqueued on `stream` behind
// the gate before the host has read it: a closed gate makes it return at
// once, an open one lets the host's round trip on the gate overlap it.
void launch_pose_2d2d_spec(const GeoArgs& a, hipStream_t stream);
// hs (optional): a second stream.  The host has seen the gate's result (both
// streams may read it); the E and H chains are enqueued interleaved, the
// longer H chain on `stream` behind launch_pose_2d2d_spec's launch (h_spec)
// and the E chain on hs — or, without h_spec, the H chain on hs and the E
// chain on `stream`; SelectMotion runs behind the H chain once the E chain's
// event `e_done` has passed, and when that is hs, `join` (behind
// SelectMotion) is waited for by `stream`.  Returns the stream SelectMotion
// ran on (read the result there).
hipStream_t launch_pose_2d2d_body(const GeoArgs& a, hipStream_t stream, hipStream_t hs = nullptr,
                                  hipEvent_t e_done = nullptr, hipEvent_t join = nullptr, bool h_spec = false);

}  // namespace viso
