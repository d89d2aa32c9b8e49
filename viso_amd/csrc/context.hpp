// viso_amd — context object behind the C ABI.
#pragma once

#include <chrono>
#include <deque>
#include <vector>

#include "../../include/viso/viso_c.h"
#include "geometry.hpp"
#include "kernels.hpp"
#include "staging.hpp"
#include "trace.hpp"

namespace viso {

struct DevBuf {
    void* ptr = nullptr;
    size_t bytes = 0;
    int ensure(size_t need);
    void release();
    template <class T>
    T* as() const { return (T*)ptr; }
};

// HIP-event timing of selected kernels on the context stream.
struct Timing {
    bool enabled = false;
    uint32_t mask = 0xffffffffu;  // kernel ids timed when enabled
    bool on(int kernel) const { return enabled && ((mask >> kernel) & 1u); }
    int64_t launches[VISO_KERNEL_COUNT] = {};
    double total_ms[VISO_KERNEL_COUNT] = {};
    struct Pending {
        int kernel;
        hipEvent_t a, b;
    };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> pool;

    hipEvent_t get_event() {
        if (!pool.empty()) {
            hipEvent_t e = pool.back();
            pool.pop_back();
            return e;
        }
        hipEvent_t e = nullptr;
        (void)hipEventCreate(&e);
        return e;
    }
    int collect() {
        for (auto& p : pending) {
            if (hipEventSynchronize(p.b) != hipSuccess) return VISO_ERR_HIP;
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, p.a, p.b) != hipSuccess) return VISO_ERR_HIP;
            launches[p.kernel] += 1;
            total_ms[p.kernel] += (double)ms;
            pool.push_back(p.a);
            pool.push_back(p.b);
        }
        pending.clear();
        return VISO_OK;
    }
    void reset() {
        for (int i = 0; i < VISO_KERNEL_COUNT; ++i) {
            launches[i] = 0;
            total_ms[i] = 0.0;
        }
    }
    void destroy() {
        collect();
        for (auto e : pool) (void)hipEventDestroy(e);
        pool.clear();
    }
};

// Bump sub-allocator over one DevBuf (stage entry points).
struct Bump {
    size_t off = 0;
    size_t take(size_t bytes) {
        size_t o = off;
        off += (bytes + 255) & ~(size_t)255;
        return o;
    }
};

struct TimedRegion {
    RoctxRange range;
    Timing& t;
    int kernel;
    hipStream_t s;
    hipEvent_t a = nullptr, b = nullptr;
    TimedRegion(Timing& t_, int k, hipStream_t s_) : range(phase_name(k)), t(t_), kernel(k), s(s_) {
        if (t.on(kernel)) {
            a = t.get_event();
            b = t.get_event();
            (void)hipEventRecord(a, s);
        }
    }
    ~TimedRegion() {
        if (a && b) {
            (void)hipEventRecord(b, s);
            t.pending.push_back({kernel, a, b});
        }
    }
};

// (dev, VISO_HOST_TIMES=1) host time of viso_process_frame by phase: 0
// ingest (the pinned copy inside it is HostStage::copy_us), 1 OnNewFrame's
// launches, 2 the call's end (LK batching, epoch); printed at destroy
struct HostTimes {
    bool on = false;
    double us[3] = {0, 0, 0};
    int64_t calls = 0;
    struct Clock {
        HostTimes& h;
        std::chrono::steady_clock::time_point t;
        explicit Clock(HostTimes& h_) : h(h_) {
            if (h.on) {
                t = std::chrono::steady_clock::now();
                ++h.calls;
            }
        }
        void lap(int k) {
            if (!h.on) return;
            const auto n = std::chrono::steady_clock::now();
            h.us[k] += std::chrono::duration<double, std::micro>(n - t).count();
            t = n;
        }
    };
};

// (dev, VISO_HOST_TIMELINE=1) device timestamps of the host-frame path: per
// mark (frame, kind) an event recorded on the mark's stream; printed at
// destroy relative to the first (kinds: 0 upload start, 1 upload end, 2
// pyramid end, 3 chain start, 4 chain end)
struct DevTimeline {
    bool on = false;
    struct Mark {
        int64_t frame;
        int kind;
        hipEvent_t e;
    };
    std::vector<Mark> marks;
    void mark(int64_t frame, int kind, hipStream_t s) {
        if (!on || marks.size() > 20000) return;
        hipEvent_t e = nullptr;
        if (hipEventCreate(&e) != hipSuccess) return;
        (void)hipEventRecord(e, s);
        marks.push_back({frame, kind, e});
    }
};

}  // namespace viso

namespace viso {
// One pyramid slot of the frame pool.  Level 0 is either in the slot or
// borrowed from the caller's device buffer (batched ingest).
struct SlotRec {
    const uint8_t* l0 = nullptr;
    bool borrowed = false;
    int refs = 0;
    int64_t lk_use = -1;  // last lk_stream batch that reads it (lk_seq numbering)
    int64_t free_epoch = -1;  // the ingest call (epoch) during which it was freed
    int log_index = -1;       // a tracking frame's pose-log index (< 0: not logged)
};
constexpr int kEpochRing = 16;
constexpr int kEpochStride = 8;  // calls per epoch record (end_epoch)
constexpr int kLkRing = 64;
}  // namespace viso

struct viso_ctx {
    viso_params p{};
    int device = 0;
    hipStream_t stream = nullptr;
    viso::PyrGeom geom{};
    viso::Timing timing;
    // scratch for the stage-level entry points
    viso::DevBuf scratch_a, scratch_b, scratch_c, scratch_d;

    // ---------------- frame pool (Keyframe objects; include/keyframe.h:10-123)
    int n_slots = 0;
    viso::DevBuf slot_pool;   // n_slots x geom.slot bytes
    viso::DevBuf slot_pose;   // n_slots x 12 doubles (Keyframe R_, T_)
    std::vector<viso::SlotRec> slots;
    std::deque<int> free_slots;  // FIFO: the longest-free slot is reused first
    int ref_slot = -1, last_slot = -1;  // init_.ref_frame, last_frame
    std::vector<int> kf_slots;          // Map::keyframes_
    // the last ingest pyramid's tail launch: level-0 bytes it copied into the
    // pool (PyrOwn; 0 or w x h) and background-LK words it cleared
    int tail_copy_bytes = 0, tail_zero_ints = 0;
    int ident_slot = -1;  // the ingest's pyramid wrote this frame's Keyframe-ctor pose (PyrOwn)
    // the ingest's pyramid launch(es) with its last frame's PyrOwn (level 0
    // owned, identity pose outside tracking)
    void launch_ingest_pyramid(const uint8_t* const* l0, uint8_t* const* dst, const int* sl, int n,
                               bool bg_words = false, hipStream_t st = nullptr);

    // ---------------- initialisation tracks (Viso::Initialization, include/viso.h:33-41)
    viso::DevBuf kp1, kp2, kp1b, kp2b, track_success, n_track_dev;
    viso::FastScratch fast;
    // the detection frame's FAST tiles fused into its one-image ingest's
    // level-1 launch (FastPre; fast_pre_slot: that frame's slot, or -1)
    viso::FastPre fast_pre;
    int fast_pre_slot = -1;
    viso::DevBuf fast_rows;
    int n_track = 0;             // < 0: on the device only (ntrack_pending)
    bool ntrack_pending = false;  // a re-detection frame's count not read yet
    hipEvent_t ntrack_evt = nullptr;  // behind the FAST frame's count store into h_int[3]
    hipEvent_t gate_evt = nullptr;    // behind the 2D-2D gate (the host waits for it alone)
    // the last 2D-2D gate read: its frame count since the reference frame
    // (0: none since the last re-detection), open or not, its disparity
    int gate_cnt = 0;
    bool gate_open = false;
    double gate_disp = 0.0;
    int gate_spec_mode = -1;  // VISO_GATE_SPEC (tests): 0 never, 1 always, -1 predicted
    int resolve_ntrack();
    bool success_valid = false;
    int frame_cnt = 0;
    double initR[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    double initT[3] = {0, 0, 0};
    double Kinv[9] = {0};

    // ---------------- geometry (PoseEstimation2d2d + SelectMotion)
    viso::DevBuf geo_buf;
    viso::GeoArgs geo{};
    viso::GeoCtl* h_ctl = nullptr;  // pinned
    int* h_int = nullptr;           // pinned scratch ints
    // their device-side addresses (kernels store the FAST frame's count and
    // the 2D-2D control block there directly: no copy launch per frame)
    int* h_int_dev = nullptr;
    viso::GeoCtl* h_ctl_dev = nullptr;
    double* h_dbl = nullptr;        // pinned scratch doubles (64)
    double* h_poses = nullptr;      // pinned staging of the pose log (viso_get_poses)
    double* h_poses_dev = nullptr;  // its device address (the direct kernels log into it too)
    size_t h_poses_cap = 0;         // poses it holds
    // poses of h_poses that are final once the context stream has passed the
    // calls that produced them: advanced by stage_poses (viso_synchronize)
    // and viso_get_poses.  Entries below h_poses_cap are written into h_poses
    // by the direct kernels themselves (log_host); the buffer grows
    // geometrically in viso_get_poses (up to max_poses)
    size_t poses_staged = 0;
    double* log_host(int index) const {  // the direct launch's log_host for a log index
        return index >= 0 && (size_t)index < h_poses_cap ? h_poses_dev : nullptr;
    }
    int stage_poses();

    // ---------------- map (Map / MapPoint, include/map.h, map_point.h)
    viso::DevBuf map_pts;  // kMaxMapPoints x 3
    int n_map = 0;
    viso::DevBuf kf_poses;  // kMaxKeyframes x 12

    // ---------------- tracking (kRunning)
    viso::DevBuf direct_buf;  // direct-pose scratch (kernels.hpp DirectScratch)
    viso::DirectScratch direct{};
    viso::DevBuf direct_stats;  // 4 levels x 50 doubles
    // LKAlignment only feeds the display (src/viso.cpp:121-135): tracking
    // frames queue in lk_pending (slot held) and run as one batched launch
    // (up to kLkBatch frames) when the ingest call ends; outputs of batch
    // frame f at row f.  Batches of viso_process_frames_device run on the
    // context stream after the chunk's direct-pose chain; single-frame calls
    // use lk_stream so the host's next frame overlaps them.
    std::vector<int> lk_pending;
    int lk_last_rows = 0;  // frames in the last launched batch
    int lk_last_pts = 0;   // map points of the last launched batch
    viso::DevBuf lk_pair, lk_succ, lk_before, lk_after;  // kLkBatch x kMaxMapPoints
    // per-map LK templates (keyframe choice + per-level template / H^-1),
    // computed once when the map is created (launch_lk_template)
    viso::DevBuf lk_tmpl, lk_tmpl_h, lk_tmpl_kf, lk_tmpl_uv;
    hipStream_t lk_stream = nullptr;
    hipEvent_t lk_ring[viso::kLkRing] = {};  // recorded after each lk_stream batch
    viso::HostStage stage;  // pinned staging of host-ingested frames (ingest_host)
    viso::HostTimes host_times;
    viso::DevTimeline dev_tl;
    // Host uploads run on their own stream (created at the first one, with a
    // hardware queue of its own when a CU-masked stream can be made), so a
    // frame's DMA overlaps the previous frame's chain.  A slot's last readers
    // on the context stream were all enqueued by the end of the ingest call
    // that freed it: every ingest call ends an epoch with an event there.
    hipStream_t up_stream = nullptr;
    int64_t epoch = 0;
    hipEvent_t epoch_evt[viso::kEpochRing] = {};
    int64_t epoch_rec_call[viso::kEpochRing] = {};  // the call (epoch) each record was made at
    int64_t epoch_nrec = 0;                         // records made
    int64_t epoch_last_rec = -(1LL << 40);          // the call of the latest record
    int wait_freed(int64_t fe, hipStream_t st);
    hipEvent_t epoch_now = nullptr;  // a slot freed in the current call (rare)
    int end_epoch();
    int create_up_stream();
    int upload_host(int s, const uint8_t* grey, int32_t w, int32_t h, int32_t stride, bool pyramid);
    // PoseEstimation2d2d's E path runs on lk_stream beside the H path (no LK
    // alignment runs while initialising): fork / join events
    hipEvent_t geo_fork = nullptr, geo_join = nullptr;
    int64_t lk_seq = 0;                      // lk_stream batches launched
    int64_t lk_done = 0;                     // batches the host has seen complete (all < lk_done)
    int64_t lk_waited_ctx = 0, lk_waited_up = 0;  // batches the context / upload stream already wait for
    int order_after_lk(int64_t use, hipStream_t st);
    // The last tracking frame's final direct-pose solve (F) is deferred: it
    // runs fused into the next tracking frame's L(3), or alone when the
    // ingest call ends (resolve_direct).  Its frame and `last` slots are held.
    bool dpend = false;
    int dpend_cur = -1, dpend_last = -1, dpend_log = -1;
    viso::DevBuf pose_log;  // max_poses x 12
    int n_poses = 0;
    // the per-frame log (viso_set_frame_log): max_poses x 4 doubles {level-0
    // nGood, level-0 cost, LK pairs, LK successes} per logged tracking frame;
    // null when off
    viso::DevBuf frame_log;
    double* flog() const { return (double*)frame_log.ptr; }
    // the LK columns of the frames in batch rows 0.. (their slots), on `s`
    int count_lk(const std::vector<int>& row_slots, hipStream_t s);

    // ---------------- stereo initialisation (viso_set_stereo; the repo's own
    // replacement of the 2D-2D init, no reference counterpart)
    double stereo_base = 0.0;  // metres; > 0 enables it
    int stereo_max_disp = 0, stereo_min_disp = 1;
    // level 0 of the right image of the frame on_new_frame is processing
    // (null: none); only the stereo initialisation reads it
    const uint8_t* right_l0 = nullptr;
    viso::DevBuf st_flag, st_pts;
    // stereo keyframe insertion (viso_set_keyframes; the repo's own map
    // maintenance): checked every kf_interval-th
    // tracking frame (0 = off), inserting when level-0 nGood is below
    // kf_permille / 1000 of the map
    int kf_interval = 0, kf_permille = 0;
    int64_t track_cnt = 0;
    // photometric BA after each keyframe insertion (viso_set_bundle_adjust;
    // ba.hip): LM iterations (0 = off) and each map point's host keyframe
    int ba_iterations = 0;
    std::vector<int32_t> point_host;
    viso::DevBuf point_host_dev, ba_scratch;
    int sync_point_hosts(int first);
    int bundle_adjust();
    int stereo_points_into(int cur, double* out, int cap, int* kept);
    int insert_keyframe(int cur);

    // ---------------- state (include/viso.h:44)
    int state = VISO_STATE_INITIALIZATION;
    int64_t frames = 0;
    double stats[16] = {0};
    bool ran_tracking = false;

    int create_streams();
    int init();
    void release();
    // frame pool
    int acquire_slot(hipStream_t lk_wait = nullptr);
    void hold(int slot);
    void drop(int slot);
    void set_role(int& role, int slot);
    viso::FrameDev frame(int slot) const;
    uint8_t* slot_base(int slot) const;
    double* pose_of(int slot) const;
    int own_level0(int slot);
    // map creation from the stereo pair (cur, right_slot); *made = 0 when
    // there are too few stereo points (the mono path then runs)
    int stereo_init(int cur, bool* made);
    // per-map LK templates (after a map is created)
    int build_lk_templates();
    // OnNewFrame on a frame whose pyramid is already built in `slot`
    int on_new_frame(int slot);
    // one ingest chunk (viso_process_frames_device; queued host frames)
    int ingest_chunk(const std::vector<int>& sl, const std::vector<const uint8_t*>& l0,
                     const std::vector<const uint8_t*>& right, bool overlap_tail = false);
    // (pyramid: the frame's pyramid too, on the upload stream)
    int ingest_host(const uint8_t* grey, int32_t w, int32_t h, int32_t stride, int* slot_out, bool pyramid = false);
    // launch LKAlignment of every pending tracking frame (on `s`)
    int flush_lk(hipStream_t s);
    // launch the pending final solve, if any
    int resolve_direct();
    // end of an ingest call: pending final solve, then the LK batch on `s`
    // (overlap: a chunk follows — its drain runs on lk_stream, bg_end)
    int finish_call(hipStream_t s, bool overlap = false);
    // end of a host-frame call (viso_process_frame / _stereo) while
    // tracking: the final solve stays pending (the next frame's L(3) runs
    // it, as inside a device chunk) and the LK alignment of every queued
    // frame but the last goes out in batches; settle() launches what is
    // pending before anything reads it or changes what it depends on
    // (getters, viso_synchronize, setters, stage calls, device ingest)
    int finish_host_call();
    int settle();
    // host frames queued while tracking (slots, uploaded, held), run as chunks
    std::vector<int> host_q;
    int host_chunk = -1;  // frames per queued chunk (VISO_HOST_CHUNK; 0 off; -1 unread)
    bool host_queue_eligible();
    int queue_host_frame(const uint8_t* grey, int32_t w, int32_t h, int32_t stride);
    int flush_host_q();
    int host_lk_batch() const;
    // host batches in the background-grid geometry (VISO_HOST_LK; -1 unread)
    int host_lk_mode = -1;
    bool host_lk_grid();
    viso::DevBuf hbg_buf;  // their words (ready flags up, heads, leftover header, error)
    int host_grid_args(viso::LkAlignArgs& a, hipStream_t s);
    // LK batch of lk_pending on `s` (all but the last frame: keep_last)
    int flush_lk_frames(hipStream_t s, bool keep_last);
    // LK alignment of a device-ingest chunk in the background of its
    // direct-pose chain (track.hip lk_item_kernel): bg_begin after the chunk's
    // pyramid when the context is tracking (frames of the chunk: their slots),
    // bg_end once the chunk's last pose is launched
    bool bg_eligible();
    bool bg_on();  // the background mode itself (VISO_LK_BG, serialised kernels, the side queue)
    bool lk_dedicated = false, up_dedicated = false;  // lk_stream / up_stream CU-masked (queue of their own)
    // (zeroed: the chunk's pyramid launch cleared the words)
    int bg_begin(const std::vector<int>& chunk, bool zeroed = false);
    int bg_end(bool drain = true, bool overlap = false);
    // the grid's buffer, event and kernel warm-up (context init)
    int bg_prepare();
    // after a host sync: VISO_ERR_HIP if a background launch since the last
    // check timed out waiting for a pose (its LK outputs are then invalid)
    int bg_check();
    int bg_launch();
    bool bg_unchecked = false;
    bool bg_active = false;
    bool bg_launched = false;  // bg_begin cleared the words; the grid is launched after frame 0
    // two sets of the grid's words, alternating chunks (the previous chunk's
    // grid and, when overlapped, its drain still read theirs on lk_stream);
    // bg_set_seq: the lk_stream batch that last read each set (-1: none)
    int bg_set = 1;
    int64_t bg_set_seq[2] = {-1, -1};
    int* bg_words_of(int set) const;
    int tail_mode = -1;  // VISO_LK_TAIL (read once)
    bool tail_overlap_on();
    int bg_mode = -1;        // VISO_LK_BG: 0 off, 1 on (read once; -1 unread)
    int bg_nb = 0;           // frames of the chunk
    int bg_cur = -1;         // chunk index of the frame on_new_frame is processing
    int dpend_bg = -1;       // chunk index of the pending final solve's frame
    int n_cu = 0;            // compute units (one background workgroup each)
    std::vector<int> bg_slots;  // tracking frames held until the kernel is done
    viso::DevBuf bg_buf;        // ready flags [kLkBatch], next item, error
    hipEvent_t bg_done = nullptr;
    viso::LkAlignArgs bg_args{};  // the chunk's launch (the drain reuses it)
    int* bg_ready(int idx) const {
        return (bg_active && idx >= 0) ? bg_args.bg_ready + idx : nullptr;  // (the chunk's word set)
    }
    // LKAlignment arguments common to the template and alignment launches
    viso::LkAlignArgs lk_args();
};
