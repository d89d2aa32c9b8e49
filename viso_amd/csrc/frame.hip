// viso_amd — the per-frame path: Viso::OnNewFrame (src/viso.cpp:7-145) as a
// host state machine over device-resident state.
//
// All pixel/point work is on the GPU; the host only sequences launches.
// Tracking frames (kRunning) never synchronise: the direct pose (5 launches,
// direct.hip) is queued back to back and the pose stays in HBM (pose log);
// LK alignment of the call's tracking frames runs as one batched launch when
// the ingest call ends (flush_lk).  Initialisation frames
// synchronise once (to read the PoseEstimation2d2d result block) because the
// state transition (src/viso.cpp:76-98) decides which kernels the next frame
// runs.  Frames live in a slot pool (device pyramids + device poses); the
// reference's shared_ptr<Keyframe> roles (ref_frame, last_frame, map
// keyframes) are slot reference counts.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#include "context.hpp"

using namespace viso;

namespace {

// Eigen 3x3 inverse (compute_inverse<..., 3>): cofactors times 1/det;
// K_inv = K.inverse() (include/viso.h:50).
void eigen_inverse3(const double* m, double* inv) {
    auto M = [&](int i, int j) { return m[3 * i + j]; };
    auto cof = [&](int i, int j) {
        int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
        return M(i1, j1) * M(i2, j2) - M(i1, j2) * M(i2, j1);
    };
    double c0[3] = {cof(0, 0), cof(1, 0), cof(2, 0)};
    double det = (c0[0] * M(0, 0) + c0[1] * M(1, 0)) + c0[2] * M(2, 0);
    double invdet = 1.0 / det;
    inv[0] = c0[0] * invdet;
    inv[1] = c0[1] * invdet;
    inv[2] = c0[2] * invdet;
    inv[3] = cof(0, 1) * invdet;
    inv[4] = cof(1, 1) * invdet;
    inv[5] = cof(2, 1) * invdet;
    inv[6] = cof(0, 2) * invdet;
    inv[7] = cof(1, 2) * invdet;
    inv[8] = cof(2, 2) * invdet;
}

const double kIdentityPose[12] = {1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0};

}  // namespace

// Flags of the events that only order GPU work against GPU work (cross-
// stream waits; the host never reads memory behind them): no timing, and
// (VISO_EVENT_FENCE=device / none) a device-scope release or no system-
// scope fence instead of the default system-scope fence, whose cache
// writeback and invalidation sit on the waiting stream (hip_runtime_api.h
// hipEventDisableSystemFence).  Events the host waits on before reading what
// kernels stored into pinned memory (ntrack_evt, gate_evt) keep the default.
static unsigned gpu_event_flags() {
    static const unsigned f = [] {
        const char* e = getenv("VISO_EVENT_FENCE");
        unsigned x = hipEventDisableTiming;
        if (e && e[0] == 'd') x |= hipEventReleaseToDevice;
        if (e && e[0] == 'n') x |= hipEventDisableSystemFence;
        return x;
    }();
    return f;
}

// ------------------------------------------------------------------ lifecycle
int viso_ctx::init() {
    const PyrGeom& g = geom;
    const int cap = p.max_features;
    // left + right of a chunk, roles; the free list is FIFO (the longest-free
    // slot is reused first, so side-stream LK reads are long finished)
    n_slots = 2 * p.batch_frames + 8;
    int rc = slot_pool.ensure(g.slot * (size_t)n_slots);
    if (!rc) rc = slot_pose.ensure(sizeof(double) * 12 * (size_t)n_slots);
    if (rc) return rc;
    slots.assign((size_t)n_slots, SlotRec{});
    free_slots.clear();
    for (int s = 0; s < n_slots; ++s) free_slots.push_back(s);
    // tracks
    const size_t kbytes = sizeof(float2) * (size_t)cap;
    if (!rc) rc = kp1.ensure(kbytes);
    if (!rc) rc = kp2.ensure(kbytes);
    if (!rc) rc = kp1b.ensure(kbytes);
    if (!rc) rc = kp2b.ensure(kbytes);
    if (!rc) rc = track_success.ensure((size_t)cap);
    if (!rc) rc = n_track_dev.ensure(256);
    if (!rc) rc = fast_rows.ensure(fast_scratch_bytes(g.w[0], g.h[0]));
    if (rc) return rc;
    fast = fast_scratch_at(fast_rows.ptr, g.w[0], g.h[0]);
    // geometry
    {
        Bump b;
        const size_t o_p1 = b.take(24 * (size_t)cap), o_p2 = b.take(24 * (size_t)cap),
                     o_q1 = b.take(16 * (size_t)cap), o_q2 = b.take(16 * (size_t)cap),
                     o_ctl = b.take(sizeof(GeoCtl)),
                     o_em = b.take(72 * (size_t)std::max(p.ransac_e_iters, 1)),
                     o_ev = b.take((size_t)std::max(p.ransac_e_iters, 1)),
                     o_ec = b.take(4 * (size_t)std::max(p.ransac_e_iters, 1)),
                     o_emk = b.take((size_t)cap),
                     o_hm = b.take(72 * (size_t)std::max(p.ransac_h_iters, 1)),
                     o_hv = b.take((size_t)std::max(p.ransac_h_iters, 1)),
                     o_hc = b.take(4 * (size_t)std::max(p.ransac_h_iters, 1)),
                     o_hmk = b.take((size_t)cap), o_si = b.take((size_t)kMaxCandidates * cap),
                     o_sp = b.take(24 * (size_t)kMaxCandidates * cap), o_in = b.take((size_t)cap),
                     o_po = b.take(24 * (size_t)cap), o_rp = b.take(8 * 24), o_rpg = b.take(16),
                     o_hmom = b.take(8 * 45 * (size_t)cap), o_hM = b.take(8 * 81);
        rc = geo_buf.ensure(b.off);
        if (rc) return rc;
        char* base = (char*)geo_buf.ptr;
        GeoArgs& a = geo;
        std::memset(&a, 0, sizeof(a));
        a.n_dev = (const int*)n_track_dev.ptr;
        a.p1 = (double*)(base + o_p1);
        a.p2 = (double*)(base + o_p2);
        a.q1 = (double*)(base + o_q1);
        a.q2 = (double*)(base + o_q2);
        a.ctl = (GeoCtl*)(base + o_ctl);
        a.e_models = (double*)(base + o_em);
        a.e_valid = (uint8_t*)(base + o_ev);
        a.e_counts = (int*)(base + o_ec);
        a.e_mask = (uint8_t*)(base + o_emk);
        a.h_models = (double*)(base + o_hm);
        a.h_valid = (uint8_t*)(base + o_hv);
        a.h_counts = (int*)(base + o_hc);
        a.h_mask = (uint8_t*)(base + o_hmk);
        a.sel_in = (uint8_t*)(base + o_si);
        a.sel_pts = (double*)(base + o_sp);
        a.inliers = (uint8_t*)(base + o_in);
        a.points_out = (double*)(base + o_po);
        a.rp = (double*)(base + o_rp);
        a.rp_good = (int*)(base + o_rpg);
        a.hm = (double*)(base + o_hmom);
        a.hM = (double*)(base + o_hM);
        a.cap = cap;
        const double K[9] = {p.fx, 0, p.cx, 0, p.fy, p.cy, 0, 0, 1};
        eigen_inverse3(K, Kinv);
        for (int k = 0; k < 9; ++k) a.Kinv[k] = Kinv[k];
        a.K[0] = p.fx;
        a.K[1] = p.fy;
        a.K[2] = p.cx;
        a.K[3] = p.cy;
        a.disparity_thresh = p.disparity_squared_thresh;
        a.proj_thresh = p.projection_error_thresh;
        a.parallax_thresh = p.parallax_thresh;
        a.confidence = p.ransac_confidence;
        // thresh = projection_error_thresh / sqrt(fx^2 + fy^2) (src/viso.cpp:191);
        // OpenCV findInliers compares against (float)(thresh * thresh)
        const double thr = p.projection_error_thresh / std::sqrt(p.fx * p.fx + p.fy * p.fy);
        a.t2 = (float)(thr * thr);
        a.seed = p.ransac_seed;
        a.e_iters = p.ransac_e_iters;
        a.h_iters = p.ransac_h_iters;
    }
    VISO_HIP_CHECK(hipHostMalloc((void**)&h_ctl, sizeof(GeoCtl)));
    VISO_HIP_CHECK(hipHostMalloc((void**)&h_int, 64 * sizeof(int)));
    VISO_HIP_CHECK(hipHostMalloc((void**)&h_dbl, 256 * sizeof(double)));
    std::memset(h_int, 0, 64 * sizeof(int));
    VISO_HIP_CHECK(hipHostGetDevicePointer((void**)&h_int_dev, h_int, 0));
    VISO_HIP_CHECK(hipHostGetDevicePointer((void**)&h_ctl_dev, h_ctl, 0));
    geo.host_ctl = h_ctl_dev;
    // map + tracking
    if (!rc) rc = map_pts.ensure(24 * (size_t)kMaxMapPoints);
    if (!rc) rc = kf_poses.ensure(96 * (size_t)kMaxKeyframes);
    if (!rc) rc = direct_buf.ensure(direct_scratch_bytes());
    if (!rc) rc = direct_stats.ensure(4 * 50 * 8);
    if (!rc) rc = lk_pair.ensure(4 * (size_t)kMaxMapPoints * kLkBatch);
    if (!rc) rc = lk_succ.ensure((size_t)kMaxMapPoints * kLkBatch);
    if (!rc) rc = lk_before.ensure(16 * (size_t)kMaxMapPoints * kLkBatch);
    if (!rc) rc = lk_after.ensure(16 * (size_t)kMaxMapPoints * kLkBatch);
    // the LK-alignment templates at their largest map (96 MiB): a map's
    // creation (an initialisation frame, timed as one) then allocates nothing
    if (!rc) rc = lk_tmpl.ensure((size_t)kMaxMapPoints * kLevels * 192 * 8);
    if (!rc) rc = lk_tmpl_h.ensure((size_t)kMaxMapPoints * kLevels * 4 * 8);
    if (!rc) rc = lk_tmpl_kf.ensure((size_t)kMaxMapPoints * 4);
    if (!rc) rc = lk_tmpl_uv.ensure((size_t)kMaxMapPoints * 16);
    if (!rc) rc = pose_log.ensure(96 * (size_t)std::max(p.max_poses, 1));
    if (rc) return rc;
    direct = direct_scratch_at(direct_buf.ptr);
    for (int i = 0; i < kLkRing; ++i) VISO_HIP_CHECK(hipEventCreateWithFlags(&lk_ring[i], gpu_event_flags()));
    // the background LK grid's resources and its kernel's first launch, here
    // rather than in the first tracking chunk (a hipMalloc, the kernel's
    // dynamic-LDS attribute and code-object load would otherwise land in that
    // chunk: ~0.1 ms)
    VISO_HIP_CHECK(hipEventCreateWithFlags(&geo_fork, gpu_event_flags()));
    VISO_HIP_CHECK(hipEventCreateWithFlags(&geo_join, gpu_event_flags()));
    VISO_HIP_CHECK(hipEventCreateWithFlags(&ntrack_evt, hipEventDisableTiming));
    VISO_HIP_CHECK(hipEventCreateWithFlags(&gate_evt, hipEventDisableTiming));
    for (auto& e : epoch_evt) VISO_HIP_CHECK(hipEventCreateWithFlags(&e, gpu_event_flags()));
    VISO_HIP_CHECK(hipEventCreateWithFlags(&epoch_now, gpu_event_flags()));
    if (const char* e = getenv("VISO_GATE_SPEC")) gate_spec_mode = e[0] == '1' ? 1 : 0;
    rc = bg_prepare();
    if (rc) return rc;
    // the pose getter's pinned staging (viso_get_poses)
    h_poses_cap = (size_t)std::min(std::max(p.max_poses, 1), 4096);
    VISO_HIP_CHECK(hipHostMalloc((void**)&h_poses, 96 * h_poses_cap));
    VISO_HIP_CHECK(hipHostGetDevicePointer((void**)&h_poses_dev, h_poses, 0));
    VISO_HIP_CHECK(hipMemsetAsync(n_track_dev.ptr, 0, 256, stream));
    VISO_HIP_CHECK(hipStreamSynchronize(stream));
    return VISO_OK;
}

void viso_ctx::release() {
    if (lk_stream) (void)hipStreamSynchronize(lk_stream);
    if (up_stream) (void)hipStreamSynchronize(up_stream);
    timing.destroy();
    for (auto& e : lk_ring) {
        if (e) (void)hipEventDestroy(e);
        e = nullptr;
    }
    if (bg_done) (void)hipEventDestroy(bg_done);
    bg_done = nullptr;
    for (hipEvent_t* e : {&geo_fork, &geo_join, &ntrack_evt, &gate_evt}) {
        if (*e) (void)hipEventDestroy(*e);
        *e = nullptr;
    }
    if (lk_stream) (void)hipStreamDestroy(lk_stream);
    lk_stream = nullptr;
    for (auto& e : epoch_evt) {
        if (e) (void)hipEventDestroy(e);
        e = nullptr;
    }
    if (epoch_now) (void)hipEventDestroy(epoch_now);
    epoch_now = nullptr;
    DevBuf* bufs[] = {&scratch_a, &scratch_b, &scratch_c, &scratch_d, &slot_pool, &slot_pose,
                      &kp1, &kp2, &kp1b, &kp2b, &track_success, &n_track_dev, &fast_rows,
                      &geo_buf, &map_pts, &kf_poses, &direct_buf, &direct_stats,
                      &bg_buf, &lk_pair, &lk_succ, &lk_before, &lk_after, &lk_tmpl, &lk_tmpl_h,
                      &lk_tmpl_kf, &lk_tmpl_uv, &pose_log, &frame_log, &hbg_buf};
    for (DevBuf* b : bufs) b->release();
    if (h_ctl) (void)hipHostFree(h_ctl);
    if (h_int) (void)hipHostFree(h_int);
    if (h_dbl) (void)hipHostFree(h_dbl);
    if (h_poses) (void)hipHostFree(h_poses);
    stage.release();
    if (up_stream) (void)hipStreamDestroy(up_stream);
    up_stream = nullptr;
    h_ctl = nullptr;
    h_int = nullptr;
    h_dbl = nullptr;
    h_poses = nullptr;
    h_poses_dev = nullptr;
    h_poses_cap = 0;
}

// The context stream and the LK-alignment side stream (single-frame calls).
// The side stream gets a hardware queue of its own: a stream created with a
// CU mask (here every CU) is never mapped onto a queue another stream uses,
// while plain streams share the process's few queues (GPU_MAX_HW_QUEUES)
// round-robin — and a chunk-resident LK grid on a queue shared with the
// context stream would sit in front of the very chain it waits for.  When
// the masked stream cannot be made, the background mode stays off.
int viso_ctx::create_streams() {
    if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return VISO_ERR_HIP;
    int cus = 0;
    const char* q = getenv("VISO_LK_QUEUE");  // dev: "shared" = a plain stream
    if (!(q && q[0] == 's') &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0) {
        std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0u);
        for (int c = 0; c < cus; ++c) mask[(size_t)c / 32] |= 1u << (c % 32);
        if (hipExtStreamCreateWithCUMask(&lk_stream, (uint32_t)mask.size(), mask.data()) != hipSuccess)
            lk_stream = nullptr;
        lk_dedicated = lk_stream != nullptr;
    }
    if (!lk_stream) {
        (void)hipGetLastError();
        if (!(q && q[0] == 's')) bg_mode = 0;
        if (hipStreamCreateWithFlags(&lk_stream, hipStreamNonBlocking) != hipSuccess) return VISO_ERR_HIP;
    }
    return VISO_OK;
}

// The upload stream (host ingest), with a hardware queue of its own when a
// CU-masked stream can be made (a plain stream may share the context
// stream's queue, behind the chain it should overlap: still correct).
int viso_ctx::create_up_stream() {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0) {
        std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0u);
        for (int c = 0; c < cus; ++c) mask[(size_t)c / 32] |= 1u << (c % 32);
        if (hipExtStreamCreateWithCUMask(&up_stream, (uint32_t)mask.size(), mask.data()) != hipSuccess)
            up_stream = nullptr;
        up_dedicated = up_stream != nullptr;
    }
    if (!up_stream) {
        (void)hipGetLastError();
        if (hipStreamCreateWithFlags(&up_stream, hipStreamNonBlocking) != hipSuccess) return VISO_ERR_HIP;
    }
    return VISO_OK;
}

// ------------------------------------------------------------------ frame pool
int viso_ctx::acquire_slot(hipStream_t lk_wait) {
    if (free_slots.empty()) return -1;
    int s = free_slots.front();
    free_slots.pop_front();
    // lk_stream may still read this slot's previous frame: order the reuse
    // (on the stream that writes it first: the context stream, or the upload
    // stream) behind that batch (a no-op wait in steady state; a later batch
    // on the same stream also implies completion)
    if (order_after_lk(slots[(size_t)s].lk_use, lk_wait ? lk_wait : stream)) {
        free_slots.push_front(s);
        return -1;
    }
    const int64_t fe = slots[(size_t)s].free_epoch;
    slots[(size_t)s] = SlotRec{};
    slots[(size_t)s].l0 = slot_base(s);
    slots[(size_t)s].free_epoch = fe;
    return s;
}

// Order `st` behind lk_stream batch `use` — unless the host already knows it
// is complete (a query of its event, or of a later one) or `st` already waits
// for it or a later batch.  A cross-queue wait is a barrier packet costing the
// waiting queue ~6-10 us even when its event completed long ago (round 6),
// and a device-ingest caller past the pool's first lap reuses a slot per
// frame.  Batches older than the event ring are covered by its oldest event
// (lk_stream runs them in order).
int viso_ctx::order_after_lk(int64_t use, hipStream_t st) {
    if (use < 0 || use >= lk_seq || use < lk_done) return VISO_OK;
    int64_t* waited = st == stream ? &lk_waited_ctx : st == up_stream ? &lk_waited_up : nullptr;
    if (waited && use < *waited) return VISO_OK;
    const int64_t e = (lk_seq - use <= kLkRing) ? use : lk_seq - kLkRing;
    const hipError_t q = hipEventQuery(lk_ring[e % kLkRing]);
    if (q == hipSuccess) {
        lk_done = std::max(lk_done, e + 1);
        return VISO_OK;
    }
    if (q != hipErrorNotReady) return VISO_ERR_HIP;
    (void)hipGetLastError();  // (the query's own status)
    VISO_HIP_CHECK(hipStreamWaitEvent(st, lk_ring[e % kLkRing], 0));
    if (waited) *waited = e + 1;
    return VISO_OK;
}

// The end of an ingest call: an event behind its work on the context stream
// (the reuse of a slot it freed is ordered behind it on the upload stream).
// Every event record on the context stream costs it a marker packet (~6-10
// us of the queue's time on MI355X, gpurun_out/r06h: a host-frame caller paid
// one per frame), so an epoch is recorded only every kEpochStride calls; a
// slot's reuse waits for the oldest record made at or after the call that
// freed it (wait_freed).
int viso_ctx::end_epoch() {
    if (epoch - epoch_last_rec >= kEpochStride) {
        const int k = (int)(epoch_nrec % kEpochRing);
        VISO_HIP_CHECK(hipEventRecord(epoch_evt[k], stream));
        epoch_rec_call[k] = epoch;
        epoch_last_rec = epoch;
        ++epoch_nrec;
    }
    ++epoch;
    return VISO_OK;
}

// Order work on `st` behind the context-stream work of call fe (the call
// that freed a slot): the oldest epoch record made at or after it (records
// are in call order on the in-order context stream), else — freed after the
// last record — a record now, behind everything enqueued so far.
int viso_ctx::wait_freed(int64_t fe, hipStream_t st) {
    if (fe < 0) return VISO_OK;
    const int64_t m = std::min<int64_t>(epoch_nrec, kEpochRing);
    for (int64_t j = epoch_nrec - m; j < epoch_nrec; ++j) {
        const int k = (int)(j % kEpochRing);
        if (epoch_rec_call[k] >= fe) {
            // (no barrier packet when the host sees the record complete)
            const hipError_t q = hipEventQuery(epoch_evt[k]);
            if (q == hipSuccess) return VISO_OK;
            if (q != hipErrorNotReady) return VISO_ERR_HIP;
            (void)hipGetLastError();
            VISO_HIP_CHECK(hipStreamWaitEvent(st, epoch_evt[k], 0));
            return VISO_OK;
        }
    }
    VISO_HIP_CHECK(hipEventRecord(epoch_now, stream));
    VISO_HIP_CHECK(hipStreamWaitEvent(st, epoch_now, 0));
    return VISO_OK;
}

// Host frame -> slot s's level 0 through the pinned staging, on the upload
// stream: behind the slot's last readers (its lk_stream batch: acquire_slot;
// the context stream's: the epoch that freed it), and the context stream
// waits for the DMA before the frame's pyramid.
int viso_ctx::upload_host(int s, const uint8_t* grey, int32_t w, int32_t h, int32_t stride, bool pyramid) {
    if (int rc = wait_freed(slots[(size_t)s].free_epoch, up_stream)) return rc;
    {
        TimedRegion t(timing, VISO_KERNEL_UPLOAD, up_stream);
        dev_tl.mark(frames, 0, up_stream);
        VISO_HIP_CHECK(stage.upload(slot_base(s), grey, w, h, stride, up_stream, true));
        dev_tl.mark(frames, 1, up_stream);
    }
    if (pyramid) {
        // the frame's pyramid behind its upload, on the same stream: both
        // beside the previous frame's chain
        uint8_t* slot = slot_base(s);
        const uint8_t* l0 = slot;
        launch_ingest_pyramid(&l0, &slot, &s, 1, false, up_stream);
        VISO_HIP_CHECK(hipGetLastError());
        dev_tl.mark(frames, 2, up_stream);
    }
    // one event behind the DMA (and the pyramid): the staging buffer's reuse
    // and the context stream's wait share it — each record is a marker packet
    // on its queue and each cross-queue wait a barrier packet (round 6: ~6-10
    // us of a queue's time each, gpurun_out/r06h), and this path pays them per
    // frame
    VISO_HIP_CHECK(stage.commit(up_stream));
    VISO_HIP_CHECK(hipStreamWaitEvent(stream, stage.last, 0));
    return VISO_OK;
}

void viso_ctx::hold(int s) {
    if (s >= 0) slots[(size_t)s].refs += 1;
}

void viso_ctx::drop(int s) {
    if (s < 0) return;
    SlotRec& r = slots[(size_t)s];
    if (--r.refs == 0) {
        r.free_epoch = epoch;
        free_slots.push_back(s);
    }
}

void viso_ctx::set_role(int& role, int s) {
    if (role == s) return;
    hold(s);
    drop(role);
    role = s;
}

uint8_t* viso_ctx::slot_base(int s) const { return (uint8_t*)slot_pool.ptr + geom.slot * (size_t)s; }

double* viso_ctx::pose_of(int s) const { return (double*)slot_pose.ptr + 12 * (size_t)s; }

FrameDev viso_ctx::frame(int s) const {
    FrameDev f = frame_from_base(slot_base(s), geom);
    f.l[0] = slots[(size_t)s].l0;
    return f;
}

// A retained frame must not keep pointing into the caller's buffer.
int viso_ctx::own_level0(int s) {
    if (s < 0) return VISO_OK;
    SlotRec& r = slots[(size_t)s];
    if (!r.borrowed) return VISO_OK;
    VISO_HIP_CHECK(hipMemcpyAsync(slot_base(s), r.l0, (size_t)geom.w[0] * geom.h[0],
                                  hipMemcpyDeviceToDevice, stream));
    r.l0 = slot_base(s);
    r.borrowed = false;
    return VISO_OK;
}

// ready flags [kLkBatch], eight heads on lines of their own, 32 spare words,
// leftover list (cursor, count, ..., 4096 items); + 32 words past them: the
// error word and the drain's item count, kept across chunks (sticky) until
// bg_check reads and clears them
static constexpr size_t kBgWords = kLkBatch + 8 * 32 + 32 + 32 + 4096;

// The ingest's pyramid.  Its last frame is last_frame when the call ends, so
// its level 0 would be copied into its slot at the end anyway (own_level0):
// the tail launch copies it instead (small chunks; a large one's bands would
// serialise the copy), and outside tracking also writes that
// frame's Keyframe-ctor pose (R = I, T = 0; on_new_frame skips its launch) —
// a frame-by-frame caller pays two launches fewer per frame.
void viso_ctx::launch_ingest_pyramid(const uint8_t* const* l0, uint8_t* const* dst, const int* sl, int n,
                                     bool bg_words, hipStream_t st) {
    if (!st) st = stream;
    const int s = sl[n - 1];
    PyrOwn own{n - 1, state != VISO_STATE_RUNNING ? pose_of(s) : nullptr, false};
    if (n == 1 && st == stream && fast_pre_slot == s && fast_pre.img) own.fast = &fast_pre;
    if (bg_words) {  // the chunk's background-LK words (bg_begin), cleared by the tail launch
        // (the set the next chunk uses: two sets alternate, so the previous
        // chunk's grid and drain, which may still run on lk_stream, read the
        // other; this one's last readers, two chunks back, are ordered first)
        const int set = bg_set ^ 1;
        (void)order_after_lk(bg_set_seq[set], st);
        own.zero = bg_words_of(set);
        own.n_zero = (int)kBgWords;
    }
    ident_slot = own.ident_pose ? s : -1;
    {
        TimedRegion t(timing, VISO_KERNEL_PYRAMID, st);
        launch_pyramid_frames(geom, l0, dst, n, st, &own);
    }
    // (viso_get_config [6], [7]: what the tail launch did beside the levels)
    tail_copy_bytes = own.copied ? (int)((size_t)geom.w[0] * geom.h[0]) : 0;
    tail_zero_ints = own.n_zero;
    SlotRec& r = slots[(size_t)s];
    if (r.borrowed && own.copied) {
        r.l0 = slot_base(s);
        r.borrowed = false;
    }
}

int viso_ctx::ingest_host(const uint8_t* grey, int32_t w, int32_t h, int32_t stride, int* slot_out, bool pyramid) {
    if (w != p.width || h != p.height || stride < w || !grey) return VISO_ERR_ARG;
    if (!up_stream) {
        int rc = create_up_stream();
        if (rc) return rc;
    }
    int s = acquire_slot(up_stream);
    if (s < 0) return VISO_ERR_CAPACITY;
    // through pinned staging (staging.hpp: a pageable hipMemcpy2DAsync
    // measured 3.25 ms per 1242x375 frame), on the upload stream
    const int rc = upload_host(s, grey, w, h, stride, pyramid);
    if (rc) {
        hold(s);
        drop(s);
        return rc;
    }
    *slot_out = s;
    return VISO_OK;
}

// ------------------------------------------------------------------ LKAlignment batch
LkAlignArgs viso_ctx::lk_args() {
    const PyrGeom& g = geom;
    LkAlignArgs a{};
    a.n_kf = (int)kf_slots.size();
    for (int j = 0; j < a.n_kf; ++j) a.kf[j] = frame(kf_slots[(size_t)j]);
    a.kf_poses = (const double*)kf_poses.ptr;
    a.points = (const double*)map_pts.ptr;
    a.n = n_map;
    a.K[0] = p.fx;
    a.K[1] = p.fy;
    a.K[2] = p.cx;
    a.K[3] = p.cy;
    a.thresh = p.photometric_error_thresh;
    for (int l = 0; l < kLevels; ++l) {
        a.g.w[l] = g.w[l];
        a.g.h[l] = g.h[l];
        a.g.off[l] = g.off[l];
    }
    a.tmpl = (double*)lk_tmpl.ptr;
    a.tmpl_h = (double*)lk_tmpl_h.ptr;
    a.tmpl_kf = (int32_t*)lk_tmpl_kf.ptr;
    a.tmpl_uv = (double*)lk_tmpl_uv.ptr;
    a.fast = p.precision == VISO_PRECISION_FAST ? 1 : 0;
    return a;
}

int viso_ctx::flush_lk(hipStream_t ls) { return flush_lk_frames(ls, false); }

int viso_ctx::flush_lk_frames(hipStream_t ls, bool keep_last) {
    if (lk_pending.empty() || (keep_last && lk_pending.size() < 2)) return VISO_OK;
    int kept = -1;
    if (keep_last) {
        kept = lk_pending.back();
        lk_pending.pop_back();
    }
    LkAlignArgs a = lk_args();
    a.n_frames = (int)lk_pending.size();
    for (int f = 0; f < a.n_frames; ++f) {
        a.frames[f].cur = frame(lk_pending[(size_t)f]);
        a.frames[f].pose = pose_of(lk_pending[(size_t)f]);
    }
    a.out_stride = kMaxMapPoints;
    a.pair_kf = (int32_t*)lk_pair.ptr;
    a.success = (uint8_t*)lk_succ.ptr;
    a.uv_before = (double*)lk_before.ptr;
    a.uv_after = (double*)lk_after.ptr;
    const bool side = ls != stream;
    if (side) {
        // the frames' poses come from the context stream
        VISO_HIP_CHECK(hipEventRecord(lk_ring[lk_seq % kLkRing], stream));
        VISO_HIP_CHECK(hipStreamWaitEvent(ls, lk_ring[lk_seq % kLkRing], 0));
    } else if (lk_seq > 0) {
        // the outputs may still be read by the last side batch's getters:
        // order behind the last side batch
        if (int rc = order_after_lk(lk_seq - 1, stream)) return rc;
    }
    // A host-frame caller's batch (side stream, beside the next frames'
    // chains): the chunk-resident grid's geometry — one workgroup per CU in
    // each CU's spare wave slots, below the chain's priority — with every
    // frame's ready flag already up (their poses are final), instead of a
    // full-occupancy launch whose workgroups hold the CUs the next frame's
    // direct launches need (VISO_HOST_LK=batch: the latter).
    const bool grid = side && host_lk_grid();
    if (grid) {
        if (int rc = host_grid_args(a, ls)) return rc;
    }
    {
        TimedRegion t(timing, VISO_KERNEL_LKALIGN, ls);
        if (grid)
            launch_lk_bg(a, n_cu, ls);
        else
            launch_lk_align(a, ls);
    }
    VISO_HIP_CHECK(hipGetLastError());
    if (int rc = count_lk(lk_pending, ls)) return rc;
    lk_last_rows = a.n_frames;
    lk_last_pts = n_map;  // a later keyframe insertion grows n_map, not these rows
    if (side) {
        VISO_HIP_CHECK(hipEventRecord(lk_ring[lk_seq % kLkRing], ls));
        for (int s : lk_pending) slots[(size_t)s].lk_use = lk_seq;
        for (int s : kf_slots) slots[(size_t)s].lk_use = lk_seq;
        ++lk_seq;
    }
    for (int s : lk_pending) drop(s);
    lk_pending.clear();
    if (kept >= 0) lk_pending.push_back(kept);
    return VISO_OK;
}

bool viso_ctx::host_lk_grid() {
    if (host_lk_mode < 0) {
        const char* e = getenv("VISO_HOST_LK");
        host_lk_mode = (e && e[0] == 'b') ? 0 : 1;
    }
    return host_lk_mode && bg_on() && direct_fits_background() && lk_tmpl.ptr;
}

// The words of a host batch's resident grid (their own buffer: a device-
// ingest chunk's words are cleared on the context stream while this grid may
// still run on the side stream): ready flags all up (set once), the heads and
// the leftover header cleared per batch on the batch's stream; at most two
// such batches outstanding (the grid shares the chain's CUs, so a caller far
// ahead of it would otherwise hold ever more frame slots).
int viso_ctx::host_grid_args(LkAlignArgs& a, hipStream_t ls) {
    constexpr size_t kHdr = 8 * 32 + 32 + 32;  // heads + leftover header
    if (!hbg_buf.ptr) {
        if (int rc = hbg_buf.ensure(sizeof(int) * (kBgWords + 32))) return rc;
        VISO_HIP_CHECK(hipMemsetAsync(hbg_buf.ptr, 0, sizeof(int) * (kBgWords + 32), ls));
        VISO_HIP_CHECK(hipMemsetD32Async((hipDeviceptr_t)hbg_buf.ptr, 1, kLkBatch, ls));
    }
    if (lk_seq >= 2) VISO_HIP_CHECK(hipEventSynchronize(lk_ring[(lk_seq - 2) % kLkRing]));
    int* w = (int*)hbg_buf.ptr;
    VISO_HIP_CHECK(hipMemsetAsync(w + kLkBatch, 0, sizeof(int) * kHdr, ls));
    a.bg_ready = w;
    a.bg_next = w + kLkBatch;
    a.bg_left = a.bg_next + 8 * 32 + 32;
    a.bg_err = w + kBgWords;
    a.bg_err_host = h_int_dev + 32;
    a.bg_items = a.n_frames * n_map;
    bg_unchecked = true;
    return VISO_OK;
}

// Frames of LK alignment a host-frame caller may leave queued: each holds its
// slot, so the pool keeps room for the roles (ref, last, keyframes) and the
// next frames.
int viso_ctx::host_lk_batch() const {
    const int room = (n_slots - (int)kf_slots.size() - 6) / 2;
    return std::max(1, std::min(8, room));
}

int viso_ctx::finish_host_call() {
    // outside tracking, and with keyframe insertion (its decision reads the
    // frame's nGood at once), as every other call
    if (state != VISO_STATE_RUNNING || kf_interval > 0 || bg_active) return finish_call(lk_stream);
    // the queued frames but the last have their final poses on the context
    // stream by now (each one's final solve ran in its successor's L(3))
    if ((int)lk_pending.size() > host_lk_batch()) return flush_lk_frames(lk_stream, true);
    return VISO_OK;
}

int viso_ctx::settle() {
    if (!host_q.empty()) {
        VISO_HIP_CHECK(hipSetDevice(device));
        if (int rc = flush_host_q()) return rc;
    }
    if (!dpend && lk_pending.empty()) return VISO_OK;
    VISO_HIP_CHECK(hipSetDevice(device));
    return finish_call(lk_stream);
}

// Host frames while tracking (viso_process_frame): each call only uploads its
// frame (the DMA on the upload stream) and queues it; queued frames run as a
// device-ingest chunk (ingest_chunk: one batched pyramid launch, the
// background LK grid, one cross-queue wait for the DMAs) once host_chunk are
// queued, or at once when the context's previous chunk has finished (so a
// caller slower than the GPU gets each frame started right away), and
// whenever anything else is called (settle).  Per frame that leaves the
// chain and the DMA; per chunk the pyramid launch pair, the grid and its end.
// VISO_HOST_CHUNK=0 turns it off (the frame-by-frame path below).
bool viso_ctx::host_queue_eligible() {
    if (host_chunk < 0) {
        const char* e = getenv("VISO_HOST_CHUNK");
        host_chunk = e ? std::max(0, std::min(kLkBatch, atoi(e))) : 16;
    }
    return host_chunk > 0 && state == VISO_STATE_RUNNING && kf_interval <= 0 && bg_on() &&
           direct_fits_background() && n_map > 0 && lk_tmpl.ptr;
}

int viso_ctx::queue_host_frame(const uint8_t* grey, int32_t w, int32_t h, int32_t stride) {
    if (w != p.width || h != p.height || stride < w || !grey) return VISO_ERR_ARG;
    // per-frame work left by the frame-by-frame path first (in order)
    if (dpend || !lk_pending.empty()) {
        if (int rc = finish_call(lk_stream)) return rc;
    }
    if (!up_stream) {
        if (int rc = create_up_stream()) return rc;
    }
    int s = acquire_slot(up_stream);
    if (s < 0 && !host_q.empty()) {  // the queue holds the pool's last slots
        if (int rc = flush_host_q()) return rc;
        s = acquire_slot(up_stream);
    }
    if (s < 0) return VISO_ERR_CAPACITY;
    if (int rc = wait_freed(slots[(size_t)s].free_epoch, up_stream)) {
        hold(s);
        drop(s);
        return rc;
    }
    {
        TimedRegion t(timing, VISO_KERNEL_UPLOAD, up_stream);
        const hipError_t e = stage.upload(slot_base(s), grey, w, h, stride, up_stream);
        if (e != hipSuccess) {
            hold(s);
            drop(s);
            return VISO_ERR_HIP;
        }
    }
    hold(s);  // queued
    host_q.push_back(s);
    bool idle = true;
    if (lk_seq > 0) {
        // the previous chunk's end: its grid's event (lk_stream), recorded after
        // the chunk's last pose
        const hipError_t q = hipEventQuery(lk_ring[(lk_seq - 1) % kLkRing]);
        if (q == hipErrorNotReady) {
            (void)hipGetLastError();
            idle = false;
        } else if (q != hipSuccess) {
            return VISO_ERR_HIP;
        }
    }
    if ((int)host_q.size() >= host_chunk || idle) return flush_host_q();
    return VISO_OK;
}

int viso_ctx::flush_host_q() {
    if (host_q.empty()) return VISO_OK;
    std::vector<int> sl;
    sl.swap(host_q);
    // the chunk's DMAs (the upload stream is in order: its last one)
    if (hipStreamWaitEvent(stream, stage.last, 0) != hipSuccess) {
        for (int s : sl) drop(s);
        return VISO_ERR_HIP;
    }
    std::vector<const uint8_t*> l0;
    for (int s : sl) l0.push_back(slot_base(s));
    return ingest_chunk(sl, l0, {}, tail_overlap_on());
}

int viso_ctx::resolve_direct() {
    if (!dpend) return VISO_OK;
    const double K[4] = {p.fx, p.fy, p.cx, p.cy};
    launch_direct_final(frame(dpend_last), frame(dpend_cur), geom, K, (const double*)map_pts.ptr,
                        n_map, pose_of(dpend_last), direct, (double*)direct_stats.ptr,
                        pose_of(dpend_cur), dpend_log >= 0 ? (double*)pose_log.ptr : nullptr,
                        dpend_log, stream, p.precision, bg_ready(dpend_bg), log_host(dpend_log), flog());
    VISO_HIP_CHECK(hipGetLastError());
    drop(dpend_cur);
    drop(dpend_last);
    dpend = false;
    return VISO_OK;
}

int viso_ctx::finish_call(hipStream_t ls, bool overlap) {
    int rc = resolve_direct();
    if (rc) {
        // still tear the background state down (its held frames, the pending
        // ready-flag owner), so the next call does not inherit a dead chunk
        if (bg_active) (void)bg_end(false);
        return rc;
    }
    if (bg_active) {
        rc = bg_end(true, overlap);
        if (rc) return rc;
    }
    return flush_lk(ls);
}

// Every pose of the log is final once an ingest call has ended (the last
// frame's by its final solve, launched in finish_call): viso_synchronize
// copies the new ones into the pinned staging ahead of its stream sync, so a
// viso_get_poses after it reads host memory instead of making its own device
// round trip (enqueued per ingest call instead, the copy cost frame-by-frame
// callers ~10 us per frame).
int viso_ctx::stage_poses() {
    const size_t m = std::min((size_t)n_poses, (size_t)std::max(p.max_poses, 0));
    if (m <= poses_staged || m > h_poses_cap || !h_poses) return VISO_OK;
    // the direct kernels logged every pose below h_poses_cap into h_poses
    // too (log_host): nothing to copy
    if (h_poses_dev) {
        poses_staged = m;
        return VISO_OK;
    }
    VISO_HIP_CHECK(hipMemcpyAsync(h_poses + 12 * poses_staged, (const double*)pose_log.ptr + 12 * poses_staged,
                                  96 * (m - poses_staged), hipMemcpyDeviceToHost, stream));
    poses_staged = m;
    return VISO_OK;
}

// Background LK alignment: eligible when the context is
// tracking at the chunk's start with a map and its LK templates, no keyframe
// insertion can change the map mid-chunk, and the direct pose's workgroup
// leaves a CU room for the background one (direct_fits_background).  Every
// frame of such a chunk is a tracking frame, so every ready flag is raised:
// frame f's by frame f+1's merged level-3 launch, the last by the final solve.
bool viso_ctx::bg_eligible() { return bg_on() && direct_fits_background() && state == VISO_STATE_RUNNING && n_map > 0 &&
                                      lk_tmpl.ptr && kf_interval <= 0 && !dpend && lk_pending.empty(); }

// (VISO_LK_TAIL=0: every chunk's drain on the context stream, as round 5)
bool viso_ctx::tail_overlap_on() {
    if (tail_mode < 0) {
        const char* e = getenv("VISO_LK_TAIL");
        tail_mode = (e && e[0] == '0') ? 0 : 1;
    }
    return tail_mode != 0;
}

int* viso_ctx::bg_words_of(int set) const { return (int*)bg_buf.ptr + (size_t)set * kBgWords; }

bool viso_ctx::bg_on() {
    if (bg_mode < 0) {
        // off on request, and when kernels are serialised (the resident grid
        // would wait out its flag timeouts behind the chain it waits for)
        const char* e = getenv("VISO_LK_BG");
        const char* ser = getenv("AMD_SERIALIZE_KERNEL");
        const char* blk = getenv("HIP_LAUNCH_BLOCKING");
        bg_mode = (e && e[0] == '0') || (ser && ser[0] && ser[0] != '0') || (blk && blk[0] && blk[0] != '0') ? 0 : 1;
    }
    return bg_mode != 0;
}


int viso_ctx::bg_prepare() {
    VISO_HIP_CHECK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device));
    VISO_HIP_CHECK(hipEventCreateWithFlags(&bg_done, gpu_event_flags()));
    // two word sets (alternating chunks) + the sticky error words
    int rc = bg_buf.ensure(sizeof(int) * (2 * kBgWords + 32));
    if (rc) return rc;
    VISO_HIP_CHECK(hipMemsetAsync(bg_buf.ptr, 0, sizeof(int) * (2 * kBgWords + 32), stream));
    warm_lk_bg(stream);
    // lk_stream's first dispatch (its hardware queue is brought up then) and
    // a cross-stream event hand-off, here rather than in the first chunk's
    // background launch
    VISO_HIP_CHECK(hipEventRecord(geo_fork, stream));
    VISO_HIP_CHECK(hipStreamWaitEvent(lk_stream, geo_fork, 0));
    warm_lk_bg(lk_stream);
    VISO_HIP_CHECK(hipEventRecord(geo_join, lk_stream));
    VISO_HIP_CHECK(hipStreamWaitEvent(stream, geo_join, 0));
    VISO_HIP_CHECK(hipGetLastError());
    return VISO_OK;
}

int viso_ctx::bg_begin(const std::vector<int>& chunk, bool zeroed) {
    const int nb = (int)chunk.size();
    if (!bg_eligible() || nb < 1 || nb > kLkBatch) return VISO_OK;
    const size_t bg_words = kBgWords;
    LkAlignArgs a = lk_args();
    a.n_frames = nb;
    for (int f = 0; f < nb; ++f) {
        a.frames[f].cur = frame(chunk[(size_t)f]);
        a.frames[f].pose = pose_of(chunk[(size_t)f]);
    }
    a.out_stride = kMaxMapPoints;
    a.pair_kf = (int32_t*)lk_pair.ptr;
    a.success = (uint8_t*)lk_succ.ptr;
    a.uv_before = (double*)lk_before.ptr;
    a.uv_after = (double*)lk_after.ptr;
    const int set = bg_set ^ 1;  // (the set the pyramid tail cleared)
    a.bg_ready = bg_words_of(set);
    a.bg_next = a.bg_ready + kLkBatch;
    a.bg_left = a.bg_next + 8 * 32 + 32;
    a.bg_err = (int*)bg_buf.ptr + 2 * bg_words;
    a.bg_err_host = h_int_dev + 32;
    a.bg_items = nb * n_map;
    // tests: VISO_LK_BG_IDLE_US shortens the resident waves' patience, so the
    // leftover list and the drain carry most items
    if (const char* f = getenv("VISO_LK_BG_INJECT_FAIL")) a.bg_inject_fail = f[0] == '1';
    if (const char* idle = getenv("VISO_LK_BG_IDLE_US")) {
        const long us = strtol(idle, nullptr, 10);
        if (us > 0 && us < 1000000) a.bg_idle = (unsigned int)(us * 100);
    }
    // flags, heads and leftovers cleared by the chunk's pyramid tail launch
    // (zeroed; else a memset behind it — round 5 measured the memset's
    // launch and gaps at ~10 us of the chunk's start); the grid
    // (on the side stream's own hardware queue, create_streams) starts behind
    // them.  The grid itself is launched once the chunk's first frame is
    // enqueued (bg_launch): its host-side cost (the cross-stream wait, the
    // launch on the masked queue, ~30 us) then overlaps that frame's chain
    // instead of holding the chain's first launch back.
    if (!zeroed) {
        if (int rc = order_after_lk(bg_set_seq[set], stream)) return rc;
        VISO_HIP_CHECK(hipMemsetAsync(a.bg_ready, 0, sizeof(int) * bg_words, stream));
    }
    VISO_HIP_CHECK(hipEventRecord(bg_done, stream));
    bg_set = set;
    bg_args = a;
    bg_active = true;
    bg_unchecked = true;
    bg_launched = false;
    bg_nb = nb;
    bg_slots.clear();
    return VISO_OK;
}

// (bg_done holds the memset of bg_begin until the grid's own record below)
int viso_ctx::bg_launch() {
    if (!bg_active || bg_launched) return VISO_OK;
    bg_launched = true;
    VISO_HIP_CHECK(hipStreamWaitEvent(lk_stream, bg_done, 0));
    {
        TimedRegion t(timing, VISO_KERNEL_LKALIGN, lk_stream);
        launch_lk_bg(bg_args, n_cu, lk_stream);
    }
    VISO_HIP_CHECK(hipGetLastError());
    VISO_HIP_CHECK(hipEventRecord(bg_done, lk_stream));
    return VISO_OK;
}

int viso_ctx::bg_check() {
    if (!bg_unchecked || !bg_buf.ptr) return VISO_OK;
    // the error word is in pinned memory (bg_err_host; the drain's item
    // count too in VISO_DRAIN_COUNT builds, copied behind the drain): final
    // once the context stream has passed the drain and the grid (bg_end)
    VISO_HIP_CHECK(hipStreamSynchronize(stream));
    const int w[2] = {h_int[32], h_int[33]};
    bg_unchecked = false;
    if (w[0] || w[1]) {
        VISO_HIP_CHECK(hipMemsetAsync(bg_args.bg_err, 0, 2 * sizeof(int), stream));
        h_int[32] = h_int[33] = 0;
    }
    if (getenv("VISO_LK_BG_STATS"))  // dev: how much of the last chunk the drain carried
        fprintf(stderr, "viso lk-bg: %d frames x %d points, drain ran %d items (builds with VISO_DRAIN_COUNT), error %d\n",
                bg_nb, n_map, w[1], w[0]);
    return w[0] ? VISO_ERR_HIP : VISO_OK;
}

// The chunk's last pose is launched: the items the resident grid has not
// taken run on the rest of the chip (the drain, behind the final solve on the
// context stream), then the context stream waits for the resident grid (its
// outputs, the held frames), which is the latest LK batch of the flush_lk
// bookkeeping.
int viso_ctx::bg_end(bool drain, bool overlap) {
    // a chunk whose first frame ended in an error before bg_launch (drain =
    // false) has no grid: bg_done still marks the memset, so the waits below
    // hold nothing back
    if (drain) {
        const int rc = bg_launch();
        if (rc) return rc;
    }
    // (drain = false: the error path of finish_call; the chunk's last pose was
    // not launched, so no drain runs: the resident grid's waves give their
    // items back and leave, and the context stream only waits for them)
    if (drain && overlap) {
        // a chunk another one follows: the drain goes on lk_stream behind the
        // resident grid, in the grid's geometry (one workgroup per CU beside
        // the chain's), so the chunk's LK tail (its last frame's points, whose
        // pose the final solve gives) overlaps the next chunk's pyramid and
        // chain instead of holding the context stream ~60-70 us
        LkAlignArgs d = bg_args;
        d.bg_drain = 1;
        launch_lk_bg(d, n_cu, lk_stream);
        VISO_HIP_CHECK(hipGetLastError());
        VISO_HIP_CHECK(hipEventRecord(bg_done, lk_stream));
    } else if (drain) {
        LkAlignArgs d = bg_args;
        d.bg_drain = 1;
        launch_lk_drain(d, 3 * n_cu, stream);
        VISO_HIP_CHECK(hipGetLastError());
    }
    // The context stream does not wait for the resident grid here (a
    // barrier packet at every chunk's end, on the chain's queue): what it
    // protects — the grid's words, cleared by the next chunk's pyramid tail —
    // is ordered there (bg_grid_pending); slot reuse and the batched LK
    // launch by their own lk_use / lk_seq ordering (order_after_lk); the
    // getters synchronise lk_stream.  The per-frame log's count reads the
    // rows on the context stream, so it keeps the wait.
    if (drain && flog()) {
        VISO_HIP_CHECK(hipStreamWaitEvent(stream, bg_done, 0));
        if (int rc = count_lk(bg_slots, stream)) return rc;
    } else if (!drain) {
        VISO_HIP_CHECK(hipStreamWaitEvent(stream, bg_done, 0));
    }
    // the error word reaches h_int[32] from the failing wave itself
    // (bg_err_host); the drain's item count (dev builds) by a copy
#ifdef VISO_DRAIN_COUNT
    VISO_HIP_CHECK(hipMemcpyAsync(h_int + 32, bg_args.bg_err, 2 * sizeof(int), hipMemcpyDeviceToHost, stream));
#endif
    lk_last_rows = bg_nb;
    lk_last_pts = n_map;
    VISO_HIP_CHECK(hipEventRecord(lk_ring[lk_seq % kLkRing], lk_stream));
    for (int s : bg_slots) slots[(size_t)s].lk_use = lk_seq;
    for (int s : kf_slots) slots[(size_t)s].lk_use = lk_seq;
    // (the words' last readers: this batch's grid, and its drain when it ran
    // on lk_stream; a drain on the context stream precedes any later clearing
    // there)
    bg_set_seq[bg_set] = lk_seq;
    ++lk_seq;
    for (int s : bg_slots) drop(s);
    bg_slots.clear();
    bg_active = false;
    dpend_bg = -1;
    return VISO_OK;
}

int viso_ctx::count_lk(const std::vector<int>& row_slots, hipStream_t s) {
    if (!flog() || row_slots.empty()) return VISO_OK;
    LkCountArgs rows{};
    const int n = std::min((int)row_slots.size(), kLkBatch);
    for (int f = 0; f < n; ++f) rows.idx[f] = slots[(size_t)row_slots[(size_t)f]].log_index;
    launch_lk_count((const int32_t*)lk_pair.ptr, (const uint8_t*)lk_succ.ptr, kMaxMapPoints, n_map, n, rows, flog(),
                    s);
    VISO_HIP_CHECK(hipGetLastError());
    return VISO_OK;
}

int viso_ctx::build_lk_templates() {
    const size_t m = (size_t)std::max(n_map, 1);
    int rc = lk_tmpl.ensure(m * kLevels * 192 * 8);
    if (!rc) rc = lk_tmpl_h.ensure(m * kLevels * 4 * 8);
    if (!rc) rc = lk_tmpl_kf.ensure(m * 4);
    if (!rc) rc = lk_tmpl_uv.ensure(m * 16);
    if (rc) return rc;
    launch_lk_template(lk_args(), stream);
    return VISO_OK;
}

// FAST on the left image of `cur`, stereo points on it and right_l0, kept
// points compacted into out (<= cap, camera frame); *kept = their count
// (oracle_stereo.cpp oracle_stereo_points).  stats[1] = FAST corners.  Two
// host syncs (the corner count, the point count).
int viso_ctx::stereo_points_into(int cur, double* out, int cap, int* kept) {
    const PyrGeom& g = geom;
    // FAST into scratch (kp1b, count slot 2): the monocular init state (kp1 =
    // the reference frame's keypoints, n_track_dev[0]) must survive a stereo
    // init that finds too few points, as the oracle's local xs/ys do
    float2* corners = (float2*)kp1b.ptr;
    int* d_nfast = (int*)n_track_dev.ptr + 2;
    {
        TimedRegion t(timing, VISO_KERNEL_FAST, stream);
        launch_fast(frame(cur).l[0], g.w[0], g.h[0], p.fast_thresh, fast, corners, nullptr,
                    p.max_features, d_nfast, stream);
    }
    VISO_HIP_CHECK(hipGetLastError());
    VISO_HIP_CHECK(hipMemcpyAsync(h_int, d_nfast, sizeof(int), hipMemcpyDeviceToHost, stream));
    VISO_HIP_CHECK(hipStreamSynchronize(stream));
    const int n = std::min(h_int[0], p.max_features);
    stats[1] = n;
    int rc = st_flag.ensure((size_t)std::max(n, 1) * 4);
    if (!rc) rc = st_pts.ensure((size_t)std::max(n, 1) * 24);
    if (rc) return rc;
    const StereoCam cam{p.fx, p.fy, p.cx, p.cy, stereo_base};
    int* d_count = (int*)n_track_dev.ptr + 1;
    {
        TimedRegion t(timing, VISO_KERNEL_STEREO, stream);
        launch_stereo_points(frame(cur).l[0], right_l0, g.w[0], g.h[0], corners, n, stereo_max_disp,
                             stereo_min_disp, cam, (int*)st_flag.ptr, (double*)st_pts.ptr, out, cap, d_count,
                             stream);
    }
    VISO_HIP_CHECK(hipGetLastError());
    VISO_HIP_CHECK(hipMemcpyAsync(h_int + 2, d_count, sizeof(int), hipMemcpyDeviceToHost, stream));
    VISO_HIP_CHECK(hipStreamSynchronize(stream));
    *kept = std::min(h_int[2], cap);
    return VISO_OK;
}

// Photometric BA over every keyframe and the map (ba.hip; oracle_viso.cpp's
// insertion branch): keyframe poses and points refined in place on the
// context stream; the refined poses go back to the keyframes' frames (the
// current frame's is the next frame's `last` pose and seed).
int viso_ctx::bundle_adjust() {
    const int nk = (int)kf_slots.size();
    if (nk < 2 || n_map < 1) return VISO_OK;
    int rc = point_host_dev.ensure(4 * (size_t)kMaxMapPoints);
    if (!rc) rc = ba_scratch.ensure(ba_scratch_bytes(kMaxMapPoints));
    if (rc) return rc;
    VISO_HIP_CHECK(hipMemcpyAsync(point_host_dev.ptr, point_host.data(), 4 * (size_t)n_map, hipMemcpyHostToDevice,
                                  stream));
    const uint8_t* l0[kMaxKeyframes];
    for (int k = 0; k < nk; ++k) l0[k] = frame(kf_slots[(size_t)k]).l[0];
    const double K[4] = {p.fx, p.fy, p.cx, p.cy};
    if (launch_photometric_ba(l0, nk, geom.w[0], geom.h[0], K, (double*)kf_poses.ptr, (double*)map_pts.ptr,
                              (const int*)point_host_dev.ptr, n_map, ba_iterations, ba_scratch.ptr, nullptr,
                              stream))
        return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipGetLastError());
    for (int k = 1; k < nk; ++k)
        VISO_HIP_CHECK(hipMemcpyAsync(pose_of(kf_slots[(size_t)k]), (char*)kf_poses.ptr + 96 * k, 96,
                                      hipMemcpyDeviceToDevice, stream));
    // the host array must outlive the async upload
    VISO_HIP_CHECK(hipStreamSynchronize(stream));
    return VISO_OK;
}

// Stereo keyframe insertion (oracle_viso.cpp, the kRunning case): the frame's
// pose is final (resolve_direct) and every earlier tracking frame's LK
// alignment has been launched against the old map (flush_lk); then its
// stereo points are appended in world coordinates, it becomes a keyframe
// and the map's LK templates are rebuilt.
int viso_ctx::insert_keyframe(int cur) {
    const int cap = kMaxMapPoints - n_map;
    int m = 0;
    const double saved1 = stats[1];
    int rc = stereo_points_into(cur, (double*)map_pts.ptr + 3 * (size_t)n_map, cap, &m);
    stats[1] = saved1;
    if (rc) return rc;
    launch_points_to_world((double*)map_pts.ptr + 3 * (size_t)n_map, m, pose_of(cur), stream);
    VISO_HIP_CHECK(hipGetLastError());
    n_map += m;
    rc = own_level0(cur);
    if (rc) return rc;
    kf_slots.push_back(cur);
    hold(cur);
    VISO_HIP_CHECK(hipMemcpyAsync((char*)kf_poses.ptr + 96 * (kf_slots.size() - 1), pose_of(cur), 96,
                                  hipMemcpyDeviceToDevice, stream));
    point_host.resize((size_t)n_map, (int32_t)kf_slots.size() - 1);
    if (ba_iterations > 0) {
        rc = bundle_adjust();
        if (rc) return rc;
    }
    rc = build_lk_templates();
    if (rc) return rc;
    stats[14] = m;
    return VISO_OK;
}

// Stereo initialisation (the repo's own spec, oracle/oracle_stereo.cpp
// oracle_stereo_points + oracle_viso.cpp stereo_init): FAST on the left
// image, sub-pixel SAD disparity on the right one, metric camera points; with
// more than 50 of them the map is created at once: the frame is the only
// keyframe (R = I, T = 0), points in its camera frame, metric scale.
int viso_ctx::stereo_init(int cur, bool* made) {
    *made = false;
    int m = 0;
    int rc = stereo_points_into(cur, (double*)map_pts.ptr, kMaxMapPoints, &m);
    if (rc) return rc;
    stats[2] = m;
    if (m <= 50) return VISO_OK;
    for (int s : kf_slots) drop(s);
    kf_slots.clear();
    kf_slots.push_back(cur);
    hold(cur);
    n_map = std::min(m, kMaxMapPoints);
    point_host.assign((size_t)n_map, 0);
    VISO_HIP_CHECK(hipMemcpyAsync(kf_poses.ptr, pose_of(cur), 96, hipMemcpyDeviceToDevice, stream));
    rc = build_lk_templates();
    if (rc) return rc;
    state = p.enable_tracking ? VISO_STATE_RUNNING : VISO_STATE_FINISHED;
    stats[3] = -2;  // stereo initialisation
    stats[12] = 1;
    *made = true;
    return VISO_OK;
}

// ------------------------------------------------------------------ OnNewFrame
int viso_ctx::on_new_frame(int cur) {
    RoctxRange range("viso:frame");
    const PyrGeom& g = geom;
    hold(cur);  // the "cur_frame" shared_ptr, released on every return
    struct CurRef {
        viso_ctx* c;
        int s;
        ~CurRef() { c->drop(s); }
    } cur_ref{this, cur};
    for (int k = 0; k < 16; ++k) stats[k] = 0;
    // Keyframe ctor: R = I, T = 0 (a tracking frame overwrites it below)
    // (written by the ingest's pyramid launch for its last frame, PyrOwn)
    if (state != VISO_STATE_RUNNING && cur != ident_slot) launch_set_pose(pose_of(cur), kIdentityPose, stream);
    if (cur == ident_slot) ident_slot = -1;
    const double K[4] = {p.fx, p.fy, p.cx, p.cy};
    bool counted = true;  // ++init_.frame_cnt at the end of kInitialization
    switch (state) {
        case VISO_STATE_INITIALIZATION: {
            if (stereo_base > 0 && right_l0) {
                bool made = false;
                const int rc = stereo_init(cur, &made);
                if (rc) return rc;
                if (made) break;  // no ++frame_cnt, as after the mono map creation
            }
            if (frame_cnt > 0 && frame_cnt <= p.reinitialize_after) {
                stats[3] = -1;
                // n_track < 0: the re-detection frame before this one left its
                // count on the device only; the KLT and the compaction read it
                // there (capped at max_features) — unless its copy has landed
                // already (a caller that synchronised in between): then the
                // exact count, without waiting
                if (ntrack_pending) {
                    const hipError_t q = hipEventQuery(ntrack_evt);
                    if (q == hipSuccess) {
                        n_track = std::min(h_int[3], p.max_features);
                        if (stats[1] == -1) stats[1] = n_track;
                        ntrack_pending = false;
                    } else if (q == hipErrorNotReady) {
                        (void)hipGetLastError();  // (only the query's own status)
                    } else {
                        return VISO_ERR_HIP;
                    }
                }
                const int n = n_track;
                if (n != 0) {
                    TimedRegion t(timing, VISO_KERNEL_KLT, stream);
                    if (n > 0)
                        launch_klt(frame(ref_slot), frame(cur), g, (const float2*)kp1.ptr,
                                   (float2*)kp2.ptr, (uint8_t*)track_success.ptr, n,
                                   p.photometric_error_thresh, stream);
                    else
                        launch_klt_dev(frame(ref_slot), frame(cur), g, (const float2*)kp1.ptr,
                                       (float2*)kp2.ptr, (uint8_t*)track_success.ptr, (const int*)n_track_dev.ptr,
                                       p.max_features, p.photometric_error_thresh, stream);
                }
                // erase failed tracks (src/viso.cpp:23-40) into the other
                // track buffers, which become kp1 / kp2 — in the gate's launch
                CompactIn ci;
                ci.in1 = (const float2*)kp1.ptr;
                ci.in2 = (const float2*)kp2.ptr;
                ci.success = (const uint8_t*)track_success.ptr;
                ci.n = n >= 0 ? n : -p.max_features;
                ci.out1 = (float2*)kp1b.ptr;
                ci.out2 = (float2*)kp2b.ptr;
                ci.n_out = (int*)n_track_dev.ptr;
                ntrack_pending = false;
                std::swap(kp1, kp1b);
                std::swap(kp2, kp2b);
                success_valid = false;
                geo.kp1 = (const float2*)kp1.ptr;
                geo.kp2 = (const float2*)kp2.ptr;
                geo.p1_in = geo.p2_in = nullptr;
                // the gates of PoseEstimation2d2d (src/viso.cpp:184, 216) are read
                // first: most initialisation frames stop there (too little
                // disparity yet), and then none of the ~17 RANSAC / motion
                // kernels is launched; a frame past the gates pays one more
                // host round trip
                {
                    TimedRegion t(timing, VISO_KERNEL_RANSAC, stream);
                    launch_compact_gate(ci, geo, stream);
                }
                VISO_HIP_CHECK(hipGetLastError());
                // the gate mirrors the control block into h_ctl itself.  When
                // it is likely open, the H hypotheses go behind it before it
                // is read (a closed gate returns them at once), so the host's
                // round trip overlaps them: likely = the last frame's gate
                // was open, or its disparity extrapolated to this frame (it
                // grows about with the square of the frames since the
                // reference one) comes within 25 % of the threshold.  A wrong
                // guess costs time only (a no-op launch, or the round trip)
                // (VISO_GATE_SPEC=0 / 1: never / always, for the tests of
                // the three paths)
                const int k = frame_cnt;
                const bool spec = gate_spec_mode >= 0
                                      ? gate_spec_mode == 1
                                      : gate_cnt > 0 && gate_cnt == k - 1 &&
                                            (gate_open || gate_disp * ((double)k * k) / ((double)(k - 1) * (k - 1)) *
                                                                  1.25 >=
                                                              p.disparity_squared_thresh);
                if (spec) {
                    VISO_HIP_CHECK(hipEventRecord(gate_evt, stream));
                    {
                        TimedRegion t(timing, VISO_KERNEL_RANSAC, stream);
                        launch_pose_2d2d_spec(geo, stream);
                    }
                    VISO_HIP_CHECK(hipGetLastError());
                    VISO_HIP_CHECK(hipEventSynchronize(gate_evt));
                } else {
                    VISO_HIP_CHECK(hipStreamSynchronize(stream));
                }
                gate_cnt = k;
                gate_open = h_ctl->gate != 0;
                gate_disp = h_ctl->disparity;
                if (h_ctl->gate) {
                    hipStream_t bs = stream;
                    {
                        TimedRegion t(timing, VISO_KERNEL_RANSAC, stream);
                        // the E and H chains on the two streams (lk_stream is
                        // idle: nothing of this frame was enqueued there), the
                        // H chain behind its speculative launch; the result is
                        // read on the stream SelectMotion ran on
                        bs = launch_pose_2d2d_body(geo, stream, lk_stream, geo_fork, geo_join, spec);
                    }
                    VISO_HIP_CHECK(hipGetLastError());
                    // (SelectMotion's last launch mirrors the block into h_ctl)
                    VISO_HIP_CHECK(hipStreamSynchronize(bs));
                }
                const GeoCtl& c = *h_ctl;
                n_track = c.n;
                int nr_inliers = 0;
                if (c.gate) {
                    nr_inliers = c.nr_inliers;
                    if (c.best_motion >= 0) {
                        std::memcpy(initR, c.R, sizeof(initR));
                        std::memcpy(initT, c.T, sizeof(initT));
                        success_valid = true;  // init_.success = best_inliers
                    }
                    stats[3] = c.best_motion;
                    stats[4] = c.n_cand;
                }
                stats[1] = n_track;
                stats[2] = nr_inliers;
                stats[8] = c.disparity;
                const double thresh = 0.9;
                if (n_track > 50 && nr_inliers > 0 && (nr_inliers / (double)n_track) > thresh) {
                    // map creation (src/viso.cpp:79-96)
                    for (int s : kf_slots) drop(s);
                    kf_slots.clear();
                    kf_slots.push_back(ref_slot);
                    kf_slots.push_back(cur);
                    hold(ref_slot);
                    hold(cur);
                    double pose[12];
                    std::memcpy(pose, initR, sizeof(initR));
                    std::memcpy(pose + 9, initT, sizeof(initT));
                    n_map = std::min(nr_inliers, kMaxMapPoints);
                    point_host.assign((size_t)n_map, 0);  // in keyframe 0's (ref) frame
                    // the frame's pose, the map points and the two keyframe
                    // poses in one launch (round 4: a kernel and three copies)
                    launch_map_create(pose_of(cur), pose, geo.points_out, (double*)map_pts.ptr, n_map,
                                      pose_of(ref_slot), (double*)kf_poses.ptr, stream);
                    VISO_HIP_CHECK(hipGetLastError());
                    // LK-alignment templates of the new map (constant while tracking)
                    {
                        const int rc = build_lk_templates();
                        if (rc) return rc;
                    }
                    state = p.enable_tracking ? VISO_STATE_RUNNING : VISO_STATE_FINISHED;
                    stats[12] = 1;
                    counted = false;  // `break` skips ++frame_cnt (src/viso.cpp:98)
                }
            } else {
                // re-detect (src/viso.cpp:100-108)
                // no host round trip: the FAST launch caps the count and
                // writes kp2 = kp1 on the device, the next frame's KLT reads
                // the count there, and the host learns it lazily from the
                // copy the same launch stores into h_int[3] (resolve_ntrack:
                // a getter, or the next frame once ntrack_evt has passed)
                {
                    TimedRegion t(timing, VISO_KERNEL_FAST, stream);
                    const FastDetect det{(float2*)kp2.ptr, h_int_dev + 3};
                    // (tiles already run by the ingest's level-1 launch: FastPre)
                    const bool pre = fast_pre.done && fast_pre_slot == cur;
                    launch_fast(frame(cur).l[0], g.w[0], g.h[0], p.fast_thresh, fast,
                                (float2*)kp1.ptr, nullptr, p.max_features, (int*)n_track_dev.ptr,
                                stream, &det, pre);
                    fast_pre = FastPre{};
                    fast_pre_slot = -1;
                }
                VISO_HIP_CHECK(hipGetLastError());
                VISO_HIP_CHECK(hipEventRecord(ntrack_evt, stream));
                n_track = -1;
                ntrack_pending = true;
                gate_cnt = 0;
                success_valid = false;
                set_role(ref_slot, cur);
                frame_cnt = 0;
                stats[1] = -1;  // resolve_ntrack fills it in
            }
            if (counted) ++frame_cnt;
            break;
        }
        case VISO_STATE_RUNNING: {
            // Sophus::SE3d X(last_frame->GetR(), last_frame->GetT()) (src/viso.cpp:114) is
            // seeded inside level 3; level 0 writes cur_frame->SetR/SetT(X) and
            // poses.push_back(X) (src/viso.cpp:117-118, 137)
            // (the previous tracking frame's final solve, if pending, runs
            // fused into this frame's level 3: its pose is this frame's
            // last_frame pose)
            const bool log = n_poses < p.max_poses;
            {
                TimedRegion t(timing, VISO_KERNEL_DIRECT, stream);
                DirectPrev m{};
                if (dpend) {
                    m.last = frame(dpend_last);
                    m.cur = frame(dpend_cur);
                    m.pose_last12 = pose_of(dpend_last);
                    m.pose_out = pose_of(dpend_cur);
                    m.log = dpend_log >= 0 ? (double*)pose_log.ptr : nullptr;
                    m.log_index = dpend_log;
                    m.ready = bg_ready(dpend_bg);
                    m.log_host = log_host(dpend_log);
                    m.flog = flog();
                }
                dev_tl.mark(frames, 3, stream);
                launch_direct_levels(frame(last_slot), frame(cur), g, K, (const double*)map_pts.ptr,
                                     n_map, pose_of(last_slot), pose_of(last_slot), direct,
                                     (double*)direct_stats.ptr, dpend ? &m : nullptr, stream, p.precision,
                                     bg_active);
                dev_tl.mark(frames, 4, stream);
            }
            if (dpend) {
                drop(dpend_cur);
                drop(dpend_last);
            }
            dpend = true;
            dpend_cur = cur;
            dpend_last = last_slot;
            hold(cur);
            hold(last_slot);
            dpend_log = log ? n_poses : -1;
            slots[(size_t)cur].log_index = dpend_log;
            dpend_bg = bg_active ? bg_cur : -1;
            if (log) ++n_poses;
            // LKAlignment (src/viso.cpp:121, 768-843): run by the chunk's
            // background kernel, or queued for the batched launch at the end
            // of this ingest call
            hold(cur);
            if (bg_active) {
                bg_slots.push_back(cur);
            } else {
                lk_pending.push_back(cur);
                if ((int)lk_pending.size() == kLkBatch) {
                    int rc = finish_call(stream);
                    if (rc) return rc;
                }
            }
            ran_tracking = true;
            // stereo keyframe insertion (oracle_viso.cpp): every
            // kf_interval-th tracking frame, one host sync for its nGood
            ++track_cnt;
            stats[15] = (double)kf_slots.size();  // before a possible insertion, as the oracle
            if (kf_interval > 0 && right_l0 && stereo_base > 0 && track_cnt % kf_interval == 0 &&
                (int)kf_slots.size() < kMaxKeyframes) {
                int rc = finish_call(stream);
                if (rc) return rc;
                VISO_HIP_CHECK(hipMemcpyAsync(h_dbl, direct_stats.ptr, sizeof(double), hipMemcpyDeviceToHost,
                                              stream));
                VISO_HIP_CHECK(hipStreamSynchronize(stream));
                if (h_dbl[0] < kf_permille * (double)n_map / 1000.0) {
                    rc = insert_keyframe(cur);
                    if (rc) return rc;
                    stats[15] = (double)kf_slots.size();
                }
            }
            break;
        }
        default:
            break;
    }
    VISO_HIP_CHECK(hipGetLastError());
    set_role(last_slot, cur);  // last_frame = cur_frame (src/viso.cpp:144)
    ++frames;
    stats[0] = state;
    stats[5] = frame_cnt;
    stats[11] = (double)frames;
    stats[13] = success_valid ? 1 : 0;
    return VISO_OK;
}

// One ingest chunk (the frames' slots, held by the caller's hold; their level
// 0 at l0[i] — borrowed from the caller's device buffer, or already in the
// slot; right[i] the right image or null): the chunk's pyramids in one
// batched launch, the background LK grid when eligible, OnNewFrame per frame,
// then the chunk's end.  Releases the chunk's holds, also on an error.
int viso_ctx::ingest_chunk(const std::vector<int>& sl, const std::vector<const uint8_t*>& l0,
                           const std::vector<const uint8_t*>& right, bool overlap_tail) {
    const int nb = (int)sl.size();
    std::vector<uint8_t*> dst;
    for (int s : sl) dst.push_back(slot_base(s));
    // a background-LK chunk's words are cleared by the pyramid's tail
    // launch (bg_begin then makes no memset launch)
    const bool bg = bg_eligible() && nb <= kLkBatch;
    // a one-frame chunk whose frame starts with FAST (the monocular
    // initialisation's detection frame, src/viso.cpp:100-108: no reference
    // keypoints to track yet) runs the FAST tiles in the pyramid's level-1
    // launch (FastPre); on_new_frame then only orders them
    fast_pre = FastPre{};
    fast_pre_slot = -1;
    if (nb == 1 && state == VISO_STATE_INITIALIZATION && !(stereo_base > 0 && !right.empty() && right[0]) &&
        !(frame_cnt > 0 && frame_cnt <= p.reinitialize_after)) {
        fast_pre.img = l0[0];
        fast_pre.w = geom.w[0];
        fast_pre.h = geom.h[0];
        fast_pre.thresh = p.fast_thresh;
        fast_pre.s = fast;
        fast_pre_slot = sl[0];
    }
    launch_ingest_pyramid(l0.data(), dst.data(), sl.data(), nb, bg);
    if (hipGetLastError() != hipSuccess) {
        for (int s : sl) drop(s);
        return VISO_ERR_HIP;
    }
    // (the background words' memset stays behind the pyramid: issued
    // ahead of it, the chain ran at half speed in 3 of 6 bench runs,
    // profiles/r05_bg_order_ab.log)
    if (const int rc = bg_begin(sl, bg)) {
        for (int s : sl) drop(s);
        return rc;
    }
    // end of the chunk, also on an error: launch what still reads the
    // chunk's borrowed frames (the pending final solve, the LK batch),
    // give retained frames their own level 0, release the chunk's holds
    auto end_chunk = [&](int rc) -> int {
        fast_pre = FastPre{};  // (consumed by its frame's FAST, or unused)
        fast_pre_slot = -1;
        const int r1 = finish_call(stream, overlap_tail && !rc);
        if (!rc) rc = r1;
        const int roles[2] = {ref_slot, last_slot};
        for (int r : roles) {
            const int r2 = own_level0(r);
            if (!rc) rc = r2;
        }
        for (int s : kf_slots) {
            const int r2 = own_level0(s);
            if (!rc) rc = r2;
        }
        for (int s : sl) drop(s);
        return rc;
    };
    for (int i = 0; i < nb; ++i) {
        right_l0 = right.empty() ? nullptr : right[(size_t)i];
        bg_cur = i;
        const int rc = on_new_frame(sl[(size_t)i]);
        right_l0 = nullptr;
        if (rc) return end_chunk(rc);
        if (i == 0) {
            const int r2 = bg_launch();
            if (r2) return end_chunk(r2);
        }
    }
    // the last frame's final solve, then the chunk's LKAlignment batch
    // behind the chunk (the GPU is free then; beside the next chunk it
    // would take the CU resources the latency-bound direct chain needs)
    return end_chunk(VISO_OK);
}

// ------------------------------------------------------------------ C ABI
extern "C" {

int viso_process_frame(viso_ctx* c, const uint8_t* grey, int32_t width, int32_t height,
                       int32_t stride) {
    if (!c) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(c->device));
    HostTimes::Clock ht(c->host_times);
    if (c->host_queue_eligible()) {
        // tracking: queue the frame (its DMA), run queued frames as chunks
        int rc = c->queue_host_frame(grey, width, height, stride);
        ht.lap(0);
        const int re = c->end_epoch();
        return rc ? rc : re;
    }
    if (int rc = c->flush_host_q()) return rc;  // (frames queued before: in order)
    int s = -1;
    // upload and pyramid on the upload stream (ingest_host)
    int rc = c->ingest_host(grey, width, height, stride, &s, true);
    ht.lap(0);
    if (rc) return rc;
    rc = c->on_new_frame(s);
    ht.lap(1);
    if (rc) return rc;
    rc = c->finish_host_call();
    const int re = c->end_epoch();
    ht.lap(2);
    return rc ? rc : re;
}

int viso_process_stereo(viso_ctx* c, const uint8_t* left, const uint8_t* right,
                        const int32_t dims[3]) {
    if (!c || !left || !right || !dims) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(c->device));
    if (int rc = c->flush_host_q()) return rc;  // (frames queued before: in order)
    int sl = -1, sr = -1;
    int rc = c->ingest_host(left, dims[0], dims[1], dims[2], &sl, true);
    if (rc) return rc;
    rc = c->ingest_host(right, dims[0], dims[1], dims[2], &sr, false);
    if (rc) {
        c->hold(sl);
        c->drop(sl);
        return rc;
    }
    // the right image feeds the stereo initialisation (viso_set_stereo), which
    // reads its level 0 only: no pyramid is built for it; the reference path
    // runs on the left image only
    c->hold(sr);
    c->right_l0 = c->slot_base(sr);
    rc = c->on_new_frame(sl);
    c->right_l0 = nullptr;
    c->drop(sr);
    if (rc) return rc;
    rc = c->finish_host_call();
    const int re = c->end_epoch();
    return rc ? rc : re;
}

int viso_process_frames_device(viso_ctx* c, const uint8_t* d_left, const uint8_t* d_right,
                               int32_t n, size_t frame_stride) {
    if (!c || !d_left || n < 0) return VISO_ERR_ARG;
    if (int rc = c->settle()) return rc;  // (host-frame work left pending)
    if (frame_stride < (size_t)c->geom.w[0] * c->geom.h[0]) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(c->device));
    const int B = c->p.batch_frames;
    for (int f0 = 0, nb = 0; f0 < n; f0 += nb) {
        RoctxRange range("viso:ingest_chunk");
        // a tracking context's chunks run LK alignment in the background,
        // which covers at most kLkBatch frames: chunks are cut to that
        nb = std::min(c->bg_eligible() ? std::min(B, kLkBatch) : B, n - f0);
        std::vector<int> sl;
        std::vector<const uint8_t*> l0, right;
        // left images only: the right image is read at level 0, in place, by
        // the stereo initialisation (no stage consumes a right pyramid)
        for (int i = 0; i < nb; ++i) {
            const int s = c->acquire_slot();
            if (s < 0) {
                for (int x : sl) c->drop(x);
                return VISO_ERR_CAPACITY;
            }
            const int f = f0 + i;
            const uint8_t* src = d_left + frame_stride * (size_t)f;
            c->slots[(size_t)s].l0 = src;
            c->slots[(size_t)s].borrowed = true;
            c->hold(s);  // pending in this chunk
            sl.push_back(s);
            l0.push_back(src);
            right.push_back(d_right ? d_right + frame_stride * (size_t)f : nullptr);
        }
        if (int rc = c->ingest_chunk(sl, l0, right, f0 + nb < n && c->tail_overlap_on())) return rc;
    }
    return c->end_epoch();
}

int viso_get_state(viso_ctx* c, int32_t* state) {
    if (!c || !state) return VISO_ERR_ARG;
    *state = c->state;
    return VISO_OK;
}

int viso_get_poses(viso_ctx* c, double* Tcw12, size_t cap, size_t* n) {
    if (!c) return VISO_ERR_ARG;
    if (int rc = c->settle()) return rc;  // (host-frame work left pending)
    // the count is host state (one pose per launched tracking frame): asking
    // for it alone needs no device round trip
    if (n) *n = (size_t)c->n_poses;
    // (the log keeps the first max_poses poses)
    const size_t m = std::min(std::min(cap, (size_t)c->n_poses), (size_t)std::max(c->p.max_poses, 0));
    if (m == 0 || !Tcw12) return VISO_OK;
    VISO_HIP_CHECK(hipSetDevice(c->device));
    // through a pinned staging buffer: one DMA and one stream sync (a
    // pageable destination is copied through the runtime's own staging)
    if (c->poses_staged >= m) {
        // staged behind the calls that produced them (stage_poses): the
        // stream's sync makes the copy visible
        VISO_HIP_CHECK(hipStreamSynchronize(c->stream));
        std::memcpy(Tcw12, c->h_poses, 96 * m);
        return VISO_OK;
    }
    if (c->h_poses_cap < m) {
        // geometric growth (up to max_poses): the kernels then mirror the
        // poses logged after this call into the new buffer (log_host), and
        // stage_poses keeps the staged path, instead of a reallocation and
        // full copy on every later read
        const size_t cap_max = (size_t)std::max(c->p.max_poses, 1);
        const size_t want = std::min(cap_max, std::max(m, std::max((size_t)4096, 2 * c->h_poses_cap)));
        VISO_HIP_CHECK(hipStreamSynchronize(c->stream));  // no staged copy in flight into the old buffer
        if (c->h_poses) VISO_HIP_CHECK(hipHostFree(c->h_poses));
        c->h_poses = nullptr;
        c->h_poses_dev = nullptr;
        c->h_poses_cap = 0;
        c->poses_staged = 0;
        VISO_HIP_CHECK(hipHostMalloc((void**)&c->h_poses, 96 * want));
        VISO_HIP_CHECK(hipHostGetDevicePointer((void**)&c->h_poses_dev, c->h_poses, 0));
        c->h_poses_cap = want;
    }
    VISO_HIP_CHECK(hipMemcpyAsync(c->h_poses, c->pose_log.ptr, 96 * m, hipMemcpyDeviceToHost, c->stream));
    VISO_HIP_CHECK(hipStreamSynchronize(c->stream));
    c->poses_staged = std::max(c->poses_staged, m);
    std::memcpy(Tcw12, c->h_poses, 96 * m);
    return VISO_OK;
}

int viso_get_points(viso_ctx* c, double* xyz, size_t cap, size_t* n) {
    if (!c) return VISO_ERR_ARG;
    if (int rc = c->settle()) return rc;  // (host-frame work left pending)
    VISO_HIP_CHECK(hipSetDevice(c->device));
    const size_t m = std::min(cap, (size_t)c->n_map);
    if (m > 0 && xyz)
        VISO_HIP_CHECK(hipMemcpyAsync(xyz, c->map_pts.ptr, 24 * m, hipMemcpyDeviceToHost, c->stream));
    VISO_HIP_CHECK(hipStreamSynchronize(c->stream));
    if (n) *n = (size_t)c->n_map;
    return VISO_OK;
}

// A re-detection frame's corner count, read lazily (on_new_frame leaves it
// on the device and copies it to pinned h_int[3] behind the frame).
int viso_ctx::resolve_ntrack() {
    if (!ntrack_pending) return VISO_OK;
    VISO_HIP_CHECK(hipStreamSynchronize(stream));
    n_track = std::min(h_int[3], p.max_features);
    if (stats[1] == -1) stats[1] = n_track;
    ntrack_pending = false;
    return VISO_OK;
}

int viso_get_init_tracks(viso_ctx* c, float* kp1, float* kp2, uint8_t* success, size_t cap,
                         size_t* n) {
    if (!c) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(c->device));
    if (int rc = c->resolve_ntrack()) return rc;
    const size_t m = std::min(cap, (size_t)c->n_track);
    if (m > 0) {
        if (kp1) VISO_HIP_CHECK(hipMemcpyAsync(kp1, c->kp1.ptr, 8 * m, hipMemcpyDeviceToHost, c->stream));
        if (kp2) VISO_HIP_CHECK(hipMemcpyAsync(kp2, c->kp2.ptr, 8 * m, hipMemcpyDeviceToHost, c->stream));
        if (success) {
            if (c->success_valid)
                VISO_HIP_CHECK(hipMemcpyAsync(success, c->geo.inliers, m, hipMemcpyDeviceToHost, c->stream));
            else
                std::memset(success, 0, m);
        }
    }
    VISO_HIP_CHECK(hipStreamSynchronize(c->stream));
    if (n) *n = (size_t)c->n_track;
    return VISO_OK;
}

int viso_get_alignment(viso_ctx* c, int32_t* pair_kf, uint8_t* success, double* uv_before,
                       double* uv_after, size_t cap, size_t* n) {
    if (!c) return VISO_ERR_ARG;
    if (int rc = c->settle()) return rc;  // (host-frame work left pending)
    VISO_HIP_CHECK(hipSetDevice(c->device));
    VISO_HIP_CHECK(hipStreamSynchronize(c->lk_stream));
    if (int rc = c->bg_check()) return rc;
    const size_t m = c->ran_tracking ? std::min(cap, (size_t)c->lk_last_pts) : 0;
    const size_t o = (size_t)std::max(c->lk_last_rows - 1, 0) * kMaxMapPoints;
    if (m > 0) {
        if (pair_kf) VISO_HIP_CHECK(hipMemcpyAsync(pair_kf, (int32_t*)c->lk_pair.ptr + o, 4 * m, hipMemcpyDeviceToHost, c->stream));
        if (success) VISO_HIP_CHECK(hipMemcpyAsync(success, (uint8_t*)c->lk_succ.ptr + o, m, hipMemcpyDeviceToHost, c->stream));
        if (uv_before) VISO_HIP_CHECK(hipMemcpyAsync(uv_before, (double*)c->lk_before.ptr + 2 * o, 16 * m, hipMemcpyDeviceToHost, c->stream));
        if (uv_after) VISO_HIP_CHECK(hipMemcpyAsync(uv_after, (double*)c->lk_after.ptr + 2 * o, 16 * m, hipMemcpyDeviceToHost, c->stream));
    }
    VISO_HIP_CHECK(hipStreamSynchronize(c->stream));
    if (n) *n = c->ran_tracking ? (size_t)c->lk_last_pts : 0;
    return VISO_OK;
}

int viso_get_frame_stats(viso_ctx* c, double out[16]) {
    if (!c || !out) return VISO_ERR_ARG;
    if (int rc = c->settle()) return rc;  // (host-frame work left pending)
    VISO_HIP_CHECK(hipSetDevice(c->device));
    if (int rc = c->resolve_ntrack()) return rc;
    std::memcpy(out, c->stats, sizeof(c->stats));
    if (c->state == VISO_STATE_RUNNING && c->stats[12] == 0 && c->ran_tracking) {
        // last frame was a tracking frame: level-0 direct stats + LK counts
        VISO_HIP_CHECK(hipStreamSynchronize(c->lk_stream));
        if (int rc = c->bg_check()) return rc;
        const int m = c->lk_last_pts;
        const size_t o = (size_t)std::max(c->lk_last_rows - 1, 0) * kMaxMapPoints;
        std::vector<int32_t> pk((size_t)m);
        std::vector<uint8_t> sc((size_t)m);
        if (m > 0) {
            VISO_HIP_CHECK(hipMemcpyAsync(pk.data(), (int32_t*)c->lk_pair.ptr + o, 4 * (size_t)m, hipMemcpyDeviceToHost, c->stream));
            VISO_HIP_CHECK(hipMemcpyAsync(sc.data(), (uint8_t*)c->lk_succ.ptr + o, (size_t)m, hipMemcpyDeviceToHost, c->stream));
        }
        VISO_HIP_CHECK(hipMemcpyAsync(c->h_dbl, c->direct_stats.ptr, 2 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
        VISO_HIP_CHECK(hipStreamSynchronize(c->stream));
        int pairs = 0, succ = 0;
        for (int i = 0; i < m; ++i) {
            pairs += pk[(size_t)i] >= 0;
            succ += sc[(size_t)i];
        }
        out[6] = pairs;
        out[7] = succ;
        out[9] = c->h_dbl[0];
        out[10] = c->h_dbl[1];
    }
    return VISO_OK;
}

int viso_get_config(viso_ctx* c, int32_t info[8]) {
    if (!c || !info) return VISO_ERR_ARG;
    for (int k = 0; k < 8; ++k) info[k] = 0;
    info[0] = c->bg_on() && direct_fits_background() ? 1 : 0;
    info[1] = c->lk_dedicated ? 1 : 0;
    info[2] = c->up_stream ? (c->up_dedicated ? 1 : 0) : -1;
    info[3] = c->n_slots;
    info[4] = c->flog() ? 1 : 0;
    info[5] = c->p.batch_frames;
    info[6] = c->tail_copy_bytes;
    info[7] = c->tail_zero_ints;
    return VISO_OK;
}

int viso_set_frame_log(viso_ctx* c, int32_t enable) {
    if (!c) return VISO_ERR_ARG;
    if (int rc = c->settle()) return rc;  // (host-frame work left pending)
    VISO_HIP_CHECK(hipSetDevice(c->device));
    if (!enable) {
        VISO_HIP_CHECK(hipStreamSynchronize(c->stream));
        if (c->lk_stream) VISO_HIP_CHECK(hipStreamSynchronize(c->lk_stream));
        c->frame_log.release();
        return VISO_OK;
    }
    if (c->flog()) return VISO_OK;
    const size_t bytes = 32 * (size_t)std::max(c->p.max_poses, 1);
    if (int rc = c->frame_log.ensure(bytes)) return rc;
    // NaN until a frame's entry is written (frames logged before the log was on)
    VISO_HIP_CHECK(hipMemsetAsync(c->frame_log.ptr, 0xff, bytes, c->stream));
    return VISO_OK;
}

int viso_get_frame_log(viso_ctx* c, double* rows, size_t cap, size_t* n) {
    if (!c) return VISO_ERR_ARG;
    if (!c->flog()) return VISO_ERR_STATE;
    if (int rc = c->settle()) return rc;  // (host-frame work left pending)
    VISO_HIP_CHECK(hipSetDevice(c->device));
    const size_t total = std::min((size_t)c->n_poses, (size_t)std::max(c->p.max_poses, 0));
    if (n) *n = total;
    // the LK columns of a side-stream batch are written on lk_stream
    if (c->lk_stream) VISO_HIP_CHECK(hipStreamSynchronize(c->lk_stream));
    const size_t m = std::min(cap, total);
    if (m > 0 && rows)
        VISO_HIP_CHECK(hipMemcpyAsync(rows, c->frame_log.ptr, 32 * m, hipMemcpyDeviceToHost, c->stream));
    VISO_HIP_CHECK(hipStreamSynchronize(c->stream));
    return c->bg_check();
}

int viso_pose_2d2d(viso_ctx* c, const double* p1, const double* p2, int32_t n, double R[9],
                   double T[3], uint8_t* inliers, double* points3d, double* candidates,
                   double stats[8]) {
    if (!c || n < 0 || n > c->p.max_features || !R || !T || !stats) return VISO_ERR_ARG;
    if (int rc = c->settle()) return rc;  // (host-frame work left pending)
    if (n > 0 && (!p1 || !p2)) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(c->device));
    int rc = c->scratch_d.ensure(48 * (size_t)std::max(n, 1) + 512);
    if (rc) return rc;
    double* d_p1 = (double*)c->scratch_d.ptr;
    double* d_p2 = d_p1 + 3 * (size_t)std::max(n, 1);
    if (n > 0) {
        VISO_HIP_CHECK(hipMemcpyAsync(d_p1, p1, 24 * (size_t)n, hipMemcpyHostToDevice, c->stream));
        VISO_HIP_CHECK(hipMemcpyAsync(d_p2, p2, 24 * (size_t)n, hipMemcpyHostToDevice, c->stream));
    }
    c->h_int[2] = n;
    VISO_HIP_CHECK(hipMemcpyAsync(c->n_track_dev.ptr, &c->h_int[2], sizeof(int), hipMemcpyHostToDevice, c->stream));
    GeoArgs a = c->geo;
    a.p1_in = d_p1;
    a.p2_in = d_p2;
    {
        TimedRegion t(c->timing, VISO_KERNEL_RANSAC, c->stream);
        launch_pose_2d2d(a, c->stream, &c->timing);
    }
    VISO_HIP_CHECK(hipGetLastError());
    // (the gate and SelectMotion mirror the control block into h_ctl)
    VISO_HIP_CHECK(hipStreamSynchronize(c->stream));
    const GeoCtl& g = *c->h_ctl;
    for (int k = 0; k < 8; ++k) stats[k] = 0;
    stats[3] = g.disparity;
    if (!g.gate) {
        // early return (src/viso.cpp:184, 216): R, T, inliers untouched; the
        // disparity gate's value is still reported when it was computed
        if (n < 10) stats[3] = 0;
        return VISO_OK;
    }
    stats[0] = g.nr_inliers;
    stats[1] = g.best_motion;
    stats[2] = g.n_cand;
    stats[4] = g.e_count;
    stats[5] = g.h_count;
    stats[6] = g.e_iters;
    stats[7] = g.h_iters;
    if (g.best_motion >= 0) {
        std::memcpy(R, g.R, sizeof(g.R));
        std::memcpy(T, g.T, sizeof(g.T));
    }
    if (candidates)
        for (int m = 0; m < g.n_cand; ++m)  // the E path's slot 0, the H path's from slot 1
            std::memcpy(candidates + 12 * m, g.cand[m < g.e_ncand ? 0 : 1 + (m - g.e_ncand)], 96);
    if (n > 0 && (inliers || points3d)) {
        std::vector<uint8_t> in((size_t)n);
        VISO_HIP_CHECK(hipMemcpy(in.data(), a.inliers, (size_t)n, hipMemcpyDeviceToHost));
        if (inliers) std::memcpy(inliers, in.data(), (size_t)n);
        if (points3d) {
            std::vector<double> comp(3 * (size_t)std::max(g.nr_inliers, 1));
            if (g.nr_inliers > 0)
                VISO_HIP_CHECK(hipMemcpy(comp.data(), a.points_out, 24 * (size_t)g.nr_inliers,
                                         hipMemcpyDeviceToHost));
            int k = 0;
            for (int i = 0; i < n; ++i) {
                for (int j = 0; j < 3; ++j) points3d[3 * i + j] = in[(size_t)i] ? comp[(size_t)3 * k + j] : 0.0;
                k += in[(size_t)i] ? 1 : 0;
            }
        }
    }
    return VISO_OK;
}

}  // extern "C"
