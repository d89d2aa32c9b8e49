// viso_amd — the multi-camera photometric rig behind include/viso/viso_rig.h
// (spec: oracle/oracle_rig.cpp).  Host sequencing only:
// per timestep one pyramid launch for all cameras, then the rig direct pose
// (direct.hip launch_rig_direct: L(3..0) + F); the stereo initialisation
// (FAST + stereo points per camera) synchronises twice per camera, once.
#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/viso/viso_rig.h"
#include "context.hpp"

using namespace viso;

static_assert(VISO_RIG_MAX_CAMS == kMaxRigCams, "rig camera limit");

namespace {

// Tc = E T (oracle_rig_compose; the device's rig_compose)
void rig_compose_host(const double* E, const double* T, double* out) {
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j)
            out[3 * i + j] = (E[3 * i] * T[j] + E[3 * i + 1] * T[3 + j]) + E[3 * i + 2] * T[6 + j];
        out[9 + i] = ((E[3 * i] * T[9] + E[3 * i + 1] * T[10]) + E[3 * i + 2] * T[11]) + E[9 + i];
    }
}

// Ad(E) = [[Re, [te]x Re], [0, Re]] (oracle_rig_adjoint)
void rig_adjoint_host(const double* E, double* Ad) {
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

const double kIdentity12[12] = {1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0};

}  // namespace

struct viso_rig {
    viso_params p{};
    int device = 0;
    int n = 0;
    hipStream_t stream = nullptr;
    PyrGeom geom{};
    double E[kMaxRigCams][12] = {};
    DevBuf pyr;      // 2 x n pyramid slots (level 0 owned): buffer b, camera c at (b * n + c)
    int cur = 0;     // buffer of the current timestep
    DevBuf ext, ad;  // n x 12, n x 36
    DevBuf map;      // n x kMaxMapPoints x 3 (world)
    int n_pts[kMaxRigCams] = {};
    DevBuf scratch;  // n x rig_scratch_bytes()
    DevBuf state, rig_pose, cam_last, stats, log;
    int n_poses = 0;
    // stereo initialisation
    double base = 0.0;
    int max_disp = 128, min_disp = 1;
    FastScratch fast;
    DevBuf fast_rows, kp, st_flag, st_pts, counts;
    int* h_int = nullptr;
    DevBuf staging;  // host-image upload (viso_rig_process)
    int state_ = VISO_STATE_INITIALIZATION;
    // the last tracked timestep's final level-0 solve (F), deferred into the
    // next timestep's L(3) within one ingest call, else launched by flush()
    bool pending = false;
    RigCamDev pending_cams[kMaxRigCams];
    int pending_log = -1;

    uint8_t* slot(int b, int c) const { return (uint8_t*)pyr.ptr + geom.slot * (size_t)(b * n + c); }
    int init();
    void release();
    int stereo_init(const uint8_t* const* right_l0, bool* made);
    int step(const uint8_t* const* left_l0, const uint8_t* const* right_l0);
    int flush();
};

int viso_rig::flush() {
    if (!pending) return VISO_OK;
    pending = false;
    const double K[4] = {p.fx, p.fy, p.cx, p.cy};
    const int rc = launch_rig_direct(pending_cams, n, geom, K, (double*)state.ptr, (const double*)rig_pose.ptr,
                                     (double*)stats.ptr, (double*)rig_pose.ptr,
                                     pending_log >= 0 ? (double*)log.ptr : nullptr, pending_log,
                                     (double*)cam_last.ptr, stream, p.precision, 0, -1, /*levels=*/0,
                                     /*final_solve=*/1);
    if (rc) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipGetLastError());
    return VISO_OK;
}

int viso_rig::init() {
    const PyrGeom& g = geom;
    int rc = pyr.ensure(geom.slot * 2 * (size_t)n);
    if (!rc) rc = ext.ensure(96 * (size_t)n);
    if (!rc) rc = ad.ensure(288 * (size_t)n);
    if (!rc) rc = map.ensure(24 * (size_t)kMaxMapPoints * n);
    if (!rc) rc = scratch.ensure(rig_scratch_bytes() * (size_t)n);
    if (!rc) rc = state.ensure(8 * 8 * (kLevels + 1));
    if (!rc) rc = rig_pose.ensure(96);
    if (!rc) rc = cam_last.ensure(96 * (size_t)n);
    if (!rc) rc = stats.ensure(8 * 200);
    if (!rc) rc = log.ensure(96 * (size_t)std::max(p.max_poses, 1));
    if (!rc) rc = kp.ensure(sizeof(float2) * (size_t)p.max_features);
    if (!rc) rc = counts.ensure(256);
    if (!rc) rc = fast_rows.ensure(fast_scratch_bytes(g.w[0], g.h[0]));
    if (rc) return rc;
    fast = fast_scratch_at(fast_rows.ptr, g.w[0], g.h[0]);
    VISO_HIP_CHECK(hipHostMalloc((void**)&h_int, 64 * sizeof(int)));
    std::vector<double> Ad(36 * (size_t)n);
    for (int c = 0; c < n; ++c) rig_adjoint_host(E[c], &Ad[36 * (size_t)c]);
    VISO_HIP_CHECK(hipMemcpyAsync(ext.ptr, E, 96 * (size_t)n, hipMemcpyHostToDevice, stream));
    VISO_HIP_CHECK(hipMemcpyAsync(ad.ptr, Ad.data(), 288 * (size_t)n, hipMemcpyHostToDevice, stream));
    VISO_HIP_CHECK(hipMemsetAsync(stats.ptr, 0, 8 * 200, stream));
    VISO_HIP_CHECK(hipStreamSynchronize(stream));
    return VISO_OK;
}

void viso_rig::release() {
    if (stream) (void)hipStreamSynchronize(stream);
    DevBuf* bufs[] = {&pyr, &ext, &ad, &map, &scratch, &state, &rig_pose, &cam_last, &stats, &log,
                      &fast_rows, &kp, &st_flag, &st_pts, &counts, &staging};
    for (DevBuf* b : bufs) b->release();
    if (h_int) (void)hipHostFree(h_int);
    h_int = nullptr;
    if (stream) (void)hipStreamDestroy(stream);
    stream = nullptr;
}

// Every camera's stereo points of the current timestep into its map (world
// = rig frame at T = I); more than 50 in all start tracking.
int viso_rig::stereo_init(const uint8_t* const* right_l0, bool* made) {
    *made = false;
    const PyrGeom& g = geom;
    int total = 0;
    int m[kMaxRigCams] = {};
    for (int c = 0; c < n; ++c) {
        const uint8_t* left = slot(cur, c);
        int* d_nfast = (int*)counts.ptr;
        launch_fast(left, g.w[0], g.h[0], p.fast_thresh, fast, (float2*)kp.ptr, nullptr, p.max_features, d_nfast,
                    stream);
        VISO_HIP_CHECK(hipGetLastError());
        VISO_HIP_CHECK(hipMemcpyAsync(h_int, d_nfast, sizeof(int), hipMemcpyDeviceToHost, stream));
        VISO_HIP_CHECK(hipStreamSynchronize(stream));
        const int nf = std::min(h_int[0], p.max_features);
        int rc = st_flag.ensure((size_t)std::max(nf, 1) * 4);
        if (!rc) rc = st_pts.ensure((size_t)std::max(nf, 1) * 24);
        if (rc) return rc;
        const StereoCam cam{p.fx, p.fy, p.cx, p.cy, base};
        double* out = (double*)map.ptr + 3 * (size_t)kMaxMapPoints * c;
        int* d_count = (int*)counts.ptr + 1;
        launch_stereo_points(left, right_l0[c], g.w[0], g.h[0], (const float2*)kp.ptr, nf, max_disp, min_disp, cam,
                             (int*)st_flag.ptr, (double*)st_pts.ptr, out, kMaxMapPoints, d_count, stream);
        VISO_HIP_CHECK(hipGetLastError());
        VISO_HIP_CHECK(hipMemcpyAsync(h_int + 1, d_count, sizeof(int), hipMemcpyDeviceToHost, stream));
        VISO_HIP_CHECK(hipStreamSynchronize(stream));
        m[c] = std::min(h_int[1], kMaxMapPoints);
        // X = Re^T (X_c - te)
        launch_points_to_world(out, m[c], (const double*)ext.ptr + 12 * c, stream);
        VISO_HIP_CHECK(hipGetLastError());
        total += m[c];
    }
    if (total <= 50) return VISO_OK;
    for (int c = 0; c < n; ++c) n_pts[c] = m[c];
    std::vector<double> last(12 * (size_t)n);
    for (int c = 0; c < n; ++c) rig_compose_host(E[c], kIdentity12, &last[12 * (size_t)c]);
    VISO_HIP_CHECK(hipMemcpyAsync(cam_last.ptr, last.data(), 96 * (size_t)n, hipMemcpyHostToDevice, stream));
    VISO_HIP_CHECK(hipMemcpyAsync(rig_pose.ptr, kIdentity12, 96, hipMemcpyHostToDevice, stream));
    VISO_HIP_CHECK(hipStreamSynchronize(stream));  // the host arrays above
    *made = true;
    return VISO_OK;
}

int viso_rig::step(const uint8_t* const* left_l0, const uint8_t* const* right_l0) {
    RoctxRange range("rig:timestep");
    const PyrGeom& g = geom;
    const size_t npx = (size_t)g.w[0] * g.h[0];
    const uint8_t* l0[kMaxRigCams];
    uint8_t* dst[kMaxRigCams];
    for (int c = 0; c < n; ++c) {
        VISO_HIP_CHECK(hipMemcpyAsync(slot(cur, c), left_l0[c], npx, hipMemcpyDeviceToDevice, stream));
        l0[c] = left_l0[c];
        dst[c] = slot(cur, c);
    }
    launch_pyramid_frames(g, l0, dst, n, stream);
    VISO_HIP_CHECK(hipGetLastError());
    if (state_ == VISO_STATE_INITIALIZATION) {
        if (right_l0 && base > 0) {
            bool made = false;
            const int rc = stereo_init(right_l0, &made);
            if (rc) return rc;
            if (made) state_ = VISO_STATE_RUNNING;
        }
    } else {
        RigCamDev cams[kMaxRigCams];
        const double K[4] = {p.fx, p.fy, p.cx, p.cy};
        for (int c = 0; c < n; ++c) {
            RigCamDev& d = cams[c];
            d.last = frame_from_base(slot(1 - cur, c), g);
            d.cur = frame_from_base(slot(cur, c), g);
            d.points = (const double*)map.ptr + 3 * (size_t)kMaxMapPoints * c;
            d.n = n_pts[c];
            d.pose_last12 = (const double*)cam_last.ptr + 12 * c;
            for (int k = 0; k < 12; ++k) d.E[k] = E[c][k];
            d.Ad = (const double*)ad.ptr + 36 * c;
            d.scratch = (char*)scratch.ptr + rig_scratch_bytes() * (size_t)c;
        }
        const bool logged = n_poses < p.max_poses;
        // L(3..0); this timestep's F is deferred (merged into the next
        // timestep's L(3), or flushed at the end of the ingest call)
        const int rc = launch_rig_direct(cams, n, g, K, (double*)state.ptr, (const double*)rig_pose.ptr,
                                         (double*)stats.ptr, (double*)rig_pose.ptr, (double*)log.ptr, n_poses,
                                         (double*)cam_last.ptr, stream, p.precision, pending ? 1 : 0,
                                         pending ? pending_log : -1, /*levels=*/1, /*final_solve=*/0);
        if (rc) return VISO_ERR_ARG;
        VISO_HIP_CHECK(hipGetLastError());
        pending = true;
        for (int c = 0; c < n; ++c) pending_cams[c] = cams[c];
        pending_log = logged ? n_poses : -1;
        if (logged) ++n_poses;
    }
    cur = 1 - cur;
    return VISO_OK;
}

extern "C" {

int viso_rig_create(const viso_params* p, int32_t n_cams, const double* extrinsics, int device, viso_rig** out) {
    if (!p || !out || !extrinsics || n_cams < 1 || n_cams > kMaxRigCams) return VISO_ERR_ARG;
    *out = nullptr;
    if (p->width < 16 || p->height < 16 || p->max_features <= 0) return VISO_ERR_ARG;
    if (p->precision != VISO_PRECISION_FAITHFUL && p->precision != VISO_PRECISION_FAST) return VISO_ERR_ARG;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= device) return VISO_ERR_NODEVICE;
    VISO_HIP_CHECK(hipSetDevice(device));
    viso_rig* r = new (std::nothrow) viso_rig();
    if (!r) return VISO_ERR_ARG;
    r->p = *p;
    r->device = device;
    r->n = n_cams;
    r->geom = make_geom(p->width, p->height);
    for (int c = 0; c < n_cams; ++c)
        for (int k = 0; k < 12; ++k) r->E[c][k] = extrinsics[12 * c + k];
    if (hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking) != hipSuccess) {
        delete r;
        return VISO_ERR_HIP;
    }
    const int rc = r->init();
    if (rc) {
        r->release();
        delete r;
        return rc;
    }
    *out = r;
    return VISO_OK;
}

int viso_rig_destroy(viso_rig* r) {
    if (!r) return VISO_ERR_ARG;
    (void)hipSetDevice(r->device);
    r->release();
    delete r;
    return VISO_OK;
}

int viso_rig_set_stereo(viso_rig* r, double baseline, int32_t max_disp, int32_t min_disp) {
    if (!r || !(baseline > 0) || max_disp < 1 || max_disp > 255 || min_disp < 0 || min_disp > max_disp)
        return VISO_ERR_ARG;
    r->base = baseline;
    r->max_disp = max_disp;
    r->min_disp = min_disp;
    return VISO_OK;
}

int viso_rig_process_device(viso_rig* r, const uint8_t* d_left, const uint8_t* d_right, int32_t n_steps,
                            size_t frame_stride) {
    if (!r || !d_left || n_steps < 0) return VISO_ERR_ARG;
    if (frame_stride < (size_t)r->geom.w[0] * r->geom.h[0]) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(r->device));
    for (int s = 0; s < n_steps; ++s) {
        const uint8_t* L[kMaxRigCams];
        const uint8_t* R[kMaxRigCams];
        for (int c = 0; c < r->n; ++c) {
            const size_t o = frame_stride * ((size_t)s * r->n + c);
            L[c] = d_left + o;
            R[c] = d_right ? d_right + o : nullptr;
        }
        const int rc = r->step(L, d_right ? R : nullptr);
        if (rc) {
            r->flush();
            return rc;
        }
    }
    return r->flush();  // the last timestep's final solve
}

int viso_rig_process(viso_rig* r, const uint8_t* const* lefts, const uint8_t* const* rights,
                     const int32_t dims[3]) {
    if (!r || !lefts || !dims) return VISO_ERR_ARG;
    const int w = dims[0], h = dims[1], stride = dims[2];
    if (w != r->p.width || h != r->p.height || stride < w) return VISO_ERR_ARG;
    for (int c = 0; c < r->n; ++c)
        if (!lefts[c] || (rights && !rights[c])) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(r->device));
    const size_t npx = (size_t)w * h;
    const int imgs = rights ? 2 * r->n : r->n;
    int rc = r->staging.ensure(npx * imgs);
    if (rc) return rc;
    // the previous timestep's copies have left the staging buffer
    VISO_HIP_CHECK(hipStreamSynchronize(r->stream));
    uint8_t* base = (uint8_t*)r->staging.ptr;
    for (int c = 0; c < r->n; ++c) {
        VISO_HIP_CHECK(hipMemcpy2DAsync(base + npx * c, (size_t)w, lefts[c], (size_t)stride, (size_t)w, (size_t)h,
                                        hipMemcpyHostToDevice, r->stream));
        if (rights)
            VISO_HIP_CHECK(hipMemcpy2DAsync(base + npx * (r->n + c), (size_t)w, rights[c], (size_t)stride, (size_t)w,
                                            (size_t)h, hipMemcpyHostToDevice, r->stream));
    }
    const uint8_t* L[kMaxRigCams];
    const uint8_t* R[kMaxRigCams];
    for (int c = 0; c < r->n; ++c) {
        L[c] = base + npx * c;
        R[c] = base + npx * (r->n + c);
    }
    rc = r->step(L, rights ? R : nullptr);
    const int rf = r->flush();  // one timestep per call: its final solve now
    return rc ? rc : rf;
}

int viso_rig_synchronize(viso_rig* r) {
    if (!r) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(r->device));
    VISO_HIP_CHECK(hipStreamSynchronize(r->stream));
    return VISO_OK;
}

int viso_rig_get_state(viso_rig* r, int32_t* state) {
    if (!r || !state) return VISO_ERR_ARG;
    *state = r->state_;
    return VISO_OK;
}

int viso_rig_get_poses(viso_rig* r, double* T12, size_t cap, size_t* n) {
    if (!r) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(r->device));
    const size_t m = std::min(cap, (size_t)r->n_poses);
    if (m > 0 && T12) VISO_HIP_CHECK(hipMemcpyAsync(T12, r->log.ptr, 96 * m, hipMemcpyDeviceToHost, r->stream));
    VISO_HIP_CHECK(hipStreamSynchronize(r->stream));
    if (n) *n = (size_t)r->n_poses;
    return VISO_OK;
}

int viso_rig_get_points(viso_rig* r, int32_t cam, double* xyz, size_t cap, size_t* n) {
    if (!r || cam < 0 || cam >= r->n) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(r->device));
    const size_t m = std::min(cap, (size_t)r->n_pts[cam]);
    if (m > 0 && xyz)
        VISO_HIP_CHECK(hipMemcpyAsync(xyz, (const double*)r->map.ptr + 3 * (size_t)kMaxMapPoints * cam, 24 * m,
                                      hipMemcpyDeviceToHost, r->stream));
    VISO_HIP_CHECK(hipStreamSynchronize(r->stream));
    if (n) *n = (size_t)r->n_pts[cam];
    return VISO_OK;
}

int viso_rig_get_level_stats(viso_rig* r, double out[200]) {
    if (!r || !out) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(r->device));
    VISO_HIP_CHECK(hipMemcpyAsync(out, r->stats.ptr, 8 * 200, hipMemcpyDeviceToHost, r->stream));
    VISO_HIP_CHECK(hipStreamSynchronize(r->stream));
    return VISO_OK;
}

}  // extern "C"
