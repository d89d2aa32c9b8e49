// viso_amd — host context and C ABI (include/viso/viso_c.h).
//
// The context owns one HIP stream and all device memory of one sequence.
// Host code here is the orchestration the reference does in
// Viso::OnNewFrame (src/viso.cpp:7-145); every pixel/point loop runs in the
// gfx950 kernels of image.hip / track.hip / direct.hip / geometry.hip.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <new>
#include <vector>

#include "context.hpp"

using namespace viso;

namespace viso {

int DevBuf::ensure(size_t need) {
    if (need <= bytes) return VISO_OK;
    if (ptr) {
        VISO_HIP_CHECK(hipFree(ptr));
        ptr = nullptr;
        bytes = 0;
    }
    size_t b = std::max<size_t>(need, 256);
    VISO_HIP_CHECK(hipMalloc(&ptr, b));
    bytes = b;
    return VISO_OK;
}

void DevBuf::release() {
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    bytes = 0;
}

}  // namespace viso

static int check_device_present() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return VISO_ERR_NODEVICE;
    return VISO_OK;
}

extern "C" {

#ifndef VISO_SOURCE_HASH
#define VISO_SOURCE_HASH "unknown"
#endif
// "viso_amd <version> gfx950 (HIP) src:<hash>": the hash of the sources the
// library was built from (viso_amd/build.py source_hash)
const char* viso_version(void) { return "viso_amd 0.1 gfx950 (HIP) src:" VISO_SOURCE_HASH; }

int viso_default_params(viso_params* p, double fx, double fy, double cx, double cy, int32_t width,
                        int32_t height) {
    if (!p) return VISO_ERR_ARG;
    std::memset(p, 0, sizeof(*p));
    p->fx = fx;
    p->fy = fy;
    p->cx = cx;
    p->cy = cy;
    p->width = width;
    p->height = height;
    p->reinitialize_after = 10;          // include/viso.h:20
    p->fast_thresh = 50;                 // include/viso.h:21
    p->projection_error_thresh = 0.3;    // include/viso.h:22
    p->parallax_thresh = 1.0;            // include/viso.h:23
    p->disparity_squared_thresh = 225.0; // include/viso.h:24
    p->photometric_error_thresh = (4.0 * 2) * (4.0 * 2) * 15 * 15;  // include/viso.h:26
    p->enable_tracking = 0;
    p->ransac_e_iters = 1000;
    p->ransac_h_iters = 2000;
    p->ransac_confidence = 0.99;
    p->ransac_seed = 0x5eed5eedULL;
    p->max_features = 32768;
    p->max_poses = 65536;
    p->batch_frames = 64;
    p->precision = VISO_PRECISION_FAITHFUL;
    return VISO_OK;
}

int viso_pyramid_dims(int32_t width, int32_t height, int32_t dims[8], size_t* total_bytes) {
    if (width < 8 || height < 8 || !dims) return VISO_ERR_ARG;
    PyrGeom g = make_geom(width, height);
    for (int l = 0; l < kLevels; ++l) {
        dims[2 * l] = g.w[l];
        dims[2 * l + 1] = g.h[l];
    }
    if (total_bytes) *total_bytes = g.bytes;
    return VISO_OK;
}

int viso_create(const viso_params* p, int device, viso_ctx** out) {
    if (!p || !out) return VISO_ERR_ARG;
    *out = nullptr;
    if (p->width < 16 || p->height < 16 || p->width > kMaxWidth) return VISO_ERR_ARG;
    if (p->max_features <= 0 || p->max_features > 65536 || p->batch_frames <= 0) return VISO_ERR_ARG;
    if (p->precision != VISO_PRECISION_FAITHFUL && p->precision != VISO_PRECISION_FAST) return VISO_ERR_ARG;
    int rc = check_device_present();
    if (rc != VISO_OK) return rc;
    VISO_HIP_CHECK(hipSetDevice(device));
    viso_ctx* c = new (std::nothrow) viso_ctx();
    if (!c) return VISO_ERR_ARG;
    c->p = *p;
    c->device = device;
    if (const char* e = getenv("VISO_HOST_TIMES")) c->host_times.on = c->stage.timed = e[0] == '1';
    if (const char* e = getenv("VISO_HOST_TIMELINE")) c->dev_tl.on = e[0] == '1';
    c->geom = make_geom(p->width, p->height);
    if (c->create_streams() != VISO_OK) {
        delete c;
        return VISO_ERR_HIP;
    }
    rc = c->init();
    if (rc != VISO_OK) {
        viso_destroy(c);
        return rc;
    }
    *out = c;
    return VISO_OK;
}

int viso_destroy(viso_ctx* c) {
    if (!c) return VISO_ERR_ARG;
    (void)hipSetDevice(c->device);
    if (c->dev_tl.on && !c->dev_tl.marks.empty()) {
        (void)hipDeviceSynchronize();
        const hipEvent_t e0 = c->dev_tl.marks[0].e;
        int64_t fr = -1;
        fprintf(stderr, "viso device timeline (us from the first mark): frame: upload start / end, pyramid end, "
                        "chain start / end\n");
        for (auto& m : c->dev_tl.marks) {
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, e0, m.e);
            if (m.frame != fr) {
                fprintf(stderr, "%s%lld:", fr >= 0 ? "\n" : "", (long long)m.frame);
                fr = m.frame;
            }
            fprintf(stderr, " %d@%.1f", m.kind, 1e3 * ms);
        }
        fprintf(stderr, "\n");
        for (auto& m : c->dev_tl.marks) (void)hipEventDestroy(m.e);
        c->dev_tl.marks.clear();
    }
    if (c->host_times.on && c->host_times.calls > 0) {
        const double n = (double)c->host_times.calls;
        fprintf(stderr, "viso host times: %lld frame calls, us per call: ingest %.1f (pinned copy %.1f), "
                        "OnNewFrame %.1f, end %.1f\n",
                (long long)c->host_times.calls, c->host_times.us[0] / n, c->stage.copy_us / n,
                c->host_times.us[1] / n, c->host_times.us[2] / n);
    }
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    c->release();
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return VISO_OK;
}

int viso_synchronize(viso_ctx* c) {
    if (!c) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(c->device));
    // what host-frame calls left pending (their last final solve, queued LK)
    if (int rc = c->settle()) return rc;
    // the pose log's new entries ride this sync into pinned memory, so a
    // viso_get_poses after it makes no device round trip of its own
    {
        const int rc = c->stage_poses();
        if (rc) return rc;
    }
    VISO_HIP_CHECK(hipStreamSynchronize(c->stream));
    if (c->lk_stream) VISO_HIP_CHECK(hipStreamSynchronize(c->lk_stream));
    return c->bg_check();
}

int viso_timing_enable(viso_ctx* c, int32_t enable) {
    if (!c) return VISO_ERR_ARG;
    c->timing.enabled = enable != 0;
    return VISO_OK;
}

int viso_timing_select(viso_ctx* c, uint32_t kernel_mask) {
    if (!c) return VISO_ERR_ARG;
    c->timing.mask = kernel_mask;
    return VISO_OK;
}

int viso_timing_get(viso_ctx* c, int32_t kernel, int64_t* launches, double* total_ms) {
    if (!c || kernel < 0 || kernel >= VISO_KERNEL_COUNT) return VISO_ERR_ARG;
    // what host-frame calls left pending (the last frame's final solve and
    // LK batch) is launched and timed first
    if (int r = c->settle()) return r;
    int rc = c->timing.collect();
    if (rc != VISO_OK) return rc;
    if (launches) *launches = c->timing.launches[kernel];
    if (total_ms) *total_ms = c->timing.total_ms[kernel];
    return VISO_OK;
}

// ----------------------------------------------------------- stage entry points
int viso_pyramid(viso_ctx* c, const uint8_t* images, int32_t n, int32_t width, int32_t height,
                 uint8_t* out) {
    if (!c || !images || !out || n <= 0 || width < 8 || height < 8) return VISO_ERR_ARG;
    if (int rc = c->settle()) return rc;  // (host-frame work left pending)
    VISO_HIP_CHECK(hipSetDevice(c->device));
    PyrGeom g = make_geom(width, height);
    int rc = c->scratch_a.ensure(g.slot * (size_t)n);
    if (rc) return rc;
    uint8_t* d = (uint8_t*)c->scratch_a.ptr;
    const size_t l0 = (size_t)width * height;
    for (int i = 0; i < n; ++i)
        VISO_HIP_CHECK(hipMemcpyAsync(d + g.slot * i, images + l0 * i, l0, hipMemcpyHostToDevice,
                                      c->stream));
    {
        TimedRegion t(c->timing, VISO_KERNEL_PYRAMID, c->stream);
        launch_pyramid(g, d, n, g.slot, c->stream);
    }
    VISO_HIP_CHECK(hipGetLastError());
    for (int i = 0; i < n; ++i)
        VISO_HIP_CHECK(hipMemcpyAsync(out + g.bytes * i, d + g.slot * i, g.bytes,
                                      hipMemcpyDeviceToHost, c->stream));
    VISO_HIP_CHECK(hipStreamSynchronize(c->stream));
    return VISO_OK;
}

int viso_fast(viso_ctx* c, const uint8_t* image, int32_t width, int32_t height, int32_t thresh,
              int32_t* xs, int32_t* ys, int32_t* scores, size_t cap, size_t* n) {
    if (!c || !image || width < 8 || height < 8 || width > kMaxWidth) return VISO_ERR_ARG;
    if (int rc = c->settle()) return rc;  // (host-frame work left pending)
    VISO_HIP_CHECK(hipSetDevice(c->device));
    const size_t npx = (size_t)width * height;
    const size_t kcap = std::max<size_t>(cap, 1);
    int rc = c->scratch_a.ensure(npx);
    if (!rc) rc = c->scratch_b.ensure(fast_scratch_bytes(width, height));
    if (!rc) rc = c->scratch_c.ensure(sizeof(int4) * kcap + sizeof(int));
    if (rc) return rc;
    uint8_t* d_img = (uint8_t*)c->scratch_a.ptr;
    FastScratch s = fast_scratch_at(c->scratch_b.ptr, width, height);
    int4* d_raw = (int4*)c->scratch_c.ptr;
    int* d_n = (int*)((char*)c->scratch_c.ptr + sizeof(int4) * kcap);
    VISO_HIP_CHECK(hipMemcpyAsync(d_img, image, npx, hipMemcpyHostToDevice, c->stream));
    {
        TimedRegion t(c->timing, VISO_KERNEL_FAST, c->stream);
        launch_fast(d_img, width, height, thresh, s, nullptr, d_raw, (int)kcap, d_n, c->stream);
    }
    VISO_HIP_CHECK(hipGetLastError());
    int total = 0;
    VISO_HIP_CHECK(hipMemcpyAsync(&total, d_n, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    VISO_HIP_CHECK(hipStreamSynchronize(c->stream));
    size_t m = std::min<size_t>((size_t)total, cap);
    if (m > 0) {
        std::vector<int4> raw(m);
        VISO_HIP_CHECK(hipMemcpy(raw.data(), d_raw, sizeof(int4) * m, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < m; ++i) {
            if (xs) xs[i] = raw[i].x;
            if (ys) ys[i] = raw[i].y;
            if (scores) scores[i] = raw[i].z;
        }
    }
    if (n) *n = (size_t)total;
    return VISO_OK;
}

}  // extern "C"


// ----------------------------------------------------------- tracking stages
extern "C" {

int viso_klt(viso_ctx* c, const uint8_t* ref_pyr, const uint8_t* cur_pyr, int32_t width,
             int32_t height, const float* kp1, float* kp2, uint8_t* success, int32_t n) {
    if (!c || !ref_pyr || !cur_pyr || n < 0 || width < 16 || height < 16) return VISO_ERR_ARG;
    if (int rc = c->settle()) return rc;  // (host-frame work left pending)
    if (n == 0) return VISO_OK;
    if (!kp1 || !kp2 || !success) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(c->device));
    PyrGeom g = make_geom(width, height);
    Bump b;
    size_t o_ref = b.take(g.bytes), o_cur = b.take(g.bytes), o_k1 = b.take(8 * (size_t)n),
           o_k2 = b.take(8 * (size_t)n), o_s = b.take((size_t)n);
    int rc = c->scratch_a.ensure(b.off);
    if (rc) return rc;
    char* base = (char*)c->scratch_a.ptr;
    VISO_HIP_CHECK(hipMemcpyAsync(base + o_ref, ref_pyr, g.bytes, hipMemcpyHostToDevice, c->stream));
    VISO_HIP_CHECK(hipMemcpyAsync(base + o_cur, cur_pyr, g.bytes, hipMemcpyHostToDevice, c->stream));
    VISO_HIP_CHECK(hipMemcpyAsync(base + o_k1, kp1, 8 * (size_t)n, hipMemcpyHostToDevice, c->stream));
    VISO_HIP_CHECK(hipMemcpyAsync(base + o_k2, kp2, 8 * (size_t)n, hipMemcpyHostToDevice, c->stream));
    {
        TimedRegion t(c->timing, VISO_KERNEL_KLT, c->stream);
        launch_klt(frame_from_base((const uint8_t*)(base + o_ref), g),
                   frame_from_base((const uint8_t*)(base + o_cur), g), g,
                   (const float2*)(base + o_k1), (float2*)(base + o_k2), (uint8_t*)(base + o_s), n,
                   c->p.photometric_error_thresh, c->stream);
    }
    VISO_HIP_CHECK(hipGetLastError());
    VISO_HIP_CHECK(hipMemcpyAsync(kp2, base + o_k2, 8 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    VISO_HIP_CHECK(hipMemcpyAsync(success, base + o_s, (size_t)n, hipMemcpyDeviceToHost, c->stream));
    VISO_HIP_CHECK(hipStreamSynchronize(c->stream));
    return VISO_OK;
}

int viso_direct_pose(viso_ctx* c, const uint8_t* last_pyr, const uint8_t* cur_pyr, int32_t width,
                     int32_t height, const double* points, int32_t n, const double pose_last[12],
                     double pose_io[12]) {
    if (!c || !last_pyr || !cur_pyr || !pose_last || !pose_io || n < 0 || n > kMaxMapPoints)
        return VISO_ERR_ARG;
    if (int rc = c->settle()) return rc;  // (host-frame work left pending)
    if (n > 0 && !points) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(c->device));
    PyrGeom g = make_geom(width, height);
    Bump b;
    size_t o_l = b.take(g.bytes), o_c = b.take(g.bytes), o_p = b.take(24 * (size_t)std::max(n, 1)),
           o_pl = b.take(96), o_pio = b.take(96), o_ds = b.take(direct_scratch_bytes());
    int rc = c->scratch_a.ensure(b.off);
    if (rc) return rc;
    char* base = (char*)c->scratch_a.ptr;
    VISO_HIP_CHECK(hipMemcpyAsync(base + o_l, last_pyr, g.bytes, hipMemcpyHostToDevice, c->stream));
    VISO_HIP_CHECK(hipMemcpyAsync(base + o_c, cur_pyr, g.bytes, hipMemcpyHostToDevice, c->stream));
    if (n > 0)
        VISO_HIP_CHECK(hipMemcpyAsync(base + o_p, points, 24 * (size_t)n, hipMemcpyHostToDevice, c->stream));
    VISO_HIP_CHECK(hipMemcpyAsync(base + o_pl, pose_last, 96, hipMemcpyHostToDevice, c->stream));
    VISO_HIP_CHECK(hipMemcpyAsync(base + o_pio, pose_io, 96, hipMemcpyHostToDevice, c->stream));
    const double K[4] = {c->p.fx, c->p.fy, c->p.cx, c->p.cy};
    {
        TimedRegion t(c->timing, VISO_KERNEL_DIRECT, c->stream);
        launch_direct_pose(frame_from_base((const uint8_t*)(base + o_l), g),
                           frame_from_base((const uint8_t*)(base + o_c), g), g, K,
                           (const double*)(base + o_p), n, (const double*)(base + o_pl),
                           (const double*)(base + o_pio), direct_scratch_at(base + o_ds), nullptr,
                           (double*)(base + o_pio), nullptr, -1, c->stream, c->p.precision);
    }
    VISO_HIP_CHECK(hipGetLastError());
    VISO_HIP_CHECK(hipMemcpyAsync(pose_io, base + o_pio, 96, hipMemcpyDeviceToHost, c->stream));
    VISO_HIP_CHECK(hipStreamSynchronize(c->stream));
    return VISO_OK;
}

int viso_lk_align(viso_ctx* c, const uint8_t* kf_pyrs, const double* kf_poses, int32_t n_kf,
                  const uint8_t* cur_pyr, const double cur_pose[12], int32_t width, int32_t height,
                  const double* points, int32_t n, int32_t* pair_kf, uint8_t* success,
                  double* uv_before, double* uv_after) {
    if (!c || !kf_pyrs || !kf_poses || n_kf <= 0 || n_kf > kMaxKeyframes || !cur_pyr || !cur_pose ||
        n < 0)
        return VISO_ERR_ARG;
    if (int rc = c->settle()) return rc;  // (host-frame work left pending)
    if (n == 0) return VISO_OK;
    if (!points || !pair_kf || !success || !uv_before || !uv_after) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(c->device));
    PyrGeom g = make_geom(width, height);
    Bump b;
    size_t o_kf = b.take(g.bytes * (size_t)n_kf), o_kp = b.take(96 * (size_t)n_kf),
           o_c = b.take(g.bytes), o_cp = b.take(96), o_p = b.take(24 * (size_t)n),
           o_pk = b.take(4 * (size_t)n), o_s = b.take((size_t)n), o_ub = b.take(16 * (size_t)n),
           o_ua = b.take(16 * (size_t)n);
    int rc = c->scratch_a.ensure(b.off);
    if (rc) return rc;
    char* base = (char*)c->scratch_a.ptr;
    VISO_HIP_CHECK(hipMemcpyAsync(base + o_kf, kf_pyrs, g.bytes * (size_t)n_kf, hipMemcpyHostToDevice, c->stream));
    VISO_HIP_CHECK(hipMemcpyAsync(base + o_kp, kf_poses, 96 * (size_t)n_kf, hipMemcpyHostToDevice, c->stream));
    VISO_HIP_CHECK(hipMemcpyAsync(base + o_c, cur_pyr, g.bytes, hipMemcpyHostToDevice, c->stream));
    VISO_HIP_CHECK(hipMemcpyAsync(base + o_cp, cur_pose, 96, hipMemcpyHostToDevice, c->stream));
    VISO_HIP_CHECK(hipMemcpyAsync(base + o_p, points, 24 * (size_t)n, hipMemcpyHostToDevice, c->stream));
    LkAlignArgs a{};
    for (int j = 0; j < n_kf; ++j) a.kf[j] = frame_from_base((const uint8_t*)(base + o_kf + g.bytes * j), g);
    a.kf_poses = (const double*)(base + o_kp);
    a.n_kf = n_kf;
    a.n_frames = 1;
    a.frames[0].cur = frame_from_base((const uint8_t*)(base + o_c), g);
    a.frames[0].pose = (const double*)(base + o_cp);
    a.out_stride = 0;
    a.points = (const double*)(base + o_p);
    a.n = n;
    a.K[0] = c->p.fx;
    a.K[1] = c->p.fy;
    a.K[2] = c->p.cx;
    a.K[3] = c->p.cy;
    a.thresh = c->p.photometric_error_thresh;
    for (int l = 0; l < kLevels; ++l) {
        a.g.w[l] = g.w[l];
        a.g.h[l] = g.h[l];
        a.g.off[l] = g.off[l];
    }
    a.pair_kf = (int32_t*)(base + o_pk);
    a.success = (uint8_t*)(base + o_s);
    a.uv_before = (double*)(base + o_ub);
    a.uv_after = (double*)(base + o_ua);
    {
        TimedRegion t(c->timing, VISO_KERNEL_LKALIGN, c->stream);
        launch_lk_align(a, c->stream);
    }
    VISO_HIP_CHECK(hipGetLastError());
    VISO_HIP_CHECK(hipMemcpyAsync(pair_kf, base + o_pk, 4 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    VISO_HIP_CHECK(hipMemcpyAsync(success, base + o_s, (size_t)n, hipMemcpyDeviceToHost, c->stream));
    VISO_HIP_CHECK(hipMemcpyAsync(uv_before, base + o_ub, 16 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    VISO_HIP_CHECK(hipMemcpyAsync(uv_after, base + o_ua, 16 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    VISO_HIP_CHECK(hipStreamSynchronize(c->stream));
    return VISO_OK;
}

}  // extern "C"

extern "C" int viso_set_stereo(viso_ctx* c, double baseline, int32_t max_disp, int32_t min_disp) {
    if (!c || !(baseline >= 0) || (baseline > 0 && (max_disp < 2 || min_disp < 1 || min_disp >= max_disp)))
        return VISO_ERR_ARG;
    if (int rc = c->settle()) return rc;  // (host-frame work left pending)
    c->stereo_base = baseline;
    c->stereo_max_disp = max_disp;
    c->stereo_min_disp = min_disp;
    return VISO_OK;
}

extern "C" int viso_set_keyframes(viso_ctx* c, int32_t interval, int32_t ngood_permille) {
    if (!c || interval < 0 || ngood_permille < 0 || ngood_permille > 1000) return VISO_ERR_ARG;
    if (int rc = c->settle()) return rc;  // (host-frame work left pending)
    c->kf_interval = interval;
    c->kf_permille = ngood_permille;
    return VISO_OK;
}

extern "C" int viso_set_bundle_adjust(viso_ctx* c, int32_t iterations) {
    if (!c || iterations < 0 || iterations > 100) return VISO_ERR_ARG;
    if (int rc = c->settle()) return rc;  // (host-frame work left pending)
    c->ba_iterations = iterations;
    return VISO_OK;
}

extern "C" int viso_photometric_ba(viso_ctx* c, const uint8_t* const* kf_images, int32_t n_kf, double* kf_poses,
                                   double* points, const int32_t* host, int32_t n, int32_t iterations,
                                   double* report) {
    if (!c || !kf_images || !kf_poses || !points || !host) return VISO_ERR_ARG;
    if (int rc = c->settle()) return rc;  // (host-frame work left pending)
    // n bounded as the pipeline's map (the block trees' stack depth and the
    // launch grids are sized for kMaxMapPoints)
    if (n_kf < 2 || n_kf > kMaxKeyframes || n < 1 || n > kMaxMapPoints || iterations < 1 || iterations > 100)
        return VISO_ERR_ARG;
    for (int i = 0; i < n; ++i)
        if (host[i] < 0 || host[i] >= n_kf) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(c->device));
    const int w = c->p.width, h = c->p.height;
    const size_t npx = (size_t)w * h;
    Bump b;
    const size_t o_img = b.take(npx * n_kf), o_pose = b.take(96 * (size_t)n_kf), o_pts = b.take(24 * (size_t)n),
                 o_host = b.take(4 * (size_t)n), o_rep = b.take(32 * (size_t)iterations);
    int rc = c->scratch_a.ensure(b.off);
    if (!rc) rc = c->ba_scratch.ensure(ba_scratch_bytes(n));
    if (rc) return rc;
    char* base = (char*)c->scratch_a.ptr;
    const uint8_t* l0[kMaxKeyframes];
    for (int k = 0; k < n_kf; ++k) {
        VISO_HIP_CHECK(hipMemcpyAsync(base + o_img + npx * k, kf_images[k], npx, hipMemcpyHostToDevice, c->stream));
        l0[k] = (const uint8_t*)(base + o_img + npx * k);
    }
    VISO_HIP_CHECK(hipMemcpyAsync(base + o_pose, kf_poses, 96 * (size_t)n_kf, hipMemcpyHostToDevice, c->stream));
    VISO_HIP_CHECK(hipMemcpyAsync(base + o_pts, points, 24 * (size_t)n, hipMemcpyHostToDevice, c->stream));
    VISO_HIP_CHECK(hipMemcpyAsync(base + o_host, host, 4 * (size_t)n, hipMemcpyHostToDevice, c->stream));
    const double K[4] = {c->p.fx, c->p.fy, c->p.cx, c->p.cy};
    if (launch_photometric_ba(l0, n_kf, w, h, K, (double*)(base + o_pose), (double*)(base + o_pts),
                              (const int*)(base + o_host), n, iterations, c->ba_scratch.ptr,
                              (double*)(base + o_rep), c->stream))
        return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipGetLastError());
    VISO_HIP_CHECK(hipMemcpyAsync(kf_poses, base + o_pose, 96 * (size_t)n_kf, hipMemcpyDeviceToHost, c->stream));
    VISO_HIP_CHECK(hipMemcpyAsync(points, base + o_pts, 24 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    if (report)
        VISO_HIP_CHECK(hipMemcpyAsync(report, base + o_rep, 32 * (size_t)iterations, hipMemcpyDeviceToHost, c->stream));
    VISO_HIP_CHECK(hipStreamSynchronize(c->stream));
    return VISO_OK;
}

extern "C" int viso_stereo_match(viso_ctx* c, const uint8_t* left, const uint8_t* right,
                                 int32_t width, int32_t height, const int32_t* xs,
                                 const int32_t* ys, int32_t n, int32_t max_disp,
                                 int32_t* disparity, int32_t* sad) {
    if (!c || !left || !right || width < 8 || height < 8 || n < 0 || max_disp < 0)
        return VISO_ERR_ARG;
    if (int rc = c->settle()) return rc;  // (host-frame work left pending)
    if (n == 0) return VISO_OK;
    if (!xs || !ys || !disparity || !sad) return VISO_ERR_ARG;
    VISO_HIP_CHECK(hipSetDevice(c->device));
    const size_t npx = (size_t)width * height;
    Bump b;
    const size_t o_l = b.take(npx), o_r = b.take(npx), o_x = b.take(4 * (size_t)n),
                 o_y = b.take(4 * (size_t)n), o_d = b.take(4 * (size_t)n), o_s = b.take(4 * (size_t)n);
    int rc = c->scratch_a.ensure(b.off);
    if (rc) return rc;
    char* base = (char*)c->scratch_a.ptr;
    VISO_HIP_CHECK(hipMemcpyAsync(base + o_l, left, npx, hipMemcpyHostToDevice, c->stream));
    VISO_HIP_CHECK(hipMemcpyAsync(base + o_r, right, npx, hipMemcpyHostToDevice, c->stream));
    VISO_HIP_CHECK(hipMemcpyAsync(base + o_x, xs, 4 * (size_t)n, hipMemcpyHostToDevice, c->stream));
    VISO_HIP_CHECK(hipMemcpyAsync(base + o_y, ys, 4 * (size_t)n, hipMemcpyHostToDevice, c->stream));
    {
        TimedRegion t(c->timing, VISO_KERNEL_STEREO, c->stream);
        launch_stereo_sad((const uint8_t*)(base + o_l), (const uint8_t*)(base + o_r), width, height,
                          (const int*)(base + o_x), (const int*)(base + o_y), n, max_disp,
                          (int*)(base + o_d), (int*)(base + o_s), c->stream);
    }
    VISO_HIP_CHECK(hipGetLastError());
    VISO_HIP_CHECK(hipMemcpyAsync(disparity, base + o_d, 4 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    VISO_HIP_CHECK(hipMemcpyAsync(sad, base + o_s, 4 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    VISO_HIP_CHECK(hipStreamSynchronize(c->stream));
    return VISO_OK;
}
