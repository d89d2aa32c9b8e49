// viso_amd — host image upload through pinned staging.
//
// Frames handed over in host memory (viso_process_frame / _stereo,
// viso_svo_process, the drop-in's FrameSequence::RunOnce -> OnNewFrame
// pattern, include/frame_sequence.h:25-38) are usually pageable.  A pageable
// hipMemcpy2DAsync goes through the runtime's own staging, row by row:
// measured 3.25 ms per 1242x375 image on MI355X.  Here the CPU copies the
// rows into a pinned buffer (one of a ring) and one DMA moves it; an event per
// buffer orders its reuse behind that DMA.
#pragma once

#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstring>

namespace viso {

struct HostStage {
    static constexpr int kRing = 8;
    uint8_t* buf[kRing] = {};
    size_t cap[kRing] = {};
    hipEvent_t ev[kRing] = {};
    bool used[kRing] = {};
    int next = 0;
    hipEvent_t last = nullptr;  // the latest upload's event (behind its DMA on s)
    double copy_us = 0.0;       // (VISO_HOST_TIMES) host time in the row copies
    bool timed = false;

    int pending = -1;  // a buffer whose reuse event the caller records (upload(defer))

    // The buffer's reuse event, recorded by the caller on `s` behind work that
    // follows the DMA on the same stream (its pyramid): one marker per frame
    // on that stream instead of two (each record is a marker packet).
    hipError_t commit(hipStream_t s) {
        if (pending < 0) return hipSuccess;
        const int k = pending;
        pending = -1;
        hipError_t e = hipEventRecord(ev[k], s);
        if (e != hipSuccess) return e;
        used[k] = true;
        last = ev[k];
        return hipSuccess;
    }

    // rows [0, h) of w bytes at src (row pitch stride) -> dst (packed), on s;
    // defer: the reuse event is left to commit()
    hipError_t upload(uint8_t* dst, const uint8_t* src, int w, int h, int stride, hipStream_t s, bool defer = false) {
        const size_t bytes = (size_t)w * (size_t)h;
        const int k = next;
        next = (next + 1) % kRing;
        hipError_t e;
        if (used[k] && (e = hipEventSynchronize(ev[k])) != hipSuccess) return e;  // its last DMA is done
        if (cap[k] < bytes) {
            if (buf[k] && (e = hipHostFree(buf[k])) != hipSuccess) return e;
            buf[k] = nullptr;
            cap[k] = 0;
            if ((e = hipHostMalloc((void**)&buf[k], bytes)) != hipSuccess) return e;
            cap[k] = bytes;
        }
        if (!ev[k] && (e = hipEventCreateWithFlags(&ev[k], hipEventDisableTiming)) != hipSuccess) return e;
        const auto t0 = timed ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point{};
        if (stride == w)
            std::memcpy(buf[k], src, bytes);
        else
            for (int y = 0; y < h; ++y) std::memcpy(buf[k] + (size_t)y * w, src + (size_t)y * stride, (size_t)w);
        if (timed)
            copy_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        if ((e = hipMemcpyAsync(dst, buf[k], bytes, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
        if (defer) {
            pending = k;
            return hipSuccess;
        }
        if ((e = hipEventRecord(ev[k], s)) != hipSuccess) return e;
        used[k] = true;
        last = ev[k];
        return hipSuccess;
    }

    void release() {
        for (int k = 0; k < kRing; ++k) {
            if (ev[k]) {
                (void)hipEventSynchronize(ev[k]);
                (void)hipEventDestroy(ev[k]);
            }
            if (buf[k]) (void)hipHostFree(buf[k]);
            buf[k] = nullptr;
            ev[k] = nullptr;
            cap[k] = 0;
            used[k] = false;
        }
        last = nullptr;
    }
};

}  // namespace viso
