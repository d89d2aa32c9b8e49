// viso_amd — context object behind the C ABI.
#pragma once

#include <vector>

#include "../../include/viso/viso_c.h"
#include "kernels.hpp"

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

struct TimedRegion {
    Timing& t;
    int kernel;
    hipStream_t s;
    hipEvent_t a = nullptr, b = nullptr;
    TimedRegion(Timing& t_, int k, hipStream_t s_) : t(t_), kernel(k), s(s_) {
        if (t.enabled) {
            a = t.get_event();
            b = t.get_event();
            (void)hipEventRecord(a, s);
        }
    }
    ~TimedRegion() {
        if (t.enabled && a && b) {
            (void)hipEventRecord(b, s);
            t.pending.push_back({kernel, a, b});
        }
    }
};

}  // namespace viso

struct viso_ctx {
    viso_params p{};
    int device = 0;
    hipStream_t stream = nullptr;
    viso::PyrGeom geom{};
    viso::Timing timing;
    // scratch for the stage-level entry points
    viso::DevBuf scratch_a, scratch_b, scratch_c, scratch_d;

    int init();
    void release();
};
