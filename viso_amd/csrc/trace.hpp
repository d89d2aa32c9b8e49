// viso_amd — roctx ranges around the per-frame phases (SURVEY.md §5
// "Tracing": the reference has a Timer it never instantiates).  Enabled by
// VISO_ROCTX=1 in the environment (read once); off, a range costs one
// branch.  Collected by `rocprofv3 --marker-trace` (the ranges name the
// phase: viso:frame, viso:ingest, viso:pyramid, viso:direct, viso:lkalign,
// svo:batch, rig:timestep, ...).
#pragma once

#include <cstdlib>

#include <rocprofiler-sdk-roctx/roctx.h>

namespace viso {

inline bool roctx_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("VISO_ROCTX");
        return e && *e && *e != '0';
    }();
    return on;
}

struct RoctxRange {
    bool on;
    explicit RoctxRange(const char* name) : on(roctx_enabled()) {
        if (on) roctxRangePushA(name);
    }
    ~RoctxRange() {
        if (on) roctxRangePop();
    }
    RoctxRange(const RoctxRange&) = delete;
    RoctxRange& operator=(const RoctxRange&) = delete;
};

// range names of the VISO_KERNEL_* phases (TimedRegion)
inline const char* phase_name(int kernel) {
    static const char* const names[] = {"viso:pyramid", "viso:fast",  "viso:klt",    "viso:ransac",
                                        "viso:select",  "viso:direct", "viso:lkalign", "viso:stereo",
                                        "viso:upload"};
    return (kernel >= 0 && kernel < 9) ? names[kernel] : "viso:phase";
}

}  // namespace viso
