// viso_amd — header-only C++ facade of the multi-camera photometric rig on
// the reference path (viso_rig.h).
#ifndef VISO_RIG_HPP
#define VISO_RIG_HPP

#include <array>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "viso_rig.h"

namespace viso {

class VisoRig {
public:
    using Pose = std::array<double, 12>;
    // p: shared single-camera parameters; extrinsics: n_cams x 12 (rig -> camera)
    VisoRig(const viso_params& p, int n_cams, const double* extrinsics, int device = 0) : n_(n_cams) {
        check(viso_rig_create(&p, n_cams, extrinsics, device, &r_), "viso_rig_create");
    }
    ~VisoRig() {
        if (r_) viso_rig_destroy(r_);
    }
    VisoRig(const VisoRig&) = delete;
    VisoRig& operator=(const VisoRig&) = delete;

    void SetStereo(double baseline, int max_disp = 128, int min_disp = 1) {
        check(viso_rig_set_stereo(r_, baseline, max_disp, min_disp), "viso_rig_set_stereo");
    }
    // one timestep; rights may be null once tracking
    void process(const uint8_t* const* lefts, const uint8_t* const* rights, const int32_t* dims) {
        check(viso_rig_process(r_, lefts, rights, dims), "viso_rig_process");
    }
    std::vector<Pose> poses() const {
        size_t n = 0;
        check(viso_rig_get_poses(r_, nullptr, 0, &n), "viso_rig_get_poses");
        std::vector<Pose> out(n);
        if (n) check(viso_rig_get_poses(r_, out.front().data(), n, &n), "viso_rig_get_poses");
        return out;
    }
    int state() const {
        int32_t s = 0;
        check(viso_rig_get_state(r_, &s), "viso_rig_get_state");
        return s;
    }
    int cameras() const { return n_; }

private:
    static void check(int rc, const char* what) {
        if (rc != VISO_OK) throw std::runtime_error(std::string(what) + " failed: " + std::to_string(rc));
    }
    viso_rig* r_ = nullptr;
    int n_;
};

}  // namespace viso

#endif
