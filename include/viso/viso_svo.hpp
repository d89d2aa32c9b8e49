// viso_amd — header-only C++ facade of the north-star stereo VO (viso_svo.h)
// with the class names the north star gives: VisualOdometryStereo
// (process(left, right, dims), getMotion(), poses) and Matcher
// (pushBack(left, right), matchFeatures(), getMatches()); plus the
// multi-camera VisualOdometryStereoRig (BASELINE.json configs[4]).  The spec
// is the repo's own (oracle/oracle_svo.cpp).  No Eigen /
// OpenCV types: poses and motions are std::array<double, 12> (R row-major, t).
#ifndef VISO_SVO_HPP
#define VISO_SVO_HPP

#include <array>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "viso_svo.h"

namespace viso {

inline void svo_check(int rc, const char* what) {
    if (rc != VISO_OK) throw std::runtime_error(std::string(what) + " failed: " + std::to_string(rc));
}

class VisualOdometryStereo {
public:
    using Motion = std::array<double, 12>;
    // one match {u_l1, v_l1, u_r1, v_r1, u_l2, v_l2, u_r2, v_r2}
    using Match = std::array<int32_t, 8>;

    explicit VisualOdometryStereo(const viso_svo_params& p, int device = 0) {
        svo_check(viso_svo_create(&p, device, &s_), "viso_svo_create");
    }
    // defaults (viso_svo_default_params) for a rectified pair
    VisualOdometryStereo(int width, int height, double fx, double fy, double cu, double cv, double base,
                         int device = 0) {
        viso_svo_params p;
        svo_check(viso_svo_default_params(&p, width, height, fx, fy, cu, cv, base), "viso_svo_default_params");
        svo_check(viso_svo_create(&p, device, &s_), "viso_svo_create");
    }
    ~VisualOdometryStereo() {
        if (s_) viso_svo_destroy(s_);
    }
    VisualOdometryStereo(const VisualOdometryStereo&) = delete;
    VisualOdometryStereo& operator=(const VisualOdometryStereo&) = delete;

    // true when a motion was estimated for this pair
    bool process(const uint8_t* left, const uint8_t* right, const int32_t* dims) {
        int32_t ok = 0;
        svo_check(viso_svo_process(s_, left, right, dims, &ok), "viso_svo_process");
        return ok != 0;
    }
    Motion getMotion() const {
        Motion m{};
        svo_check(viso_svo_get_motion(s_, m.data()), "viso_svo_get_motion");
        return m;
    }
    std::vector<Motion> poses() const {
        size_t n = 0;
        svo_check(viso_svo_get_poses(s_, nullptr, 0, &n), "viso_svo_get_poses");
        std::vector<Motion> out(n);
        if (n) svo_check(viso_svo_get_poses(s_, out.front().data(), n, &n), "viso_svo_get_poses");
        return out;
    }
    std::vector<Match> getMatches(std::vector<uint8_t>* inliers = nullptr) const {
        size_t n = 0;
        svo_check(viso_svo_get_matches(s_, nullptr, nullptr, 0, &n), "viso_svo_get_matches");
        std::vector<Match> out(n);
        std::vector<uint8_t> in(n ? n : 1);
        if (n) svo_check(viso_svo_get_matches(s_, out.front().data(), in.data(), n, &n), "viso_svo_get_matches");
        if (inliers) inliers->assign(in.begin(), in.begin() + (long)n);
        return out;
    }
    viso_svo* handle() const { return s_; }

protected:
    VisualOdometryStereo() = default;
    viso_svo* s_ = nullptr;
};

// Matcher: pushBack(left, right) per stereo pair; after two pairs,
// matchFeatures() runs the circular matching + bucketing of the last two
// and getMatches() returns them (the engine's matching pass on its own pairs).
class Matcher {
public:
    explicit Matcher(const viso_svo_params& p, int device = 0) : vo_(p, device), dims_{p.width, p.height, p.width} {}
    void pushBack(const uint8_t* left, const uint8_t* right) {
        vo_.process(left, right, dims_);
        ++pushed_;
    }
    // the matches of the last two pairs (false before two pairs were pushed)
    bool matchFeatures() { return pushed_ >= 2; }
    std::vector<VisualOdometryStereo::Match> getMatches() const { return vo_.getMatches(); }

private:
    VisualOdometryStereo vo_;
    int32_t dims_[3];
    int pushed_ = 0;
};

// n_cams rigid stereo cameras (viso_svo_rig_create), one rig motion per timestep
class VisualOdometryStereoRig : public VisualOdometryStereo {
public:
    VisualOdometryStereoRig(const viso_svo_params& p, int n_cams, const double* extrinsics, int device = 0)
        : n_(n_cams) {
        svo_check(viso_svo_rig_create(&p, n_cams, extrinsics, device, &s_), "viso_svo_rig_create");
    }
    bool process(const uint8_t* const* lefts, const uint8_t* const* rights, const int32_t* dims) {
        int32_t ok = 0;
        svo_check(viso_svo_rig_process(s_, lefts, rights, dims, &ok), "viso_svo_rig_process");
        return ok != 0;
    }
    int cameras() const { return n_; }

private:
    int n_;
};

}  // namespace viso

#endif
