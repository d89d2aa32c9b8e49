// viso_amd — header-only C++ facade over the C ABI (viso_c.h) that keeps the
// reference's class names and call shapes, so code written against
// Seasandwpy/viso compiles with minimal changes:
//   Keyframe(mat)                     include/keyframe.h:28-46 (raw grey buffer
//                                     instead of cv::Mat)
//   FrameSequence::FrameHandler       include/frame_sequence.h:13-16
//   FrameSequence::RunOnce()          include/frame_sequence.h:25-38 (loader
//                                     callback instead of cv::imread)
//   Viso(fx, fy, cx, cy)              include/viso.h:47-52
//   Viso::OnNewFrame(Keyframe::Ptr)   src/viso.cpp:7-145
//   Viso::poses                       include/viso.h:54 (Tcw, R row-major + t)
//   Viso::GetPoints()                 include/viso.h:60-67
//   StereoViso::process(left, right, dims)   the reference path with the
//                                     stereo initialisation (viso_set_stereo)
// The north-star VisualOdometryStereo / Matcher (the SVO engine) are in
// viso_svo.hpp, the multi-camera photometric rig (VisoRig) in viso_rig.hpp.
// No Eigen / Sophus / OpenCV types: poses are std::array<double, 12>.
#ifndef VISO_HPP
#define VISO_HPP

#include <array>
#include <cstdint>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "viso_c.h"

namespace viso {

inline void check(int rc, const char* what) {
    if (rc != VISO_OK) throw std::runtime_error(std::string(what) + " failed: " + std::to_string(rc));
}

using Pose = std::array<double, 12>;  // R (row-major 3x3) + t: Pc = R * Pw + t
using V3d = std::array<double, 3>;

class Keyframe {
public:
    using Ptr = std::shared_ptr<Keyframe>;
    Keyframe(const uint8_t* grey, int width, int height, int stride)
        : id_(next_id_++), w_(width), h_(height), data_(grey, grey + (size_t)stride * height),
          stride_(stride) {}
    long GetId() const { return id_; }
    static long GetNextId() { return next_id_; }
    const uint8_t* Data() const { return data_.data(); }
    int Width() const { return w_; }
    int Height() const { return h_; }
    int Stride() const { return stride_; }

private:
    static inline long next_id_ = 0;
    long id_;
    int w_, h_;
    std::vector<uint8_t> data_;
    int stride_;
};

class FrameSequence {
public:
    class FrameHandler {
    public:
        virtual ~FrameHandler() = default;
        virtual void OnNewFrame(Keyframe::Ptr keyframe) = 0;
    };
    // loader(path, &grey, &w, &h) -> false when the file does not exist
    using Loader = std::function<bool(const std::string&, std::vector<uint8_t>*, int*, int*)>;
    FrameSequence(std::string location, FrameHandler* handler, Loader loader)
        : location_(std::move(location)), handler_(handler), loader_(std::move(loader)) {}
    void RunOnce() {
        const std::string file = location_ + std::to_string(Keyframe::GetNextId() + 1) + ".png";
        std::vector<uint8_t> grey;
        int w = 0, h = 0;
        if (loader_(file, &grey, &w, &h))
            handler_->OnNewFrame(std::make_shared<Keyframe>(grey.data(), w, h, w));
    }

private:
    std::string location_;
    FrameHandler* handler_;
    Loader loader_;
};

class Viso : public FrameSequence::FrameHandler {
public:
    Viso(double fx, double fy, double cx, double cy, int width, int height, int device = 0,
         bool enable_tracking = false) {
        viso_params p;
        check(viso_default_params(&p, fx, fy, cx, cy, width, height), "viso_default_params");
        p.enable_tracking = enable_tracking ? 1 : 0;
        check(viso_create(&p, device, &ctx_), "viso_create");
    }
    explicit Viso(const viso_params& p, int device = 0) { check(viso_create(&p, device, &ctx_), "viso_create"); }
    ~Viso() override {
        if (ctx_) viso_destroy(ctx_);
    }
    Viso(const Viso&) = delete;
    Viso& operator=(const Viso&) = delete;

    void OnNewFrame(Keyframe::Ptr cur) override {
        check(viso_process_frame(ctx_, cur->Data(), cur->Width(), cur->Height(), cur->Stride()),
              "viso_process_frame");
    }

    // The pose log.  The reference exposes it as a public field
    // (`std::vector<Sophus::SE3d> poses`, include/viso.h:54; src/main.cpp:50
    // passes `viso.poses` to DrawMap and iterates it), so `poses` is a member
    // that reads like that field -- `viso.poses.size()`, `viso.poses[i]`,
    // `for (auto& Tcw : viso.poses)`, `const std::vector<Pose>& p =
    // viso.poses` -- and also keeps the call form `viso.poses()`.  Every use
    // copies the log from the device (synchronising the context); range-for
    // and indexing work on that snapshot, refreshed by size() / begin().
    class PoseLog {
       public:
        explicit PoseLog(const Viso* v) : v_(v) {}
        PoseLog(const PoseLog&) = delete;
        PoseLog& operator=(const PoseLog&) = delete;
        std::vector<Pose> operator()() const { return v_->fetch_poses(); }
        operator std::vector<Pose>() const { return v_->fetch_poses(); }
        size_t size() const { return refresh().size(); }
        bool empty() const { return size() == 0; }
        const Pose& operator[](size_t i) const { return cache_.size() > i ? cache_[i] : refresh()[i]; }
        std::vector<Pose>::const_iterator begin() const { return refresh().begin(); }
        std::vector<Pose>::const_iterator end() const { return cache_.end(); }

       private:
        const std::vector<Pose>& refresh() const {
            cache_ = v_->fetch_poses();
            return cache_;
        }
        const Viso* v_;
        mutable std::vector<Pose> cache_;
    };
    PoseLog poses{this};

    std::vector<V3d> GetPoints() const {
        size_t n = 0;
        check(viso_get_points(ctx_, nullptr, 0, &n), "viso_get_points");
        std::vector<V3d> out(n);
        if (n) check(viso_get_points(ctx_, out.front().data(), n, &n), "viso_get_points");
        return out;
    }

    std::vector<Pose> fetch_poses() const {
        size_t n = 0;
        check(viso_get_poses(ctx_, nullptr, 0, &n), "viso_get_poses");
        std::vector<Pose> out(n);
        if (n) check(viso_get_poses(ctx_, out.front().data(), n, &n), "viso_get_poses");
        return out;
    }

    int state() const {
        int32_t s = 0;
        check(viso_get_state(ctx_, &s), "viso_get_state");
        return s;
    }

    viso_ctx* handle() const { return ctx_; }

protected:
    viso_ctx* ctx_ = nullptr;
};

// The reference path fed with stereo pairs: the left image drives
// OnNewFrame; while initialising, the right image gives the metric stereo
// initialisation (viso_set_stereo, enabled with SetStereo) in place of the
// 2D-2D one (src/viso.cpp:178-256).
class StereoViso : public Viso {
public:
    using Viso::Viso;
    void SetStereo(double baseline, int max_disp = 128, int min_disp = 1) {
        check(viso_set_stereo(ctx_, baseline, max_disp, min_disp), "viso_set_stereo");
    }
    bool process(const uint8_t* left, const uint8_t* right, const int32_t* dims) {
        return viso_process_stereo(ctx_, left, right, dims) == VISO_OK;
    }
};

}  // namespace viso

#endif
