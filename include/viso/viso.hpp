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

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <mutex>
#include <vector>

#include "viso_c.h"

namespace viso {

inline void check(int rc, const char* what) {
    if (rc != VISO_OK) throw std::runtime_error(std::string(what) + " failed: " + std::to_string(rc));
}

using Pose = std::array<double, 12>;  // R (row-major 3x3) + t: Pc = R * Pw + t
using V3d = std::array<double, 3>;
using V2d = std::array<double, 2>;
using M3d = std::array<double, 9>;  // row-major

// cv::KeyPoint's fields (Keyframe::Keypoints / AddKeypoint)
struct KeyPoint {
    float x = 0.f, y = 0.f;  // pt
    float size = 0.f, angle = -1.f, response = 0.f;
    int octave = 0, class_id = -1;
};

// One pyramid level as the reference reads a cv::Mat: data, cols, rows, step
// (continuous: step == cols for levels 1..3, the caller's stride for level 0).
struct GreyView {
    const uint8_t* data = nullptr;
    int cols = 0, rows = 0;
    size_t step = 0;
};

namespace detail {
// A library context per image size that builds Keyframe pyramids with the
// same pyrDown kernels as the frame path (viso_pyramid).  Keyframe has no
// device argument (the reference's Keyframe(cv::Mat) has none), so these
// contexts live on device 0; they are created once per size, shared by every
// thread (the cache is guarded by a mutex) and released only at process exit.
inline viso_ctx* pyramid_ctx(int w, int h) {
    struct Entry {
        int w, h;
        viso_ctx* ctx;
    };
    static std::mutex mu;
    static std::vector<Entry> cache;
    std::lock_guard<std::mutex> lock(mu);
    for (const Entry& e : cache)
        if (e.w == w && e.h == h) return e.ctx;
    viso_params p;
    check(viso_default_params(&p, 1.0, 1.0, 0.0, 0.0, w, h), "viso_default_params");
    viso_ctx* c = nullptr;
    check(viso_create(&p, 0, &c), "viso_create");
    cache.push_back(Entry{w, h, c});
    return c;
}
}  // namespace detail

// include/keyframe.h:10-123.  The frame is a raw grey buffer instead of a
// cv::Mat; the accessors keep the reference's names, arguments and
// arithmetic (GetPixelValue's int() base with floor weights, :50-57;
// GetGradient's central differences, :59-64; Project, :82-89; IsInside,
// :71-80; ViewingAngle, :93-98), so a FrameHandler written against the
// reference compiles.  The pyramid (:37-45) is built on first use by the
// library's pyrDown kernels; taps outside a level's buffer read 0 (the
// reference reads past the cv::Mat there).  These are per-call host helpers
// for handler code: the tracking path never calls them.
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

    // include/keyframe.h:102
    GreyView Mat() const { return GreyView{data_.data(), w_, h_, (size_t)stride_}; }
    // include/keyframe.h:112: levels 0..3 (level 0 is the frame itself)
    const std::vector<GreyView>& Pyramids() const {
        if (pyr_views_.empty()) build_pyramid();
        return pyr_views_;
    }
    // include/keyframe.h:110
    double GetScale(int level) const { return kScales[level]; }

    // include/keyframe.h:50-57
    double GetPixelValue(const double& x, const double& y, int level = 0) const {
        const GreyView& m = Pyramids()[level];
        const long long n = (long long)m.step * m.rows;
        const long long base = (long long)(int)y * (long long)m.step + (long long)(int)x;
        auto tap = [&](long long i) -> double { return (i >= 0 && i < n) ? (double)m.data[i] : 0.0; };
        const double xx = x - std::floor(x);
        const double yy = y - std::floor(y);
        return double((1 - xx) * (1 - yy) * tap(base) + xx * (1 - yy) * tap(base + 1) +
                      (1 - xx) * yy * tap(base + (long long)m.step) + xx * yy * tap(base + (long long)m.step + 1));
    }
    // include/keyframe.h:59-64
    V2d GetGradient(const double& u, const double& v, int level = 0) const {
        const double dx = 0.5 * (GetPixelValue(u + 1, v, level) - GetPixelValue(u - 1, v, level));
        const double dy = 0.5 * (GetPixelValue(u, v + 1, level) - GetPixelValue(u, v - 1, level));
        return V2d{dx, dy};
    }
    // include/keyframe.h:82-89 (Pc = R Pw + T, then K at the level's scale)
    V2d Project(const V3d& point, int level) const {
        double uv1[3];
        for (int i = 0; i < 3; ++i)
            uv1[i] = (R_[3 * i] * point[0] + R_[3 * i + 1] * point[1]) + R_[3 * i + 2] * point[2] + T_[i];
        const double z = uv1[2];
        for (int i = 0; i < 3; ++i) uv1[i] /= z;
        const double u = kScales[level] * (uv1[0] * K_[0] + K_[2]);
        const double v = kScales[level] * (uv1[1] * K_[4] + K_[5]);
        return V2d{u, v};
    }
    // include/keyframe.h:71-80 (level sizes: Pyramids()[level])
    bool IsInside(const double& u, const double& v, int level = 0) const {
        const GreyView& m = Pyramids()[level];
        return u >= 0 && u < m.cols && v >= 0 && v < m.rows;
    }
    bool IsInside(const V3d& point, int level = 0) const {
        const V2d uv = Project(point, level);
        return IsInside(uv[0], uv[1], level);
    }
    // include/keyframe.h:93-98: angle between the ray to Pw and the camera's z axis
    double ViewingAngle(const V3d& Pw) const {
        double Pc[3];
        for (int i = 0; i < 3; ++i)
            Pc[i] = (R_[3 * i] * Pw[0] + R_[3 * i + 1] * Pw[1]) + R_[3 * i + 2] * Pw[2] + T_[i];
        const double norm = std::sqrt(Pc[0] * Pc[0] + Pc[1] * Pc[1] + Pc[2] * Pc[2]);
        return std::acos(Pc[2] / norm);
    }
    // include/keyframe.h:100-108 (R row-major, K row-major 3x3)
    std::vector<KeyPoint>& Keypoints() { return keypoints_; }
    int AddKeypoint(const KeyPoint& kp) {
        keypoints_.push_back(kp);
        return (int)keypoints_.size();
    }
    M3d GetR() const { return R_; }
    V3d GetT() const { return T_; }
    void SetR(const M3d& R) { R_ = R; }
    void SetT(const V3d& T) { T_ = T; }
    M3d GetK() const { return K_; }
    void SetK(const M3d& K) { K_ = K; }

private:
    static constexpr double kScales[4] = {1.0, 0.5, 0.25, 0.125};  // include/keyframe.h:22
    void build_pyramid() const {
        // level 0 continuous for viso_pyramid, then levels 1..3 from the device
        std::vector<uint8_t> l0((size_t)w_ * h_);
        for (int y = 0; y < h_; ++y)
            std::copy(data_.begin() + (size_t)y * stride_, data_.begin() + (size_t)y * stride_ + w_,
                      l0.begin() + (size_t)y * w_);
        int32_t dims[8];
        size_t total = 0;
        check(viso_pyramid_dims(w_, h_, dims, &total), "viso_pyramid_dims");
        pyr_.resize(total);
        check(viso_pyramid(detail::pyramid_ctx(w_, h_), l0.data(), 1, w_, h_, pyr_.data()), "viso_pyramid");
        pyr_views_.clear();
        pyr_views_.push_back(Mat());
        size_t off = (size_t)dims[0] * dims[1];
        for (int l = 1; l < 4; ++l) {
            pyr_views_.push_back(GreyView{pyr_.data() + off, dims[2 * l], dims[2 * l + 1], (size_t)dims[2 * l]});
            off += (size_t)dims[2 * l] * dims[2 * l + 1];
        }
    }
    static inline long next_id_ = 0;
    long id_;
    int w_, h_;
    std::vector<uint8_t> data_;
    int stride_;
    M3d R_{1, 0, 0, 0, 1, 0, 0, 0, 1};  // include/keyframe.h:34-35
    V3d T_{0, 0, 0};
    M3d K_{0, 0, 0, 0, 0, 0, 0, 0, 1};
    std::vector<KeyPoint> keypoints_;
    mutable std::vector<uint8_t> pyr_;
    mutable std::vector<GreyView> pyr_views_;
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
    // viso.poses` -- and also keeps the call form `viso.poses()`.  size()
    // asks the library for the count only (no copy); indexing and iteration
    // read a host snapshot that is re-downloaded only when the count has
    // changed since it was taken (entries below the count are final once the
    // library reports them), so `for (i < poses.size()) poses[i]` costs one
    // download per new frame, not one per call.
    class PoseLog {
       public:
        explicit PoseLog(const Viso* v) : v_(v) {}
        PoseLog(const PoseLog&) = delete;
        PoseLog& operator=(const PoseLog&) = delete;
        std::vector<Pose> operator()() const { return v_->fetch_poses(); }
        operator std::vector<Pose>() const { return v_->fetch_poses(); }
        size_t size() const { return v_->num_poses(); }
        bool empty() const { return size() == 0; }
        const Pose& operator[](size_t i) const { return current()[i]; }
        std::vector<Pose>::const_iterator begin() const { return current().begin(); }
        // both iterators come from the same snapshot whichever is evaluated first
        std::vector<Pose>::const_iterator end() const { return current().end(); }

       private:
        const std::vector<Pose>& current() const {
            if (cache_.size() != v_->num_poses()) cache_ = v_->fetch_poses();
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

    size_t num_poses() const {
        size_t n = 0;
        check(viso_get_poses(ctx_, nullptr, 0, &n), "viso_get_poses");
        return n;
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
