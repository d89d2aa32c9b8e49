// TEST INFRASTRUCTURE ONLY — shared helpers of the CPU oracle (see viso_oracle.h).
#ifndef VISO_ORACLE_COMMON_HPP
#define VISO_ORACLE_COMMON_HPP

#include <cmath>
#include <cstddef>
#include <cstdint>
#include <memory>
#include <vector>

namespace oracle {

constexpr int kLevels = 4;
constexpr double kScales[kLevels] = {1.0, 0.5, 0.25, 0.125};  // include/keyframe.h:22
constexpr int kHalfPatch = 4;                                  // include/viso.h:25

struct PyrView {
    const uint8_t* base;
    int w[kLevels], h[kLevels];
    size_t off[kLevels];
    const uint8_t* level(int l) const { return base + off[l]; }
};

inline void pyramid_dims(int w, int h, int* ws, int* hs, size_t* offs) {
    size_t off = 0;
    for (int l = 0; l < kLevels; ++l) {
        if (l > 0) {
            // cv::Size(cols * 0.5, rows * 0.5): double -> int truncation (keyframe.h:43)
            w = (int)(w * 0.5);
            h = (int)(h * 0.5);
        }
        ws[l] = w;
        hs[l] = h;
        offs[l] = off;
        off += (size_t)w * (size_t)h;
    }
}

inline PyrView make_view(const uint8_t* base, int w, int h) {
    PyrView v;
    v.base = base;
    pyramid_dims(w, h, v.w, v.h, v.off);
    return v;
}

// Canonical pairwise tree sum over n leaves padded with +0.0 to a power of two.
inline double tree_sum(const double* v, int n) {
    if (n <= 0) return 0.0;
    int p = 1;
    while (p < n) p <<= 1;
    // small trees (the 64-pixel patch sums, map tiles) on the stack: the
    // CPU baseline times this restatement, so it must not be dominated by
    // allocations the reference's running sums never make
    double stack[256];
    std::vector<double> heap;
    double* t = stack;
    if (p > 256) {
        heap.assign((size_t)p, 0.0);
        t = heap.data();
    }
    for (int i = 0; i < n; ++i) t[i] = v[i];
    for (int i = n; i < p; ++i) t[i] = 0.0;
    for (int s = 1; s < p; s <<= 1)
        for (int i = 0; i < p; i += 2 * s) t[i] = t[i] + t[i + s];
    return t[0];
}

// The direct pose's 64-pixel patch sums (round 3): the pairwise tree with
// the levels in descending stride order (p + 32 first, then + 16, ... + 1),
// the device's reduce_scatter_28_desc.
inline double tree_sum_desc64(const double* v) {
    double t[64];
    for (int i = 0; i < 64; ++i) t[i] = v[i];
    for (int s = 32; s >= 1; s >>= 1)
        for (int i = 0; i < s; ++i) t[i] = t[i] + t[i + s];
    return t[0];
}

// Canonical order of a sum over MAP POINTS (the direct pose's 28 sums and
// the rig's per-camera sums): points in tiles of T = min(64, max(1,
// ceil(n / groups))) consecutive points, each tile a pairwise tree
// (tree_sum over its count), then the pairwise tree over the ceil(n / T)
// tile sums.  The device gives one workgroup per tile (groups = 256 for the
// direct pose: one tile per CU; 256 / pow2(n_cams) per rig camera), so the
// order is independent of the launch but fills the chip; pairwise trees
// with zero padding make the device's 64-lane and 256-lane trees equal to
// these.
inline int map_tile(int n, int groups) {
    int t = (n + groups - 1) / groups;
    if (t < 1) t = 1;
    if (t > 64) t = 64;
    return t;
}

// the two-level sum over tiles of T points (the last tile ragged)
inline double map_tree_sum_tiles(const double* v, int n, int T) {
    if (n <= 0) return 0.0;
    const int nt = (n + T - 1) / T;
    std::vector<double> heap;
    double stack[256];
    double* tiles = stack;
    if (nt > 256) {
        heap.resize((size_t)nt);
        tiles = heap.data();
    }
    for (int t = 0; t < nt; ++t) {
        const int c = (t + 1) * T <= n ? T : n - t * T;
        tiles[t] = tree_sum(v + (size_t)t * T, c);
    }
    return tree_sum(tiles, nt);
}

inline double map_tree_sum(const double* v, int n, int groups) {
    return n <= 0 ? 0.0 : map_tree_sum_tiles(v, n, map_tile(n, groups));
}

// Summation order switch (oracle_set_sum_order, viso_oracle.h).  0: the
// canonical pairwise tree the device reproduces bit for bit; 1: "literal",
// the reference's own running sums in loop order (H += ..., b += ...,
// cost += ... at src/viso.cpp:308-310, 727-729, 888-890; disparity and mean
// depth at :199-201, :622-625).  Literal mode exists to measure the drift the
// tree substitution causes (tests/test_literal_drift.py); the GPU is checked
// against the tree mode.
inline int& sum_literal() {
    thread_local int mode = 0;  // per calling thread
    return mode;
}

// Running sum in index order, starting from 0 (Eigen's Zero() then +=).
// The reference's cost model, for the copies-included CPU baseline (SURVEY.md
// §8(d); bench.py cpu_baseline_faithful).  Map::GetPoints() and
// Map::Keyframes() return std::vector<shared_ptr> BY VALUE (include/map.h:
// 18-19), and the reference calls them inside its loops: the loop condition
// `i < map_.GetPoints().size()` and `map_.GetPoints()[i]` per point in
// DirectPoseEstimationSingleLayer (src/viso.cpp:688,690) and LKAlignment
// (:774,776), `auto keyframes = map_.Keyframes()` per point in LKAlignment
// (:787) — O(N^2) shared_ptr copies per pass.  With ref_copies().on the
// oracle makes the same copies of a mirror of the map (the arithmetic is
// untouched; off by default).
struct RefCopies {
    bool on = false;
    std::vector<std::shared_ptr<const int>> pts, kfs;
};
inline RefCopies& ref_copies() {
    static RefCopies r;
    return r;
}
inline void ref_sink(size_t v) {
    static volatile size_t s;
    s = s + v;
}
inline std::vector<std::shared_ptr<const int>> ref_mirror(std::vector<std::shared_ptr<const int>>& m, int n) {
    while ((int)m.size() < n) m.push_back(std::make_shared<const int>((int)m.size()));
    if ((int)m.size() > n) m.resize((size_t)n);
    return m;  // by value, as Map::GetPoints() / Keyframes()
}
// `i < map_.GetPoints().size()`
inline void ref_points_cond(int n) {
    if (ref_copies().on) ref_sink(ref_mirror(ref_copies().pts, n).size());
}
// `map_.GetPoints()[i]`
inline void ref_points_at(int n, int i) {
    if (ref_copies().on) ref_sink((size_t)*ref_mirror(ref_copies().pts, n)[(size_t)i]);
}
// `auto keyframes = map_.Keyframes()`
inline void ref_keyframes(int nk) {
    if (ref_copies().on) ref_sink(ref_mirror(ref_copies().kfs, nk).size());
}

inline double running_sum(const double* v, int n) {
    double s = 0.0;
    for (int i = 0; i < n; ++i) s = s + v[i];
    return s;
}

// The sum of n per-item terms in the active order (tree or literal).
inline double acc_sum(const double* v, int n) {
    return sum_literal() ? running_sum(v, n) : tree_sum(v, n);
}

// The same for a 64-pixel patch summed by the descending-stride tree (LK
// alignment's per-iteration sums, round 3).
inline double acc_sum_desc64(const double* v) {
    return sum_literal() ? running_sum(v, 64) : tree_sum_desc64(v);
}

// GetPixelValue (include/common.h:35-42, include/keyframe.h:50-57).  Base
// pointer uses int() truncation, weights use x - floor(x).  Taps outside the
// continuous level buffer read 0 (reference: reads outside the cv::Mat).
inline double sample(const uint8_t* img, int w, int h, double x, double y) {
    long long base;
    bool finite = (x > -1e9 && x < 1e9 && y > -1e9 && y < 1e9);
    long long n = (long long)w * (long long)h;
    if (finite)
        base = (long long)(int)y * (long long)w + (long long)(int)x;
    else
        base = -(1LL << 40);
    auto tap = [&](long long idx) -> double {
        return (idx >= 0 && idx < n) ? (double)img[idx] : 0.0;
    };
    double xx = x - std::floor(x);
    double yy = y - std::floor(y);
    double d0 = tap(base), d1 = tap(base + 1), d2 = tap(base + w), d3 = tap(base + w + 1);
    return double((1 - xx) * (1 - yy) * d0 + xx * (1 - yy) * d1 + (1 - xx) * yy * d2 +
                  xx * yy * d3);
}

inline void gradient(const uint8_t* img, int w, int h, double u, double v, double& gx,
                     double& gy) {
    // include/common.h:44-49
    gx = 0.5 * (sample(img, w, h, u + 1, v) - sample(img, w, h, u - 1, v));
    gy = 0.5 * (sample(img, w, h, u, v + 1) - sample(img, w, h, u, v - 1));
}

// Pose as (R row-major, t).  Tcw convention: Pc = R * Pw + t (keyframe.h:84).
struct Pose {
    double R[9];
    double t[3];
};

inline void mat3_vec(const double* R, const double* p, double* out) {
    // Eigen coefficient order: (R(i,0)*p0 + R(i,1)*p1) + R(i,2)*p2
    for (int i = 0; i < 3; ++i) out[i] = R[3 * i + 0] * p[0] + R[3 * i + 1] * p[1] + R[3 * i + 2] * p[2];
}

// Keyframe::Project (include/keyframe.h:82-89)
inline void project(const Pose& T, const double K[4], const double* P, int level, double& u,
                    double& v) {
    double uv1[3];
    mat3_vec(T.R, P, uv1);
    uv1[0] = uv1[0] + T.t[0];
    uv1[1] = uv1[1] + T.t[1];
    uv1[2] = uv1[2] + T.t[2];
    double z = uv1[2];
    uv1[0] = uv1[0] / z;
    uv1[1] = uv1[1] / z;
    u = kScales[level] * (uv1[0] * K[0] + K[2]);
    v = kScales[level] * (uv1[1] * K[1] + K[3]);
}

// Keyframe::IsInside(u, v, level) (include/keyframe.h:77-80)
inline bool is_inside(double u, double v, int w, int h) {
    return u >= 0 && u < w && v >= 0 && v < h;
}

// counter-based RNG used by the RANSAC samplers (identical on the device)
inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

}  // namespace oracle

#endif
