// TEST INFRASTRUCTURE ONLY (see viso_oracle.h) — a driver for the
// AddressSanitizer / UndefinedBehaviorSanitizer build of the oracle
// (`make -C oracle sanitize`, run by tests/test_oracle_sanitize.py).
//
// The reference has two undefined behaviours on its hot path that the
// oracle restates as defined ones: the uninitialised
// `init_.frame_cnt` (include/viso.h:38; the oracle starts it at 0) and the
// unguarded `data[step + 1]` bilinear taps past the cv::Mat
// (include/common.h:35-41; the oracle reads 0 outside the level buffer).
// This driver runs every oracle path over a procedural scene whose camera
// drifts to the image border (so patches and taps leave the buffer) with the
// sanitizers armed: the monocular initialisation (FAST, KLT, 2D-2D RANSAC,
// SelectMotion), stereo initialisation and tracking (direct pose, LK
// alignment, keyframe insertion) in both summation orders, and the
// multi-camera rig.  Exit status 0 and no sanitizer report = clean.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "viso_oracle.h"

namespace {

constexpr int W = 320, H = 160;

// block-noise texture (8 px blocks) sampled bilinearly at a sub-pixel shift
struct Texture {
    int tw = 1024, th = 512;
    std::vector<uint8_t> t;
    Texture() : t((size_t)tw * th) {
        uint64_t s = 0x9E3779B97F4A7C15ULL;
        std::vector<uint8_t> blocks((size_t)(tw / 8) * (th / 8));
        for (auto& b : blocks) {
            s ^= s << 13;
            s ^= s >> 7;
            s ^= s << 17;
            b = (uint8_t)(s >> 56);
        }
        for (int y = 0; y < th; ++y)
            for (int x = 0; x < tw; ++x) t[(size_t)y * tw + x] = blocks[(size_t)(y / 8) * (tw / 8) + x / 8];
    }
    uint8_t at(double x, double y) const {
        const int ix = (int)std::floor(x), iy = (int)std::floor(y);
        const double fx = x - ix, fy = y - iy;
        auto p = [&](int a, int b) {
            a = std::min(std::max(a, 0), tw - 1);
            b = std::min(std::max(b, 0), th - 1);
            return (double)t[(size_t)b * tw + a];
        };
        const double v = (1 - fx) * (1 - fy) * p(ix, iy) + fx * (1 - fy) * p(ix + 1, iy) +
                         (1 - fx) * fy * p(ix, iy + 1) + fx * fy * p(ix + 1, iy + 1);
        return (uint8_t)std::lround(v);
    }
};

void render(const Texture& tex, double ox, double oy, double zoom, std::vector<uint8_t>& img) {
    img.resize((size_t)W * H);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) img[(size_t)y * W + x] = tex.at(ox + x * zoom, oy + y * zoom);
}

int run_viso(const Texture& tex, bool stereo, int literal) {
    oracle_set_sum_order(literal);
    oracle_params p;
    oracle_default_params(&p, 300.0, 300.0, W / 2.0, H / 2.0, W, H);
    p.enable_tracking = 1;
    oracle_viso* v = oracle_viso_create(&p);
    if (!v) return 1;
    if (stereo) {
        oracle_viso_set_stereo(v, 0.5, 64, 1);
        oracle_viso_set_keyframes(v, 2, 900);
    }
    std::vector<uint8_t> L, R;
    for (int f = 0; f < 10; ++f) {
        // the view drifts right and zooms in (forward motion), leaving the map
        const double ox = 40 + 9.0 * f, oy = 30 + 1.5 * f, zoom = 0.77 - 0.01 * f;
        render(tex, ox, oy, zoom, L);
        if (stereo) {
            render(tex, ox + 12.0, oy, zoom, R);
            oracle_viso_on_new_stereo(v, L.data(), R.data());
        } else {
            oracle_viso_on_new_frame(v, L.data());
        }
    }
    std::printf("%s%s: state %d, poses %d, points %d\n", stereo ? "stereo" : "mono", literal ? " (literal)" : "",
                oracle_viso_state(v), oracle_viso_num_poses(v), oracle_viso_num_points(v));
    oracle_viso_destroy(v);
    oracle_set_sum_order(0);
    return 0;
}

int run_rig(const Texture& tex) {
    const double E[24] = {1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0,
                          0.9848077530, 0, -0.1736481777, 0, 1, 0, 0.1736481777, 0, 0.9848077530, -0.2, 0, 0};
    const double K[4] = {300.0, 300.0, W / 2.0, H / 2.0};
    oracle_rig* r = oracle_rig_create(2, W, H, K, 50, E, 0.5, 64, 1);
    if (!r) return 1;
    std::vector<uint8_t> L0, L1, R0, R1;
    for (int f = 0; f < 4; ++f) {
        render(tex, 40 + 3.0 * f, 30, 0.77, L0);
        render(tex, 400 + 3.0 * f, 60, 0.77, L1);
        render(tex, 52 + 3.0 * f, 30, 0.77, R0);
        render(tex, 412 + 3.0 * f, 60, 0.77, R1);
        const uint8_t* ls[2] = {L0.data(), L1.data()};
        const uint8_t* rs[2] = {R0.data(), R1.data()};
        oracle_rig_process(r, ls, f == 0 ? rs : nullptr);
    }
    std::printf("rig: state %d, poses %d, points %d + %d\n", oracle_rig_state(r), oracle_rig_num_poses(r),
                oracle_rig_num_points(r, 0), oracle_rig_num_points(r, 1));
    oracle_rig_destroy(r);
    return 0;
}

}  // namespace

int main() {
    Texture tex;
    int rc = 0;
    rc |= run_viso(tex, false, 0);
    rc |= run_viso(tex, true, 0);
    rc |= run_viso(tex, true, 1);
    rc |= run_rig(tex);
    std::printf(rc ? "FAILED\n" : "sancheck ok\n");
    return rc;
}
