// Compile/link check of the C++ facades (include/viso/viso.hpp, viso_svo.hpp,
// viso_rig.hpp) against the C ABI; with a GPU (any argument) it runs a few
// synthetic frames through each engine.
#include <cmath>
#include <cstdio>
#include <vector>

#include "viso/viso.hpp"
#include "viso/viso_rig.hpp"
#include "viso/viso_svo.hpp"
#include "viso/viso_synth.h"

// A FrameHandler written against the reference's Keyframe accessors
// (include/keyframe.h:50-112): it samples every frame the way Viso's loops do.
struct SamplingHandler : viso::FrameSequence::FrameHandler {
    double acc = 0.0;
    void OnNewFrame(viso::Keyframe::Ptr kf) override {
        kf->SetK({718.856, 0, 607.19, 0, 718.856, 185.22, 0, 0, 1});
        const viso::V3d P{1.0, -0.5, 12.0};
        for (int level = 0; level < 4; ++level) {
            if (!kf->IsInside(P, level)) continue;
            const viso::V2d uv = kf->Project(P, level);
            const viso::V2d g = kf->GetGradient(uv[0], uv[1], level);
            acc += kf->GetPixelValue(uv[0], uv[1], level) + g[0] + g[1] + kf->GetScale(level);
        }
        acc += kf->ViewingAngle(P) + (double)kf->Mat().cols + (double)kf->Pyramids().size();
    }
};

// Keyframe accessors on frame 0 -> `path`: the four pyramid levels (as
// Pyramids() returns them), then per sample (x, y, level): GetPixelValue,
// GetGradient (2) -- compared with the oracle by tests/test_stereo_abi.py.
static int dump_keyframe(const uint8_t* img, int W, int H, const char* path) {
    viso::Keyframe kf(img, W, H, W);
    const auto& pyr = kf.Pyramids();
    if (pyr.size() != 4 || kf.Mat().data != kf.Data()) return 1;
    std::FILE* f = std::fopen(path, "wb");
    if (!f) return 1;
    for (const auto& m : pyr) std::fwrite(m.data, 1, m.step * m.rows, f);
    const double xs[5] = {10.25, 100.5, 333.75, 64.0, 140.125};
    const double ys[5] = {7.5, 40.25, 20.0, 80.75, 30.5};
    for (int level = 0; level < 4; ++level)
        for (int k = 0; k < 5; ++k) {
            const double s = kf.GetScale(level);
            const double x = xs[k] * s * 2.0, y = ys[k] * s * 2.0;
            const viso::V2d g = kf.GetGradient(x, y, level);
            const double v[3] = {kf.GetPixelValue(x, y, level), g[0], g[1]};
            std::fwrite(v, sizeof(double), 3, f);
        }
    // Project / IsInside / ViewingAngle with a pose and K (include/keyframe.h:82-98)
    kf.SetR({0.8, -0.6, 0, 0.6, 0.8, 0, 0, 0, 1});
    kf.SetT({0.1, -0.2, 0.3});
    kf.SetK({718.856, 0, 607.19, 0, 718.856, 185.22, 0, 0, 1});
    const viso::V3d P{1.0, -0.5, 12.0};
    for (int level = 0; level < 4; ++level) {
        const viso::V2d uv = kf.Project(P, level);
        const double v[3] = {uv[0], uv[1], kf.IsInside(P, level) ? 1.0 : 0.0};
        std::fwrite(v, sizeof(double), 3, f);
    }
    const double va = kf.ViewingAngle(P);
    std::fwrite(&va, sizeof(double), 1, f);
    std::fclose(f);
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::printf("facade ok (link only)\n");
        return 0;
    }
    const int W = 1242, H = 375;
    viso_synth_params sp;
    viso_synth_default(&sp, W, H);
    std::vector<uint8_t> l(W * H), r(W * H);
    const int32_t dims[3] = {W, H, W};
    viso_synth_render(&sp, 0, 0, l.data(), 4);
    if (argc > 2 && dump_keyframe(l.data(), W, H, argv[2])) return 1;
    {
        // the reference's plugin shape: FrameSequence -> FrameHandler(Keyframe::Ptr)
        SamplingHandler h;
        viso::FrameSequence seq("frame", &h, [&](const std::string&, std::vector<uint8_t>* g, int* w, int* hh) {
            *g = l;
            *w = W;
            *hh = H;
            return true;
        });
        seq.RunOnce();
        if (!(h.acc == h.acc) || h.acc == 0.0) return 1;
        std::printf("handler: %.6f\n", h.acc);
    }
    // the reference path, stereo-initialised
    viso::StereoViso vo(sp.fx, sp.fy, sp.cx, sp.cy, W, H, 0, true);
    vo.SetStereo(sp.baseline);
    // the north-star stereo VO
    viso::VisualOdometryStereo svo(W, H, sp.fx, sp.fy, sp.cx, sp.cy, sp.baseline);
    int svo_ok = 0;
    for (int f = 0; f < 6; ++f) {
        viso_synth_render(&sp, f, 0, l.data(), 4);
        viso_synth_render(&sp, f, 1, r.data(), 4);
        if (!vo.process(l.data(), r.data(), dims)) return 1;
        svo_ok += svo.process(l.data(), r.data(), dims) ? 1 : 0;
    }
    std::printf("viso: state %d points %zu poses %zu\n", vo.state(), vo.GetPoints().size(), vo.poses().size());
    // the reference's field form (src/main.cpp:50, :75): viso.poses, iterated
    {
        const std::vector<viso::Pose>& log = vo.poses;
        size_t n = 0;
        for (const auto& Tcw : vo.poses) n += (Tcw[0] == Tcw[0]) ? 1 : 0;
        if (n != log.size() || vo.poses.size() != log.size() || (n && vo.poses[n - 1] != log[n - 1])) return 1;
    }
    std::printf("svo: ok %d poses %zu matches %zu\n", svo_ok, svo.poses().size(), svo.getMatches().size());
    // the photometric rig, 2 cameras
    const int nc = 2;
    double E[2 * 12];
    for (int c = 0; c < nc; ++c) viso_synth_rig_extrinsic(c, nc, E + 12 * c);
    viso_params p;
    viso::check(viso_default_params(&p, sp.fx, sp.fy, sp.cx, sp.cy, W, H), "viso_default_params");
    viso::VisoRig rig(p, nc, E);
    rig.SetStereo(sp.baseline);
    std::vector<uint8_t> ls(nc * W * H), rs(nc * W * H);
    for (int f = 0; f < 3; ++f) {
        const uint8_t* L[2];
        const uint8_t* R[2];
        for (int c = 0; c < nc; ++c) {
            viso_synth_rig_render(&sp, f, nc, c, 0, ls.data() + c * W * H, 4);
            viso_synth_rig_render(&sp, f, nc, c, 1, rs.data() + c * W * H, 4);
            L[c] = ls.data() + c * W * H;
            R[c] = rs.data() + c * W * H;
        }
        rig.process(L, R, dims);
    }
    std::printf("rig: state %d poses %zu\n", rig.state(), rig.poses().size());
    return (vo.poses().empty() || svo_ok < 4 || rig.poses().size() != 2) ? 1 : 0;
}
