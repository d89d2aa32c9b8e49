// Compile/link check of the C++ facades (include/viso/viso.hpp, viso_svo.hpp,
// viso_rig.hpp) against the C ABI; with a GPU (any argument) it runs a few
// synthetic frames through each engine.
#include <cstdio>
#include <vector>

#include "viso/viso.hpp"
#include "viso/viso_rig.hpp"
#include "viso/viso_svo.hpp"
#include "viso/viso_synth.h"

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
