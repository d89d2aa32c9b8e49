// Compile/link check of the C++ facade (include/viso/viso.hpp) against the
// C ABI; run with a GPU it processes a few synthetic frames.
#include <cstdio>
#include <vector>

#include "viso/viso.hpp"
#include "viso/viso_synth.h"

int main(int argc, char** argv) {
    if (argc < 2) {
        std::printf("facade ok (link only)\n");
        return 0;
    }
    viso_synth_params sp;
    viso_synth_default(&sp, 1242, 375);
    viso::VisualOdometryStereo vo(sp.fx, sp.fy, sp.cx, sp.cy, 1242, 375, 0, true);
    std::vector<uint8_t> l(1242 * 375), r(1242 * 375);
    const int32_t dims[3] = {1242, 375, 1242};
    for (int f = 0; f < 10; ++f) {
        viso_synth_render(&sp, f, 0, l.data(), 4);
        viso_synth_render(&sp, f, 1, r.data(), 4);
        if (!vo.process(l.data(), r.data(), dims)) return 1;
    }
    std::printf("state %d points %zu poses %zu\n", vo.state(), vo.GetPoints().size(), vo.poses().size());
    return vo.poses().empty() ? 1 : 0;
}
