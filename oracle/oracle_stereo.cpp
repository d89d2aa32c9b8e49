// TEST INFRASTRUCTURE ONLY — CPU restatement of the repo's stereo SAD stage
// (viso_amd/csrc/stereo.hip).  North-star stage with no reference
// counterpart: "parity unpinned vs reference" (SURVEY.md §8a).
#include <cstdlib>

#include "viso_oracle.h"

extern "C" void oracle_stereo_match(const uint8_t* L, const uint8_t* R, int w, int h,
                                    const int32_t* xs, const int32_t* ys, int n, int max_disp,
                                    int32_t* disp, int32_t* best_sad) {
    for (int i = 0; i < n; ++i) {
        const int x = xs[i], y = ys[i];
        if (!(x - 4 >= 0 && x + 3 < w && y - 4 >= 0 && y + 3 < h)) {
            disp[i] = -1;
            best_sad[i] = -1;
            continue;
        }
        int bd = -1, bs = 0;
        const int dmax = max_disp < x - 4 ? max_disp : x - 4;
        for (int d = 0; d <= dmax; ++d) {
            int s = 0;
            for (int dx = -4; dx < 4; ++dx)
                for (int dy = -4; dy < 4; ++dy)
                    s += std::abs((int)L[(size_t)(y + dy) * w + x + dx] -
                                  (int)R[(size_t)(y + dy) * w + x - d + dx]);
            if (bd < 0 || s < bs) {
                bd = d;
                bs = s;
            }
        }
        disp[i] = bd;
        best_sad[i] = bs;
    }
}
