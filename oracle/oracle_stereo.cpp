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

namespace {
int sad_at(const uint8_t* L, const uint8_t* R, int w, int x, int y, int d) {
    int s = 0;
    for (int dx = -4; dx < 4; ++dx)
        for (int dy = -4; dy < 4; ++dy)
            s += std::abs((int)L[(size_t)(y + dy) * w + x + dx] - (int)R[(size_t)(y + dy) * w + x - d + dx]);
    return s;
}
}  // namespace

// Stereo initialisation (the repo's own spec; viso_amd/csrc/stereo.hip
// stereo_points_kernel): the SAD winner d of each keypoint (as above), kept
// iff min_disp <= d < dmax (dmax = min(max_disp, x - 4)) so that both
// neighbours exist; parabola through SAD(d-1), SAD(d), SAD(d+1):
// dd = d + (s- - s+) / (2 (s- - 2 s0 + s+)) (the denominator is > 0: d is the
// unique-from-below minimum); Z = fx * base / dd, X = (x - cx) * Z / fx,
// Y = (y - cy) * Z / fy.  Points of the kept keypoints in keypoint order.
extern "C" int oracle_stereo_points(const uint8_t* L, const uint8_t* R, int w, int h,
                                    const int32_t* xs, const int32_t* ys, int n, int max_disp,
                                    int min_disp, const double K[4], double base, double* pts) {
    int m = 0;
    for (int i = 0; i < n; ++i) {
        int32_t d, s0;
        oracle_stereo_match(L, R, w, h, xs + i, ys + i, 1, max_disp, &d, &s0);
        const int x = xs[i], y = ys[i];
        const int dmax = max_disp < x - 4 ? max_disp : x - 4;
        if (d < 0 || d < min_disp || d < 1 || d >= dmax) continue;
        const int sm = sad_at(L, R, w, x, y, d - 1), sp = sad_at(L, R, w, x, y, d + 1);
        const int den = sm - 2 * s0 + sp;
        const double dd = (double)d + (double)(sm - sp) / (2.0 * (double)den);
        const double z = K[0] * base / dd;
        pts[3 * m] = ((double)x - K[2]) * z / K[0];
        pts[3 * m + 1] = ((double)y - K[3]) * z / K[1];
        pts[3 * m + 2] = z;
        ++m;
    }
    return m;
}
