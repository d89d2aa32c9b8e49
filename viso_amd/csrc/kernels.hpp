// viso_amd — host-side launcher declarations (one translation unit per stage).
#pragma once

#include "common.hpp"

namespace viso {

// ---------------------------------------------------------------- image pass
// Builds levels 1..3 of n_images pyramids; image i's level-0 bytes live at
// base + i*img_stride (levels follow, PyrGeom offsets).
void launch_pyramid(const PyrGeom& g, uint8_t* base, int n_images, size_t img_stride,
                    hipStream_t stream);

struct FastScratch {
    int* row_count = nullptr;   // [h]
    int4* row_list = nullptr;   // [h * fast_row_cap(w)]
};
size_t fast_row_cap(int w);
// FAST + NMS on a level-0 image; writes up to cap keypoints (float2 and/or
// raw int4 {x, y, score, 0}) and the total count to *n_out (device).
void launch_fast(const uint8_t* img, int w, int h, int thresh, FastScratch& s, float2* kp_out,
                 int4* raw_out, int cap, int* n_out, hipStream_t stream);

}  // namespace viso
