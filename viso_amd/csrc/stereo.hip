// viso_amd — stereo stage of the north-star process(left, right) facade.
// No reference counterpart (the reference is monocular); the
// spec and its CPU restatement are the repo's own (oracle_stereo_match).
//
// For each left keypoint (x, y) the 8x8 patch (x-4..x+3, y-4..y+3, the
// reference's patch convention) is compared by SAD with the right image
// along the same row (rectified pair) for disparities d = 0..max_disp while
// x - d - 4 >= 0; the winner is the smallest SAD, ties -> smallest d.
// Keypoints whose left patch leaves the image get disparity -1.
//
// Mapping: one wave per keypoint, lane = candidate disparity (chunks of 64);
// the left patch is staged once in LDS (64 bytes), each lane streams its
// right patch from L1/L2; argmin by a packed (sad << 16 | d) wave min.
// Integer work: bit-exact.
#include "kernels.hpp"

namespace viso {

namespace {

__global__ __launch_bounds__(256) void stereo_sad_kernel(const uint8_t* __restrict__ L,
                                                         const uint8_t* __restrict__ R, int w,
                                                         int h, const int* __restrict__ xs,
                                                         const int* __restrict__ ys, int n,
                                                         int max_disp, int* __restrict__ disp,
                                                         int* __restrict__ best_sad) {
    __shared__ uint8_t s_patch[4][64];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + wave;
    if (i >= n) return;
    const int x = xs[i], y = ys[i];
    const bool ok = x - 4 >= 0 && x + 3 < w && y - 4 >= 0 && y + 3 < h;
    if (!ok) {
        if (lane == 0) {
            disp[i] = -1;
            best_sad[i] = -1;
        }
        return;
    }
    // left patch: lane p = (dx+4)*8 + (dy+4)
    {
        const int dx = (lane >> 3) - 4, dy = (lane & 7) - 4;
        s_patch[wave][lane] = L[(size_t)(y + dy) * w + (x + dx)];
    }
    __builtin_amdgcn_wave_barrier();
    const int dmax = min(max_disp, x - 4);
    unsigned long long best = ~0ULL;
    for (int d0 = 0; d0 <= dmax; d0 += 64) {
        const int d = d0 + lane;
        if (d <= dmax) {
            int sad = 0;
            for (int dx = -4; dx < 4; ++dx)
                for (int dy = -4; dy < 4; ++dy) {
                    const int l = s_patch[wave][(dx + 4) * 8 + (dy + 4)];
                    const int r = R[(size_t)(y + dy) * w + (x - d + dx)];
                    sad += abs(l - r);
                }
            const unsigned long long key = ((unsigned long long)sad << 32) | (unsigned)d;
            best = key < best ? key : best;
        }
    }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const unsigned long long o = __shfl_xor(best, off, 64);
        best = o < best ? o : best;
    }
    if (lane == 0) {
        disp[i] = (int)(best & 0xffffffffULL);
        best_sad[i] = (int)(best >> 32);
    }
}

}  // namespace

void launch_stereo_sad(const uint8_t* left, const uint8_t* right, int w, int h, const int* xs,
                       const int* ys, int n, int max_disp, int* disp, int* sad,
                       hipStream_t stream) {
    if (n <= 0) return;
    stereo_sad_kernel<<<(n + 3) / 4, 256, 0, stream>>>(left, right, w, h, xs, ys, n, max_disp,
                                                       disp, sad);
}

}  // namespace viso
