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

// Stereo initialisation points (the repo's own spec, restated in
// oracle/oracle_stereo.cpp oracle_stereo_points): wave per FAST keypoint,
// lane = candidate disparity; the winner's two neighbours SAD(d-1), SAD(d+1)
// by a lane-per-pixel pass; sub-pixel parabola, metric depth, camera point.
// Writes flag[i] (1 = kept) and pts[i] (3 doubles) per keypoint.
__device__ inline int wave_sum_i(int v) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) v += __shfl_xor(v, off, 64);
    return v;
}

__global__ __launch_bounds__(256) void stereo_points_kernel(const uint8_t* __restrict__ L,
                                                            const uint8_t* __restrict__ R, int w, int h,
                                                            const float2* __restrict__ kp, int n,
                                                            int max_disp, int min_disp, StereoCam cam,
                                                            int* __restrict__ flag,
                                                            double* __restrict__ pts) {
    __shared__ uint8_t s_patch[4][64];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + wave;
    if (i >= n) return;
    const int x = (int)kp[i].x, y = (int)kp[i].y;
    const int dmax = min(max_disp, x - 4);
    const bool ok = x - 4 >= 0 && x + 3 < w && y - 4 >= 0 && y + 3 < h && dmax >= 2;
    if (!ok) {
        if (lane == 0) flag[i] = 0;
        return;
    }
    const int pdx = (lane >> 3) - 4, pdy = (lane & 7) - 4;
    const int lpx = L[(size_t)(y + pdy) * w + (x + pdx)];
    s_patch[wave][lane] = (uint8_t)lpx;
    __builtin_amdgcn_wave_barrier();
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
    const int d = (int)(best & 0xffffffffULL), s0 = (int)(best >> 32);
    const bool keep = d >= min_disp && d >= 1 && d < dmax;
    if (!keep) {
        if (lane == 0) flag[i] = 0;
        return;
    }
    // neighbours: lane = patch pixel (d - 1 and d + 1 stay inside 0..dmax)
    const size_t ro = (size_t)(y + pdy) * w + (x + pdx);
    const int sm = wave_sum_i(abs(lpx - (int)R[ro - (d - 1)]));
    const int sp = wave_sum_i(abs(lpx - (int)R[ro - (d + 1)]));
    if (lane == 0) {
        const int den = sm - 2 * s0 + sp;
        const double dd = (double)d + (double)(sm - sp) / (2.0 * (double)den);
        const double z = cam.fx * cam.base / dd;
        pts[3 * (size_t)i] = ((double)x - cam.cx) * z / cam.fx;
        pts[3 * (size_t)i + 1] = ((double)y - cam.cy) * z / cam.fy;
        pts[3 * (size_t)i + 2] = z;
        flag[i] = 1;
    }
}

// Ordered compaction of the kept points (one workgroup of 1024 threads):
// out[j] = pts of the j-th kept keypoint, j < cap; *count = number kept
// (uncapped).
__global__ __launch_bounds__(1024) void stereo_compact_kernel(const int* __restrict__ flag,
                                                              const double* __restrict__ pts, int n,
                                                              double* __restrict__ out, int cap,
                                                              int* __restrict__ count) {
    __shared__ int s_w[16];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int base = 0;
    for (int i0 = 0; i0 < n; i0 += 1024) {
        const int i = i0 + tid;
        const int f = i < n ? flag[i] : 0;
        int incl = f;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(incl, o, 64);
            if (lane >= o) incl += t;
        }
        if (lane == 63) s_w[wave] = incl;
        __syncthreads();
        int wb = 0, tot = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int t = s_w[k];
            wb += k < wave ? t : 0;
            tot += t;
        }
        __syncthreads();
        const int j = base + wb + incl - f;
        if (f && j < cap) {
            out[3 * (size_t)j] = pts[3 * (size_t)i];
            out[3 * (size_t)j + 1] = pts[3 * (size_t)i + 1];
            out[3 * (size_t)j + 2] = pts[3 * (size_t)i + 2];
        }
        base += tot;
    }
    if (tid == 0) *count = base;
}

// Stereo keyframe insertion: camera-frame points -> world, Pw = R^T (Pc - T)
// with the keyframe's Tcw pose (oracle_viso.cpp restates the same order).
__global__ __launch_bounds__(256) void points_to_world_kernel(double* __restrict__ pts, int n,
                                                              const double* __restrict__ pose) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const double d0 = pts[3 * (size_t)i] - pose[9], d1 = pts[3 * (size_t)i + 1] - pose[10],
                 d2 = pts[3 * (size_t)i + 2] - pose[11];
#pragma unroll
    for (int k = 0; k < 3; ++k) pts[3 * (size_t)i + k] = (pose[k] * d0 + pose[3 + k] * d1) + pose[6 + k] * d2;
}

}  // namespace

void launch_points_to_world(double* pts, int n, const double* pose12, hipStream_t stream) {
    if (n > 0) points_to_world_kernel<<<(n + 255) / 256, 256, 0, stream>>>(pts, n, pose12);
}

void launch_stereo_points(const uint8_t* left, const uint8_t* right, int w, int h, const float2* kp,
                          int n, int max_disp, int min_disp, const StereoCam& cam, int* flag,
                          double* pts, double* out, int cap, int* count, hipStream_t stream) {
    if (n > 0)
        stereo_points_kernel<<<(n + 3) / 4, 256, 0, stream>>>(left, right, w, h, kp, n, max_disp,
                                                              min_disp, cam, flag, pts);
    stereo_compact_kernel<<<1, 1024, 0, stream>>>(flag, pts, n, out, cap, count);
}

void launch_stereo_sad(const uint8_t* left, const uint8_t* right, int w, int h, const int* xs,
                       const int* ys, int n, int max_disp, int* disp, int* sad,
                       hipStream_t stream) {
    if (n <= 0) return;
    stereo_sad_kernel<<<(n + 3) / 4, 256, 0, stream>>>(left, right, w, h, xs, ys, n, max_disp,
                                                       disp, sad);
}

}  // namespace viso
