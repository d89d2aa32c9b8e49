// viso_amd — direct photometric 6-DoF Gauss-Newton pose for gfx950
// (DirectPoseEstimationSingleLayer / MultiLayer + dPixeldXi,
// src/viso.cpp:640-766).
//
// One level = two launches:
//  1. direct_tiles_kernel: one wave per map point, lane = patch pixel.  The
//     wave forms J = -grad^T * dPixel/dXi for its 64 pixels and reduces the
//     28 sums (21 upper-triangle J J^T, 6 -e J, e^2) with the canonical DPP
//     wave tree; a workgroup's 4 points form one tile, (p0 + p1) + (p2 + p3).
//  2. direct_solve_kernel (one workgroup): canonical tree over the tiles
//     (independent coalesced loads, k-major layout), then on one lane:
//     H^-1 (PartialPivLU), SE3::exp(update) * T21, cost / nGood and the
//     NaN / cost-increase / relative-decrease checks of :741-753.
// The sum order is the canonical pairwise tree over (point, pixel), so the
// result is independent of the launch geometry and equal to the oracle's.
// As shipped the loop takes exactly one GN step per level (cost is never
// reset, src/viso.cpp:673); the rare continuation (a level
// whose photometric cost is exactly 0) is executed faithfully by the solve
// workgroup itself, re-running the tiles.
// Frame-level fusions: level 3 seeds T21 = SE3(last R, last t)
// (src/viso.cpp:114) inside both kernels; level 0's solve writes
// cur_frame R,t and appends the pose log (src/viso.cpp:117-118, 137).
#include "device_math.hpp"
#include "kernels.hpp"

namespace viso {

namespace {

constexpr int kSums = 28;
constexpr int kTile = 4;           // points per tile = waves per workgroup
constexpr int kMaxTiles = 4096;    // kMaxMapPoints / kTile
constexpr int kChunk = kMaxTiles / 256;

struct DirectArgs {
    FrameDev last;
    FrameDev cur;
    PyrDev g;
    Intrinsics K;
    const double* points;
    int n;
    const double* pose_last;
    double* se3;  // 7 doubles in/out
    int seed_from_last;
    int level;
    int n_tiles;
    int tile_stride;  // k-major layout: tile_part[k * tile_stride + tile]
    double* tile_part;
    int* tile_good;
    double* stats;
    double* pose_out;  // level 0: cur pose (12)
    double* log;
    int* log_count;
};

// dPixeldXi (src/viso.cpp:640-658)
__device__ inline void d_pixel_d_xi(const Intrinsics& K, const double* pose, const double* P,
                                    double scale, double* J) {
    double Pc[3];
    mat3_vec(pose, P, Pc);
    Pc[0] = Pc[0] + pose[9];
    Pc[1] = Pc[1] + pose[10];
    Pc[2] = Pc[2] + pose[11];
    const double x = Pc[0], y = Pc[1], z = Pc[2];
    const double fx = K.fx * scale, fy = K.fy * scale;
    const double zz = z * z, xy = x * y;
    J[0] = fx / z;
    J[1] = 0;
    J[2] = -fx * x / zz;
    J[3] = -fx * xy / zz;
    J[4] = fx + fx * x * x / zz;
    J[5] = -fx * y / z;
    J[6] = 0;
    J[7] = fy / z;
    J[8] = -fy * y / zz;
    J[9] = -fy - fy * y * y / zz;
    J[10] = fy * xy / zz;
    J[11] = fy * x / z;
}

// The 28 sums of one map point (wave-wide; identical in every lane).
__device__ inline bool direct_point(const DirectArgs& a, const double* cur_pose, int i,
                                    double* s) {
    const int lane = threadIdx.x & 63;
    const int px = (lane >> 3) - 4, py = (lane & 7) - 4;
    const int l = a.level;
    const double scale = kScale[l];
    const int w = a.g.w[l], h = a.g.h[l];
    const double P[3] = {a.points[3 * i], a.points[3 * i + 1], a.points[3 * i + 2]};
    double ur, vr, uc, vc;
    project_px(a.pose_last, a.K, P, scale, ur, vr);
    project_px(cur_pose, a.K, P, scale, uc, vc);
    const double hp = 4.0;
    const bool good = inside_px(ur - hp, vr - hp, w, h) && inside_px(ur + hp, vr + hp, w, h) &&
                      inside_px(uc - hp, vc - hp, w, h) && inside_px(uc + hp, vc + hp, w, h);
    if (!good) return false;
    double Jp[12];
    d_pixel_d_xi(a.K, cur_pose, P, scale, Jp);
    const uint8_t* L = a.last.l[l];
    const uint8_t* C = a.cur.l[l];
    const double error = sample_px(L, w, h, ur + px, vr + py) - sample_px(C, w, h, uc + px, vc + py);
    double g0, g1;
    gradient_px(C, w, h, uc + px, vc + py, g0, g1);
    double J[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) J[k] = -g0 * Jp[k] + -g1 * Jp[6 + k];
    int idx = 0;
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int c = r; c < 6; ++c) s[idx++] = wave_tree_sum_dpp(J[r] * J[c]);
#pragma unroll
    for (int k = 0; k < 6; ++k) s[21 + k] = wave_tree_sum_dpp(-error * J[k]);
    s[27] = wave_tree_sum_dpp(error * error);
    return true;
}

// T21 at the start of this launch: the running state, or SE3(R, t) of the
// last frame's pose for the first level (Sophus::SE3d(R, t): R -> quaternion)
__device__ inline void start_state(const DirectArgs& a, double* st) {
    if (a.seed_from_last) {
        double q[4];
        quat_from_matrix(a.pose_last, q);
        for (int k = 0; k < 4; ++k) st[k] = q[k];
        st[4] = a.pose_last[9];
        st[5] = a.pose_last[10];
        st[6] = a.pose_last[11];
    } else {
        for (int k = 0; k < 7; ++k) st[k] = a.se3[k];
    }
}

__device__ inline void state_to_pose(const double* st, double* pose) {
    double q[4] = {st[0], st[1], st[2], st[3]};
    quat_to_matrix(q, pose);
    pose[9] = st[4];
    pose[10] = st[5];
    pose[11] = st[6];
}

// Tile b (kTile points): 28 sums -> tile_part (k-major), good count -> tile_good.
// Called by a whole 256-thread workgroup.
__device__ void direct_tile(const DirectArgs& a, const double* cur_pose, int b, double* s_pts,
                            int* s_good4) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int i = b * kTile + wave;
    double s[kSums];
    bool good = false;
    if (i < a.n) good = direct_point(a, cur_pose, i, s);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < kSums; ++k) s_pts[wave * kSums + k] = good ? s[k] : 0.0;
        s_good4[wave] = good ? 1 : 0;
    }
    __syncthreads();
    if (threadIdx.x < kSums) {
        const int k = threadIdx.x;
        const double v = (s_pts[0 * kSums + k] + s_pts[1 * kSums + k]) +
                         (s_pts[2 * kSums + k] + s_pts[3 * kSums + k]);
        a.tile_part[(size_t)k * a.tile_stride + b] = v;
    }
    if (threadIdx.x == 0) a.tile_good[b] = (s_good4[0] + s_good4[1]) + (s_good4[2] + s_good4[3]);
    __syncthreads();
}

__global__ __launch_bounds__(256) void direct_tiles_kernel(DirectArgs a) {
    __shared__ double s_pose[12];
    __shared__ double s_pts[kTile * kSums];
    __shared__ int s_good4[kTile];
    if (threadIdx.x == 0) {
        double st[7];
        start_state(a, st);
        state_to_pose(st, s_pose);
    }
    __syncthreads();
    double pose[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) pose[k] = s_pose[k];
    direct_tile(a, pose, blockIdx.x, s_pts, s_good4);
}

// Canonical tree over the tiles: thread t owns the aligned chunk
// [t*C, (t+1)*C) (C = P_tiles/256, a power of two <= kChunk; a 16-leaf tree
// whose extra leaves are +0.0 equals the C-leaf tree), then lanes and waves.
__device__ void reduce_tiles(const DirectArgs& a, double* S, int* n_good, double* s_red) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int t = threadIdx.x;
    int P = 256;
    while (P < a.n_tiles) P <<= 1;
    const int C = P / 256;
    for (int k = 0; k < kSums; ++k) {
        const double* src = a.tile_part + (size_t)k * a.tile_stride;
        double v[kChunk];
#pragma unroll
        for (int j = 0; j < kChunk; ++j) {
            const int tile = t * C + j;
            v[j] = (j < C && tile < a.n_tiles) ? src[tile] : 0.0;
        }
#pragma unroll
        for (int sft = 1; sft < kChunk; sft <<= 1)
#pragma unroll
            for (int j = 0; j < kChunk; j += 2 * sft) v[j] = v[j] + v[j + sft];
        const double r = wave_tree_sum_dpp(v[0]);
        if (lane == 0) s_red[wave * kSums + k] = r;
    }
    int gsum = 0;
    for (int j = 0; j < C; ++j) {
        const int tile = t * C + j;
        gsum += tile < a.n_tiles ? a.tile_good[tile] : 0;
    }
    gsum = wave_sum_int(gsum);
    __shared__ int s_g[4];
    if (lane == 0) s_g[wave] = gsum;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 0; k < kSums; ++k)
            S[k] = (s_red[0 * kSums + k] + s_red[1 * kSums + k]) +
                   (s_red[2 * kSums + k] + s_red[3 * kSums + k]);
        *n_good = (s_g[0] + s_g[1]) + (s_g[2] + s_g[3]);
    }
    __syncthreads();
}

__global__ __launch_bounds__(256) void direct_solve_kernel(DirectArgs a) {
    __shared__ double s_red[4 * kSums];
    __shared__ double S[kSums];
    __shared__ int s_ngood;
    __shared__ double s_pose[12];
    __shared__ double s_pts[kTile * kSums];
    __shared__ int s_good4[kTile];
    __shared__ int s_continue;
    __shared__ double s_state[7], s_best[7];
    __shared__ double s_cost, s_lastCost;
    if (threadIdx.x == 0) {
        start_state(a, s_state);
        for (int k = 0; k < 7; ++k) s_best[k] = s_state[k];
        s_cost = 0.0;
        s_lastCost = 0.0;
    }
    __syncthreads();
    for (int iter = 0; iter < 100; ++iter) {
        if (iter > 0) {
            // continuation (faithful, rare): this workgroup recomputes every tile
            if (threadIdx.x == 0) state_to_pose(s_state, s_pose);
            __syncthreads();
            double pose[12];
            for (int k = 0; k < 12; ++k) pose[k] = s_pose[k];
            for (int b = 0; b < a.n_tiles; ++b) direct_tile(a, pose, b, s_pts, s_good4);
            __threadfence_block();
            __syncthreads();
        }
        reduce_tiles(a, S, &s_ngood, s_red);
        if (threadIdx.x == 0) {
            double H[36], b[6];
            int idx = 0;
            for (int r = 0; r < 6; ++r)
                for (int c = r; c < 6; ++c) {
                    H[6 * r + c] = S[idx];
                    H[6 * c + r] = S[idx];
                    ++idx;
                }
            for (int k = 0; k < 6; ++k) b[k] = S[21 + k];
            double cost = s_cost + S[27];
            double inv[36], update[6];
            inverse6(H, inv);
            for (int r = 0; r < 6; ++r) {
                double s = inv[6 * r] * b[0];
                for (int c = 1; c < 6; ++c) s = s + inv[6 * r + c] * b[c];
                update[r] = s;
            }
            SE3d T21;
            for (int k = 0; k < 4; ++k) T21.q[k] = s_state[k];
            for (int k = 0; k < 3; ++k) T21.t[k] = s_state[4 + k];
            T21 = se3_mul(se3_exp(update), T21);
            for (int k = 0; k < 4; ++k) s_state[k] = T21.q[k];
            for (int k = 0; k < 3; ++k) s_state[4 + k] = T21.t[k];
            cost /= s_ngood;
            const double lastCost = s_lastCost;
            if (a.stats) {
                a.stats[0] = s_ngood;
                a.stats[1] = cost;
                for (int k = 0; k < 36; ++k) a.stats[2 + k] = H[k];
                for (int k = 0; k < 6; ++k) a.stats[38 + k] = b[k];
                for (int k = 0; k < 6; ++k) a.stats[44 + k] = update[k];
            }
            int cont = 1;
            if (isnan(update[0])) {
                for (int k = 0; k < 7; ++k) s_state[k] = s_best[k];
                cont = 0;
            } else if (iter > 0 && cost > lastCost) {
                for (int k = 0; k < 7; ++k) s_state[k] = s_best[k];
                cont = 0;
            } else if ((1 - cost / (double)lastCost) < 0.005) {
                cont = 0;
            } else {
                for (int k = 0; k < 7; ++k) s_best[k] = s_state[k];
                s_lastCost = cost;
            }
            s_cost = cost;
            s_continue = cont;
        }
        __syncthreads();
        if (!s_continue) break;
    }
    if (threadIdx.x == 0) {
        for (int k = 0; k < 7; ++k) a.se3[k] = s_state[k];
        if (a.pose_out) {
            double p[12];
            state_to_pose(s_state, p);
            for (int k = 0; k < 12; ++k) a.pose_out[k] = p[k];
            if (a.log && a.log_count) {
                const int c = *a.log_count;
                for (int k = 0; k < 12; ++k) a.log[12 * c + k] = p[k];
                *a.log_count = c + 1;
            }
        }
    }
}

__global__ void se3_from_pose_kernel(const double* pose, double* se3) {
    if (threadIdx.x != 0) return;
    double q[4];
    quat_from_matrix(pose, q);
    for (int k = 0; k < 4; ++k) se3[k] = q[k];
    se3[4] = pose[9];
    se3[5] = pose[10];
    se3[6] = pose[11];
}

__global__ void se3_to_pose_kernel(const double* se3, double* pose, double* log, int* log_count) {
    if (threadIdx.x != 0) return;
    double p[12];
    state_to_pose(se3, p);
    for (int k = 0; k < 12; ++k) pose[k] = p[k];
    if (log && log_count) {
        const int c = *log_count;
        for (int k = 0; k < 12; ++k) log[12 * c + k] = p[k];
        *log_count = c + 1;
    }
}

struct Pose12v {
    double v[12];
};

__global__ void set_pose_kernel(double* dst, Pose12v p) {
    if (threadIdx.x < 12) dst[threadIdx.x] = p.v[threadIdx.x];
}

}  // namespace

void launch_set_pose(double* dst, const double src[12], hipStream_t stream) {
    Pose12v p;
    for (int k = 0; k < 12; ++k) p.v[k] = src[k];
    set_pose_kernel<<<1, 64, 0, stream>>>(dst, p);
}

void launch_direct_level(const FrameDev& last_pyr, const FrameDev& cur_pyr, const PyrGeom& g,
                         const double K[4], const double* points, int n,
                         const double* pose_last12, double* se3_state, int level,
                         DirectScratch& s, double* stats, hipStream_t stream,
                         bool seed_from_last, double* pose_out, double* log, int* log_count) {
    DirectArgs a;
    a.last = last_pyr;
    a.cur = cur_pyr;
    a.g = make_pyrdev(g);
    a.K = Intrinsics{K[0], K[1], K[2], K[3]};
    a.points = points;
    a.n = n;
    a.pose_last = pose_last12;
    a.se3 = se3_state;
    a.seed_from_last = seed_from_last ? 1 : 0;
    a.level = level;
    a.n_tiles = (n + kTile - 1) / kTile;
    a.tile_stride = kMaxTiles;
    a.tile_part = s.tile_part;
    a.tile_good = s.tile_good;
    a.stats = stats;
    a.pose_out = pose_out;
    a.log = log;
    a.log_count = log_count;
    if (a.n_tiles > 0) direct_tiles_kernel<<<a.n_tiles, 256, 0, stream>>>(a);
    direct_solve_kernel<<<1, 256, 0, stream>>>(a);
}

size_t direct_scratch_bytes() { return (size_t)kSums * kMaxTiles * 8 + (size_t)kMaxTiles * 4; }

void launch_se3_from_pose(const double* pose12, double* se3_state, hipStream_t stream) {
    se3_from_pose_kernel<<<1, 64, 0, stream>>>(pose12, se3_state);
}

void launch_se3_to_pose(const double* se3_state, double* pose12, double* log, int* log_count,
                        hipStream_t stream) {
    se3_to_pose_kernel<<<1, 64, 0, stream>>>(se3_state, pose12, log, log_count);
}

}  // namespace viso
