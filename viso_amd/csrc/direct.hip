// viso_amd — direct photometric 6-DoF Gauss-Newton pose for gfx950
// (DirectPoseEstimationSingleLayer / MultiLayer + dPixeldXi,
// src/viso.cpp:640-766).
//
// One level = two launches:
//  1. direct_tiles_kernel (8 waves): one wave per map point at a time, lane =
//     patch pixel.  The wave forms J = -grad^T * dPixel/dXi for its 64 pixels
//     and reduces the 28 sums (21 upper-triangle J J^T, 6 -e J, e^2) with the
//     canonical DPP wave tree.  A workgroup owns an aligned tile of
//     T = max(8, P/256) points (P = next pow2 of the point count), so there
//     are at most 256 tiles; the tile's 28 sums are a tree over its points,
//     stored tile-major.
//  2. direct_solve_kernel (one workgroup): thread t loads tile t's 28 sums in
//     one burst; canonical tree over tiles (DPP wave tree, then the 4 waves);
//     PartialPivLU of H on one lane, the six inverse columns on six lanes
//     (column-oriented forward/backward substitution), update rows on six
//     lanes, SE3::exp(update) * T21, cost / nGood and the checks of :741-753.
// The sum order is the canonical pairwise tree over (point, pixel), so the
// result is independent of the launch geometry and equal to the oracle's.
// As shipped the loop takes exactly one GN step per level (cost is never
// reset, src/viso.cpp:673); the rare continuation (a level
// whose photometric cost is exactly 0) is executed faithfully by the solve
// workgroup itself, re-running every tile.
// Frame-level fusions: level 3 seeds T21 = SE3(last R, last t)
// (src/viso.cpp:114) inside both kernels; level 0's solve writes
// cur_frame R,t and appends the pose log (src/viso.cpp:117-118, 137).
#include "device_math.hpp"
#include "kernels.hpp"

namespace viso {

namespace {

constexpr int kSums = 28;
constexpr int kWaves = 8;         // waves per tiles workgroup
constexpr int kMaxTiles = 256;
constexpr int kMaxTile = kMaxMapPoints / kMaxTiles;  // 64 points

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
    int tile;     // points per tile (power of two, >= kWaves)
    int n_tiles;  // <= 256
    double* tile_part;  // tile-major [tile][28]
    int* tile_good;
    double* stats;
    double* pose_out;  // level 0: cur pose (12)
    double* log;
    int log_index;  // < 0: no log append
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

// The 28 sums of one map point by reduce-scatter: returns good; lane l < 32
// with *idx >= 0 holds sum *idx in *out.
__device__ inline bool direct_point_rs(const DirectArgs& a, const double* cur_pose, int i,
                                       double* out, int* idx) {
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
    double leaf[kSums];
    int e = 0;
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int c = r; c < 6; ++c) leaf[e++] = J[r] * J[c];
#pragma unroll
    for (int k = 0; k < 6; ++k) leaf[21 + k] = -error * J[k];
    leaf[27] = error * error;
    *out = reduce_scatter_28(leaf, idx);
    return true;
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

// Tile b (a.tile points): 28 sums -> tile_part[b], good count -> tile_good[b].
// Called by every thread of a workgroup of `nwaves` waves.
__device__ void direct_tile(const DirectArgs& a, const double* cur_pose, int b, int nwaves,
                            double* s_pts, int* s_good) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int T = a.tile;
    if (threadIdx.x == 0) *s_good = 0;
    __syncthreads();
    int good_cnt = 0;
    for (int local = wave; local < T; local += nwaves) {
        const int i = b * T + local;
        double f = 0.0;
        int idx = -1;
        bool good = false;
        if (i < a.n) good = direct_point_rs(a, cur_pose, i, &f, &idx);
        if (!good) {
            if (lane < kSums) s_pts[local * kSums + lane] = 0.0;
        } else if (lane < 32 && idx >= 0) {
            s_pts[local * kSums + idx] = f;
        }
        good_cnt += good ? 1 : 0;
    }
    if (lane == 0 && good_cnt) atomicAdd(s_good, good_cnt);
    __syncthreads();
    // tree over the tile's T points (lanes >= T hold +0.0)
    for (int k = wave; k < kSums; k += nwaves) {
        const double v = lane < T ? s_pts[lane * kSums + k] : 0.0;
        const double r = wave_tree_sum_dpp(v);
        if (lane == 0) a.tile_part[(size_t)b * kSums + k] = r;
    }
    if (threadIdx.x == 0) a.tile_good[b] = *s_good;
    __syncthreads();
}

__global__ __launch_bounds__(kWaves * 64) void direct_tiles_kernel(DirectArgs a) {
    __shared__ double s_pose[12];
    __shared__ double s_pts[kMaxTile * kSums];
    __shared__ int s_good;
    if (threadIdx.x == 0) {
        double st[7];
        start_state(a, st);
        state_to_pose(st, s_pose);
    }
    __syncthreads();
    double pose[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) pose[k] = s_pose[k];
    direct_tile(a, pose, blockIdx.x, kWaves, s_pts, &s_good);
}

// Canonical tree over <= 256 tiles: thread t holds tile t (zeros beyond).
__device__ void reduce_tiles(const DirectArgs& a, double* S, int* n_good, double* s_red,
                             int* s_g) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int t = threadIdx.x;
    double v[kSums];
    if (t < a.n_tiles) {
        const double2* src = reinterpret_cast<const double2*>(a.tile_part + (size_t)t * kSums);
#pragma unroll
        for (int k = 0; k < kSums / 2; ++k) {
            const double2 d = src[k];
            v[2 * k] = d.x;
            v[2 * k + 1] = d.y;
        }
    } else {
#pragma unroll
        for (int k = 0; k < kSums; ++k) v[k] = 0.0;
    }
    int g = t < a.n_tiles ? a.tile_good[t] : 0;
#pragma unroll
    for (int k = 0; k < kSums; ++k) {
        const double r = wave_tree_sum_dpp(v[k]);
        if (lane == 0) s_red[wave * kSums + k] = r;
    }
    g = wave_sum_int(g);
    if (lane == 0) s_g[wave] = g;
    __syncthreads();
    if (threadIdx.x < kSums) {
        const int k = threadIdx.x;
        S[k] = (s_red[0 * kSums + k] + s_red[1 * kSums + k]) + (s_red[2 * kSums + k] + s_red[3 * kSums + k]);
    }
    if (threadIdx.x == 0) *n_good = (s_g[0] + s_g[1]) + (s_g[2] + s_g[3]);
    __syncthreads();
}

__global__ __launch_bounds__(256) void direct_solve_kernel(DirectArgs a) {
    __shared__ double s_red[4 * kSums];
    __shared__ double S[kSums];
    __shared__ int s_ngood;
    __shared__ int s_g[4];
    __shared__ double s_pose[12];
    __shared__ double s_pts[kMaxTile * kSums];
    __shared__ int s_good;
    __shared__ int s_continue;
    __shared__ double s_state[7], s_best[7];
    __shared__ double s_cost, s_lastCost;
    __shared__ double s_lu[36], s_inv[36], s_upd[6];
    __shared__ int s_tr[6];
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
            for (int b = 0; b < a.n_tiles; ++b) direct_tile(a, pose, b, 4, s_pts, &s_good);
            __threadfence_block();
            __syncthreads();
        }
        reduce_tiles(a, S, &s_ngood, s_red, s_g);
        // ---- H.inverse() (Eigen PartialPivLU): factor on lane 0 ...
        if (threadIdx.x == 0) {
            double lu[36];
            int idx = 0;
            for (int r = 0; r < 6; ++r)
                for (int c = r; c < 6; ++c) {
                    lu[6 * r + c] = S[idx];
                    lu[6 * c + r] = S[idx];
                    ++idx;
                }
            for (int k = 0; k < 6; ++k) {
                int p = k;
                double best = fabs(lu[6 * k + k]);
                for (int i = k + 1; i < 6; ++i) {
                    const double s = fabs(lu[6 * i + k]);
                    if (s > best) {
                        best = s;
                        p = i;
                    }
                }
                s_tr[k] = p;
                if (best != 0.0) {
                    if (p != k)
                        for (int j = 0; j < 6; ++j) {
                            const double tmp = lu[6 * k + j];
                            lu[6 * k + j] = lu[6 * p + j];
                            lu[6 * p + j] = tmp;
                        }
                    for (int i = k + 1; i < 6; ++i) lu[6 * i + k] = lu[6 * i + k] / lu[6 * k + k];
                }
                for (int i = k + 1; i < 6; ++i)
                    for (int j = k + 1; j < 6; ++j) lu[6 * i + j] = lu[6 * i + j] - lu[6 * i + k] * lu[6 * k + j];
            }
            for (int e = 0; e < 36; ++e) s_lu[e] = lu[e];
        }
        __syncthreads();
        // ... one lane per column: X = P*I, forward (unit L), backward (U)
        if (threadIdx.x < 6) {
            const int c = threadIdx.x;
            double x[6];
            for (int i = 0; i < 6; ++i) x[i] = (i == c) ? 1.0 : 0.0;
            for (int k = 0; k < 6; ++k) {
                const int p = s_tr[k];
                if (p != k) {
                    const double tmp = x[k];
                    x[k] = x[p];
                    x[p] = tmp;
                }
            }
            for (int j = 0; j < 6; ++j)
                for (int i = j + 1; i < 6; ++i) x[i] = x[i] - s_lu[6 * i + j] * x[j];
            for (int j = 5; j >= 0; --j) {
                x[j] = x[j] / s_lu[6 * j + j];
                for (int i = 0; i < j; ++i) x[i] = x[i] - s_lu[6 * i + j] * x[j];
            }
            for (int i = 0; i < 6; ++i) s_inv[6 * i + c] = x[i];
        }
        __syncthreads();
        // update = H^-1 * b, one lane per row
        if (threadIdx.x < 6) {
            const int r = threadIdx.x;
            double s = s_inv[6 * r] * S[21];
            for (int c = 1; c < 6; ++c) s = s + s_inv[6 * r + c] * S[21 + c];
            s_upd[r] = s;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            double update[6];
            for (int k = 0; k < 6; ++k) update[k] = s_upd[k];
            double cost = s_cost + S[27];
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
                int idx = 0;
                for (int r = 0; r < 6; ++r)
                    for (int c = r; c < 6; ++c) {
                        a.stats[2 + 6 * r + c] = S[idx];
                        a.stats[2 + 6 * c + r] = S[idx];
                        ++idx;
                    }
                for (int k = 0; k < 6; ++k) a.stats[38 + k] = S[21 + k];
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
            if (a.log && a.log_index >= 0)
                for (int k = 0; k < 12; ++k) a.log[12 * (size_t)a.log_index + k] = p[k];
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

__global__ void se3_to_pose_kernel(const double* se3, double* pose, double* log, int log_index) {
    if (threadIdx.x != 0) return;
    double p[12];
    state_to_pose(se3, p);
    for (int k = 0; k < 12; ++k) pose[k] = p[k];
    if (log && log_index >= 0)
        for (int k = 0; k < 12; ++k) log[12 * (size_t)log_index + k] = p[k];
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
                         bool seed_from_last, double* pose_out, double* log, int log_index) {
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
    int P = 1;
    while (P < n) P <<= 1;
    a.tile = P / kMaxTiles > kWaves ? P / kMaxTiles : kWaves;
    a.n_tiles = (n + a.tile - 1) / a.tile;
    a.tile_part = s.tile_part;
    a.tile_good = s.tile_good;
    a.stats = stats;
    a.pose_out = pose_out;
    a.log = log;
    a.log_index = log ? log_index : -1;
    if (a.n_tiles > 0) direct_tiles_kernel<<<a.n_tiles, kWaves * 64, 0, stream>>>(a);
    direct_solve_kernel<<<1, 256, 0, stream>>>(a);
}

size_t direct_scratch_bytes() { return (size_t)kSums * kMaxTiles * 8 + (size_t)kMaxTiles * 4 + 256; }

void launch_se3_from_pose(const double* pose12, double* se3_state, hipStream_t stream) {
    se3_from_pose_kernel<<<1, 64, 0, stream>>>(pose12, se3_state);
}

void launch_se3_to_pose(const double* se3_state, double* pose12, double* log, int log_index,
                        hipStream_t stream) {
    se3_to_pose_kernel<<<1, 64, 0, stream>>>(se3_state, pose12, log, log ? log_index : -1);
}

}  // namespace viso
