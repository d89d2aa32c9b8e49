// viso_amd — deterministic synthetic stereo sequence (KITTI-like geometry).
//
// KITTI is not available offline, so tests and bench.py use
// this renderer: a box-shaped scene (back wall, two side walls, ground
// plane) textured with seeded block noise + smooth value noise, seen by a
// rectified stereo pair (baseline 0.54 m, KITTI seq-00 intrinsics by
// default) moving on a smooth oscillating trajectory.  Each pixel is the
// mean of a 2x2 supersample plus +-2 grey levels of hashed noise, so FAST
// scores rarely tie.  Pure integer hashing + double arithmetic: the same
// bytes on every host.  Host-only code (not part of the GPU hot path).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/viso/viso_synth.h"

namespace {

inline uint64_t h64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

inline double cell_value(uint64_t seed, int plane, long long a, long long b) {
    uint64_t k = h64(seed * 0x1000193ULL + (uint64_t)plane * 0x51ED27ULL) ^
                 h64((uint64_t)(a * 73856093LL) ^ (uint64_t)(b * 19349663LL));
    return (double)(h64(k) & 255ULL);
}

inline double texture(const viso_synth_params& p, int plane, double a, double b) {
    const double cs = p.block_m;
    long long ia = (long long)std::floor(a / cs), ib = (long long)std::floor(b / cs);
    double block = cell_value(p.seed, plane, ia, ib);
    const double ss = p.block_m * 7.3;
    double fa = a / ss, fb = b / ss;
    long long ja = (long long)std::floor(fa), jb = (long long)std::floor(fb);
    double ta = fa - (double)ja, tb = fb - (double)jb;
    double v00 = cell_value(p.seed + 1, plane, ja, jb), v10 = cell_value(p.seed + 1, plane, ja + 1, jb);
    double v01 = cell_value(p.seed + 1, plane, ja, jb + 1), v11 = cell_value(p.seed + 1, plane, ja + 1, jb + 1);
    double smooth = (1 - tb) * ((1 - ta) * v00 + ta * v10) + tb * ((1 - ta) * v01 + ta * v11);
    return 0.72 * block + 0.28 * smooth;
}

void rot_ypr(double yaw, double pitch, double roll, double* R) {
    // world -> camera rotation from yaw (about y), pitch (about x), roll (about z)
    double cy = std::cos(yaw), sy = std::sin(yaw);
    double cp = std::cos(pitch), sp = std::sin(pitch);
    double cr = std::cos(roll), sr = std::sin(roll);
    double Ry[9] = {cy, 0, sy, 0, 1, 0, -sy, 0, cy};
    double Rx[9] = {1, 0, 0, 0, cp, -sp, 0, sp, cp};
    double Rz[9] = {cr, -sr, 0, sr, cr, 0, 0, 0, 1};
    double T[9], Rwc[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            T[3 * i + j] = 0;
            for (int k = 0; k < 3; ++k) T[3 * i + j] += Ry[3 * i + k] * Rx[3 * k + j];
        }
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            Rwc[3 * i + j] = 0;
            for (int k = 0; k < 3; ++k) Rwc[3 * i + j] += T[3 * i + k] * Rz[3 * k + j];
        }
    // R (camera <- world) = Rwc^T
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R[3 * i + j] = Rwc[3 * j + i];
}

}  // namespace

extern "C" {

void viso_synth_default(viso_synth_params* p, int width, int height) {
    std::memset(p, 0, sizeof(*p));
    p->width = width;
    p->height = height;
    // KITTI odometry sequence 00 calib.txt P0 (public dataset fact)
    p->fx = 718.856;
    p->fy = 718.856;
    p->cx = 607.1928 * width / 1241.0;
    p->cy = 185.2157 * height / 376.0;
    p->baseline = 0.54;
    p->seed = 0;
    p->block_m = 0.45;
    p->wall_x = 9.0;
    p->wall_z = 32.0;
    p->ground_y = 1.65;
    p->pitch0 = 6.0 * 3.14159265358979323846 / 180.0;
    p->yaw_amp = 4.0 * 3.14159265358979323846 / 180.0;
    p->yaw_period = 100.0;
    p->x_amp = 0.30;
    p->x_period = 140.0;
    p->z_amp = 0.40;
    p->z_period = 160.0;
    p->noise = 2;
}

void rig_extrinsic(int cam, int n_cams, double* E12);

int viso_synth_pose(const viso_synth_params* p, int frame, int cam, double* Rt12) {
    const double two_pi = 6.28318530717958647692;
    double f = (double)frame;
    double yaw = p->yaw_amp * std::sin(two_pi * f / p->yaw_period);
    double pitch = p->pitch0 +0.2 * p->yaw_amp * std::sin(two_pi * f / (1.7 * p->yaw_period));
    double roll = 0.1 * p->yaw_amp * std::sin(two_pi * f / (2.3 * p->yaw_period));
    double C[3] = {p->x_amp * std::sin(two_pi * f / p->x_period),
                   0.05 * std::sin(two_pi * f / (0.9 * p->x_period)),
                   p->z_amp * std::sin(two_pi * f / p->z_period)};
    double R[9];
    rot_ypr(yaw, pitch, roll, R);
    // t = -R C ; right camera: +baseline along the camera x axis
    double t[3];
    for (int i = 0; i < 3; ++i) t[i] = -(R[3 * i] * C[0] + R[3 * i + 1] * C[1] + R[3 * i + 2] * C[2]);
    if (cam == 1) t[0] -= p->baseline;
    std::memcpy(Rt12, R, sizeof(R));
    std::memcpy(Rt12 + 9, t, sizeof(t));
    return 0;
}

// Rig of n_cams stereo cameras (BASELINE.json configs[4]): camera c is yawed by
// (c - (n-1)/2) * 20 deg and sits (c - (n-1)/2) * 0.35 m along the rig x axis;
// E_c maps rig -> camera c (left): P_c = Re P_rig + te.  The rig frame is the
// trajectory camera of viso_synth_pose(frame, 0).
void rig_extrinsic(int cam, int n_cams, double* E12) {
    const double k = (double)cam - 0.5 * (double)(n_cams - 1);
    const double a = k * 20.0 * 3.14159265358979323846 / 180.0;
    const double c = std::cos(a), sn = std::sin(a);
    const double Re[9] = {c, 0.0, -sn, 0.0, 1.0, 0.0, sn, 0.0, c};  // camera <- rig, yaw about y
    const double pos[3] = {0.35 * k, 0.0, 0.0};
    std::memcpy(E12, Re, sizeof(Re));
    for (int i = 0; i < 3; ++i) E12[9 + i] = -((Re[3 * i] * pos[0] + Re[3 * i + 1] * pos[1]) + Re[3 * i + 2] * pos[2]);
}

int viso_synth_rig_extrinsic(int cam, int n_cams, double* E12) {
    if (!E12 || n_cams < 1 || cam < 0 || cam >= n_cams) return -1;
    rig_extrinsic(cam, n_cams, E12);
    return 0;
}

// camera (cam, side) of the rig at `frame`: Tcw = E_c * Trig_w (+ baseline for the right image)
int viso_synth_rig_pose(const viso_synth_params* p, int frame, int n_cams, int cam, int side, double* Rt12) {
    if (!p || !Rt12 || n_cams < 1 || cam < 0 || cam >= n_cams) return -1;
    double T[12], E[12];
    viso_synth_pose(p, frame, 0, T);
    rig_extrinsic(cam, n_cams, E);
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j)
            Rt12[3 * i + j] = (E[3 * i] * T[j] + E[3 * i + 1] * T[3 + j]) + E[3 * i + 2] * T[6 + j];
        Rt12[9 + i] = ((E[3 * i] * T[9] + E[3 * i + 1] * T[10]) + E[3 * i + 2] * T[11]) + E[9 + i];
    }
    if (side == 1) Rt12[9] -= p->baseline;
    return 0;
}

static void render_rows(const viso_synth_params* p, const double* Rt, int frame, int cam, uint8_t* out,
                        int y0, int y1) {
    const double* R = Rt;
    // camera centre C = -R^T t
    double C[3];
    for (int i = 0; i < 3; ++i) C[i] = -(R[i] * Rt[9] + R[3 + i] * Rt[10] + R[6 + i] * Rt[11]);
    const int w = p->width;
    static const double so[2] = {-0.25, 0.25};
    for (int v = y0; v < y1; ++v) {
        for (int u = 0; u < w; ++u) {
            double acc = 0;
            for (int sy = 0; sy < 2; ++sy)
                for (int sx = 0; sx < 2; ++sx) {
                    double dc[3] = {((double)u + so[sx] - p->cx) / p->fx, ((double)v + so[sy] - p->cy) / p->fy, 1.0};
                    // world direction d = R^T dc
                    double d[3];
                    for (int i = 0; i < 3; ++i) d[i] = R[i] * dc[0] + R[3 + i] * dc[1] + R[6 + i] * dc[2];
                    double best = 1e30;
                    int plane = -1;
                    double hit[3] = {0, 0, 0};
                    auto test = [&](int axis, double val, int id) {
                        if (std::fabs(d[axis]) < 1e-12) return;
                        double tt = (val - C[axis]) / d[axis];
                        if (tt > 0.1 && tt < best) {
                            best = tt;
                            plane = id;
                            for (int i = 0; i < 3; ++i) hit[i] = C[i] + tt * d[i];
                        }
                    };
                    test(2, p->wall_z, 0);    // back wall
                    test(0, -p->wall_x, 1);   // left wall
                    test(0, p->wall_x, 2);    // right wall
                    test(1, p->ground_y, 3);  // ground (y down)
                    double val;
                    if (plane < 0 || best > 200.0) {
                        val = 150.0 + 40.0 * dc[1];
                    } else if (plane == 0) {
                        val = texture(*p, 0, hit[0], hit[1]);
                    } else if (plane == 1 || plane == 2) {
                        val = texture(*p, plane, hit[2], hit[1]);
                    } else {
                        val = texture(*p, 3, hit[0], hit[2]);
                    }
                    acc += val;
                }
            double g = acc * 0.25;
            if (p->noise > 0) {
                uint64_t k = h64(((uint64_t)frame << 40) ^ ((uint64_t)cam << 38) ^ ((uint64_t)v << 16) ^ (uint64_t)u ^
                                 (p->seed * 0x2545F4914F6CDD1DULL));
                g += (double)((int)(k % (uint64_t)(2 * p->noise + 1)) - p->noise);
            }
            int gi = (int)std::lround(g);
            out[(size_t)v * w + u] = (uint8_t)(gi < 0 ? 0 : (gi > 255 ? 255 : gi));
        }
    }
}

static int render(const viso_synth_params* p, const double* Rt, int frame, int noise_cam, uint8_t* out,
                  int threads) {
    if (threads <= 1) {
        render_rows(p, Rt, frame, noise_cam, out, 0, p->height);
        return 0;
    }
    std::vector<std::thread> ts;
    int rows = (p->height + threads - 1) / threads;
    for (int i = 0; i < threads; ++i) {
        int y0 = i * rows, y1 = std::min(p->height, y0 + rows);
        if (y0 >= y1) break;
        ts.emplace_back(render_rows, p, Rt, frame, noise_cam, out, y0, y1);
    }
    for (auto& t : ts) t.join();
    return 0;
}

int viso_synth_render(const viso_synth_params* p, int frame, int cam, uint8_t* out, int threads) {
    if (!p || !out || p->width <= 0 || p->height <= 0) return -1;
    double Rt[12];
    viso_synth_pose(p, frame, cam, Rt);
    return render(p, Rt, frame, cam, out, threads);
}

int viso_synth_rig_render(const viso_synth_params* p, int frame, int n_cams, int cam, int side, uint8_t* out,
                          int threads) {
    if (!p || !out || p->width <= 0 || p->height <= 0) return -1;
    double Rt[12];
    if (viso_synth_rig_pose(p, frame, n_cams, cam, side, Rt)) return -1;
    // pixel noise keyed by (camera, side) as well (cam field: 2 bits side+cam)
    return render(p, Rt, frame, 2 * cam + side, out, threads);
}

}  // extern "C"
