// viso_amd — device-side geometry: projection (Keyframe::Project), the
// Sophus/Eigen SE(3) operations of the direct-pose path and the 6x6
// PartialPivLU inverse, written for one lane (wave-uniform control flow).
// Operation order follows the reference source.
#pragma once

#include "common.hpp"

namespace viso {

__device__ constexpr double kScale[kLevels] = {1.0, 0.5, 0.25, 0.125};  // keyframe.h:22

struct PyrDev {
    int w[kLevels], h[kLevels];
    unsigned long long off[kLevels];
};

inline PyrDev make_pyrdev(const PyrGeom& g) {
    PyrDev p;
    for (int l = 0; l < kLevels; ++l) {
        p.w[l] = g.w[l];
        p.h[l] = g.h[l];
        p.off[l] = g.off[l];
    }
    return p;
}

struct Intrinsics {
    double fx, fy, cx, cy;
};

// Keyframe::Project (include/keyframe.h:82-89); pose = R row-major + t
__device__ inline void project_px(const double* pose, const Intrinsics& K, const double* P,
                                  double scale, double& u, double& v) {
    double uv[3];
    mat3_vec(pose, P, uv);
    uv[0] = uv[0] + pose[9];
    uv[1] = uv[1] + pose[10];
    uv[2] = uv[2] + pose[11];
    const double z = uv[2];
    const double x = uv[0] / z, y = uv[1] / z;
    u = scale * (x * K.fx + K.cx);
    v = scale * (y * K.fy + K.cy);
}

// Keyframe::IsInside(u, v, level) (include/keyframe.h:77-80)
__device__ inline bool inside_px(double u, double v, int w, int h) {
    return u >= 0 && u < w && v >= 0 && v < h;
}

// ---------------------------------------------------------------- SE(3)
struct SE3d {
    double q[4];  // x, y, z, w
    double t[3];
};

__device__ inline void quat_from_matrix(const double* m, double* q) {
    double t = (m[0] + m[4]) + m[8];
    if (t > 0.0) {
        t = sqrt(t + 1.0);
        q[3] = 0.5 * t;
        t = 0.5 / t;
        q[0] = (m[7] - m[5]) * t;
        q[1] = (m[2] - m[6]) * t;
        q[2] = (m[3] - m[1]) * t;
    } else {
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > m[3 * i + i]) i = 2;
        int j = (i + 1) % 3;
        int k = (j + 1) % 3;
        t = sqrt(m[3 * i + i] - m[3 * j + j] - m[3 * k + k] + 1.0);
        double qq[3];
        qq[i] = 0.5 * t;
        t = 0.5 / t;
        q[3] = (m[3 * k + j] - m[3 * j + k]) * t;
        qq[j] = (m[3 * j + i] + m[3 * i + j]) * t;
        qq[k] = (m[3 * k + i] + m[3 * i + k]) * t;
        q[0] = qq[0];
        q[1] = qq[1];
        q[2] = qq[2];
    }
}

__device__ inline void quat_to_matrix(const double* q, double* r) {
    const double x = q[0], y = q[1], z = q[2], w = q[3];
    const double tx = 2.0 * x, ty = 2.0 * y, tz = 2.0 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w;
    const double txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    r[0] = 1.0 - (tyy + tzz);
    r[1] = txy - twz;
    r[2] = txz + twy;
    r[3] = txy + twz;
    r[4] = 1.0 - (txx + tzz);
    r[5] = tyz - twx;
    r[6] = txz - twy;
    r[7] = tyz + twx;
    r[8] = 1.0 - (txx + tyy);
}

__device__ inline void quat_mul(const double* a, const double* b, double* o) {
    const double w = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
    const double x = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
    const double y = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
    const double z = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
    o[0] = x;
    o[1] = y;
    o[2] = z;
    o[3] = w;
}

__device__ inline void quat_rotate(const double* q, const double* v, double* o) {
    double uv[3] = {q[1] * v[2] - q[2] * v[1], q[2] * v[0] - q[0] * v[2], q[0] * v[1] - q[1] * v[0]};
    uv[0] = uv[0] + uv[0];
    uv[1] = uv[1] + uv[1];
    uv[2] = uv[2] + uv[2];
    const double c0 = q[1] * uv[2] - q[2] * uv[1];
    const double c1 = q[2] * uv[0] - q[0] * uv[2];
    const double c2 = q[0] * uv[1] - q[1] * uv[0];
    o[0] = v[0] + q[3] * uv[0] + c0;
    o[1] = v[1] + q[3] * uv[1] + c1;
    o[2] = v[2] + q[3] * uv[2] + c2;
}

__device__ inline SE3d se3_mul(const SE3d& a, const SE3d& b) {
    SE3d r;
    double rt[3];
    quat_rotate(a.q, b.t, rt);
    r.t[0] = a.t[0] + rt[0];
    r.t[1] = a.t[1] + rt[1];
    r.t[2] = a.t[2] + rt[2];
    quat_mul(a.q, b.q, r.q);
    const double sq = ((r.q[0] * r.q[0] + r.q[1] * r.q[1]) + r.q[2] * r.q[2]) + r.q[3] * r.q[3];
    if (sq != 1.0) {
        const double f = 2.0 / (1.0 + sq);
        for (int i = 0; i < 4; ++i) r.q[i] = r.q[i] * f;
    }
    return r;
}

__device__ inline SE3d se3_exp(const double* a) {
    const double eps = 1e-10;
    const double* w = a + 3;
    const double theta_sq = (w[0] * w[0] + w[1] * w[1]) + w[2] * w[2];
    const double theta = sqrt(theta_sq);
    const double half_theta = 0.5 * theta;
    double imag, real;
    if (theta < eps) {
        const double theta_po4 = theta_sq * theta_sq;
        imag = 0.5 - (1.0 / 48.0) * theta_sq + (1.0 / 3840.0) * theta_po4;
        real = 1.0 - 0.5 * theta_sq + (1.0 / 384.0) * theta_po4;
    } else {
        imag = sin(half_theta) / theta;
        real = cos(half_theta);
    }
    SE3d r;
    r.q[0] = imag * w[0];
    r.q[1] = imag * w[1];
    r.q[2] = imag * w[2];
    r.q[3] = real;
    double V[9];
    if (theta < eps) {
        quat_to_matrix(r.q, V);
    } else {
        const double O[9] = {0.0, -w[2], w[1], w[2], 0.0, -w[0], -w[1], w[0], 0.0};
        double O2[9];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                O2[3 * i + j] = (O[3 * i + 0] * O[0 + j] + O[3 * i + 1] * O[3 + j]) + O[3 * i + 2] * O[6 + j];
        const double th2 = theta * theta;
        const double c1 = (1.0 - cos(theta)) / th2;
        const double c2 = (theta - sin(theta)) / (th2 * theta);
        for (int i = 0; i < 9; ++i) {
            const double id = (i % 4 == 0) ? 1.0 : 0.0;
            V[i] = (id + c1 * O[i]) + c2 * O2[i];
        }
    }
    mat3_vec(V, a, r.t);
    return r;
}

__device__ inline void se3_to_pose12(const SE3d& s, double* p) {
    quat_to_matrix(s.q, p);
    p[9] = s.t[0];
    p[10] = s.t[1];
    p[11] = s.t[2];
}

// Eigen 6x6 inverse() through PartialPivLU (see oracle_se3.hpp::inverse6)
__device__ inline void inverse6(const double* Hin, double* x) {
    double lu[36];
    for (int i = 0; i < 36; ++i) lu[i] = Hin[i];
    int tr[6];
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
        tr[k] = p;
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
    for (int i = 0; i < 36; ++i) x[i] = (i % 7 == 0) ? 1.0 : 0.0;
    for (int k = 0; k < 6; ++k)
        if (tr[k] != k)
            for (int j = 0; j < 6; ++j) {
                const double tmp = x[6 * k + j];
                x[6 * k + j] = x[6 * tr[k] + j];
                x[6 * tr[k] + j] = tmp;
            }
    for (int c = 0; c < 6; ++c) {
        for (int j = 0; j < 6; ++j)
            for (int i = j + 1; i < 6; ++i) x[6 * i + c] = x[6 * i + c] - lu[6 * i + j] * x[6 * j + c];
        for (int j = 5; j >= 0; --j) {
            x[6 * j + c] = x[6 * j + c] / lu[6 * j + j];
            for (int i = 0; i < j; ++i) x[6 * i + c] = x[6 * i + c] - lu[6 * i + j] * x[6 * j + c];
        }
    }
}

}  // namespace viso
