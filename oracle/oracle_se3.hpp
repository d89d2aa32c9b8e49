// TEST INFRASTRUCTURE ONLY — restatement of the Sophus/Eigen pieces the
// reference's direct-pose path uses (src/viso.cpp:114-118, :685-686, :735-737):
// Sophus::SE3d(R, t), SE3d::exp, SE3d * SE3d, rotationMatrix(), and
// Eigen's 6x6 inverse() (PartialPivLU).  Version-dependent third-party code;
// parity vs Sophus/Eigen is unpinned.
#ifndef VISO_ORACLE_SE3_HPP
#define VISO_ORACLE_SE3_HPP

#include <cmath>

#include "oracle_common.hpp"

namespace oracle {

struct SE3 {
    double q[4];  // x, y, z, w (Eigen coefficient order)
    double t[3];
};

// Eigen::Quaternion(const Matrix3&) (Shepperd's method, Eigen/src/Geometry/Quaternion.h)
inline void quat_from_matrix(const double* m, double* q) {
    double t = (m[0] + m[4]) + m[8];
    if (t > 0.0) {
        t = std::sqrt(t + 1.0);
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
        t = std::sqrt(m[3 * i + i] - m[3 * j + j] - m[3 * k + k] + 1.0);
        q[i] = 0.5 * t;
        t = 0.5 / t;
        q[3] = (m[3 * k + j] - m[3 * j + k]) * t;
        q[j] = (m[3 * j + i] + m[3 * i + j]) * t;
        q[k] = (m[3 * k + i] + m[3 * i + k]) * t;
    }
}

// Eigen QuaternionBase::toRotationMatrix
inline void quat_to_matrix(const double* q, double* r) {
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

// Eigen quaternion product a * b
inline void quat_mul(const double* a, const double* b, double* o) {
    const double w = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
    const double x = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
    const double y = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
    const double z = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
    o[0] = x;
    o[1] = y;
    o[2] = z;
    o[3] = w;
}

// Eigen QuaternionBase::_transformVector: v + w*uv + vec x uv, uv = 2 * (vec x v)
inline void quat_rotate(const double* q, const double* v, double* o) {
    double uv[3] = {q[1] * v[2] - q[2] * v[1], q[2] * v[0] - q[0] * v[2], q[0] * v[1] - q[1] * v[0]};
    uv[0] = uv[0] + uv[0];
    uv[1] = uv[1] + uv[1];
    uv[2] = uv[2] + uv[2];
    double c[3] = {q[1] * uv[2] - q[2] * uv[1], q[2] * uv[0] - q[0] * uv[2], q[0] * uv[1] - q[1] * uv[0]};
    o[0] = v[0] + q[3] * uv[0] + c[0];
    o[1] = v[1] + q[3] * uv[1] + c[1];
    o[2] = v[2] + q[3] * uv[2] + c[2];
}

inline SE3 se3_from_Rt(const double* R, const double* t) {
    SE3 s;
    quat_from_matrix(R, s.q);
    s.t[0] = t[0];
    s.t[1] = t[1];
    s.t[2] = t[2];
    return s;
}

// Sophus SE3 a * b: t = a.t + a.so3 * b.t ; so3 = a.so3 * b.so3 (renormalised
// by 2/(1+|q|^2) when |q|^2 != 1, Sophus SO3Base::operator*=)
inline SE3 se3_mul(const SE3& a, const SE3& b) {
    SE3 r;
    double rt[3];
    quat_rotate(a.q, b.t, rt);
    r.t[0] = a.t[0] + rt[0];
    r.t[1] = a.t[1] + rt[1];
    r.t[2] = a.t[2] + rt[2];
    quat_mul(a.q, b.q, r.q);
    double sq = ((r.q[0] * r.q[0] + r.q[1] * r.q[1]) + r.q[2] * r.q[2]) + r.q[3] * r.q[3];
    if (sq != 1.0) {
        double f = 2.0 / (1.0 + sq);
        for (int i = 0; i < 4; ++i) r.q[i] = r.q[i] * f;
    }
    return r;
}

// Sophus SE3::exp(a), a = [upsilon(3); omega(3)]
inline SE3 se3_exp(const double* a) {
    const double eps = 1e-10;
    const double* w = a + 3;
    double theta_sq = (w[0] * w[0] + w[1] * w[1]) + w[2] * w[2];
    double theta = std::sqrt(theta_sq);
    double half_theta = 0.5 * theta;
    double imag, real;
    if (theta < eps) {
        double theta_po4 = theta_sq * theta_sq;
        imag = 0.5 - (1.0 / 48.0) * theta_sq + (1.0 / 3840.0) * theta_po4;
        real = 1.0 - 0.5 * theta_sq + (1.0 / 384.0) * theta_po4;
    } else {
        double s = std::sin(half_theta);
        imag = s / theta;
        real = std::cos(half_theta);
    }
    SE3 r;
    r.q[0] = imag * w[0];
    r.q[1] = imag * w[1];
    r.q[2] = imag * w[2];
    r.q[3] = real;
    double V[9];
    if (theta < eps) {
        quat_to_matrix(r.q, V);
    } else {
        // V = I + (1-cos)/theta^2 * Omega + (theta - sin)/theta^3 * Omega^2
        double O[9] = {0.0, -w[2], w[1], w[2], 0.0, -w[0], -w[1], w[0], 0.0};
        double O2[9];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                O2[3 * i + j] = (O[3 * i + 0] * O[0 + j] + O[3 * i + 1] * O[3 + j]) + O[3 * i + 2] * O[6 + j];
        double th2 = theta * theta;
        double c1 = (1.0 - std::cos(theta)) / th2;
        double c2 = (theta - std::sin(theta)) / (th2 * theta);
        for (int i = 0; i < 9; ++i) {
            double id = (i % 4 == 0) ? 1.0 : 0.0;
            V[i] = (id + c1 * O[i]) + c2 * O2[i];
        }
    }
    mat3_vec(V, a, r.t);
    return r;
}

// Eigen 6x6 inverse through PartialPivLU (pivot = first largest |a|), then
// column-oriented forward (unit L) / backward (U) substitution.
inline void inverse6(const double* Hin, double* inv) {
    double lu[36];
    for (int i = 0; i < 36; ++i) lu[i] = Hin[i];
    int tr[6];
    for (int k = 0; k < 6; ++k) {
        int p = k;
        double best = std::fabs(lu[6 * k + k]);
        for (int i = k + 1; i < 6; ++i) {
            double s = std::fabs(lu[6 * i + k]);
            if (s > best) {
                best = s;
                p = i;
            }
        }
        tr[k] = p;
        if (best != 0.0) {
            if (p != k)
                for (int j = 0; j < 6; ++j) {
                    double tmp = lu[6 * k + j];
                    lu[6 * k + j] = lu[6 * p + j];
                    lu[6 * p + j] = tmp;
                }
            for (int i = k + 1; i < 6; ++i) lu[6 * i + k] = lu[6 * i + k] / lu[6 * k + k];
        }
        for (int i = k + 1; i < 6; ++i)
            for (int j = k + 1; j < 6; ++j) lu[6 * i + j] = lu[6 * i + j] - lu[6 * i + k] * lu[6 * k + j];
    }
    // X = P * I
    double x[36];
    for (int i = 0; i < 36; ++i) x[i] = (i % 7 == 0) ? 1.0 : 0.0;
    for (int k = 0; k < 6; ++k)
        if (tr[k] != k)
            for (int j = 0; j < 6; ++j) {
                double tmp = x[6 * k + j];
                x[6 * k + j] = x[6 * tr[k] + j];
                x[6 * tr[k] + j] = tmp;
            }
    for (int c = 0; c < 6; ++c) {
        for (int j = 0; j < 6; ++j)  // forward, unit lower
            for (int i = j + 1; i < 6; ++i) x[6 * i + c] = x[6 * i + c] - lu[6 * i + j] * x[6 * j + c];
        for (int j = 5; j >= 0; --j) {  // backward, upper
            x[6 * j + c] = x[6 * j + c] / lu[6 * j + j];
            for (int i = 0; i < j; ++i) x[6 * i + c] = x[6 * i + c] - lu[6 * i + j] * x[6 * j + c];
        }
    }
    for (int i = 0; i < 36; ++i) inv[i] = x[i];
}

// One DirectPoseEstimationSingleLayer call on the SE3 state (oracle_track.cpp).
// stats (may be null): [nGood, cost, H(36), b(6), update(6)] of the last iteration.
void direct_layer(const uint8_t* last_pyr, const uint8_t* cur_pyr, int w, int h, const double* K,
                  const double* points, int n, const double* pose_last12, SE3& T21, int level,
                  double* stats);

}  // namespace oracle

#endif
