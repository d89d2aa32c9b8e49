// TEST INFRASTRUCTURE ONLY — small dense linear algebra used by the oracle's
// geometry stage.  These are the repo's deterministic stand-ins for
// Eigen::JacobiSVD<M4d> (src/viso.cpp:425) and for the SVD / eigen / solver
// calls inside OpenCV's findEssentialMat, findHomography, recoverPose and
// decomposeHomographyMat (src/viso.cpp:221-244).  The device code
// (viso_amd/csrc/linalg.hpp) implements the same algorithms in the same
// operation order; parity vs Eigen/OpenCV themselves is unpinned.
#ifndef VISO_ORACLE_LINALG_HPP
#define VISO_ORACLE_LINALG_HPP

#include <cmath>

namespace oracle {

// One-sided (Hestenes) Jacobi on an n x n matrix A (row-major, n <= 4):
// returns the right singular vector of the smallest singular value.
template <int N>
inline void null_vector_jacobi(const double* Ain, double* v_out) {
    double U[N * N], V[N * N];
    for (int i = 0; i < N * N; ++i) {
        U[i] = Ain[i];
        V[i] = (i % (N + 1) == 0) ? 1.0 : 0.0;
    }
    for (int sweep = 0; sweep < 40; ++sweep) {
        bool rotated = false;
        for (int p = 0; p < N - 1; ++p)
            for (int q = p + 1; q < N; ++q) {
                double alpha = 0, beta = 0, gamma = 0;
                for (int i = 0; i < N; ++i) {
                    alpha = alpha + U[N * i + p] * U[N * i + p];
                    beta = beta + U[N * i + q] * U[N * i + q];
                    gamma = gamma + U[N * i + p] * U[N * i + q];
                }
                if (gamma == 0.0 || std::fabs(gamma) <= 1e-15 * std::sqrt(alpha * beta)) continue;
                rotated = true;
                double zeta = (beta - alpha) / (2.0 * gamma);
                double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
                double c = 1.0 / std::sqrt(1.0 + t * t);
                double s = c * t;
                for (int i = 0; i < N; ++i) {
                    double up = U[N * i + p], uq = U[N * i + q];
                    U[N * i + p] = c * up - s * uq;
                    U[N * i + q] = s * up + c * uq;
                    double vp = V[N * i + p], vq = V[N * i + q];
                    V[N * i + p] = c * vp - s * vq;
                    V[N * i + q] = s * vp + c * vq;
                }
            }
        if (!rotated) break;
    }
    int k = 0;
    double best = 0;
    for (int j = 0; j < N; ++j) {
        double nn = 0;
        for (int i = 0; i < N; ++i) nn = nn + U[N * i + j] * U[N * i + j];
        if (j == 0 || nn < best) {
            best = nn;
            k = j;
        }
    }
    for (int i = 0; i < N; ++i) v_out[i] = V[N * i + k];
}

// Cyclic Jacobi eigen-decomposition of a symmetric N x N matrix (row-major).
// evals sorted descending, evecs column j = eigenvector of evals[j].
template <int N>
inline void jacobi_eigen(const double* Ain, double* evals, double* evecs) {
    double A[N * N], V[N * N];
    for (int i = 0; i < N * N; ++i) {
        A[i] = Ain[i];
        V[i] = (i % (N + 1) == 0) ? 1.0 : 0.0;
    }
    for (int sweep = 0; sweep < 50; ++sweep) {
        double off = 0, diag = 0;
        for (int p = 0; p < N; ++p) {
            diag = diag + A[N * p + p] * A[N * p + p];
            for (int q = p + 1; q < N; ++q) off = off + A[N * p + q] * A[N * p + q];
        }
        if (off <= 1e-30 * diag || off == 0.0) break;
        for (int p = 0; p < N - 1; ++p)
            for (int q = p + 1; q < N; ++q) {
                double apq = A[N * p + q];
                if (apq == 0.0) continue;
                double theta = (A[N * q + q] - A[N * p + p]) / (2.0 * apq);
                double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
                double c = 1.0 / std::sqrt(t * t + 1.0);
                double s = t * c;
                for (int k = 0; k < N; ++k) {  // columns p, q
                    double akp = A[N * k + p], akq = A[N * k + q];
                    A[N * k + p] = c * akp - s * akq;
                    A[N * k + q] = s * akp + c * akq;
                }
                for (int k = 0; k < N; ++k) {  // rows p, q
                    double apk = A[N * p + k], aqk = A[N * q + k];
                    A[N * p + k] = c * apk - s * aqk;
                    A[N * q + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < N; ++k) {
                    double vkp = V[N * k + p], vkq = V[N * k + q];
                    V[N * k + p] = c * vkp - s * vkq;
                    V[N * k + q] = s * vkp + c * vkq;
                }
            }
    }
    // selection sort, descending (stable on ties)
    int idx[N];
    for (int i = 0; i < N; ++i) idx[i] = i;
    for (int i = 0; i < N; ++i) {
        int m = i;
        for (int j = i + 1; j < N; ++j)
            if (A[N * idx[j] + idx[j]] > A[N * idx[m] + idx[m]]) m = j;
        int tmp = idx[i];
        idx[i] = idx[m];
        idx[m] = tmp;
    }
    for (int j = 0; j < N; ++j) {
        evals[j] = A[N * idx[j] + idx[j]];
        for (int i = 0; i < N; ++i) evecs[N * i + j] = V[N * i + idx[j]];
    }
}

// Parallel-ordered (round-robin) Jacobi eigen-decomposition of a symmetric
// N x N matrix: the device's ordering of the 9 x 9 H-refine moment matrix
// (viso_amd/csrc/linalg.hpp jacobi_eigen_rr9).  Players 0..N-1 (+ a dummy
// when N is odd) in M - 1 rounds of the circle method: round r pairs
// arr[i] with arr[M-1-i], arr = {0, 1 + (j - 1 + r) mod (M-1) for j = 1..M-1};
// pairs with the dummy are dropped.  Within a round every rotation (c, s) is
// computed from the round's starting A (a pair with a_pq == 0 is skipped),
// then every column pair of A is rotated, then every row pair, then the
// column pairs of V -- the same operations a lane per (pair, index) does on
// the device.  Sweep test, stop rule and the descending sort as
// jacobi_eigen.
template <int N>
inline void jacobi_eigen_rr(const double* Ain, double* evals, double* evecs) {
    constexpr int M = N + (N & 1), R = M - 1, P = M / 2;
    double A[N * N], V[N * N];
    for (int i = 0; i < N * N; ++i) {
        A[i] = Ain[i];
        V[i] = (i % (N + 1) == 0) ? 1.0 : 0.0;
    }
    for (int sweep = 0; sweep < 50; ++sweep) {
        double off = 0, diag = 0;
        for (int p = 0; p < N; ++p) {
            diag = diag + A[N * p + p] * A[N * p + p];
            for (int q = p + 1; q < N; ++q) off = off + A[N * p + q] * A[N * p + q];
        }
        if (off <= 1e-30 * diag || off == 0.0) break;
        for (int r = 0; r < R; ++r) {
            int arr[M];
            arr[0] = 0;
            for (int j = 1; j < M; ++j) arr[j] = 1 + (j - 1 + r) % (M - 1);
            int pp[P], qq[P];
            double cc[P], ss[P];
            bool act[P];
            for (int i = 0; i < P; ++i) {
                const int a = arr[i], b = arr[M - 1 - i];
                pp[i] = a < b ? a : b;
                qq[i] = a < b ? b : a;
                act[i] = qq[i] < N && A[N * pp[i] + qq[i]] != 0.0;
                cc[i] = ss[i] = 0.0;
                if (!act[i]) continue;
                const int p = pp[i], q = qq[i];
                const double apq = A[N * p + q];
                const double theta = (A[N * q + q] - A[N * p + p]) / (2.0 * apq);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
                cc[i] = 1.0 / std::sqrt(t * t + 1.0);
                ss[i] = t * cc[i];
            }
            for (int i = 0; i < P; ++i) {  // columns of A
                if (!act[i]) continue;
                const int p = pp[i], q = qq[i];
                const double c = cc[i], s = ss[i];
                for (int k = 0; k < N; ++k) {
                    const double akp = A[N * k + p], akq = A[N * k + q];
                    A[N * k + p] = c * akp - s * akq;
                    A[N * k + q] = s * akp + c * akq;
                }
            }
            for (int i = 0; i < P; ++i) {  // rows of A
                if (!act[i]) continue;
                const int p = pp[i], q = qq[i];
                const double c = cc[i], s = ss[i];
                for (int k = 0; k < N; ++k) {
                    const double apk = A[N * p + k], aqk = A[N * q + k];
                    A[N * p + k] = c * apk - s * aqk;
                    A[N * q + k] = s * apk + c * aqk;
                }
            }
            for (int i = 0; i < P; ++i) {  // columns of V
                if (!act[i]) continue;
                const int p = pp[i], q = qq[i];
                const double c = cc[i], s = ss[i];
                for (int k = 0; k < N; ++k) {
                    const double vkp = V[N * k + p], vkq = V[N * k + q];
                    V[N * k + p] = c * vkp - s * vkq;
                    V[N * k + q] = s * vkp + c * vkq;
                }
            }
        }
    }
    int idx[N];
    for (int i = 0; i < N; ++i) idx[i] = i;
    for (int i = 0; i < N; ++i) {
        int m = i;
        for (int j = i + 1; j < N; ++j)
            if (A[N * idx[j] + idx[j]] > A[N * idx[m] + idx[m]]) m = j;
        int tmp = idx[i];
        idx[i] = idx[m];
        idx[m] = tmp;
    }
    for (int j = 0; j < N; ++j) {
        evals[j] = A[N * idx[j] + idx[j]];
        for (int i = 0; i < N; ++i) evecs[N * i + j] = V[N * i + idx[j]];
    }
}

// Null vector of an 8 x 9 system by Gauss-Jordan elimination with complete
// pivoting (first maximal |a| in row-major scan).  Returns false when the
// system has rank < 8 (degenerate minimal sample).
inline bool null_vector_8x9(const double* Ain, double* e) {
    double M[8 * 9];
    for (int i = 0; i < 72; ++i) M[i] = Ain[i];
    int cp[9];
    for (int j = 0; j < 9; ++j) cp[j] = j;
    for (int k = 0; k < 8; ++k) {
        int pr = k, pc = k;
        double best = -1.0;
        for (int r = k; r < 8; ++r)
            for (int c = k; c < 9; ++c) {
                double a = std::fabs(M[9 * r + c]);
                if (a > best) {
                    best = a;
                    pr = r;
                    pc = c;
                }
            }
        if (!(best > 1e-300)) return false;
        if (pr != k)
            for (int j = 0; j < 9; ++j) {
                double tmp = M[9 * k + j];
                M[9 * k + j] = M[9 * pr + j];
                M[9 * pr + j] = tmp;
            }
        if (pc != k) {
            for (int r = 0; r < 8; ++r) {
                double tmp = M[9 * r + k];
                M[9 * r + k] = M[9 * r + pc];
                M[9 * r + pc] = tmp;
            }
            int tmp = cp[k];
            cp[k] = cp[pc];
            cp[pc] = tmp;
        }
        const double piv = M[9 * k + k];
        for (int j = k + 1; j < 9; ++j) M[9 * k + j] = M[9 * k + j] / piv;
        M[9 * k + k] = 1.0;
        for (int r = 0; r < 8; ++r) {
            if (r == k) continue;
            const double f = M[9 * r + k];
            if (f == 0.0) continue;
            for (int j = k + 1; j < 9; ++j) M[9 * r + j] = M[9 * r + j] - f * M[9 * k + j];
            M[9 * r + k] = 0.0;
        }
    }
    double ep[9];
    for (int k = 0; k < 8; ++k) ep[k] = -M[9 * k + 8];
    ep[8] = 1.0;
    for (int j = 0; j < 9; ++j) e[cp[j]] = ep[j];
    return true;
}

inline double det3(const double* m) {
    return m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) +
           m[2] * (m[3] * m[7] - m[4] * m[6]);
}

inline void matmul3(const double* a, const double* b, double* o) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            o[3 * i + j] = (a[3 * i + 0] * b[0 + j] + a[3 * i + 1] * b[3 + j]) + a[3 * i + 2] * b[6 + j];
}

inline void transpose3(const double* a, double* o) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) o[3 * j + i] = a[3 * i + j];
}

// SVD of a 3x3 matrix through the eigen-decomposition of A^T A:
// A = U diag(s) V^T, s descending; U's first two columns are A v_i / s_i,
// the third is u0 x u1 (A of rank >= 2 assumed; callers check s[1] > 0).
inline void svd3(const double* A, double* U, double* s, double* V) {
    double At[9], AtA[9], ev[3];
    transpose3(A, At);
    matmul3(At, A, AtA);
    jacobi_eigen<3>(AtA, ev, V);
    for (int i = 0; i < 3; ++i) s[i] = std::sqrt(ev[i] > 0 ? ev[i] : 0.0);
    for (int j = 0; j < 2; ++j) {
        double v[3] = {V[j], V[3 + j], V[6 + j]};
        double u[3];
        u[0] = A[0] * v[0] + A[1] * v[1] + A[2] * v[2];
        u[1] = A[3] * v[0] + A[4] * v[1] + A[5] * v[2];
        u[2] = A[6] * v[0] + A[7] * v[1] + A[8] * v[2];
        double inv = s[j] > 0 ? 1.0 / s[j] : 0.0;
        U[j] = u[0] * inv;
        U[3 + j] = u[1] * inv;
        U[6 + j] = u[2] * inv;
    }
    U[2] = U[3] * U[7] - U[6] * U[4];
    U[5] = U[6] * U[1] - U[0] * U[7];
    U[8] = U[0] * U[4] - U[3] * U[1];
}

}  // namespace oracle

#endif
