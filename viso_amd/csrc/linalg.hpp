// viso_amd — small dense linear algebra for the geometry kernels, one lane
// each: one-sided Jacobi null vector (Triangulate's JacobiSVD,
// src/viso.cpp:425), cyclic Jacobi symmetric eigen-decomposition, complete-
// pivot Gauss-Jordan null vector of an 8x9 system, 3x3 SVD via A^T A.
// Same algorithms and operation order as the oracle's.
#pragma once

#include "common.hpp"

namespace viso {

template <int N>
__device__ inline void null_vector_jacobi(const double* Ain, double* v_out) {
    double U[N * N], V[N * N];
#pragma unroll
    for (int i = 0; i < N * N; ++i) {
        U[i] = Ain[i];
        V[i] = (i % (N + 1) == 0) ? 1.0 : 0.0;
    }
    for (int sweep = 0; sweep < 40; ++sweep) {
        bool rotated = false;
#pragma unroll
        for (int p = 0; p < N - 1; ++p)
#pragma unroll
            for (int q = p + 1; q < N; ++q) {
                double alpha = 0, beta = 0, gamma = 0;
#pragma unroll
                for (int i = 0; i < N; ++i) {
                    alpha = alpha + U[N * i + p] * U[N * i + p];
                    beta = beta + U[N * i + q] * U[N * i + q];
                    gamma = gamma + U[N * i + p] * U[N * i + q];
                }
                if (gamma == 0.0 || fabs(gamma) <= 1e-15 * sqrt(alpha * beta)) continue;
                rotated = true;
                const double zeta = (beta - alpha) / (2.0 * gamma);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                const double c = 1.0 / sqrt(1.0 + t * t);
                const double s = c * t;
#pragma unroll
                for (int i = 0; i < N; ++i) {
                    const double up = U[N * i + p], uq = U[N * i + q];
                    U[N * i + p] = c * up - s * uq;
                    U[N * i + q] = s * up + c * uq;
                    const double vp = V[N * i + p], vq = V[N * i + q];
                    V[N * i + p] = c * vp - s * vq;
                    V[N * i + q] = s * vp + c * vq;
                }
            }
        if (!rotated) break;
    }
    int k = 0;
    double best = 0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        double nn = 0;
#pragma unroll
        for (int i = 0; i < N; ++i) nn = nn + U[N * i + j] * U[N * i + j];
        if (j == 0 || nn < best) {
            best = nn;
            k = j;
        }
    }
#pragma unroll
    for (int j = 0; j < N; ++j)
        if (j == k)
#pragma unroll
            for (int i = 0; i < N; ++i) v_out[i] = V[N * i + j];
}

template <int N>
__device__ inline void jacobi_eigen(const double* Ain, double* evals, double* evecs) {
    // every index below is a compile-time constant (all loops unrolled but
    // the sweeps), so A and V live in registers instead of scratch
    double A[N * N], V[N * N];
#pragma unroll
    for (int i = 0; i < N * N; ++i) {
        A[i] = Ain[i];
        V[i] = (i % (N + 1) == 0) ? 1.0 : 0.0;
    }
    for (int sweep = 0; sweep < 50; ++sweep) {
        double off = 0, diag = 0;
#pragma unroll
        for (int p = 0; p < N; ++p) {
            diag = diag + A[N * p + p] * A[N * p + p];
#pragma unroll
            for (int q = p + 1; q < N; ++q) off = off + A[N * p + q] * A[N * p + q];
        }
        if (off <= 1e-30 * diag || off == 0.0) break;
#pragma unroll
        for (int p = 0; p < N - 1; ++p)
#pragma unroll
            for (int q = p + 1; q < N; ++q) {
                const double apq = A[N * p + q];
                if (apq == 0.0) continue;
                const double theta = (A[N * q + q] - A[N * p + p]) / (2.0 * apq);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0);
                const double s = t * c;
#pragma unroll
                for (int k = 0; k < N; ++k) {
                    const double akp = A[N * k + p], akq = A[N * k + q];
                    A[N * k + p] = c * akp - s * akq;
                    A[N * k + q] = s * akp + c * akq;
                }
#pragma unroll
                for (int k = 0; k < N; ++k) {
                    const double apk = A[N * p + k], aqk = A[N * q + k];
                    A[N * p + k] = c * apk - s * aqk;
                    A[N * q + k] = s * apk + c * aqk;
                }
#pragma unroll
                for (int k = 0; k < N; ++k) {
                    const double vkp = V[N * k + p], vkq = V[N * k + q];
                    V[N * k + p] = c * vkp - s * vkq;
                    V[N * k + q] = s * vkp + c * vkq;
                }
            }
    }
    // descending eigenvalues, the first maximum first (a selection sort of
    // the diagonal with the columns of V carried along by predicated swaps)
    double d[N];
#pragma unroll
    for (int i = 0; i < N; ++i) d[i] = A[N * i + i];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        int m = i;
        double dm = d[i];
#pragma unroll
        for (int j = i + 1; j < N; ++j)
            if (d[j] > dm) {
                m = j;
                dm = d[j];
            }
#pragma unroll
        for (int j = i + 1; j < N; ++j)
            if (j == m) {
                const double td = d[i];
                d[i] = d[j];
                d[j] = td;
#pragma unroll
                for (int r = 0; r < N; ++r) {
                    const double tv = V[N * r + i];
                    V[N * r + i] = V[N * r + j];
                    V[N * r + j] = tv;
                }
            }
    }
#pragma unroll
    for (int j = 0; j < N; ++j) {
        evals[j] = d[j];
#pragma unroll
        for (int i = 0; i < N; ++i) evecs[N * i + j] = V[N * i + j];
    }
}

__device__ inline bool null_vector_8x9(const double* Ain, double* e) {
    double M[8 * 9];
    for (int i = 0; i < 72; ++i) M[i] = Ain[i];
    int cp[9];
    for (int j = 0; j < 9; ++j) cp[j] = j;
    for (int k = 0; k < 8; ++k) {
        int pr = k, pc = k;
        double best = -1.0;
        for (int r = k; r < 8; ++r)
            for (int c = k; c < 9; ++c) {
                const double a = fabs(M[9 * r + c]);
                if (a > best) {
                    best = a;
                    pr = r;
                    pc = c;
                }
            }
        if (!(best > 1e-300)) return false;
        if (pr != k)
            for (int j = 0; j < 9; ++j) {
                const double tmp = M[9 * k + j];
                M[9 * k + j] = M[9 * pr + j];
                M[9 * pr + j] = tmp;
            }
        if (pc != k) {
            for (int r = 0; r < 8; ++r) {
                const double tmp = M[9 * r + k];
                M[9 * r + k] = M[9 * r + pc];
                M[9 * r + pc] = tmp;
            }
            const int tmp = cp[k];
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

// null_vector_8x9 on one wave: lane l owns elements l and 64 + l (l < 8) of
// the row-major 8x9 matrix (A[0] / A[1] on entry, the eliminated matrix on
// return) and performs exactly the sequential routine's operations on them:
// the complete pivot is the first maximum |M| of the trailing submatrix in
// row-major order (a (value, index) wave maximum; NaN is never chosen), the
// row / column swaps are a permuted re-read of the matrix staged in `lds`
// (72 doubles, the wave's own), the pivot row divided by the pivot, and
// every other row r with f = M[r][k] != 0 updated as M[r][j] - f * M[k][j].
// On success every lane receives the null vector in e[9].
__device__ inline bool null_vector_8x9_wave(double (&A)[2], double* lds, double* e) {
    const int lane = threadIdx.x & 63;
    const int i0 = lane, i1 = 64 + lane;  // element i1 exists for lane < 8
    const int r0 = i0 / 9, c0 = i0 - 9 * r0, r1 = 7, c1 = i1 - 63;
    const bool has1 = lane < 8;
    int cp = lane;  // lane j < 9: the column permutation cp[j]
    for (int k = 0; k < 8; ++k) {
        // ---- pivot: the first maximum of |M[r][c]|, r >= k, c >= k
        double best = -2.0;
        int bi = 1 << 20;
        if (r0 >= k && c0 >= k) {
            const double a = fabs(A[0]);
            best = a > -1.0 ? a : -1.0;
            bi = i0;
        }
        if (has1 && c1 >= k) {
            const double a = fabs(A[1]);
            const double v = a > -1.0 ? a : -1.0;
            if (v > best) {
                best = v;
                bi = i1;
            }
        }
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const double ob = __shfl_xor(best, d);
            const int oi = __shfl_xor(bi, d);
            if (ob > best || (ob == best && oi < bi)) {
                best = ob;
                bi = oi;
            }
        }
        if (!(best > 1e-300)) return false;  // wave-uniform
        const int pr = bi / 9, pc = bi - 9 * pr;
        // ---- stage, then re-read through the row swap k <-> pr and column swap k <-> pc
        __builtin_amdgcn_wave_barrier();
        lds[i0] = A[0];
        if (has1) lds[i1] = A[1];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
        __builtin_amdgcn_wave_barrier();
        auto src = [&](int r, int c) {
            const int rr = r == k ? pr : (r == pr ? k : r);
            const int cc = c == k ? pc : (c == pc ? k : c);
            return lds[9 * rr + cc];
        };
        const double piv = src(k, k);
        double m0 = src(r0, c0), f0 = src(r0, k), p0 = src(k, c0);
        double m1 = 0.0, p1 = 0.0, f1 = 0.0;
        if (has1) {
            m1 = src(r1, c1);
            f1 = src(r1, k);
            p1 = src(k, c1);
        }
        {
            const int ck = __shfl(cp, k), cpc = __shfl(cp, pc);
            if (lane == k) cp = cpc;
            if (lane == pc) cp = ck;
        }
        // ---- normalise the pivot row, eliminate the other rows
        auto upd = [&](int r, int c, double m, double f, double p) -> double {
            if (r == k) return c > k ? m / piv : (c == k ? 1.0 : m);
            if (c < k || f == 0.0) return m;
            return c == k ? 0.0 : m - f * (p / piv);
        };
        A[0] = upd(r0, c0, m0, f0, p0);
        if (has1) A[1] = upd(r1, c1, m1, f1, p1);
    }
    // e[cp[j]] = ep[j]: ep[k] = -M[k][8] (k < 8), ep[8] = 1
    __builtin_amdgcn_wave_barrier();
    if (c0 == 8) lds[r0] = -A[0];
    if (has1 && c1 == 8) lds[r1] = -A[1];
    if (lane == 8) lds[8] = 1.0;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    const double epj = lane < 9 ? lds[lane] : 0.0;
    __builtin_amdgcn_wave_barrier();
    if (lane < 9) lds[16 + cp] = epj;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < 9; ++j) e[j] = lds[16 + j];
    return true;
}

__device__ inline double det3(const double* m) {
    return m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) +
           m[2] * (m[3] * m[7] - m[4] * m[6]);
}

__device__ inline void matmul3(const double* a, const double* b, double* o) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            o[3 * i + j] = (a[3 * i + 0] * b[0 + j] + a[3 * i + 1] * b[3 + j]) + a[3 * i + 2] * b[6 + j];
}

__device__ inline void transpose3(const double* a, double* o) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) o[3 * j + i] = a[3 * i + j];
}

__device__ inline void svd3(const double* A, double* U, double* s, double* V) {
    double At[9], AtA[9], ev[3];
    transpose3(A, At);
    matmul3(At, A, AtA);
    jacobi_eigen<3>(AtA, ev, V);
    for (int i = 0; i < 3; ++i) s[i] = sqrt(ev[i] > 0 ? ev[i] : 0.0);
    for (int j = 0; j < 2; ++j) {
        const double v0 = V[j], v1 = V[3 + j], v2 = V[6 + j];
        const double u0 = A[0] * v0 + A[1] * v1 + A[2] * v2;
        const double u1 = A[3] * v0 + A[4] * v1 + A[5] * v2;
        const double u2 = A[6] * v0 + A[7] * v1 + A[8] * v2;
        const double inv = s[j] > 0 ? 1.0 / s[j] : 0.0;
        U[j] = u0 * inv;
        U[3 + j] = u1 * inv;
        U[6 + j] = u2 * inv;
    }
    U[2] = U[3] * U[7] - U[6] * U[4];
    U[5] = U[6] * U[1] - U[0] * U[7];
    U[8] = U[0] * U[4] - U[3] * U[1];
}

// Viso::Triangulate with P1 = [I|0], P2 = [R|T]: homogeneous null vector.
__device__ inline void triangulate_h(const double* R, const double* T, double x1, double y1,
                                     double x2, double y2, double* X) {
    const double P2[12] = {R[0], R[1], R[2], T[0], R[3], R[4], R[5], T[1], R[6], R[7], R[8], T[2]};
    const double P1[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    double A[16];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        A[j] = x1 * P1[8 + j] - P1[j];
        A[4 + j] = y1 * P1[8 + j] - P1[4 + j];
        A[8 + j] = x2 * P2[8 + j] - P2[j];
        A[12 + j] = y2 * P2[8 + j] - P2[4 + j];
    }
    null_vector_jacobi<4>(A, X);
}

// Block-wide (T threads, a power of two >= 64) canonical pairwise tree over
// n leaves: leaf(i) for i < n, +0.0 beyond.  Each thread reduces an aligned
// chunk of C = max(1, P/T) leaves with the binary-counter form of the same
// tree, then lanes and the T/64 waves combine pairwise in index order — the
// same tree for any T (padding leaves are +0.0: exact).  s_red holds T/64
// doubles.  Result valid in every thread.
template <int T = 256, class F>
__device__ inline double block_tree_sum(int n, F leaf, double* s_red) {
    static_assert(T >= 64 && (T & (T - 1)) == 0, "block_tree_sum: power-of-two block");
    constexpr int W = T / 64;
    int P = 1;
    while (P < n) P <<= 1;
    const int C = P > T ? P / T : 1;
    const int t = threadIdx.x;
    double stack[16];
    int sp = 0;
    for (int j = 0; j < C; ++j) {
        const int i = t * C + j;
        double x = i < n ? leaf(i) : 0.0;
        for (int k = j; k & 1; k >>= 1) x = stack[--sp] + x;
        stack[sp++] = x;
    }
    double v = stack[0];
    v = wave_tree_sum(v);
    const int wave = t >> 6;
    __syncthreads();
    if ((t & 63) == 0) s_red[wave] = v;
    __syncthreads();
    double l[W];
#pragma unroll
    for (int k = 0; k < W; ++k) l[k] = s_red[k];
#pragma unroll
    for (int w = W; w > 1; w >>= 1)
#pragma unroll
        for (int k = 0; k < w / 2; ++k) l[k] = l[2 * k] + l[2 * k + 1];
    __syncthreads();
    return l[0];
}

}  // namespace viso
