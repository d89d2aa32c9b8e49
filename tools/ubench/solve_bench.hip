// Micro-benchmark of the direct-pose level solve (dev tool; not part of the
// library): one workgroup runs a solve of viso_amd/csrc/direct_solve.hpp
// REPS times on a fixed symmetric positive-definite H / b and reports the
// mean s_memrealtime ticks (100 MHz) per solve, plus the result bits so that
// variants can be checked for bit-identity.
// Build: hipcc -O3 -ffp-contract=off --offload-arch=gfx950 -I include -I viso_amd/csrc
//        tools/ubench/solve_bench.hip -o tools/ubench/solve_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "direct_solve.hpp"

using namespace viso;

#ifdef VISO_PROBE
__device__ unsigned long long g_probe[128];
#endif

#ifndef REPS
#define REPS 200
#endif

template <int MODE>  // 0 replicated LU (round 4), 1 LDL^T (fast mode), 2 lane-per-element LU
__global__ void bench(const double* S28, const double* st7, double* out, unsigned long long* ticks) {
    __shared__ SolveLds L;
    const int lane = threadIdx.x & 63;
    unsigned long long acc = 0, clk = 0;
    for (int r = 0; r < REPS; ++r) {
        if (threadIdx.x < kSolveSums) L.S[threadIdx.x] = S28[threadIdx.x];
        if (threadIdx.x == 0) {
            for (int k = 0; k < 7; ++k) L.state[k] = L.best[k] = st7[k];
            L.cost = 0.0;
            L.last_cost = 0.0;
            L.cont = 0;
            L.ngood = 1000;
        }
        __syncthreads();
        if (threadIdx.x < 64) {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            const unsigned long long c0 = __builtin_amdgcn_s_memtime();
#ifdef VISO_PROBE
            unsigned long long stamps[4] = {t0, t0, t0, t0};
            if (MODE == 1)
                solve_wave0_ldlt(L, 0, nullptr, stamps);
            else if (MODE == 2)
                solve_wave0_lane(L, 0, nullptr, stamps);
            else
                solve_wave0_rep(L, 0, nullptr, stamps);
#else
            if (MODE == 1)
                solve_wave0_ldlt(L, 0, nullptr);
            else if (MODE == 2)
                solve_wave0_lane(L, 0, nullptr);
            else
                solve_wave0_rep(L, 0, nullptr);
#endif
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            acc += __builtin_amdgcn_s_memrealtime() - t0;
            clk += __builtin_amdgcn_s_memtime() - c0;
#ifdef VISO_PROBE
            if (lane == 0)
                for (int k = 0; k < 4; ++k) g_probe[k] += stamps[k] - t0;
#endif
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        ticks[0] = acc;
        ticks[1] = clk;
        for (int k = 0; k < 7; ++k) out[k] = L.state[k];
        out[7] = L.cost;
    }
}

int main() {
    // an SPD H (J^T J of 200 random 6-vectors with the photometric scales)
    double H[36] = {0}, b[6] = {0};
    srand(7);
    for (int n = 0; n < 200; ++n) {
        double J[6];
        for (int k = 0; k < 6; ++k) J[k] = ((rand() % 20001) - 10000) * (k < 3 ? 1e-1 : 3e1) / 1e4;
        const double e = ((rand() % 2001) - 1000) / 100.0;
        for (int i = 0; i < 6; ++i) {
            for (int j = 0; j < 6; ++j) H[6 * i + j] += J[i] * J[j];
            b[i] += -e * J[i];
        }
    }
    double S[28];
    int idx = 0;
    for (int r = 0; r < 6; ++r)
        for (int c = r; c < 6; ++c) S[idx++] = H[6 * r + c];
    for (int k = 0; k < 6; ++k) S[21 + k] = b[k] * 1e-3;
    S[27] = 1234.5;
    const double st[7] = {0.01, -0.02, 0.005, 0.9997, 0.3, -0.1, 1.2};
    double *dS, *dst, *dout;
    unsigned long long* dt;
    hipMalloc(&dS, sizeof(S));
    hipMalloc(&dst, sizeof(st));
    hipMalloc(&dout, 8 * sizeof(double));
    hipMalloc(&dt, 2 * sizeof(unsigned long long));
    hipMemcpy(dS, S, sizeof(S), hipMemcpyHostToDevice);
    hipMemcpy(dst, st, sizeof(st), hipMemcpyHostToDevice);
    static const char* names[3] = {"LU", "LDLT", "laneLU"};
    for (int variant = 0; variant < 6; ++variant) {
        const int threads = (variant & 1) ? 512 : 64;
        const int mode = variant >> 1;
        for (int rep = 0; rep < 2; ++rep) {
            if (mode == 1)
                bench<1><<<1, threads>>>(dS, dst, dout, dt);
            else if (mode == 2)
                bench<2><<<1, threads>>>(dS, dst, dout, dt);
            else
                bench<0><<<1, threads>>>(dS, dst, dout, dt);
            hipDeviceSynchronize();
        }
        unsigned long long tt[2];
        double out[8];
        hipMemcpy(tt, dt, sizeof(tt), hipMemcpyDeviceToHost);
        const unsigned long long t = tt[0];
        printf("  shader clock %.2f GHz (%.0f clocks per solve)\n", tt[1] / (10.0 * t), (double)tt[1] / REPS);
        hipMemcpy(out, dout, sizeof(out), hipMemcpyDeviceToHost);
        unsigned long long bits = 0;
        for (int k = 0; k < 8; ++k) {
            unsigned long long u;
            memcpy(&u, &out[k], 8);
            bits = bits * 1000003ULL + u;
        }
#ifdef VISO_PROBE
        {
            unsigned long long pr[8];
            hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_probe), sizeof(pr));
            hipMemset(dt, 0, 8);
            static unsigned long long zero[128] = {};
            hipMemcpyToSymbol(HIP_SYMBOL(g_probe), zero, sizeof(zero));
            printf("  phases (us from start, cumulative): LU %.3f inverse %.3f update %.3f exp %.3f\n",
                   10.0 * pr[0] / (3.0 * REPS) / 1e3, 10.0 * pr[1] / (3.0 * REPS) / 1e3,
                   10.0 * pr[2] / (3.0 * REPS) / 1e3, 10.0 * pr[3] / (3.0 * REPS) / 1e3);
        }
#endif
        printf("%s threads %d: %.3f us per solve; result hash %016llx state %.17g %.17g %.17g\n",
               names[mode], threads, 10.0 * (double)t / REPS / 1e3, bits, out[0], out[4], out[7]);
    }
    return 0;
}
