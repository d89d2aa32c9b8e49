// Probe of v_mfma_f64_16x16x4_f64's arithmetic (dev tool; not part of the
// library): D = A(16x4) B(4x16) + C on random operands, compared bit for bit
// with CPU models of the accumulation, and the latency of a chain of
// dependent MFMAs.  Layout (cdna_hip_programming.md): A/B one f64 per lane
// (A[i][k] in lane i + 16 k, B[k][j] in lane j + 16 k), C/D four f64 per
// lane, D[row][col] with col = lane & 15, row = (lane >> 4) + 4 r.
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench/mfma_f64_probe.hip -o tools/ubench/mfma_f64_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

typedef double v4d __attribute__((ext_vector_type(4)));

__global__ void mfma_once(const double* A, const double* B, const double* C, double* D, int reps,
                          unsigned long long* ticks) {
    const int lane = threadIdx.x;
    const double a = A[lane], b = B[lane];
    v4d c;
    for (int r = 0; r < 4; ++r) c[r] = C[lane + 64 * r];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    v4d d = c;
    for (int i = 0; i < reps; ++i) d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d, 0, 0, 0);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < 4; ++r) D[lane + 64 * r] = d[r];
    if (lane == 0) ticks[0] = t1 - t0;
}

static double rnd(std::mt19937_64& g) {
    std::uniform_real_distribution<double> u(-1.0, 1.0);
    const double m = u(g);
    std::uniform_int_distribution<int> e(-20, 20);
    return std::ldexp(m, e(g));
}

int main() {
    std::mt19937_64 g(12345);
    const int trials = 200;
    int match[5] = {0, 0, 0, 0, 0};
    double *dA, *dB, *dC, *dD;
    unsigned long long* dt;
    hipMalloc(&dA, 64 * 8);
    hipMalloc(&dB, 64 * 8);
    hipMalloc(&dC, 256 * 8);
    hipMalloc(&dD, 256 * 8);
    hipMalloc(&dt, 8);
    long long total = 0;
    for (int t = 0; t < trials; ++t) {
        double A[64], B[64], C[256], D[256];
        for (int i = 0; i < 64; ++i) {
            A[i] = rnd(g);
            B[i] = rnd(g);
        }
        for (int i = 0; i < 256; ++i) C[i] = (t % 3 == 0) ? 0.0 : rnd(g);
        hipMemcpy(dA, A, sizeof(A), hipMemcpyHostToDevice);
        hipMemcpy(dB, B, sizeof(B), hipMemcpyHostToDevice);
        hipMemcpy(dC, C, sizeof(C), hipMemcpyHostToDevice);
        mfma_once<<<1, 64>>>(dA, dB, dC, dD, 1, dt);
        hipMemcpy(D, dD, sizeof(D), hipMemcpyDeviceToHost);
        for (int lane = 0; lane < 64; ++lane)
            for (int r = 0; r < 4; ++r) {
                const int col = lane & 15, row = (lane >> 4) + 4 * r;
                const double c = C[lane + 64 * r];
                double p[4];
                for (int k = 0; k < 4; ++k) p[k] = 0;
                // models
                double m0 = c;  // k-ordered fma chain
                for (int k = 0; k < 4; ++k) m0 = std::fma(A[row + 16 * k], B[k * 16 + col], m0);
                double m1 = c;  // reverse-ordered fma chain
                for (int k = 3; k >= 0; --k) m1 = std::fma(A[row + 16 * k], B[k * 16 + col], m1);
                double m2 = c;  // rounded products, running sum
                for (int k = 0; k < 4; ++k) m2 = m2 + A[row + 16 * k] * B[k * 16 + col];
                // exact sum of the four products and c, one rounding (long double as a proxy)
                long double acc = (long double)c;
                for (int k = 0; k < 4; ++k) acc += (long double)A[row + 16 * k] * (long double)B[k * 16 + col];
                const double m3 = (double)acc;
                // pairwise products fma: (p0 + p1) + (p2 + p3) + c
                double q01 = std::fma(A[row], B[col], A[row + 16] * B[16 + col]);
                double q23 = std::fma(A[row + 32], B[32 + col], A[row + 48] * B[48 + col]);
                const double m4 = (q01 + q23) + c;
                const double got = D[lane + 64 * r];
                match[0] += memcmp(&got, &m0, 8) == 0;
                match[1] += memcmp(&got, &m1, 8) == 0;
                match[2] += memcmp(&got, &m2, 8) == 0;
                match[3] += memcmp(&got, &m3, 8) == 0;
                match[4] += memcmp(&got, &m4, 8) == 0;
                total++;
                (void)p;
            }
    }
    printf("{\"values\": %lld, \"fma_chain_k_ascending\": %d, \"fma_chain_k_descending\": %d, "
           "\"rounded_products_running_sum\": %d, \"single_rounding\": %d, \"pairwise\": %d}\n",
           total, match[0], match[1], match[2], match[3], match[4]);
    // dependent-chain latency
    for (int reps : {16, 64, 256}) {
        mfma_once<<<1, 64>>>(dA, dB, dC, dD, reps, dt);
        hipDeviceSynchronize();
        mfma_once<<<1, 64>>>(dA, dB, dC, dD, reps, dt);
        unsigned long long tk = 0;
        hipMemcpy(&tk, dt, 8, hipMemcpyDeviceToHost);
        printf("{\"chain\": %d, \"memtime_ticks\": %llu, \"ticks_per_mfma\": %.2f}\n", reps, tk, (double)tk / reps);
    }
    return 0;
}
