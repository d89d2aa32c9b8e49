// Micro-benchmark of the dependent-launch boundary (dev tool; not part of the
// library): chains of launches of empty-bodied kernels
// with the direct pose's launch geometry (247 workgroups x 1,024 threads,
// 68 KB LDS, 128 VGPRs, a ~600-byte by-value argument struct behind three
// preloaded scalars) and variants that drop one property at a time.  Per
// variant: host-timed microseconds per launch over a chain, and from
// s_memrealtime stamps (100 MHz) the gap between the last workgroup's exit
// of launch i and block 0's entry of launch i + 1 (the ring probe's
// "boundary"), and the entry -> last exit span of a launch.
// Build: hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-kernarg-preload-count=5
//        tools/ubench/boundary_bench.hip -o tools/ubench/boundary_bench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                             \
        }                                                                         \
    } while (0)

constexpr int kRing = 4096;
__device__ unsigned long long g_entry[kRing];
__device__ unsigned long long g_exit[kRing];
__device__ unsigned long long g_first_exit[kRing];
// PLAIN mode (-DPLAIN_STAMPS): exit stamps by plain stores to one slot per
// block (no same-address atomics: 247 serialised atomicMax / atomicMin per
// launch take several us after the last stamp and were counted as "gap")
constexpr int kMaxBlocks = 256;
__device__ unsigned long long g_exit_blk[kRing][kMaxBlocks];

template <int AB>
struct Args {
    int seq;
    int spin;  // ticks (100 MHz) every block waits before its exit stamp
    int pad[AB / 4];
};

template <int THREADS, int LDS, bool VG128, int AB>
__global__ __launch_bounds__(THREADS) void chain_kernel(const double* __restrict__ pre, const int* __restrict__ g,
                                                        int hdr, Args<AB> a) {
    __shared__ double s[LDS / 8 > 0 ? LDS / 8 : 1];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const int slot = a.seq & (kRing - 1);
    if (blockIdx.x == 0 && threadIdx.x == 0) g_entry[slot] = t0;
    if (VG128) asm volatile("v_mov_b32 v127, 0" ::: "v127");
    if (LDS > 0) {
        s[threadIdx.x % (LDS / 8)] = (double)threadIdx.x;
        __syncthreads();
        if (s[(threadIdx.x + 1) % (LDS / 8)] < -1.0 && pre) ((double*)pre)[0] = 1.0;  // never true
    }
    if (a.spin > 0)
        while (__builtin_amdgcn_s_memrealtime() < t0 + (unsigned long long)a.spin) __builtin_amdgcn_s_sleep(2);
    if (threadIdx.x == 0) {
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
#ifdef PLAIN_STAMPS
        g_exit_blk[slot][blockIdx.x] = t1;
#else
        atomicMax(&g_exit[slot], t1);
        atomicMin(&g_first_exit[slot], t1);
#endif
    }
    (void)g;
    (void)hdr;
}

struct Result {
    double us_per_launch, gap_p50, gap_mean, span_p50;
};

template <int THREADS, int LDS, bool VG128, int AB>
int run(const char* name, int blocks, int n, Result* out, int spin = 0, bool graph = false) {
    std::vector<unsigned long long> zero(kRing, 0), big(kRing, ~0ull);
    CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_exit), zero.data(), sizeof(unsigned long long) * kRing));
    CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_first_exit), big.data(), sizeof(unsigned long long) * kRing));
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    Args<AB> a{};
    a.spin = spin;
    double* pre = nullptr;
    int* g = nullptr;
    for (int w = 0; w < 50; ++w) {  // warm-up (code object, queues)
        a.seq = kRing - 1;
        chain_kernel<THREADS, LDS, VG128, AB><<<blocks, THREADS, 0, st>>>(pre, g, 0, a);
    }
    CHECK(hipStreamSynchronize(st));
    CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_exit), zero.data(), sizeof(unsigned long long) * kRing));
    CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_first_exit), big.data(), sizeof(unsigned long long) * kRing));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipGraphExec_t gx = nullptr;
    if (graph) {
        hipGraph_t gr;
        CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int i = 0; i < n; ++i) {
            a.seq = i;
            chain_kernel<THREADS, LDS, VG128, AB><<<blocks, THREADS, 0, st>>>(pre, g, i, a);
        }
        CHECK(hipStreamEndCapture(st, &gr));
        CHECK(hipGraphInstantiate(&gx, gr, nullptr, nullptr, 0));
        CHECK(hipGraphLaunch(gx, st));  // warm replay
        CHECK(hipStreamSynchronize(st));
        CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_exit), zero.data(), sizeof(unsigned long long) * kRing));
    }
    CHECK(hipEventRecord(e0, st));
    if (graph) {
        CHECK(hipGraphLaunch(gx, st));
    } else {
        for (int i = 0; i < n; ++i) {
            a.seq = i;
            chain_kernel<THREADS, LDS, VG128, AB><<<blocks, THREADS, 0, st>>>(pre, g, i, a);
        }
    }
    CHECK(hipEventRecord(e1, st));
    CHECK(hipStreamSynchronize(st));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> en(kRing), ex(kRing);
    CHECK(hipMemcpyFromSymbol(en.data(), HIP_SYMBOL(g_entry), sizeof(unsigned long long) * kRing));
    CHECK(hipMemcpyFromSymbol(ex.data(), HIP_SYMBOL(g_exit), sizeof(unsigned long long) * kRing));
#ifdef PLAIN_STAMPS
    {
        std::vector<unsigned long long> eb((size_t)kRing * kMaxBlocks);
        CHECK(hipMemcpyFromSymbol(eb.data(), HIP_SYMBOL(g_exit_blk), sizeof(unsigned long long) * eb.size()));
        for (int i = 0; i < n; ++i) {
            unsigned long long m = 0;
            for (int b = 0; b < blocks; ++b) m = std::max(m, eb[(size_t)i * kMaxBlocks + b]);
            ex[i] = m;
        }
    }
#endif
    std::vector<double> gap, span;
    for (int i = 1; i < n; ++i) gap.push_back((double)(en[i] - ex[i - 1]) / 100.0);
    for (int i = 0; i < n; ++i) span.push_back((double)(ex[i] - en[i]) / 100.0);
    std::sort(gap.begin(), gap.end());
    std::sort(span.begin(), span.end());
    double gm = 0;
    for (double v : gap) gm += v;
    out->us_per_launch = 1e3 * ms / n;
    out->gap_p50 = gap[gap.size() / 2];
    out->gap_mean = gm / gap.size();
    out->span_p50 = span[span.size() / 2];
    printf("{\"variant\": \"%s\", \"spin_us\": %.1f, \"graph\": %d, \"blocks\": %d, \"threads\": %d, \"lds\": %d, \"vgpr128\": %d, \"arg_bytes\": %d, "
           "\"us_per_launch\": %.3f, \"gap_p50_us\": %.3f, \"gap_mean_us\": %.3f, \"span_p50_us\": %.3f}\n",
           name, spin / 100.0, (int)graph, blocks, THREADS, LDS, (int)VG128, AB, out->us_per_launch, out->gap_p50, out->gap_mean, out->span_p50);
    CHECK(hipStreamDestroy(st));
    return 0;
}

int main() {
    const int n = 400;
    Result r;
    int rc = 0;
    // the direct pose's geometry
    rc |= run<1024, 68 * 1024, true, 600>("direct-like", 247, n, &r);
    rc |= run<1024, 68 * 1024, true, 16>("small-args", 247, n, &r);
    rc |= run<1024, 0, true, 600>("no-lds", 247, n, &r);
    rc |= run<1024, 68 * 1024, false, 600>("few-vgprs", 247, n, &r);
    rc |= run<1024, 0, false, 16>("1024-bare", 247, n, &r);
    rc |= run<512, 34 * 1024, true, 600>("512-threads", 247, n, &r);
    rc |= run<256, 17 * 1024, true, 600>("256-threads", 247, n, &r);
    rc |= run<256, 0, false, 16>("256-bare", 256, n, &r);
    rc |= run<64, 0, false, 16>("64-bare", 256, n, &r);
    rc |= run<1024, 68 * 1024, true, 600>("direct-like-again", 247, n, &r);
    // kernels long enough (10 us) that the host stays ahead: the GPU-side boundary
    rc |= run<1024, 68 * 1024, true, 600>("direct-like-10us", 247, n, &r, 1000);
    rc |= run<256, 0, false, 16>("256-bare-10us", 256, n, &r, 1000);
    rc |= run<1024, 68 * 1024, true, 600>("direct-like-graph", 247, n, &r, 0, true);
    rc |= run<1024, 68 * 1024, true, 600>("direct-like-10us-graph", 247, n, &r, 1000, true);
    rc |= run<256, 0, false, 16>("256-bare-graph", 256, n, &r, 0, true);
    return rc;
}
