// Micro-benchmark of cross-launch hand-offs that hide the dependent-launch
// boundary (dev tool; not part of the library).  A chain of N launches with
// the direct pose's geometry (247 workgroups x 1,024 threads, 68 KB LDS), each
// spinning `work` ticks, where launch k must see launch k-1 complete:
//   base   — one stream, ordinary in-order launches (the kernel boundary);
//   anyord — one stream, hipExtLaunchKernelGGL(..., hipExtAnyOrderLaunch),
//            ordering by an in-kernel wait on a completion counter;
//   2str   — launches alternating over two streams (two hardware queues), the
//            same in-kernel wait: launch k's dispatch overlaps launch k-1.
// Hand-off protocol (MI355X_MICROARCH.md, inter-workgroup visibility, row 1):
// every workgroup stores its payload words with sc1 (agent-scope relaxed
// atomic stores), waits vmcnt(0), barriers, then one lane adds 1 to a
// monotonically increasing agent-scope counter; the next launch's thread 0
// polls the counter with sc1 loads until it reaches the cumulative block count
// of the launches before it, the workgroup barriers, and every check load of
// the previous launch's payload is an sc1 load.  Every wait is bounded (50 ms
// of s_memrealtime): a timeout is counted, never a hang.  The check reads 8
// words of other workgroups' payload per workgroup and counts stale values.
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench/overlap_bench.hip -o tools/ubench/overlap_bench
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                           \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
            return 1;                                                                      \
        }                                                                                  \
    } while (0)

constexpr int kBlocks = 247;
constexpr int kRing = 4096;
__device__ unsigned long long g_entry[kRing];  // block 0 entry per launch
__device__ unsigned long long g_go[kRing];     // block 0 after its wait
__device__ unsigned long long g_exit[kRing];   // last exit per launch
__device__ unsigned int g_err[4];              // timeouts, stale reads

struct Args {
    unsigned long long* counter;  // monotonically increasing
    unsigned long long target;    // counter value meaning "launch seq - 1 complete"
    unsigned int* payload;        // [2][kBlocks][64]
    int seq;
    int work;  // ticks
    int wait;  // 0: no in-kernel wait (ordinary chain)
};

// VG128: the kernel holds 128 VGPRs like the direct pose, so one 1,024-thread
// workgroup fills a CU and the next launch's workgroups can only land where
// the previous launch's have exited.
template <bool VG128>
__global__ __launch_bounds__(1024) void chain_kernel(Args a) {
    __shared__ double s[68 * 1024 / 8];
    __shared__ int s_ok;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (VG128) asm volatile("v_mov_b32 v127, 0" ::: "v127");
    const int slot = a.seq & (kRing - 1);
    if (blockIdx.x == 0 && threadIdx.x == 0) g_entry[slot] = t0;
    s[threadIdx.x] = (double)threadIdx.x;
    if (a.wait && threadIdx.x == 0) {
        unsigned long long c = 0;
        while (true) {
            c = __hip_atomic_load(a.counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (c >= a.target) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 > 5000000ull) {  // 50 ms
                atomicAdd(&g_err[0], 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x == 0) g_go[slot] = __builtin_amdgcn_s_memrealtime();
    // check: 8 words of the previous launch's payload, from other workgroups
    if (a.seq > 0 && threadIdx.x < 8) {
        const int src = (blockIdx.x + 1 + 31 * threadIdx.x) % kBlocks;
        const unsigned int* prev = a.payload + (size_t)((a.seq - 1) & 1) * kBlocks * 64;
        const unsigned int v = __hip_atomic_load(prev + src * 64 + threadIdx.x, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
        if (v != (unsigned int)(a.seq - 1) * 1000u + (unsigned int)src) atomicAdd(&g_err[1], 1u);
    }
    const unsigned long long tw = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - tw < (unsigned long long)a.work) __builtin_amdgcn_s_sleep(2);
    // publish
    if (threadIdx.x < 64) {
        unsigned int* mine = a.payload + (size_t)(a.seq & 1) * kBlocks * 64 + blockIdx.x * 64;
        __hip_atomic_store(mine + threadIdx.x, (unsigned int)a.seq * 1000u + blockIdx.x, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicAdd(a.counter, 1ull);
        atomicMax(&g_exit[slot], __builtin_amdgcn_s_memrealtime());
    }
    if (s[(threadIdx.x + 1) % 1024] < -1.0) s_ok = 1;  // keeps the LDS allocation
}

template <bool VG128>
int run(const char* name, int mode, int n, int work) {
    std::vector<unsigned long long> zero(kRing, 0);
    unsigned int zerr[4] = {0, 0, 0, 0};
    CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_exit), zero.data(), sizeof(unsigned long long) * kRing));
    CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_err), zerr, sizeof(zerr)));
    unsigned long long* counter;
    unsigned int* payload;
    CHECK(hipMalloc(&counter, sizeof(unsigned long long)));
    CHECK(hipMalloc(&payload, sizeof(unsigned int) * 2 * kBlocks * 64));
    CHECK(hipMemset(counter, 0, sizeof(unsigned long long)));
    CHECK(hipMemset(payload, 0xff, sizeof(unsigned int) * 2 * kBlocks * 64));
    hipStream_t st[2];
    CHECK(hipStreamCreateWithFlags(&st[0], hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&st[1], hipStreamNonBlocking));
    CHECK(hipDeviceSynchronize());
    auto launch = [&](int i) {
        Args a;
        a.counter = counter;
        a.target = (unsigned long long)kBlocks * (unsigned long long)i;
        a.payload = payload;
        a.seq = i;
        a.work = work;
        a.wait = mode != 0;
        if (mode == 0)
            chain_kernel<VG128><<<kBlocks, 1024, 0, st[0]>>>(a);
        else if (mode == 1)
            hipExtLaunchKernelGGL(chain_kernel<VG128>, dim3(kBlocks), dim3(1024), 0, st[0], nullptr, nullptr,
                                  hipExtAnyOrderLaunch, a);
        else
            chain_kernel<VG128><<<kBlocks, 1024, 0, st[i & 1]>>>(a);
    };
    const auto h0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) launch(i);
    CHECK(hipDeviceSynchronize());
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h0).count();
    std::vector<unsigned long long> en(kRing), go(kRing), ex(kRing);
    CHECK(hipMemcpyFromSymbol(en.data(), HIP_SYMBOL(g_entry), sizeof(unsigned long long) * kRing));
    CHECK(hipMemcpyFromSymbol(go.data(), HIP_SYMBOL(g_go), sizeof(unsigned long long) * kRing));
    CHECK(hipMemcpyFromSymbol(ex.data(), HIP_SYMBOL(g_exit), sizeof(unsigned long long) * kRing));
    CHECK(hipMemcpyFromSymbol(zerr, HIP_SYMBOL(g_err), sizeof(zerr)));
    std::vector<double> gap, span;
    for (int i = 1; i < n; ++i) gap.push_back(((double)go[i] - (double)ex[i - 1]) / 100.0);
    for (int i = 1; i < n; ++i) span.push_back(((double)ex[i] - (double)ex[i - 1]) / 100.0);
    std::sort(gap.begin(), gap.end());
    std::sort(span.begin(), span.end());
    printf("{\"variant\": \"%s\", \"vgpr128\": %d, \"work_us\": %.1f, \"launches\": %d, \"host_us_per_launch\": %.3f, "
           "\"exit_to_exit_p50_us\": %.3f, \"prev_exit_to_go_p50_us\": %.3f, \"prev_exit_to_go_p10_us\": %.3f, "
           "\"timeouts\": %u, \"stale_reads\": %u}\n",
           name, (int)VG128, work / 100.0, n, us / n, span[span.size() / 2], gap[gap.size() / 2], gap[gap.size() / 10], zerr[0],
           zerr[1]);
    CHECK(hipStreamDestroy(st[0]));
    CHECK(hipStreamDestroy(st[1]));
    CHECK(hipFree(counter));
    CHECK(hipFree(payload));
    return 0;
}

int main() {
    int rc = 0;
    const int n = 300;
    for (int work : {0, 900}) {
        rc |= run<true>("base", 0, n, work);
        rc |= run<true>("anyord", 1, n, work);
        rc |= run<true>("2str", 2, n, work);
        rc |= run<false>("2str", 2, n, work);
    }
    return rc;
}
