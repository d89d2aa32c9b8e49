// Micro-benchmark (dev tool; not part of the library): the level-to-level
// hand-off of the direct pose's chain as (K) a dependent kernel launch vs
// (P) an in-launch grid synchronisation of a persistent grid, with the direct
// pose's geometry (247 workgroups x 1,024 threads, 68 KB LDS: one per CU) and
// its payload (28 doubles per workgroup, every workgroup reading all 247 x 28).
//
// P: per level every workgroup stores its 28 partials with sc1 stores (wave 0,
// lanes 0-27), waits vmcnt(0), and one lane adds to its XCD's shard of an
// arrival counter (agent-scope atomic add; eight shards on lines of their
// own, HW_REG_XCC_ID).  Wave 0 polls the eight shards with sc1 loads (one
// lane per shard) until their sum reaches 247 x (level + 1), then loads all
// partials with sc1 loads (MI355X_MICROARCH.md, the hand-off table's first
// row: one lane per storing workgroup signals after the wave's vmcnt(0); the
// polling wave loads after its poll matched, the other waves after a
// workgroup barrier it joins).  Double-buffered partials.  Every wait is
// bounded (an error word).
// K: one launch per level: load the previous level's partials (plain loads),
// reduce, store own partials (plain stores).
// Stamps (s_memrealtime, 100 MHz) by plain stores to per-block slots.
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench/gridsync_bench.hip -o tools/ubench/gridsync_bench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                                  \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));             \
            return 1;                                                                             \
        }                                                                                         \
    } while (0)

constexpr int kBlocks = 247, kThreads = 1024, kSums = 28, kMaxLv = 512;
constexpr unsigned long long kWaitTicks = 5000000ull;  // 50 ms

struct Buf {
    double* part;                    // [2][kBlocks][32]
    unsigned* cnt;                   // 8 shards x 32 words
    int* err;
    unsigned long long* t_arr;       // [kMaxLv][kBlocks]
    unsigned long long* t_rel;       // [kMaxLv][kBlocks]
    unsigned long long* t_done;      // [kMaxLv][kBlocks]
    double* sink;
};

__device__ inline double reduce_partials(const double* p, bool sc1) {
    // waves 0-3: lane l of wave w sums column l % 28 over the blocks b = w, w + 4, ...
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    double s = 0.0;
    if (w < 4 && l < kSums) {
        for (int b = w; b < kBlocks; b += 4) {
            const double* q = p + (size_t)b * 32 + l;
            s += sc1 ? __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *q;
        }
    }
    return s;
}

template <int SPIN>
__global__ __launch_bounds__(kThreads) void persist_kernel(Buf B, int levels) {
    __shared__ double lds[68 * 1024 / 8];
    __shared__ int s_ok;
    const int t = threadIdx.x, w = t >> 6, l = t & 63, b = blockIdx.x;
    const int xcc = (int)(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 7);
    double acc = 0.0;
    for (int lv = 0; lv < levels; ++lv) {
        // "work": optional spin, then the partials
        if (SPIN > 0) {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            while (__builtin_amdgcn_s_memrealtime() < t0 + SPIN) __builtin_amdgcn_s_sleep(1);
        }
        double* dst = B.part + (size_t)(lv & 1) * kBlocks * 32;
        if (w == 0) {
            if (l < kSums)
                __hip_atomic_store(dst + (size_t)b * 32 + l, acc + (double)(lv * 100 + b), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const unsigned long long ta = __builtin_amdgcn_s_memrealtime();
            if (l == 0) {
                __hip_atomic_fetch_add(B.cnt + xcc * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                B.t_arr[(size_t)lv * kBlocks + b] = ta;
            }
            // poll the eight shards (lane k reads shard k)
            const unsigned target = (unsigned)kBlocks * (unsigned)(lv + 1);
            const unsigned long long tw = __builtin_amdgcn_s_memrealtime();
            int ok = 1;
            for (;;) {
                unsigned v = 0;
                if (l < 8) v = __hip_atomic_load(B.cnt + l * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                // sum of lanes 0-7
                v += __shfl_xor(v, 1);
                v += __shfl_xor(v, 2);
                v += __shfl_xor(v, 4);
                v = __builtin_amdgcn_readfirstlane(v);
                if (v >= target) break;
                if (__builtin_amdgcn_s_memrealtime() - tw > kWaitTicks) {
                    ok = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (l == 0) {
                B.t_rel[(size_t)lv * kBlocks + b] = __builtin_amdgcn_s_memrealtime();
                s_ok = ok;
                if (!ok) atomicOr(B.err, 1);
            }
        }
        __syncthreads();
        if (!s_ok) return;
        const double s = reduce_partials(dst, true);
        if (w < 4 && l < kSums) lds[w * 32 + l] = s;
        __syncthreads();
        if (w == 0 && l < kSums) acc = ((lds[l] + lds[32 + l]) + lds[64 + l]) + lds[96 + l];
        if (t == 0) B.t_done[(size_t)lv * kBlocks + b] = __builtin_amdgcn_s_memrealtime();
    }
    if (w == 0 && l < kSums) B.sink[(size_t)b * 32 + l] = acc;
}

template <int SPIN>
__global__ __launch_bounds__(kThreads) void step_kernel(Buf B, int lv) {
    __shared__ double lds[68 * 1024 / 8];
    const int t = threadIdx.x, w = t >> 6, l = t & 63, b = blockIdx.x;
    if (t == 0) B.t_rel[(size_t)lv * kBlocks + b] = __builtin_amdgcn_s_memrealtime();  // entry
    double acc = 0.0;
    if (lv > 0) {
        const double s = reduce_partials(B.part + (size_t)((lv - 1) & 1) * kBlocks * 32, false);
        if (w < 4 && l < kSums) lds[w * 32 + l] = s;
        __syncthreads();
        if (w == 0 && l < kSums) acc = ((lds[l] + lds[32 + l]) + lds[64 + l]) + lds[96 + l];
    }
    if (t == 0) B.t_done[(size_t)lv * kBlocks + b] = __builtin_amdgcn_s_memrealtime();
    if (SPIN > 0) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__builtin_amdgcn_s_memrealtime() < t0 + SPIN) __builtin_amdgcn_s_sleep(1);
    }
    if (w == 0 && l < kSums) B.part[(size_t)(lv & 1) * kBlocks * 32 + (size_t)b * 32 + l] = acc + (double)(lv * 100 + b);
    __syncthreads();
    if (t == 0) B.t_arr[(size_t)lv * kBlocks + b] = __builtin_amdgcn_s_memrealtime();  // exit
}

static double pct(std::vector<double> v, double p) {
    std::sort(v.begin(), v.end());
    return v[(size_t)(p * (v.size() - 1))];
}

template <int SPIN>
int run(const char* name, bool persistent, int levels) {
    Buf B{};
    CHECK(hipMalloc(&B.part, sizeof(double) * 2 * kBlocks * 32));
    CHECK(hipMalloc(&B.cnt, sizeof(unsigned) * 8 * 32));
    CHECK(hipMalloc(&B.err, sizeof(int)));
    CHECK(hipMalloc(&B.t_arr, sizeof(unsigned long long) * kMaxLv * kBlocks));
    CHECK(hipMalloc(&B.t_rel, sizeof(unsigned long long) * kMaxLv * kBlocks));
    CHECK(hipMalloc(&B.t_done, sizeof(unsigned long long) * kMaxLv * kBlocks));
    CHECK(hipMalloc(&B.sink, sizeof(double) * kBlocks * 32));
    hipStream_t st;
    CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int rep = 0; rep < 2; ++rep) {  // rep 0 warms up
        CHECK(hipMemsetAsync(B.cnt, 0, sizeof(unsigned) * 8 * 32, st));
        CHECK(hipMemsetAsync(B.err, 0, sizeof(int), st));
        CHECK(hipMemsetAsync(B.part, 0, sizeof(double) * 2 * kBlocks * 32, st));
        CHECK(hipEventRecord(e0, st));
        if (persistent) {
            persist_kernel<SPIN><<<kBlocks, kThreads, 0, st>>>(B, levels);
        } else {
            for (int lv = 0; lv < levels; ++lv) step_kernel<SPIN><<<kBlocks, kThreads, 0, st>>>(B, lv);
        }
        CHECK(hipEventRecord(e1, st));
        CHECK(hipStreamSynchronize(st));
    }
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    int err = 0;
    CHECK(hipMemcpy(&err, B.err, sizeof(int), hipMemcpyDeviceToHost));
    std::vector<unsigned long long> ta((size_t)kMaxLv * kBlocks), tr(ta.size()), td(ta.size());
    CHECK(hipMemcpy(ta.data(), B.t_arr, sizeof(unsigned long long) * ta.size(), hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(tr.data(), B.t_rel, sizeof(unsigned long long) * ta.size(), hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(td.data(), B.t_done, sizeof(unsigned long long) * ta.size(), hipMemcpyDeviceToHost));
    // hand-off latency: the last arrival (P) / last exit (K) of level lv -> the
    // first / median / last release (P) or entry (K) of level lv + 1 (P: of lv),
    // then -> partials reduced
    std::vector<double> first, med, last, red;
    for (int lv = 1; lv < levels; ++lv) {
        const int la = persistent ? lv : lv - 1;
        unsigned long long amax = 0;
        for (int b = 0; b < kBlocks; ++b) amax = std::max(amax, ta[(size_t)la * kBlocks + b]);
        std::vector<double> r, d;
        for (int b = 0; b < kBlocks; ++b) {
            r.push_back(((double)tr[(size_t)lv * kBlocks + b] - (double)amax) / 100.0);
            d.push_back(((double)td[(size_t)lv * kBlocks + b] - (double)amax) / 100.0);
        }
        std::sort(r.begin(), r.end());
        first.push_back(r.front());
        med.push_back(r[r.size() / 2]);
        last.push_back(r.back());
        red.push_back(pct(d, 1.0));
    }
    printf("{\"variant\": \"%s\", \"spin_us\": %.1f, \"levels\": %d, \"err\": %d, \"us_per_level\": %.3f, "
           "\"release_first_p50\": %.3f, \"release_median_p50\": %.3f, \"release_last_p50\": %.3f, "
           "\"reduced_last_p50\": %.3f}\n",
           name, SPIN / 100.0, levels, err, 1e3 * ms / levels, pct(first, 0.5), pct(med, 0.5), pct(last, 0.5),
           pct(red, 0.5));
    CHECK(hipFree(B.part));
    CHECK(hipFree(B.cnt));
    CHECK(hipFree(B.err));
    CHECK(hipFree(B.t_arr));
    CHECK(hipFree(B.t_rel));
    CHECK(hipFree(B.t_done));
    CHECK(hipFree(B.sink));
    CHECK(hipStreamDestroy(st));
    return err ? 2 : 0;
}

int main() {
    int dev_cu = 0;
    CHECK(hipDeviceGetAttribute(&dev_cu, hipDeviceAttributeMultiprocessorCount, 0));
    if (dev_cu < kBlocks) {
        fprintf(stderr, "needs >= %d CUs (have %d)\n", kBlocks, dev_cu);
        return 1;
    }
    int rc = 0;
    rc |= run<0>("kernel-chain", false, 400);
    rc |= run<1000>("kernel-chain-10us", false, 400);
    rc |= run<0>("persistent-sharded", true, 400);
    rc |= run<1000>("persistent-sharded-10us", true, 400);
    return rc;
}
