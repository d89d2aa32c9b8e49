// Dev tool (not part of the library): which CUs does a CU-masked stream
// (hipExtStreamCreateWithCUMask) run on?  For several 256-bit masks it
// launches 2048 short workgroups and reports, per XCD (HW_REG_XCC_ID), how
// many distinct CUs (HW_REG_HW_ID se/sh/cu) ran at least one of them.
// Build: hipcc -O2 --offload-arch=gfx950 tools/ubench/cu_mask_probe.hip -o tools/ubench/cu_mask_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <set>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

__global__ void where(unsigned* out) {
    // HW_REG_HW_ID (4), all 32 bits; HW_REG_XCC_ID (20), low 4 bits
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);
    // a little work so the workgroups spread over the CUs
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < 200) __builtin_amdgcn_s_sleep(2);
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = hw;
        out[2 * blockIdx.x + 1] = xcc;
    }
}

static int run(const char* name, const std::vector<unsigned>& mask, int ncu) {
    hipStream_t s;
    CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
    const int nb = 2048;
    unsigned* d = nullptr;
    CK(hipMalloc(&d, 8 * nb));
    CK(hipMemsetAsync(d, 0xff, 8 * nb, s));
    where<<<nb, 64, 0, s>>>(d);
    CK(hipGetLastError());
    std::vector<unsigned> h(2 * nb);
    CK(hipMemcpyAsync(h.data(), d, 8 * nb, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    std::set<unsigned> cus[16];
    for (int b = 0; b < nb; ++b) {
        const unsigned hw = h[2 * b], x = h[2 * b + 1] & 15;
        const unsigned cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
        cus[x].insert((se << 8) | (sh << 4) | cu);
    }
    int bits = 0;
    for (unsigned m : mask) bits += __builtin_popcount(m);
    std::printf("%-28s bits %3d  CUs per XCC:", name, bits);
    int tot = 0;
    for (int x = 0; x < 8; ++x) {
        std::printf(" %2zu", cus[x].size());
        tot += (int)cus[x].size();
    }
    std::printf("  total %d\n", tot);
    // first workgroups' placement
    std::printf("    blocks 0..15 xcc:");
    for (int b = 0; b < 16; ++b) std::printf(" %u", h[2 * b + 1] & 15);
    std::printf("\n");
    CK(hipFree(d));
    CK(hipStreamDestroy(s));
    (void)ncu;
    return 0;
}

// the CUs (xcc, se, sh, cu) a masked stream ran on
static int cu_set(const std::vector<unsigned>& mask, std::set<unsigned>& out) {
    hipStream_t s;
    CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
    const int nb = 4096;
    unsigned* d = nullptr;
    CK(hipMalloc(&d, 8 * nb));
    where<<<nb, 64, 0, s>>>(d);
    CK(hipGetLastError());
    std::vector<unsigned> h(2 * nb);
    CK(hipMemcpyAsync(h.data(), d, 8 * nb, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    for (int b = 0; b < nb; ++b) {
        const unsigned hw = h[2 * b], x = h[2 * b + 1] & 15;
        out.insert((x << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15));
    }
    CK(hipFree(d));
    CK(hipStreamDestroy(s));
    return 0;
}

__global__ void spin(unsigned long long ticks, unsigned* out) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
    if (threadIdx.x == 0) out[blockIdx.x] = 1;
}

// two streams each running a 1 ms spin kernel: concurrent (~1 ms) or
// serialised (~2 ms)?
static int concurrency(const char* name, hipStream_t a, hipStream_t b, int na, int nb) {
    unsigned* d = nullptr;
    CK(hipMalloc(&d, 4 * 1024));
    for (int rep = 0; rep < 2; ++rep) {
        CK(hipDeviceSynchronize());
        const auto t0 = std::chrono::steady_clock::now();
        spin<<<na, 256, 0, a>>>(100000, d);
        spin<<<nb, 256, 0, b>>>(100000, d + 512);
        CK(hipStreamSynchronize(a));
        CK(hipStreamSynchronize(b));
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (rep == 1) std::printf("%-34s two 1-ms kernels: %.2f ms\n", name, ms);
    }
    CK(hipFree(d));
    return 0;
}

int main() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int ncu = p.multiProcessorCount;
    const int words = (ncu + 31) / 32;
    std::printf("CUs %d (%s)\n", ncu, p.gcnArchName);
    auto make = [&](auto pred) {
        std::vector<unsigned> m((size_t)words, 0u);
        for (int i = 0; i < ncu; ++i)
            if (pred(i)) m[(size_t)(i / 32)] |= 1u << (i % 32);
        return m;
    };
    int rc = 0;
    rc |= run("all", make([](int) { return true; }), ncu);
    rc |= run("bits 0..127", make([](int i) { return i < 128; }), ncu);
    rc |= run("bits 0..31", make([](int i) { return i < 32; }), ncu);
    rc |= run("bits 0..7", make([](int i) { return i < 8; }), ncu);
    rc |= run("even bits", make([](int i) { return (i & 1) == 0; }), ncu);
    rc |= run("i%32 < 20", make([](int i) { return i % 32 < 20; }), ncu);
    rc |= run("i/8 % 4 != 3", make([](int i) { return (i / 8) % 4 != 3; }), ncu);
    rc |= run("i < 160", make([](int i) { return i < 160; }), ncu);
    // complementary masks: disjoint CU sets?
    for (int split : {128, 160, 192}) {
        std::set<unsigned> a, b;
        rc |= cu_set(make([&](int i) { return i < split; }), a);
        rc |= cu_set(make([&](int i) { return i >= split; }), b);
        int common = 0;
        for (unsigned x : a) common += b.count(x) ? 1 : 0;
        std::printf("split %d: |A| %zu |B| %zu common %d\n", split, a.size(), b.size(), common);
    }
    {
        hipStream_t a, b;
        CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
        CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
        rc |= concurrency("unmasked non-blocking pair", a, b, 160, 96);
        CK(hipStreamDestroy(a));
        CK(hipStreamDestroy(b));
        auto ma = make([](int i) { return i < 160; });
        auto mb = make([](int i) { return i >= 160; });
        CK(hipExtStreamCreateWithCUMask(&a, (uint32_t)ma.size(), ma.data()));
        CK(hipExtStreamCreateWithCUMask(&b, (uint32_t)mb.size(), mb.data()));
        rc |= concurrency("masked pair 160/96", a, b, 160, 96);
        CK(hipStreamDestroy(a));
        CK(hipStreamDestroy(b));
        // masked after two other streams exist (as in the library)
        hipStream_t x, y;
        CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
        CK(hipStreamCreateWithFlags(&y, hipStreamNonBlocking));
        CK(hipExtStreamCreateWithCUMask(&a, (uint32_t)ma.size(), ma.data()));
        CK(hipExtStreamCreateWithCUMask(&b, (uint32_t)mb.size(), mb.data()));
        rc |= concurrency("masked pair beside 2 streams", a, b, 160, 96);
        unsigned got[8] = {0};
        CK(hipExtStreamGetCUMask(a, 8, got));
        std::printf("mask a read back: %08x %08x %08x %08x %08x %08x %08x %08x\n", got[0], got[1], got[2], got[3], got[4], got[5], got[6], got[7]);
    }
    return rc;
}
