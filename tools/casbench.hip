// casbench.hip -- what pass C's register raise costs (standalone diagnostic;
// not part of libsketch): per op, load a random 32-bit word of a 1.6 GB table
// (the C3 register slab) and raise one of its bytes by a CAS whose expected
// value is the loaded word (retry on failure) -- pass C's pre-check + CAS.
//   rand     : addresses uniform over the whole table
//   win<W>   : op i goes to window i*W/n of W equal windows (the grid sweeps the
//              windows in order, so the live footprint is ~1.6 GB / W)
//   small    : uniform over the first 100 MB
//   xcd      : the table cut in 8 regions, block b raising only in region b % 8
//              (blocks are dealt round-robin to the 8 XCDs: every line is
//              raised from one XCD only)
//   xcd_l2   : as xcd over the first 16 MB (2 MB per XCD: each XCD's region
//              fits its 4 MB L2) -- does an XCD-local raise resolve in L2?
// Prints G ops/s for 7.3M and 58M ops.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

__device__ __forceinline__ uint64_t sm64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ULL;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t red(uint64_t r, uint64_t n) { return (uint64_t(uint32_t(r)) * n) >> 32; }

constexpr int U = 2;

__global__ void __launch_bounds__(256) k_raise(uint32_t *t, uint64_t nwords, uint64_t n, uint32_t nwin,
                                               uint64_t seed, int xcd) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x * U;
    const uint64_t wwords = nwords / (xcd ? 8 : nwin);
    for (uint64_t i = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) * U; i < n; i += stride) {
        uint32_t *p[U];
        uint32_t cur[U], sh[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t r = sm64(seed ^ (i + u));
            const uint64_t win = xcd ? blockIdx.x % 8 : (i + u) * nwin / n;
            p[u] = &t[win * wwords + red(r, wwords)];
            sh[u] = uint32_t(r >> 62) * 8;
        }
#pragma unroll
        for (int u = 0; u < U; u++) cur[u] = p[u][0];
#pragma unroll
        for (int u = 0; u < U; u++) {
            uint32_t old = cur[u];
            for (;;) {
                const uint32_t b = (old >> sh[u]) & 0xffu;
                if (b >= 250) break;
                const uint32_t prev = atomicCAS(p[u], old, (old & ~(0xffu << sh[u])) | ((b + 1) << sh[u]));
                if (prev == old) break;
                old = prev;
            }
        }
    }
}

template <typename F>
static double median_ms(F f) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    std::vector<float> v;
    for (int r = 0; r < 5; r++) {
        CK(hipEventRecord(a));
        f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        v.push_back(ms);
    }
    std::sort(v.begin(), v.end());
    return v[2];
}

int main() {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const uint64_t big = 1600ull << 20, small = 100ull << 20;
    uint32_t *t = nullptr;
    CK(hipMalloc(&t, big));
    CK(hipMemset(t, 0, big));
    const unsigned grid = unsigned(cus) * 8;
    printf("{");
    const char *sep = "";
    for (uint64_t n : {7300000ull, 58400000ull}) {
        struct M { const char *name; uint64_t bytes; uint32_t nwin; int xcd; } modes[] = {
            {"rand", big, 1, 0}, {"win4", big, 4, 0}, {"win16", big, 16, 0}, {"win64", big, 64, 0},
            {"small", small, 1, 0}, {"xcd", big, 1, 1}, {"xcd_l2", 16ull << 20, 1, 1}};
        for (auto &m : modes) {
            const double ms = median_ms([&] {
                hipLaunchKernelGGL(k_raise, dim3(grid), dim3(256), 0, 0, t, m.bytes / 4, n, m.nwin, 1234, m.xcd);
            });
            printf("%s\"%s_%lluM_Gps\": %.2f", sep, m.name, (unsigned long long)(n / 1000000), n / ms / 1e6);
            sep = ", ";
        }
    }
    printf("}\n");
    CK(hipFree(t));
    return 0;
}
