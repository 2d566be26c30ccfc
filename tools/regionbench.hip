// regionbench.hip -- prices a slab-region-ordered pass C before building one
// (standalone diagnostic, not part of libsketch).
//
// Pass C's mix per valid swipe: one random 4-B pre-check load of a register
// word, then (about half the time) a CAS on the same word.  Measured here on
// a 1.6 GB table (the C3 slab) with 14.4 M accesses per launch:
//   random  : every access anywhere in the table (today's pass C);
//   blocks  : one launch whose blocks are region major (block b works in
//             region b * R / nblocks, R regions of table / R bytes), so the
//             resident blocks share one or two regions at a time;
//   launches: R launches, one per region.
// Prints one JSON object; every time is the median of 5 timed repetitions.
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

constexpr int U = 4;  // accesses per lane per block
constexpr int T = 256;

// block b: accesses [b * T * U, (b + 1) * T * U) of n; region = b * R / nblocks
// (R = 1: the whole table); word index = region base + random below rwords
__global__ void __launch_bounds__(T) k_mix(uint32_t *t, uint64_t rwords, uint32_t R, uint32_t region0,
                                           uint64_t n, uint64_t seed) {
    const uint32_t nb = gridDim.x;
    const uint32_t region = region0 + uint32_t(uint64_t(blockIdx.x) * R / nb);
    uint32_t *base = t + uint64_t(region) * rwords;
    uint32_t *p[U];
    uint32_t v[U];
    bool cas[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint64_t i = (uint64_t(blockIdx.x) * U + u) * T + threadIdx.x;
        const uint64_t r = sm64(seed ^ i);
        p[u] = base + ((uint64_t(uint32_t(r)) * rwords) >> 32);
        cas[u] = i < n && ((r >> 40) & 1);
        v[u] = i < n ? __builtin_nontemporal_load(p[u]) : 0;
    }
#pragma unroll
    for (int u = 0; u < U; u++)
        if (cas[u]) (void)atomicCAS(p[u], v[u], v[u] + 1);
}

template <typename F>
static double median_ms(F f) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
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
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return v[2];
}

int main() {
    CK(hipSetDevice(0));
    const uint64_t bytes = 1600ull << 20;  // the C3 register slab
    const uint64_t words = bytes / 4;
    const uint64_t n = 14400000ull;  // pre-check loads per C3 step
    uint32_t *t = nullptr;
    CK(hipMalloc(&t, bytes));
    CK(hipMemset(t, 0, bytes));
    const unsigned nblk = unsigned((n + T * U - 1) / (T * U));
    printf("{\"table_MB\": %llu, \"accesses\": %llu", (unsigned long long)(bytes >> 20), (unsigned long long)n);
    double ms = median_ms([&] { hipLaunchKernelGGL(k_mix, dim3(nblk), dim3(T), 0, 0, t, words, 1u, 0u, n, 7); });
    printf(", \"random_ms\": %.4f", ms);
    for (uint32_t R : {4u, 8u, 16u, 32u}) {
        const uint64_t rw = words / R;
        ms = median_ms([&] { hipLaunchKernelGGL(k_mix, dim3(nblk), dim3(T), 0, 0, t, rw, R, 0u, n, 11); });
        printf(", \"blocks_R%u_ms\": %.4f", R, ms);
        const uint64_t nr = n / R;
        const unsigned nbr = unsigned((nr + T * U - 1) / (T * U));
        ms = median_ms([&] {
            for (uint32_t r = 0; r < R; r++)
                hipLaunchKernelGGL(k_mix, dim3(nbr), dim3(T), 0, 0, t, rw, 1u, r, nr, 13 + r);
        });
        printf(", \"launches_R%u_ms\": %.4f", R, ms);
    }
    printf("}\n");
    CK(hipFree(t));
    return 0;
}
