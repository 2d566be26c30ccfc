// randbench.hip -- the gfx950 rates that bound K1's variants (roofline
// denominators; standalone diagnostic, not part of libsketch).
//
//   gather  : one random 4-B load per lane (a random line each) over a table
//             of T bytes -- L2-, Infinity-Cache- and HBM-resident T;
//   cas     : one random 32-bit atomicCAS per lane over T (the HLL register
//             update of the finish pass);
//   umax    : one random no-return atomicMax per lane over T;
//   store8  : one random byte store per lane over T;
//   lds8    : random ds_read_u8 from a 64 / 128 KiB LDS image, 16 waves per CU
//             (the probe of the LDS variants), reads per second chip-wide;
//   stream  : 16-B-per-lane streaming read and copy (HBM reference).
// Prints one JSON object; every rate is the median of 5 timed repetitions.
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

// r mod n by a multiply (n < 2^32): no 64-bit division in the timed loop
__device__ __forceinline__ uint64_t red(uint64_t r, uint64_t n) { return (uint64_t(uint32_t(r)) * n) >> 32; }

// U independent random accesses per lane per iteration
constexpr int U = 8;

__global__ void __launch_bounds__(256) k_gather(const uint32_t *t, uint64_t nwords, uint64_t n,
                                                uint32_t *sink, uint64_t seed) {
    uint32_t acc = 0;
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x * U;
    for (uint64_t i = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) * U; i < n; i += stride) {
        uint32_t v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = t[red(sm64(seed ^ (i + u)), nwords)];
#pragma unroll
        for (int u = 0; u < U; u++) acc ^= v[u];
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

__global__ void __launch_bounds__(256) k_cas(uint32_t *t, uint64_t nwords, uint64_t n, uint64_t seed) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x * U;
    for (uint64_t i = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) * U; i < n; i += stride) {
        uint32_t *p[U];
        uint32_t old[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t r = sm64(seed ^ (i + u));
            p[u] = &t[red(r, nwords)];
            old[u] = uint32_t(r >> 40);
        }
#pragma unroll
        for (int u = 0; u < U; u++) old[u] = atomicCAS(p[u], old[u], old[u] + 1);
        if (old[0] == 0xdeadbeefu) t[0] = 1;
    }
}

__global__ void __launch_bounds__(256) k_umax(uint32_t *t, uint64_t nwords, uint64_t n, uint64_t seed) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x * U;
    for (uint64_t i = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) * U; i < n; i += stride) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t r = sm64(seed ^ (i + u));
            atomicMax(&t[red(r, nwords)], uint32_t(r >> 58));
        }
    }
}

__global__ void __launch_bounds__(256) k_store8(uint8_t *t, uint64_t nbytes, uint64_t n, uint64_t seed) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x * U;
    for (uint64_t i = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) * U; i < n; i += stride) {
#pragma unroll
        for (int u = 0; u < U; u++) t[red(sm64(seed ^ (i + u)), nbytes)] = 1;
    }
}

// random ds_read_u8 over an LDS image of B bytes; each lane walks its own
// xorshift address chain (the address of read j+1 does not depend on read j)
template <int B>
__global__ void __launch_bounds__(1024) k_lds8(const uint8_t *src, uint64_t reads_per_lane,
                                               uint32_t *sink) {
    __shared__ uint8_t img[B];
    for (int i = threadIdx.x * 16; i < B; i += blockDim.x * 16)
        *reinterpret_cast<uint4 *>(&img[i]) = *reinterpret_cast<const uint4 *>(&src[i]);
    __syncthreads();
    uint32_t x[U], acc = 0;
#pragma unroll
    for (int u = 0; u < U; u++) x[u] = uint32_t(sm64(blockIdx.x * 1024 + threadIdx.x + u * 977));
    for (uint64_t j = 0; j < reads_per_lane; j += U) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            acc += img[x[u] % B];
            x[u] ^= x[u] << 13;
            x[u] ^= x[u] >> 17;
            x[u] ^= x[u] << 5;
        }
    }
    if (acc == 0x12345u) sink[0] = acc;
}

__global__ void __launch_bounds__(256) k_stream(const uint4 *p, uint64_t nq, uint4 *dst, uint32_t *sink) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < nq; i += uint64_t(gridDim.x) * blockDim.x) {
        const uint4 v = p[i];
        if (dst) dst[i] = v;
        else acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
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
    int dev = 0, cus = 0;
    CK(hipSetDevice(dev));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, dev));
    cus = prop.multiProcessorCount;
    const uint64_t big = 1600ull << 20;  // the C3 register slab (1.6 GB)
    uint8_t *buf = nullptr, *buf2 = nullptr;
    uint32_t *sink = nullptr;
    CK(hipMalloc(&buf, big));
    CK(hipMalloc(&buf2, big));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(buf, 0, big));
    const unsigned grid = unsigned(cus) * 8;
    const uint64_t n = 64ull << 20;  // accesses per launch
    printf("{\"device\": \"%s\", \"cus\": %d", prop.name, cus);
    const uint64_t sizes[] = {2ull << 20, 20ull << 20, 200ull << 20, big};
    const char *names[] = {"2MB", "20MB", "200MB", "1600MB"};
    for (int s = 0; s < 4; s++) {
        const uint64_t nw = sizes[s] / 4;
        double ms = median_ms([&] { hipLaunchKernelGGL(k_gather, dim3(grid), dim3(256), 0, 0, (const uint32_t *)buf, nw, n, sink, 7); });
        printf(", \"gather4_%s_Gps\": %.2f", names[s], n / ms / 1e6);
        ms = median_ms([&] { hipLaunchKernelGGL(k_cas, dim3(grid), dim3(256), 0, 0, (uint32_t *)buf, nw, n, 11); });
        printf(", \"cas_%s_Gps\": %.2f", names[s], n / ms / 1e6);
        ms = median_ms([&] { hipLaunchKernelGGL(k_umax, dim3(grid), dim3(256), 0, 0, (uint32_t *)buf, nw, n, 13); });
        printf(", \"umax_%s_Gps\": %.2f", names[s], n / ms / 1e6);
        ms = median_ms([&] { hipLaunchKernelGGL(k_store8, dim3(grid), dim3(256), 0, 0, buf, sizes[s], n, 17); });
        printf(", \"store8_%s_Gps\": %.2f", names[s], n / ms / 1e6);
    }
    {
        const uint64_t rpl = 4096;
        const uint64_t total = uint64_t(cus) * 2 * 1024 * rpl;
        double ms = median_ms([&] { hipLaunchKernelGGL(k_lds8<65536>, dim3(cus * 2), dim3(1024), 0, 0, buf, rpl, sink); });
        printf(", \"lds8_64K_2blk_Gps\": %.1f", total / ms / 1e6);
        const uint64_t total1 = uint64_t(cus) * 1024 * rpl;
        ms = median_ms([&] { hipLaunchKernelGGL(k_lds8<131072>, dim3(cus), dim3(1024), 0, 0, buf, rpl, sink); });
        printf(", \"lds8_128K_1blk_Gps\": %.1f", total1 / ms / 1e6);
    }
    {
        const uint64_t nq = big / 16;
        double ms = median_ms([&] { hipLaunchKernelGGL(k_stream, dim3(grid), dim3(256), 0, 0, (const uint4 *)buf, nq, (uint4 *)nullptr, sink); });
        printf(", \"stream_read_TBps\": %.2f", big / ms / 1e9);
        ms = median_ms([&] { hipLaunchKernelGGL(k_stream, dim3(grid), dim3(256), 0, 0, (const uint4 *)buf, nq, (uint4 *)buf2, sink); });
        printf(", \"stream_copy_TBps\": %.2f", 2.0 * big / ms / 1e9);
    }
    printf("}\n");
    CK(hipFree(buf));
    CK(hipFree(buf2));
    CK(hipFree(sink));
    return 0;
}
