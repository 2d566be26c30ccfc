// runbench.hip -- what reading short runs costs on gfx950 (standalone
// diagnostic for the partitioned K1's pass B; not part of libsketch).
//
// A 704 MB buffer of u32 "records" is cut into tiles of `stride` records; a
// run is the first `len` records of a tile (the runs of one slice in the
// partitioned K1 are `len` ~ 37 records long, one per 11264-record tile).
// Every variant reads every run once and XORs the records (kept live):
//   stream4   contiguous, 4 B per lane (reference)
//   stream16  contiguous, 16 B per lane (reference)
//   run64x4   one run per wave instruction round: 64 lanes x 4 B
//   run8x16   8 runs per instruction, 8 lanes x 16 B each (pass B v6)
//   run16x16  4 runs per instruction, 16 lanes x 16 B each
// Prints GB/s of run bytes (len * 4 per tile) for each variant and len.
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

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rs(const void *p, uint32_t nbytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, int(nbytes), 0x00020000);
}
constexpr uint32_t kOOR = 0x80000000u;

__global__ void __launch_bounds__(1024) k_stream4(const uint32_t *p, uint32_t n, uint32_t *sink) {
    uint32_t acc = 0;
    for (uint32_t i = blockIdx.x * 1024 + threadIdx.x; i < n; i += gridDim.x * 1024) acc ^= p[i];
    if (acc == 0x1234567u) sink[0] = acc;
}
__global__ void __launch_bounds__(1024) k_stream16(const uint4 *p, uint32_t n4, uint32_t *sink) {
    uint32_t acc = 0;
    for (uint32_t i = blockIdx.x * 1024 + threadIdx.x; i < n4; i += gridDim.x * 1024) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x1234567u) sink[0] = acc;
}

// The runs of a tile are its `stride / len` consecutive pieces of `len`
// records (slices); wave work items are (slice, group of tiles), slice major,
// so a wave reads one slice's runs of consecutive tiles (as pass B does).

// one wave reads one run per round: 64 lanes x 4 B, two rounds (len <= 128)
__global__ void __launch_bounds__(1024) k_run64x4(const uint32_t *p, uint32_t ntiles, uint32_t stride,
                                                  uint32_t len, uint32_t *sink) {
    const __amdgpu_buffer_rsrc_t r = rs(p, ntiles * stride * 4);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t gw = blockIdx.x * 16 + (threadIdx.x >> 6), nw = gridDim.x * 16;
    const uint32_t ns = stride / len, items = ns * ntiles;
    uint32_t acc = 0;
    for (uint32_t it = gw; it < items; it += nw * 2) {
        uint32_t v[4];
#pragma unroll
        for (uint32_t h = 0; h < 2; h++) {
            const uint32_t ii = it + h * nw;
            const uint32_t sl = ii / ntiles, t = ii % ntiles;
#pragma unroll
            for (uint32_t c = 0; c < 2; c++) {
                const uint32_t i = c * 64 + lane;
                v[c * 2 + h] = __builtin_amdgcn_raw_buffer_load_b32(
                    r, (ii < items && i < len) ? (t * stride + sl * len + i) * 4 : kOOR, 0, 0);
            }
        }
        acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
    }
    if (acc == 0x1234567u) sink[0] = acc;
}

// L lanes per run, 16 B per lane, 64/L runs (consecutive tiles of one slice)
// per instruction, R rounds; runs start at their natural (unaligned)
// position, or (aligned) at a 128-B boundary
template <int L, int R>
__global__ void __launch_bounds__(1024) k_runLx16(const uint32_t *p, uint32_t ntiles, uint32_t stride,
                                                  uint32_t len, uint32_t aligned, uint32_t *sink) {
    const __amdgpu_buffer_rsrc_t r = rs(p, ntiles * stride * 4);
    constexpr uint32_t G = 64 / L;
    const uint32_t lane = threadIdx.x & 63, k = lane / L, q = lane % L;
    const uint32_t gw = blockIdx.x * 16 + (threadIdx.x >> 6), nw = gridDim.x * 16;
    const uint32_t ns = stride / len, ngr = ntiles / G, items = ns * ngr;
    uint32_t acc = 0;
    for (uint32_t it = gw; it < items; it += nw) {
        const uint32_t sl = it / ngr, t = (it % ngr) * G + k;
        const uint32_t b = aligned ? sl * ((len + 31) & ~31u) : sl * len;
        const uint32_t s0 = b & ~3u, e = b + len;
        uint4 v[R];
        const uint32_t rounds = (e - s0 + L * 4 - 1) / (L * 4);  // <= R
#pragma unroll
        for (uint32_t c = 0; c < R; c++) {
            const uint32_t i = s0 + c * L * 4 + q * 4;
            v[c] = c < rounds ? __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                 r, i < e ? (t * stride + i) * 4 : kOOR, 0, 0)) : uint4{0, 0, 0, 0};
        }
#pragma unroll
        for (uint32_t c = 0; c < R; c++) acc ^= v[c].x ^ v[c].y ^ v[c].z ^ v[c].w;
    }
    if (acc == 0x1234567u) sink[0] = acc;
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
    const uint32_t stride = 11264, ntiles = 15625;
    const size_t bytes = size_t(ntiles) * stride * 4;
    uint32_t *p = nullptr, *sink = nullptr;
    CK(hipMalloc(&p, bytes + 4096));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(p, 1, bytes));
    const unsigned grid = cus * 2;
    printf("{\"stream4_GBps\": %.0f", bytes / median_ms([&] {
        hipLaunchKernelGGL(k_stream4, dim3(grid), dim3(1024), 0, 0, p, uint32_t(bytes / 4), sink); }) / 1e6);
    printf(", \"stream16_GBps\": %.0f", bytes / median_ms([&] {
        hipLaunchKernelGGL(k_stream16, dim3(grid), dim3(1024), 0, 0, (const uint4 *)p, uint32_t(bytes / 16), sink); }) / 1e6);
    for (uint32_t len : {37u, 74u, 120u}) {
        const double rb = double(ntiles) * (stride / len) * len * 4;
        printf(", \"run64x4_%u_GBps\": %.0f", len, rb / median_ms([&] {
            hipLaunchKernelGGL(k_run64x4, dim3(grid), dim3(1024), 0, 0, p, ntiles, stride, len, sink); }) / 1e6);
        printf(", \"run8x16_%u_GBps\": %.0f", len, rb / median_ms([&] {
            hipLaunchKernelGGL((k_runLx16<8, 6>), dim3(grid), dim3(1024), 0, 0, p, ntiles, stride, len, 0u, sink); }) / 1e6);
        printf(", \"run8x16_%u_aligned_GBps\": %.0f", len, rb / median_ms([&] {
            hipLaunchKernelGGL((k_runLx16<8, 6>), dim3(grid), dim3(1024), 0, 0, p, ntiles, stride, len, 1u, sink); }) / 1e6);
        printf(", \"run16x16_%u_GBps\": %.0f", len, rb / median_ms([&] {
            hipLaunchKernelGGL((k_runLx16<16, 4>), dim3(grid), dim3(1024), 0, 0, p, ntiles, stride, len, 0u, sink); }) / 1e6);
    }
    printf("}\n");
    CK(hipFree(p));
    CK(hipFree(sink));
    return 0;
}
