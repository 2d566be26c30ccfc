// fetchcal.hip -- calibrate rocprofv3's FETCH_SIZE (and TCC_MISS / TCC_EA0_RDREQ)
// against known memory footprints, one kernel per access kind the partitioned
// K1's pass B issues (standalone diagnostic; not part of libsketch).
//
// MI355X_MICROARCH.md (HBM section): FETCH_SIZE = TCC_EA0_RDREQ x 64 B and
// reports half of a 16-B-per-lane streaming read; other widths are
// uncalibrated.  Pass B mixes three kinds, so one blanket factor cannot price
// it.  Each kernel below touches a number of distinct 128-B lines known on the
// host (over a 704 MB buffer, far above the 256 MiB Infinity Cache, so no
// line is served on chip between kernels), and prints it with its time:
//
//   stream16   every line of the buffer, 16 B per lane (the image copy, the
//              record pieces)
//   line4      one 4-B load per line, consecutive lines per lane (run
//              boundaries: 8 lanes read 8 consecutive words, other lanes far)
//   sector4    one 4-B load per 64-B half line
//   runs       pass B's record reads exactly: runs of `len` u32 records at
//              their natural 4-B offsets in tiles of 11264 records (151 runs per
//              tile), each run read as 16-B pieces of 8 lanes from the 128-B
//              line holding its start; reported lines = every (run, line)
//              pair read (a line shared by two runs is read twice)
//   runs_al    the same runs with each start rounded up to a 128-B line
//              (pass A writing sentinel-padded runs)
//
//   wstream16 / wbytes / wline4   stores: 16 B per lane over every line, 1 B
//              per lane contiguous, one 4-B word per line (WRITE_SIZE)
//
// tools/fetchcal_summary.py divides the PMC per kernel by these counts.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                               \
    do {                                                                    \
        hipError_t e_ = (x);                                                \
        if (e_ != hipSuccess) {                                             \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
            exit(1);                                                        \
        }                                                                   \
    } while (0)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rs(const void *p, uint32_t nbytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, int(nbytes), 0x00020000);
}
constexpr uint32_t kOOR = 0x80000000u;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(1024) k_stream16(const uint32_t *p, uint32_t n16, uint32_t *sink) {
    const __amdgpu_buffer_rsrc_t r = rs(p, n16 * 16);
    uint32_t acc = 0;
    for (uint32_t i = blockIdx.x * 1024 + threadIdx.x; i < n16; i += gridDim.x * 1024) {
        const uint4 v = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, i * 16, 0, 0));
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x1234567u) sink[0] = acc;
}

// one 4-B word every `step` bytes (128: one per line, 64: one per half line)
__global__ void __launch_bounds__(1024) k_strided4(const uint32_t *p, uint32_t nwords, uint32_t step_words,
                                                   uint32_t *sink) {
    const __amdgpu_buffer_rsrc_t r = rs(p, nwords * 4);
    uint32_t acc = 0;
    const uint32_t n = nwords / step_words;
    for (uint32_t i = blockIdx.x * 1024 + threadIdx.x; i < n; i += gridDim.x * 1024)
        acc ^= __builtin_amdgcn_raw_buffer_load_b32(r, i * step_words * 4, 0, 0);
    if (acc == 0x1234567u) sink[0] = acc;
}

// pass B's run reads: work item = (run, 8 consecutive tiles), run-major (a
// wave reads one run index of 8 consecutive tiles per round, as pass B reads
// one slice pair of 8 tiles); start[t * nr + j], start[t * nr + nr] = end
template <int R>
__global__ void __launch_bounds__(1024) k_runs(const uint32_t *p, uint32_t nbytes, const uint32_t *start,
                                               uint32_t ntiles, uint32_t nr, uint32_t stride, uint32_t *sink) {
    const __amdgpu_buffer_rsrc_t r = rs(p, nbytes);
    const uint32_t lane = threadIdx.x & 63, k = lane / 8, q = lane % 8;
    const uint32_t gw = blockIdx.x * 16 + (threadIdx.x >> 6), nw = gridDim.x * 16;
    const uint32_t ng = ntiles / 8, items = nr * ng;
    uint32_t acc = 0;
    for (uint32_t it = gw; it < items; it += nw) {
        const uint32_t j = it / ng, t = (it % ng) * 8 + k;
        const uint32_t b = start[t * (nr + 1) + j], e = start[t * (nr + 1) + j + 1];
        const uint32_t s0 = b & ~31u;
        for (uint32_t c0 = 0; s0 + c0 * 32 < e; c0 += R) {
            uint4 v[R];
#pragma unroll
            for (uint32_t c = 0; c < R; c++) {
                const uint32_t i = s0 + (c0 + c) * 32 + q * 4;
                v[c] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                    r, i < e ? (t * stride + i) * 4 : kOOR, 0, 2));
            }
#pragma unroll
            for (uint32_t c = 0; c < R; c++) acc ^= v[c].x ^ v[c].y ^ v[c].z ^ v[c].w;
        }
    }
    if (acc == 0x1234567u) sink[0] = acc;
}

// writes (WRITE_SIZE calibration): 16 B per lane over every line (pass A's
// record copy-out), 1 B per lane contiguous (pass C's answers), one 4-B word
// per 128-B line (a scattered partial-line store)
__global__ void __launch_bounds__(1024) k_wstream16(uint32_t *p, uint32_t n16) {
    const __amdgpu_buffer_rsrc_t r = rs(p, n16 * 16);
    for (uint32_t i = blockIdx.x * 1024 + threadIdx.x; i < n16; i += gridDim.x * 1024)
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{i, i, i, i}, r, i * 16, 0, 2);
}
__global__ void __launch_bounds__(1024) k_wbytes(uint32_t *p, uint32_t n) {
    const __amdgpu_buffer_rsrc_t r = rs(p, n);
    for (uint32_t i = blockIdx.x * 1024 + threadIdx.x; i < n; i += gridDim.x * 1024)
        __builtin_amdgcn_raw_buffer_store_b8(uint8_t(i), r, i, 0, 0);
}
__global__ void __launch_bounds__(1024) k_wstrided4(uint32_t *p, uint32_t nwords, uint32_t step_words) {
    const __amdgpu_buffer_rsrc_t r = rs(p, nwords * 4);
    const uint32_t n = nwords / step_words;
    for (uint32_t i = blockIdx.x * 1024 + threadIdx.x; i < n; i += gridDim.x * 1024)
        __builtin_amdgcn_raw_buffer_store_b32(i, r, i * step_words * 4, 0, 0);
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
    const uint32_t stride = 11264, ntiles = 15624, nr = 151;  // C3: 16M swipes, k = 11, 151 slice pairs
    const size_t bytes = size_t(ntiles) * stride * 4;
    uint32_t *p = nullptr, *sink = nullptr, *st = nullptr;
    CK(hipMalloc(&p, bytes + 4096));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(p, 1, bytes));
    const unsigned grid = cus * 2;
    const double lines_all = double(bytes) / 128;
    // every launch runs 6 times (1 + 5 timed): PMC per dispatch equals one run
    printf("{\"buffer_bytes\": %zu", bytes);
    printf(", \"stream16\": {\"ms\": %.4f, \"lines\": %.0f}", median_ms([&] {
        hipLaunchKernelGGL(k_stream16, dim3(grid), dim3(1024), 0, 0, p, uint32_t(bytes / 16), sink); }), lines_all);
    printf(", \"line4\": {\"ms\": %.4f, \"lines\": %.0f}", median_ms([&] {
        hipLaunchKernelGGL(k_strided4, dim3(grid), dim3(1024), 0, 0, p, uint32_t(bytes / 4), 32u, sink); }), lines_all);
    printf(", \"sector4\": {\"ms\": %.4f, \"lines\": %.0f, \"sectors\": %.0f}", median_ms([&] {
        hipLaunchKernelGGL(k_strided4, dim3(grid), dim3(1024), 0, 0, p, uint32_t(bytes / 4), 16u, sink); }),
        lines_all, 2 * lines_all);
    // run lengths as pass B sees them: 11264 records of a tile over 151 pairs
    // (multinomial, drawn with a fixed LCG), natural or line-aligned starts
    std::vector<uint32_t> hs(size_t(ntiles) * (nr + 1));
    for (int al = 0; al < 2; al++) {
        uint64_t s = 0x9E3779B97F4A7C15ull;
        double lines = 0, recs = 0;
        for (uint32_t t = 0; t < ntiles; t++) {
            std::vector<uint32_t> cnt(nr, 0);
            for (uint32_t i = 0; i < 11264; i++) {
                s = s * 6364136223846793005ull + 1442695040888963407ull;
                cnt[uint32_t((s >> 33) % nr)]++;
            }
            uint32_t pos = 0;
            for (uint32_t j = 0; j < nr; j++) {
                if (al) pos = (pos + 31) & ~31u;
                hs[size_t(t) * (nr + 1) + j] = pos;
                if (cnt[j]) lines += ((pos + cnt[j] - 1) >> 5) - (pos >> 5) + 1;
                recs += cnt[j];
                pos += cnt[j];
            }
            hs[size_t(t) * (nr + 1) + nr] = pos;
            if (pos > (al ? stride + 32 * nr : stride)) { fprintf(stderr, "tile overflow\n"); return 1; }
        }
        const uint32_t tstride = al ? stride + 32 * nr : stride;
        const size_t need = size_t(ntiles) * tstride * 4;
        uint32_t *q = p;
        if (need > bytes) {
            CK(hipMalloc(&q, need + 4096));
            CK(hipMemset(q, 1, need));
        }
        if (!st) CK(hipMalloc(&st, hs.size() * 4));
        CK(hipMemcpy(st, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
        printf(", \"%s\": {\"ms\": %.4f, \"lines\": %.0f, \"record_bytes\": %.0f}", al ? "runs_al" : "runs",
               median_ms([&] {
                   hipLaunchKernelGGL((k_runs<4>), dim3(grid), dim3(1024), 0, 0, q, uint32_t(need), st, ntiles, nr,
                                      tstride, sink);
               }),
               lines, recs * 4);
        if (q != p) CK(hipFree(q));
    }
    const size_t wb = bytes / 4;  // 176 MB of bytes: the answers' shape
    printf(", \"wstream16\": {\"ms\": %.4f, \"lines\": %.0f, \"bytes\": %zu}", median_ms([&] {
        hipLaunchKernelGGL(k_wstream16, dim3(grid), dim3(1024), 0, 0, p, uint32_t(bytes / 16)); }), lines_all, bytes);
    printf(", \"wbytes\": {\"ms\": %.4f, \"lines\": %.0f, \"bytes\": %zu}", median_ms([&] {
        hipLaunchKernelGGL(k_wbytes, dim3(grid), dim3(1024), 0, 0, p, uint32_t(wb)); }), double(wb) / 128, wb);
    printf(", \"wline4\": {\"ms\": %.4f, \"lines\": %.0f, \"bytes\": %.0f}", median_ms([&] {
        hipLaunchKernelGGL(k_wstrided4, dim3(grid), dim3(1024), 0, 0, p, uint32_t(bytes / 4), 32u); }), lines_all,
        lines_all * 4);
    printf("}\n");
    CK(hipFree(p));
    CK(hipFree(st));
    CK(hipFree(sink));
    return 0;
}
