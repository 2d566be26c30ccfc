// launchbench.hip -- what is K1's fixed per-launch cost made of?  (diagnostic,
// not part of libsketch).  Back-to-back launches on one stream, timed with
// events: an empty 1-wave kernel, an empty kernel with K1's shape (256 x 1024
// threads, 135 KiB dynamic LDS), the same shape staging a 135 KiB image by
// LDS-DMA (+ barrier), and the staging kernel again on two alternating
// streams and replayed from a hipGraph.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void k_empty(int *sink) {
    if (threadIdx.x == 12345) sink[0] = 1;
}

__global__ void __launch_bounds__(1024) k_shape(int *sink) {
    extern __shared__ unsigned char img[];
    if (threadIdx.x == 12345) sink[0] = img[0];
}

template <int P>
__global__ void __launch_bounds__(1024) k_stage(const unsigned char *src, unsigned nbytes, int *sink) {
    extern __shared__ __attribute__((aligned(16))) unsigned char img[];
    const unsigned wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char *>(src), 0, int(nbytes), 0x00020000);
#pragma unroll
    for (int j = 0; j < P; j++) {
        const unsigned p = wave + 16 * j;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void *)(img + p * 1024), 16, int(p * 1024 + lane * 16), 0, 0, 0);
    }
    __syncthreads();
    if (img[(threadIdx.x * 131) % (P * 16 * 1024)] == 0xEE && threadIdx.x == 99999) sink[0] = 1;
}

template <typename F>
static float time_it(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int i = 0; i < 5; i++) f(i);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; i++) f(i);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps * 1000.f;
}

int main() {
    int *sink; unsigned char *src;
    CK(hipMalloc(&sink, 64));
    const unsigned nbytes = 138240;
    CK(hipMalloc(&src, nbytes));
    CK(hipMemset(src, 0x5a, nbytes));
    CK(hipFuncSetAttribute((const void *)k_shape, hipFuncAttributeMaxDynamicSharedMemorySize, 152 * 1024));
    CK(hipFuncSetAttribute((const void *)k_stage<9>, hipFuncAttributeMaxDynamicSharedMemorySize, 152 * 1024));
    hipDeviceProp_t pr; CK(hipGetDeviceProperties(&pr, 0));
    const int cus = pr.multiProcessorCount;
    const size_t lds = 135 * 1024;
    printf("CUs=%d\n", cus);
    float t;
    t = time_it([&](int) { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, 0, sink); }, 500);
    printf("empty 1x64                      %7.2f us/launch\n", t);
    t = time_it([&](int) { hipLaunchKernelGGL(k_empty, dim3(cus), dim3(1024), 0, 0, sink); }, 500);
    printf("empty %dx1024, no LDS          %7.2f us/launch\n", cus, t);
    t = time_it([&](int) { hipLaunchKernelGGL(k_shape, dim3(cus), dim3(1024), lds, 0, sink); }, 500);
    printf("empty %dx1024, 135 KiB LDS     %7.2f us/launch\n", cus, t);
    t = time_it([&](int) { hipLaunchKernelGGL(k_stage<9>, dim3(cus), dim3(1024), lds, 0, src, nbytes, sink); }, 500);
    printf("stage 135 KiB by LDS-DMA        %7.2f us/launch\n", t);
    hipStream_t s2[2];
    CK(hipStreamCreateWithFlags(&s2[0], hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2[1], hipStreamNonBlocking));
    {
        hipEvent_t a, b;
        CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a, s2[0]));
        CK(hipStreamWaitEvent(s2[1], a, 0));
        for (int i = 0; i < 500; i++) hipLaunchKernelGGL(k_stage<9>, dim3(cus), dim3(1024), lds, s2[i & 1], src, nbytes, sink);
        hipEvent_t c; CK(hipEventCreate(&c)); CK(hipEventRecord(c, s2[1]));
        CK(hipStreamWaitEvent(s2[0], c, 0));
        CK(hipEventRecord(b, s2[0]));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        printf("stage, 2 alternating streams    %7.2f us/launch\n", ms / 500 * 1000.f);
    }
    {
        hipGraph_t g; hipGraphExec_t ge;
        hipStream_t cs; CK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
        CK(hipStreamBeginCapture(cs, hipStreamCaptureModeGlobal));
        for (int i = 0; i < 100; i++) hipLaunchKernelGGL(k_stage<9>, dim3(cus), dim3(1024), lds, cs, src, nbytes, sink);
        CK(hipStreamEndCapture(cs, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, cs));
        CK(hipStreamSynchronize(cs));
        hipEvent_t a, b;
        CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
        CK(hipEventRecord(a, cs));
        for (int i = 0; i < 5; i++) CK(hipGraphLaunch(ge, cs));
        CK(hipEventRecord(b, cs));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        printf("stage, hipGraph of 100 launches %7.2f us/launch\n", ms / 500 * 1000.f);
    }
    return 0;
}
