// valurate.hip -- issue cost of the VALU instructions K1 is made of, on
// gfx950 (diagnostic, not part of libsketch).  Each kernel runs a loop of 16
// independent instances of one instruction per iteration in every wave of a
// full chip (256 CUs x 8 waves per SIMD); reports cycles per wave-instruction
// per SIMD (clock from s_memtime inside the kernel).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int kIters = 2048;

#define REP16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

template <int OP>
__global__ void __launch_bounds__(256) k_rate(unsigned *out, unsigned long long *clk, unsigned seed) {
    unsigned v[16], w[16];
    unsigned long long q[16];
    double f[16];
#pragma unroll
    for (int i = 0; i < 16; i++) {
        v[i] = threadIdx.x * 7 + i + seed;
        w[i] = v[i] ^ 0x9e3779b9u;
        q[i] = (unsigned long long)v[i] << 20 | w[i];
        f[i] = double(v[i]);
    }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; it++) {
#define OPV(i)                                                                                     \
    if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[i]) : "v"(w[i]));       \
    if constexpr (OP == 1) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(v[i]) : "v"(w[i]));   \
    if constexpr (OP == 2) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(v[i]) : "v"(w[i]));   \
    if constexpr (OP == 3) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(q[i]) : "v"(v[i]), "v"(w[i]) : "vcc"); \
    if constexpr (OP == 4) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(q[i]) : "v"(q[(i + 1) & 15])); \
    if constexpr (OP == 5) asm volatile("v_fma_f64 %0, %0, %0, %0" : "+v"(f[i]));                \
    if constexpr (OP == 6) asm volatile("v_cmp_lt_u64 vcc, %0, %1" :: "v"(q[i]), "v"(q[(i + 1) & 15]) : "vcc"); \
    if constexpr (OP == 7) asm volatile("v_alignbit_b32 %0, %0, %1, %1" : "+v"(v[i]) : "v"(w[i])); \
    if constexpr (OP == 8) asm volatile("v_lshrrev_b64 %0, 15, %0" : "+v"(q[i]));
        REP16(OPV)
#undef OPV
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned acc = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) acc ^= v[i] ^ unsigned(q[i]) ^ unsigned(f[i]);
    if (acc == 0x12345678u) out[0] = acc;
    if (threadIdx.x == 0) atomicMax(clk, t1 - t0);
}

static const char *names[] = {"v_add_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32",
                              "v_lshl_add_u64", "v_fma_f64", "v_cmp_lt_u64", "v_alignbit_b32",
                              "v_lshrrev_b64"};

template <int OP>
static void run(int cus, unsigned *out, unsigned long long *clk) {
    CK(hipMemset(clk, 0, 8));
    const int blocks = cus * 8;  // 8 x 256 threads per CU = 8 waves per SIMD
    hipLaunchKernelGGL(k_rate<OP>, dim3(blocks), dim3(256), 0, 0, out, clk, 1u);
    CK(hipDeviceSynchronize());
    CK(hipMemset(clk, 0, 8));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL(k_rate<OP>, dim3(blocks), dim3(256), 0, 0, out, clk, 2u);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    unsigned long long c; CK(hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost));
    // per SIMD: 8 waves x kIters x 16 instructions
    const double instr_per_simd = 8.0 * kIters * 16;
    printf("%-16s %6.2f cyc/wave-instr/SIMD (s_memtime)   %6.2f ns/instr/SIMD (events %.3f ms)\n",
           names[OP], double(c) / instr_per_simd, ms * 1e6 / instr_per_simd, ms);
}

int main() {
    unsigned *out; unsigned long long *clk;
    CK(hipMalloc(&out, 64)); CK(hipMalloc(&clk, 64));
    hipDeviceProp_t pr; CK(hipGetDeviceProperties(&pr, 0));
    printf("CUs=%d clock %d kHz\n", pr.multiProcessorCount, pr.clockRate);
    run<0>(pr.multiProcessorCount, out, clk);
    run<1>(pr.multiProcessorCount, out, clk);
    run<2>(pr.multiProcessorCount, out, clk);
    run<3>(pr.multiProcessorCount, out, clk);
    run<4>(pr.multiProcessorCount, out, clk);
    run<5>(pr.multiProcessorCount, out, clk);
    run<6>(pr.multiProcessorCount, out, clk);
    run<7>(pr.multiProcessorCount, out, clk);
    run<8>(pr.multiProcessorCount, out, clk);
    return 0;
}
