// Microbenchmark: issue cost of the fp64 VALU instructions the B/F sweep uses,
// on gfx950.  Each kernel runs 8 independent chains of one instruction in a
// loop (inline asm so nothing is folded), 256 CUs x 8 waves; prints cycles per
// wave-instruction per SIMD = elapsed_cycles * SIMDs / instructions.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CHAIN8(INSN)                                                                                  \
    asm volatile(INSN : "+v"(a0) : "v"(b), "v"(c)); asm volatile(INSN : "+v"(a1) : "v"(b), "v"(c)); \
    asm volatile(INSN : "+v"(a2) : "v"(b), "v"(c)); asm volatile(INSN : "+v"(a3) : "v"(b), "v"(c)); \
    asm volatile(INSN : "+v"(a4) : "v"(b), "v"(c)); asm volatile(INSN : "+v"(a5) : "v"(b), "v"(c)); \
    asm volatile(INSN : "+v"(a6) : "v"(b), "v"(c)); asm volatile(INSN : "+v"(a7) : "v"(b), "v"(c));

#define KERNEL(NAME, INSN)                                                              \
    __global__ __launch_bounds__(256) void NAME(double* out, int iters) {               \
        double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,    \
               a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, b = 1.0000001, c = 0.5;           \
        for (int i = 0; i < iters; ++i) { CHAIN8(INSN) CHAIN8(INSN) }                   \
        out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;   \
    }

#define KERNEL32(NAME, INSN)                                                            \
    __global__ __launch_bounds__(256) void NAME(double* out, int iters) {               \
        float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,     \
              a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, b = 1.0000001f, c = 0.5f;         \
        for (int i = 0; i < iters; ++i) { CHAIN8(INSN) CHAIN8(INSN) }                   \
        out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;   \
    }
#define CHAIN8_LD(INSN)                                                                                \
    asm volatile(INSN : "+v"(a0) : "v"(e)); asm volatile(INSN : "+v"(a1) : "v"(e));                  \
    asm volatile(INSN : "+v"(a2) : "v"(e)); asm volatile(INSN : "+v"(a3) : "v"(e));                  \
    asm volatile(INSN : "+v"(a4) : "v"(e)); asm volatile(INSN : "+v"(a5) : "v"(e));                  \
    asm volatile(INSN : "+v"(a6) : "v"(e)); asm volatile(INSN : "+v"(a7) : "v"(e));
#define CHAIN8_CVT(INSN)                                                                               \
    asm volatile(INSN : "=v"(r0) : "v"(a0)); asm volatile(INSN : "=v"(r1) : "v"(a1));                \
    asm volatile(INSN : "=v"(r2) : "v"(a2)); asm volatile(INSN : "=v"(r3) : "v"(a3));                \
    asm volatile(INSN : "=v"(r4) : "v"(a4)); asm volatile(INSN : "=v"(r5) : "v"(a5));                \
    asm volatile(INSN : "=v"(r6) : "v"(a6)); asm volatile(INSN : "=v"(r7) : "v"(a7));

KERNEL(k_fma, "v_fma_f64 %0, %0, %1, %2")
KERNEL(k_mul, "v_mul_f64 %0, %0, %1")
KERNEL(k_add, "v_add_f64 %0, %0, %1")
KERNEL(k_max, "v_max_f64 %0, %0, %1")
KERNEL(k_rndne, "v_rndne_f64 %0, %0")
KERNEL(k_rsq, "v_rsq_f64 %0, %0")
__global__ __launch_bounds__(256) void k_ldexp(double* out, int iters) {
    double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    int e = 0;
    for (int i = 0; i < iters; ++i) { CHAIN8_LD("v_ldexp_f64 %0, %0, %1") CHAIN8_LD("v_ldexp_f64 %0, %0, %1") }
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}
KERNEL(k_fract, "v_fract_f64 %0, %0")
KERNEL32(k_fma_f32, "v_fma_f32 %0, %0, %1, %2")
KERNEL32(k_mov_dpp, "v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1")
KERNEL32(k_cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
__global__ __launch_bounds__(256) void k_cvt(double* out, int iters) {
    double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    int r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0, r5 = 0, r6 = 0, r7 = 0;
    for (int i = 0; i < iters; ++i) { CHAIN8_CVT("v_cvt_i32_f64 %0, %1") CHAIN8_CVT("v_cvt_i32_f64 %0, %1") }
    out[blockIdx.x * 256 + threadIdx.x] = r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7;
}

int main() {
    double* out;
    hipMalloc(&out, 256 * 256 * 8 * sizeof(double));
    int cus = 256, wpb = 4, blocks = cus * 2;  // 8 waves per CU = 2 per SIMD
    const int iters = 4096;
    struct K { const char* n; void (*f)(double*, int); } ks[] = {
        {"v_fma_f64", k_fma}, {"v_mul_f64", k_mul}, {"v_add_f64", k_add}, {"v_max_f64", k_max},
        {"v_rndne_f64", k_rndne}, {"v_rsq_f64", k_rsq}, {"v_ldexp_f64", k_ldexp}, {"v_fract_f64", k_fract},
        {"v_fma_f32", k_fma_f32}, {"v_mov_b32_dpp", k_mov_dpp}, {"v_cvt_i32_f64", k_cvt}, {"v_cndmask_b32", k_cndmask}};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    int clk_khz = 0;
    hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
    for (auto& k : ks) {
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 64);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        double winsts = (double)blocks * wpb * iters * 16;  // wave-instructions
        double simd_cycles = ms * 1e-3 * 2.4e9 * cus * 4;  // at 2.4 GHz
        printf("%-16s %.3f ms  %.2f cycles/wave-instr/SIMD (at 2.4 GHz)\n", k.n, ms, simd_cycles / winsts);
    }
    printf("clock attr %d kHz\n", clk_khz);
    return 0;
}
