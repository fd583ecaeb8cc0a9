// Microbenchmark: dependent-chain latency and one-wave issue cost of the instructions
// the B/F sweep is made of, on gfx950.  One workgroup of one wave on one CU; the
// cycle counter (s_memtime) brackets 512 instructions in inline asm:
//   dep  : one chain, each instruction reads the previous result  -> latency
//   ind8 : eight independent chains interleaved                   -> one wave's issue cost
// Prints cycles per instruction.  Speed-only diagnostic.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define R8(X) X X X X X X X X
#define R64(X) R8(R8(X))

#define DEP_KERNEL(NAME, INSN)                                                     \
    __global__ void NAME(double* out, long long* cyc) {                            \
        double a = threadIdx.x * 1e-3 + 1.0, b = 1.0000001, c = 0.5;             \
        __builtin_amdgcn_s_waitcnt(0);                                            \
        long long t0 = __builtin_amdgcn_s_memtime();                              \
        R8(R64(asm volatile(INSN : "+v"(a) : "v"(b), "v"(c));))                   \
        long long t1 = __builtin_amdgcn_s_memtime();                              \
        out[threadIdx.x] = a;                                                     \
        if (threadIdx.x == 0) cyc[0] = t1 - t0;                                   \
    }

#define IND_KERNEL(NAME, INSN)                                                                        \
    __global__ void NAME(double* out, long long* cyc) {                                               \
        double a0 = threadIdx.x + 1.0, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, \
               a6 = a0 + 6, a7 = a0 + 7, b = 1.0000001, c = 0.5;                                     \
        long long t0 = __builtin_amdgcn_s_memtime();                                                 \
        R64(asm volatile(INSN : "+v"(a0) : "v"(b), "v"(c)); asm volatile(INSN : "+v"(a1) : "v"(b), "v"(c)); \
            asm volatile(INSN : "+v"(a2) : "v"(b), "v"(c)); asm volatile(INSN : "+v"(a3) : "v"(b), "v"(c)); \
            asm volatile(INSN : "+v"(a4) : "v"(b), "v"(c)); asm volatile(INSN : "+v"(a5) : "v"(b), "v"(c)); \
            asm volatile(INSN : "+v"(a6) : "v"(b), "v"(c)); asm volatile(INSN : "+v"(a7) : "v"(b), "v"(c));) \
        long long t1 = __builtin_amdgcn_s_memtime();                                                 \
        out[threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;                                   \
        if (threadIdx.x == 0) cyc[0] = t1 - t0;                                                      \
    }

#define DEP32(NAME, INSN)                                                          \
    __global__ void NAME(double* out, long long* cyc) {                            \
        int a = threadIdx.x + 1, b = 3, c = 5;                                    \
        long long t0 = __builtin_amdgcn_s_memtime();                              \
        R8(R64(asm volatile(INSN : "+v"(a) : "v"(b), "v"(c));))                   \
        long long t1 = __builtin_amdgcn_s_memtime();                              \
        out[threadIdx.x] = a;                                                     \
        if (threadIdx.x == 0) cyc[0] = t1 - t0;                                   \
    }
#define IND32(NAME, INSN)                                                                             \
    __global__ void NAME(double* out, long long* cyc) {                                               \
        int a0 = threadIdx.x + 1, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,    \
            a6 = a0 + 6, a7 = a0 + 7, b = 3, c = 5;                                                  \
        long long t0 = __builtin_amdgcn_s_memtime();                                                 \
        R64(asm volatile(INSN : "+v"(a0) : "v"(b), "v"(c)); asm volatile(INSN : "+v"(a1) : "v"(b), "v"(c)); \
            asm volatile(INSN : "+v"(a2) : "v"(b), "v"(c)); asm volatile(INSN : "+v"(a3) : "v"(b), "v"(c)); \
            asm volatile(INSN : "+v"(a4) : "v"(b), "v"(c)); asm volatile(INSN : "+v"(a5) : "v"(b), "v"(c)); \
            asm volatile(INSN : "+v"(a6) : "v"(b), "v"(c)); asm volatile(INSN : "+v"(a7) : "v"(b), "v"(c));) \
        long long t1 = __builtin_amdgcn_s_memtime();                                                 \
        out[threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;                                   \
        if (threadIdx.x == 0) cyc[0] = t1 - t0;                                                      \
    }

DEP_KERNEL(d_fma, "v_fma_f64 %0, %0, %1, %2")
DEP_KERNEL(d_mul, "v_mul_f64 %0, %0, %1")
DEP_KERNEL(d_add, "v_add_f64 %0, %0, %1")
DEP_KERNEL(d_rsq, "v_rsq_f64 %0, %0")
DEP_KERNEL(d_min, "v_min_f64 %0, %0, %1")
DEP32(d_dpp, "v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1")
IND_KERNEL(i_fma, "v_fma_f64 %0, %0, %1, %2")
IND_KERNEL(i_mul, "v_mul_f64 %0, %0, %1")
IND_KERNEL(i_add, "v_add_f64 %0, %0, %1")
IND_KERNEL(i_rsq, "v_rsq_f64 %0, %0")
IND32(i_dpp, "v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1")
IND32(i_and, "v_and_b32 %0, %0, %1")
DEP32(d_and, "v_and_b32 %0, %0, %1")
DEP32(d_cnd, "v_cndmask_b32 %0, %0, %1, vcc")

IND32(i_rsq32, "v_rsq_f32 %0, %0")
IND_KERNEL(i_sqrt64, "v_sqrt_f64 %0, %0")
IND_KERNEL(i_rcp64, "v_rcp_f64 %0, %0")
// one transcendental + three independent FMAs per group: does v_rsq_f64 overlap plain VALU?
__global__ void mix_rsq_fma(double* out, long long* cyc) {
    double a0 = threadIdx.x + 1.0, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, b = 1.0000001, c = 0.5;
    long long t0 = __builtin_amdgcn_s_memtime();
    R64(asm volatile("v_rsq_f64 %0, %0" : "+v"(a0)); asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a1) : "v"(b), "v"(c));
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a2) : "v"(b), "v"(c));
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a3) : "v"(b), "v"(c));
        asm volatile("v_rsq_f64 %0, %0" : "+v"(a0)); asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a1) : "v"(b), "v"(c));
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a2) : "v"(b), "v"(c));
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a3) : "v"(b), "v"(c));)
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a0 + a1 + a2 + a3;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    double* out;
    long long* cyc;
    if (hipMalloc(&out, 64 * sizeof(double)) != hipSuccess || hipMalloc(&cyc, sizeof(long long)) != hipSuccess) return 1;
    struct K {
        const char* n;
        void (*f)(double*, long long*);
        int insts;
    } ks[] = {{"dep v_fma_f64", d_fma, 512}, {"dep v_mul_f64", d_mul, 512}, {"dep v_add_f64", d_add, 512},
              {"dep v_rsq_f64", d_rsq, 512}, {"dep v_min_f64", d_min, 512}, {"dep v_mov_b32_dpp", d_dpp, 512},
              {"ind8 v_fma_f64", i_fma, 512}, {"ind8 v_mul_f64", i_mul, 512}, {"ind8 v_add_f64", i_add, 512},
              {"ind8 v_rsq_f64", i_rsq, 512}, {"ind8 v_mov_b32_dpp", i_dpp, 512}, {"ind8 v_and_b32", i_and, 512}, {"dep v_and_b32", d_and, 512}, {"dep v_cndmask_b32", d_cnd, 512},
              {"ind8 v_rsq_f32", i_rsq32, 512}, {"ind8 v_sqrt_f64", i_sqrt64, 512}, {"ind8 v_rcp_f64", i_rcp64, 512},
              {"mix rsq_f64+3 fma (per group of 4)", mix_rsq_fma, 128}};
    for (auto& k : ks) {
        long long best = -1;
        for (int rep = 0; rep < 5; ++rep) {
            hipLaunchKernelGGL(k.f, dim3(1), dim3(64), 0, 0, out, cyc);
            long long c;
            if (hipMemcpy(&c, cyc, sizeof c, hipMemcpyDeviceToHost) != hipSuccess) return 1;
            if (best < 0 || c < best) best = c;
        }
        printf("%-22s %6.2f cycles/instr (s_memtime ticks, best of 5)\n", k.n, (double)best / k.insts);
    }
    return 0;
}
