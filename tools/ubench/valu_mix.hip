// Microbenchmark: VALU issue cost per SIMD on gfx950 by instruction class and by waves per
// SIMD (W = 1..4), the numbers the class-weighted issue bound of the B/F sweep needs
// (is a 32-bit op -- DPP move, bfi, lshl_add -- 2 cycles across waves
// while fp64 is 4?).  Each kernel runs 8 independent chains (ILP 8) of a 16-instruction
// body; every wave times itself with s_memtime (shader clock, so DVFS does not enter) and
// the report is cycles per wave-instruction per SIMD = block elapsed (first start to last end
// of its waves) / (W * instructions per wave), median over blocks.  One block of 256 W threads
// per CU (each block allocates 96 KB of LDS, so no CU holds two): the block's waves are dealt
// round-robin over the CU's 4 SIMDs, so every SIMD holds exactly W waves for the whole run.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/valu_mix.hip -o tools/ubench/valu_mix
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define D8(I) I(d0) I(d1) I(d2) I(d3) I(d4) I(d5) I(d6) I(d7)
#define F8(I) I(f0) I(f1) I(f2) I(f3) I(f4) I(f5) I(f6) I(f7)

#define FMA64(x) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define MUL64(x) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(x) : "v"(b));
#define RSQ64(x) asm volatile("v_rsq_f64 %0, %0" : "+v"(x));
#define RCP64(x) asm volatile("v_rcp_f64 %0, %0" : "+v"(x));
#define DPP32(x) asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x));
#define AND32(x) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x) : "v"(k));
#define LSHLADD32(x) asm volatile("v_lshl_add_u32 %0, %0, 4, %1" : "+v"(x) : "v"(k));
#define BFI32(x) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(x) : "v"(k), "v"(k2));
#define FMA32(x) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(fb), "v"(fc));
#define CND32(x) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(k));
#define CNDS(x) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x) : "v"(k), "s"(smask));
#define MOV32(x) asm volatile("v_mov_b32 %0, %1" : "=v"(x) : "v"(x));
#define MOV64(x) asm volatile("v_mov_b64 %0, %1" : "=v"(x) : "v"(x));
#define MIN64(x) asm volatile("v_min_f64 %0, %0, %1" : "+v"(x) : "v"(b));
#define RSQ32(f) asm volatile("v_rsq_f32 %0, %0" : "+v"(f));
#define CVTF(x, f) asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(f) : "v"(x));
#define CVTD(x, f) asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(x) : "v"(f));

// 16-instruction bodies
#define BODY_fma64 D8(FMA64) D8(FMA64)
#define BODY_mul64 D8(MUL64) D8(MUL64)
#define BODY_rsq64 D8(RSQ64) D8(RSQ64)
#define BODY_rcp64 D8(RCP64) D8(RCP64)
#define BODY_dpp32 F8(DPP32) F8(DPP32)
#define BODY_and32 F8(AND32) F8(AND32)
#define BODY_lshladd32 F8(LSHLADD32) F8(LSHLADD32)
#define BODY_bfi32 F8(BFI32) F8(BFI32)
#define BODY_fma32 F8(FMA32) F8(FMA32)
#define BODY_cnd32 F8(CND32) F8(CND32)
#define BODY_cnds F8(CNDS) F8(CNDS)
#define BODY_mov32 F8(MOV32) F8(MOV32)
#define BODY_mov64 D8(MOV64) D8(MOV64)
#define BODY_min64 D8(MIN64) D8(MIN64)
#define BODY_fma64_cnds D8(FMA64) F8(CNDS)
// mixes (16 instructions each)
#define BODY_fma64_dpp32 D8(FMA64) F8(DPP32)
#define BODY_fma64_and32 D8(FMA64) F8(AND32)
#define BODY_fma64_bfi32 D8(FMA64) F8(BFI32)
#define BODY_fma64x3_dpp32 FMA64(d0) FMA64(d1) FMA64(d2) DPP32(f0) FMA64(d3) FMA64(d4) FMA64(d5) DPP32(f1) \
    FMA64(d6) FMA64(d7) FMA64(d0) DPP32(f2) FMA64(d1) FMA64(d2) FMA64(d3) DPP32(f3)
#define BODY_rsq64_fma64x7 RSQ64(d0) FMA64(d1) FMA64(d2) FMA64(d3) FMA64(d4) FMA64(d5) FMA64(d6) FMA64(d7) \
    RSQ64(d1) FMA64(d0) FMA64(d2) FMA64(d3) FMA64(d4) FMA64(d5) FMA64(d6) FMA64(d7)
// round 6: an fp64 reciprocal square root seeded through fp32 (cvt, v_rsq_f32, cvt) against v_rsq_f64
#define BODY_rsq32 F8(RSQ32) F8(RSQ32)
#define BODY_cvt_pair CVTF(d0, f0) CVTF(d1, f1) CVTF(d2, f2) CVTF(d3, f3) CVTF(d4, f4) CVTF(d5, f5) CVTF(d6, f6) \
    CVTF(d7, f7) CVTD(d0, f0) CVTD(d1, f1) CVTD(d2, f2) CVTD(d3, f3) CVTD(d4, f4) CVTD(d5, f5) CVTD(d6, f6) CVTD(d7, f7)
#define BODY_rsq32seq_fma64x5 CVTF(d0, f0) FMA64(d1) FMA64(d2) RSQ32(f0) FMA64(d3) FMA64(d4) CVTD(d0, f0) FMA64(d5) \
    CVTF(d6, f1) FMA64(d1) FMA64(d2) RSQ32(f1) FMA64(d3) FMA64(d4) CVTD(d6, f1) FMA64(d5)
// dependent pairs: 4 chains of fma64 (ILP 4) and 2 chains (ILP 2)
#define BODY_fma64_ilp4 FMA64(d0) FMA64(d1) FMA64(d2) FMA64(d3) FMA64(d0) FMA64(d1) FMA64(d2) FMA64(d3) \
    FMA64(d0) FMA64(d1) FMA64(d2) FMA64(d3) FMA64(d0) FMA64(d1) FMA64(d2) FMA64(d3)
#define BODY_fma64_ilp2 FMA64(d0) FMA64(d1) FMA64(d0) FMA64(d1) FMA64(d0) FMA64(d1) FMA64(d0) FMA64(d1) \
    FMA64(d0) FMA64(d1) FMA64(d0) FMA64(d1) FMA64(d0) FMA64(d1) FMA64(d0) FMA64(d1)
#define BODY_fma64_ilp1 FMA64(d0) FMA64(d0) FMA64(d0) FMA64(d0) FMA64(d0) FMA64(d0) FMA64(d0) FMA64(d0) \
    FMA64(d0) FMA64(d0) FMA64(d0) FMA64(d0) FMA64(d0) FMA64(d0) FMA64(d0) FMA64(d0)

#define KERNEL(NAME)                                                                                    \
    __global__ __launch_bounds__(1024) void k_##NAME(long long* cyc, double* out, int iters) {         \
        extern __shared__ double lds_pad[];                                                             \
        double d0 = threadIdx.x, d1 = d0 + 1, d2 = d0 + 2, d3 = d0 + 3, d4 = d0 + 4, d5 = d0 + 5,       \
               d6 = d0 + 6, d7 = d0 + 7, b = 1.0000001, c = 0.5;                                       \
        float f0 = threadIdx.x, f1 = f0 + 1, f2 = f0 + 2, f3 = f0 + 3, f4 = f0 + 4, f5 = f0 + 5,        \
              f6 = f0 + 6, f7 = f0 + 7, fb = 1.0000001f, fc = 0.5f;                                     \
        int k = 0x0f0f0f0f, k2 = (int)threadIdx.x;                                                      \
        unsigned long long smask = __ballot((threadIdx.x & 1) != 0);                                    \
        asm volatile("s_mov_b64 vcc, -1" ::: "vcc");                                                    \
        __syncthreads();                                                                                \
        const long long t0 = __builtin_readcyclecounter();                                              \
        for (int i = 0; i < iters; ++i) { BODY_##NAME }                                                 \
        const long long t1 = __builtin_readcyclecounter();                                              \
        if ((threadIdx.x & 63) == 0) {                                                                  \
            cyc[2 * (blockIdx.x * 16 + (threadIdx.x >> 6))] = t0;                                       \
            cyc[2 * (blockIdx.x * 16 + (threadIdx.x >> 6)) + 1] = t1;                                   \
        }                                                                                               \
        if (threadIdx.x == 0) lds_pad[0] = d0;                                                          \
        out[blockIdx.x * 1024 + threadIdx.x] = d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7 +                 \
                                              (double)(f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7) + k + k2; \
    }

KERNEL(fma64) KERNEL(mul64) KERNEL(rsq64) KERNEL(rcp64) KERNEL(dpp32) KERNEL(and32) KERNEL(lshladd32)
KERNEL(bfi32) KERNEL(fma32) KERNEL(cnd32) KERNEL(fma64_dpp32) KERNEL(fma64_and32) KERNEL(fma64_bfi32)
KERNEL(fma64x3_dpp32) KERNEL(rsq64_fma64x7) KERNEL(fma64_ilp4) KERNEL(fma64_ilp2) KERNEL(fma64_ilp1)
KERNEL(cnds) KERNEL(mov32) KERNEL(mov64) KERNEL(min64) KERNEL(fma64_cnds) KERNEL(rsq32) KERNEL(cvt_pair)
KERNEL(rsq32seq_fma64x5)

int main() {
    struct K { const char* n; void (*f)(long long*, double*, int); } ks[] = {
        {"fma64", k_fma64}, {"mul64", k_mul64}, {"rsq64", k_rsq64}, {"rcp64", k_rcp64},
        {"dpp32", k_dpp32}, {"and32", k_and32}, {"lshladd32", k_lshladd32}, {"bfi32", k_bfi32},
        {"fma32", k_fma32}, {"cnd32", k_cnd32}, {"fma64+dpp32 (1:1)", k_fma64_dpp32},
        {"fma64+and32 (1:1)", k_fma64_and32}, {"fma64+bfi32 (1:1)", k_fma64_bfi32},
        {"fma64x3+dpp32 (3:1)", k_fma64x3_dpp32}, {"rsq64+fma64x7 (1:7)", k_rsq64_fma64x7},
        {"fma64 ILP4", k_fma64_ilp4}, {"fma64 ILP2", k_fma64_ilp2}, {"fma64 ILP1", k_fma64_ilp1},
        {"cndmask_e64 (sgpr mask)", k_cnds}, {"mov32", k_mov32}, {"mov64", k_mov64}, {"min64", k_min64},
        {"fma64+cndmask_e64 (1:1)", k_fma64_cnds}, {"rsq32", k_rsq32}, {"cvt f64>f32>f64", k_cvt_pair},
        {"(cvt,rsq32,cvt)x2+fma64x10", k_rsq32seq_fma64x5}};
    const int cus = 256, iters = 2048;
    const size_t lds = 96 * 1024;
    long long* cyc;
    double* out;
    (void)hipMalloc(&cyc, cus * 16 * 2 * sizeof(long long));
    (void)hipMalloc(&out, cus * 1024 * sizeof(double));
    std::vector<long long> h(cus * 16 * 2);
    printf("cycles per wave-instruction per SIMD (s_memtime; one block per CU, W waves per SIMD; median over "
           "blocks; 16 instr x %d iters per wave)\n", iters);
    printf("%-22s %8s %8s %8s %8s\n", "body", "W=1", "W=2", "W=3", "W=4");
    for (auto& k : ks) {
        (void)hipFuncSetAttribute((const void*)k.f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        printf("%-22s", k.n);
        for (int W = 1; W <= 4; ++W) {
            const int threads = 256 * W, waves = 4 * W;
            hipLaunchKernelGGL(k.f, dim3(cus), dim3(threads), lds, 0, cyc, out, 64);  // warm
            hipLaunchKernelGGL(k.f, dim3(cus), dim3(threads), lds, 0, cyc, out, iters);
            (void)hipMemcpy(h.data(), cyc, h.size() * sizeof(long long), hipMemcpyDeviceToHost);
            std::vector<double> per;
            for (int b = 0; b < cus; ++b) {
                long long lo = h[2 * (b * 16)], hi = h[2 * (b * 16) + 1];
                for (int w = 1; w < waves; ++w) {
                    lo = std::min(lo, h[2 * (b * 16 + w)]);
                    hi = std::max(hi, h[2 * (b * 16 + w) + 1]);
                }
                per.push_back((double)(hi - lo) / ((double)W * iters * 16));
            }
            std::nth_element(per.begin(), per.begin() + per.size() / 2, per.end());
            printf(" %8.2f", per[per.size() / 2]);
        }
        printf("\n");
    }
    return 0;
}
