// fp64 elementary functions for the NNGP covariance / Cholesky kernels.
//
// The covariance plug-in (pyNNGP/nngp.py:6,12 -- `cov`, called at :82 and :96)
// is evaluated ~m(m+1)/2 times per location, so exp and sqrt dominate the
// B/F sweep.  These versions are branch-free and specialised to the ranges the
// sweep uses, each within ~1.5 ulp:
//   * sigma2 exp(-phi d) = sigma2 2^(x/256), x = -256 phi log2(e) d, split as
//     x = 256 n + j + f (|f| <= 1/2, 0 <= j < 256): one FMA against the 1.5*2^52
//     "magic" constant rounds x to the integer k = 256 n + j (its low dword IS k),
//     one FMA gives f, a degree-4 polynomial gives 2^(f/256), a 256-entry table
//     (sigma2 2^(j/256), in LDS) and one ldexp finish it.  11 VALU ops + 1 LDS read
//     instead of the 16 of a degree-11 polynomial on |f| <= 1/2.
//   * d = sqrt(d2) and 1/sqrt(pivot): v_rsq_f64 plus a second-order correction
//     (below); d2 carries a 2^-1000 floor from the distance FMA, so no clamp is
//     needed against d2 == 0 (exp(-phi 2^-500) == 1 in fp64).
// The exponent is bounded by clamping d2 at d2max, where sigma2 2^-1080 has
// underflowed; far-away padding points (nngp_internal.h) land there.
// The same source compiles on the host (NNGP_MATH_HOST) so
// tests/test_math_host.py measures the ulp error against libm without a GPU.
#pragma once

#include "exp2_table.h"

#ifdef NNGP_MATH_HOST
#include <math.h>
#include <string.h>
#include <stdint.h>
#define NNGP_FN static inline
#define NNGP_HD static inline
static inline double nngp_rsq_approx(double x) {
    // emulate v_rsq_f64's relative error (measured on gfx950: up to 2^-24.2,
    // tools/ubench/rsq_acc.hip) with either sign, so the refinement is tested at it
    double y = 1.0 / sqrt(x);
    uint64_t u;
    memcpy(&u, &x, 8);
    return y * ((u >> 7) & 1 ? 1.0 + 0x1p-24 : 1.0 - 0x1p-24);
}
static inline int32_t nngp_lo_dword(double t) {
    uint64_t u;
    memcpy(&u, &t, 8);
    return (int32_t)(uint32_t)u;
}
static const double kExp2Tab[256] = NNGP_EXP2_TAB;
#else
#include <hip/hip_runtime.h>
#define NNGP_FN __device__ __forceinline__
#define NNGP_HD __host__ __device__ __forceinline__
NNGP_FN double nngp_rsq_approx(double x) { return __builtin_amdgcn_rsq(x); }
NNGP_FN int32_t nngp_lo_dword(double t) { return (int32_t)(uint32_t)(__double_as_longlong(t) & 0xffffffffll); }
static __device__ const double kExp2Tab[256] = NNGP_EXP2_TAB;
#endif

#define NNGP_LOG2E 0x1.71547652b82fep+0
#define NNGP_EXP_MAGIC 0x1.8p52
#define NNGP_D2_FLOOR 0x1p-1000
#define NNGP_EXP_TAB_N 256

// Covariance parameters, built once on the host (nngp_cov_params) and passed by value.
struct CovParams {
    double q[4];     // (2^(f/256) - 1) / f ~= q0 + q1 f + q2 f^2 + q3 f^3, |f| <= 1/2
    double nphi256;  // -256 phi log2(e): table units of the exponent per unit distance
    double d2max;    // squared distance at which sigma2 2^(nphi256 d / 256) has underflowed
    double phi;      // phi (Matern-3/2 needs phi d)
    double diag;     // sigma2 + tau2
    double sigma2;
};

NNGP_HD CovParams nngp_cov_params(double sigma2, double phi, double tau2) {
    const double q[4] = NNGP_EXP2_Q;
    CovParams p;
    for (int k = 0; k < 4; ++k) p.q[k] = q[k];
    p.nphi256 = -256.0 * (phi * NNGP_LOG2E);
    const double dmax = 1080.0 / (phi * NNGP_LOG2E);  // 2^-1080 sigma2 == 0 (or a negligible subnormal)
    p.d2max = dmax * dmax;
    p.phi = phi;
    p.diag = sigma2 + tau2;
    p.sigma2 = sigma2;
    return p;
}

#ifndef NNGP_MATH_HOST
// Fill the block's LDS table tab[j] = sigma2 2^(j/256) (every thread of the block calls it).
NNGP_FN void nngp_exp_table_load(double* tab, double sigma2) {
    for (int j = threadIdx.x; j < NNGP_EXP_TAB_N; j += blockDim.x) tab[j] = sigma2 * kExp2Tab[j];
    __syncthreads();
}
#else
static inline void nngp_exp_table_load(double* tab, double sigma2) {
    for (int j = 0; j < NNGP_EXP_TAB_N; ++j) tab[j] = sigma2 * kExp2Tab[j];
}
#endif

// sigma2 2^(nphi256 d / 256) for 0 <= nphi256 d / 256 ... i.e. d in [0, sqrt(d2max)]
NNGP_FN double nngp_exp_tab(const CovParams& P, const double* tab, double d) {
    const double t = fma(P.nphi256, d, NNGP_EXP_MAGIC);  // 1.5 2^52 + k, k = rint(nphi256 d)
    const double k = t - NNGP_EXP_MAGIC;                  // exact
    const double f = fma(P.nphi256, d, -k);               // |f| <= 1/2
    const int32_t ki = nngp_lo_dword(t);                  // k as an integer
    const double T = tab[ki & (NNGP_EXP_TAB_N - 1)];      // sigma2 2^(j/256)
    double q = fma(P.q[3], f, P.q[2]);
    q = fma(q, f, P.q[1]);
    q = fma(q, f, P.q[0]);
    const double fq = f * q;                              // 2^(f/256) - 1
    return ldexp(fma(T, fq, T), ki >> 8);                 // floor(k / 256)
}

// v_rsq_f64 is only good to ~2^-24 (measured), so one plain Newton step would leave
// ~1.5 * 2^-48 relative error.  Both refinements instead use the second-order series
// in e = 1 - x y^2 (|e| ~ 2^-23; the e^3 term is below 2^-66):
//   sqrt(x)   = s (1 - e')^(-1/2), s = x y, e' = 1 - s y:  s (1 + e'/2 + 3 e'^2 / 8)
//   1/sqrt(x) = y (1 - e)^(-1/2)                        :  y (1 + e/2 + 3 e^2 / 8)
// 5 ops each (one plain Newton step is 4; two are 8), within ~1 ulp.

// sqrt(x) for x >= 2^-1000
NNGP_FN double nngp_sqrt(double x) {
    const double y = nngp_rsq_approx(x);
    const double s = x * y;
    const double e = fma(-s, y, 1.0);
    const double g = e * fma(0.375, e, 0.5);
    return fma(s, g, s);
}

// 1/sqrt(x) for a positive pivot
NNGP_FN double nngp_rsqrt(double x) {
    const double y = nngp_rsq_approx(x);
    const double e = fma(-(x * y), y, 1.0);
    const double g = e * fma(0.375, e, 0.5);
    return fma(y, g, y);
}

// Covariance kinds (the reference's `cov` plug-in, nngp.py:6,12):
//   0 exponential  sigma2 * exp(-phi d)
//   1 matern32     sigma2 * (1 + phi d) * exp(-phi d)
// d2 from nngp_d2 (>= 2^-1000); tab from nngp_exp_table_load(tab, P.sigma2).
template <int KIND>
NNGP_FN double nngp_cov_d2(const CovParams& P, const double* tab, double d2) {
    const double d = nngp_sqrt(fmin(d2, P.d2max));
    const double e = nngp_exp_tab(P, tab, d);
    if (KIND == 1) {
        const double pd = P.phi * d;
        return fma(pd, e, e);
    }
    return e;
}

// squared Euclidean distance between two points, floored at 2^-1000 (exact otherwise:
// dy^2 + 2^-1000 rounds to dy^2 unless dy^2 < 2^-947)
NNGP_FN double nngp_d2(double ax, double ay, double bx, double by) {
    const double dx = ax - bx;
    const double dy = ay - by;
    return fma(dx, dx, fma(dy, dy, NNGP_D2_FLOOR));
}
