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

// Covariance kinds (the reference's `cov` plug-in, nngp.py:6,12; the spNNGP family), u = phi d:
#define NNGP_KIND_EXPONENTIAL 0  // sigma2 e^-u
#define NNGP_KIND_MATERN32 1     // sigma2 (1 + u) e^-u
#define NNGP_KIND_MATERN52 2     // sigma2 (1 + u + u^2 / 3) e^-u
#define NNGP_KIND_GAUSSIAN 3     // sigma2 e^-u^2          (no square root: the exponent is phi^2 d^2)
#define NNGP_KIND_SPHERICAL 4    // sigma2 (1 - 3u/2 + u^3/2) for u < 1, else 0   (no exponential)
#define NNGP_N_KINDS 5
// Runtime kind (the m = 25..32 kernels, one instantiation for all five kinds): every kind as
// p(u) e, p(u) = 1 + c1 u + c2 u^2 + c3 u^3 with u = min(phi d, umax), e = 2^(nphi256 g / 256) with
// g = d (g = d^2 for the gaussian kind; nphi256 = 0, i.e. e = 1, for the spherical kind).
#define NNGP_KIND_GENERIC 5

// Covariance parameters, built once on the host (nngp_cov_params) and passed by value.
struct CovParams {
    double q[4];     // (2^(f/256) - 1) / f ~= q0 + q1 f + q2 f^2 + q3 f^3, |f| <= 1/2
    double nphi256;  // table units of the exponent per unit of its variable: -256 log2(e) phi
                     // (variable d) or -256 log2(e) phi^2 (gaussian: variable d^2)
    double d2max;    // squared distance beyond which the covariance is 0 (underflowed / past the range)
    double phi;
    double diag;     // sigma2 + tau2
    double sigma2;
    double c[3];     // NNGP_KIND_GENERIC: polynomial coefficients c1, c2, c3 of the kind
    double umax;     // NNGP_KIND_GENERIC: u = phi d is clamped at umax (1 for the spherical kind)
    int gauss;       // NNGP_KIND_GENERIC: the exponent's variable is d^2 (gaussian), else d
};

NNGP_HD CovParams nngp_cov_params(int kind, double sigma2, double phi, double tau2) {
    const double q[4] = NNGP_EXP2_Q;
    CovParams p;
    for (int k = 0; k < 4; ++k) p.q[k] = q[k];
    if (kind == NNGP_KIND_GAUSSIAN) {
        p.nphi256 = -256.0 * (phi * phi * NNGP_LOG2E);
        p.d2max = 1080.0 / (phi * phi * NNGP_LOG2E);  // sigma2 2^-1080: zero (or a negligible subnormal)
    } else if (kind == NNGP_KIND_SPHERICAL) {
        p.nphi256 = 0.0;
        p.d2max = 4.0 / (phi * phi);  // any d2 past (1/phi)^2 gives 0; the clamp keeps sqrt in range
    } else {
        p.nphi256 = -256.0 * (phi * NNGP_LOG2E);
        // 2^-1080 sigma2 == 0; the polynomial factor of the Matern kinds (<= 1 + u + u^2/3 at
        // u ~ 750) leaves it a subnormal far below any pivot
        const double dmax = 1080.0 / (phi * NNGP_LOG2E);
        p.d2max = dmax * dmax;
    }
    p.phi = phi;
    p.diag = sigma2 + tau2;
    p.sigma2 = sigma2;
    p.c[0] = kind == NNGP_KIND_MATERN32 || kind == NNGP_KIND_MATERN52 ? 1.0 : kind == NNGP_KIND_SPHERICAL ? -1.5 : 0.0;
    p.c[1] = kind == NNGP_KIND_MATERN52 ? 1.0 / 3.0 : 0.0;
    p.c[2] = kind == NNGP_KIND_SPHERICAL ? 0.5 : 0.0;
    p.umax = kind == NNGP_KIND_SPHERICAL ? 1.0 : 1e300;
    p.gauss = kind == NNGP_KIND_GAUSSIAN;
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

// Covariance of kind KIND (NNGP_KIND_*) at squared distance d2 (from nngp_d2, >= 2^-1000);
// tab from nngp_exp_table_load(tab, P.sigma2) (unused by the spherical kind).
template <int KIND>
NNGP_FN double nngp_cov_d2(const CovParams& P, const double* tab, double d2) {
    const double x = fmin(d2, P.d2max);
    if (KIND == NNGP_KIND_GAUSSIAN) return nngp_exp_tab(P, tab, x);  // sigma2 2^(nphi256 d2 / 256)
    const double d = nngp_sqrt(x);
    if (KIND == NNGP_KIND_GENERIC) {  // runtime kind (nngp_cov_unit's generic branch, sigma2 in the table)
        const double e = nngp_exp_tab(P, tab, P.gauss ? x : d);
        const double u = fmin(P.phi * d, P.umax);
        return fma(u, fma(u, fma(u, P.c[2], P.c[1]), P.c[0]), 1.0) * e;
    }
    if (KIND == NNGP_KIND_SPHERICAL) {
        const double u = fmin(P.phi * d, 1.0);                       // u = 1: the polynomial is exactly 0
        const double p = fma(u, fma(0.5 * u, u, -1.5), 1.0);         // 1 + u (u^2 / 2 - 3/2)
        return P.sigma2 * p;
    }
    const double e = nngp_exp_tab(P, tab, d);
    if (KIND == NNGP_KIND_MATERN32) {
        const double pd = P.phi * d;
        return fma(pd, e, e);
    }
    if (KIND == NNGP_KIND_MATERN52) {
        const double u = P.phi * d;
        const double p = fma(fma(u, 1.0 / 3.0, 1.0), u, 1.0);       // 1 + u + u^2 / 3
        return p * e;
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

// ---------------------------------------------------------------- unit-variance covariances
// The persistent kernels (bf_pairb) factor the unit-variance block R + (tau2 / sigma2) I and
// scale F by sigma2 at the end (B and the value residual are scale-invariant).  With unit
// variance every table entry 2^(j/256) lies in [1, 2), so 2^n can be applied by adding n to
// the exponent field instead of an ldexp: the LDS table stores 2^(j/256) with (j << 12)
// pre-subtracted from its high dword, and for k = 256 n + j the high dword of
// 2^(j/256) 2^n is (stored high dword) + (k << 12) -- one v_lshl_add_u32 instead of an
// ashr + v_ldexp_f64.  The exponent argument is clamped so that n >= -1023 (below).
//
// The clamp sits at k = -261888.25 (rounded: -1023 * 256, table entry j = 0): there the high
// dword is exactly 0 and the covariance is +0.0, so far-away padding points decouple EXACTLY
// (their rows and columns stay 0 through the elimination and B is 0 in padded slots without a
// mask; the 1/4 margin absorbs the rounding of phi, d2max and the square root).  Between
// k = -261887 and -261633 (n = -1023) the exponent field is 0 and the entry reads as a subnormal
// below 2^-1022 -- a covariance that small is 0 for every purpose of the factorisation.
#define NNGP_UNIT_CLAMP (1023.0 + 1.0 / 1024.0)
NNGP_HD CovParams nngp_cov_params_unit(int kind, double phi, double tau2_over_sigma2) {
    CovParams p = nngp_cov_params(kind, 1.0, phi, tau2_over_sigma2);
    if (kind == NNGP_KIND_GAUSSIAN) {
        p.d2max = NNGP_UNIT_CLAMP / (phi * phi * NNGP_LOG2E);
    } else if (kind != NNGP_KIND_SPHERICAL) {
        const double dmax = NNGP_UNIT_CLAMP / (phi * NNGP_LOG2E);
        p.d2max = dmax * dmax;
    }
    return p;
}

NNGP_FN double nngp_exp_unit(const CovParams& P, const double* tab, double u) {
    const double t = fma(P.nphi256, u, NNGP_EXP_MAGIC);  // 1.5 2^52 + k, k = rint(nphi256 u) >= -1021 * 256
    const double k = t - NNGP_EXP_MAGIC;
    const double f = fma(P.nphi256, u, -k);               // |f| <= 1/2
    const int32_t ki = nngp_lo_dword(t);
    const double Tadj = tab[ki & (NNGP_EXP_TAB_N - 1)];   // 2^(j/256), high dword - (j << 12)
#ifdef NNGP_MATH_HOST
    uint64_t bits;
    memcpy(&bits, &Tadj, 8);
    bits += (uint64_t)((uint32_t)ki << 12) << 32;         // high dword += k << 12 (mod 2^32)
    double Ts;
    memcpy(&Ts, &bits, 8);
#else
    const long long tb = __double_as_longlong(Tadj);
    const int32_t hi = (int32_t)(tb >> 32) + (int32_t)((uint32_t)ki << 12);
    const double Ts = __hiloint2double(hi, (int32_t)(tb & 0xffffffffll));  // 2^(j/256) 2^n
#endif
    // the coefficients as literals (not CovParams fields): the persistent kernels re-materialise
    // them instead of pinning 8 more SGPRs for the whole tile loop
    constexpr double Q[4] = NNGP_EXP2_Q;
    double q = fma(Q[3], f, Q[2]);
    q = fma(q, f, Q[1]);
    q = fma(q, f, Q[0]);
    return fma(Ts, f * q, Ts);
}

// unit-variance covariance of kind KIND at squared distance d2 (tab: nngp_exp_table_load_unit)
template <int KIND>
NNGP_FN double nngp_cov_unit(const CovParams& P, const double* tab, double d2) {
    const double x = fmin(d2, P.d2max);
    if (KIND == NNGP_KIND_GAUSSIAN) return nngp_exp_unit(P, tab, x);
    const double d = nngp_sqrt(x);
    if (KIND == NNGP_KIND_SPHERICAL) {
        const double u = fmin(P.phi * d, 1.0);
        return fma(u, fma(0.5 * u, u, -1.5), 1.0);
    }
    if (KIND == NNGP_KIND_GENERIC) {
        // exponential: p = 1 exactly; Matern-5/2 and spherical: the same polynomial operations as
        // their own kinds below; Matern-3/2: (1 + u) e, one more rounding than e + u e
        const double e = nngp_exp_unit(P, tab, P.gauss ? x : d);
        const double u = fmin(P.phi * d, P.umax);
        return fma(u, fma(u, fma(u, P.c[2], P.c[1]), P.c[0]), 1.0) * e;
    }
    const double e = nngp_exp_unit(P, tab, d);
    if (KIND == NNGP_KIND_MATERN32) return fma(P.phi * d, e, e);
    if (KIND == NNGP_KIND_MATERN52) {
        const double u = P.phi * d;
        return fma(fma(u, 1.0 / 3.0, 1.0), u, 1.0) * e;
    }
    return e;
}

#ifndef NNGP_MATH_HOST
// Split fill for a 256-thread block (one entry per thread): fetch the entry early, store it
// (and synchronise) once other loads are in flight -- vmcnt retires loads in order, so the
// store waits only for this load, not for loads issued after it.
NNGP_FN double nngp_exp_table_entry_unit(int j) {
    const long long b = __double_as_longlong(kExp2Tab[j]);
    return __hiloint2double((int32_t)(b >> 32) - (j << 12), (int32_t)(b & 0xffffffffll));
}
NNGP_FN double nngp_exp_table_fetch_unit() { return nngp_exp_table_entry_unit((int)threadIdx.x & (NNGP_EXP_TAB_N - 1)); }
NNGP_FN void nngp_exp_table_store_unit(double* tab, double v) {
    if (threadIdx.x < NNGP_EXP_TAB_N) tab[threadIdx.x] = v;
    __syncthreads();
}

// LDS table for nngp_exp_unit (every thread of the block calls it)
NNGP_FN void nngp_exp_table_load_unit(double* tab) {
    for (int j = threadIdx.x; j < NNGP_EXP_TAB_N; j += blockDim.x) {
        const long long b = __double_as_longlong(kExp2Tab[j]);
        tab[j] = __hiloint2double((int32_t)(b >> 32) - (j << 12), (int32_t)(b & 0xffffffffll));
    }
    __syncthreads();
}
#else
static inline void nngp_exp_table_load_unit(double* tab) {
    for (int j = 0; j < NNGP_EXP_TAB_N; ++j) {
        uint64_t b;
        memcpy(&b, &kExp2Tab[j], 8);
        b -= (uint64_t)((uint32_t)j << 12) << 32;
        memcpy(&tab[j], &b, 8);
    }
}
#endif
