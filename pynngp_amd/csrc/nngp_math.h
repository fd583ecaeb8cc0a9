// fp64 elementary functions for the NNGP covariance / Cholesky kernels.
//
// The covariance plug-in (pyNNGP/nngp.py:6,12 -- `cov`, called at :82 and :96)
// is evaluated ~m(m+1)/2 times per location, so exp and sqrt dominate the
// B/F sweep.  These versions are branch-free and specialised to the ranges the
// sweep uses, each within ~1 ulp:
//   * exp(-phi d) = 2^(-phi log2(e) d): one clamp, one rndne, one sub, an 11-FMA Horner
//     polynomial for 2^f on |f| <= 1/2 whose coefficients already carry sigma2
//     (host-precomputed, passed by value so they live in SGPRs), one ldexp;
//   * d = sqrt(d2): v_rsq_f64 plus one coupled Newton step (d2 clamped below at
//     2^-1000 so d never becomes NaN; exp(-phi 2^-500) == 1 in fp64);
//   * 1/sqrt(pivot): v_rsq_f64 plus two Newton steps.
// The same source compiles on the host (NNGP_MATH_HOST) so
// tests/test_math_host.py measures the ulp error against libm without a GPU.
#pragma once

#ifdef NNGP_MATH_HOST
#include <math.h>
#define NNGP_FN static inline
#define NNGP_HD static inline
static inline double nngp_rsq_approx(double x) {
    // emulate v_rsq_f64's ~2^-29 relative accuracy so the refinement is tested
    double y = 1.0 / sqrt(x);
    return y * (1.0 + 0x1p-29);
}
#else
#include <hip/hip_runtime.h>
#define NNGP_FN __device__ __forceinline__
#define NNGP_HD __host__ __device__ __forceinline__
NNGP_FN double nngp_rsq_approx(double x) { return __builtin_amdgcn_rsq(x); }
#endif

// 2^f on [-1/2, 1/2]: near-minimax degree-11 polynomial (max rel. error
// 1.9e-16 incl. Horner rounding), i.e. exp(r) on |r| <= ln2/2 with r = f ln2.
#define NNGP_EXP2_COEFS                                                                                       \
    {0x1.0000000000000p+0, 0x1.62e42fefa39efp-1, 0x1.ebfbdff82c62cp-3, 0x1.c6b08d70493edp-5,                  \
     0x1.3b2ab6fb8f172p-7, 0x1.5d87fe7b457bap-10, 0x1.4309133b29912p-13, 0x1.ffcbf0bb9f2ccp-17,               \
     0x1.62bf690de5049p-20, 0x1.b53a806e484cbp-24, 0x1.e6a9c6fa19eb0p-28, 0x1.cd7d769448dd6p-32}

#define NNGP_LOG2E 0x1.71547652b82fep+0
#define NNGP_LN2 0x1.62e42fefa39efp-1

// Covariance parameters, built once on the host (nngp_cov_params) and passed by value.
struct CovParams {
    double c[12];  // sigma2 * (2^f polynomial coefficients)
    double nphi2;  // -phi * log2(e): exponent of 2 per unit distance
    double phi;    // phi (Matern-3/2 needs phi d)
    double diag;   // sigma2 + tau2
    double sigma2;
};

NNGP_HD CovParams nngp_cov_params(double sigma2, double phi, double tau2) {
    const double q[12] = NNGP_EXP2_COEFS;
    CovParams p;
    for (int k = 0; k < 12; ++k) p.c[k] = sigma2 * q[k];
    p.nphi2 = -(phi * NNGP_LOG2E);
    p.phi = phi;
    p.diag = sigma2 + tau2;
    p.sigma2 = sigma2;
    return p;
}

// sigma2 * 2^x for x <= 0.  x is clamped at -1080 first: the result underflows
// to (practically) 0 there, and v_ldexp_f64 must not see the saturated
// v_cvt_i32_f64 of a huge |x| (it does not return 0 for it on gfx950).
NNGP_FN double nngp_scaled_exp2(const CovParams& P, double x) {
    x = fmax(x, -1080.0);
    const double n = rint(x);
    const double f = x - n;  // exact
    double p = P.c[11];
    p = fma(p, f, P.c[10]);
    p = fma(p, f, P.c[9]);
    p = fma(p, f, P.c[8]);
    p = fma(p, f, P.c[7]);
    p = fma(p, f, P.c[6]);
    p = fma(p, f, P.c[5]);
    p = fma(p, f, P.c[4]);
    p = fma(p, f, P.c[3]);
    p = fma(p, f, P.c[2]);
    p = fma(p, f, P.c[1]);
    p = fma(p, f, P.c[0]);
    return ldexp(p, (int)n);
}

// sqrt(d2) for d2 >= 0, ~1 ulp; d2 below 2^-1000 is treated as 2^-1000.
NNGP_FN double nngp_sqrt(double d2) {
    const double x = fmax(d2, 0x1p-1000);
    const double y = nngp_rsq_approx(x);
    const double s = x * y;
    const double h = 0.5 * y;
    const double e = fma(-s, h, 0.5);
    return fma(s, e, s);
}

// 1/sqrt(x) for a positive pivot: two Newton steps on v_rsq_f64.
NNGP_FN double nngp_rsqrt(double x) {
    double y = nngp_rsq_approx(x);
    double t = fma(-(x * y), y, 1.0);
    y = fma(0.5 * y, t, y);
    t = fma(-(x * y), y, 1.0);
    y = fma(0.5 * y, t, y);
    return y;
}

// Covariance kinds (the reference's `cov` plug-in, nngp.py:6,12):
//   0 exponential  sigma2 * exp(-phi d)
//   1 matern32     sigma2 * (1 + phi d) * exp(-phi d)
template <int KIND>
NNGP_FN double nngp_cov_d2(const CovParams& P, double d2) {
    const double d = nngp_sqrt(d2);
    if (KIND == 1) {
        const double pd = P.phi * d;
        const double e = nngp_scaled_exp2(P, pd * -NNGP_LOG2E);
        return fma(pd, e, e);
    }
    return nngp_scaled_exp2(P, P.nphi2 * d);
}

// squared Euclidean distance between two points
NNGP_FN double nngp_d2(double ax, double ay, double bx, double by) {
    const double dx = ax - bx;
    const double dy = ay - by;
    return fma(dx, dx, dy * dy);
}
