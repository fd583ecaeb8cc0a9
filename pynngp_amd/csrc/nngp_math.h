// fp64 elementary functions for the NNGP covariance / Cholesky kernels.
//
// The covariance plug-in (pyNNGP/nngp.py:6,12 -- `cov`, called at :82 and :96)
// is evaluated ~m(m+1)/2 times per location, so exp and sqrt dominate the
// B/F sweep.  These are branch-free versions specialised to the ranges the
// sweep uses (exp of a non-positive argument, sqrt of a squared distance,
// rsqrt of a Cholesky pivot), each ~1 ulp, built on the gfx950 v_rsq_f64 /
// v_ldexp_f64 / v_rndne_f64 instructions.  The same source compiles on the host
// (NNGP_MATH_HOST) so tests/test_math_host.py can measure the ulp error
// against libm without a GPU.
#pragma once

#ifdef NNGP_MATH_HOST
#include <math.h>
#define NNGP_FN static inline
static inline double nngp_rsq_approx(double x) {
    // emulate v_rsq_f64's ~2^-29 relative accuracy so the refinement is tested
    double y = 1.0 / sqrt(x);
    return y * (1.0 + 0x1p-29);
}
#else
#include <hip/hip_runtime.h>
#define NNGP_FN __device__ __forceinline__
NNGP_FN double nngp_rsq_approx(double x) { return __builtin_amdgcn_rsq(x); }
#endif

// exp(x) for x <= 0.  Arguments below -708 return exp(-708) ~ 3.3e-308
// (a covariance that small is zero at fp64 resolution of sigma2).
// Reduction x = n ln2 + r, |r| <= ln2/2; near-minimax degree-11 polynomial
// (max rel. error 1.8e-16 incl. rounding); result scaled by 2^n.
NNGP_FN double nngp_exp_neg(double x) {
    x = fmax(x, -708.0);
    const double n = rint(x * 0x1.71547652b82fep+0);
    double r = fma(-n, 0x1.62e42fefa39efp-1, x);
    r = fma(-n, 0x1.abc9e3b39803fp-56, r);
    double p = 0x1.965a188f6715ep-26;
    p = fma(p, r, 0x1.29068f4350904p-22);
    p = fma(p, r, 0x1.71f037d278010p-19);
    p = fma(p, r, 0x1.a019286d70301p-16);
    p = fma(p, r, 0x1.a019f82f0dce0p-13);
    p = fma(p, r, 0x1.6c16c1b74f231p-10);
    p = fma(p, r, 0x1.111111131d4d8p-7);
    p = fma(p, r, 0x1.555555553db56p-5);
    p = fma(p, r, 0x1.5555555554bb5p-3);
    p = fma(p, r, 0x1.0000000000052p-1);
    p = fma(p, r, 1.0);
    p = fma(p, r, 1.0);
    return ldexp(p, (int)n);
}

// sqrt(x) for x >= 0 (a squared distance).  x below 2^-1000 returns 0: the
// covariance of two points 1e-150 apart equals sigma2 in fp64 either way.
// One coupled Newton-Raphson step on v_rsq_f64 plus a final residual correction.
NNGP_FN double nngp_sqrt(double x) {
    const double y = nngp_rsq_approx(x);
    double s = x * y;
    double h = 0.5 * y;
    const double e = fma(-s, h, 0.5);
    s = fma(s, e, s);
    h = fma(h, e, h);
    const double d = fma(-s, s, x);
    s = fma(d, h, s);
    return x > 0x1p-1000 ? s : 0.0;
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
// kind is wave-uniform, so the select costs one fma + one cndmask pair.
NNGP_FN double nngp_cov(int kind, double d, double sigma2, double phi) {
    const double pd = phi * d;
    const double e = sigma2 * nngp_exp_neg(-pd);
    return kind == 1 ? fma(pd, e, e) : e;
}

// Euclidean distance between two points.
NNGP_FN double nngp_dist(double ax, double ay, double bx, double by) {
    const double dx = ax - bx;
    const double dy = ay - by;
    return nngp_sqrt(fma(dx, dx, dy * dy));
}
