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
#include "rgamma_series.h"

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
#define NNGP_KIND_MATERN 5       // sigma2 u^nu K_nu(u) / (2^(nu-1) Gamma(nu)), any smoothness nu (spNNGP's
                                 // "matern"; nu = 1/2, 3/2, 5/2 give the exponential / Matern-3/2 / -5/2 kinds)
#define NNGP_N_KINDS 6
#define NNGP_MATERN_NU_MAX 50.0
#define NNGP_MATERN_X_SWITCH 1.5  // Temme below, the continued fraction above (the most accurate split, tests/test_matern.py)
// Runtime kind (the m = 25..32 kernels, one instantiation for kinds 0..4): every kind as
// p(u) e, p(u) = 1 + c1 u + c2 u^2 + c3 u^3 with u = min(phi d, umax), e = 2^(nphi256 g / 256) with
// g = d (g = d^2 for the gaussian kind; nphi256 = 0, i.e. e = 1, for the spherical kind).
#define NNGP_KIND_GENERIC 7
// Covariance blocks from memory (nngp_bf_sweep_blocks: a caller-evaluated covariance; bf_pairb.h)
#define NNGP_KIND_BLOCKS 8

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
    // NNGP_KIND_MATERN (nngp_matern_setup): nu = nl + mu, |mu| <= 1/2; Temme's Gamma_1(mu), Gamma_2(mu),
    // Gamma(1 + mu), Gamma(1 - mu), mu pi / sin(mu pi), and the scale 2^(1 - nl) / Gamma(nu)
    double nu, mu, mg1, mg2, mgp, mgm, mfac, mscale;
    int mnl;
    // NNGP_KIND_MATERN on the fused pair kernel (nngp_matern_table_setup, nngp_matern_tab): t = mphi2 d^2,
    // the table's first octave exponent and octave count
    double mphi2;
    int mt_e0, mt_noct;
    // ... below the table (t < 2^mt_e0) when the octaves from 1 - rho < eps would not fit (nu < ~0.45):
    // rho = 1 - mt_A t^nu (mt_series = 1), else rho = 1 there
    double mt_A;
    int mt_series;
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
    } else if (kind == NNGP_KIND_MATERN) {
        p.nphi256 = 0.0;
        // u = 1500 (+ 30 nu below, nngp_matern_setup): e^-u underflows, so the covariance is exactly 0
        // (far-away padding points decouple) and u^nu stays finite
        p.d2max = (1500.0 / phi) * (1500.0 / phi);
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
    p.nu = p.mu = p.mg1 = p.mg2 = p.mgp = p.mgm = p.mfac = p.mscale = 0.0;
    p.mnl = 0;
    p.mphi2 = 0.0;
    p.mt_e0 = p.mt_noct = 0;
    p.mt_A = 0.0;
    p.mt_series = 0;
    return p;
}

// ---------------------------------------------------------------- Matern, general smoothness nu
// rho(u) = u^nu K_nu(u) / (2^(nu-1) Gamma(nu)), u = phi d (spNNGP's parameterisation: nu = 3/2 is
// (1 + u) e^-u).  nu = nl + mu with nl = floor(nu + 1/2), |mu| <= 1/2.  K_mu and K_{mu+1} come from
// Temme's series (u <= 1.5) or the Thompson-Barnett continued fraction (u > 1.5), K_nu from the upward
// recurrence.  Everything is carried scaled, J_k = u^k (u/2)^mu K_{mu+k}(u), so that
//   rho(u) = 2^(1 - nl) / Gamma(nu) * J_nl,   J_{k+1} = 2 (mu + k) J_k + u^2 J_{k-1}
// (positive terms only) and the small-u limit (J_nl -> 2^(nl-1) Gamma(nu)) involves no large
// exponential: the scaling removes the (u/2)^-mu of Temme's p-series exactly.
// Host part: the per-theta constants (1 / Gamma(1 +- mu) from the entire series of
// rgamma_series.h, so Temme's Gamma_1 = (1/Gamma(1-mu) - 1/Gamma(1+mu)) / (2 mu) is its odd part
// without cancellation).
NNGP_HD void nngp_matern_setup(CovParams& p, double nu) {
    const double a[NNGP_RGAMMA_N] = NNGP_RGAMMA_COEF;
    const double nlf = floor(nu + 0.5);
    const double mu = nu - nlf;
    double gp = 0.0, gm = 0.0, g1 = 0.0, g2 = 0.0;  // 1/Gamma(1+mu), 1/Gamma(1-mu), odd / even parts
    for (int k = NNGP_RGAMMA_N - 1; k >= 0; --k) {
        gp = fma(gp, mu, a[k]);
        gm = fma(gm, -mu, a[k]);
    }
    for (int k = NNGP_RGAMMA_N - 1 - ((NNGP_RGAMMA_N - 1) % 2 == 0); k >= 1; k -= 2) g1 = fma(g1, mu * mu, a[k]);
    for (int k = NNGP_RGAMMA_N - 1 - ((NNGP_RGAMMA_N - 1) % 2 == 1); k >= 0; k -= 2) g2 = fma(g2, mu * mu, a[k]);
    p.nu = nu;
    p.mu = mu;
    p.mnl = (int)nlf;
    p.mg1 = -g1;  // Gamma_1(mu) = -sum_{k odd} a_k mu^(k-1)
    p.mg2 = g2;   // Gamma_2(mu) = sum_{k even} a_k mu^k
    p.mgp = 1.0 / gp;  // Gamma(1 + mu)
    p.mgm = 1.0 / gm;  // Gamma(1 - mu)
    const double pm = 3.141592653589793 * mu;
    p.mfac = mu == 0.0 ? 1.0 : pm / sin(pm);
    // Gamma(nu) = Gamma(1 + mu) prod_{j=1}^{nl-1} (j + mu)   (nl = 0: Gamma(mu) = Gamma(1 + mu) / mu)
    double gnu = p.mgp;
    if (p.mnl == 0) gnu /= mu;
    for (int j = 1; j < p.mnl; ++j) gnu *= (double)j + mu;
    p.mscale = ldexp(1.0, 1 - p.mnl) / gnu;
    const double umax = 1500.0 + 30.0 * nu;
    p.d2max = (umax / p.phi) * (umax / p.phi);
}

NNGP_HD CovParams nngp_cov_params_nu(int kind, double sigma2, double phi, double tau2, double nu) {
    CovParams p = nngp_cov_params(kind, sigma2, phi, tau2);
    if (kind == NNGP_KIND_MATERN) nngp_matern_setup(p, nu);
    return p;
}

// sinh(s) / s (a series below |s| = 1/2, where sinh loses bits to the cancellation of its exponentials)
NNGP_HD double nngp_sinhc(double s) {
    if (fabs(s) < 0.5) {
        const double z = s * s;  // sum_k z^k / (2k + 1)!, k <= 8: the next term is below 2^-70
        double t = 1.0 / 355687428096000.0;  // 1/17!
        t = fma(t, z, 1.0 / 1307674368000.0);
        t = fma(t, z, 1.0 / 6227020800.0);
        t = fma(t, z, 1.0 / 39916800.0);
        t = fma(t, z, 1.0 / 362880.0);
        t = fma(t, z, 1.0 / 5040.0);
        t = fma(t, z, 1.0 / 120.0);
        t = fma(t, z, 1.0 / 6.0);
        return fma(t, z, 1.0);
    }
    return sinh(s) / s;
}

// J_0 = (x/2)^mu K_mu(x), J_1 = x (x/2)^mu K_{mu+1}(x) for x > 0
NNGP_HD void nngp_matern_j01(const CovParams& P, double x, double& j0, double& j1) {
    const double mu = P.mu;
    if (x <= NNGP_MATERN_X_SWITCH) {
        // Temme (1975): K_mu = sum_k c_k f_k, K_{mu+1} = (2/x) sum_k c_k (p_k - k f_k), c_k = (x^2/4)^k / k!,
        // f_0 = (mu pi / sin mu pi) (Gamma_1 cosh s + Gamma_2 L sinh(s) / s), s = mu L, L = ln(2/x),
        // p_0 = (x/2)^-mu Gamma(1+mu) / 2, q_0 = (x/2)^mu Gamma(1-mu) / 2,
        // f_k = (k f_{k-1} + p_{k-1} + q_{k-1}) / (k^2 - mu^2), p_k = p_{k-1} / (k - mu), q_k = q_{k-1} / (k + mu);
        // here every f, p, q carries the factor E = (x/2)^mu = e^-s
        const double L = -log(0.5 * x);
        const double s = mu * L;
        const double E = exp(-s);
        double f = P.mfac * (P.mg1 * (0.5 * fma(E, E, 1.0)) + P.mg2 * L * (E * nngp_sinhc(s)));
        double pk = 0.5 * P.mgp;
        double qk = 0.5 * (E * E) * P.mgm;
        const double hh = 0.25 * x * x;
        double c = 1.0, s0 = f, s1 = pk;
        for (int k = 1; k < 60; ++k) {
            const double dk = (double)k;
            f = (dk * f + pk + qk) / fma(dk, dk, -mu * mu);
            c *= hh / dk;
            pk /= dk - mu;
            qk /= dk + mu;
            const double t0 = c * f, t1 = c * fma(-dk, f, pk);
            s0 += t0;
            s1 += t1;
            if (fabs(t0) <= 0x1p-56 * fabs(s0) && fabs(t1) <= 0x1p-56 * fabs(s1)) break;
        }
        j0 = s0;
        j1 = 2.0 * s1;
    } else {
        // Thompson & Barnett (1987), Steed's evaluation of the continued fraction for K_{mu+1} / K_mu
        // together with the sum S giving K_mu = sqrt(pi / 2x) e^-x / S (x > 1.5: a few dozen terms)
        const double a1 = 0.25 - mu * mu;
        double b = 2.0 * (1.0 + x), d = 1.0 / b, dh = d, h = d;
        double q0 = 0.0, q1 = 1.0, q = a1, c = a1, a = -a1, S = fma(q, dh, 1.0);
        for (int i = 1; i < 400; ++i) {
            const double di = (double)i;
            a -= 2.0 * di;
            c = -a * c / (di + 1.0);
            const double qn = (q0 - b * q1) / a;
            q0 = q1;
            q1 = qn;
            q = fma(c, qn, q);
            b += 2.0;
            d = 1.0 / fma(a, d, b);
            dh = fma(b, d, -1.0) * dh;
            h += dh;
            const double dS = q * dh;
            S += dS;
            if (fabs(dS) <= 0x1p-56 * fabs(S)) break;
        }
        const double E = exp(mu * log(0.5 * x));
        j0 = E * sqrt(1.5707963267948966 / x) * exp(-x) / S;
        j1 = j0 * (mu + x + 0.5 - a1 * h);
    }
}

// rho(u) for u >= 0 (u = 0: the limit 1)
NNGP_HD double nngp_matern_rho(const CovParams& P, double u) {
    if (!(u > 0.0)) return 1.0;
    double j0, j1;
    nngp_matern_j01(P, u, j0, j1);
    if (P.mnl == 0) return P.mscale * j0;
    const double u2 = u * u;
    for (int k = 1; k < P.mnl; ++k) {
        const double j2 = fma(2.0 * (P.mu + (double)k), j1, u2 * j0);
        j0 = j1;
        j1 = j2;
    }
    return P.mscale * j1;
}

// ---------------------------------------------------------------- Matern-nu by table (bf_pairb)
// The fused pair kernel evaluates rho from a per-launch table in t = u^2 = phi^2 d^2 (no square root,
// no Bessel loop).  Octave o of t -- t in [2^(e0+o-1), 2^(e0+o)), o = (frexp exponent of t) - e0 -- is
// split into NNGP_MT_K bins by its top mantissa bits; each bin holds a degree-(NNGP_MT_NC - 1)
// polynomial in the bin's local variable f in [0, 1): the Chebyshev interpolant of rho at NNGP_MT_NC
// nodes (values from nngp_matern_rho), in monomial form.  Octave 0 holds rho = 1 (every t below it
// has 1 - rho < NNGP_MT_EPS) and octave noct - 1 holds rho = 0 (rho < NNGP_MT_EPS beyond): coincident
// points give exactly 1, far-away padding points exactly 0 (decoupled).  Interpolation error against
// mpmath (nu = 0.5 .. 50, 8 bins per octave of degree 9 since round 5: ~1e-16; 4 of degree 13: 1.2e-17)
// absolute, well under what the table inherits from
// accuracy of nngp_matern_rho (<= 1.3e-15 absolute).  Per covariance: 11 VALU for the index and the
// local variable, NNGP_MT_NC - 1 FMAs, NNGP_MT_NC / 2 LDS reads of 16 B (8 x 10 measured 9-12 % faster
// than 4 x 14 -- 5 reads and 9 FMAs against 7 and 13 -- and 16 x 8 slower: every block copies the table
// into LDS, 77 KB, profiles/r05m).  The octaves from 1 - rho < eps to
// rho < eps fit NNGP_MT_MAX_OCT for nu >= NNGP_MT_NU_MIN; smaller nu start the table at 2^-64 and take
// the small-t expansion below it (NNGP_MT_SERIES_E): every nu in (0, 50] runs on the pair kernel.
#define NNGP_MT_K 8
#define NNGP_MT_NC 10
#define NNGP_MT_MAX_OCT 160
#define NNGP_MT_EPS 1e-18
#define NNGP_MT_NU_MIN 0.4
#define NNGP_MT_BYTES(noct) ((size_t)(noct) * NNGP_MT_K * NNGP_MT_NC * sizeof(double))

// a bound on 1 - rho(sqrt(t)) for small t from the expansion rho = 1 - A t^nu - t / (4 (1 - nu)) + ...,
// A = Gamma(1 - nu) / (4^nu Gamma(1 + nu)) (u^nu K_nu(u) through I_-nu and I_nu), with margin; near
// nu = 1, where the two terms cancel into (t / 4) ln(1 / t), a bound of that form
NNGP_HD double nngp_matern_small_bound(double nu, double t) {
    const double d1 = fabs(1.0 - nu);
    if (d1 < 0.05) return 6.0 * pow(t, fmin(nu, 1.0)) * (fabs(log(t)) + 5.0);
    double b = 0.25 * t / d1;
    if (nu < 1.95) b += fabs(tgamma(1.0 - nu)) / (pow(4.0, nu) * tgamma(1.0 + nu)) * pow(t, nu);
    return 2.0 * b;
}

// Below the table.  For small nu the octaves down to 1 - rho < eps are too many (rho = 1 - A t^nu + ...
// reaches 1 - 1e-18 only at t ~ 1e-18^(1/nu): ~200 octaves at nu = 0.3), so from NNGP_MT_SERIES_E down
// the kernel uses the expansion (u = sqrt t; u^nu K_nu(u) through I_{-nu} and I_nu):
//   rho = 1 + t / (4 (1 - nu)) - A t^nu (1 + t / (4 (1 + nu))) + O(t^2),  A = Gamma(1 - nu) / (4^nu Gamma(1 + nu)),
// where below t = 2^-64 every term but 1 - A t^nu is under 1e-19: rho = 1 - A t^nu (one pow per such
// covariance -- near-coincident points, phi d < 2^-32 -- on a branch the other lanes skip).
#define NNGP_MT_SERIES_E (-64)
// 1 - A t^nu below the table: a real call on the GPU (ocml's pow would otherwise be inlined at each of a
// fully unrolled kernel's hundreds of covariance sites -- 4x the code -- for a branch that near-coincident
// points alone take)
// points, and coincident points -- t at point_d2's floor times phi^2 -- are exactly 1 (1 - A t^nu there is
// not for a tiny nu: 1 - 1e-3 at nu = 0.01)
#ifdef NNGP_MATH_HOST
static inline double nngp_matern_below(double A, double t, double nu, double mphi2) {
    return t <= NNGP_D2_FLOOR * mphi2 ? 1.0 : fma(-A, pow(t, nu), 1.0);
}
#else
__device__ __attribute__((noinline)) static double nngp_matern_below(double A, double t, double nu, double mphi2) {
    return t <= NNGP_D2_FLOOR * mphi2 ? 1.0 : fma(-A, pow(t, nu), 1.0);
}
#endif

// table extent for P (nngp_matern_setup done): returns false when it would exceed NNGP_MT_MAX_OCT
NNGP_HD bool nngp_matern_table_setup(CovParams& p) {
    p.mphi2 = p.phi * p.phi;
    int ez = 1;  // smallest E with rho(sqrt(2^E)) < eps (rho decreases)
    while (ez < 1100 && !(nngp_matern_rho(p, sqrt(ldexp(1.0, ez))) < NNGP_MT_EPS)) ++ez;
    int e0 = 0;  // largest E <= 0 with the small-t bound below eps at 2^E (the bound increases with t)
    while (e0 > -1074 && !(nngp_matern_small_bound(p.nu, ldexp(1.0, e0)) < NNGP_MT_EPS)) --e0;
    p.mt_series = 0;
    p.mt_A = 0.0;
    // (every nu < 0.9 whose table would reach below 2^-64, not only those past NNGP_MT_MAX_OCT: ~45 fewer
    // octaves at nu = 0.5 -- 25 KB less LDS per block, the occupancy advice r04 asked about)
    if (p.nu < 0.9 && e0 < NNGP_MT_SERIES_E) {
        e0 = NNGP_MT_SERIES_E;  // the series serves t < 2^e0
        p.mt_series = 1;
        p.mt_A = tgamma(1.0 - p.nu) / (pow(4.0, p.nu) * tgamma(1.0 + p.nu));
    }
    p.mt_e0 = e0;
    p.mt_noct = ez - e0 + 2;
    return p.mt_noct <= NNGP_MT_MAX_OCT;
}

// Chebyshev nodes of a bin in its local variable f: (1 + cos(pi (k + 1/2) / NC)) / 2, k = 0 .. NC-1
NNGP_HD double nngp_matern_node(int k) { return 0.5 * (1.0 + cos(3.141592653589793 * (k + 0.5) / NNGP_MT_NC)); }

// t at local variable f of bin b (octave o = b / K, j = b % K): 2^(e0 + o - 1) (1 + (j + f) / K)
NNGP_HD double nngp_matern_bin_t(const CovParams& p, int b, double f) {
    const int o = b / NNGP_MT_K, j = b % NNGP_MT_K;
    return ldexp(1.0 + (j + f) / NNGP_MT_K, p.mt_e0 + o - 1);
}

// costab[j NC + k] = cos(pi j (k + 1/2) / NC): the discrete cosine transform of the node values
NNGP_HD void nngp_matern_costab(double* costab) {
    for (int j = 0; j < NNGP_MT_NC; ++j)
        for (int k = 0; k < NNGP_MT_NC; ++k) costab[j * NNGP_MT_NC + k] = cos(3.141592653589793 * j * (k + 0.5) / NNGP_MT_NC);
}

// monomial coefficients in f of bin b's interpolant from rho at the bin's nodes (rho_nodes[k] at
// nngp_matern_node(k)); octave 0 = 1, the last octave = 0
NNGP_HD void nngp_matern_bin_fit(const CovParams& p, int b, const double* rho_nodes, const double* costab,
                                 double* coef) {
    const int o = b / NNGP_MT_K;
    for (int k = 0; k < NNGP_MT_NC; ++k) coef[k] = 0.0;
    if (o == 0) {
        coef[0] = 1.0;
        return;
    }
    if (o >= p.mt_noct - 1) return;
    // Chebyshev coefficients c_j in x = 2 f - 1, then sum_j c_j T_j(2 f - 1) in powers of f.  The transform
    // runs on the deviations from a middle node's value, which is added to the constant term last: every
    // c_j then carries rounding noise of the bin's variation only, not of rho itself (transforming rho
    // directly left ~NC ulp of noise in the sum over j, 2.5e-15 near rho = 1)
    const double vref = rho_nodes[NNGP_MT_NC / 2];
    double tprev[NNGP_MT_NC], tcur[NNGP_MT_NC], tnext[NNGP_MT_NC];
    for (int k = 0; k < NNGP_MT_NC; ++k) tprev[k] = tcur[k] = 0.0;
    tprev[0] = 1.0;             // T_0 = 1
    tcur[0] = -1.0;             // T_1 = 2 f - 1
    tcur[1] = 2.0;
    for (int j = 0; j < NNGP_MT_NC; ++j) {
        double c = 0.0;
        for (int k = 0; k < NNGP_MT_NC; ++k) c = fma(rho_nodes[k] - vref, costab[j * NNGP_MT_NC + k], c);
        c *= (j == 0 ? 1.0 : 2.0) / NNGP_MT_NC;
        const double* T = j == 0 ? tprev : tcur;
        for (int k = 0; k < NNGP_MT_NC; ++k) coef[k] = fma(c, T[k], coef[k]);
        if (j >= 1) {  // T_{j+1} = 2 (2 f - 1) T_j - T_{j-1}
            for (int k = 0; k < NNGP_MT_NC; ++k)
                tnext[k] = 4.0 * (k > 0 ? tcur[k - 1] : 0.0) - 2.0 * tcur[k] - tprev[k];
            for (int k = 0; k < NNGP_MT_NC; ++k) {
                tprev[k] = tcur[k];
                tcur[k] = tnext[k];
            }
        }
    }
    coef[0] += vref;
}

// rho(phi d) from the table (tab: the launch's table, 16-B aligned), d2 = d^2 from the distance.
// t is clamped far past the last octave (rho = 0 there): a padding point's d2 ~ (m + 1)^2 1e300 times a
// large phi^2 overflows to inf, whose frexp exponent (0 on the GPU) and mantissa (inf) would index the
// table out of range and give NaN instead of an exact 0 (advice r04)
NNGP_HD double nngp_matern_tab(const CovParams& P, const double* tab, double d2) {
    const double t = fmin(d2 * P.mphi2, 0x1p1000);
#ifdef NNGP_MATH_HOST
    int ex;
    const double mant = frexp(t, &ex);
    const double s = mant * (2.0 * NNGP_MT_K);  // [K, 2K)
    const double f = s - floor(s);
#else
    const int ex = __builtin_amdgcn_frexp_exp(t);
    const double s = __builtin_amdgcn_frexp_mant(t) * (2.0 * NNGP_MT_K);
    const double f = __builtin_amdgcn_fract(s);
#endif
    const int j = (int)s - NNGP_MT_K;
    if (P.mt_series && ex <= P.mt_e0) return nngp_matern_below(P.mt_A, t, P.nu, P.mphi2);  // below the table (rare)
    int o = ex - P.mt_e0;
    o = o < 0 ? 0 : (o > P.mt_noct - 1 ? P.mt_noct - 1 : o);
    const double* c = tab + (o * NNGP_MT_K + j) * NNGP_MT_NC;
#ifdef NNGP_MATH_HOST
    double r = c[NNGP_MT_NC - 1];
#pragma unroll
    for (int k = NNGP_MT_NC - 2; k >= 0; --k) r = fma(r, f, c[k]);
#else
    // the same Horner order from 16-byte pairs (a bin's NC coefficients start 16-byte aligned: one load
    // each from LDS or global memory)
    static_assert(NNGP_MT_NC % 2 == 0, "coefficient pairs");
    const double2* c2 = (const double2*)c;
    double2 v = c2[NNGP_MT_NC / 2 - 1];
    double r = fma(v.y, f, v.x);
#pragma unroll
    for (int h = NNGP_MT_NC / 2 - 2; h >= 0; --h) {
        v = c2[h];
        r = fma(fma(r, f, v.y), f, v.x);
    }
#endif
    return r;
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
    if (KIND == NNGP_KIND_MATERN) return P.sigma2 * nngp_matern_rho(P, P.phi * d);
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
    // the polynomial before the table value is first used: the LDS read (bank-conflicted random
    // lookups) gets the polynomial's latency to land in (round 4, profiles/r04u: -0.8 %, same bits).
    // The coefficients as literals (not CovParams fields): the persistent kernels re-materialise
    // them instead of pinning 8 more SGPRs for the whole tile loop
    constexpr double Q[4] = NNGP_EXP2_Q;
    double q = fma(Q[3], f, Q[2]);
    q = fma(q, f, Q[1]);
    q = fma(q, f, Q[0]);
    const double fq = f * q;
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
    return fma(Ts, fq, Ts);
}

// unit-variance covariance of kind KIND at squared distance d2 (tab: nngp_exp_table_load_unit)
template <int KIND>
NNGP_FN double nngp_cov_unit(const CovParams& P, const double* tab, double d2) {
    if (KIND == NNGP_KIND_MATERN) return nngp_matern_tab(P, tab, d2);  // tab: the Matern table
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
