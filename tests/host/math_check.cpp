// Host build of pynngp_amd/csrc/nngp_math.h (NNGP_MATH_HOST) for tests/test_math_host.py:
// prints the max ulp / relative errors of the kernels' table exp (sigma2 table and the
// unit-variance exponent-add table), sqrt, rsqrt and every covariance kind against long
// double references over random arguments in the ranges the sweeps use, one "name value"
// pair per line, then "special <0|1>" for the exact special values.
#define NNGP_MATH_HOST
#include "../../pynngp_amd/csrc/nngp_math.h"
#include <stdio.h>
#include <stdlib.h>

static double ulp_err(double a, long double ref) {
    if (ref == 0) return a == 0 ? 0 : 1e30;
    double r = (double)ref;
    double u = nextafter(fabs(r), INFINITY) - fabs(r);
    return (double)(fabsl((long double)a - ref) / u);
}

static long double cov_ref(int kind, long double s2, long double phi, long double d) {
    const long double u = phi * d;
    switch (kind) {
        case 1: return s2 * (1 + u) * expl(-u);
        case 2: return s2 * (1 + u + u * u / 3) * expl(-u);
        case 3: return s2 * expl(-u * u);
        case 4: return u < 1 ? s2 * (1 - 1.5L * u + 0.5L * u * u * u) : 0.0L;
        default: return s2 * expl(-u);
    }
}

template <int K>
static double cov_dispatch(bool unit, const CovParams& P, const double* tab, double d2) {
    return unit ? nngp_cov_unit<K>(P, tab, d2) : nngp_cov_d2<K>(P, tab, d2);
}

static double cov_any(int kind, bool unit, const CovParams& P, const double* tab, double d2) {
    switch (kind) {
        case 1: return cov_dispatch<1>(unit, P, tab, d2);
        case 2: return cov_dispatch<2>(unit, P, tab, d2);
        case 3: return cov_dispatch<3>(unit, P, tab, d2);
        case 4: return cov_dispatch<4>(unit, P, tab, d2);
        default: return cov_dispatch<0>(unit, P, tab, d2);
    }
}

// unit-variance covariance: exactly 1 at coincident points; far-away padding points decouple
// exactly (the clamp lands on a zero high dword, nngp_math.h), and every distance near the
// clamp (exponent below -1022) gives a finite value in [0, 1e-300] (<= 2^-1022 times the
// Matern polynomial), exactly 0 beyond it
static int unit_special(int kind, const CovParams& P, const double* tab, double same, double far) {
    const double c0 = cov_any(kind, true, P, tab, same), cf = cov_any(kind, true, P, tab, far);
    int ok = c0 == 1.0 && cf == 0.0;
    const double d2a = P.d2max * 0.999, d2b = P.d2max * 1.02;
    for (int i = 0; i <= 4000; ++i) {
        const double d2 = d2a + (d2b - d2a) * i / 4000.0;
        const double c = cov_any(kind, true, P, tab, d2);
        ok = ok && c >= 0.0 && c <= 1e-300 && (d2 < P.d2max || c == 0.0);
    }
    return ok;
}

int main() {
    double me = 0, meu = 0, ms = 0, mr = 0, mc[5] = {0, 0, 0, 0, 0}, mcu[5] = {0, 0, 0, 0, 0};
    srand(1);
    const double s2 = 1.7, phi = 13.0;
    CovParams P = nngp_cov_params(0, s2, phi, 0.1);
    double tab[NNGP_EXP_TAB_N];
    nngp_exp_table_load(tab, 1.0);  // unit table: exp error alone
    double tab2[NNGP_EXP_TAB_N];
    nngp_exp_table_load(tab2, s2);
    double tabu[NNGP_EXP_TAB_N];
    nngp_exp_table_load_unit(tabu);
    CovParams Pk[5], Pu[5];
    for (int k = 0; k < 5; ++k) {
        Pk[k] = nngp_cov_params(k, s2, phi, 0.1);
        Pu[k] = nngp_cov_params_unit(k, phi, 0.1 / s2);
    }
    for (int t = 0; t < 2000000; t++) {
        double u = (double)rand() / RAND_MAX, w = (double)rand() / RAND_MAX;
        double d = u * 5.0;  // exponent down to -94
        long double x = (long double)P.nphi256 * d / 256.0L;
        double q = ulp_err(nngp_exp_tab(P, tab, d), exp2l(x));
        if (q > me) me = q;
        q = ulp_err(nngp_exp_unit(Pu[0], tabu, d), exp2l((long double)Pu[0].nphi256 * d / 256.0L));
        if (q > meu) meu = q;
        double s = u * u * (t % 3 ? 1.0 : 1e-20) + 1e-290;
        q = ulp_err(nngp_sqrt(s), sqrtl((long double)s));
        if (q > ms) ms = q;
        q = ulp_err(nngp_rsqrt(s + 0.1), 1.0L / sqrtl((long double)s + 0.1L));
        if (q > mr) mr = q;
        // distances up to ~0.2 (u = phi d up to ~2.6): where the factorisation is sensitive
        const double sc = 0.15;
        double d2 = nngp_d2(u * sc, w * sc, 0.0, 0.0);
        long double dd = sqrtl((long double)(u * sc) * (u * sc) + (long double)(w * sc) * (w * sc));
        for (int k = 0; k < 5; ++k) {
            const long double r = cov_ref(k, s2, phi, dd);
            if (r == 0) continue;
            // relative to sigma2: the scale every entry of the block is compared against
            q = (double)(fabsl(cov_any(k, false, Pk[k], tab2, d2) - r) / s2);
            if (q > mc[k]) mc[k] = q;
            q = (double)(fabsl(s2 * cov_any(k, true, Pu[k], tabu, d2) - r) / s2);
            if (q > mcu[k]) mcu[k] = q;
        }
    }
    // exact special values used by the kernels: coincident points, far-away padding points
    int ok = nngp_exp_tab(P, tab2, 0.0) == s2 && nngp_cov_d2<0>(P, tab2, nngp_d2(0.3, 0.4, 0.3, 0.4)) == s2 &&
             nngp_cov_d2<1>(P, tab2, nngp_d2(0.3, 0.4, 0.3, 0.4)) == s2 &&
             nngp_cov_d2<0>(P, tab2, nngp_d2(1e150, 0.0, 0.5, 0.5)) == 0.0 &&
             nngp_cov_d2<0>(P, tab2, nngp_d2(64e150, 0.0, 1e150, 0.0)) == 0.0 && nngp_rsqrt(1.0) == 1.0;
    for (int k = 0; k < 5; ++k) {
        const double same = nngp_d2(0.3, 0.4, 0.3, 0.4), far = nngp_d2(1e150, 0.0, 0.5, 0.5);
        ok = ok && unit_special(k, Pu[k], tabu, same, far);
    }
    printf("exp2_ulp %.6g\nexp2_unit_ulp %.6g\nsqrt_ulp %.6g\nrsqrt_ulp %.6g\n", me, meu, ms, mr);
    for (int k = 0; k < 5; ++k) printf("cov%d_rel %.6g\ncov%d_unit_rel %.6g\n", k, mc[k], k, mcu[k]);
    printf("special %d\n", ok);
    return 0;
}
