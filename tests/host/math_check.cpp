// Host build of pynngp_amd/csrc/nngp_math.h (NNGP_MATH_HOST) for tests/test_math_host.py:
// prints the max ulp / relative errors of the kernel's table exp, sqrt, rsqrt and covariance
// against libm (long double references) over random arguments in the ranges the sweep uses.
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

int main() {
    double me = 0, ms = 0, mr = 0, mc0 = 0, mc1 = 0;
    srand(1);
    const double s2 = 1.7, phi = 13.0;
    CovParams P = nngp_cov_params(s2, phi, 0.1);
    double tab[NNGP_EXP_TAB_N];
    nngp_exp_table_load(tab, 1.0);  // unit table: exp error alone
    double tab2[NNGP_EXP_TAB_N];
    nngp_exp_table_load(tab2, s2);
    for (int t = 0; t < 4000000; t++) {
        double u = (double)rand() / RAND_MAX, w = (double)rand() / RAND_MAX;
        double d = u * 5.0;  // exponent down to -94
        long double x = (long double)P.nphi256 * d / 256.0L;
        double q = ulp_err(nngp_exp_tab(P, tab, d), exp2l(x));
        if (q > me) me = q;
        double s = u * u * (t % 3 ? 1.0 : 1e-20) + 1e-290;
        q = ulp_err(nngp_sqrt(s), sqrtl((long double)s));
        if (q > ms) ms = q;
        q = ulp_err(nngp_rsqrt(s + 0.1), 1.0L / sqrtl((long double)s + 0.1L));
        if (q > mr) mr = q;
        double d2 = nngp_d2(u, w, 0.0, 0.0);
        long double dd = sqrtl((long double)u * u + (long double)w * w);
        long double r0 = s2 * expl(-phi * dd), r1 = s2 * (1 + phi * dd) * expl(-phi * dd);
        q = (double)(fabsl(nngp_cov_d2<0>(P, tab2, d2) - r0) / r0);
        if (q > mc0) mc0 = q;
        q = (double)(fabsl(nngp_cov_d2<1>(P, tab2, d2) - r1) / r1);
        if (q > mc1) mc1 = q;
    }
    // exact special values used by the kernels: coincident points, far-away padding points
    int ok = nngp_exp_tab(P, tab2, 0.0) == s2 && nngp_cov_d2<0>(P, tab2, nngp_d2(0.3, 0.4, 0.3, 0.4)) == s2 &&
             nngp_cov_d2<1>(P, tab2, nngp_d2(0.3, 0.4, 0.3, 0.4)) == s2 &&
             nngp_cov_d2<0>(P, tab2, nngp_d2(1e150, 0.0, 0.5, 0.5)) == 0.0 &&
             nngp_cov_d2<0>(P, tab2, nngp_d2(64e150, 0.0, 1e150, 0.0)) == 0.0 && nngp_rsqrt(1.0) == 1.0;
    printf("%.6g %.6g %.6g %.6g %.6g %d\n", me, ms, mr, mc0, mc1, ok);
    return 0;
}
