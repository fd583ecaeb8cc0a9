// Host build of pynngp_amd/csrc/nngp_math.h (NNGP_MATH_HOST) for tests/test_math_host.py:
// prints the max ulp / relative errors of the kernel's exp2, sqrt, rsqrt and covariance
// against libm over random arguments in the ranges the sweep uses.
#define NNGP_MATH_HOST
#include "../../pynngp_amd/csrc/nngp_math.h"
#include <stdio.h>
#include <stdlib.h>

static double ulp_err(double a, double ref) {
    if (ref == 0) return a == 0 ? 0 : 1e30;
    double u = nextafter(fabs(ref), INFINITY) - fabs(ref);
    return fabs(a - ref) / u;
}

int main() {
    double me = 0, ms = 0, mr = 0, mc0 = 0, mc1 = 0;
    srand(1);
    const double s2 = 1.7, phi = 13.0;
    CovParams P = nngp_cov_params(s2, phi, 0.1);
    for (int t = 0; t < 4000000; t++) {
        double u = (double)rand() / RAND_MAX, w = (double)rand() / RAND_MAX;
        double x = -u * 60.0;
        double q = ulp_err(nngp_scaled_exp2(P, x) / s2, exp2(x));
        if (q > me) me = q;
        double s = u * u * (t % 3 ? 1.0 : 1e-20) + 1e-290;
        q = ulp_err(nngp_sqrt(s), sqrt(s));
        if (q > ms) ms = q;
        q = ulp_err(nngp_rsqrt(s + 0.1), 1.0 / sqrt(s + 0.1));
        if (q > mr) mr = q;
        double d2 = u * u + w * w, dd = sqrt(d2);
        double r0 = s2 * exp(-phi * dd), r1 = s2 * (1 + phi * dd) * exp(-phi * dd);
        q = fabs(nngp_cov_d2<0>(P, d2) - r0) / r0;
        if (q > mc0) mc0 = q;
        q = fabs(nngp_cov_d2<1>(P, d2) - r1) / r1;
        if (q > mc1) mc1 = q;
    }
    // exact special values used by the kernels
    int ok = nngp_scaled_exp2(P, 0.0) == s2 * 1.0 && nngp_scaled_exp2(P, -1e150 * 13.0) == 0.0 &&
             nngp_cov_d2<0>(P, 0.0) == P.c[0] && nngp_cov_d2<0>(P, 1e300) == 0.0 && nngp_rsqrt(1.0) == 1.0;
    printf("%.6g %.6g %.6g %.6g %.6g %d\n", me, ms, mr, mc0, mc1, ok);
    return 0;
}
