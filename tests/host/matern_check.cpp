// Host build of the general-smoothness Matern correlation of pynngp_amd/csrc/nngp_math.h
// (NNGP_MATH_HOST) for tests/test_matern.py: reads "nu u" pairs from stdin and prints
// rho(u) = u^nu K_nu(u) / (2^(nu-1) Gamma(nu)) as a hex float per line.
#define NNGP_MATH_HOST
#include "../../pynngp_amd/csrc/nngp_math.h"
#include <stdio.h>

int main() {
    double nu, u;
    while (scanf("%lf %lf", &nu, &u) == 2) {
        CovParams P = nngp_cov_params_nu(NNGP_KIND_MATERN, 1.0, 1.0, 0.0, nu);
        printf("%a\n", nngp_matern_rho(P, u));
    }
    return 0;
}
