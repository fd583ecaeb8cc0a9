// Host build of the Matern-nu table path of pynngp_amd/csrc/nngp_math.h (NNGP_MATH_HOST) for
// tests/test_matern.py: reads "nu u" pairs from stdin; per nu it builds the table exactly as the
// device builder does (nngp_matern_table_setup, rho at the bins' Chebyshev nodes, nngp_matern_bin_fit)
// and prints rho(u) = nngp_matern_tab(P, table, u^2) (phi = 1) as a hex float with the table's octave
// count, or "nan 0" when the table would not fit (nu below the fast kernel's range).
#define NNGP_MATH_HOST
#include "../../pynngp_amd/csrc/nngp_math.h"
#include <stdio.h>
#include <vector>

int main() {
    double nu, u, last_nu = -1.0;
    CovParams P{};
    bool ok = false;
    std::vector<double> tab;
    double costab[NNGP_MT_NC * NNGP_MT_NC];
    nngp_matern_costab(costab);
    while (scanf("%lf %lf", &nu, &u) == 2) {
        if (nu != last_nu) {
            P = nngp_cov_params_nu(NNGP_KIND_MATERN, 1.0, 1.0, 0.0, nu);
            ok = nngp_matern_table_setup(P);
            tab.assign((size_t)P.mt_noct * NNGP_MT_K * NNGP_MT_NC, 0.0);
            if (ok) {
                for (int b = 0; b < P.mt_noct * NNGP_MT_K; ++b) {
                    double rho[NNGP_MT_NC];
                    for (int k = 0; k < NNGP_MT_NC; ++k)
                        rho[k] = nngp_matern_rho(P, sqrt(nngp_matern_bin_t(P, b, nngp_matern_node(k))));
                    nngp_matern_bin_fit(P, b, rho, costab, &tab[(size_t)b * NNGP_MT_NC]);
                }
            }
            last_nu = nu;
        }
        // d2 = u^2 with the kernels' floor for coincident points (nngp_d2)
        const double d2 = fma(u, u, 0x1p-1000);
        if (ok)
            printf("%a %d\n", nngp_matern_tab(P, tab.data(), d2), P.mt_noct);
        else
            printf("nan 0\n");
    }
    return 0;
}
