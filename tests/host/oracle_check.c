/* Sanitizer driver for the C oracle (oracle/nngp_oracle.c), built by tests/test_sanitizers.py
 * with -fsanitize=address,undefined: every entry point on small inputs, including the edge
 * cases the tests use (m = 0, N <= m, rows past the prefix, bad rows, every kind, 1..3 dims,
 * duplicates), so an out-of-bounds access or UB in the checker itself fails loudly.
 * Prints "ok <checksum>" on success. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int oracle_knn_prior(const double *coords, int64_t n, int32_t dim, int32_t m, int64_t q0, int64_t q1, int32_t *nbr);
int oracle_knn_prior_rows(const double *coords, int64_t n, int32_t dim, int32_t m, const int64_t *rows,
                          int64_t n_rows, int32_t *nbr);
int oracle_knn_prior_kdtree_rebuild(const double *coords, int64_t n, int32_t dim, int32_t m, int64_t q0, int64_t q1,
                                    int32_t *nbr);
int oracle_bf_sweep(const double *coords, const int32_t *nbr, int64_t n, int32_t dim, int32_t m, int32_t kind,
                    const double *theta, const double *values, double *Bout, double *Fout, double *partials,
                    int64_t i0, int64_t i1);
int oracle_nngp_simulate(const int32_t *nbr, const double *B, const double *F, int64_t n, int32_t m,
                         const double *eps, double *w);

static uint64_t rng = 88172645463325252ull;
static double urand(void) {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return (double)(rng >> 11) * 0x1p-53;
}

int main(void) {
    double check = 0.0;
    const int64_t n = 700;
    for (int dim = 1; dim <= 3; ++dim) {
        for (int32_t m = 0; m <= 17; m += 17 / 3 + 1) {
            double *c = malloc(sizeof(double) * (size_t)(n * dim));
            double *y = malloc(sizeof(double) * (size_t)n);
            for (int64_t i = 0; i < n * dim; ++i) c[i] = urand();
            for (int64_t i = 0; i < n; ++i) y[i] = urand() - 0.5;
            memcpy(c + 50 * dim, c + 10 * dim, sizeof(double) * (size_t)dim); /* a duplicate point */
            const size_t nm = (size_t)(n * (m > 0 ? m : 1));
            int32_t *a = malloc(sizeof(int32_t) * nm), *b = malloc(sizeof(int32_t) * nm);
            if (oracle_knn_prior(c, n, dim, m, 0, n, a) != 0) return 1;
            if (oracle_knn_prior_kdtree_rebuild(c, n, dim, m, 0, n, b) != 0) return 2;
            if (m > 0 && memcmp(a, b, sizeof(int32_t) * (size_t)(n * m)) != 0) return 3;
            int64_t rows[4] = {n - 1, 0, 1, 333};
            if (oracle_knn_prior_rows(c, n, dim, m, rows, 4, b) != 0) return 4;
            double *B = malloc(sizeof(double) * nm), *F = malloc(sizeof(double) * (size_t)n), p[3];
            for (int kind = 0; kind < 5; ++kind) {
                const double theta[3] = {1.3, kind == 4 ? 3.0 : 7.0, 0.2};
                if (oracle_bf_sweep(c, a, n, dim, m, kind, theta, y, B, F, p, 0, n) != 0) return 5;
                check += p[0] + p[1];
                if (oracle_bf_sweep(c, a + 5 * m, n, dim, m, kind, theta, NULL, NULL, NULL, p, 5, 9) != 0) return 6;
            }
            const double th0[3] = {1.0, 5.0, 0.0};
            if (oracle_bf_sweep(c, a, n, dim, m, 0, th0, NULL, B, F, p, 0, n) != 0) return 7;
            if (p[2] >= 0.0) { /* the duplicate makes C_N singular somewhere: flagged, not a crash */
                check += p[2];
            } else {
                double *w = malloc(sizeof(double) * (size_t)n);
                if (oracle_nngp_simulate(a, B, F, n, m, y, w) != 0) return 8;
                check += w[n - 1];
                free(w);
            }
            free(c);
            free(y);
            free(a);
            free(b);
            free(B);
            free(F);
        }
    }
    printf("ok %.6g\n", check);
    return 0;
}
