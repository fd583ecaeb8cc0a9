/*
 * The C ABI of libnngp_hip.so used directly from C (no Python, no torch): the binding
 * a compiled caller of the reference's path would write.
 *
 *   capi_demo N M SEED  ->  prints "loglik <value> first_bad <i> F0 <F[n-1]>"
 *
 * Coordinates: SplitMix64 uniforms in [0,1)^2, values N(0,1) by Box-Muller from the
 * same stream (so tests/test_gpu_api.py can regenerate them); exponential covariance
 * sigma2 = 1, phi = 30, tau2 = 0.1.  Device memory from hipMalloc, default stream.
 */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../include/nngp.h"

static uint64_t sm_state;
static double uniform01(void) {
    uint64_t z = (sm_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (double)(z >> 11) * 0x1p-53;
}

#define CHECK_HIP(x)                                                  \
    do {                                                              \
        if ((x) != hipSuccess) {                                      \
            fprintf(stderr, "HIP error at %s:%d\n", __FILE__, __LINE__); \
            return 2;                                                 \
        }                                                             \
    } while (0)
#define CHECK_NNGP(x)                                                          \
    do {                                                                       \
        if ((x) != NNGP_OK) {                                                  \
            fprintf(stderr, "nngp error at %s:%d: %s\n", __FILE__, __LINE__, nngp_last_error()); \
            return 3;                                                          \
        }                                                                      \
    } while (0)

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 100000;
    const int32_t m = argc > 2 ? atoi(argv[2]) : 15;
    sm_state = argc > 3 ? strtoull(argv[3], NULL, 10) : 1;
    double* xy = (double*)malloc(sizeof(double) * 2 * n);
    double* v = (double*)malloc(sizeof(double) * n);
    for (int64_t i = 0; i < 2 * n; ++i) xy[i] = uniform01();
    for (int64_t i = 0; i < n; ++i) {
        const double u1 = uniform01() + 0x1p-54, u2 = uniform01();
        v[i] = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
    }
    double *d_xy, *d_v, *d_B, *d_F, *d_p;
    int32_t* d_nbr;
    void *ws_knn, *ws_bf;
    const size_t knn_bytes = nngp_knn_workspace_bytes(n, 2, m);
    const size_t bf_bytes = nngp_bf_sweep_workspace_bytes(n, m, NNGP_COV_EXPONENTIAL, 2, NNGP_ALGO_AUTO);
    CHECK_HIP(hipMalloc((void**)&d_xy, sizeof(double) * 2 * n));
    CHECK_HIP(hipMalloc((void**)&d_v, sizeof(double) * n));
    CHECK_HIP(hipMalloc((void**)&d_nbr, sizeof(int32_t) * n * (m > 0 ? m : 1)));
    CHECK_HIP(hipMalloc((void**)&d_B, sizeof(double) * n * (m > 0 ? m : 1)));
    CHECK_HIP(hipMalloc((void**)&d_F, sizeof(double) * n));
    CHECK_HIP(hipMalloc((void**)&d_p, sizeof(double) * 4));
    CHECK_HIP(hipMalloc(&ws_knn, knn_bytes));
    CHECK_HIP(hipMalloc(&ws_bf, bf_bytes > 0 ? bf_bytes : 256));
    CHECK_HIP(hipMemset(ws_bf, 0, 256)); /* the sweep workspace's header starts at zero (nngp.h) */
    CHECK_HIP(hipMemcpy(d_xy, xy, sizeof(double) * 2 * n, hipMemcpyHostToDevice));
    CHECK_HIP(hipMemcpy(d_v, v, sizeof(double) * n, hipMemcpyHostToDevice));

    /* NNGP._make_s_neighbor_sets (nngp.py:49-62) */
    CHECK_NNGP(nngp_knn_prior(d_xy, n, 2, m, 0, n, d_nbr, ws_knn, knn_bytes, NULL));
    /* _CNs / _Ccross / _Cs / _Bsi / _Fsi (nngp.py:73-96) + the log-likelihood for every location */
    CHECK_NNGP(nngp_bf_sweep(d_xy, n, 2, d_nbr, NULL, n, m, 0, NNGP_COV_EXPONENTIAL, 1.0, 30.0, 0.1, /*nu*/ 0.0, d_v,
                             d_B, d_F, NULL, d_p, ws_bf, bf_bytes, NNGP_ALGO_AUTO, NULL));
    double p[4], Flast;
    CHECK_HIP(hipMemcpy(p, d_p, sizeof p, hipMemcpyDeviceToHost));
    CHECK_HIP(hipMemcpy(&Flast, d_F + (n - 1), sizeof(double), hipMemcpyDeviceToHost));
    printf("loglik %.17g first_bad %lld F_last %.17g lib %s\n", nngp_loglik_from_partials(p, n), (long long)p[2],
           Flast, nngp_version());
    hipFree(d_xy);
    hipFree(d_v);
    hipFree(d_nbr);
    hipFree(d_B);
    hipFree(d_F);
    hipFree(d_p);
    hipFree(ws_knn);
    hipFree(ws_bf);
    free(xy);
    free(v);
    return p[2] >= 0 ? 4 : 0;
}
