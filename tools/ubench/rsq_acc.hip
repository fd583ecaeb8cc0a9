// Accuracy of v_rsq_f64 on gfx950: max relative error of __builtin_amdgcn_rsq(x) vs
// 1/sqrt(x) (host long double) over log-uniform x in [2^-60, 2^60] and [0.5, 2).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

__global__ void k(const double* x, double* y, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = __builtin_amdgcn_rsq(x[i]);
}

int main() {
    const int n = 1 << 22;
    std::vector<double> x(n), y(n);
    srand(7);
    for (int i = 0; i < n; ++i) {
        double u = (double)rand() / RAND_MAX;
        x[i] = (i & 1) ? ldexp(1.0, -60) * pow(2.0, 120.0 * u) : 0.5 + 1.5 * u;
    }
    double *dx, *dy;
    hipMalloc(&dx, n * 8);
    hipMalloc(&dy, n * 8);
    hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dx, dy, n);
    hipMemcpy(y.data(), dy, n * 8, hipMemcpyDeviceToHost);
    long double emax = 0;
    double xw = 0;
    for (int i = 0; i < n; ++i) {
        long double r = 1.0L / sqrtl((long double)x[i]);
        long double e = fabsl((y[i] - r) / r);
        if (e > emax) { emax = e; xw = x[i]; }
    }
    printf("v_rsq_f64 max rel err %.3Le = 2^%.2f (at x=%.17g)\n", emax, (double)log2l(emax), xw);
    return 0;
}
