// Accuracy of v_sqrt_f64 on gfx950 (__builtin_amdgcn_sqrt): error in ulps against the correctly
// rounded sqrt (host libm) over log-uniform x in [2^-1000, 2^1000], [0.5, 2) and the sweep's
// range of squared distances [2^-40, 2^4]; also the same for the kernels' current refinement
// (nngp_sqrt: v_rsq_f64 + a second-order correction, 5 VALU) for comparison.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

__global__ void k(const double* x, double* y, double* z, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double v = x[i];
    y[i] = __builtin_amdgcn_sqrt(v);
    const double r = __builtin_amdgcn_rsq(v);
    const double s = v * r;
    const double e = fma(-s, r, 1.0);
    const double g = e * fma(0.375, e, 0.5);
    z[i] = fma(s, g, s);
}

static double ulps(double got, double ref) {
    return fabs(got - ref) / (nextafter(ref, INFINITY) - ref);
}

int main() {
    const int n = 1 << 23;
    std::vector<double> x(n), y(n), z(n);
    srand(11);
    for (int i = 0; i < n; ++i) {
        double u = (double)rand() / RAND_MAX;
        switch (i % 3) {
            case 0: x[i] = ldexp(1.0, -1000) * pow(2.0, 2000.0 * u); break;
            case 1: x[i] = 0.5 + 1.5 * u; break;
            default: x[i] = ldexp(1.0, -40) * pow(2.0, 44.0 * u); break;
        }
    }
    double *dx, *dy, *dz;
    hipMalloc(&dx, n * 8);
    hipMalloc(&dy, n * 8);
    hipMalloc(&dz, n * 8);
    hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dx, dy, dz, n);
    hipMemcpy(y.data(), dy, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(z.data(), dz, n * 8, hipMemcpyDeviceToHost);
    double ey = 0, ez = 0, xy = 0, xz = 0;
    long ny = 0, nz = 0;
    for (int i = 0; i < n; ++i) {
        const double r = sqrt(x[i]);
        const double a = ulps(y[i], r), b = ulps(z[i], r);
        if (a > ey) { ey = a; xy = x[i]; }
        if (b > ez) { ez = b; xz = x[i]; }
        ny += y[i] != r;
        nz += z[i] != r;
    }
    printf("v_sqrt_f64: max %.3f ulp (x=%.17g), %ld of %d not correctly rounded\n", ey, xy, ny, n);
    printf("v_rsq_f64 + second-order correction (nngp_sqrt): max %.3f ulp (x=%.17g), %ld of %d not correctly rounded\n",
           ez, xz, nz, n);
    return 0;
}
