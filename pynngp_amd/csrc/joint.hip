// Joint-block distances for a caller-evaluated covariance (nngp_joint_dist; SURVEY.md 8(a) A2: the
// reference's `cov` is an arbitrary plug-in, nngp.py:6,12).  For nbr row t (location i = i0 + (order ?
// order[t] : t)), the joint rows a = 0..m are the m neighbour slots and the location itself (row m, from
// qcoords); entry (a, b), b <= a, of the packed lower triangle goes to
//     dist[(a (a + 1) / 2 + b) * n_rows + t]
// (entry-major, the layout nngp_bf_sweep_blocks / bf_pairb<M, NNGP_KIND_BLOCKS> reads): the Euclidean
// distance of the two points, 0 on the diagonal, +inf when either slot holds no point (index -1 or out
// of range).  The caller maps the distances through its covariance function on the GPU (any elementwise
// torch expression) and passes the result to nngp_bf_sweep_blocks.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/nngp.h"
#include "nngp_internal.h"

namespace nngp {

// A block handles kJRows consecutive rows: their (m+1) points go to LDS once (coordinates padded to
// three, a NaN marker for slots without a point), then thread k computes entries e = k / kJRows,
// e + 256 / kJRows, ... of row k % kJRows -- every store instruction writes whole 256-B runs of
// consecutive rows of one entry.  (One thread per row re-gathered each point (m+2)/2 times through
// nbr: 2.6-2.8 ms at N = 1e6, m = 15.)
constexpr int kJRows = 32;

__global__ __launch_bounds__(256) void joint_dist_kernel(const double* __restrict__ coords, int64_t n_points, int dim,
                                                         const double* __restrict__ qcoords,
                                                         const int32_t* __restrict__ nbr,
                                                         const int32_t* __restrict__ order, int64_t n_rows, int m,
                                                         int64_t i0, double* __restrict__ dist) {
    __shared__ double pts[kJRows * (NNGP_MAX_M + 1) * 3];  // [row][joint row][axis]
    const int64_t t0 = (int64_t)blockIdx.x * kJRows;
    const int nr = m + 1;
    for (int k = threadIdx.x; k < kJRows * nr; k += blockDim.x) {
        const int r = k / nr, a = k % nr;
        const int64_t t = t0 + r;
        double x[3] = {NAN, NAN, NAN};
        if (t < n_rows) {
            const double* p = nullptr;
            if (a == m) {
                p = qcoords + (i0 + (order != nullptr ? (int64_t)order[t] : t)) * dim;
            } else {
                const int32_t j = nbr[t * m + a];
                if (j >= 0 && (int64_t)j < n_points) p = coords + (int64_t)j * dim;
            }
            if (p != nullptr)
                for (int c = 0; c < 3; ++c) x[c] = c < dim ? p[c] : 0.0;
        }
        for (int c = 0; c < 3; ++c) pts[(r * nr + a) * 3 + c] = x[c];
    }
    __syncthreads();
    const int r = threadIdx.x % kJRows;
    const int64_t t = t0 + r;
    if (t >= n_rows) return;
    const int64_t ne = (int64_t)nr * (nr + 1) / 2;
    for (int64_t e = threadIdx.x / kJRows; e < ne; e += blockDim.x / kJRows) {
        int a = (int)(0.5 * (sqrt(8.0 * (double)e + 1.0) - 1.0));
        while ((int64_t)a * (a + 1) / 2 > e) --a;
        while ((int64_t)(a + 1) * (a + 2) / 2 <= e) ++a;
        const int b = (int)(e - (int64_t)a * (a + 1) / 2);
        const double* pa = pts + (r * nr + a) * 3;
        const double* pb = pts + (r * nr + b) * 3;
        double d;
        if (isnan(pa[0]) || isnan(pb[0])) {
            d = INFINITY;
        } else if (a == b) {
            d = 0.0;
        } else {
            double s = 0.0;
            for (int c = 0; c < dim; ++c) {
                const double df = pa[c] - pb[c];
                s = fma(df, df, s);
            }
            d = sqrt(s);
        }
        dist[e * n_rows + t] = d;
    }
}

// Elementwise general-smoothness Matern correlation (nngp_matern_eval): out[k] = rho(u[k]) of
// nngp_math.h (u >= 0; +inf -> 0), for a caller covariance built on it (IsotropicCovariance).
__global__ __launch_bounds__(256) void matern_eval_kernel(const double* __restrict__ u, int64_t n, const CovParams P,
                                                          double* __restrict__ out) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const double x = u[k];
    out[k] = x > 3000.0 + 30.0 * P.nu ? 0.0 : nngp_matern_rho(P, x);  // e^-x has underflowed
}

hipError_t matern_eval_launch(const double* u, int64_t n, double nu, double* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const CovParams P = nngp_cov_params_nu(NNGP_KIND_MATERN, 1.0, 1.0, 0.0, nu);
    hipLaunchKernelGGL(matern_eval_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, u, n, P, out);
    return hipGetLastError();
}

hipError_t joint_dist_launch(const double* coords, int64_t n_points, int dim, const double* qcoords,
                             const int32_t* nbr, const int32_t* order, int64_t n_rows, int m, int64_t i0, double* dist,
                             hipStream_t s) {
    if (n_rows == 0) return hipSuccess;
    hipLaunchKernelGGL(joint_dist_kernel, dim3((unsigned)((n_rows + kJRows - 1) / kJRows)), dim3(256), 0, s, coords,
                       n_points, dim, qcoords, nbr, order, n_rows, m, i0, dist);
    return hipGetLastError();
}

}  // namespace nngp
