// Per-launch table of the Matern-nu correlation for the fused pair kernel (nngp_math.h, "Matern-nu by
// table"): one block per octave of t = (phi d)^2; its 4 bins x 14 Chebyshev nodes evaluate rho with the
// direct Temme / continued-fraction evaluation (nngp_matern_rho) at full lane use, then one thread per bin
// turns the node values into the bin's monomial coefficients (nngp_matern_bin_fit, the same code as the
// host check tests/host/matern_table_check.cpp).  Stream-ordered before the sweep that reads it.
#include "nngp_internal.h"
#include "nngp_math.h"

namespace nngp {

__global__ __launch_bounds__(64) void matern_table_kernel(const CovParams P, double* __restrict__ tab) {
    static_assert(NNGP_MT_K * NNGP_MT_NC <= 64, "one node per thread");
    __shared__ double rho[NNGP_MT_K][NNGP_MT_NC];
    __shared__ double costab[NNGP_MT_NC * NNGP_MT_NC];
    const int o = blockIdx.x;
    const int tid = threadIdx.x;
    for (int i = tid; i < NNGP_MT_NC * NNGP_MT_NC; i += 64)
        costab[i] = cos(3.141592653589793 * (i / NNGP_MT_NC) * ((i % NNGP_MT_NC) + 0.5) / NNGP_MT_NC);
    if (o > 0 && o < P.mt_noct - 1 && tid < NNGP_MT_K * NNGP_MT_NC) {
        const int jb = tid / NNGP_MT_NC, k = tid % NNGP_MT_NC;
        rho[jb][k] = nngp_matern_rho(P, sqrt(nngp_matern_bin_t(P, o * NNGP_MT_K + jb, nngp_matern_node(k))));
    }
    __syncthreads();
    if (tid < NNGP_MT_K) {
        double coef[NNGP_MT_NC];
        const int b = o * NNGP_MT_K + tid;
        nngp_matern_bin_fit(P, b, rho[tid], costab, coef);
#pragma unroll
        for (int k = 0; k < NNGP_MT_NC; ++k) tab[(int64_t)b * NNGP_MT_NC + k] = coef[k];
    }
}

hipError_t matern_table_launch(const CovParams& P, double* tab, hipStream_t s) {
    hipLaunchKernelGGL(matern_table_kernel, dim3((unsigned)P.mt_noct), dim3(64), 0, s, P, tab);
    return hipGetLastError();
}

// table extent for smoothness nu (nngp_matern_table_setup at phi = 1), cached per thread for the last
// few nu: the setup evaluates rho and the small-t bound a few hundred times on the host
bool matern_table_extent(double nu, int* e0, int* noct) {
    constexpr int kSlots = 8;
    thread_local double c_nu[kSlots] = {0, 0, 0, 0, 0, 0, 0, 0};
    thread_local int c_e0[kSlots], c_noct[kSlots], c_next = 0;
    for (int i = 0; i < kSlots; ++i)
        if (c_nu[i] == nu) {
            *e0 = c_e0[i];
            *noct = c_noct[i];
            return *noct <= NNGP_MT_MAX_OCT;
        }
    CovParams p = nngp_cov_params_nu(NNGP_KIND_MATERN, 1.0, 1.0, 0.0, nu);
    nngp_matern_table_setup(p);
    c_nu[c_next] = nu;
    c_e0[c_next] = *e0 = p.mt_e0;
    c_noct[c_next] = *noct = p.mt_noct;
    c_next = (c_next + 1) % kSlots;
    return *noct <= NNGP_MT_MAX_OCT;
}

}  // namespace nngp
