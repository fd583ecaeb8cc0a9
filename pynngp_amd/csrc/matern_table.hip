// Per-launch table of the Matern-nu correlation for the fused pair kernel (nngp_math.h, "Matern-nu by
// table"), stream-ordered before the sweep that reads it.
#include "nngp_internal.h"
#include "nngp_math.h"

namespace nngp {

// One block per octave of t: its NNGP_MT_K bins x NNGP_MT_NC nodes evaluate rho with the direct evaluation
// (nngp_matern_rho; the Temme / continued-fraction loops are the kernel's critical path), then the fit of
// nngp_matern_bin_fit in parallel -- one thread per (bin, Chebyshev coefficient) for the transform of the
// deviations from the middle node's value, one per (bin, power of f) for the monomial coefficients --
// with the same sums in the same order as the serial host version.
constexpr int kMtThreads = (NNGP_MT_K * NNGP_MT_NC + 63) / 64 * 64;

__global__ __launch_bounds__(kMtThreads) void matern_table_kernel(const CovParams P, double* __restrict__ tab) {
    __shared__ double rho[NNGP_MT_K][NNGP_MT_NC];
    __shared__ double cheb[NNGP_MT_K][NNGP_MT_NC];
    __shared__ double costab[NNGP_MT_NC * NNGP_MT_NC];
    // coefficients of f^k in the shifted Chebyshev polynomial T_j(2 f - 1) (exact integers; rows j, columns
    // k): T_0 = 1, T_1 = 2 f - 1, T_{j+1} = 2 (2 f - 1) T_j - T_{j-1}, the host fit's recurrence
    __shared__ double scheb[NNGP_MT_NC][NNGP_MT_NC];
    const int o = blockIdx.x;
    const int tid = threadIdx.x;
    const int jb = tid / NNGP_MT_NC, k = tid % NNGP_MT_NC;
    const bool work = tid < NNGP_MT_K * NNGP_MT_NC;
    const int b = o * NNGP_MT_K + jb;
    if (o == 0 || o >= P.mt_noct - 1) {  // rho = 1 below the table, 0 above
        if (work) tab[(int64_t)b * NNGP_MT_NC + k] = (o == 0 && k == 0) ? 1.0 : 0.0;
        return;
    }
    for (int i = tid; i < NNGP_MT_NC * NNGP_MT_NC; i += kMtThreads)
        costab[i] = cos(3.141592653589793 * (i / NNGP_MT_NC) * ((i % NNGP_MT_NC) + 0.5) / NNGP_MT_NC);
    if (tid == 0) {  // row by row (a few hundred exact operations)
        for (int j = 0; j < NNGP_MT_NC; ++j)
            for (int k = 0; k < NNGP_MT_NC; ++k) {
                double v;
                if (j == 0) v = k == 0 ? 1.0 : 0.0;
                else if (j == 1) v = k == 0 ? -1.0 : (k == 1 ? 2.0 : 0.0);
                else v = (k > 0 ? 4.0 * scheb[j - 1][k - 1] : 0.0) - 2.0 * scheb[j - 1][k] - scheb[j - 2][k];
                scheb[j][k] = v;
            }
    }
    if (work) rho[jb][k] = nngp_matern_rho(P, sqrt(nngp_matern_bin_t(P, b, nngp_matern_node(k))));
    __syncthreads();
    if (work) {  // Chebyshev coefficient c_k of bin jb (k plays j's role here)
        const double vref = rho[jb][NNGP_MT_NC / 2];
        double c = 0.0;
#pragma unroll
        for (int i = 0; i < NNGP_MT_NC; ++i) c = fma(rho[jb][i] - vref, costab[k * NNGP_MT_NC + i], c);
        cheb[jb][k] = c * ((k == 0 ? 1.0 : 2.0) / NNGP_MT_NC);
    }
    __syncthreads();
    if (work) {  // coefficient of f^k: sum_j c_j [f^k] T_j(2 f - 1), j ascending (then the middle value)
        double a = 0.0;
#pragma unroll
        for (int j = 0; j < NNGP_MT_NC; ++j) a = fma(cheb[jb][j], scheb[j][k], a);
        if (k == 0) a += rho[jb][NNGP_MT_NC / 2];
        tab[(int64_t)b * NNGP_MT_NC + k] = a;
    }
}

hipError_t matern_table_launch(const CovParams& P, double* tab, hipStream_t s) {
    hipLaunchKernelGGL(matern_table_kernel, dim3((unsigned)P.mt_noct), dim3(kMtThreads), 0, s, P, tab);
    return hipGetLastError();
}

// the table geometry of nu (nngp_matern_table_setup: a few thousand host evaluations of rho), cached per
// thread for the last few nu: mt_e0, mt_noct, mt_series, mt_A into *p; false when it does not fit
bool matern_table_params(double nu, CovParams* p) {
    constexpr int kSlots = 8;
    thread_local double c_nu[kSlots] = {0, 0, 0, 0, 0, 0, 0, 0};
    thread_local CovParams c_p[kSlots];
    thread_local int c_next = 0;
    int hit = -1;
    for (int i = 0; i < kSlots; ++i)
        if (c_nu[i] == nu) hit = i;
    if (hit < 0) {
        CovParams q = nngp_cov_params_nu(NNGP_KIND_MATERN, 1.0, 1.0, 0.0, nu);
        nngp_matern_table_setup(q);
        hit = c_next;
        c_nu[hit] = nu;
        c_p[hit] = q;
        c_next = (c_next + 1) % kSlots;
    }
    p->mt_e0 = c_p[hit].mt_e0;
    p->mt_noct = c_p[hit].mt_noct;
    p->mt_series = c_p[hit].mt_series;
    p->mt_A = c_p[hit].mt_A;
    return p->mt_noct <= NNGP_MT_MAX_OCT;
}

bool matern_table_extent(double nu, int* e0, int* noct) {
    CovParams p{};
    const bool ok = matern_table_params(nu, &p);
    *e0 = p.mt_e0;
    *noct = p.mt_noct;
    return ok;
}

}  // namespace nngp
