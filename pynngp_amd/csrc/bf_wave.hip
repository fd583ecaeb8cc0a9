// One-wave-per-location B/F + log-likelihood kernel (the north_star layout):
// lane a owns row a of the (m+1)x(m+1) joint block in VGPRs, column values are
// broadcast with v_readlane, so any m <= 63 runs without LDS.  Same math and
// outputs as bf_lane (bf_sweep.hip, which documents the formulation and the
// reference methods nngp.py:73-96 it replaces); used for m > 16 and as the
// comparison point for the lane kernel.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nngp_math.h"
#include "nngp_internal.h"

namespace nngp {

// --------------------------------------------------------------------------
// one wave per location; lane a owns row a of the joint block (NR >= M+1 rows)
// --------------------------------------------------------------------------
// Generic path: the kind and the dimension are runtime arguments (wave-uniform, so the
// kind switch is a scalar branch and only one path runs), coordinates are zero-padded to
// three axes (the extra terms of the squared distance add exact zeros, so D = 1 / 2 give the
// bits of their own point_d2<D>): three instantiations instead of one per (kind, D).
template <int NR, int KIND>
__device__ __forceinline__ void wave_row(const CovParams& P, const double* etab, const double (&xg)[3], int lane,
                                         double (&row)[NR]) {
#pragma unroll
    for (int b = 0; b < NR; ++b) {
        double xb[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) xb[k] = wave_bcast(xg[k], b);
        const double c = nngp_cov_d2<KIND>(P, etab, point_d2<3>(xg, xb));
        row[b] = b == lane ? P.diag : c;
    }
}

// General-smoothness Matern: each entry is a Bessel-function evaluation with data-dependent loops
// (nngp_matern_rho), so the wave evaluates the joint block's M (M + 1) / 2 distinct entries once,
// spread over all 64 lanes (entry e = (a, b), a > b, e = a (a - 1) / 2 + b; the two points'
// coordinates come from lanes a and b by ds_bpermute), into this wave's LDS slice, and lane a then
// reads its row back -- instead of each lane evaluating its own row (one entry per lane and step,
// lanes past the row idle: ~1/8 of the lanes busy at m = 15).  Intra-wave LDS exchange: a
// wavefront-scope release / acquire around a wave barrier (the waves of a block run different
// numbers of locations, so no block barrier).
template <int NR>
__device__ __forceinline__ void wave_row_matern(const CovParams& P, const double (&xg)[3], int lane, int M,
                                                double* __restrict__ cb, double (&row)[NR]) {
    const int ne = (M + 1) * M / 2;
#pragma nounroll
    for (int e0 = 0; e0 < ne; e0 += 64) {  // wave-uniform trip count: the shuffles run with every lane active
        const int e = min(e0 + lane, ne - 1);
        int a = (int)(0.5 * (1.0 + sqrt(1.0 + 8.0 * (double)e)));
        while (a * (a - 1) / 2 > e) --a;
        while ((a + 1) * a / 2 <= e) ++a;
        const int b = e - a * (a - 1) / 2;
        double xa[3], xb[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            xa[k] = __shfl(xg[k], a);
            xb[k] = __shfl(xg[k], b);
        }
        if (e0 + lane < ne) cb[e] = nngp_cov_d2<NNGP_KIND_MATERN>(P, nullptr, point_d2<3>(xa, xb));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int base = lane * (lane - 1) / 2;
#pragma unroll
    for (int b = 0; b < NR; ++b) row[b] = b == lane ? P.diag : (b < lane && lane <= M ? cb[base + b] : 0.0);
    // the slice is rewritten for the next location only after every lane has read its row
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// MATERN: the general-smoothness Matern kind in an instantiation of its own (its Bessel loops would
// raise the register peak of the other kinds' kernel: 223 -> 264 VGPRs at NR = 64)
template <int NR, bool MATERN>
__global__ __launch_bounds__(256) void bf_wave(const double* __restrict__ coords, int64_t n_points, int dim, int kind,
                                               const int32_t* __restrict__ nbr, const int32_t* __restrict__ order,
                                               int64_t n_rows, int64_t i0, int M,
                                               const CovParams P, const double* __restrict__ values, const double* __restrict__ qcoords, const double* __restrict__ qvalues,
                                               double* __restrict__ Bout, double* __restrict__ Fout, double* __restrict__ Rout,
                                               double* __restrict__ bpart) {
    const int lane = threadIdx.x & 63;
    __shared__ double etab[NNGP_EXP_TAB_N];
    // MATERN: one slice of the joint block's distinct entries per wave (4 waves per block)
    constexpr int kSlice = NR * (NR - 1) / 2;
    __shared__ double cbuf[MATERN ? 4 * kSlice : 1];
    nngp_exp_table_load(etab, P.sigma2);
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t n_waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    double lf_acc = 0.0, q_acc = 0.0;  // lane 0 accumulates this wave's locations in row order
    double badp = INFINITY, badi = INFINITY;

    for (int64_t rl = wave; rl < n_rows; rl += n_waves) {
        const int64_t rr = order != nullptr ? (int64_t)order[rl] : rl;
        const int64_t i = i0 + rr;
        // lane a < M: neighbour slot a; lane M: the location itself; lanes > M: far-away identity rows
        const int32_t jr = M > 0 ? nbr[rl * M + (lane < M ? lane : 0)] : -1;  // nbr may be null for m = 0
        const int32_t j = (lane < M) ? jr : -1;
        const bool is_self = lane == M;
        const bool in_range = j >= 0 && (int64_t)j < n_points;
        const bool bad_index = j != -1 && !in_range;
        const double* pc = is_self ? qcoords + i * dim
                                   : (in_range ? coords + (int64_t)j * dim : far_point<1>(lane));  // far: (x, 0, 0)
        const double* pv = is_self ? (qvalues != nullptr ? qvalues + i : kZeroValue)
                                   : ((values != nullptr && in_range) ? values + j : kZeroValue);
        double xg[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) xg[k] = (k < dim && (k == 0 || is_self || in_range)) ? pc[k] : 0.0;
        double zv = *pv;

        // row `lane` of the joint block (entries b <= lane are meaningful)
        double row[NR];
        if constexpr (MATERN) {
            wave_row_matern<NR>(P, xg, lane, M, cbuf + (threadIdx.x >> 6) * kSlice, row);
        } else {
            switch (kind) {
                case 0: wave_row<NR, 0>(P, etab, xg, lane, row); break;
                case 1: wave_row<NR, 1>(P, etab, xg, lane, row); break;
                case 2: wave_row<NR, 2>(P, etab, xg, lane, row); break;
                case 3: wave_row<NR, 3>(P, etab, xg, lane, row); break;
                default: wave_row<NR, 4>(P, etab, xg, lane, row); break;
            }
        }
        bool bad = false;
        double ip_mine = 1.0;  // lane p keeps 1/L[p][p]
#pragma unroll
        for (int p = 0; p < NR - 1; ++p) {
            if (p < M) {
                const double piv = wave_bcast(row[p], p);
                bad |= !(piv > 0.0);
                const double ip = nngp_rsqrt(piv);
                if (lane == p) ip_mine = ip;
                row[p] *= ip;  // lane > p: L[lane][p]; lane p: sqrt(pivot)
                const double l = row[p];
                if (lane == p) zv *= ip;
                const double zp = wave_bcast(zv, p);
                if (lane > p) zv = fma(-l, zp, zv);
#pragma unroll
                for (int b = p + 1; b < NR; ++b) {
                    if (b <= M) {
                        const double lb = wave_bcast(l, b);
                        if (lane >= b) row[b] = fma(-l, lb, row[b]);
                    }
                }
            }
        }
        double F = 0.0;
#pragma unroll
        for (int b = 0; b < NR; ++b)
            if (b == M) F = wave_bcast(row[b], M);
        const double res = wave_bcast(zv, M);
        bad |= !(F > 0.0);
        if (Bout != nullptr) {
            // B = L_N^{-T} v with v = row M of L; lane a ends with b_a
            double bmine = 0.0;
#pragma unroll
            for (int a = NR - 2; a >= 0; --a) {
                if (a < M) {
                    const double term = (lane > a && lane < M) ? row[a] * bmine : 0.0;
                    const double va = wave_bcast(row[a], M);
                    const double s = va - wave_sum(term);
                    const double ipa = wave_bcast(ip_mine, a);
                    if (lane == a) bmine = s * ipa;
                }
            }
            if (lane < M) Bout[rr * M + lane] = bad ? NAN : (in_range ? bmine : 0.0);
        }
        if (lane == 0) {
            if (Fout != nullptr) Fout[rr] = bad ? NAN : F;
            if (Rout != nullptr) Rout[rr] = bad ? NAN : res;
            lf_acc += log(F);
            q_acc += res * res / F;
            if (bad) badp = fmin(badp, (double)i);
        }
        if (__any(bad_index) && lane == 0) badi = fmin(badi, (double)i);
    }
    block_partials_store(lf_acc, q_acc, badp, badi, bpart, blockIdx.x);
}

template <int NR>
static void launch_wave(const BfArgs& a, const CovParams& P, int64_t n_blocks, hipStream_t s) {
    auto kern = a.kind == NNGP_KIND_MATERN ? bf_wave<NR, true> : bf_wave<NR, false>;
    hipLaunchKernelGGL(kern, dim3((unsigned)n_blocks), dim3(256), 0, s, a.coords, a.n_points, a.dim,
                       a.kind, a.nbr, a.order, a.n_rows, a.i0, a.m, P, a.values, a.qcoords, a.qvalues, a.B, a.F, a.R,
                       a.bpart);
}

int64_t bf_wave_blocks(int64_t n_rows) {
    // persistent grid of 4-wave blocks: at most 2048 blocks (256 CUs x 32 waves), about one wave per location
    const int64_t b = (n_rows + 3) / 4;
    return b < 1 ? 1 : (b > 2048 ? 2048 : b);
}

// every kind and dimension: the generic path (any m <= 63)
bool bf_wave_launch(const BfArgs& a, const CovParams& P, int64_t nb, hipStream_t s) {
    if (a.dim < 1 || a.dim > 3 || a.kind < 0 || a.kind > NNGP_KIND_MATERN) return false;
    if (a.m + 1 <= 16)
        launch_wave<16>(a, P, nb, s);
    else if (a.m + 1 <= 32)
        launch_wave<32>(a, P, nb, s);
    else if (a.m + 1 <= 64)
        launch_wave<64>(a, P, nb, s);
    else
        return false;
    return true;
}

}  // namespace nngp
