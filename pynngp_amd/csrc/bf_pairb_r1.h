// Round-1 bf_pairb (non-persistent, sigma2 table, per-tile log), kept as algo 7 ("pairb_r1")
// for same-box A/B measurements against the round-2 kernel.
// B/F + log-likelihood sweep, two lanes per location, 2x2-blocked elimination
// ("pairb").  Same formulation and outputs as bf_lane / bf_group (bf_sweep.hip
// documents it and the reference methods nngp.py:73-96 it replaces): the
// (m+1)x(m+1) joint block [[C_N + tau2 I, c], [c^T, sigma2 + tau2]] with the value
// column appended, m elimination steps, B = L_N^{-T} v.
//
// The joint rows come in pairs (2t, 2t+1); lane q of a location's lane pair owns
// rows a = 2s + q ("local row s").  Row a stores its lower-triangle entries pair
// by pair in OWN-PARITY-FIRST order:
//     R[s][t][0] = entry (a, 2t + q)        (same parity as the lane)
//     R[s][t][1] = entry (a, 2t + 1 - q)    (the partner lane's parity)
// (t = s: [0] is the diagonal, [1] is (2s+1, 2s) in lane 1 and unused in lane 0).
// With that layout every step of a 2x2-blocked Cholesky addresses the same
// registers in both lanes, and the only cross-lane traffic is
//   * the diagonal 2x2 block of pair t (three DPP broadcasts), factored redundantly
//     by both lanes;
//   * one DPP swap ([1,0,3,2]) of each later local row's two panel entries, after
//     which a row's update reads its own lane's panel for the same-parity column
//     and the swapped panel for the other one;
// i.e. ~4 DPP moves per row pair and block step instead of a broadcast per column
// and step (bf_group<M, KIND, 2>).  The back-substitution uses the same trick: a
// lane's partial sums for columns (2t+q, 2t+1-q) combine as acc0 + swap(acc1).
// Covariances: lane q computes its own rows; partner coordinates come from one swap
// per pair.  Rows past M are far-away (decoupled) padding points.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bf_group.h"
#include "bf_pairb.h"
#include "nngp_internal.h"
#include "nngp_math.h"

namespace nngp {
namespace r1 {

template <int KIND, int VAR>
__device__ __forceinline__ double cov(const CovParams& P, const double* tab, double d2) {
    if (VAR & 1) return nngp_cov_unit<KIND>(P, tab, d2);
    return nngp_cov_d2<KIND>(P, tab, d2);
}


// Occupancy: up to m = NNGP_PAIRB_TWO_WAVES_MAX the compiler is asked for two waves per SIMD
// (<= 256 VGPRs): m = 16 / 17 then fit in 248 / 252 VGPRs without spills instead of
// 264 / 266 (one wave per SIMD).  Beyond it the block needs more registers than that.

// VAR (A/B of the round-2 changes one at a time): bit 0 -- unit-variance covariances
// (nngp_cov_unit, F scaled by sigma2 at the end); bit 1 -- a tile record with the log
// deferred to the fold (pairb_tile_store / bf_finalize_pairb) instead of log per lane.
template <int M, int KIND, int VAR>
__global__ __launch_bounds__(256) NNGP_PAIRB_ATTR void bf_pairb(const double2* __restrict__ coords, int64_t n_points,
                                                const int32_t* __restrict__ nbr, const int32_t* __restrict__ order,
                                                int64_t n_rows, int64_t i0, const CovParams Pc,
                                                const double* __restrict__ values, const double2* __restrict__ qcoords,
                                                const double* __restrict__ qvalues, double* __restrict__ Bout,
                                                double* __restrict__ Fout, double* __restrict__ Rout,
                                                double* __restrict__ bpart, double sigma2, int32_t* __restrict__ lexp) {
    static_assert(M >= 1 && M <= 24, "pairb instantiated for 1 <= m <= 24");
    constexpr int NR = M + 1;         // joint rows 0..M (row M = the location)
    constexpr int NP = (NR + 1) / 2;  // row pairs
    constexpr int T = M / 2;          // pairs made of two neighbour rows: full 2x2 block steps
    __shared__ double etab[NNGP_EXP_TAB_N];
    if (VAR & 1)
        nngp_exp_table_load_unit(etab);
    else
        nngp_exp_table_load(etab, Pc.sigma2);

    const int64_t blk = xcd_logical_block(blockIdx.x, gridDim.x);
    const int64_t tid = blk * blockDim.x + threadIdx.x;
    const int q = (int)(threadIdx.x & 1);
    const bool q1 = q == 1;
    const int64_t r = tid >> 1;
    const bool live = r < n_rows;
    const int64_t rl = live ? r : n_rows - 1;
    const int64_t rr = order != nullptr ? (int64_t)order[rl] : rl;
    const int64_t i = i0 + rr;

    // ---- gathers (branch-free, as bf_group): own rows a = 2s + q
    int32_t jn[NP];
#pragma unroll
    for (int s = 0; s < NP; ++s) {
        const int a = 2 * s + q;
        jn[s] = nbr[rl * M + (a < M ? a : M - 1)];
    }
    double ox[NP], oy[NP], z[NP];
    bool oval[NP];
    bool bad_index = false;
#pragma unroll
    for (int s = 0; s < NP; ++s) {
        const int a = 2 * s + q;
        const int32_t j = a < M ? jn[s] : -1;
        const bool in_range = j >= 0 && (int64_t)j < n_points;
        bad_index |= j >= 0 && !in_range;
        oval[s] = in_range;
        const bool self = a == M;
        const double2* pc = self ? qcoords + i : (in_range ? coords + j : kFarPoints + (a & 63));
        const double* pv = self ? (qvalues != nullptr ? qvalues + i : kZeroValue)
                                : ((values != nullptr && in_range) ? values + j : kZeroValue);
        const double2 x = *pc;
        ox[s] = x.x;
        oy[s] = x.y;
        z[s] = *pv;
    }

    // ---- covariances in own-parity-first order
    double R[NP][NP][2];
    {
        double px[NP], py[NP];
#pragma unroll
        for (int t = 0; t < NP; ++t) {
            px[t] = pr_swap(ox[t]);
            py[t] = pr_swap(oy[t]);
        }
#pragma unroll
        for (int s = 0; s < NP; ++s) {
#pragma unroll
            for (int t = 0; t < s; ++t) {
                R[s][t][0] = cov<KIND, VAR>(Pc, etab, nngp_d2(ox[s], oy[s], ox[t], oy[t]));
                R[s][t][1] = cov<KIND, VAR>(Pc, etab, nngp_d2(ox[s], oy[s], px[t], py[t]));
            }
            R[s][s][0] = Pc.diag;
            const double c = cov<KIND, VAR>(Pc, etab, nngp_d2(ox[s], oy[s], px[s], py[s]));
            R[s][s][1] = q1 ? c : 0.0;
        }
    }

    // ---- 2x2-blocked right-looking elimination of the neighbour columns 0..M-1.
    // After block step t: lane q's R[t][t][0] = 1 / L[2t+q][2t+q], R[t][t][1] = L[2t+1][2t]
    // (both lanes), rows s > t hold their panel entries (L[a][2t+q], L[a][2t+1-q]) and z[t]
    // the forward-solved value of row 2t+q.
    bool bad = false;
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const double a00 = pr_from0(R[t][t][0]);
        const double a11 = pr_from1(R[t][t][0]);
        const double a10 = pr_from1(R[t][t][1]);
        bad |= !(a00 > 0.0);
        const double i00 = nngp_rsqrt(a00);
        const double l10 = a10 * i00;
        const double s11 = fma(-l10, l10, a11);
        bad |= !(s11 > 0.0);
        const double i11 = nngp_rsqrt(s11);
        const double w0 = pr_from0(z[t]) * i00;
        const double w1 = fma(-l10, w0, pr_from1(z[t])) * i11;
        R[t][t][0] = pr_sel(q1, i11, i00);
        R[t][t][1] = l10;
        z[t] = pr_sel(q1, w1, w0);
        // panel map (L[a][2t], L[a][2t+1]) = (A[a][2t], A[a][2t+1]) U, U = [[i00, u01], [0, i11]],
        // written in own-parity-first coordinates: Y0 = X0 c00 + X1 c10, Y1 = X0 c01 + X1 c11
        const double u01 = -(l10 * i00) * i11;
        const double c00 = pr_sel(q1, i11, i00), c10 = pr_sel(q1, u01, 0.0);
        const double c01 = pr_sel(q1, 0.0, u01), c11 = pr_sel(q1, i00, i11);
        const double wS = pr_sel(q1, w1, w0), wO = pr_sel(q1, w0, w1);
#pragma unroll
        for (int s = t + 1; s < NP; ++s) {
            const double x0 = R[s][t][0], x1 = R[s][t][1];
            const double y0 = fma(x0, c00, x1 * c10);
            const double y1 = fma(x0, c01, x1 * c11);
            R[s][t][0] = y0;
            R[s][t][1] = y1;
            z[s] = fma(-y0, wS, fma(-y1, wO, z[s]));
        }
        // trailing update: same-parity slots read this lane's panel, other-parity slots the swapped one
#pragma unroll
        for (int u = t + 1; u < NP; ++u) {
            const double S0 = R[u][t][0], S1 = R[u][t][1];
            const double P0 = pr_swap(S0), P1 = pr_swap(S1);
#pragma unroll
            for (int s = u; s < NP; ++s) {
                const double y0 = R[s][t][0], y1 = R[s][t][1];
                R[s][u][0] = fma(-y0, S0, fma(-y1, S1, R[s][u][0]));
                R[s][u][1] = fma(-y0, P1, fma(-y1, P0, R[s][u][1]));
            }
        }
    }

    // ---- last pair: (M-1, M) for odd M (one more column), (M, padding) for even M
    double F, res;
    if (M % 2 == 1) {
        const double a00 = pr_from0(R[T][T][0]);
        const double a11 = pr_from1(R[T][T][0]);
        const double a10 = pr_from1(R[T][T][1]);
        bad |= !(a00 > 0.0);
        const double i00 = nngp_rsqrt(a00);
        const double l10 = a10 * i00;
        F = fma(-l10, l10, a11);
        const double w0 = pr_from0(z[T]) * i00;
        res = fma(-l10, w0, pr_from1(z[T]));
        R[T][T][0] = i00;  // lane 0: 1 / L[M-1][M-1]
        R[T][T][1] = l10;  // L[M][M-1]
    } else {
        F = pr_from0(R[T][T][0]);
        res = pr_from0(z[T]);
    }
    bad |= !(F > 0.0);
    if (VAR & 1) F *= sigma2;

    if (Bout != nullptr) {
        // B = L_N^{-T} v, v = row M of L (lane M % 2, local row M / 2).  Lane q ends with
        // bown[s] = B_{2s+q}.
        constexpr int SM = M / 2;
        constexpr bool VQ1 = (M % 2) == 1;  // row M sits in lane 1
        double bown[NP];
#pragma unroll
        for (int s = 0; s < NP; ++s) bown[s] = 0.0;
        if (M % 2 == 1) bown[T] = R[T][T][1] * R[T][T][0];  // lane 0: B_{M-1} = L[M][M-1] / L[M-1][M-1]
#pragma unroll
        for (int t = T - 1; t >= 0; --t) {
            // partial sums over this lane's rows b = 2u + q, 2t + 2 <= b < M
            double acc0 = 0.0, acc1 = 0.0;
#pragma unroll
            for (int u = t + 1; u < NP; ++u) {
                if (2 * u >= M) continue;  // both rows of the pair are past the neighbour rows
                const bool row_ok = 2 * u + 1 < M;  // else only lane 0's row is a neighbour row
                double bu = bown[u];
                if (!row_ok) bu = q1 ? 0.0 : bu;
                acc0 = fma(R[u][t][0], bu, acc0);
                acc1 = fma(R[u][t][1], bu, acc1);
            }
            const double tot = acc0 + pr_swap(acc1);  // sum_b L[b][2t+q] B_b
            // v_{2t+q}: row M's own-parity entry is slot [t][0] in lane M%2, slot [t][1] in the other
            const double vrow0 = R[SM][t][0], vrow1 = R[SM][t][1];
            double v;
            if (VQ1) {
                v = pr_sel(q1, vrow0, pr_swap(vrow1));
            } else {
                v = pr_sel(q1, pr_swap(vrow1), vrow0);
            }
            const double iown = R[t][t][0];
            const double bx = (v - tot) * iown;      // lane 1: B_{2t+1}
            const double b1 = pr_swap(bx);           // lane 0: B_{2t+1}
            const double l10 = R[t][t][1];
            const double b0 = fma(-(l10 * iown), b1, bx);  // lane 0: B_{2t}
            bown[t] = pr_sel(q1, bx, b0);
        }
        if (live) {
#pragma unroll
            for (int s = 0; s < NP; ++s) {
                const int a = 2 * s + q;
                if (a < M) Bout[rr * M + a] = bad ? NAN : (oval[s] ? bown[s] : 0.0);
            }
        }
    }
    const bool lead = live && !q1;
    if (Fout != nullptr && lead) Fout[rr] = bad ? NAN : F;
    if (Rout != nullptr && lead) Rout[rr] = bad ? NAN : res;

    if (VAR & 2) {
        __shared__ double sh[2][4][5];
        pairb_tile_store(lead ? __builtin_amdgcn_frexp_mant(F) : 1.0, lead ? __builtin_amdgcn_frexp_exp(F) : 0,
                         lead ? res * res * pr_rcp(F) : 0.0, (lead && bad) ? (double)i : INFINITY,
                         (live && bad_index) ? (double)i : INFINITY, sh, 0, (double4*)bpart, lexp, blk);
        __syncthreads();
        if (threadIdx.x == 0) pairb_tile_fold(sh, 0, (double4*)bpart, lexp, blk);
        return;
    }
    double lf = 0.0, qq = 0.0, badp = INFINITY, badi = INFINITY;
    if (lead) {
        lf = log(F);
        qq = res * res / F;
        if (bad) badp = (double)i;
    }
    if (live && bad_index) badi = (double)i;
    block_partials_store(lf, qq, badp, badi, bpart, blk);
}

template <int M, int KIND, int VAR>
static void launch_pairb_mk(const BfArgs& a, const CovParams& Pc, hipStream_t s) {
    const int64_t blocks = (a.n_rows * 2 + 255) / 256;
    hipLaunchKernelGGL((bf_pairb<M, KIND, VAR>), dim3((unsigned)blocks), dim3(256), 0, s, (const double2*)a.coords,
                       a.n_points, a.nbr, a.order, a.n_rows, a.i0, Pc, a.values, (const double2*)a.qcoords, a.qvalues,
                       a.B, a.F, a.R, a.bpart, a.sigma2, pairb_lexp(a.bpart, a.n_rows));
}



}  // namespace r1
}  // namespace nngp
