// B/F + log-likelihood sweep with P lanes per location (P = 1, 2, 4).
//
// Same formulation and outputs as bf_lane (bf_sweep.hip documents it and the
// reference methods nngp.py:73-96 it replaces): the (m+1)x(m+1) joint block
// [[C_N + tau2 I, c], [c^T, sigma2 + tau2]] with the value column appended, m
// right-looking elimination steps, B = L_N^{-T} v.
//
// Why P > 1: with one lane per location the whole joint block lives in one
// lane's VGPRs (136 doubles at m = 15), which pins the kernel at one wave per
// SIMD and leaves every latency exposed.  Here the block's rows are dealt
// cyclically over the P lanes of a group (lane q owns rows a = P*s + q), so a
// lane holds ~1/P of it and two or more waves fit per SIMD.  Column values move
// between the lanes of a group with DPP quad_perm broadcasts (the groups are
// aligned inside DPP quads), never through LDS:
//   * build: every lane computes the covariances of its own rows (~1/P of the
//     pairs) against the group-broadcast neighbour coordinates;
//   * step p: the pivot and column p are broadcast from their owner lanes, each
//     lane updates its own rows;
//   * back-substitution: per-lane partial dot products + a group butterfly sum.
// Rows are padded to a multiple of P with far-away (decoupled) slots.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nngp_math.h"
#include "nngp_internal.h"

namespace nngp {

template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const long long u = __double_as_longlong(v);
    // bound_ctrl: every lane reads a valid source lane, so no "old" value (and no init mov) is needed
    const int lo = __builtin_amdgcn_mov_dpp((int)(u & 0xffffffffll), CTRL, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(u >> 32), CTRL, 0xf, 0xf, true);
    return __hiloint2double(hi, lo);
}

// value of v in lane `src` of this lane's P-group (src folds to a constant after unrolling)
template <int P>
__device__ __forceinline__ double grp_bcast(double v, int src) {
    if (P == 1) return v;
    if (P == 2) return src == 0 ? dpp_f64<0xA0>(v) : dpp_f64<0xF5>(v);  // quad_perm [s,s,s+2,s+2]
    switch (src) {                                                      // quad_perm [s,s,s,s]
        case 0:
            return dpp_f64<0x00>(v);
        case 1:
            return dpp_f64<0x55>(v);
        case 2:
            return dpp_f64<0xAA>(v);
        default:
            return dpp_f64<0xFF>(v);
    }
}

// sum of v over the P lanes of the group (same value, same rounding, in every lane)
template <int P>
__device__ __forceinline__ double grp_sum(double v) {
    if (P == 1) return v;
    v = v + dpp_f64<0xB1>(v);  // quad_perm [1,0,3,2]
    if (P == 4) v = v + dpp_f64<0x4E>(v);  // quad_perm [2,3,0,1]
    return v;
}

// D = 2: 2-D ordinates (one 16-byte load per point); D = 0: runtime dimension 1..3 held as three
// coordinates, with KIND = NNGP_KIND_GENERIC the runtime-kind covariance (nngp_math.h) -- the
// m = 25..32 kernels for every kind and dimension.  KIND = NNGP_KIND_BLOCKS: the joint block's
// covariances are read from cblk (nngp_bf_sweep_blocks at m = 25..32; the layout bf_pairb.h's
// blocks kernel reads: entry (a, b), b <= a <= M, of nbr row t at cblk[(a (a+1)/2 + b) n_rows + t]),
// no coordinates are gathered, and slots without a point decouple exactly (0 off the diagonal, 1 on
// it) whatever the caller stored there.
template <int M, int KIND, int P, int D = 2>
__global__ __launch_bounds__(256) void bf_group(const double* __restrict__ coords, int64_t n_points,
                                                const int32_t* __restrict__ nbr, const int32_t* __restrict__ order,
                                                int64_t n_rows, int64_t i0,
                                                const CovParams Pc, const double* __restrict__ values, const double* __restrict__ qcoords, const double* __restrict__ qvalues,
                                                double* __restrict__ Bout, double* __restrict__ Fout, double* __restrict__ Rout,
                                                double* __restrict__ bpart, int dim, const double* __restrict__ cblk) {
    static_assert(D == 0 || D == 2, "bf_group: 2-D or runtime dimension");
    constexpr bool CM = KIND == NNGP_KIND_BLOCKS;
    // KIND == NNGP_KIND_MATERN: rho from the launch's Matern table (cblk, copied to dynamic LDS; nngp_math.h
    // "Matern-nu by table"), sigma2 rho per entry -- the general-smoothness Matern at m = 25..32
    constexpr bool MT = KIND == NNGP_KIND_MATERN;
    extern __shared__ double4 grp_mtab[];
    static_assert(!CM || M <= 32, "the validity mask holds one bit per neighbour slot");
    constexpr int NR = M + 1;               // joint rows 0..M (row M = the location)
    constexpr int S = (NR + P - 1) / P;     // local rows per lane
    constexpr int DA = point_arity<D>();
    const int ds = D == 0 ? dim : 2;
    __shared__ double etab[MT ? 1 : NNGP_EXP_TAB_N];
    if constexpr (MT) {
        const int n4 = Pc.mt_noct * (NNGP_MT_K * NNGP_MT_NC / 4);
        const double4* g = (const double4*)cblk;
        for (int k = (int)threadIdx.x; k < n4; k += blockDim.x) grp_mtab[k] = g[k];
        __syncthreads();
    } else if constexpr (!CM) {
        nngp_exp_table_load(etab, Pc.sigma2);
    }
    // the covariance of one entry at squared distance d2
    auto cov = [&](double d2) -> double {
        if constexpr (MT) return Pc.sigma2 * nngp_matern_tab(Pc, (const double*)grp_mtab, d2);
        else return nngp_cov_d2<KIND>(Pc, etab, d2);
    };
    const int64_t blk = xcd_logical_block(blockIdx.x, gridDim.x);
    const int64_t tid = blk * blockDim.x + threadIdx.x;
    const int q = (int)(threadIdx.x % P);
    const int64_t r = tid / P;
    const bool live = r < n_rows;
    const int64_t rl = live ? r : n_rows - 1;
    const int64_t rr = order != nullptr ? (int64_t)order[rl] : rl;
    const int64_t i = i0 + rr;

    // ---- own rows a = P*s + q: neighbour slot (a < M), the location (a == M), padding (a > M)
    // branch-free loads: neighbour slots first (clamped slot for the self/padding rows),
    // then every gather unconditionally from a resolved address (far-point / zero tables
    // for invalid and padding slots), so the compiler issues them back to back
    int32_t jn[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int a = P * s + q;
        jn[s] = nbr[rl * M + (a < M ? a : M - 1)];
    }
    double o[S][DA], z[S];
    bool oval[S];
    bool bad_index = false;
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int a = P * s + q;
        const int32_t j = a < M ? jn[s] : -1;
        const bool in_range = j >= 0 && (int64_t)j < n_points;
        bad_index |= j != -1 && !in_range;
        oval[s] = in_range;
        const bool self = a == M;
        const double* pc = self ? qcoords + i * ds : (in_range ? coords + (int64_t)j * ds : far_point<DA>(a));
        const double* pv = self ? (qvalues != nullptr ? qvalues + i : kZeroValue)
                                : ((values != nullptr && in_range) ? values + j : kZeroValue);
        if constexpr (CM) {
        } else if constexpr (D == 0) {
            load_point_rt(pc, dim, o[s]);
        } else {
            load_point<D>(pc, o[s]);
        }
        z[s] = *pv;
    }

    // ---- joint block rows: R[s][b], b < min(P*s + P, NR)
    double R[S][NR];
    if constexpr (CM) {
        // vm: bit a set when neighbour slot a < M holds a point (this lane's slots, then the group's
        // by two DPP ORs); row M (the location) always does, padding rows a > M never
        uint32_t vm = 0;
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int a = P * s + q;
            vm |= (a < M && oval[s]) ? (1u << (a & 31)) : 0u;
        }
        if constexpr (P > 1) vm |= (uint32_t)__builtin_amdgcn_mov_dpp((int)vm, 0xB1, 0xf, 0xf, true);
        if constexpr (P > 2) vm |= (uint32_t)__builtin_amdgcn_mov_dpp((int)vm, 0x4E, 0xf, 0xf, true);
        auto has = [&](int a) -> bool { return a == M || (a < M && ((vm >> (a & 31)) & 1u)); };
        const double* cb = cblk + rl;
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int a = P * s + q;
            const bool ha = has(a);
#pragma unroll
            for (int b = 0; b < NR; ++b) {
                if (b >= P * s + P) continue;  // beyond this local row's width
                if (b > a) {                   // (diagonal block, upper part)
                    R[s][b] = 0.0;
                    continue;
                }
                const bool ok = ha && has(b);
                const int64_t e = ok ? (int64_t)((a * (a + 1)) / 2 + b) : 0;  // in range either way
                const double v = cb[e * n_rows];
                R[s][b] = ok ? v : (b == a ? 1.0 : 0.0);
            }
        }
    } else {
        double X[NR][DA];
#pragma unroll
        for (int b = 0; b < NR; ++b)
#pragma unroll
            for (int k = 0; k < DA; ++k) X[b][k] = grp_bcast<P>(o[b / P][k], b % P);
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int a = P * s + q;
#pragma unroll
            for (int b = 0; b < NR; ++b) {
                if (b >= P * s + P) continue;  // beyond this local row's width
                if (b < P * s) {
                    R[s][b] = cov(point_d2<DA>(o[s], X[b]));
                } else if (b < P * s + P - 1) {  // diagonal block: lane-dependent
                    // (the self entry's value is not used: under the Matern table it would take the small-nu
                    // branch's call for its zero distance, once per row group, so it evaluates d2 = 1 instead)
                    const double d2 = point_d2<DA>(o[s], X[b]);
                    const double c = cov(MT && b == a ? 1.0 : d2);
                    R[s][b] = b < a ? c : (b == a ? Pc.diag : 0.0);
                } else {
                    R[s][b] = b == a ? Pc.diag : 0.0;
                }
            }
        }
    }

    // ---- right-looking elimination; the owner of row p keeps 1/L[p][p] in R[p/P][p]
    bool bad = false;
#pragma unroll
    for (int p = 0; p < M; ++p) {
        const int qp = p % P, sp = p / P;
        const double piv = grp_bcast<P>(R[sp][p], qp);
        bad |= !(piv > 0.0);
        const double ip = nngp_rsqrt(piv);
        R[sp][p] = q == qp ? ip : R[sp][p] * ip;
#pragma unroll
        for (int s = sp + 1; s < S; ++s) R[s][p] *= ip;
        z[sp] = q == qp ? z[sp] * ip : z[sp];
        const double zp = grp_bcast<P>(z[sp], qp);
        double lb[NR];
#pragma unroll
        for (int b = p + 1; b < NR; ++b) lb[b] = grp_bcast<P>(R[b / P][p], b % P);
#pragma unroll
        for (int s = sp; s < S; ++s) {
#pragma unroll
            for (int b = p + 1; b < NR; ++b) {
                if (b >= P * s + P) continue;
                R[s][b] = fma(-R[s][p], lb[b], R[s][b]);
            }
            if (s == sp) {
                if (P > 1) z[s] = q > qp ? fma(-R[s][p], zp, z[s]) : z[s];
            } else {
                z[s] = fma(-R[s][p], zp, z[s]);
            }
        }
    }
    const double F = grp_bcast<P>(R[M / P][M], M % P);
    const double res = grp_bcast<P>(z[M / P], M % P);
    bad |= !(F > 0.0);

    if (Bout != nullptr) {
        // B = L_N^{-T} v, v = row M of L; lane q ends with bown[s] = b_{P*s+q}
        double bown[S];
#pragma unroll
        for (int s = 0; s < S; ++s) bown[s] = 0.0;
#pragma unroll
        for (int a = M - 1; a >= 0; --a) {
            double part = 0.0;
#pragma unroll
            for (int s = 0; s < S; ++s) {
                if (P * s + P - 1 <= a) continue;  // every row of this local row is <= a
                const int ar = P * s + q;
                const double t = R[s][a] * bown[s];
                part = (ar > a && ar < M) ? part + t : part;
            }
            const double tot = grp_sum<P>(part);
            const double va = grp_bcast<P>(R[M / P][a], M % P);
            const double iva = grp_bcast<P>(R[a / P][a], a % P);
            const double ba = (va - tot) * iva;
            bown[a / P] = q == a % P ? ba : bown[a / P];
        }
        if (live) {
#pragma unroll
            for (int s = 0; s < S; ++s) {
                const int a = P * s + q;
                if (a < M) Bout[rr * M + a] = bad ? NAN : (oval[s] ? bown[s] : 0.0);
            }
        }
    }
    const bool lead = live && q == 0;
    if (Fout != nullptr && lead) Fout[rr] = bad ? NAN : F;
    if (Rout != nullptr && lead) Rout[rr] = bad ? NAN : res;

    double lf = 0.0, qq = 0.0, badp = INFINITY, badi = INFINITY;
    if (lead) {
        lf = log(F);
        qq = res * res / F;
        if (bad) badp = (double)i;
    }
    if (live && bad_index) badi = (double)i;
    block_partials_store(lf, qq, badp, badi, bpart, blk);
}

template <int M, int KIND, int P, int D = 2>
static void launch_group_mkp(const BfArgs& a, const CovParams& Pc, hipStream_t s) {
    const int64_t blocks = (a.n_rows * P + 255) / 256;
    const size_t lds = KIND == NNGP_KIND_MATERN ? NNGP_MT_BYTES(Pc.mt_noct) : 0;
    hipLaunchKernelGGL((bf_group<M, KIND, P, D>), dim3((unsigned)blocks), dim3(256), lds, s, a.coords, a.n_points, a.nbr,
                       a.order, a.n_rows, a.i0, Pc, a.values, a.qcoords, a.qvalues, a.B, a.F, a.R, a.bpart, a.dim,
                       a.cblk);
}

// one (M, P): the 2-D exponential / Matern-3/2 kernels, and one runtime-kind, runtime-dimension
// kernel for the other kinds and dimensions; returns false for other m
template <int M, int P>
static bool launch_group_if(const BfArgs& a, const CovParams& Pc, hipStream_t s) {
    if (a.m != M) return false;
    if (a.dim == 2 && a.kind == 1)
        launch_group_mkp<M, 1, P>(a, Pc, s);
    else if (a.dim == 2 && a.kind == 0)
        launch_group_mkp<M, 0, P>(a, Pc, s);
    else
        launch_group_mkp<M, NNGP_KIND_GENERIC, P, 0>(a, Pc, s);
    return true;
}

// general-smoothness Matern from the launch's table (a.cblk, bf_launch) at m = 25..32 (bf_quad_matern_*.hip:
// units of their own, these fully unrolled kernels compile for minutes each)
template <int M>
static bool launch_group_matern_if(const BfArgs& a, const CovParams& Pc, hipStream_t s) {
    if (a.m != M) return false;
    launch_group_mkp<M, NNGP_KIND_MATERN, 4, 0>(a, Pc, s);
    return true;
}

// covariance blocks from memory at m = 25..32 (nngp_bf_sweep_blocks; bf_quad_blocks.hip)
template <int M>
static bool launch_group_blocks_if(const BfArgs& a, hipStream_t s) {
    if (a.m != M) return false;
    launch_group_mkp<M, NNGP_KIND_BLOCKS, 4>(a, nngp_cov_params(0, 1.0, 1.0, 0.0), s);
    return true;
}

}  // namespace nngp
