// NNGP B/F + log-likelihood sweep on gfx950 (CDNA4).
//
// Reference path (bwpriest/pyNNGP, /root/reference; stubs there):
//   _CNs(i)    nngp.py:78-82  C_{N(s_i)}            -> rows/cols 0..m-1 of the joint block
//   _Ccross(i) nngp.py:84-86  C_{s_i,N(s_i)}        -> row m of the joint block
//   _Cs(i)     nngp.py:92-96  C_{s_i,s_i}           -> entry (m, m)
//   _Bsi(i)    nngp.py:73-76  B_i = c^T C_N^{-1}    -> back-substitution on L_N
//   _Fsi(i)    nngp.py:88-90  F_i = C_ii - c^T C_N^{-1} c -> last pivot of the joint block
// plus the log-likelihood sweep the reference never wrote.
//
// Formulation: factor the (m+1)x(m+1) joint block
//   J = [[C_N + tau2 I, c], [c^T, sigma2 + tau2]]   with the value column [v_N; v_i]
// appended.  After m right-looking elimination steps the last row of L holds
// v = L_N^{-1} c, the last pivot is F_i and the last entry of the value column
// is r_i = v_i - B_i v_N(i).  B_i = L_N^{-T} v needs one more back-solve.
// Neighbour slots with index -1 become identity rows (decoupled, exact).
//
// Two kernels, same math, same outputs (bf_wave lives in bf_wave.hip):
//   bf_lane<M>   one LANE per location, the whole joint block in VGPRs, fully
//                unrolled for a compile-time M <= 16.  64 locations per wave;
//                every lane does useful fp64 work on every instruction.
//   bf_wave<NR>  one WAVE per location (the north_star layout): lane a owns row a
//                of the joint block in VGPRs; column values are broadcast with
//                v_readlane.  Any M <= 63.  Generic path / comparison point.
// Every kernel writes one record per 256-thread block (sum log F, sum r^2/F,
// first bad-pivot row, first bad-index row) into a workspace slab; bf_finalize
// folds the slab in a fixed order (bit-reproducible, no pre-initialised state).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nngp_math.h"
#include "nngp_internal.h"
#include "bf_pairb.h"

namespace nngp {


// --------------------------------------------------------------------------
// one lane per location
// --------------------------------------------------------------------------
template <int M, int KIND>
__global__ __launch_bounds__(256) void bf_lane(const double2* __restrict__ coords, int64_t n_points,
                                               const int32_t* __restrict__ nbr, const int32_t* __restrict__ order,
                                               int64_t n_rows, int64_t i0,
                                               const CovParams P, const double* __restrict__ values, const double2* __restrict__ qcoords, const double* __restrict__ qvalues,
                                               double* __restrict__ Bout, double* __restrict__ Fout, double* __restrict__ Rout,
                                               double* __restrict__ bpart) {
    constexpr int N1 = M + 1;  // joint block order
    __shared__ double etab[NNGP_EXP_TAB_N];
    nngp_exp_table_load(etab, P.sigma2);
    const int64_t blk = xcd_logical_block(blockIdx.x, gridDim.x);
    const int64_t r = blk * blockDim.x + threadIdx.x;
    const bool live = r < n_rows;
    const int64_t rl = live ? r : n_rows - 1;
    const int64_t rr = order != nullptr ? (int64_t)order[rl] : rl;
    const int64_t i = i0 + rr;

    // branch-free loads: neighbour rows first, then every gather unconditionally
    // (invalid slots read a far point / a zero value from tables in global memory)
    bool valid[M];
    int32_t jn[M];
    bool bad_index = false;
#pragma unroll
    for (int a = 0; a < M; ++a) jn[a] = nbr[rl * M + a];
    double px[N1], py[N1], z[N1];
#pragma unroll
    for (int a = 0; a < M; ++a) {
        const int32_t j = jn[a];
        const bool v = j >= 0 && (int64_t)j < n_points;
        bad_index |= j != -1 && !v;
        valid[a] = v;
        const double2 x = *(v ? coords + j : kFarPoints + a);
        px[a] = x.x;
        py[a] = x.y;
        z[a] = *((values != nullptr && v) ? values + j : kZeroValue);
    }
    {
        const double2 x = qcoords[i];
        px[M] = x.x;
        py[M] = x.y;
        z[M] = *(qvalues != nullptr ? qvalues + i : kZeroValue);
    }

    // joint block, lower triangle (A[a][b], b <= a)
    double A[N1][N1];
#pragma unroll
    for (int a = 0; a < N1; ++a) {
#pragma unroll
        for (int b = 0; b < a; ++b) A[a][b] = nngp_cov_d2<KIND>(P, etab, nngp_d2(px[a], py[a], px[b], py[b]));
        A[a][a] = P.diag;
    }

    // right-looking elimination of the M neighbour columns (value column z appended)
    double inv[M];
    bool bad = false;
#pragma unroll
    for (int p = 0; p < M; ++p) {
        bad |= !(A[p][p] > 0.0);
        const double ip = nngp_rsqrt(A[p][p]);
        inv[p] = ip;
#pragma unroll
        for (int a = p + 1; a < N1; ++a) A[a][p] *= ip;
        z[p] *= ip;
#pragma unroll
        for (int a = p + 1; a < N1; ++a) {
#pragma unroll
            for (int b = p + 1; b <= a; ++b) A[a][b] = fma(-A[a][p], A[b][p], A[a][b]);
            z[a] = fma(-A[a][p], z[p], z[a]);
        }
    }
    const double F = A[M][M];
    const double res = z[M];
    bad |= !(F > 0.0);

    if (Bout != nullptr) {
        // B = L_N^{-T} v, v = row M of L
        double bb[M];
#pragma unroll
        for (int a = M - 1; a >= 0; --a) {
            double s = A[M][a];
#pragma unroll
            for (int q = a + 1; q < M; ++q) s = fma(-A[q][a], bb[q], s);
            bb[a] = s * inv[a];
        }
        if (live) {
#pragma unroll
            for (int a = 0; a < M; ++a) Bout[rr * M + a] = bad ? NAN : (valid[a] ? bb[a] : 0.0);
        }
    }
    if (Fout != nullptr && live) Fout[rr] = bad ? NAN : F;
    if (Rout != nullptr && live) Rout[rr] = bad ? NAN : res;

    double lf = 0.0, q = 0.0, badp = INFINITY, badi = INFINITY;
    if (live) {
        lf = log(F);
        q = res * res / F;
        if (bad) badp = (double)i;
        if (bad_index) badi = (double)i;
    }
    block_partials_store(lf, q, badp, badi, bpart, blk);
}

// --------------------------------------------------------------------------
// fixed-order reduction of the per-block partial records -> partials[4]
// --------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void bf_finalize(const double* __restrict__ bpart, int64_t n_blocks,
                                                    double* __restrict__ partials) {
    // Fixed order: thread t folds records t, t + 1024, t + 2048, ... (each wave reads
    // contiguous 2 KB per round; up to 8 rounds in flight before the first use), then
    // a fixed xor-butterfly inside each wave and a fixed fold over the 16 waves.
    __shared__ double sh[16][4];
    const int t = threadIdx.x;
    const double4* rec = (const double4*)bpart;
    double a = 0.0, b = 0.0, c = INFINITY, d = INFINITY;
    for (int64_t k0 = t; k0 < n_blocks; k0 += 8 * 1024) {
        double4 r[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t k = k0 + (int64_t)u * 1024;
            r[u] = k < n_blocks ? rec[k] : make_double4(0.0, 0.0, INFINITY, INFINITY);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            a += r[u].x;
            b += r[u].y;
            c = fmin(c, r[u].z);
            d = fmin(d, r[u].w);
        }
    }
    a = wave_sum(a);
    b = wave_sum(b);
    c = wave_min(c);
    d = wave_min(d);
    if ((t & 63) == 0) {
        sh[t >> 6][0] = a;
        sh[t >> 6][1] = b;
        sh[t >> 6][2] = c;
        sh[t >> 6][3] = d;
    }
    __syncthreads();
    if (t == 0) {
        a = 0.0, b = 0.0, c = INFINITY, d = INFINITY;
        for (int w = 0; w < 16; ++w) {
            a += sh[w][0];
            b += sh[w][1];
            c = fmin(c, sh[w][2]);
            d = fmin(d, sh[w][3]);
        }
        partials[0] = a;
        partials[1] = b;
        partials[2] = c == INFINITY ? -1.0 : c;
        partials[3] = d == INFINITY ? -1.0 : d;
    }
}

// the separate fold of bf_pairb's tile records (pairb_fold_records, bf_pairb.h): one block of kPairbThreads
// threads, a fixed order
// The tile count comes from the workspace header the sweep wrote; a count outside [0, bound] means the
// workspace does not hold a pair-kernel sweep of n_rows rows (e.g. a deferred Matern sweep that ran on the
// wavefront kernel, finalised as PAIRB): the fold then reads nothing and the partials are NaN (advice r04).
__global__ __launch_bounds__(kPairbThreads) void bf_finalize_pairb(const double4* __restrict__ rec,
                                                                   const int32_t* __restrict__ lexp,
                                                                   const int64_t* __restrict__ hdr, int64_t bound,
                                                                   double* __restrict__ partials) {
    __shared__ double sh[kPairbWaves][5];
    const int64_t n = hdr[0];
    if (n < 0 || n > bound) {
        if (threadIdx.x == 0) {
            partials[0] = partials[1] = NAN;
            partials[2] = partials[3] = -1.0;
        }
        return;
    }
    pairb_fold_records(rec, lexp, n, partials, sh);
}

hipError_t bf_finalize_pairb_launch(void* ws, int64_t n_rows, double* partials, hipStream_t s) {
    hipLaunchKernelGGL(bf_finalize_pairb, dim3(1), dim3(kPairbThreads), 0, s, (const double4*)pairb_rec(ws),
                       pairb_lexp(ws, n_rows), (const int64_t*)pairb_hdr(ws), pairb_tiles_bound(n_rows), partials);
    return hipGetLastError();
}

// Rank-order combination of all-gathered partials: sums for [0], [1], smallest non-negative (else -1)
// for the bad-row flags [2], [3].  g is (world, n_slots, 4) rank-major (an all-gather of each rank's
// (n_slots, 4) block: a batch of independent sweeps in one collective); one thread per slot.
__global__ __launch_bounds__(64) void combine_partials_kernel(const double* __restrict__ g, int world,
                                                              int64_t n_slots, double* __restrict__ out) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_slots) return;
    double a = 0.0, b = 0.0, c = INFINITY, d = INFINITY;
    for (int r = 0; r < world; ++r) {
        const double* p = g + 4 * ((int64_t)r * n_slots + k);
        a += p[0];
        b += p[1];
        if (p[2] >= 0.0) c = fmin(c, p[2]);
        if (p[3] >= 0.0) d = fmin(d, p[3]);
    }
    out[4 * k] = a;
    out[4 * k + 1] = b;
    out[4 * k + 2] = c == INFINITY ? -1.0 : c;
    out[4 * k + 3] = d == INFINITY ? -1.0 : d;
}

hipError_t combine_partials_launch(const double* gathered, int world, int64_t n_slots, double* out, hipStream_t s) {
    if (n_slots == 0) return hipSuccess;
    hipLaunchKernelGGL(combine_partials_kernel, dim3((unsigned)((n_slots + 63) / 64)), dim3(64), 0, s, gathered, world,
                       n_slots, out);
    return hipGetLastError();
}

// --------------------------------------------------------------------------
// launch
// --------------------------------------------------------------------------
template <int M, int KIND>
static void launch_lane(const BfArgs& a, const CovParams& P, hipStream_t s) {
    const int64_t blocks = (a.n_rows + 255) / 256;
    hipLaunchKernelGGL((bf_lane<M, KIND>), dim3((unsigned)blocks), dim3(256), 0, s, (const double2*)a.coords,
                       a.n_points, a.nbr, a.order, a.n_rows, a.i0, P, a.values, (const double2*)a.qcoords, a.qvalues, a.B, a.F, a.R, a.bpart);
}

int64_t bf_lane_blocks(int64_t n_rows) { return (n_rows + 255) / 256; }

template <int KIND>
static bool launch_lane_m(const BfArgs& a, const CovParams& P, hipStream_t s) {
    switch (a.m) {
#define NNGP_LANE_CASE(MM)              \
    case MM:                            \
        launch_lane<MM, KIND>(a, P, s); \
        return true;
        NNGP_LANE_CASE(1) NNGP_LANE_CASE(2) NNGP_LANE_CASE(3) NNGP_LANE_CASE(4) NNGP_LANE_CASE(5)
        NNGP_LANE_CASE(6) NNGP_LANE_CASE(7) NNGP_LANE_CASE(8) NNGP_LANE_CASE(9) NNGP_LANE_CASE(10)
        NNGP_LANE_CASE(11) NNGP_LANE_CASE(12) NNGP_LANE_CASE(13) NNGP_LANE_CASE(14) NNGP_LANE_CASE(15)
        NNGP_LANE_CASE(16)
#undef NNGP_LANE_CASE
        default:
            return false;
    }
}

int64_t bf_record_count(int64_t n_rows, int algo, int m) {
    if (n_rows == 0) return 0;
    if (algo == kAlgoLane) return bf_lane_blocks(n_rows);
    if (algo == kAlgoPairB) return pairb_tiles_bound(n_rows);
    if (algo == kAlgoQuad) return bf_group_blocks(n_rows, 4);
    return bf_wave_blocks(n_rows);
}

hipError_t bf_finalize_launch(const double* bpart, int64_t n_records, double* partials, hipStream_t s) {
    hipLaunchKernelGGL(bf_finalize, dim3(1), dim3(1024), 0, s, bpart, n_records, partials);
    return hipGetLastError();
}

// a.partials == nullptr: leave the per-block records in a.bpart (bf_finalize_launch later)
hipError_t bf_launch(const BfArgs& a, int algo, hipStream_t s) {
    if (a.n_rows == 0)  // empty shard: partials = [0, 0, -1, -1]
        return a.partials != nullptr ? bf_finalize_launch(a.bpart, 0, a.partials, s) : hipSuccess;
    const CovParams P = nngp_cov_params_nu(a.kind, a.sigma2, a.phi, a.tau2, a.nu);
    bool ok;
    int64_t nb;
    if (algo == kAlgoLane) {
        ok = a.dim == 2 && (a.kind == 1 ? launch_lane_m<1>(a, P, s) : a.kind == 0 && launch_lane_m<0>(a, P, s));
        nb = bf_lane_blocks(a.n_rows);
    } else if (algo == kAlgoPairB) {
        // unit-variance factorisation (nngp_cov_unit), F scaled by sigma2 in the kernel
        CovParams Pu = nngp_cov_params_unit(a.kind, a.phi, a.tau2 / a.sigma2);
        BfArgs b = a;
        if (a.kind == NNGP_KIND_MATERN) {
            // the launch's Matern table (a function of nu only: t = phi^2 d^2) after the tile records
            nngp_matern_setup(Pu, a.nu);
            Pu.mphi2 = a.phi * a.phi;
            if (!matern_table_params(a.nu, &Pu)) return hipErrorInvalidValue;
            double* tab = (double*)((char*)a.bpart + bf_pairb_workspace_bytes(a.n_rows));
            hipError_t e = matern_table_launch(Pu, tab, s);
            if (e != hipSuccess) return e;
            b.cblk = tab;
        }
        ok = bf_pairb_launch(b, Pu, s);
        if (!ok) return hipErrorInvalidValue;
        hipError_t e = hipGetLastError();
        if (e != hipSuccess || a.partials == nullptr) return e;
        return bf_finalize_pairb_launch(a.bpart, a.n_rows, a.partials, s);
    } else if (algo == kAlgoQuad) {
        nb = bf_group_blocks(a.n_rows, 4);
        if (a.kind == NNGP_KIND_MATERN) {
            // the launch's Matern table after the block records (as the pair kernel's after its tile records)
            CovParams Pm = P;
            Pm.mphi2 = a.phi * a.phi;
            if (!matern_table_params(a.nu, &Pm)) return hipErrorInvalidValue;
            double* tab = (double*)((char*)a.bpart + ((size_t)nb * 4 * sizeof(double) + 255) / 256 * 256);
            hipError_t e = matern_table_launch(Pm, tab, s);
            if (e != hipSuccess) return e;
            BfArgs b = a;
            b.cblk = tab;
            ok = bf_group_launch(b, Pm, 4, s);
        } else {
            ok = bf_group_launch(a, P, 4, s);
        }
    } else {
        nb = bf_wave_blocks(a.n_rows);
        ok = bf_wave_launch(a, P, nb, s);
    }
    if (!ok) return hipErrorInvalidValue;
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || a.partials == nullptr) return e;
    return bf_finalize_launch(a.bpart, nb, a.partials, s);
}

// a planned sweep (pair_plan.h): the plan's regions through the planned kernel, the direct ones through
// the unplanned kernel (same tiling, same records), then the fold
hipError_t bf_launch_planned(const BfArgs& a, const PlanLaunch& pl, hipStream_t s) {
    if (a.n_rows == 0)
        return a.partials != nullptr ? bf_finalize_launch(a.bpart, 0, a.partials, s) : hipSuccess;
    const CovParams Pu = nngp_cov_params_unit(a.kind, a.phi, a.tau2 / a.sigma2);
    if (pl.n_planned > 0 && !bf_pairb_planned_launch(a, Pu, pl, s)) return hipErrorInvalidValue;
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (pl.n_direct > 0) {
        BfArgs b = a;
        b.tiles = pl.direct;
        b.n_tiles = pl.n_regions;
        b.n_tile_list = pl.n_direct;
        if (!bf_pairb_launch(b, Pu, s)) return hipErrorInvalidValue;
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (a.partials == nullptr) return hipSuccess;
    return bf_finalize_pairb_launch(a.bpart, a.n_rows, a.partials, s);
}

}  // namespace nngp
