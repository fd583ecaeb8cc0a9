// B/F + log-likelihood sweep, two lanes per location, 2x2-blocked elimination
// ("pairb").  Same formulation and outputs as bf_lane / bf_group (bf_sweep.hip
// documents it and the reference methods nngp.py:73-96 it replaces): the
// (m+1)x(m+1) joint block [[C_N + tau2 I, c], [c^T, sigma2 + tau2]] with the value
// column appended, m elimination steps, B = L_N^{-T} v.
//
// Layout.  The joint rows come in pairs (2t, 2t+1); lane q of a location's lane pair
// owns rows a = 2s + q ("local row s").  Row a stores its lower-triangle entries pair
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
//
// Round 2 (profiles/r02b: the kernel keeps the VALU pipe busy, so only fewer
// instructions per location make it faster):
//   * unit-variance covariances (nngp_cov_unit: the exponent of 2^n is added to the
//     table entry's exponent field, one integer op instead of ashr + ldexp), F scaled
//     by sigma2 at the end (B and the residual are scale-invariant);
//   * one partial record per 128-location tile: sum log F leaves the kernel as the
//     tile's mantissa product and exponent sum (frexp), and the ~100-instruction log is
//     taken once per record by the fold (bf_finalize_pairb), not per lane;
//     r^2 / F through v_rcp_f64 + a refinement (pr_rcp) instead of the IEEE divide.
//   Second pass: no value column (r = v_i - B v_N), within-pair covariances split across the
//   pair, exact-zero far points, scalar-pivot LDL^T (reciprocal pivots, unit factor); see
//   DESIGN.md 4.1 for each step's measured effect and the variants rejected.
//   One block per tile, hardware-scheduled: persistent grids (static ranges, ranges with
//   issue-priority balancing, tiles claimed from per-XCD counters) all measured slower
//   (profiles/r02j, r02l, r02m).
// D = coordinate dimension (1..3), KIND = covariance kind (nngp_math.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "bf_group.h"
#include "nngp_internal.h"
#include "nngp_math.h"
#include "pair_plan.h"

namespace nngp {

// Design constants (each measured; the rejected alternatives -- partner exchanges through ds_swizzle, the
// Matern table read from global memory, values parked in LDS, left-looking at three waves per SIMD, balanced
// tilings, the fused record fold -- are described in DESIGN.md 4.1 / 4.2a / 5 and live as patches under
// tools/variants/ for tools/build_variant.sh, not as switches here).
//
// The within-pair covariance split (below) up to m = kPairbDedupMax: it keeps the partner coordinates live
// longer (+20 VGPRs at m = 15), which costs spills past m = 17.
constexpr int kPairbDedupMax = 17;
// (A 2x2-block LDL^T -- one reciprocal of det D_t per block step instead of two pivot square roots, -4.3 %
// VALU -- was measured and rejected: L = X D_t^{-1} multiplies by entries ~1/delta for a nearly singular pair
// block where the Cholesky factor's are ~1/sqrt(delta), and F lost accuracy: 2e-9 relative vs the oracle at
// Matern-3/2, tau2 = 0, m = 8, beyond the 1e-10 bound.)
// Scalar-pivot LDL^T in the 2x2-blocked layout (reciprocals, unit factor) instead of the Cholesky factor
// (inverse square roots) for the right-looking kernels: -44 VALU per wave at m = 15 (-1.7 %), -0.6 % time
// (same-box A/B), every GPU parity test unchanged.  (Until round 6 the right-looking Matern-nu / blocks kernels
// at m = 18 kept the Cholesky form: the two-wave register budget was tight there, 80 -> 216 B of scratch;
// every kind is left-looking at m = 18 now.)
// Left-looking elimination (m in [kPairbLeftMin, 32], the fused kinds): column pair by column pair, each
// column's covariances evaluated when it is reached and updated from the finished columns, so the trailing
// block and every coordinate are never live at once; the finished factor rows 0..KL-1 wait in LDS for the
// back-substitution.  The register peak is the factor's later rows instead of the whole joint block plus
// coordinates: m = 18..22 run at two waves per SIMD (m = 18: 0.273 vs 0.413 ms per 1e6 rows right-looking
// with 224 B of scratch, profiles/r05z5; m = 16 / 17 tie and stay right-looking) (right-looking: one; 0.352 /
// 0.392 / 0.566 vs 0.457 / 0.544 / 0.639 ms per 1e6 rows at m = 19 / 20 / 22, profiles/r03e; m = 21 0.416 vs
// 0.552, profiles/r05z2); from m = kPairbLeftOneWaveMin the left-looking kernel runs at one wave with more
// rows in LDS (its peak no longer fits 256 registers): m = 23 / 24 0.604 / 0.696 vs 0.659 / 0.732
// right-looking (profiles/r05z2).
constexpr int kPairbLeftMin = 18;
constexpr int kPairbLeftOneWaveMin = 23;
constexpr int kPairbLeftLdsRows = 5;    // factor rows in LDS at two waves per SIMD (123 KB of 160 per CU)
constexpr int kPairbLeftLdsRows1W = 7;  // ... and at one wave per SIMD (with the late state in LDS)
// The general-nu Matern kind (its covariances from the launch's LDS table) is left-looking at m = 18 only, at
// one wave per SIMD with 6 factor rows beside its <= 35 KB table: 0.694 vs 0.849 ms per 10^6 rows right-looking
// (two waves, 736 B of scratch); from m = 19 its table evaluation's registers spill in the left-looking form
// (224 - 1,344 B per lane at m = 20..24) and the right-looking one-wave kernel is faster: m = 19 0.699 vs 0.688,
// m = 20 0.890 vs 0.780, m = 24 2.56 vs 1.31 (profiles/r06n, nu = 1.3).  (At two waves per SIMD the
// left-looking Matern kernel spilled 1-2 KB per lane.)  The covariance-blocks kind is left-looking at m = 18..24:
// column pair u's entries are read from the caller's block array when the column is reached -- 0.50 / 0.53 /
// 0.54 / 1.28 / 1.56 / 2.41 / 2.71 ms per 10^6 rows at m = 18..24 against 1.19 / 1.76 / 2.04 / 2.07 / 2.44 / 2.48 /
// 2.83 right-looking (profiles/r06p; m = 18..20 at two waves without spills); the four-lane kernel keeps 25..32.
constexpr int kPairbLeftMaternM = 18;
constexpr int kPairbLeftLdsRowsMT = 6;
constexpr bool pairb_left(int m) { return m >= kPairbLeftMin && m <= 32; }
// the same for a kernel of covariance kind `kind` (the Matern-table kernels left-looking at m =
// kPairbLeftMaternM only, the covariance-blocks ones up to m = 24: the four-lane kernel serves them above)
constexpr bool pairb_lk(int m, int kind) {
    return pairb_left(m) && (kind != NNGP_KIND_MATERN || m == kPairbLeftMaternM) &&
           (kind != NNGP_KIND_BLOCKS || m <= 24);
}
// static per-phase budgets (tools/isa_phases.py): tools/variants/phases.h defines NNGP_PHASE to fence the
// phases with named markers (hipcc -include tools/variants/phases.h); a product build leaves them empty
#ifndef NNGP_PHASE
#define NNGP_PHASE(name)
#endif
__device__ __forceinline__ double pr_swap(double v) { return dpp_f64<0xB1>(v); }   // partner lane's v
__device__ __forceinline__ double pr_from0(double v) { return dpp_f64<0xA0>(v); }  // lane 0's v
__device__ __forceinline__ double pr_from1(double v) { return dpp_f64<0xF5>(v); }  // lane 1's v
__device__ __forceinline__ double pr_sel(bool q1, double v1, double v0) { return q1 ? v1 : v0; }
// the same select as a bit-field insert under an opaque lane mask: a plain select of two entries
// of one register array becomes an array access at a lane-dependent index, which LLVM lowers
// to a compare / select chain over the whole array
__device__ __forceinline__ double pr_pick(uint32_t mask1, double v1, double v0) {
    const long long a = __double_as_longlong(v1), b = __double_as_longlong(v0);
    const uint32_t lo = ((uint32_t)a & mask1) | ((uint32_t)b & ~mask1);
    const uint32_t hi = ((uint32_t)(a >> 32) & mask1) | ((uint32_t)(b >> 32) & ~mask1);
    return __hiloint2double((int)hi, (int)lo);
}

// Occupancy: up to m = kPairbTwoWavesMax the compiler is asked for two waves per SIMD (<= 256 VGPRs):
// m = 16 / 17 fit without spills; m = 18 (the right-looking blocks kind, round 5) spilled 20 dwords and
// still runs ~30 % faster than at one wave per SIMD (0.314 vs 0.435 ms per 10^6 rows, profiles/r02ap).  From
// m = 20 (342 VGPRs) the right-looking kernels' forced spills (91 dwords) cost more than the second wave gains
// (+52 % at m = 20, 2-3x at m = 22 / 24).  Three waves per SIMD (<= 168 VGPRs) up to m = kPairbThreeWavesMax:
// m = 12 / 13 fit in 162 / 164 VGPRs (-3.7 % cycles at m = 13); forced at m = 14 / 15 the 31 / 35 spilled
// dwords cost more (+10 % / +37 %, profiles/r02y).
constexpr int kPairbTwoWavesMax = 18;
constexpr int kPairbThreeWavesMax = 13;
// waves per SIMD the kernel for (m, kind) is built for: blocks per CU
constexpr int pairb_waves_per_simd(int m, int kind) {
    return m <= kPairbThreeWavesMax ? 3
           : (pairb_lk(m, kind) && kind == NNGP_KIND_MATERN) ? 1
           : (m <= kPairbTwoWavesMax || (pairb_lk(m, kind) && m < kPairbLeftOneWaveMin)) ? 2
                                                                                          : 1;
}
#define NNGP_PAIRB_ATTR \
    __attribute__((amdgpu_waves_per_eu(pairb_waves_per_simd(M, KIND), M <= kPairbThreeWavesMax ? 3 : 2)))

// Threads per block (one tile of up to kPairbThreads / 2 locations per block).  256 measured fastest:
// 128 / 64 threads (table fill per block, 2x / 4x the tile records) took +0.9 % / +2.6 % at
// config 3 and +5 % / +1 % at config 2 (same-box A/B).
constexpr int kPairbThreads = 256;
constexpr int kPairbWaves = kPairbThreads / 64;
constexpr int kPairbTile = kPairbThreads / 2;  // locations per tile (at most)
constexpr int kDeviceCUs = 256;                 // MI355X (gfx950): 8 XCDs x 32 CUs

// Tiling of n_rows locations: ceil(n / 128) tiles of q or q + 1 rows (the sweep writes the tile count into
// the workspace header, where the record fold reads it).  (Tiles balanced to whole rounds of the device's
// block slots were measured and not kept, round 4, profiles/r04d: +4 % at config 3, no gain at config 2.)
struct PairbTiling {
    int64_t tiles, q, rem;  // tiles; tile t holds q + (t < rem) rows starting at t q + min(t, rem)
};
inline PairbTiling pairb_tiling(int64_t n_rows, int m, int kind) {
    (void)m;
    (void)kind;
    const int64_t T = (n_rows + kPairbTile - 1) / kPairbTile;
    if (T == 0) return {0, 0, 0};
    return {T, n_rows / T, n_rows % T};
}
// record slots a sweep of n_rows may use (workspace sizing; kept at the ABI-2 bound, which also covered the
// balanced tilings, so workspace sizes do not change)
inline int64_t pairb_tiles_bound(int64_t n_rows) {
    const int64_t T = (n_rows + kPairbTile - 1) / kPairbTile;
    const int64_t b = T + 3 * kDeviceCUs - 1 < n_rows / 97 ? T + 3 * kDeviceCUs - 1 : n_rows / 97;
    return b > T ? b : T;
}

// Tile record fold: wave butterflies (fixed order), then the 4 waves in order by thread 0.
// lm: product of the lanes' F mantissas (each in [0.5, 1); 128 of them stay above 2^-128),
// renormalised once; le: their exponent sum.  rec[tile] = (mantissa, sum r^2/F, first
// bad-pivot row, first bad-index row), lexp[tile] = exponent sum.  sh[par] lets a
// multi-tile caller double-buffer the exchange (one barrier per tile).
__device__ __forceinline__ void pairb_tile_store(double lm, int le, double qq, double badp, double badi,
                                                 double (*sh)[kPairbWaves][5], int par, double4* __restrict__ rec,
                                                 int32_t* __restrict__ lexp, int64_t tile) {
#pragma unroll
    for (int o = 32; o > 1; o >>= 1) {  // the terms sit in the even (lead) lanes: lane 0 needs no xor-1 step
        lm *= __shfl_xor(lm, o);
        le += __shfl_xor(le, o);
        qq += __shfl_xor(qq, o);
    }
    if (__any(badp != INFINITY || badi != INFINITY)) {  // wave-uniform; rare
        badp = wave_min(badp);
        badi = wave_min(badi);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sh[par][w][0] = lm;
        sh[par][w][1] = (double)le;
        sh[par][w][2] = qq;
        sh[par][w][3] = badp;
        sh[par][w][4] = badi;
    }
}

__device__ __forceinline__ void pairb_tile_fold(double (*sh)[kPairbWaves][5], int par, double4* __restrict__ rec,
                                                int32_t* __restrict__ lexp, int64_t tile) {
    double lm = 1.0, le = 0.0, qq = 0.0, bp = INFINITY, bi = INFINITY;
#pragma unroll
    for (int k = 0; k < kPairbWaves; ++k) {
        lm *= sh[par][k][0];
        le += sh[par][k][1];
        qq += sh[par][k][2];
        bp = fmin(bp, sh[par][k][3]);
        bi = fmin(bi, sh[par][k][4]);
    }
    rec[tile] = make_double4(__builtin_amdgcn_frexp_mant(lm), qq, bp, bi);
    lexp[tile] = (int32_t)le + __builtin_amdgcn_frexp_exp(lm);
}

// ---- the fixed-order fold of the tile records (the finalize kernel, kPairbThreads threads).
// rec[t] = (mantissa product m_t in [1/2, 1), sum r^2/F, bad-pivot row, bad-index row), lexp[t] =
// exponent sum e_t.  sum log F = log(prod_t m_t) + (sum_t e_t) ln 2: the mantissas are multiplied
// (renormalised by frexp after every product, exponents summed exactly as integers) and ONE log is
// taken at the end -- a log per record made the single-block fold 10 us at 7,813 records.
// Row reduction (16 lanes) by four DPP steps -- quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror,
// row_mirror -- after which every lane of a row holds the row's result (each step combines a lane
// with one partner, a op b == b op a, so all 16 lanes agree bit for bit); the four row results are
// then read from lanes 0, 16, 32, 48 and combined in that order.
template <int OP>  // 0: sum, 1: product, 2: min
__device__ __forceinline__ double fold_op(double a, double b) {
    return OP == 0 ? a + b : OP == 1 ? a * b : fmin(a, b);
}
template <int OP>
__device__ __forceinline__ double wave_fold_dpp(double v) {
    v = fold_op<OP>(v, dpp_f64<0xB1>(v));
    v = fold_op<OP>(v, dpp_f64<0x4E>(v));
    v = fold_op<OP>(v, dpp_f64<0x141>(v));
    v = fold_op<OP>(v, dpp_f64<0x140>(v));
    const long long u = __double_as_longlong(v);
    double r[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        r[k] = __hiloint2double(__builtin_amdgcn_readlane((int)(u >> 32), 16 * k),
                                __builtin_amdgcn_readlane((int)(u & 0xffffffffll), 16 * k));
    return fold_op<OP>(fold_op<OP>(r[0], r[1]), fold_op<OP>(r[2], r[3]));
}

// m in [1/2, 1) and its exponent moved into e (exact: e holds integers far below 2^53)
__device__ __forceinline__ void mant_norm(double& m, double& e) {
    e += (double)__builtin_amdgcn_frexp_exp(m);
    m = __builtin_amdgcn_frexp_mant(m);
}

__device__ __forceinline__ void pairb_fold_records(const double4* __restrict__ rec, const int32_t* __restrict__ lexp,
                                                   int64_t n_tiles, double* __restrict__ partials,
                                                   double (*sh)[5]) {
    constexpr int NT = kPairbThreads;
    const int t = threadIdx.x;
    double a = 1.0, e = 0.0, b = 0.0, c = INFINITY, d = INFINITY;  // a: mantissa product, e: exponent sum
    // 8 records per thread in flight per round; a product of 8 mantissas in [1/2, 1) stays above 2^-8:
    // one renormalisation per round
    for (int64_t k0 = t; k0 < n_tiles; k0 += 8 * NT) {
        double4 r[8];
        int32_t x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t k = k0 + (int64_t)u * NT;
            r[u] = k < n_tiles ? rec[k] : make_double4(1.0, 0.0, INFINITY, INFINITY);
            x[u] = k < n_tiles ? lexp[k] : 0;
        }
        double pm = 1.0;
        int32_t pe = 0;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            pm *= r[u].x;
            pe += x[u];
            b += r[u].y;
            c = fmin(c, r[u].z);
            d = fmin(d, r[u].w);
        }
        a *= pm;
        e += (double)pe;
        mant_norm(a, e);
    }
    // one wave: 64 mantissas in [1/2, 1) multiply to no less than 2^-64
    a = wave_fold_dpp<1>(a);
    e = wave_fold_dpp<0>(e);
    mant_norm(a, e);
    b = wave_fold_dpp<0>(b);
    c = wave_fold_dpp<2>(c);
    d = wave_fold_dpp<2>(d);
    if ((t & 63) == 0) {
        sh[t >> 6][0] = a;
        sh[t >> 6][1] = e;
        sh[t >> 6][2] = b;
        sh[t >> 6][3] = c;
        sh[t >> 6][4] = d;
    }
    __syncthreads();
    if (t == 0) {  // the wave results in wave order
        a = 1.0, e = 0.0, b = 0.0, c = INFINITY, d = INFINITY;
#pragma unroll
        for (int w = 0; w < NT / 64; ++w) {
            a *= sh[w][0];
            e += sh[w][1];
            b += sh[w][2];
            c = fmin(c, sh[w][3]);
            d = fmin(d, sh[w][4]);
        }
        partials[0] = fma(e, 0.6931471805599453, log(a));
        partials[1] = b;
        partials[2] = c == INFINITY ? -1.0 : c;
        partials[3] = d == INFINITY ? -1.0 : d;
    }
}

// 1/x to ~1 ulp for a positive normal x: v_rcp_f64 (~2^-26) and one second-order correction
// y (1 + e + e^2), e = 1 - x y (3 ops; the e^3 term is below 2^-78; two Newton steps are 4)
__device__ __forceinline__ double pr_rcp(double x) {
    const double y = __builtin_amdgcn_rcp(x);
    const double e = fma(-x, y, 1.0);
    return fma(y, fma(e, e, e), y);
}

// KIND == NNGP_KIND_BLOCKS (nngp_bf_sweep_blocks): the joint block's covariances are read from
// cblk instead of evaluated -- a user covariance (any isotropic function of distance, evaluated on the
// GPU by the caller over nngp_joint_dist's distances): entry (a, b), b <= a <= M, of nbr row t at
// cblk[(a (a + 1) / 2 + b) * n_rows + t] (entry-major: one load instruction reads 32 consecutive
// rows).  Slots with an invalid neighbour index are decoupled exactly (0 off the diagonal, 1 on it)
// whatever the caller's values there; sigma2 = 1 (the blocks are the covariances themselves).
// Wave pair plans (pair_plan.h): PL = true reads each wave's distinct covariance pairs and its lanes' entry maps
// from the plan instead of gathering coordinates per location; tiles != null lists the tiles (regions) this
// launch sweeps (the planned and the direct launches of a planned sweep), n_tiles = all regions.
struct PairPlanArgs {
    const uint8_t* slots = nullptr;   // region slots (pair_plan.h), region r at slots + r * slot_bytes
    const int32_t* tiles = nullptr;   // logical block -> region, or null (block b sweeps tile b)
    int64_t slot_bytes = 0;
    int64_t n_tiles = 0;              // regions of the whole sweep (the record fold's count)
};

template <int M, int KIND, int D, bool PL = false>
__global__ __launch_bounds__(kPairbThreads) NNGP_PAIRB_ATTR void bf_pairb(const double* __restrict__ coords, int64_t n_points,
                                                const int32_t* __restrict__ nbr, const int32_t* __restrict__ order,
                                                int64_t n_rows, int64_t i0, const CovParams Pc, double sigma2,
                                                const double* __restrict__ values, const double* __restrict__ qcoords,
                                                const double* __restrict__ qvalues, double* __restrict__ Bout,
                                                double* __restrict__ Fout, double* __restrict__ Rout,
                                                double4* __restrict__ rec, int32_t* __restrict__ lexp, int dim,
                                                const double* __restrict__ cblk, int64_t tq, int64_t trem,
                                                int64_t* __restrict__ hdr, const PairPlanArgs pp) {
    static_assert(M >= 1 && M <= 32, "pairb instantiated for 1 <= m <= 32");
    static_assert(D >= 0 && D <= 3, "0 (runtime dimension) <= D <= 3");
    constexpr bool CM = KIND == NNGP_KIND_BLOCKS;
    constexpr bool MT = KIND == NNGP_KIND_MATERN;  // cblk: the launch's Matern table (matern_table.hip)
    constexpr int DA = point_arity<D>();  // coordinates held per point
    const int ds = D == 0 ? dim : D;      // row stride of coords / qcoords
    constexpr int NR = M + 1;         // joint rows 0..M (row M = the location)
    constexpr int NP = (NR + 1) / 2;  // row pairs
    constexpr int T = M / 2;          // pairs made of two neighbour rows: full 2x2 block steps
    constexpr bool LEFT = !PL && pairb_lk(M, KIND);  // (the planned kernel is right-looking)
    static_assert(!PL || (!CM && !MT && !LEFT && D >= 1 && M >= kPlanMinM && M <= kPlanMaxM),
                  "pair plans: the right-looking fused kinds, 1 <= D <= 3");
    // the planned kernel's LDS (pair_plan.h): one slice per wave -- the wave's distinct covariances from its
    // head (slot 0: the exact zero), the wave's points at its end
    constexpr int PSL = PL ? plan_slice_bytes(M) : 16;
    __shared__ __attribute__((aligned(16))) double wsl[PL ? kPairbWaves * PSL / 8 : 1];
    // (no value column in the elimination: the residual is r = v_i - B v_N after the back-substitution, the
    // oracle's own formula -- 5 % fewer VALU at m = 15 than forward-solving the values through it)
    constexpr bool SLDL = !LEFT;
    constexpr int KL0 = MT ? kPairbLeftLdsRowsMT
                           : (M >= kPairbLeftOneWaveMin ? kPairbLeftLdsRows1W : kPairbLeftLdsRows);
    constexpr int KL = !LEFT ? 0 : (KL0 < M / 2 - 1 ? KL0 : M / 2 - 1);
    // the left-looking kernel's LDS in one object: the exp table first (its reads fold the base into the
    // 16-bit offset field; the LDS lowering sorts separate objects by size, which put it above 64 KB), the
    // finished factor rows, then the late state -- the neighbour indices (its values are gathered late),
    // the row, the bad-index flag: held in registers through its factorisation they spilled 13 dwords per
    // lane to scratch, written once and reloaded at the end (+95 B of HBM writes per location at m = 20,
    // profiles/r04e)
    constexpr int LXW = (NP + 3 + 1) / 2;  // doubles per thread of the late state
    __shared__ double lbuf[LEFT ? NNGP_EXP_TAB_N + (KL * (KL + 1) + LXW) * kPairbThreads : 1];
    double(*const lrow)[kPairbThreads] = (double(*)[kPairbThreads])(lbuf + NNGP_EXP_TAB_N);
    int32_t(*const lidx)[kPairbThreads] =
        (int32_t(*)[kPairbThreads])(lbuf + NNGP_EXP_TAB_N + KL * (KL + 1) * kPairbThreads);
    __shared__ double etab_own[MT || LEFT ? 1 : NNGP_EXP_TAB_N];
    double* const etab = LEFT ? lbuf : etab_own;
    extern __shared__ double4 pairb_mtab[];  // MT: the Matern table (dynamic LDS, NNGP_MT_BYTES(noct))
    const double* ctab = MT ? (const double*)pairb_mtab : etab;
    // table entries per thread (threads past the table's 256 entries of a 512-thread block fetch
    // entry j - 256 and do not store it)
    constexpr int kTabPer = kPairbThreads >= NNGP_EXP_TAB_N ? 1 : NNGP_EXP_TAB_N / kPairbThreads;
    static_assert(kPairbThreads >= NNGP_EXP_TAB_N || kTabPer * kPairbThreads == NNGP_EXP_TAB_N, "table fill");
    double etab_entry[kTabPer];
    if constexpr (!CM && !MT) {
#pragma unroll
        for (int e = 0; e < kTabPer; ++e)
            etab_entry[e] = nngp_exp_table_entry_unit(((int)threadIdx.x + e * kPairbThreads) & (NNGP_EXP_TAB_N - 1));
    }

    __shared__ double sh[1][kPairbWaves][5];
    const int64_t ltile = xcd_logical_block(blockIdx.x, gridDim.x);
    const int64_t tile = pp.tiles != nullptr ? (int64_t)__builtin_amdgcn_readfirstlane(pp.tiles[ltile]) : ltile;
    if (blockIdx.x == 0 && threadIdx.x == 0) hdr[0] = pp.tiles != nullptr ? pp.n_tiles : gridDim.x;  // for the record fold
    const int q = (int)(threadIdx.x & 1);
    const bool q1 = q == 1;
    const bool lead0 = !q1;
    const double wq1 = q1 ? 1.0 : 0.0, wq0 = 1.0 - wq1;
    uint32_t mask1 = q1 ? 0xffffffffu : 0u;
    asm volatile("" : "+v"(mask1));  // opaque to the optimizer (see pr_pick)
    {
        const int64_t lr = threadIdx.x >> 1;  // the tile's local row (pairb_tiling)
        const int64_t r = tile * tq + (tile < trem ? tile : trem) + lr;
        const bool live = lr < tq + (tile < trem ? 1 : 0);
        const int64_t rl = live ? r : n_rows - 1;
        // branch-free (a branch here makes the compiler drain every outstanding load, the
        // early exp-table fetch included, at the join): without an order, read nbr's word
        const int32_t ov = (order != nullptr ? order : nbr)[rl];
        const int64_t rr = order != nullptr ? (int64_t)ov : rl;
        const int64_t i = i0 + rr;

        // ---- gathers (branch-free, as bf_group): own rows a = 2s + q
        int32_t jn[NP];
#pragma unroll
        for (int s = 0; s < NP; ++s) {
            const int a = 2 * s + q;
            jn[s] = nbr[rl * M + (a < M ? a : M - 1)];
        }
        double o[NP][DA], z[NP];
        // one unsigned compare per slot (a negative index is out of range as a huge unsigned);
        // an index >= n_points anywhere in the row shows in the row's largest index, one below -1
        // (only -1 pads a row) in its smallest (n_points >= 2^31: every non-negative int32 index is
        // in range)
        const uint32_t n32 = n_points < (int64_t)0x80000000ll ? (uint32_t)n_points : 0x80000000u;
        int32_t jmax = -1, jmin = -1;
#pragma unroll
        for (int s = 0; s < NP; ++s) {
            const int a = 2 * s + q;
            const int32_t j = a < M ? jn[s] : -1;
            jmax = max(jmax, j);
            jmin = min(jmin, j);
            const bool in_range = (uint32_t)j < n32;
            const bool self = a == M;
            const double* pc = self ? qcoords + i * ds : (in_range ? coords + (int64_t)j * ds : far_point<DA>(a));
            const double* pv = self ? (qvalues != nullptr ? qvalues + i : kZeroValue)
                                    : ((values != nullptr && in_range) ? values + j : kZeroValue);
            if constexpr (CM || PL) {
            } else if constexpr (D == 0) {
                load_point_rt(pc, dim, o[s]);
            } else {
                load_point<D>(pc, o[s]);
            }
            if constexpr (!LEFT) z[s] = *pv;  // (the left-looking kernel gathers the values late)
        }
        const bool bad_index = (int64_t)jmax >= n_points || jmin < -1;
        if constexpr (LEFT) {  // the late state waits in LDS (read back by this thread only)
#pragma unroll
            for (int s = 0; s < NP; ++s) lidx[s][threadIdx.x] = jn[s];
            lidx[NP][threadIdx.x] = (int32_t)(uint32_t)(uint64_t)rr;
            lidx[NP + 1][threadIdx.x] = (int32_t)(uint32_t)((uint64_t)rr >> 32);
            lidx[NP + 2][threadIdx.x] = bad_index ? 1 : 0;
        }

        // the exp table entry was fetched before the gathers; storing it here lets its load and
        // the barrier overlap the gathers' latency instead of preceding it
        if constexpr (MT) {
            const int n4 = Pc.mt_noct * (NNGP_MT_K * NNGP_MT_NC / 4);
            const double4* g = (const double4*)cblk;
            for (int k = (int)threadIdx.x; k < n4; k += kPairbThreads) pairb_mtab[k] = g[k];
            __syncthreads();
        } else if constexpr (!CM && !PL) {
#pragma unroll
            for (int e = 0; e < kTabPer; ++e)
                if (kPairbThreads <= NNGP_EXP_TAB_N || threadIdx.x < NNGP_EXP_TAB_N)
                    etab[threadIdx.x + e * kPairbThreads] = etab_entry[e];
            __syncthreads();
        }

        double R[NP][NP][2];
        bool bad = false;
        bool stale_plan = false;  // PL: the plan was built for other neighbour sets (flagged as a bad index)
        double Fu, res;
        if constexpr (PL) {
            // ---- the wave's plan (pair_plan.h), wave-private after the table barrier: the map, the U list and
            // the pair words are streamed in at once (fixed offsets in the wave's slot, no dependent header
            // read), the U points' coordinates are the one dependent gather, staged at the end of the wave's
            // LDS slice; each distinct pair is evaluated once by one lane into the slice's head; the joint
            // block is read through the lane's map.  No block barrier after the table's.
            constexpr int CHE = plan_map_chunks(M);
            constexpr int PS = plan_ps(DA);
            constexpr int UK = plan_ucap(M) / 64;  // U-list rounds (max)
            constexpr int64_t WSB = plan_wave_slot_bytes(M);
            const int wv = (int)(threadIdx.x >> 6), L = (int)(threadIdx.x & 63);
            const uint8_t* wsp = pp.slots + tile * pp.slot_bytes + (int64_t)__builtin_amdgcn_readfirstlane(wv) * WSB;
            // (wave-uniform: scalar loads and branches)
            const int nU0 = __builtin_amdgcn_readfirstlane(((const int32_t*)wsp)[0]);
            const int nE0 = __builtin_amdgcn_readfirstlane(((const int32_t*)wsp)[1]);
            const int st0 = __builtin_amdgcn_readfirstlane(((const int32_t*)wsp)[2]);
            // a foreign or damaged plan stays inside the slice and comes out NaN
            const bool over = st0 != 0 || nU0 < 0 || nU0 > plan_ucap(M) || nE0 < 0 || nE0 > plan_ecap(M) ||
                              !plan_fits(nU0, nE0, PS, PSL);
            const int nU = over ? 0 : nU0, nE = over ? 0 : nE0;
            bad = over;
            const __amdgpu_buffer_rsrc_t srd =
                __builtin_amdgcn_make_buffer_rsrc((void*)wsp, (short)0, (int)WSB, 0x00020000);
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            uint32_t mw[4 * CHE];
#pragma unroll
            for (int c = 0; c < CHE; ++c) {
                const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(srd, plan_map_off(M) + 16 * L, c * 64 * 16, 0);
                mw[4 * c] = v.x;
                mw[4 * c + 1] = v.y;
                mw[4 * c + 2] = v.z;
                mw[4 * c + 3] = v.w;
            }
            const uint32_t ck = __builtin_amdgcn_raw_buffer_load_b32(srd, plan_chk_off(M) + 4 * L, 0, 0);
            // (every round, without waiting for the header: the builder zero-fills the list)
            int32_t ug[UK];
#pragma unroll
            for (int k = 0; k < UK; ++k)
                ug[k] = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(srd, plan_u_off() + 4 * L, 256 * k, 0);
            // pair rounds in groups of PG = 4 (the builder zero-fills the words of the last group and keeps its
            // slots below the points): a group's words are one 16-byte load per lane (lane-major in the slot)
            static_assert(kPlanPairGroup == 4, "one 16-byte word load per lane and group");
            constexpr int PG = kPlanPairGroup;
            constexpr int KG = plan_pair_groups(M);  // groups (max)
            const int ngr = (nE + 64 * PG - 1) / (64 * PG);                 // wave-uniform
            // (the first two groups without waiting for the header: the loop starts from them)
            u32x4 wg[KG];
#pragma unroll
            for (int g = 0; g < KG; ++g)
                wg[g] = (g < 2 || g < ngr) ? __builtin_amdgcn_raw_buffer_load_b128(srd, plan_pair_off(M) + 16 * L, 1024 * g, 0)
                                           : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
            for (int e = 0; e < kTabPer; ++e)
                if (kPairbThreads <= NNGP_EXP_TAB_N || threadIdx.x < NNGP_EXP_TAB_N)
                    etab[threadIdx.x + e * kPairbThreads] = etab_entry[e];
            __syncthreads();
            NNGP_PHASE(plan_points);
            char* const sl = (char*)wsl + wv * PSL;  // this wave's slice
            const int cb = PSL - nU * PS;            // its points' base
#pragma unroll
            for (int k = 0; k < UK; ++k) {
                if (64 * k < nU) {  // wave-uniform
                    const uint32_t g = (uint32_t)ug[k] < (uint32_t)n_points ? (uint32_t)ug[k] : 0u;
                    double x[DA];
                    load_point<DA>(coords + (int64_t)g * ds, x);
                    if (L + 64 * k < nU) {
                        double* pd = (double*)(sl + cb + (L + 64 * k) * PS);
                        if constexpr (DA == 2) {
                            *(double2*)pd = make_double2(x[0], x[1]);
                        } else {
#pragma unroll
                            for (int c = 0; c < DA; ++c) pd[c] = x[c];
                        }
                    }
                }
            }
            // group g's words (g >= 2) wait in the covariance slots of group g - 2, [8 + 2048 (g - 2), + 1024):
            // the loop reads them at the start of half g - 2, before that half's stores
#pragma unroll
            for (int g = 2; g < KG; ++g)
                if (g < ngr) *(u32x4*)(sl + 8 + 2048 * (g - 2) + 16 * L) = wg[g];
            // (a wave's LDS operations complete in order; the barrier keeps the compiler's order)
            asm volatile("" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            NNGP_PHASE(plan_pairs);
            // the wave's distinct pairs: a loop over groups, software-pipelined -- group g + 1's words and point
            // reads are in flight while group g is evaluated (the unplanned kernel's nngp_cov_unit on the same
            // operands: (a - b)^2 == (b - a)^2 bit for bit)
            auto pair_points = [&](const u32x4 w4, double (*xa)[DA], double (*xb)[DA]) {
                const uint32_t w[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
                for (int j = 0; j < PG; ++j) {
                    const double* pa = (const double*)(sl + (w[j] & 0xffffu));
                    const double* pb = (const double*)(sl + (w[j] >> 16));
                    if constexpr (DA == 2) {
                        const double2 va = *(const double2*)pa, vb = *(const double2*)pb;
                        xa[j][0] = va.x;
                        xa[j][1] = va.y;
                        xb[j][0] = vb.x;
                        xb[j][1] = vb.y;
                    } else {
#pragma unroll
                        for (int c = 0; c < DA; ++c) {
                            xa[j][c] = pa[c];
                            xb[j][c] = pb[c];
                        }
                    }
                }
            };
            // one group's covariances from its points into its slots
            auto pair_covs = [&](int g, double (*xa)[DA], double (*xb)[DA]) {
#pragma unroll
                for (int j = 0; j < PG; ++j)
                    *(double*)(sl + 8 * (1 + L + 64 * (PG * g + j))) =
                        nngp_cov_unit<KIND>(Pc, ctab, point_d2<DA>(xa[j], xb[j]));
            };
            // (past the last group: group 0's words, valid point offsets, read for nothing)
            const u32x4 w0g = wg[0];
            auto group_words = [&](int g) -> u32x4 {
                return g < ngr ? *(const u32x4*)(sl + 8 + 2048 * (g - 2) + 16 * L) : w0g;
            };
            double xa0[PG][DA], xb0[PG][DA], xa1[PG][DA], xb1[PG][DA];
            pair_points(wg[0], xa0, xb0);
            // two groups per trip, the point registers and the word registers alternating (no copies): at a
            // trip's start x0 holds group g's points and wA group g + 1's words; each half reads the words two
            // groups ahead and the points one group ahead of the group it evaluates
            u32x4 wA = wg[KG > 1 ? 1 : 0], wB;
#pragma unroll 1
            for (int g = 0; g < ngr; g += 2) {
                wB = group_words(g + 2);
                pair_points(wA, xa1, xb1);
                pair_covs(g, xa0, xb0);
                if (g + 1 >= ngr) break;  // wave-uniform
                wA = group_words(g + 3);
                pair_points(wB, xa0, xb0);
                pair_covs(g + 1, xa1, xb1);
            }
            if (L == 0) *(double*)sl = 0.0;  // the exact-zero slot
            asm volatile("" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            NNGP_PHASE(plan_fill);
            // the joint block in the unplanned kernel's register order (pair_plan.h plan_entry): entry e's
            // slice byte offset is u16 half e & 1 of map word e >> 1
            auto rd = [&](int e) -> double {
                const uint32_t off = (e & 1) ? (mw[e >> 1] >> 16) : (mw[e >> 1] & 0xffffu);
                return *(const double*)(sl + off);
            };
            int e = 0;
#pragma unroll
            for (int s = 0; s < NP; ++s) {
#pragma unroll
                for (int t = 0; t < s; ++t) {
                    R[s][t][0] = rd(e++);
                    R[s][t][1] = rd(e++);
                }
                R[s][s][0] = Pc.diag;
                R[s][s][1] = rd(e++);
            }
            // the plan belongs to this nbr / order: the lane's checksum (pair_plan.h plan_chk_*)
            uint32_t h = plan_chk_init((uint32_t)(uint64_t)rr);
#pragma unroll
            for (int s = 0; s < NP; ++s) h = plan_chk_step(h, jn[s], s);
            const int stale = h != ck ? 1 : 0;
            stale_plan = (stale | __builtin_amdgcn_mov_dpp(stale, 0xB1, 0xf, 0xf, true)) != 0;  // either lane of the pair
        }
        // ---- covariances from the caller's blocks (CM), own-parity-first order.  vm: bit a set when
        // joint row a holds a point (a valid neighbour slot, or a = M); this lane's rows, then the
        // partner's by one swap
        uint32_t vm = 0;
        if constexpr (CM) {
#pragma unroll
            for (int s = 0; s < NP; ++s) {
                const int a = 2 * s + q;
                const bool ok = a == M || (a < M && (uint32_t)jn[s] < n32);
                vm |= ok ? (1u << a) : 0u;
            }
            vm |= (uint32_t)__builtin_amdgcn_mov_dpp((int)vm, 0xB1, 0xf, 0xf, true);
        }
        const double* cb = cblk + rl;
        // lane 0 reads entry (a0, b0), lane 1 (a1, b1) -- compile-time after unrolling, so each load
        // costs two selects and an address multiply-add; 0 unless both rows hold points
        auto ldc2 = [&](int a0, int b0, int a1, int b1) -> double {
            const int e0 = (a0 * (a0 + 1) >> 1) + b0, e1 = (a1 * (a1 + 1) >> 1) + b1;
            const uint32_t need = q1 ? ((1u << a1) | (1u << b1)) : ((1u << a0) | (1u << b0));
            const bool ok = (vm & need) == need;
            const int64_t e = ok ? (q1 ? e1 : e0) : 0;  // an in-range address either way (branch-free)
            const double v = cb[e * n_rows];
            return ok ? v : 0.0;
        };
        if constexpr (CM && !LEFT) {
#pragma unroll
            for (int s = 0; s < NP; ++s) {
                const int a0 = 2 * s, a1 = 2 * s + 1;
#pragma unroll
                for (int t = 0; t < s; ++t) {
                    R[s][t][0] = ldc2(a0, 2 * t, a1, 2 * t + 1);      // (a, 2t + q)
                    R[s][t][1] = ldc2(a0, 2 * t + 1, a1, 2 * t);      // (a, 2t + 1 - q)
                }
                const double dg = ldc2(a0, a0, a1, a1);
                R[s][s][0] = ((vm >> (2 * s + q)) & 1u) ? dg : 1.0;   // a decoupled row: identity
                const double w = ldc2(a0, a0, a1, a0);               // (2s+1, 2s), read from lane 1 only
                R[s][s][1] = q1 ? w : 0.0;
            }
        }
        if constexpr (!LEFT) {
        NNGP_PHASE(covariances);
        // ---- unit-variance covariances in own-parity-first order
        if constexpr (!CM && !PL) {
            double p[NP][DA];
#pragma unroll
            for (int t = 0; t < NP; ++t)
#pragma unroll
                for (int k = 0; k < DA; ++k) p[t][k] = pr_swap(o[t][k]);
#pragma unroll
            for (int s = 0; s < NP; ++s) {
#pragma unroll
                for (int t = 0; t < s; ++t) {
                    R[s][t][0] = nngp_cov_unit<KIND>(Pc, ctab, point_d2<DA>(o[s], o[t]));
                    R[s][t][1] = nngp_cov_unit<KIND>(Pc, ctab, point_d2<DA>(o[s], p[t]));
                }
                R[s][s][0] = Pc.diag;
            }
            // the within-pair entries (2s+1, 2s) are read from lane 1 only (lane 0's R[s][s][1] is
            // never used): of each two pairs, lane 0 evaluates the first and lane 1 the second, and
            // lane 0's value moves to lane 1 -- half the evaluations of one per pair in both lanes
#pragma unroll
            for (int s0 = 0; s0 < NP; s0 += 2) {
                const int s1 = s0 + 1;
                if (M <= kPairbDedupMax && s1 < NP) {
                    double a[DA], b[DA];
#pragma unroll
                    for (int k = 0; k < DA; ++k) {
                        a[k] = pr_pick(mask1, o[s1][k], o[s0][k]);
                        b[k] = pr_pick(mask1, p[s1][k], p[s0][k]);
                    }
                    const double c = nngp_cov_unit<KIND>(Pc, ctab, point_d2<DA>(a, b));
                    R[s1][s1][1] = c;
                    R[s0][s0][1] = pr_from0(c);
                } else {
                    R[s0][s0][1] = nngp_cov_unit<KIND>(Pc, ctab, point_d2<DA>(o[s0], p[s0]));
                    if (s1 < NP) R[s1][s1][1] = nngp_cov_unit<KIND>(Pc, ctab, point_d2<DA>(o[s1], p[s1]));
                }
            }
        }

        // ---- 2x2-blocked right-looking elimination of the neighbour columns 0..M-1.
        // After block step t: lane q's R[t][t][0] = 1 / L[2t+q][2t+q], R[t][t][1] = L[2t+1][2t]
        // (both lanes), rows s > t hold their panel entries (L[a][2t+q], L[a][2t+1-q]) and z[t]
        // the forward-solved value of row 2t+q.
        NNGP_PHASE(elimination);
        if constexpr (SLDL) {
            // 2x2-blocked scalar-pivot LDL^T: per pair t the pivots d00 and e11 = d11 - l d10 (l =
            // d10 / d00) need a reciprocal each instead of an inverse square root.  Each later row's
            // panel X becomes W = X L_D^{-T} (its column 2t+1 loses l times column 2t) in place; in
            // the update of row pair u the partner's side is Q_u = W_u diag(1/d00, 1/e11), which is
            // also row u's entry of the unit factor and replaces W_u once pair u is done.  Like the
            // Cholesky form the first column is one product and the second one subtraction away
            // from X (no 2x2 inverse with 1/det entries, which lost accuracy: see the note above).
#pragma unroll
            for (int t = 0; t < T; ++t) {
                const double d00 = pr_from0(R[t][t][0]);
                const double d11 = pr_from1(R[t][t][0]);
                const double d10 = pr_from1(R[t][t][1]);
                bad |= !(d00 > 0.0);
                const double r00 = pr_rcp(d00);
                const double l10 = d10 * r00;
                const double e11 = fma(-l10, d10, d11);
                bad |= !(e11 > 0.0);
                const double r11 = pr_rcp(e11);
                R[t][t][1] = l10;  // L[2t+1][2t] of the unit factor
                const double town = pr_sel(q1, r11, r00), toth = pr_sel(q1, r00, r11);
                const double g1 = -l10 * wq1, g0 = -l10 * wq0;
#pragma unroll
                for (int s = t + 1; s < NP; ++s) {
                    const double x0 = R[s][t][0], x1 = R[s][t][1];
                    R[s][t][0] = fma(g1, x1, x0);
                    R[s][t][1] = fma(g0, x0, x1);
                }
#pragma unroll
                for (int u = t + 1; u < NP; ++u) {
                    const double Q0 = R[u][t][0] * town, Q1 = R[u][t][1] * toth;
                    const double P0 = pr_swap(Q0), P1 = pr_swap(Q1);
#pragma unroll
                    for (int s = u; s < NP; ++s) {
                        const double w0 = R[s][t][0], w1 = R[s][t][1];
                        R[s][u][0] = fma(-w0, Q0, fma(-w1, Q1, R[s][u][0]));
                        R[s][u][1] = fma(-w0, P1, fma(-w1, P0, R[s][u][1]));
                    }
                    R[u][t][0] = Q0;
                    R[u][t][1] = Q1;
                }
            }
        } else {
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
            R[t][t][0] = pr_sel(q1, i11, i00);
            R[t][t][1] = l10;
            // panel map (L[a][2t], L[a][2t+1]) = (A[a][2t], A[a][2t+1]) U, U = [[i00, u01], [0, i11]],
            // written in own-parity-first coordinates: Y0 = X0 c00 + X1 c10, Y1 = X0 c01 + X1 c11
            const double u01 = -(l10 * i00) * i11;
            // c10 / c01 = u01 in one lane, 0 in the other: one multiply by the lane's 0/1 weight each
            // instead of a two-dword select
            const double c00 = pr_sel(q1, i11, i00), c10 = u01 * wq1;
            const double c01 = u01 * wq0, c11 = pr_sel(q1, i00, i11);
#pragma unroll
            for (int s = t + 1; s < NP; ++s) {
                const double x0 = R[s][t][0], x1 = R[s][t][1];
                const double y0 = fma(x0, c00, x1 * c10);
                const double y1 = fma(x0, c01, x1 * c11);
                R[s][t][0] = y0;
                R[s][t][1] = y1;
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
        }

        NNGP_PHASE(lastpair);
        // ---- last pair: (M-1, M) for odd M (one more column), (M, padding) for even M
        if (M % 2 == 1 && SLDL) {
            const double a00 = pr_from0(R[T][T][0]);
            const double a11 = pr_from1(R[T][T][0]);
            const double a10 = pr_from1(R[T][T][1]);
            bad |= !(a00 > 0.0);
            const double l10 = a10 * pr_rcp(a00);  // L[M][M-1] of the unit factor = B_{M-1}
            Fu = fma(-l10, a10, a11);
            R[T][T][0] = 1.0;
            R[T][T][1] = l10;
        } else if (M % 2 == 1) {
            const double a00 = pr_from0(R[T][T][0]);
            const double a11 = pr_from1(R[T][T][0]);
            const double a10 = pr_from1(R[T][T][1]);
            bad |= !(a00 > 0.0);
            const double i00 = nngp_rsqrt(a00);
            const double l10 = a10 * i00;
            Fu = fma(-l10, l10, a11);
            R[T][T][0] = i00;  // lane 0: 1 / L[M-1][M-1]
            R[T][T][1] = l10;  // L[M][M-1]
        } else {
            Fu = pr_from0(R[T][T][0]);
        }
        } else {
            // ---- left-looking 2x2-blocked Cholesky (kPairbLeftMin): step u evaluates column
            // pair u's covariances for rows s >= u, subtracts the finished column pairs t < u (the
            // same 2x2 block products as the right-looking update, reordered), factors the diagonal
            // block and maps the panel.  Row pair u is then final; rows < KL move to LDS.
            NNGP_PHASE(leftlooking);
            double pnext[DA], wpnext = 0.0;  // pair u+1's partner coordinates / within-pair entry
#pragma unroll
            for (int u = 0; u < NP; ++u) {
                if constexpr (CM) {  // column pair u's entries from the caller's blocks
#pragma unroll
                    for (int s = u + 1; s < NP; ++s) {
                        R[s][u][0] = ldc2(2 * s, 2 * u, 2 * s + 1, 2 * u + 1);      // (a, 2u + q)
                        R[s][u][1] = ldc2(2 * s, 2 * u + 1, 2 * s + 1, 2 * u);      // (a, 2u + 1 - q)
                    }
                    const double dg = ldc2(2 * u, 2 * u, 2 * u + 1, 2 * u + 1);
                    R[u][u][0] = ((vm >> (2 * u + q)) & 1u) ? dg : 1.0;  // a decoupled row: identity
                    const double wv = ldc2(2 * u, 2 * u, 2 * u + 1, 2 * u);  // (2u+1, 2u), read from lane 1 only
                    R[u][u][1] = q1 ? wv : 0.0;
                } else {
                double pu[DA];
#pragma unroll
                for (int k = 0; k < DA; ++k) pu[k] = (u % 2 == 1) ? pnext[k] : pr_swap(o[u][k]);
#pragma unroll
                for (int s = u + 1; s < NP; ++s) {
                    R[s][u][0] = nngp_cov_unit<KIND>(Pc, ctab, point_d2<DA>(o[s], o[u]));
                    R[s][u][1] = nngp_cov_unit<KIND>(Pc, ctab, point_d2<DA>(o[s], pu));
                }
                R[u][u][0] = Pc.diag;
                // the within-pair entry (2u+1, 2u) is read from lane 1 only: for pairs u, u+1 (u even)
                // lane 0 evaluates pair u's and lane 1 pair u+1's, and lane 0's moves over (as the
                // right-looking kernel's split)
                if (u % 2 == 0 && u + 1 < NP) {
                    double a[DA], b[DA];
#pragma unroll
                    for (int k = 0; k < DA; ++k) {
                        pnext[k] = pr_swap(o[u + 1][k]);
                        a[k] = pr_pick(mask1, o[u + 1][k], o[u][k]);
                        b[k] = pr_pick(mask1, pnext[k], pu[k]);
                    }
                    wpnext = nngp_cov_unit<KIND>(Pc, ctab, point_d2<DA>(a, b));
                    R[u][u][1] = pr_from0(wpnext);
                } else if (u % 2 == 1) {
                    R[u][u][1] = wpnext;
                } else {
                    R[u][u][1] = nngp_cov_unit<KIND>(Pc, ctab, point_d2<DA>(o[u], pu));  // (2u+1, 2u): lane 1's
                }
                }
#pragma unroll
                for (int t = 0; t < u; ++t) {
                    const double S0 = R[u][t][0], S1 = R[u][t][1];
                    const double P0 = pr_swap(S0), P1 = pr_swap(S1);
#pragma unroll
                    for (int s = u; s < NP; ++s) {
                        const double y0 = R[s][t][0], y1 = R[s][t][1];
                        R[s][u][0] = fma(-y0, S0, fma(-y1, S1, R[s][u][0]));
                        R[s][u][1] = fma(-y0, P1, fma(-y1, P0, R[s][u][1]));
                    }
                }
                if (u < T) {
                    const double a00 = pr_from0(R[u][u][0]);
                    const double a11 = pr_from1(R[u][u][0]);
                    const double a10 = pr_from1(R[u][u][1]);
                    bad |= !(a00 > 0.0);
                    const double i00 = nngp_rsqrt(a00);
                    const double l10 = a10 * i00;
                    const double s11 = fma(-l10, l10, a11);
                    bad |= !(s11 > 0.0);
                    const double i11 = nngp_rsqrt(s11);
                    R[u][u][0] = pr_sel(q1, i11, i00);
                    R[u][u][1] = l10;
                    const double u01 = -(l10 * i00) * i11;
                    const double c00 = pr_sel(q1, i11, i00), c10 = u01 * wq1;
                    const double c01 = u01 * wq0, c11 = pr_sel(q1, i00, i11);
#pragma unroll
                    for (int s = u + 1; s < NP; ++s) {
                        const double x0 = R[s][u][0], x1 = R[s][u][1];
                        R[s][u][0] = fma(x0, c00, x1 * c10);
                        R[s][u][1] = fma(x0, c01, x1 * c11);
                    }
                } else if (M % 2 == 1) {  // u = T: the pair (M-1, M)
                    const double a00 = pr_from0(R[T][T][0]);
                    const double a11 = pr_from1(R[T][T][0]);
                    const double a10 = pr_from1(R[T][T][1]);
                    bad |= !(a00 > 0.0);
                    const double i00 = nngp_rsqrt(a00);
                    const double l10 = a10 * i00;
                    Fu = fma(-l10, l10, a11);
                    R[T][T][0] = i00;
                    R[T][T][1] = l10;
                } else {  // u = T: the pair (M, padding)
                    Fu = pr_from0(R[T][T][0]);
                }
                if (u < KL) {
#pragma unroll
                    for (int t = 0; t <= u; ++t) {
                        lrow[u * (u + 1) + 2 * t][threadIdx.x] = R[u][t][0];
                        lrow[u * (u + 1) + 2 * t + 1][threadIdx.x] = R[u][t][1];
                    }
                }
            }
        }
        // factor entry (row pair u, column pair t, slot k) for the back-substitution (rows < KL of
        // the left-looking factor from LDS; u, t, k are compile-time after unrolling)
        auto RB = [&](int u, int t, int k) -> double {
            if (u < KL) return lrow[u * (u + 1) + 2 * t + k][threadIdx.x];
            return R[u][t][k];
        };
        bad |= !(Fu > 0.0);
        const double F = Fu * sigma2;  // the unit-variance pivot scaled back
        int64_t rrl = rr, il = i;
        bool bidx = bad_index || stale_plan;
        if constexpr (LEFT) {
            // (the fence keeps the compiler from forwarding the stores' registers past the factorisation)
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            rrl = (int64_t)(((uint64_t)(uint32_t)lidx[NP + 1][threadIdx.x] << 32) | (uint32_t)lidx[NP][threadIdx.x]);
            il = i0 + rrl;
            bidx = lidx[NP + 2][threadIdx.x] != 0;
        }

        {
            // B = L_N^{-T} v, v = row M of L (lane M % 2, local row M / 2).  Lane q ends with
            // bown[s] = B_{2s+q}.
            constexpr int SM = M / 2;
            constexpr bool VQ1 = (M % 2) == 1;  // row M sits in lane 1
            NNGP_PHASE(backsub);
            if constexpr (LEFT) {
                // the values are read only by the residual: gathered here (the row's indices again,
                // cache-warm), their latency behind the back-substitution, instead of holding NP
                // registers through the factorisation
#pragma unroll
                for (int s = 0; s < NP; ++s) {
                    const int a = 2 * s + q;
                    const int32_t j = a < M ? lidx[s][threadIdx.x] : -1;
                    const bool in_range = (uint32_t)j < n32;
                    const double* pv = a == M ? (qvalues != nullptr ? qvalues + il : kZeroValue)
                                              : ((values != nullptr && in_range) ? values + j : kZeroValue);
                    z[s] = *pv;
                }
            }
            double bown[NP];
#pragma unroll
            for (int s = 0; s < NP; ++s) bown[s] = 0.0;
            if (M % 2 == 1) bown[T] = RB(T, T, 1) * RB(T, T, 0);  // lane 0: B_{M-1} = L[M][M-1] / L[M-1][M-1]
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
                    acc0 = fma(RB(u, t, 0), bu, acc0);
                    acc1 = fma(RB(u, t, 1), bu, acc1);
                }
                const double tot = acc0 + pr_swap(acc1);  // sum_b L[b][2t+q] B_b
                // v_{2t+q}: row M's own-parity entry is slot [t][0] in lane M%2, slot [t][1] in the other
                const double vrow0 = RB(SM, t, 0), vrow1 = RB(SM, t, 1);
                double v;
                if (VQ1) {
                    v = pr_sel(q1, vrow0, pr_swap(vrow1));
                } else {
                    v = pr_sel(q1, pr_swap(vrow1), vrow0);
                }
                const double l10 = RB(t, t, 1);
                double bx, b0;
                if constexpr (SLDL) {  // unit factor: B_{2t+1} = v - tot, B_{2t} = v - tot - l10 B_{2t+1}
                    bx = v - tot;
                    b0 = fma(-l10, pr_swap(bx), bx);
                } else {
                    const double iown = RB(t, t, 0);
                    bx = (v - tot) * iown;                     // lane 1: B_{2t+1}
                    b0 = fma(-(l10 * iown), pr_swap(bx), bx);  // lane 0: B_{2t}
                }
                bown[t] = pr_sel(q1, bx, b0);
            }
            NNGP_PHASE(residual);
            {
                // r = v_i - B v_N (as the oracle states it): this lane's rows a = 2s + q < M, then the pair
                double acc = 0.0;
#pragma unroll
                for (int s = 0; s < NP; ++s) {
                    if (2 * s >= M) continue;
                    double bs = bown[s];
                    if (2 * s + 1 >= M) bs = q1 ? 0.0 : bs;  // lane 1's row here is row M (or padding)
                    acc = fma(bs, z[s], acc);
                }
                const double zm = z[SM];
                const double vi = VQ1 ? pr_from1(zm) : pr_from0(zm);
                res = vi - (acc + pr_swap(acc));
            }
            NNGP_PHASE(stores);
            if (Bout != nullptr && live) {
                // padded slots hold exact zeros (far-away points decouple exactly, nngp_math.h)
                const double bscale = (bad || stale_plan) ? NAN : 1.0;
#pragma unroll
                for (int s = 0; s < NP; ++s) {
                    const int a = 2 * s + q;
                    if (a < M) Bout[rrl * M + a] = bown[s] * bscale;
                }
            }
        }
        NNGP_PHASE(tail);
        const bool lead = live && lead0;
        if (Fout != nullptr && lead) Fout[rrl] = (bad || stale_plan) ? NAN : F;
        if (Rout != nullptr && lead) Rout[rrl] = (bad || stale_plan) ? NAN : res;
        // this lane's terms of the tile record (lead lanes; a NaN F -- a bad pivot -- propagates
        // into the mantissa product as log(NaN) would; the flag is what callers check)
        pairb_tile_store(lead ? __builtin_amdgcn_frexp_mant(F) : 1.0, lead ? __builtin_amdgcn_frexp_exp(F) : 0,
                         lead ? res * res * pr_rcp(F) : 0.0, (lead && bad) ? (double)il : INFINITY,
                         (live && bidx) ? (double)il : INFINITY, sh, 0, rec, lexp, tile);
        __syncthreads();
        if (threadIdx.x == 0) pairb_tile_fold(sh, 0, rec, lexp, tile);
    }
}

// workspace: a 256-B header (int64 tile count, written by the sweep and read by the fold; the second word,
// once the ticket of a fused fold -- measured and not kept, round 4 -- stays zero), the tile records (32 B
// each) and the tile exponent sums (4 B each), sized for pairb_tiles_bound(n_rows)
inline size_t pairb_align(size_t b) { return (b + 255) & ~(size_t)255; }
constexpr size_t kPairbHeader = 256;
inline size_t bf_pairb_workspace_bytes(int64_t n_rows) {
    const int64_t t = pairb_tiles_bound(n_rows);
    return t > 0 ? kPairbHeader + pairb_align((size_t)t * 32) + pairb_align((size_t)t * 4) : 0;
}
inline int64_t* pairb_hdr(void* ws) { return (int64_t*)ws; }
inline double4* pairb_rec(void* ws) { return (double4*)((char*)ws + kPairbHeader); }
inline int32_t* pairb_lexp(void* ws, int64_t n_rows) {
    return (int32_t*)((char*)ws + kPairbHeader + pairb_align((size_t)pairb_tiles_bound(n_rows) * 32));
}

// a.tiles != null: sweep only the listed tiles (a planned sweep's direct regions, pair_plan.h), a.n_tiles
// being the whole sweep's count; the records are then the caller's to fold
template <int M, int KIND, int D, bool PL = false>
static void launch_pairb_mkd(const BfArgs& a, const CovParams& Pc, hipStream_t s, const PairPlanArgs* ppl = nullptr) {
    const size_t lds = KIND == NNGP_KIND_MATERN ? NNGP_MT_BYTES(Pc.mt_noct) : 0;
    const PairbTiling tl = pairb_tiling(a.n_rows, M, KIND);
    PairPlanArgs pp = ppl != nullptr ? *ppl : PairPlanArgs{};
    if (!PL && a.tiles != nullptr) {
        pp.tiles = a.tiles;
        pp.n_tiles = a.n_tiles;
    }
    const int64_t nb = PL ? a.n_plan_blocks : (a.tiles != nullptr ? a.n_tile_list : tl.tiles);
    if (nb == 0) return;
    hipLaunchKernelGGL((bf_pairb<M, KIND, D, PL>), dim3((unsigned)nb), dim3(kPairbThreads), lds, s, a.coords,
                       a.n_points, a.nbr, a.order, a.n_rows, a.i0, Pc, KIND == NNGP_KIND_BLOCKS ? 1.0 : a.sigma2, a.values,
                       a.qcoords, a.qvalues, a.B, a.F, a.R, pairb_rec(a.bpart), pairb_lexp(a.bpart, a.n_rows), a.dim,
                       a.cblk, tl.q, tl.rem, pairb_hdr(a.bpart), pp);
}

// the planned regions of a planned sweep (pair_plan.h; the direct ones go through bf_pairb_launch with
// a.tiles = the direct list)
template <int M, int KIND, int D>
static void launch_pairb_planned_mkd(const BfArgs& a, const CovParams& Pc, const PlanLaunch& pl, hipStream_t s) {
    PairPlanArgs pp;
    pp.slots = pl.plan + kPlanGlobalHdr;
    pp.slot_bytes = pl.slot_bytes;
    pp.n_tiles = pl.n_regions;
    pp.tiles = pl.planned;
    BfArgs b = a;
    b.n_plan_blocks = pl.n_planned;
    launch_pairb_mkd<M, KIND, D, true>(b, Pc, s, &pp);
}

template <int M, int D>
static bool launch_pairb_planned_if(const BfArgs& a, const CovParams& Pc, const PlanLaunch& pl, hipStream_t s) {
    if (a.m != M || a.dim != D) return false;
    switch (a.kind) {
        case 0: launch_pairb_planned_mkd<M, 0, D>(a, Pc, pl, s); return true;
        case 1: launch_pairb_planned_mkd<M, 1, D>(a, Pc, pl, s); return true;
        case 2: launch_pairb_planned_mkd<M, 2, D>(a, Pc, pl, s); return true;
        case 3: launch_pairb_planned_mkd<M, 3, D>(a, Pc, pl, s); return true;
        case 4: launch_pairb_planned_mkd<M, 4, D>(a, Pc, pl, s); return true;
        default: return false;
    }
}

// m = 25..32: one instantiation per m for every kind and dimension (runtime kind NNGP_KIND_GENERIC,
// runtime dimension D = 0): these fully unrolled kernels take 0.5-2.5 min each to compile, and the
// extra work per covariance (the kind's polynomial, padded coordinates) is a few percent of theirs
template <int M>
static bool launch_pairb_generic_if(const BfArgs& a, const CovParams& Pc, hipStream_t s) {
    if (a.m != M) return false;
    launch_pairb_mkd<M, NNGP_KIND_GENERIC, 0>(a, Pc, s);
    return true;
}

// covariance blocks from memory (nngp_bf_sweep_blocks; instantiated by bf_pairb_inst_blocks_*.hip)
template <int M>
static bool launch_pairb_blocks_if(const BfArgs& a, const CovParams& Pc, hipStream_t s) {
    if (a.m != M) return false;
    launch_pairb_mkd<M, NNGP_KIND_BLOCKS, 2>(a, Pc, s);
    return true;
}

// one m and dimension, every kind (instantiated by the generated bf_pairb_inst_*.hip units)
template <int M, int D>
static bool launch_pairb_if(const BfArgs& a, const CovParams& Pc, hipStream_t s) {
    if (a.m != M || a.dim != D) return false;
    switch (a.kind) {
        case 0: launch_pairb_mkd<M, 0, D>(a, Pc, s); return true;
        case 1: launch_pairb_mkd<M, 1, D>(a, Pc, s); return true;
        case 2: launch_pairb_mkd<M, 2, D>(a, Pc, s); return true;
        case 3: launch_pairb_mkd<M, 3, D>(a, Pc, s); return true;
        case 4: launch_pairb_mkd<M, 4, D>(a, Pc, s); return true;
        case NNGP_KIND_MATERN:  // the table path (left-looking at m = 18); above m = 24 the four-lane kernel
            if constexpr (M <= 24) {
                launch_pairb_mkd<M, NNGP_KIND_MATERN, D>(a, Pc, s);
                return true;
            } else {
                return false;
            }
        default: return false;
    }
}

}  // namespace nngp
