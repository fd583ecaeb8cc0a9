// Gibbs-sampler kernels for the NNGP response model.
//
// Reference: pyNNGP's NNGP.oneSample (nngp.py:98-101) calls update_wt /
// update_ws / update_y_unobserved, none of which exist; the model and the
// updates here are those of the NNGP papers the reference's docstrings name
// (Datta et al. 2016): y = X beta + w + eps, eps ~ N(0, tau2 I),
// w ~ NNGP(0, C(sigma2, phi)) with precision Q = (I - B)^T F^{-1} (I - B).
//
// Full conditional of w_i (everything else fixed):
//   prec_i = 1/tau2 + 1/F_i + sum_{j in U(i)} B_{j,i}^2 / F_j
//   lin_i  = (y_i - x_i beta)/tau2 + (B_i w_N(i))/F_i
//            + sum_{j in U(i)} B_{j,i} (w_j - sum_{l in N(j), l != i} B_{j,l} w_l) / F_j
//   w_i ~ N(lin_i / prec_i, 1 / prec_i)
// with U(i) = {j : i in N(j)} (the reverse neighbour lists).  Keeping the NNGP
// residuals r_j = w_j - B_j w_N(j) current makes each term O(1):
//   B_i w_N(i) = w_i - r_i,   w_j - sum_{l != i} B_{j,l} w_l = r_j + B_{j,i} w_i,
// and after drawing w_i' the residuals of i and of its children move by
// dw = w_i' - w_i (r_i += dw, r_j -= B_{j,i} dw).
//
// Locations of one colour of the moral graph (edges i-N(i) and between
// co-parents of a common child) never read or write each other's w / r, so a
// colour is updated in parallel without races; colours run in sequence.  Normal
// draws come from a counter-based Philox4x32-10 keyed by (seed) with counter
// (location, sweep), so a chain is reproducible bit for bit.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <math.h>
#include <stdint.h>
#include <string.h>
#include <vector>

#include "nngp_internal.h"

namespace nngp {

// ---------------------------------------------------------------- Philox4x32-10
__host__ __device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)M0 * c[0];
        const uint64_t p1 = (uint64_t)M1 * c[2];
        const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0;
        const uint32_t h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
        const uint32_t n0 = h1 ^ c[1] ^ k0, n2 = h0 ^ c[3] ^ k1;
        c[0] = n0;
        c[1] = l1;
        c[2] = n2;
        c[3] = l0;
        k0 += W0;
        k1 += W1;
    }
}

// standard normal for (seed, location, sweep): Box-Muller on two 53-bit uniforms in (0, 1)
__host__ __device__ __forceinline__ double philox_normal(uint64_t seed, uint64_t loc, uint64_t sweep) {
    uint32_t c[4] = {(uint32_t)loc, (uint32_t)(loc >> 32), (uint32_t)sweep, (uint32_t)(sweep >> 32)};
    philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const uint64_t a = ((uint64_t)c[0] << 21) ^ (c[1] >> 11);
    const uint64_t b = ((uint64_t)c[2] << 21) ^ (c[3] >> 11);
    const double u1 = ((double)(a & ((1ull << 53) - 1)) + 0.5) * 0x1p-53;
    const double u2 = ((double)(b & ((1ull << 53) - 1)) + 0.5) * 0x1p-53;
    return sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
}

// n standard normals z[i] = philox_normal(seed, i, sweep): the same stream the w sweep draws
// inline when it gets no z, precomputed in one fully parallel pass so the colour kernels'
// critical path carries no Philox rounds / log / cos.
__global__ __launch_bounds__(256) void philox_normals_kernel(int64_t n, uint64_t seed, uint64_t sweep,
                                                             double* __restrict__ z) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) z[i] = philox_normal(seed, (uint64_t)i, sweep);
}

hipError_t philox_normals_launch(int64_t n, uint64_t seed, uint64_t sweep, double* z, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(philox_normals_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, seed, sweep, z);
    return hipGetLastError();
}

// ---------------------------------------------------------------- reverse neighbour lists
__global__ __launch_bounds__(256) void rev_keys(const int32_t* __restrict__ nbr, int64_t n_entries, int64_t n,
                                                uint32_t* __restrict__ key, int32_t* __restrict__ val) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n_entries) return;
    const int32_t i = nbr[e];
    key[e] = (i >= 0 && (int64_t)i < n) ? (uint32_t)i : (uint32_t)n;  // invalid slots sort last
    val[e] = (int32_t)e;
}

__global__ __launch_bounds__(256) void rev_bounds(const uint32_t* __restrict__ key_sorted, int64_t n_entries,
                                                  int64_t n, int32_t* __restrict__ off) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    int64_t lo = 0, hi = n_entries;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if ((int64_t)key_sorted[mid] < i)
            lo = mid + 1;
        else
            hi = mid;
    }
    off[i] = (int32_t)lo;
}

__global__ __launch_bounds__(256) void rev_split(const int32_t* __restrict__ val_sorted, int64_t n_valid, int m,
                                                 int32_t* __restrict__ rev_j, int32_t* __restrict__ rev_k) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n_valid) return;
    const int32_t v = val_sorted[e];
    rev_j[e] = v / m;
    rev_k[e] = v % m;
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

static size_t rev_sort_temp(int64_t e) {
    size_t tb = 0;
    if (rocprim::radix_sort_pairs((void*)nullptr, tb, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                  (const int32_t*)nullptr, (int32_t*)nullptr, (size_t)e, 0u, 32u) != hipSuccess)
        return 0;
    return tb;
}

size_t reverse_workspace_bytes(int64_t n, int m) {
    const int64_t e = n * m;
    if (e < 1) return 256;
    const size_t tb = rev_sort_temp(e);
    if (tb == 0) return 0;
    return 4 * align256((size_t)e * 4) + align256(tb);
}

hipError_t reverse_launch(const int32_t* nbr, int64_t n, int m, int32_t* off, int32_t* rev_j, int32_t* rev_k,
                          void* workspace, hipStream_t s) {
    const int64_t e = n * m;
    char* w = (char*)workspace;
    uint32_t* key = (uint32_t*)w;
    w += align256((size_t)e * 4);
    uint32_t* key_sorted = (uint32_t*)w;
    w += align256((size_t)e * 4);
    int32_t* val = (int32_t*)w;
    w += align256((size_t)e * 4);
    int32_t* val_sorted = (int32_t*)w;
    w += align256((size_t)e * 4);
    if (e == 0) {
        hipLaunchKernelGGL(rev_bounds, dim3((unsigned)((n + 1 + 255) / 256)), dim3(256), 0, s, key_sorted, (int64_t)0,
                           n, off);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(rev_keys, dim3((unsigned)((e + 255) / 256)), dim3(256), 0, s, nbr, e, n, key, val);
    size_t tb = rev_sort_temp(e);
    hipError_t er = rocprim::radix_sort_pairs((void*)w, tb, key, key_sorted, val, val_sorted, (size_t)e, 0u, 32u, s);
    if (er != hipSuccess) return er;
    hipLaunchKernelGGL(rev_bounds, dim3((unsigned)((n + 1 + 255) / 256)), dim3(256), 0, s, key_sorted, e, n, off);
    // entries [0, off[n]) are valid; split all e (the tail past off[n] is never read)
    hipLaunchKernelGGL(rev_split, dim3((unsigned)((e + 255) / 256)), dim3(256), 0, s, val_sorted, e, m, rev_j, rev_k);
    return hipGetLastError();
}

// ---------------------------------------------------------------- moral-graph colouring (host)
int64_t color_moral_graph_host(const int32_t* nbr, const int32_t* off, const int32_t* rev_j, int64_t n, int m,
                               int32_t* color) {
    std::vector<int64_t> stamp(1024, -1);
    int32_t n_colors = 0;
    for (int64_t i = 0; i < n; ++i) {
        // mark colours of already-coloured (index < i) moral neighbours: parents N(i), children j
        // (earlier than i only when the locations were relabelled, e.g. into a spatial storage
        // order) and co-parents of children
        auto mark = [&](int32_t k) {
            if (k >= 0 && k < i) {
                const int32_t c = color[k];
                if (c >= (int32_t)stamp.size()) stamp.resize((size_t)c * 2 + 1, -1);
                stamp[c] = i;
            }
        };
        const int32_t* row = nbr + i * m;
        for (int s = 0; s < m; ++s) mark(row[s]);
        for (int32_t e = off[i]; e < off[i + 1]; ++e) {
            const int64_t j = rev_j[e];
            mark((int32_t)j);
            const int32_t* rj = nbr + j * m;
            for (int s = 0; s < m; ++s)
                if (rj[s] != i) mark(rj[s]);
        }
        int32_t c = 0;
        while (c < (int32_t)stamp.size() && stamp[c] == i) ++c;
        color[i] = c;
        if (c + 1 > n_colors) n_colors = c + 1;
        if (n_colors >= (int32_t)stamp.size()) stamp.resize(stamp.size() * 2, -1);
    }
    return n_colors;
}

// ---------------------------------------------------------------- moral-graph colouring (device)
// The same greedy colouring as color_moral_graph_host -- node i takes the smallest colour no moral
// neighbour k < i holds -- computed in parallel rounds (Jones-Plassmann with the index as priority): in a
// round every uncoloured node whose lower moral neighbours are all coloured takes its colour.  A colour
// is final once written and a node reads its neighbours only when all are final, so the result is the
// sequential greedy's, whatever the timing (a stale "uncoloured" read -- another XCD's L2 -- only defers a
// node to a later round).  Rounds = the longest index-decreasing path of the moral graph (549 at
// N = 1e6, m = 15, measured on the host: tools note in DESIGN.md 4.5); a node scans its ~m + m^2 lower
// neighbours once, when it is coloured, and stops at the first uncoloured one before.  Up to 256 colours
// (a 256-bit mask); more sets *overflow and the caller colours on the host.
__global__ __launch_bounds__(256) void color_round_kernel(const int32_t* __restrict__ nbr, const int32_t* __restrict__ off,
                                                          const int32_t* __restrict__ rev_j, int64_t n, int m,
                                                          int32_t* color, unsigned long long* __restrict__ done,
                                                          int32_t* __restrict__ overflow, int32_t* __restrict__ maxc) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    // (colours are written by other workgroups of the same launch: relaxed agent-scope atomics make the
    // "final once written, read once" argument well defined -- no re-load or speculation of a plain load)
    if (__hip_atomic_load(&color[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= 0) return;
    uint64_t used[4] = {0, 0, 0, 0};
    // true when k is a lower neighbour that is still uncoloured (not ready); marks its colour otherwise
    auto lower = [&](int64_t k) -> bool {
        if (k < 0 || k >= i) return false;
        const int32_t c = __hip_atomic_load(&color[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (c < 0) return true;
        used[(c >> 6) & 3] |= c < 256 ? (1ull << (c & 63)) : 0ull;
        return false;
    };
    const int32_t* row = nbr + i * m;
    for (int s = 0; s < m; ++s)
        if (lower(row[s])) return;
    for (int32_t e = off[i]; e < off[i + 1]; ++e) {
        const int64_t j = rev_j[e];
        if (lower(j)) return;
        const int32_t* rj = nbr + j * m;
        for (int s = 0; s < m; ++s) {
            const int64_t k = rj[s];
            if (k != i && lower(k)) return;
        }
    }
    int c = 0;
    while (c < 256 && ((used[c >> 6] >> (c & 63)) & 1ull)) ++c;
    if (c >= 256) {
        *overflow = 1;
        return;
    }
    __hip_atomic_store(&color[i], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    atomicAdd(done, 1ull);
    atomicMax(maxc, c);
}

// colour -1 everywhere, the counters zero
__global__ __launch_bounds__(256) void color_init_kernel(int32_t* __restrict__ color, int64_t n,
                                                         unsigned long long* done, int32_t* overflow, int32_t* maxc) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) color[i] = -1;
    if (i == 0) {
        *done = 0ull;
        *overflow = 0;
        *maxc = -1;
    }
}

// rounds until every node is coloured (the host reads the count every kColorCheck rounds: one
// synchronisation per check, ~40 at N = 1e6); returns the number of colours, -1 on overflow (more than
// 256 colours: colour on the host), -2 on a HIP error (*err)
int64_t color_moral_graph_device(const int32_t* nbr, const int32_t* off, const int32_t* rev_j, int64_t n, int m,
                                 int32_t* color, void* workspace, hipStream_t s, hipError_t* err) {
    constexpr int kColorCheck = 16;
    unsigned long long* done = (unsigned long long*)workspace;
    int32_t* overflow = (int32_t*)((char*)workspace + 8);
    int32_t* maxc = (int32_t*)((char*)workspace + 12);
    *err = hipSuccess;
    if (n == 0) return 0;
    const dim3 grid((unsigned)((n + 255) / 256));
    hipLaunchKernelGGL(color_init_kernel, grid, dim3(256), 0, s, color, n, done, overflow, maxc);
    struct {
        unsigned long long done;
        int32_t overflow, maxc;
    } h{0, 0, -1};
    // (a round colours at least the lowest uncoloured node: n rounds always suffice)
    for (int64_t round = 0; round <= n; round += kColorCheck) {
        for (int k = 0; k < kColorCheck; ++k)
            hipLaunchKernelGGL(color_round_kernel, grid, dim3(256), 0, s, nbr, off, rev_j, n, m, color, done, overflow,
                               maxc);
        if ((*err = hipGetLastError()) != hipSuccess) return -2;
        if ((*err = hipMemcpyAsync(&h, workspace, 16, hipMemcpyDeviceToHost, s)) != hipSuccess) return -2;
        if ((*err = hipStreamSynchronize(s)) != hipSuccess) return -2;
        if (h.overflow) return -1;
        if ((int64_t)h.done >= n) break;
    }
    return (int64_t)h.maxc + 1;
}

// ---------------------------------------------------------------- per-phi preparation
// Everything of the w full conditionals that depends on B / F only (i.e. changes only
// when a new phi is accepted) is folded once into reverse-list order:
//   Brev[e] = B_{j,i},  Grev[e] = B_{j,i} / F_j   (e in [off[i], off[i+1]), j = rev_j[e])
//   P[i]    = sum_e B_{j,i}^2 / F_j,  invF[i] = 1 / F_i
// so that, with s2 = sigma2 (F here is the unit-variance field's),
//   prec_i = 1/tau2 + (invF_i + P_i) / s2
//   lin_i  = yres_i / tau2 + [(w_i - r_i) invF_i + w_i P_i + sum_e Grev[e] r_j] / s2
// and a colour step reads one streamed double and one gathered r_j per child.
// Workgroups are dealt round-robin over the 8 XCDs (private L2s): xcd_logical_block gives
// each XCD a contiguous chunk of the grid, so spatially adjacent locations (sharing
// children and reverse-list lines) meet in one L2 (speed only; -4 % per Gibbs iteration).
// The colour kernel gives kGroup lanes to a location: the lanes split its children, a
// fixed xor-butterfly sums their terms.  32 measured best for m = 15 (~15 children per
// location): 8 lanes 1.30, 16 lanes 1.07, 32 lanes 1.05 ms per Gibbs iteration at
// N = 1e6 -- the colour steps are latency bound.
#define NNGP_GIBBS_GROUP 32
// ... each lane holding NNGP_GIBBS_PER children with their loads in flight together.  Fewer lanes
// per member with more children each (fewer waves, no second round trip for the members with more
// children than lanes) measured slower (round 3, profiles/r03s, ms per iteration at N = 1e6):
// 32 x 1 0.799, 32 x 2 0.801, 16 x 2 0.859, 8 x 4 1.012 -- the steps want every gather in its own
// lane (memory-level parallelism), not fewer waves.
#define NNGP_GIBBS_PER 1
constexpr int kGroup = NNGP_GIBBS_GROUP;
constexpr int kPer = NNGP_GIBBS_PER;
constexpr int kSpan = kGroup * kPer;

// Sum over the G lanes of an aligned group, in every lane the bits of the ASCENDING xor butterfly
// (distances 1, 2, 4, ...; the round-2 kernel summed descending, so its sums differ in the last
// bits): after the steps of distance 1 and 2 all lanes of a quad hold the same value, so a partner in the
// other half of the 8- (16-) lane group may be taken by the DPP half-row (row) mirror, l ^ 7
// (l ^ 15), instead of l ^ 4 (l ^ 8) -- the same two operands in the same order.  The quad steps and
// the mirrors are DPP moves on the VALU; l ^ 16 is one ds_swizzle (bit mode) and l ^ 32 a
// ds_bpermute: one LDS round trip instead of five.
// (the descending __shfl_xor butterfly, a ds_bpermute per step, was the A/B baseline)
template <int CTRL>
__device__ __forceinline__ double gdpp(double v) {
    const long long u = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(u & 0xffffffffll), CTRL, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(u >> 32), CTRL, 0xf, 0xf, true);
    return __hiloint2double(hi, lo);
}
template <int G>
__device__ __forceinline__ double group_sum(double v) {
    static_assert(G == 1 || G == 2 || G == 4 || G == 8 || G == 16 || G == 32 || G == 64, "group of 2^k <= 64 lanes");
    if constexpr (G >= 2) v += gdpp<0xB1>(v);   // quad_perm [1,0,3,2]: l ^ 1
    if constexpr (G >= 4) v += gdpp<0x4E>(v);   // quad_perm [2,3,0,1]: l ^ 2
    if constexpr (G >= 8) v += gdpp<0x141>(v);  // row_half_mirror: l ^ 7
    if constexpr (G >= 16) v += gdpp<0x140>(v); // row_mirror: l ^ 15
    if constexpr (G >= 32) {                    // ds_swizzle bit mode, and 0x1f, xor 0x10: l ^ 16
        const long long u = __double_as_longlong(v);
        const int lo = __builtin_amdgcn_ds_swizzle((int)(u & 0xffffffffll), 0x401F);
        const int hi = __builtin_amdgcn_ds_swizzle((int)(u >> 32), 0x401F);
        v += __hiloint2double(hi, lo);
    }
    if constexpr (G >= 64) v += __shfl_xor(v, 32);
    return v;
}

// Two passes, both streaming:
//   entries: one thread per reverse entry e: Brev[e] = B[j, k], Grev[e] = Brev[e] / Ft[j]
//            (coalesced rev_j / rev_k reads and Brev / Grev writes, B / Ft gathered from
//            rows near j's parents in the storage order);
//   rows:    kRowLanes lanes per location fold P_i over its contiguous reverse range
//            (fixed order: lane-strided partial sums + a fixed xor-butterfly), 1 / Ft_i.
// 0.183 ms per prepared phi at N = 1e6, m = 15 (tools/bench_prepare.py).  Measured and rejected
// (round 3, profiles/r03k): one fused pass (L lanes per location, U entries per lane
// in flight, P_i folded without re-reading Brev / Grev) at L x U = 4 x 4 / 8 x 2 / 16 x 1 / 16 x 2:
// 0.216 / 0.181 / 0.196 / 0.233 ms; the first version, kGroup lanes per location with one entry
// each in flight, took 267 us.
constexpr int kRowLanes = 4;

// Both passes cover the rows [row0, row1) -- the whole field, or the shard a rank of a sharded
// chain owns (nngp_gibbs_prepare_range): the entries pass walks the contiguous reverse entries
// [off[row0], off[row1]) grid-stride (their count is only known on the device).
__global__ __launch_bounds__(256) void gibbs_prepare_entries(const double* __restrict__ B,
                                                             const double* __restrict__ Ft,
                                                             const int32_t* __restrict__ rev_j,
                                                             const int32_t* __restrict__ rev_k,
                                                             const int32_t* __restrict__ off, int64_t row0,
                                                             int64_t row1, int m, double* __restrict__ Brev,
                                                             double* __restrict__ Grev) {
    const int64_t e1 = off[row1];
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = off[row0] + xcd_logical_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x; e < e1;
         e += stride) {
        const int64_t j = rev_j[e];
        const double b = B[j * m + rev_k[e]];
        Brev[e] = b;
        Grev[e] = b / Ft[j];
    }
}

__global__ __launch_bounds__(256) void gibbs_prepare_rows(const double* __restrict__ Ft,
                                                          const int32_t* __restrict__ off, int64_t row0, int64_t row1,
                                                          const double* __restrict__ Brev,
                                                          const double* __restrict__ Grev, double* __restrict__ P,
                                                          double* __restrict__ invF) {
    const int64_t t = xcd_logical_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
    const int64_t i = row0 + t / kRowLanes;
    const int l = (int)(t % kRowLanes);
    const bool live = i < row1;
    const int64_t ic = live ? i : row1 - 1;
    const int32_t e0 = off[ic], e1 = live ? off[ic + 1] : e0;
    double acc = 0.0;
    for (int32_t e = e0 + l; e < e1; e += kRowLanes) acc = fma(Brev[e], Grev[e], acc);
#pragma unroll
    for (int o = kRowLanes / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (live && l == 0) {
        P[i] = acc;
        invF[i] = 1.0 / Ft[i];
    }
}


struct GibbsPrep {
    double *Brev, *Grev, *P, *invF;
};

static GibbsPrep prep_layout(void* prep, int64_t n, int m) {
    char* w = (char*)prep;
    GibbsPrep g;
    g.Brev = (double*)w;
    w += align256((size_t)(n * m) * 8);
    g.Grev = (double*)w;
    w += align256((size_t)(n * m) * 8);
    g.P = (double*)w;
    w += align256((size_t)n * 8);
    g.invF = (double*)w;
    return g;
}

size_t gibbs_prep_bytes(int64_t n, int m) {
    return 2 * align256((size_t)(n * m) * 8) + 2 * align256((size_t)n * 8);
}

hipError_t gibbs_prepare_range_launch(const double* B, const double* Ft, const int32_t* off, const int32_t* rev_j,
                                      const int32_t* rev_k, int64_t n, int m, int64_t row0, int64_t row1, void* prep,
                                      hipStream_t s) {
    if (row1 <= row0) return hipSuccess;
    const GibbsPrep g = prep_layout(prep, n, m);
    const int64_t rows = row1 - row0;
    // grid sized for m reverse entries per row (the average); the stride loop takes the rest
    const int64_t ne = rows * (int64_t)m;
    if (ne > 0)
        hipLaunchKernelGGL(gibbs_prepare_entries, dim3((unsigned)((ne + 255) / 256)), dim3(256), 0, s, B, Ft, rev_j,
                           rev_k, off, row0, row1, m, g.Brev, g.Grev);
    hipLaunchKernelGGL(gibbs_prepare_rows, dim3((unsigned)((rows * kRowLanes + 255) / 256)), dim3(256), 0, s, Ft, off,
                       row0, row1, g.Brev, g.Grev, g.P, g.invF);
    return hipGetLastError();
}

hipError_t gibbs_prepare_launch(const double* B, const double* Ft, const int32_t* off, const int32_t* rev_j,
                                const int32_t* rev_k, const int32_t* order, int64_t n, int m, void* prep,
                                hipStream_t s) {
    (void)order;  // both passes stream the reverse lists in storage order; no visiting order needed
    return gibbs_prepare_range_launch(B, Ft, off, rev_j, rev_k, n, m, 0, n, prep, s);
}

// ---------------------------------------------------------------- colour update
// Member rows (nngp_gibbs_member_rows): per colour-ordered member g the int4 (location i, first and
// end reverse entry, 0), so a colour step starts with one coalesced 16-B load per member instead of
// members[g] and then off[i], off[i + 1] -- one dependent memory round trip less per member.
__global__ __launch_bounds__(256) void gibbs_member_rows_kernel(const int32_t* __restrict__ members, int64_t n,
                                                                const int32_t* __restrict__ off,
                                                                int4* __restrict__ rows) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n) return;
    const int32_t i = members[g];
    rows[g] = make_int4(i, off[i], off[i + 1], 0);
}

hipError_t gibbs_member_rows_launch(const int32_t* members, int64_t n, const int32_t* off, int32_t* rows,
                                    hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(gibbs_member_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, members, n, off,
                       (int4*)rows);
    return hipGetLastError();
}

// kGroup lanes per location: the lanes split its children (reverse entries), a
// fixed xor-butterfly sums their sum_e Grev[e] r_j, and every lane of the group then
// evaluates the same full conditional and the same Philox normal (no broadcast
// needed; lane 0 writes w_i, r_i), and the lanes scatter r_j -= B_{j,i} dw to their
// children.  Race-free within a colour (moral-graph colouring: no two members share a
// child, and no member is another's child).

// INLINE_Z: the normals are drawn inside the step (z == nullptr: Philox rounds, log and cos on the
// critical path); otherwise read from z.  Two instantiations because a kernel's VGPR allocation is
// static: the inline-Philox code held the z-given kernel -- the one every sampler runs -- at 70 VGPRs,
// 7 waves per SIMD; without it 46 VGPRs, the 8-wave cap (round 4, profiles/r04l: 0.8022 -> 0.7885 ms per
// Gibbs iteration at N = 1e6, median of 4 interleaved runs; the 8-wave cap binds, so asking the compiler
// for more waves per SIMD changes nothing).
// (Measured and not kept, round 6, profiles/r06e: the per-iteration streams of a colour step -- member rows,
// the reverse entries, P, 1 / F, y - X beta, the normals -- read non-temporally, to keep r in the XCDs' L2s:
// 0.829 against 0.792 ms per iteration, the colour kernel's L2 fetch unchanged at ~44 MB per launch.)
template <bool INLINE_Z>
__global__ __launch_bounds__(256) void gibbs_w_color(const int4* __restrict__ member_rows, int64_t n_members,
                                                     const double* __restrict__ Brev, const double* __restrict__ Grev,
                                                     const double* __restrict__ P, const double* __restrict__ invF,
                                                     double it2, double is2, const double* __restrict__ yres,
                                                     const double* __restrict__ noise_w,
                                                     double* __restrict__ w, double* __restrict__ r,
                                                     const int32_t* __restrict__ rev_j,
                                                     const double* __restrict__ z, uint64_t seed, uint64_t sweep,
                                                     double* __restrict__ w_out, const double* __restrict__ var,
                                                     int64_t m_cap) {
    const int64_t t = xcd_logical_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
    const int64_t g = t / kGroup;
    const int l = (int)(t % kGroup);
    const bool live = g < n_members;
    const int4 mr = member_rows[live ? g : n_members - 1];
    const int64_t i = mr.x;
    const int32_t e0 = mr.y, e1 = live ? mr.z : mr.y;
    // every load that depends only on the member row is issued at once, branch-free: the
    // member's own operands and its first child's reverse entry in one memory round trip, then
    // the child's r_j in a second (a guarded load per operand made the compiler wait for each
    // before issuing the next).  r_i is safe to read early: no other member of the colour is a
    // parent of i, so nothing else writes it during the step.
    const double wi = w[i], ri = r[i], iF = invF[i], Pi = P[i], yi = yres[i];
    const double hi = noise_w != nullptr ? noise_w[i] : 1.0;
    const double zl = z != nullptr ? z[i] : 0.0;
    if (var != nullptr) {  // (sigma2, tau2) from device memory: a graph-captured step replays with new values
        is2 = 1.0 / var[0];
        it2 = 1.0 / var[1];
    }
    // the first kSpan = kGroup * kPer children in registers (child index, B, r_j), kPer per lane
    // (children l, l + kGroup, ...), their loads issued together: the scatter below reuses them
    // without reloading (no other member of this colour touches r_j); more children (rare) take
    // the generic loops.  A slot without a child reads entry 0 (in the n*m-entry reverse arrays
    // whenever m > 0) and r_i, and discards them.
    int64_t jf[kPer];
    double bf[kPer], gf[kPer], rf[kPer];
    bool has[kPer];
#pragma unroll
    for (int c = 0; c < kPer; ++c) {
        const int32_t ef = e0 + l + c * kGroup;
        has[c] = ef < e1;
        const int64_t es = has[c] ? ef : 0;
        jf[c] = i;
        bf[c] = 0.0;
        gf[c] = 0.0;
        if (m_cap > 0) {  // kernel argument: wave-uniform
            const int32_t jr = rev_j[es];
            bf[c] = Brev[es];
            gf[c] = Grev[es];
            jf[c] = has[c] ? (int64_t)jr : i;
        }
    }
#pragma unroll
    for (int c = 0; c < kPer; ++c) rf[c] = r[jf[c]];
    double acc = 0.0;
#pragma unroll
    for (int c = 0; c < kPer; ++c) {
        rf[c] = has[c] ? rf[c] : 0.0;
        bf[c] = has[c] ? bf[c] : 0.0;
        acc = c == 0 ? (has[0] ? gf[0] * rf[0] : 0.0) : (has[c] ? fma(gf[c], rf[c], acc) : acc);
    }
    for (int32_t e = e0 + l + kSpan; e < e1; e += kGroup) acc = fma(Grev[e], r[rev_j[e]], acc);
    acc = group_sum<kGroup>(acc);
    const double it2i = noise_w != nullptr ? it2 * hi : it2;  // 1 / (tau2 / h_i)
    const double prec = fma(iF + Pi, is2, it2i);
    const double lin = fma(yi, it2i, is2 * fma(wi - ri, iF, fma(wi, Pi, acc)));
    double zi = zl;
    if constexpr (INLINE_Z) zi = philox_normal(seed, (uint64_t)i, sweep);
    const double sd = nngp_rsqrt(prec);
    const double wn = fma(zi, sd, lin / prec);
    const double dw = wn - wi;
    if (live && l == 0) {
        w[i] = wn;
        r[i] = ri + dw;
        if (w_out != nullptr) w_out[g] = wn;  // published to the other ranks of a sharded chain
    }
#pragma unroll
    for (int c = 0; c < kPer; ++c)
        if (has[c]) r[jf[c]] = fma(-bf[c], dw, rf[c]);
    for (int32_t e = e0 + l + kSpan; e < e1; e += kGroup) {
        const int64_t j = rev_j[e];
        r[j] = fma(-Brev[e], dw, r[j]);
    }
}

hipError_t gibbs_w_sweep_launch(const int32_t* member_rows, int n_colors, const int32_t* color_off_host,
                                const void* prep, int64_t n, int m, double sigma2, double tau2,
                                const double* yres, const double* noise_w, double* w, double* r,
                                const int32_t* rev_j, const double* z, uint64_t seed, uint64_t sweep, hipStream_t s) {
    const GibbsPrep g = prep_layout((void*)prep, n, m);
    for (int c = 0; c < n_colors; ++c) {
        const int64_t a = color_off_host[c], b = color_off_host[c + 1];
        if (b <= a) continue;
        const int64_t threads = (b - a) * kGroup;
        hipLaunchKernelGGL(z != nullptr ? gibbs_w_color<false> : gibbs_w_color<true>,
                           dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s,
                           (const int4*)member_rows + a, b - a, g.Brev, g.Grev, g.P, g.invF, 1.0 / tau2, 1.0 / sigma2,
                           yres, noise_w, w, r, rev_j, z, seed, sweep, nullptr, nullptr, n * (int64_t)m);
    }
    return hipGetLastError();
}

hipError_t gibbs_w_color_launch(const int32_t* member_rows, int64_t n_members, const void* prep, int64_t n, int m,
                                double sigma2, double tau2, const double* yres, const double* noise_w, double* w,
                                double* r, const int32_t* rev_j, const double* z, uint64_t seed, uint64_t sweep,
                                double* w_out, const double* var, hipStream_t s) {
    if (n_members <= 0) return hipSuccess;
    const GibbsPrep g = prep_layout((void*)prep, n, m);
    const int64_t threads = n_members * kGroup;
    hipLaunchKernelGGL(z != nullptr ? gibbs_w_color<false> : gibbs_w_color<true>,
                       dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s,
                       (const int4*)member_rows, n_members, g.Brev, g.Grev, g.P, g.invF, 1.0 / tau2, 1.0 / sigma2, yres,
                       noise_w, w, r, rev_j, z, seed, sweep, w_out, var, n * (int64_t)m);
    return hipGetLastError();
}

// ---------------------------------------------------------------- tiled colour sweep (round 6)
// pynngp_amd/gibbs_tiles.py builds the plan: spatial tiles whose footprints (each node and its children --
// the r entries its update reads and writes) are disjoint within a launch.  One workgroup per tile holds
// the footprint's r and the tile's new w in LDS, runs every colour of its nodes in order and writes r and
// w back: the residuals cross HBM once per launch instead of once per colour.  The plan is contiguous
// (SeqNNGP stores the nodes in its order): tile t's nodes are storage rows [n0, n1), colour-rank groups in
// order, so the members of a step (<= 64 of one colour) and their reverse entries are contiguous ranges.
// A step's operands -- per member 1 / F, P, y - X beta, the normal, w (and h), per reverse entry B, B / F
// and the child's local index -- are loaded by the whole block (coalesced, a few entries a thread) two
// steps ahead into registers and written to one of two LDS step buffers after the current step: the
// global latency is hidden behind two steps, and a member's children are read from LDS however many
// there are.  A block barrier ends every step (the next buffer is ready; a colour's r updates are seen by
// the next colour).  Per member the arithmetic is gibbs_w_color's (the same conditional; its 16-lane sum
// of the children's terms is a fixed butterfly of its own order).  A step costs ~1.45 us even without its
// global loads (a timing probe, tools/variants/tile_noload.patch, profiles/r06i): a tile's ~30-60 steps in
// series outlast a colour launch's ~15 us per colour over the whole field, so this sweep is opt-in
// (DESIGN.md 4.5).  (Measured and not kept: 4 lanes per member in 256-thread blocks, 2.2x slower per step --
// a member's children then cost a chain of dependent LDS reads per lane, profiles/r06j.)
constexpr int kTileThreads = 1024;
constexpr int kTileLanes = 16;                         // lanes per member
constexpr int kTileSlots = kTileThreads / kTileLanes;  // members per step (at most)
constexpr int kTileEQ = 2;                             // staged entries per thread: a step holds <= 2048
constexpr int kTileMem = 6;                            // staged values per member
constexpr int kTileMQ = (kTileMem * kTileSlots + kTileThreads - 1) / kTileThreads;  // member values a thread

struct TileRegs {
    double mv[kTileMQ];
    double g[kTileEQ], b[kTileEQ];
    int32_t loc[kTileEQ];
};

__global__ __launch_bounds__(kTileThreads) void gibbs_tile_phase(
    const int32_t* __restrict__ tiles, const int4* __restrict__ tinfo, const int32_t* __restrict__ tstep, int ecap,
    int64_t n_entries, const int32_t* __restrict__ tfp, const int32_t* __restrict__ off,
    const int32_t* __restrict__ rev_loc, const double* __restrict__ Brev, const double* __restrict__ Grev,
    const double* __restrict__ P, const double* __restrict__ invF, const double* __restrict__ yres,
    const double* __restrict__ noise_w, const double* __restrict__ z, double it2, double is2,
    double* __restrict__ w, double* __restrict__ r) {
    extern __shared__ double tile_lds[];
    const int tile = tiles[blockIdx.x];
    const int4 ta = tinfo[2 * tile], tb = tinfo[2 * tile + 1];  // rows [n0, n1), footprint, steps
    const int n0 = ta.x, nn = ta.y - ta.x, nf = ta.w - ta.z, S = tb.y - tb.x;
    const int ecp = ecap + 1;                          // + a dummy slot (unconditional staging writes)
    const int bufd = kTileMem * kTileSlots + 1 + 2 * ecp;  // doubles per step buffer
    double* const rl = tile_lds;                         // footprint r (its first nn: the tile's rows)
    double* const wl = rl + nf;                          // the tile's new w
    double* const bufs = wl + nn;                        // 2 step buffers: member values, B / F, B
    int32_t* const locs = (int32_t*)(bufs + 2 * bufd);  // 2 x (ecap + 1) local indices
    int32_t* const eo = locs + 2 * ecp;                  // nn + 1 reverse-entry offsets off[n0 + k]
    int32_t* const sk = eo + nn + 1;                     // S + 1 step starts (tile-local rows)
    const int tid = (int)threadIdx.x;
    for (int f = tid; f < nf; f += kTileThreads) rl[f] = r[tfp[ta.z + f]];
    for (int k = tid; k <= nn; k += kTileThreads) eo[k] = off[n0 + k];
    for (int q = tid; q <= S; q += kTileThreads) sk[q] = q < S ? tstep[tb.x + q] : nn;
    __syncthreads();
    // the member values this thread stages: value v = tid + 256 q is field v / 64 of member v % 64 (past
    // the 384 values: a harmless copy of the last field)
    const double* msrc[kTileMQ];
#pragma unroll
    for (int q = 0; q < kTileMQ; ++q) {
        const int mf = min((tid + kTileThreads * q) / kTileSlots, kTileMem - 1);
        msrc[q] = mf == 0 ? invF : mf == 1 ? P : mf == 2 ? yres : mf == 3 ? z : mf == 4 ? w
                : (noise_w != nullptr ? noise_w : invF);
    }
    const int mj = tid % kTileSlots;
    const int64_t ecl = n_entries > 0 ? n_entries - 1 : 0;
    // Every load is unconditional (indices clamped into range; past the last step the last step reloads,
    // unused): with no branch around them the compiler's counted waits stay exact -- a conditional load
    // made it wait for every outstanding load (vmcnt(0)) before staging the previous step, serialising the
    // pipeline (1.8 us per step, profiles/r06h).
    auto load = [&](int s, TileRegs& R) {
        const int sc = min(s, S - 1);
        const int ka = sk[sc], kb = sk[sc + 1];
        const int k = min(ka + mj, kb - 1);
#pragma unroll
        for (int q = 0; q < kTileMQ; ++q) R.mv[q] = msrc[q][n0 + k];
        const int ea = eo[ka], ne = eo[kb] - ea;
#pragma unroll
        for (int q = 0; q < kTileEQ; ++q) {
            const int x = tid + kTileThreads * q;
            const int64_t e = min((int64_t)ea + min(x, max(ne - 1, 0)), ecl);
            R.g[q] = Grev[e];
            R.b[q] = Brev[e];
            R.loc[q] = rev_loc[e];
        }
    };
    // into step buffer s & 1; unconditional too (what is not staged goes to the dummy slot), so that no
    // branch leaves a staged register "maybe pending" for the compiler's waits
    auto store = [&](int s, const TileRegs& R) {
        const int sc = max(0, min(s, S - 1));  // (before the first / past the last step: a buffer not read)
        double* const mem = bufs + (s & 1) * bufd;
        double* const G = mem + kTileMem * kTileSlots + 1;
        double* const Bb = G + ecp;
        int32_t* const L = locs + (s & 1) * ecp;
        const int ka = sk[sc], kb = sk[sc + 1];
#pragma unroll
        for (int q = 0; q < kTileMQ; ++q) {
            const int v = tid + kTileThreads * q;
            mem[v < kTileMem * kTileSlots && ka + mj < kb ? v : kTileMem * kTileSlots] = R.mv[q];
        }
        const int ne = eo[kb] - eo[ka];
#pragma unroll
        for (int q = 0; q < kTileEQ; ++q) {
            const int x = tid + kTileThreads * q;
            const int xs = x < ne ? x : ecap;
            G[xs] = R.g[q];
            Bb[xs] = R.b[q];
            L[xs] = R.loc[q];
        }
    };
    const int j = tid / kTileLanes, l = tid % kTileLanes;
    auto compute = [&](int s) {
        const double* const mem = bufs + (s & 1) * bufd;
        const double* const G = mem + kTileMem * kTileSlots + 1;
        const double* const Bb = G + ecp;
        const int32_t* const L = locs + (s & 1) * ecp;
        const int ka = sk[s], kb = sk[s + 1];
        const int k = ka + j;
        if (k >= kb) {
            (void)group_sum<kTileLanes>(0.0);  // (the butterfly is lane-collective: every lane joins)
            return;
        }
        const int ea = eo[ka], e0 = eo[k] - ea, e1 = eo[k + 1] - ea;
        double acc = 0.0;
        for (int x = e0 + l; x < e1; x += kTileLanes) acc = fma(G[x], rl[L[x]], acc);
        acc = group_sum<kTileLanes>(acc);
        const double iF = mem[j], Pi = mem[kTileSlots + j], yi = mem[2 * kTileSlots + j];
        const double zi = mem[3 * kTileSlots + j], wi = mem[4 * kTileSlots + j];
        const double ri = rl[k];
        const double it2i = noise_w != nullptr ? it2 * mem[5 * kTileSlots + j] : it2;
        const double prec = fma(iF + Pi, is2, it2i);
        const double lin = fma(yi, it2i, is2 * fma(wi - ri, iF, fma(wi, Pi, acc)));
        const double sd = nngp_rsqrt(prec);
        const double wn = fma(zi, sd, lin / prec);
        const double dw = wn - wi;
        if (l == 0) {
            wl[k] = wn;
            rl[k] = ri + dw;
        }
        for (int x = e0 + l; x < e1; x += kTileLanes) rl[L[x]] = fma(-Bb[x], dw, rl[L[x]]);
    };
    // two register sets: step s + 2 loads while step s computes; step s + 1 (loaded during step s - 1) is
    // written to its buffer after step s, before the barrier that ends it.  The loop starts two steps early
    // (no compute) so that every load and staging write sits in the loop body: a separate prologue gave the
    // loop head a merged "maybe pending" register state and early waits.
    TileRegs Ra = {}, Rb = {};
    for (int s = -2; s < S; s += 2) {
        load(s + 2, Ra);
        if (s >= 0) compute(s);
        store(s + 1, Rb);
        __syncthreads();
        if (s + 1 >= S) break;
        load(s + 3, Rb);
        if (s + 1 >= 0) compute(s + 1);
        store(s + 2, Ra);
        __syncthreads();
    }
    for (int f = tid; f < nf; f += kTileThreads) r[tfp[ta.z + f]] = rl[f];
    for (int k = tid; k < nn; k += kTileThreads) w[n0 + k] = wl[k];
}

hipError_t gibbs_tile_sweep_launch(const int32_t* tiles, const int32_t* phase_off_host, const int32_t* phase_lds_host,
                                   int n_phases, const int32_t* tinfo, const int32_t* tstep, int ecap,
                                   const int32_t* tfp, const int32_t* off, const int32_t* rev_loc, const void* prep,
                                   int64_t n, int m, int64_t n_entries, double sigma2, double tau2,
                                   const double* yres, const double* noise_w, double* w, double* r, const double* z,
                                   hipStream_t s) {
    const GibbsPrep g = prep_layout((void*)prep, n, m);
    // no reverse entries (m = 0, or no node has a child): the kernel's clamped entry loads read index 0 of
    // arrays that exist (their values are never staged)
    const double* Brev = n_entries > 0 ? g.Brev : g.P;
    const double* Grev = n_entries > 0 ? g.Grev : g.P;
    const int32_t* rloc = n_entries > 0 ? rev_loc : off;
    for (int p = 0; p < n_phases; ++p) {
        const int nt = phase_off_host[p + 1] - phase_off_host[p];
        if (nt <= 0) continue;
        hipLaunchKernelGGL(gibbs_tile_phase, dim3((unsigned)nt), dim3(kTileThreads), (size_t)phase_lds_host[p], s,
                           tiles + phase_off_host[p], (const int4*)tinfo, tstep, ecap, n_entries, tfp, off, rloc,
                           Brev, Grev, g.P, g.invF, yres, noise_w, z, 1.0 / tau2, 1.0 / sigma2, w, r);
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------- several chains, one launch per colour
// C independent chains of the same field (the same DAG, colouring and member rows; each chain its own
// B / F -- its own phi --, w, r, y - X beta, sigma2, tau2 and normals) advanced by ONE launch per colour
// (nngp_gibbs_w_sweep_chains): a colour step's fixed cost (the launch and its dependent member-row /
// reverse-entry round trips, ~5 us of the ~16 us per colour at N = 1e6) is paid once for all chains, the
// member rows and child indices are read once, and each thread has C independent gathers in flight.
// Per chain the arithmetic is gibbs_w_color's, operation for operation, so chain c's draws are
// bit-identical to running it alone.
constexpr int kMaxChains = 8;
struct ChainPtrs {
    const double* Brev[kMaxChains];
    const double* Grev[kMaxChains];
    const double* P[kMaxChains];
    const double* invF[kMaxChains];
    const double* yres[kMaxChains];
    const double* z[kMaxChains];
    double* w[kMaxChains];
    double* r[kMaxChains];
    double* wil;  // gibbs_w_color_chains_il: w and r interleaved, (n, C) row-major (chain c of location i at [i C + c])
    double* ril;
    double it2[kMaxChains], is2[kMaxChains];
};

template <int C>
__global__ __launch_bounds__(256) void gibbs_w_color_chains(const int4* __restrict__ member_rows, int64_t n_members,
                                                            const ChainPtrs cp, const double* __restrict__ noise_w,
                                                            const int32_t* __restrict__ rev_j, int64_t m_cap) {
#define CW(c, idx) cp.w[c][idx]
#define CR(c, idx) cp.r[c][idx]
    const int64_t t = xcd_logical_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
    const int64_t g = t / kGroup;
    const int l = (int)(t % kGroup);
    const bool live = g < n_members;
    const int4 mr = member_rows[live ? g : n_members - 1];
    const int64_t i = mr.x;
    const int32_t e0 = mr.y, e1 = live ? mr.z : mr.y;
    const double hi = noise_w != nullptr ? noise_w[i] : 1.0;
    double wi[C], ri[C], iF[C], Pi[C], yi[C], zl[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
        wi[c] = CW(c, i);
        ri[c] = CR(c, i);
        iF[c] = cp.invF[c][i];
        Pi[c] = cp.P[c][i];
        yi[c] = cp.yres[c][i];
        zl[c] = cp.z[c][i];
    }
    int64_t jf[kPer];
    bool has[kPer];
    double bf[C][kPer], gf[C][kPer], rf[C][kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int32_t ef = e0 + l + k * kGroup;
        has[k] = ef < e1;
        const int64_t es = has[k] ? ef : 0;
        jf[k] = i;
        int32_t jr = 0;
        if (m_cap > 0) jr = rev_j[es];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            bf[c][k] = 0.0;
            gf[c][k] = 0.0;
            if (m_cap > 0) {
                bf[c][k] = cp.Brev[c][es];
                gf[c][k] = cp.Grev[c][es];
            }
        }
        if (m_cap > 0) jf[k] = has[k] ? (int64_t)jr : i;
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k)
#pragma unroll
        for (int c = 0; c < C; ++c) rf[c][k] = CR(c, jf[k]);
#pragma unroll
    for (int c = 0; c < C; ++c) {
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            rf[c][k] = has[k] ? rf[c][k] : 0.0;
            bf[c][k] = has[k] ? bf[c][k] : 0.0;
            acc = k == 0 ? (has[0] ? gf[c][0] * rf[c][0] : 0.0) : (has[k] ? fma(gf[c][k], rf[c][k], acc) : acc);
        }
        for (int32_t e = e0 + l + kSpan; e < e1; e += kGroup) acc = fma(cp.Grev[c][e], CR(c, rev_j[e]), acc);
        acc = group_sum<kGroup>(acc);
        const double it2 = cp.it2[c], is2 = cp.is2[c];
        const double it2i = noise_w != nullptr ? it2 * hi : it2;
        const double prec = fma(iF[c] + Pi[c], is2, it2i);
        const double lin = fma(yi[c], it2i, is2 * fma(wi[c] - ri[c], iF[c], fma(wi[c], Pi[c], acc)));
        const double sd = nngp_rsqrt(prec);
        const double wn = fma(zl[c], sd, lin / prec);
        const double dw = wn - wi[c];
        if (live && l == 0) {
            CW(c, i) = wn;
            CR(c, i) = ri[c] + dw;
        }
#pragma unroll
        for (int k = 0; k < kPer; ++k)
            if (has[k]) CR(c, jf[k]) = fma(-bf[c][k], dw, rf[c][k]);
        for (int32_t e = e0 + l + kSpan; e < e1; e += kGroup) {
            const int64_t j = rev_j[e];
            CR(c, j) = fma(-cp.Brev[c][e], dw, CR(c, j));
        }
    }
}
#undef CW
#undef CR

// The interleaved form with every access to w / r of all chains as ONE run of 8C bytes (dwordx4 pairs:
// half the load / store instructions of per-chain scalars, which is what the colour step's random r_j
// traffic costs -- the interleaving alone moved the bytes but not the instruction count).  Chains inner:
// each chain's operations and their order are gibbs_w_color's (its sums, then its draw, then its
// scatter), so chain c is still bit-identical; across chains only the interleaving of independent
// operations changes.
// (rows of an odd chain count are only 8-byte aligned: scalar accesses there, the same values)
template <int C>
__device__ __forceinline__ void il_load(const double* p, double (&v)[C]) {
    if constexpr (C % 2 == 0) {
#pragma unroll
        for (int q = 0; q < C; q += 2) {
            const double2 t = *(const double2*)(p + q);
            v[q] = t.x;
            v[q + 1] = t.y;
        }
    } else {
#pragma unroll
        for (int q = 0; q < C; ++q) v[q] = p[q];
    }
}
template <int C>
__device__ __forceinline__ void il_store(double* p, const double (&v)[C]) {
    if constexpr (C % 2 == 0) {
#pragma unroll
        for (int q = 0; q < C; q += 2) *(double2*)(p + q) = make_double2(v[q], v[q + 1]);
    } else {
#pragma unroll
        for (int q = 0; q < C; ++q) p[q] = v[q];
    }
}

template <int C>
__global__ __launch_bounds__(256) void gibbs_w_color_chains_il(const int4* __restrict__ member_rows,
                                                               int64_t n_members, const ChainPtrs cp,
                                                               const double* __restrict__ noise_w,
                                                               const int32_t* __restrict__ rev_j, int64_t m_cap) {
    const int64_t t = xcd_logical_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
    const int64_t g = t / kGroup;
    const int l = (int)(t % kGroup);
    const bool live = g < n_members;
    const int4 mr = member_rows[live ? g : n_members - 1];
    const int64_t i = mr.x;
    const int32_t e0 = mr.y, e1 = live ? mr.z : mr.y;
    const double hi = noise_w != nullptr ? noise_w[i] : 1.0;
    double* __restrict__ W = cp.wil;
    double* __restrict__ R = cp.ril;
    double wi[C], ri[C], iF[C], Pi[C], yi[C], zl[C];
    il_load<C>(W + i * C, wi);
    il_load<C>(R + i * C, ri);
#pragma unroll
    for (int c = 0; c < C; ++c) {
        iF[c] = cp.invF[c][i];
        Pi[c] = cp.P[c][i];
        yi[c] = cp.yres[c][i];
        zl[c] = cp.z[c][i];
    }
    int64_t jf[kPer];
    bool has[kPer];
    double bf[C][kPer], gf[C][kPer], rf[kPer][C];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int32_t ef = e0 + l + k * kGroup;
        has[k] = ef < e1;
        const int64_t es = has[k] ? ef : 0;
        jf[k] = i;
        int32_t jr = 0;
        if (m_cap > 0) jr = rev_j[es];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            bf[c][k] = 0.0;
            gf[c][k] = 0.0;
            if (m_cap > 0) {
                bf[c][k] = cp.Brev[c][es];
                gf[c][k] = cp.Grev[c][es];
            }
        }
        if (m_cap > 0) jf[k] = has[k] ? (int64_t)jr : i;
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) il_load<C>(R + jf[k] * C, rf[k]);
    double acc[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
        double a = 0.0;
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            rf[k][c] = has[k] ? rf[k][c] : 0.0;
            bf[c][k] = has[k] ? bf[c][k] : 0.0;
            a = k == 0 ? (has[0] ? gf[c][0] * rf[k][c] : 0.0) : (has[k] ? fma(gf[c][k], rf[k][c], a) : a);
        }
        acc[c] = a;
    }
    for (int32_t e = e0 + l + kSpan; e < e1; e += kGroup) {
        double rj[C];
        il_load<C>(R + (int64_t)rev_j[e] * C, rj);
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] = fma(cp.Grev[c][e], rj[c], acc[c]);
    }
    double wn[C], dw[C], rn[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
        double a = acc[c];
        a = group_sum<kGroup>(a);
        const double it2 = cp.it2[c], is2 = cp.is2[c];
        const double it2i = noise_w != nullptr ? it2 * hi : it2;
        const double prec = fma(iF[c] + Pi[c], is2, it2i);
        const double lin = fma(yi[c], it2i, is2 * fma(wi[c] - ri[c], iF[c], fma(wi[c], Pi[c], a)));
        const double sd = nngp_rsqrt(prec);
        wn[c] = fma(zl[c], sd, lin / prec);
        dw[c] = wn[c] - wi[c];
        rn[c] = ri[c] + dw[c];
    }
    if (live && l == 0) {
        il_store<C>(W + i * C, wn);
        il_store<C>(R + i * C, rn);
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        if (has[k]) {
            double v[C];
#pragma unroll
            for (int c = 0; c < C; ++c) v[c] = fma(-bf[c][k], dw[c], rf[k][c]);
            il_store<C>(R + jf[k] * C, v);
        }
    }
    for (int32_t e = e0 + l + kSpan; e < e1; e += kGroup) {
        const int64_t j = rev_j[e];
        double rj[C];
        il_load<C>(R + j * C, rj);
#pragma unroll
        for (int c = 0; c < C; ++c) rj[c] = fma(-cp.Brev[c][e], dw[c], rj[c]);
        il_store<C>(R + j * C, rj);
    }
}

hipError_t gibbs_w_sweep_chains_launch(const int32_t* member_rows, int n_colors, const int32_t* color_off_host,
                                       int chains, const void* const* preps, int64_t n, int m, const double* sigma2,
                                       const double* tau2, const double* const* yres, const double* noise_w,
                                       double* const* w, double* const* r, const int32_t* rev_j,
                                       const double* const* z, hipStream_t s, double* w_il, double* r_il) {
    if (chains < 1 || chains > kMaxChains) return hipErrorInvalidValue;
    const bool il = w_il != nullptr;
    ChainPtrs cp{};
    cp.wil = w_il;
    cp.ril = r_il;
    for (int c = 0; c < chains; ++c) {
        const GibbsPrep g = prep_layout((void*)preps[c], n, m);
        cp.Brev[c] = g.Brev;
        cp.Grev[c] = g.Grev;
        cp.P[c] = g.P;
        cp.invF[c] = g.invF;
        cp.yres[c] = yres[c];
        cp.z[c] = z[c];
        cp.w[c] = il ? nullptr : w[c];
        cp.r[c] = il ? nullptr : r[c];
        cp.it2[c] = 1.0 / tau2[c];
        cp.is2[c] = 1.0 / sigma2[c];
    }
    for (int k = 0; k < n_colors; ++k) {
        const int64_t a = color_off_host[k], b = color_off_host[k + 1];
        if (b <= a) continue;
        const dim3 grid((unsigned)(((b - a) * kGroup + 255) / 256));
        const int4* mr = (const int4*)member_rows + a;
        const int64_t mc = n * (int64_t)m;
        switch (chains) {
#define NNGP_CHAINS_CASE(CC)                                                                                      \
    case CC:                                                                                                     \
        if (il)                                                                                                  \
            hipLaunchKernelGGL((gibbs_w_color_chains_il<CC>), grid, dim3(256), 0, s, mr, b - a, cp, noise_w,     \
                               rev_j, mc);                                                                       \
        else                                                                                                     \
            hipLaunchKernelGGL((gibbs_w_color_chains<CC>), grid, dim3(256), 0, s, mr, b - a, cp, noise_w,        \
                               rev_j, mc);                                                                       \
        break;
            NNGP_CHAINS_CASE(1) NNGP_CHAINS_CASE(2) NNGP_CHAINS_CASE(3) NNGP_CHAINS_CASE(4)
            NNGP_CHAINS_CASE(5) NNGP_CHAINS_CASE(6) NNGP_CHAINS_CASE(7) NNGP_CHAINS_CASE(8)
#undef NNGP_CHAINS_CASE
        }
    }
    return hipGetLastError();
}

// Sharded chain (nngp_gibbs_w_apply): after a colour's exchange, each rank replays the updates of the
// other ranks' members it keeps a replica of.  Row (i, e0, e1, src): w_new = wsrc[src] (the owner's
// draw), dw = w_new - w_i computed from this rank's replica of w_i -- the owner's operands, so the
// same bits -- then w_i = w_new, r_i += dw and r_j -= B_{j,i} dw over the children, exactly the
// owner's scatter (B read in place: B_{j,i} = B[j, rev_k[e]], the value the owner's Brev holds).
__global__ __launch_bounds__(256) void gibbs_w_apply_kernel(const int4* __restrict__ rows, int64_t n_rows,
                                                            const double* __restrict__ wsrc,
                                                            const double* __restrict__ B, int m,
                                                            double* __restrict__ w, double* __restrict__ r,
                                                            const int32_t* __restrict__ rev_j,
                                                            const int32_t* __restrict__ rev_k) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t g = t / kGroup;
    const int l = (int)(t % kGroup);
    if (g >= n_rows) return;
    const int4 a = rows[g];
    const int64_t i = a.x;
    const double wn = wsrc[a.w];
    const double dw = wn - w[i];
    for (int32_t e = a.y + l; e < a.z; e += kGroup) {
        const int64_t j = rev_j[e];
        r[j] = fma(-B[j * m + rev_k[e]], dw, r[j]);
    }
    if (l == 0) {
        r[i] = r[i] + dw;
        w[i] = wn;
    }
}

hipError_t gibbs_w_apply_launch(const int32_t* rows, int64_t n_rows, const double* wsrc, const double* B, int m,
                                double* w, double* r, const int32_t* rev_j, const int32_t* rev_k, hipStream_t s) {
    if (n_rows <= 0) return hipSuccess;
    const int64_t threads = n_rows * kGroup;
    hipLaunchKernelGGL(gibbs_w_apply_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s,
                       (const int4*)rows, n_rows, wsrc, B, m, w, r, rev_j, rev_k);
    return hipGetLastError();
}

// ---------------------------------------------------------------- small reductions for the conjugate steps
// out[0] = sum r_i^2 / Ft_i (sigma2 full conditional), out[1] = sum h_i (yres_i - w_i)^2 (tau2),
// out[2 + c] = sum_i h_i X[i, c] (y_i - w_i) (beta), c < p; h_i = noise_w[i] (1 when NULL).
// Fixed-order: per-block records + one fold.
__global__ __launch_bounds__(256) void gibbs_stats_blocks(int64_t n, const double* __restrict__ r,
                                                          const double* __restrict__ Ft,
                                                          const double* __restrict__ yres,
                                                          const double* __restrict__ y, const double* __restrict__ X,
                                                          int p, const double* __restrict__ w,
                                                          const double* __restrict__ noise_w,
                                                          double* __restrict__ rec) {
    __shared__ double sh[256];
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int nv = 2 + p;
    for (int v = 0; v < nv; ++v) {
        double x = 0.0;
        if (i < n) {
            if (v == 0) {
                x = r[i] * r[i] / Ft[i];
            } else if (v == 1) {
                const double e = yres[i] - w[i];
                x = e * e;
            } else {
                x = X[i * p + (v - 2)] * (y[i] - w[i]);
            }
            if (v > 0 && noise_w != nullptr) x *= noise_w[i];
        }
        sh[threadIdx.x] = x;
        __syncthreads();
        for (int o = 128; o > 0; o >>= 1) {
            if ((int)threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
            __syncthreads();
        }
        if (threadIdx.x == 0) rec[blockIdx.x * (int64_t)nv + v] = sh[0];
        __syncthreads();
    }
}

__global__ __launch_bounds__(1024) void gibbs_stats_fold(const double* __restrict__ rec, int64_t nb, int nv,
                                                         double* __restrict__ out) {
    // fixed order: thread t folds records t, t + 1024, ...; xor-butterfly per wave; 16 waves in order
    __shared__ double sh[16];
    const int t = threadIdx.x;
    for (int v = 0; v < nv; ++v) {
        double a = 0.0;
        for (int64_t b = t; b < nb; b += 1024) a += rec[b * nv + v];
        a = wave_sum(a);
        if ((t & 63) == 0) sh[t >> 6] = a;
        __syncthreads();
        if (t == 0) {
            double x = 0.0;
            for (int k = 0; k < 16; ++k) x += sh[k];
            out[v] = x;
        }
        __syncthreads();
    }
}

size_t gibbs_stats_workspace_bytes(int64_t n, int p) { return align256((size_t)((n + 255) / 256) * (2 + p) * 8); }

hipError_t gibbs_stats_launch(int64_t n, const double* r, const double* Ft, const double* yres, const double* y,
                              const double* X, int p, const double* w, const double* noise_w, double* out,
                              void* workspace, hipStream_t s) {
    const int64_t nb = (n + 255) / 256;
    if (nb == 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(gibbs_stats_blocks, dim3((unsigned)nb), dim3(256), 0, s, n, r, Ft, yres, y, X, p, w, noise_w,
                       (double*)workspace);
    hipLaunchKernelGGL(gibbs_stats_fold, dim3(1), dim3(1024), 0, s, (const double*)workspace, nb, 2 + p, out);
    return hipGetLastError();
}

}  // namespace nngp
