// Tile pair plans (pair_plan.h): built once per neighbour set and visiting order, on the GPU.
//
// One 256-thread block per region (= the pair kernel's tile: the same q / q + 1 rows of
// pairb_tiling).  Per region:
//   1. the joint points of its rows (each row's neighbours nbr[r, :] and the location i0 + order[r]
//      itself) are sorted as (global index, position) keys in LDS (bitonic); the first of each run
//      gets the next local index u = 1, 2, ... (ascending global index), invalid slots (-1, or out of
//      range) keep u = 0, and rows with an index out of range are noted (the first bad location);
//   2. every used entry (u_a, u_b) of every lane marks a bit of a 2^18-bit LDS bitmap (u <= 511: key
//      (min - 1) << 9 | (max - 1)); popcount prefix sums over the bitmap give each distinct pair its
//      rank in key order, i.e. the pair list sorted by (u_a, u_b) and an O(1) lookup per entry;
//   3. the pair words, the U list and, per lane in the kernel's fill order, the entries' LDS byte
//      offsets (8 (rank + 1); 0: exact-zero slot) and the rows' local indices are written to the
//      region's fixed-size slot.
// Regions past the caps (nU > plan_ucap or nE > plan_ecap(m, dim)) are marked direct.  A last
// single-block kernel lists planned and direct regions in order; the host reads the two counts once
// (nngp_pair_plan_build synchronises: a setup call, like the neighbour build).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nngp_internal.h"
#include "pair_plan.h"

namespace nngp {

namespace {

constexpr int kBitWords = (1 << 18) / 32;  // 8192 words: keys (u_a - 1) << 9 | (u_b - 1), u <= 511

// exclusive prefix sum over the block's 256 threads (every thread calls it); returns the total in *tot
__device__ int block_scan_excl(int v, int* sh, int* tot) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) sh[w] = x;
    __syncthreads();
    int base = 0, all = 0;
#pragma unroll
    for (int k = 0; k < kPlanThreads / 64; ++k) {
        base += k < w ? sh[k] : 0;
        all += sh[k];
    }
    __syncthreads();
    *tot = all;
    return base + x - v;
}

__global__ __launch_bounds__(kPlanThreads) void pair_plan_build_kernel(
    const int32_t* __restrict__ nbr, const int32_t* __restrict__ order, int64_t n_rows, int m, int64_t i0,
    int64_t n_points, int64_t tq, int64_t trem, uint8_t* __restrict__ plan, int64_t slot_bytes, int ucap, int ecap,
    int ps) {
    extern __shared__ uint64_t pp_lds[];
    __shared__ int scan_sh[kPlanThreads / 64];
    __shared__ double bad_sh[kPlanThreads / 64];
    const int t = threadIdx.x;
    const int64_t region = blockIdx.x;
    const int nr = (int)(tq + (region < trem ? 1 : 0));
    const int64_t r0 = region * tq + (region < trem ? region : trem);
    const int NR = m + 1, NP = plan_np(m), NE = plan_entries(m);
    const int npos = kPlanThreads / 2 * NR;  // (local row, joint row) positions
    int nsort = 1;
    while (nsort < npos) nsort <<= 1;
    uint64_t* key = pp_lds;                                      // nsort
    uint16_t* loc = (uint16_t*)(key + nsort);                    // npos (+ pad)
    uint32_t* bits = (uint32_t*)(loc + ((npos + 7) & ~7));       // kBitWords
    uint32_t* pref = bits + kBitWords;                           // kBitWords
    uint8_t* slot = plan + kPlanGlobalHdr + region * slot_bytes;

    // ---- 1. the joint points, sorted by (global index, position)
    double bad = INFINITY;
    for (int p = t; p < nsort; p += kPlanThreads) {
        uint64_t k = ~0ull;
        if (p < npos) {
            const int lr = p / NR, a = p % NR;
            if (lr < nr) {
                const int64_t r = r0 + lr;
                const int64_t rr = order != nullptr ? (int64_t)order[r] : r;
                const int64_t i = i0 + rr;
                int64_t j = i;
                if (a < m) {
                    j = nbr[r * m + a];
                    if (j >= n_points || j < -1) bad = fmin(bad, (double)i);
                }
                if (j >= 0 && j < n_points) k = ((uint64_t)j << 32) | (uint64_t)p;
            }
            loc[p] = 0;
        }
        key[p] = k;
    }
    bad = wave_min(bad);
    if ((t & 63) == 0) bad_sh[t >> 6] = bad;
    __syncthreads();
    for (int k = 2; k <= nsort; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = t; i < nsort; i += kPlanThreads) {
                const int ij = i ^ j;
                if (ij > i) {
                    const uint64_t x = key[i], y = key[ij];
                    if ((x > y) == ((i & k) == 0)) {
                        key[i] = y;
                        key[ij] = x;
                    }
                }
            }
            __syncthreads();
        }
    }
    // local indices: u = inclusive count of run starts (a thread scans a contiguous chunk)
    const int per = nsort / kPlanThreads;  // nsort >= 512 (m >= 2)
    const int c0 = t * per, c1 = c0 + per;
    int cnt = 0;
    for (int p = c0; p < c1; ++p) {
        const uint64_t k = key[p];
        const bool start = k != ~0ull && (p == 0 || (key[p - 1] >> 32) != (k >> 32));
        cnt += start ? 1 : 0;
    }
    int nU;
    int u = block_scan_excl(cnt, scan_sh, &nU);
    int32_t* ulist = (int32_t*)(slot + kPlanUOff);
    for (int p = c0; p < c1; ++p) {
        const uint64_t k = key[p];
        if (k == ~0ull) break;
        if (p == 0 || (key[p - 1] >> 32) != (k >> 32)) {
            ++u;
            if (u <= ucap) ulist[u - 1] = (int32_t)(k >> 32);
        }
        loc[k & 0xffffffffu] = (uint16_t)(u <= ucap ? u : 0);
    }
    double badr = INFINITY;
#pragma unroll
    for (int w = 0; w < kPlanThreads / 64; ++w) badr = fmin(badr, bad_sh[w]);
    int32_t* hdr = (int32_t*)slot;
    if (nU > ucap) {
        if (t == 0) {
            hdr[0] = nU;
            hdr[1] = -1;
            hdr[2] = 1;
            *(double*)(slot + kPlanHdrBadOff) = badr;
        }
        return;
    }
    for (int w = t; w < kBitWords; w += kPlanThreads) bits[w] = 0;
    __syncthreads();

    // ---- 2. mark the used pairs: thread t is lane q = t & 1 of local row t >> 1
    const int lr = t >> 1, q = t & 1;
    const bool live = lr < nr;
    auto pair_key = [&](int e, int* key_out) -> bool {
        int a, b;
        plan_entry(NP, q, e, &a, &b);
        if (!live || a < 0 || a > m || b > m) return false;
        const int ua = loc[lr * NR + a], ub = loc[lr * NR + b];
        if (ua == 0 || ub == 0) return false;
        const int lo = ua < ub ? ua : ub, hi = ua < ub ? ub : ua;
        *key_out = ((lo - 1) << 9) | (hi - 1);
        return true;
    };
    for (int e = 0; e < NE; ++e) {
        int k;
        if (pair_key(e, &k)) atomicOr(&bits[k >> 5], 1u << (k & 31));
    }
    __syncthreads();
    // ---- 3. ranks: popcount prefix over the bitmap (thread t: words [32 t, 32 t + 32))
    int pc = 0;
    for (int w = 32 * t; w < 32 * t + 32; ++w) pc += __popc(bits[w]);
    int nE;
    int base = block_scan_excl(pc, scan_sh, &nE);
    if (nE > ecap) {
        if (t == 0) {
            hdr[0] = nU;
            hdr[1] = nE;
            hdr[2] = 1;
            *(double*)(slot + kPlanHdrBadOff) = badr;
        }
        return;
    }
    uint32_t* pw = (uint32_t*)(slot + kPlanPairOff);
    for (int w = 32 * t; w < 32 * t + 32; ++w) {
        pref[w] = (uint32_t)base;
        uint32_t x = bits[w];
        while (x != 0u) {
            const int bit = __ffs(x) - 1;
            x &= x - 1u;
            const int k = (w << 5) | bit;
            // the planned kernel's LDS byte offsets of the two points (u * ps, u <= 511: < 2^16)
            pw[base++] = (uint32_t)(((k >> 9) + 1) * ps) | ((uint32_t)(((k & 511) + 1) * ps) << 16);
        }
    }
    __syncthreads();
    // ---- 4. this lane's map: entry offsets (u16 pairs in dwords, 4 dwords per chunk), then row indices
    uint32_t* mp = (uint32_t*)(slot + kPlanMapOff);
    const int CHE = plan_map_chunks(m), CHL = plan_loc_chunks(m);
    for (int c = 0; c < CHE; ++c) {
        uint32_t d[4];
        for (int k = 0; k < 4; ++k) {
            uint32_t v = 0;
            for (int h = 0; h < 2; ++h) {
                const int e = 8 * c + 2 * k + h;
                int key2;
                uint32_t off = 0;
                if (e < NE && pair_key(e, &key2)) {
                    const uint32_t wd = bits[key2 >> 5];
                    const uint32_t rank = pref[key2 >> 5] + __popc(wd & ((1u << (key2 & 31)) - 1u));
                    off = (rank + 1u) * 8u;
                }
                v |= off << (16 * h);
            }
            d[k] = v;
        }
        *(uint4*)(mp + 4 * ((int64_t)c * kPlanThreads + t)) = make_uint4(d[0], d[1], d[2], d[3]);
    }
    for (int c = 0; c < CHL; ++c) {
        uint32_t d[4];
        for (int k = 0; k < 4; ++k) {
            uint32_t v = 0;
            for (int h = 0; h < 2; ++h) {
                const int s = 8 * c + 2 * k + h, a = 2 * s + q;
                const uint32_t ua = (live && s < NP && a <= m) ? loc[lr * NR + a] : 0u;
                v |= ua << (16 * h);
            }
            d[k] = v;
        }
        *(uint4*)(mp + 4 * ((int64_t)(CHE + c) * kPlanThreads + t)) = make_uint4(d[0], d[1], d[2], d[3]);
    }
    if (t == 0) {
        hdr[0] = nU;
        hdr[1] = nE;
        hdr[2] = 0;
        *(double*)(slot + kPlanHdrBadOff) = badr;
    }
}

// planned / direct region lists in region order, and the counts into the global header
// (status: word 2 of each region slot's header, written by pair_plan_build_kernel)
__global__ __launch_bounds__(1024) void pair_plan_lists_kernel(const uint8_t* __restrict__ slots, int64_t slot_bytes,
                                                               int64_t n_regions, int32_t* __restrict__ planned,
                                                               int32_t* __restrict__ direct, PlanHeader* hdr) {
    __shared__ int sh[16];
    __shared__ int64_t carry[2];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (t == 0) carry[0] = carry[1] = 0;
    __syncthreads();
    for (int64_t b = 0; b < n_regions; b += 1024) {
        const int64_t r = b + t;
        const int st = r < n_regions ? ((const int32_t*)(slots + r * slot_bytes))[2] : -1;
        const int isp = st == 0 ? 1 : 0;
        int x = isp;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) sh[w] = x;
        __syncthreads();
        int base = 0, all = 0;
        for (int k = 0; k < 16; ++k) {
            base += k < w ? sh[k] : 0;
            all += sh[k];
        }
        const int64_t pe = carry[0] + base + x - isp;       // planned before r
        const int64_t de = carry[1] + (t - (base + x - isp));  // direct before r
        if (st == 0) planned[pe] = (int32_t)r;
        if (st == 1) direct[de] = (int32_t)r;
        __syncthreads();
        if (t == 0) {
            const int64_t nb = n_regions - b < 1024 ? n_regions - b : 1024;
            carry[0] += all;
            carry[1] += nb - all;
        }
        __syncthreads();
    }
    if (t == 0) {
        hdr->n_planned = carry[0];
        hdr->n_direct = carry[1];
    }
}

}  // namespace

size_t pair_plan_build_lds(int m) {
    const int npos = kPlanThreads / 2 * (m + 1);
    int nsort = 1;
    while (nsort < npos) nsort <<= 1;
    return (size_t)nsort * 8 + (size_t)((npos + 7) & ~7) * 2 + (size_t)kBitWords * 8;
}

hipError_t pair_plan_build_launch(const int32_t* nbr, const int32_t* order, int64_t n_rows, int m, int dim, int64_t i0,
                                  int64_t n_points, int64_t tq, int64_t trem, int ecap, void* plan, hipStream_t s) {
    const int64_t nreg = plan_regions(n_rows);
    const int64_t sb = plan_slot_bytes(m);
    uint8_t* p = (uint8_t*)plan;
    int32_t* planned = (int32_t*)(p + kPlanGlobalHdr + nreg * sb);
    int32_t* direct = planned + nreg;
    PlanHeader h{kPlanMagic, n_rows, m, dim, i0, n_points, nreg, 0, 0, sb};
    hipError_t e = hipMemcpyAsync(p, &h, sizeof h, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return e;
    if (nreg == 0) return hipSuccess;
    const size_t lds = pair_plan_build_lds(m);
    hipLaunchKernelGGL(pair_plan_build_kernel, dim3((unsigned)nreg), dim3(kPlanThreads), lds, s, nbr, order, n_rows, m,
                       i0, n_points, tq, trem, p, sb, plan_ucap(), ecap, 8 * plan_cs(dim));
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(pair_plan_lists_kernel, dim3(1), dim3(1024), 0, s, (const uint8_t*)(p + kPlanGlobalHdr), sb, nreg,
                       planned, direct, (PlanHeader*)p);
    return hipGetLastError();
}

}  // namespace nngp
