// Wave pair plans (pair_plan.h): built once per neighbour set and visiting order, on the GPU.
//
// One 256-thread block per wave (4 per region = the pair kernel's tile: the same q / q + 1 rows of
// pairb_tiling; wave w of a region holds its local rows 32 w .. 32 w + 31, lanes 2 l + q).  Per wave:
//   1. the joint points of its rows (each row's neighbours nbr[r, :] and the location i0 + order[r]
//      itself) are sorted as (global index, position) keys in LDS (bitonic); the first of each run
//      gets the next local index u = 0, 1, ... (ascending global index); invalid slots (-1, or out of
//      range) get none and read the exact-zero covariance;
//   2. every used entry (u_a, u_b) of every lane marks a bit of a 2^16-bit LDS bitmap (u < 256: key
//      min << 8 | max); popcount prefix sums over the bitmap give each distinct pair its rank k in key
//      order -- pair k is evaluated by lane k % 64 in round k / 64 into slice byte 8 (k + 1);
//   3. the U list (zero-filled to whole rounds of 64), the pair words (the points' slice byte offsets,
//      zero-filled to whole groups of kPlanPairGroup rounds; plan_pair_word's lane-major order), per
//      lane in the kernel's fill order the entries' slice byte offsets, and per lane the checksum of the
//      nbr / order words the kernel will read (pair_plan.h) are written to the wave's fixed-size slot.
// Waves past the caps (nU > plan_ucap, or the covariances and the points not fitting the slice) are
// marked; a region is planned only when all its waves are.  A last single-block kernel lists planned and
// direct regions in order; the host reads the two counts once (nngp_pair_plan_build synchronises: a
// setup call, like the neighbour build).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nngp_internal.h"
#include "pair_plan.h"

namespace nngp {

namespace {

constexpr int kBitWords = (1 << 16) / 32;  // 2048 words: keys u_a << 8 | u_b, u < 256

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

__global__ __launch_bounds__(kPlanThreads) void wave_plan_build_kernel(
    const int32_t* __restrict__ nbr, const int32_t* __restrict__ order, int64_t n_rows, int m, int64_t i0,
    int64_t n_points, int64_t tq, int64_t trem, uint8_t* __restrict__ slots, int ps) {
    extern __shared__ uint64_t pp_lds[];
    __shared__ int scan_sh[kPlanThreads / 64];
    const int t = threadIdx.x;
    const int64_t region = blockIdx.x / kPlanWaves;
    const int wv = (int)(blockIdx.x % kPlanWaves);
    const int nr = (int)(tq + (region < trem ? 1 : 0));
    const int64_t r0 = region * tq + (region < trem ? region : trem);
    const int NR = m + 1, NP = plan_np(m), NE = plan_entries(m);
    const int npos = kPlanWaveRows * NR;  // (wave row, joint row) positions
    int nsort = 1;
    while (nsort < npos) nsort <<= 1;
    uint64_t* key = pp_lds;                                      // nsort
    int16_t* loc = (int16_t*)(key + nsort);                      // npos (+ pad): local index or -1
    uint32_t* bits = (uint32_t*)(loc + ((npos + 7) & ~7));       // kBitWords
    uint32_t* pref = bits + kBitWords;                           // kBitWords
    const int64_t wsb = plan_wave_slot_bytes(m);
    uint8_t* slot = slots + (region * kPlanWaves + wv) * wsb;
    int32_t* hdr = (int32_t*)slot;
    const int slice = plan_slice_bytes(m), ecap = plan_ecap(m), ucap = plan_ucap(m);

    // ---- 1. the joint points, sorted by (global index, position)
    for (int p = t; p < nsort; p += kPlanThreads) {
        uint64_t k = ~0ull;
        if (p < npos) {
            const int l = p / NR, a = p % NR;
            const int lr = kPlanWaveRows * wv + l;
            if (lr < nr) {
                const int64_t r = r0 + lr;
                const int64_t rr = order != nullptr ? (int64_t)order[r] : r;
                int64_t j = i0 + rr;
                if (a < m) j = nbr[r * m + a];
                if (j >= 0 && j < n_points) k = ((uint64_t)j << 32) | (uint64_t)p;
            }
            loc[p] = -1;
        }
        key[p] = k;
    }
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
    // local indices: u = count of run starts before (a thread scans a contiguous chunk)
    const int per = (nsort + kPlanThreads - 1) / kPlanThreads;
    const int c0 = t * per < nsort ? t * per : nsort, c1 = c0 + per < nsort ? c0 + per : nsort;
    auto run_start = [&](int p) -> bool {
        const uint64_t k = key[p];
        return k != ~0ull && (p == 0 || (key[p - 1] >> 32) != (k >> 32));
    };
    int cnt = 0;
    for (int p = c0; p < c1; ++p) cnt += run_start(p) ? 1 : 0;
    int nU;
    int u = block_scan_excl(cnt, scan_sh, &nU) - 1;
    int32_t* ulist = (int32_t*)(slot + plan_u_off());
    for (int p = c0; p < c1; ++p) {
        const uint64_t k = key[p];
        if (k == ~0ull) break;
        if (run_start(p)) {
            ++u;
            if (u < ucap) ulist[u] = (int32_t)(k >> 32);
        }
        if (u < ucap) loc[k & 0xffffffffu] = (int16_t)u;
    }
    if (nU > ucap) {
        if (t == 0) {
            hdr[0] = nU;
            hdr[1] = -1;
            hdr[2] = 1;
        }
        return;
    }
    for (int x = nU + t; x < ucap; x += kPlanThreads) ulist[x] = 0;  // (the kernel loads every round: point 0)
    for (int w = t; w < kBitWords; w += kPlanThreads) bits[w] = 0;
    __syncthreads();

    // ---- 2. mark the used pairs: threads 0..63 are the wave's lanes (lane L: wave row L >> 1, q = L & 1)
    auto pair_key = [&](int L, int e, int* key_out) -> bool {
        const int l = L >> 1, q = L & 1;
        if (kPlanWaveRows * wv + l >= nr) return false;
        int a, b;
        plan_entry(NP, q, e, &a, &b);
        if (a < 0 || a > m || b > m) return false;
        const int ua = loc[l * NR + a], ub = loc[l * NR + b];
        if (ua < 0 || ub < 0) return false;
        *key_out = ua < ub ? (ua << 8) | ub : (ub << 8) | ua;
        return true;
    };
    for (int x = t; x < 64 * NE; x += kPlanThreads) {
        int k;
        if (pair_key(x / NE, x % NE, &k)) atomicOr(&bits[k >> 5], 1u << (k & 31));
    }
    __syncthreads();
    // ---- 3. ranks: popcount prefix over the bitmap (thread t: words [8 t, 8 t + 8))
    constexpr int WPT = kBitWords / kPlanThreads;
    int pc = 0;
    for (int w = WPT * t; w < WPT * t + WPT; ++w) pc += __popc(bits[w]);
    int nE;
    int base = block_scan_excl(pc, scan_sh, &nE);
    const int cb = slice - nU * ps;  // the points' base in the slice
    if (nE > ecap || !plan_fits(nU, nE, ps, slice)) {
        if (t == 0) {
            hdr[0] = nU;
            hdr[1] = nE;
            hdr[2] = 1;
        }
        return;
    }
    uint32_t* pw = (uint32_t*)(slot + plan_pair_off(m));
    for (int w = WPT * t; w < WPT * t + WPT; ++w) {
        pref[w] = (uint32_t)base;
        uint32_t x = bits[w];
        while (x != 0u) {
            const int bit = __ffs(x) - 1;
            x &= x - 1u;
            const int k = (w << 5) | bit;
            // the slice byte offsets of the two points (< slice <= 2^16)
            pw[plan_pair_word(base++)] = (uint32_t)(cb + (k >> 8) * ps) | ((uint32_t)(cb + (k & 255) * ps) << 16);
        }
    }
    for (int x = nE + t; x < plan_pair_slots(nE) - 1; x += kPlanThreads) pw[plan_pair_word(x)] = 0u;  // whole groups
    __syncthreads();
    // ---- 4. the lanes' maps (slice byte offsets 8 (rank + 1); 0: the exact-zero slot) and checksums
    uint32_t* mp = (uint32_t*)(slot + plan_map_off(m));
    const int CHE = plan_map_chunks(m);
    for (int x = t; x < 64 * CHE; x += kPlanThreads) {
        const int L = x & 63, c = x >> 6;
        uint32_t d[4];
        for (int k = 0; k < 4; ++k) {
            uint32_t v = 0;
            for (int h = 0; h < 2; ++h) {
                const int e = 8 * c + 2 * k + h;
                int key2;
                uint32_t off = 0;
                if (e < NE && pair_key(L, e, &key2)) {
                    const uint32_t wd = bits[key2 >> 5];
                    const uint32_t rank = pref[key2 >> 5] + __popc(wd & ((1u << (key2 & 31)) - 1u));
                    off = (rank + 1u) * 8u;
                }
                v |= off << (16 * h);
            }
            d[k] = v;
        }
        *(uint4*)(mp + 4 * ((int64_t)c * 64 + L)) = make_uint4(d[0], d[1], d[2], d[3]);
    }
    if (t < 64) {
        // the words the kernel reads for lane t (bf_pairb.h: dead lanes read the last row)
        const int lr = kPlanWaveRows * wv + (t >> 1), q = t & 1;
        const int64_t rl = lr < nr ? r0 + lr : n_rows - 1;
        const int32_t ov = (order != nullptr ? order : nbr)[rl];
        const int64_t rr = order != nullptr ? (int64_t)ov : rl;
        uint32_t h = plan_chk_init((uint32_t)(uint64_t)rr);
        for (int s = 0; s < NP; ++s) {
            const int a = 2 * s + q;
            h = plan_chk_step(h, nbr[rl * m + (a < m ? a : m - 1)], s);
        }
        ((uint32_t*)(slot + plan_chk_off(m)))[t] = h;
    }
    if (t == 0) {
        hdr[0] = nU;
        hdr[1] = nE;
        hdr[2] = 0;
    }
}

// planned / direct region lists in region order, and the counts into the global header (a region is
// planned when all its waves are: status word 2 of each wave slot, written by wave_plan_build_kernel)
__global__ __launch_bounds__(1024) void pair_plan_lists_kernel(const uint8_t* __restrict__ slots, int64_t slot_bytes,
                                                               int64_t wave_slot_bytes, int64_t n_regions,
                                                               int32_t* __restrict__ planned,
                                                               int32_t* __restrict__ direct, PlanHeader* hdr) {
    __shared__ int sh[16];
    __shared__ int64_t carry[2];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (t == 0) carry[0] = carry[1] = 0;
    __syncthreads();
    for (int64_t b = 0; b < n_regions; b += 1024) {
        const int64_t r = b + t;
        int st = -1;
        if (r < n_regions) {
            st = 0;
            for (int k = 0; k < kPlanWaves; ++k)
                st |= ((const int32_t*)(slots + r * slot_bytes + k * wave_slot_bytes))[2] != 0 ? 1 : 0;
        }
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
    const int npos = kPlanWaveRows * (m + 1);
    int nsort = 1;
    while (nsort < npos) nsort <<= 1;
    return (size_t)nsort * 8 + (size_t)((npos + 7) & ~7) * 2 + (size_t)kBitWords * 8;
}

hipError_t pair_plan_build_launch(const int32_t* nbr, const int32_t* order, int64_t n_rows, int m, int dim, int64_t i0,
                                  int64_t n_points, int64_t tq, int64_t trem, void* plan, hipStream_t s) {
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
    hipLaunchKernelGGL(wave_plan_build_kernel, dim3((unsigned)(nreg * kPlanWaves)), dim3(kPlanThreads), lds, s, nbr,
                       order, n_rows, m, i0, n_points, tq, trem, p + kPlanGlobalHdr, plan_ps(dim));
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(pair_plan_lists_kernel, dim3(1), dim3(1024), 0, s, (const uint8_t*)(p + kPlanGlobalHdr), sb,
                       plan_wave_slot_bytes(m), nreg, planned, direct, (PlanHeader*)p);
    return hipGetLastError();
}

}  // namespace nngp
