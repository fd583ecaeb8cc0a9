// Wave pair plans: covariance entries shared by the 32 locations of one wavefront, evaluated once.
//
// Reference path (bwpriest/pyNNGP, /root/reference, stubs there): _CNs / _Ccross / _Cs
// (nngp.py:78-86, 92-96) build every location's joint block C(x_a, x_b) over its neighbour set and
// itself; _Bsi / _Fsi (nngp.py:73-76, 88-90) factor it.  The pair kernel (bf_pairb.h) runs 32
// Z-order-consecutive locations per wavefront, two lanes each, and their neighbour sets overlap: at
// N = 1e6, m = 15 a wave's 32 x 120 off-diagonal joint entries hold ~1,770 distinct point pairs (46 %;
// p99 2,140, max 2,357 of 4,000 sampled waves; tools/reuse_stats.py --tile 32).  A wave plan, built
// once per neighbour set and visiting order (like the Z-order itself), lists per wave
//   * U, the wave's distinct joint points (global indices; local index u = 0 .. nU-1, ascending index),
//   * its distinct point pairs as two LDS byte offsets into the wave's slice (the pair words), in the
//     order the wave evaluates them: pair k by lane k % 64 in round k / 64 (rounds in groups of four, a
//     lane's four words of a group adjacent), its covariance stored at slice byte 8 (k + 1) (slot 0: the
//     exact zero of padding / invalid entries), and
//   * per lane, in the order the pair kernel fills its joint-block registers, the slice byte offset of
//     each entry's covariance (the entry map), plus a checksum of the lane's neighbour-index row and
//     location (checked by the kernel against nbr / order: a stale plan flags its rows instead of
//     returning the old neighbour sets' B / F).
// The planned kernel (bf_pairb<.., PL = true>) stages U's coordinates at the END of its wave's LDS slice,
// evaluates the pairs (the same nngp_cov_unit on the same operands as the unplanned kernel: covariances
// are symmetric bit for bit, (a - b)^2 == (b - a)^2) into the slice's head, and reads its joint block
// through the map; the values, the elimination and everything after are the unplanned kernel's, so
// B / F / residuals / partials are bit-identical to NNGP_ALGO_PAIRB.  Everything is wave-private: no
// block barrier between the plan loads and the fill (round 5's tile plans shared one block-wide table
// behind two __syncthreads and lost to the exposed waits).  A tile (region) whose waves
// do not all fit their slice is swept by the unplanned kernel through a tile list into the same records.
#pragma once
#include <stdint.h>

namespace nngp {

constexpr int kPlanThreads = 256;        // = kPairbThreads (bf_pairb.h): 128 locations per tile
constexpr int kPlanWaves = 4;            // waves per tile (region)
constexpr int kPlanWaveRows = 32;        // locations per wave
constexpr int kPlanMinM = 2;
constexpr int kPlanMaxM = 17;            // the right-looking two-lane kernels (m >= 18: left-looking)
constexpr int kPlanHdrBytes = 64;        // int32 nU, nE, status (0 planned, 1 over the caps)
constexpr int kPlanPairGroup = 4;        // pair rounds per step of the planned kernel's evaluation loop

__host__ __device__ constexpr int plan_np(int m) { return (m + 2) / 2; }  // row pairs of the joint block
// entries per lane: R[s][t][0..1] for t < s and R[s][s][1] (lane 1's within-pair entry; lane 0: unused)
__host__ __device__ constexpr int plan_entries(int m) { return plan_np(m) * plan_np(m); }
__host__ __device__ constexpr int plan_map_chunks(int m) { return (plan_entries(m) + 7) / 8; }  // 8 u16 per chunk
// LDS doubles per staged point
__host__ __device__ constexpr int plan_cs(int d) { return d == 1 ? 1 : d == 2 ? 2 : 4; }
__host__ __device__ constexpr int plan_ps(int d) { return 8 * plan_cs(d); }  // bytes per staged point
// blocks per CU the planned kernel runs at for m (bf_pairb.h's waves per SIMD: 4-wave blocks, 4 SIMDs)
__host__ __device__ constexpr int plan_blocks_per_cu(int m) { return m <= 13 ? 3 : 2; }
// a wave's LDS slice: the CU's 160 KB over its blocks' waves, less the block's exp table (2 KB) and
// records, in whole 256-byte units
__host__ __device__ constexpr int plan_slice_bytes(int m) {
    return ((163840 / plan_blocks_per_cu(m) - 2048 - 512) / kPlanWaves) / 256 * 256;
}
// pair groups of a wave slot (kPlanPairGroup rounds of 64 lanes each, their covariance slots within the slice)
// and the pair capacity
__host__ __device__ constexpr int plan_pair_groups(int m) { return (plan_slice_bytes(m) / 8 - 1) / (64 * kPlanPairGroup); }
__host__ __device__ constexpr int plan_ecap(int m) { return 64 * kPlanPairGroup * plan_pair_groups(m); }
// pair slots a wave's evaluation writes: whole groups of kPlanPairGroup rounds of 64 lanes, + the zero slot
__host__ __device__ constexpr int plan_pair_slots(int nE) {
    return 64 * kPlanPairGroup * ((nE + 64 * kPlanPairGroup - 1) / (64 * kPlanPairGroup)) + 1;
}
// whether a wave of nU points and nE pairs fits a slice of sb bytes (points of ps bytes at its end): the nE
// real covariances end below the points, and the last group's unused lanes -- which store past nE, over
// points no read needs any more -- still inside the slice
__host__ __device__ constexpr bool plan_fits(int nU, int nE, int ps, int sb) {
    return 8 * (nE + 1) <= sb - nU * ps && 8 * plan_pair_slots(nE) <= sb;
}
// U-list capacity of a wave slot (m = 15: nU ~125, max 186 of 4,000 sampled waves; m = 17: max 198)
__host__ __device__ constexpr int plan_ucap(int) { return 256; }
// byte offsets inside a wave slot
__host__ __device__ constexpr int plan_u_off() { return kPlanHdrBytes; }
__host__ __device__ constexpr int plan_pair_off(int m) { return plan_u_off() + 4 * plan_ucap(m); }
// pair words: group g's 4 x 64 words lane-major (lane L's four words at 1024 g + 16 L: one 16-byte load)
__host__ __device__ constexpr int plan_pair_word(int k) {
    return (k >> 8 << 8) | ((k & 63) << 2) | ((k >> 6) & 3);
}
__host__ __device__ constexpr int plan_map_off(int m) { return plan_pair_off(m) + 4 * plan_ecap(m); }
__host__ __device__ constexpr int plan_chk_off(int m) { return plan_map_off(m) + plan_map_chunks(m) * 64 * 16; }
__host__ __device__ constexpr int64_t plan_wave_slot_bytes(int m) {
    return ((int64_t)plan_chk_off(m) + 64 * 4 + 255) & ~(int64_t)255;
}
__host__ __device__ constexpr int64_t plan_slot_bytes(int m) { return kPlanWaves * plan_wave_slot_bytes(m); }

// The planned kernel's checksum of one lane: its location rr (the visiting order's value) and the
// neighbour indices it reads for its joint rows a = 2s + q (a clamped to m - 1), each rotated by a
// distinct amount.  The builder stores it per lane; the kernel recomputes it from nbr / order.
__host__ __device__ inline uint32_t plan_rotl(uint32_t x, int r) { return r == 0 ? x : (x << r) | (x >> (32 - r)); }
__host__ __device__ inline uint32_t plan_chk_init(uint32_t rr) { return plan_rotl(rr, 1) ^ 0x9e3779b9u; }
__host__ __device__ inline uint32_t plan_chk_step(uint32_t h, int32_t j, int s) {
    return h ^ plan_rotl((uint32_t)j, (5 * s + 3) & 31);
}

// Entry e of lane q (fill order of the planned kernel): (row a, column b) of the joint block, or
// a < 0 for an unused entry (lane 0's within-pair slot).  Rows / columns > m are padding.
__host__ __device__ inline void plan_entry(int np, int q, int e, int* a, int* b) {
    int s = 0;
    while (e >= 2 * s + 1) {
        e -= 2 * s + 1;
        ++s;
    }
    const int row = 2 * s + q;
    if (e < 2 * s) {
        const int t = e >> 1;
        *a = row;
        *b = (e & 1) == 0 ? 2 * t + q : 2 * t + 1 - q;
    } else {
        *a = q == 1 ? row : -1;  // within-pair entry (2s+1, 2s), read by lane 1 only
        *b = 2 * s;
    }
    (void)np;
}

// what a sweep needs on the host: the region lists' lengths (the lists themselves are in the plan)
struct PlanLaunch {
    const uint8_t* plan;      // device: global header, then the region slots, then the lists
    int64_t n_regions, n_planned, n_direct;
    int64_t slot_bytes;       // bytes per region (kPlanWaves wave slots)
    const int32_t* planned;   // device: regions swept by the planned kernel
    const int32_t* direct;    // device: regions swept by the unplanned kernel
};

// global header of a plan buffer (256 B): geometry it was built for, and the counts
struct PlanHeader {
    int64_t magic, n_rows, m, dim, i0, n_points, n_regions, n_planned, n_direct, slot_bytes;
};
constexpr int64_t kPlanMagic = 0x4e4e47505750324cll;  // "NNGPWP2L"
constexpr int64_t kPlanGlobalHdr = 256;
inline int64_t plan_regions(int64_t n_rows) { return (n_rows + 127) / 128; }
inline int64_t plan_total_bytes(int64_t n_rows, int m) {
    const int64_t nr = plan_regions(n_rows);
    return kPlanGlobalHdr + nr * plan_slot_bytes(m) + ((2 * nr * 4 + 255) & ~(int64_t)255);
}

}  // namespace nngp
