// Tile pair plans: covariance entries shared by the locations of a sweep tile, evaluated once.
//
// Reference path (bwpriest/pyNNGP, /root/reference, stubs there): _CNs / _Ccross / _Cs
// (nngp.py:78-86, 92-96) build every location's joint block C(x_a, x_b) over its neighbour set and
// itself; _Bsi / _Fsi (nngp.py:73-76, 88-90) factor it.  In the pair kernel's Z-order tiles (128
// consecutive storage rows) neighbouring locations share most of their neighbours: at N = 1e6, m = 15
// only ~36 % of a tile's 128 x 120 off-diagonal joint entries are distinct point pairs
// (tools/reuse_stats.py).  A pair plan, built once per neighbour set and visiting order (like the
// Z-order itself), lists per tile
//   * U, the tile's distinct joint points (global indices; local index u = 1..nU, 0 = "no point"),
//   * the distinct point pairs (u_a, u_b), u_a <= u_b, sorted, as the planned kernel's LDS byte offsets
//     of the two points (u * 8 plan_cs(dim): the points sit at LDS address 0), and
//   * per location lane, in the order the pair kernel fills its registers, the LDS byte offset of
//     each entry's covariance (0: the exact-zero slot of padding / invalid / unused entries) and the
//     local index of each of its joint rows (for the values).
// The planned sweep (bf_pairb<.., PL = true>) stages U's coordinates and values in LDS, evaluates each
// distinct pair once (block-cooperatively, the same nngp_cov_unit on the same operands: covariances are
// symmetric bit for bit, (a - b)^2 == (b - a)^2), and then reads its joint block from LDS; everything
// after the covariances is the unplanned kernel's code, so B / F / residuals are bit-identical to it.
// Tiles whose U or distinct pairs exceed the LDS budget are swept by the unplanned kernel ("direct"
// tiles) into the same record array, with the same tiling, so the partials are bit-identical too.
#pragma once
#include <stdint.h>

namespace nngp {

constexpr int kPlanThreads = 256;        // = kPairbThreads (bf_pairb.h): 128 locations per tile
constexpr int kPlanUMax = 512;           // LDS point slots (slot 0 = no point): nU <= 511
constexpr int kPlanEMax = 8192;          // LDS covariance slots (slot 0 = exact zero): nE <= 8191
constexpr int kPlanHdrBytes = 64;        // int32 nU, nE, status (bytes 0..11); double at kPlanHdrBadOff
constexpr int kPlanHdrBadOff = 16;       // the region's first bad-index location (or +inf): clear of the status
                                         // word (at byte 8 its low half overwrote it: direct regions read as planned)
constexpr int kPlanUOff = kPlanHdrBytes;                     // int32 U list
constexpr int kPlanPairOff = kPlanUOff + 4 * kPlanUMax;      // uint32 pair words u_a | u_b << 16
constexpr int kPlanMapOff = kPlanPairOff + 4 * kPlanEMax;    // uint4 chunks, chunk-major over the threads
constexpr int kPlanMinM = 2;
constexpr int kPlanMaxM = 18;            // the right-looking two-lane kernels (bf_pairb.h)

__host__ __device__ constexpr int plan_np(int m) { return (m + 2) / 2; }  // row pairs of the joint block
// entries per lane: R[s][t][0..1] for t < s and R[s][s][1] (lane 1's within-pair entry; lane 0: unused)
__host__ __device__ constexpr int plan_entries(int m) { return plan_np(m) * plan_np(m); }
__host__ __device__ constexpr int plan_map_chunks(int m) { return (plan_entries(m) + 7) / 8; }  // 8 u16 per chunk
__host__ __device__ constexpr int plan_loc_chunks(int m) { return (plan_np(m) + 7) / 8; }
__host__ __device__ constexpr int64_t plan_slot_bytes(int m) {
    return ((int64_t)kPlanMapOff + (int64_t)(plan_map_chunks(m) + plan_loc_chunks(m)) * kPlanThreads * 16 + 255) &
           ~(int64_t)255;
}
// LDS doubles per staged point
__host__ __device__ constexpr int plan_cs(int d) { return d == 1 ? 1 : d == 2 ? 2 : 4; }
// blocks per CU the planned kernel runs at for m (bf_pairb.h's waves per SIMD: 4-wave blocks, 4 SIMDs)
__host__ __device__ constexpr int plan_blocks_per_cu(int m) { return m <= 13 ? 3 : 2; }
// distinct-pair cap: the LDS left per block after the points, their values and the exp table, rounded
// down to whole rounds of the block's threads (the kernel allocates 256 ceil(ecap / 256) + 1 slots)
__host__ __device__ constexpr int plan_ecap_raw(int m, int d) {
    return (163840 / plan_blocks_per_cu(m) - 4096) / 8 - kPlanUMax * (plan_cs(d) + 1) - 1;
}
__host__ __device__ constexpr int plan_ecap(int m, int d) {
    return plan_ecap_raw(m, d) / kPlanThreads * kPlanThreads < kPlanEMax - 1
               ? plan_ecap_raw(m, d) / kPlanThreads * kPlanThreads
               : kPlanEMax - 1;
}
__host__ __device__ constexpr int plan_ucap() { return kPlanUMax - 1; }

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
    int64_t slot_bytes;
    const int32_t* planned;   // device: regions swept by the planned kernel
    const int32_t* direct;    // device: regions swept by the unplanned kernel
};

// global header of a plan buffer (256 B): geometry it was built for, and the counts
struct PlanHeader {
    int64_t magic, n_rows, m, dim, i0, n_points, n_regions, n_planned, n_direct, slot_bytes;
};
constexpr int64_t kPlanMagic = 0x4e4e47505041314cll;  // "NNGPPA1L"
constexpr int64_t kPlanGlobalHdr = 256;
inline int64_t plan_regions(int64_t n_rows) { return (n_rows + 127) / 128; }
inline int64_t plan_total_bytes(int64_t n_rows, int m) {
    const int64_t nr = plan_regions(n_rows);
    return kPlanGlobalHdr + nr * plan_slot_bytes(m) + ((2 * nr * 4 + 255) & ~(int64_t)255);
}

}  // namespace nngp
