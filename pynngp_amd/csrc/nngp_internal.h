// Internal declarations shared by the HIP translation units of libnngp_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nngp_math.h"
#include "pair_plan.h"

namespace nngp {

// Invalid neighbour slots (index -1) are moved "infinitely" far away: slot a sits
// at (kFar * (a + 1), 0), so every covariance involving it is sigma2 * 2^-(huge) = 0
// (ldexp underflow) and its row/column of the joint block is a decoupled diagonal
// entry.  That keeps the pair loops free of per-entry selects; B is zeroed at the
// store.  (kFar * 64)^2 stays finite.
constexpr double kFar = 1e150;
// The same far points as a global table, so a kernel gathers an invalid slot from
// here instead of selecting after the load: the gathers stay unconditional and
// the compiler issues them back to back (no exec-masked branch per slot).
static __device__ double2 kFarPoints[64] = {{1e150, 0.0}, {2e150, 0.0}, {3e150, 0.0}, {4e150, 0.0}, {5e150, 0.0}, {6e150, 0.0}, {7e150, 0.0}, {8e150, 0.0}, {9e150, 0.0}, {10e150, 0.0}, {11e150, 0.0}, {12e150, 0.0}, {13e150, 0.0}, {14e150, 0.0}, {15e150, 0.0}, {16e150, 0.0}, {17e150, 0.0}, {18e150, 0.0}, {19e150, 0.0}, {20e150, 0.0}, {21e150, 0.0}, {22e150, 0.0}, {23e150, 0.0}, {24e150, 0.0}, {25e150, 0.0}, {26e150, 0.0}, {27e150, 0.0}, {28e150, 0.0}, {29e150, 0.0}, {30e150, 0.0}, {31e150, 0.0}, {32e150, 0.0}, {33e150, 0.0}, {34e150, 0.0}, {35e150, 0.0}, {36e150, 0.0}, {37e150, 0.0}, {38e150, 0.0}, {39e150, 0.0}, {40e150, 0.0}, {41e150, 0.0}, {42e150, 0.0}, {43e150, 0.0}, {44e150, 0.0}, {45e150, 0.0}, {46e150, 0.0}, {47e150, 0.0}, {48e150, 0.0}, {49e150, 0.0}, {50e150, 0.0}, {51e150, 0.0}, {52e150, 0.0}, {53e150, 0.0}, {54e150, 0.0}, {55e150, 0.0}, {56e150, 0.0}, {57e150, 0.0}, {58e150, 0.0}, {59e150, 0.0}, {60e150, 0.0}, {61e150, 0.0}, {62e150, 0.0}, {63e150, 0.0}, {64e150, 0.0}};
static __device__ double kZeroValue[1] = {0.0};
// the same far points for 1-D and 3-D ordinates (coordinate 0 at (a + 1) 1e150, the rest 0)
static __device__ double kFarPoints1[64] = {1e150, 2e150, 3e150, 4e150, 5e150, 6e150, 7e150, 8e150, 9e150, 10e150, 11e150, 12e150, 13e150, 14e150, 15e150, 16e150, 17e150, 18e150, 19e150, 20e150, 21e150, 22e150, 23e150, 24e150, 25e150, 26e150, 27e150, 28e150, 29e150, 30e150, 31e150, 32e150, 33e150, 34e150, 35e150, 36e150, 37e150, 38e150, 39e150, 40e150, 41e150, 42e150, 43e150, 44e150, 45e150, 46e150, 47e150, 48e150, 49e150, 50e150, 51e150, 52e150, 53e150, 54e150, 55e150, 56e150, 57e150, 58e150, 59e150, 60e150, 61e150, 62e150, 63e150, 64e150};
static __device__ double kFarPoints3[64 * 3] = {1e150, 0.0, 0.0, 2e150, 0.0, 0.0, 3e150, 0.0, 0.0, 4e150, 0.0, 0.0, 5e150, 0.0, 0.0, 6e150, 0.0, 0.0, 7e150, 0.0, 0.0, 8e150, 0.0, 0.0, 9e150, 0.0, 0.0, 10e150, 0.0, 0.0, 11e150, 0.0, 0.0, 12e150, 0.0, 0.0, 13e150, 0.0, 0.0, 14e150, 0.0, 0.0, 15e150, 0.0, 0.0, 16e150, 0.0, 0.0, 17e150, 0.0, 0.0, 18e150, 0.0, 0.0, 19e150, 0.0, 0.0, 20e150, 0.0, 0.0, 21e150, 0.0, 0.0, 22e150, 0.0, 0.0, 23e150, 0.0, 0.0, 24e150, 0.0, 0.0, 25e150, 0.0, 0.0, 26e150, 0.0, 0.0, 27e150, 0.0, 0.0, 28e150, 0.0, 0.0, 29e150, 0.0, 0.0, 30e150, 0.0, 0.0, 31e150, 0.0, 0.0, 32e150, 0.0, 0.0, 33e150, 0.0, 0.0, 34e150, 0.0, 0.0, 35e150, 0.0, 0.0, 36e150, 0.0, 0.0, 37e150, 0.0, 0.0, 38e150, 0.0, 0.0, 39e150, 0.0, 0.0, 40e150, 0.0, 0.0, 41e150, 0.0, 0.0, 42e150, 0.0, 0.0, 43e150, 0.0, 0.0, 44e150, 0.0, 0.0, 45e150, 0.0, 0.0, 46e150, 0.0, 0.0, 47e150, 0.0, 0.0, 48e150, 0.0, 0.0, 49e150, 0.0, 0.0, 50e150, 0.0, 0.0, 51e150, 0.0, 0.0, 52e150, 0.0, 0.0, 53e150, 0.0, 0.0, 54e150, 0.0, 0.0, 55e150, 0.0, 0.0, 56e150, 0.0, 0.0, 57e150, 0.0, 0.0, 58e150, 0.0, 0.0, 59e150, 0.0, 0.0, 60e150, 0.0, 0.0, 61e150, 0.0, 0.0, 62e150, 0.0, 0.0, 63e150, 0.0, 0.0, 64e150, 0.0, 0.0};

// ---------------------------------------------------------------- D-dimensional points
// Ordinates are fp64 (n, D) row-major (the reference's KDTree takes any dimension,
// nngp.py:55-61).  D = 2 loads a point with one 16-byte load.
// D = 0: the dimension is a runtime argument (1..3) and points are held as 3 coordinates, the
// missing ones 0 (the m = 25..32 kernels: one instantiation for every dimension).  The 3-D far
// points serve every runtime dimension (their first coordinate is the far one).
template <int D>
__device__ __forceinline__ const double* far_point(int a) {
    if constexpr (D == 1) return kFarPoints1 + (a & 63);
    else if constexpr (D == 2) return (const double*)(kFarPoints + (a & 63));
    else return kFarPoints3 + 3 * (a & 63);
}
template <int D>
constexpr int point_arity() { return D == 0 ? 3 : D; }

template <int D>
__device__ __forceinline__ void load_point(const double* __restrict__ p, double (&x)[D]) {
    if constexpr (D == 2) {
        const double2 v = *(const double2*)p;
        x[0] = v.x;
        x[1] = v.y;
    } else {
#pragma unroll
        for (int k = 0; k < D; ++k) x[k] = p[k];
    }
}

// a point of runtime dimension dim (1..3) as 3 coordinates (the missing ones read 0 from a table,
// branch-free)
__device__ __forceinline__ void load_point_rt(const double* __restrict__ p, int dim, double (&x)[3]) {
#pragma unroll
    for (int k = 0; k < 3; ++k) x[k] = *(k < dim ? p + k : kZeroValue);
}

// squared distance for the covariance, floored at 2^-1000 (nngp_d2's order for D = 2:
// the last coordinate first, each term one FMA)
template <int D>
__device__ __forceinline__ double point_d2(const double (&a)[D], const double (&b)[D]) {
    double acc = NNGP_D2_FLOOR;
#pragma unroll
    for (int k = D - 1; k >= 0; --k) {
        const double t = a[k] - b[k];
        acc = fma(t, t, acc);
    }
    return acc;
}

constexpr int kAlgoAuto = 0;
constexpr int kAlgoLane = 1;
constexpr int kAlgoWave = 2;
// (3 was the two-lane bf_group and 7 the round-1 bf_pairb: comparison kernels, no longer built)
constexpr int kAlgoQuad = 4;  // bf_group, 4 lanes per location (m = 25..32, 2-D exponential / Matern-3/2)
constexpr int kAlgoPairB = 5; // bf_pairb, 2 lanes per location, 2x2-blocked elimination (m = 1..32)
constexpr int kLaneMaxM = 16;

struct BfArgs {
    const double* coords;  // (n_points, dim) row-major
    int64_t n_points;
    const int32_t* nbr;  // (n_rows, m), -1 padded; row t is location i0 + (order ? order[t] : t)
    int64_t n_rows;
    int64_t i0;
    int m;
    int kind;
    int dim;                   // coordinate dimension (1..3)
    double sigma2, phi, tau2;
    double nu;                 // smoothness of NNGP_KIND_MATERN (unused by the other kinds)
    const int32_t* order;      // (n_rows,) local row of nbr row t (nngp_row_order layout), or null (identity)
    const double* values;      // (n_points,) or null
    const double* qcoords;     // coordinates of the locations themselves: coords (sweep) or query points (cross)
    const double* qvalues;     // values at the locations: values (sweep), query values or null (cross)
    double* B;                 // (n_rows, m) or null
    double* F;                 // (n_rows,) or null
    double* R;                 // (n_rows,) residuals v_i - B_i v_N(i), or null
    double* partials;          // [4]
    double* bpart;             // 4 doubles per block: sum log F, sum r^2/F, first bad-pivot row, first bad-index row
    const double* cblk = nullptr;  // NNGP_KIND_BLOCKS: the joint blocks' covariances (bf_pairb.h), entry-major
    // pair kernel, planned sweeps (pair_plan.h): sweep only the n_tile_list tiles listed in `tiles` (of
    // n_tiles in all), or, for the planned launch, n_plan_blocks regions of the plan
    const int32_t* tiles = nullptr;
    int64_t n_tiles = 0, n_tile_list = 0, n_plan_blocks = 0;
};

int64_t bf_record_count(int64_t n_rows, int algo, int m);
hipError_t bf_finalize_launch(const double* bpart, int64_t n_records, double* partials, hipStream_t s);
hipError_t bf_finalize_pairb_launch(void* ws, int64_t n_rows, double* partials, hipStream_t s);
hipError_t bf_launch(const BfArgs& a, int algo, hipStream_t s);
hipError_t combine_partials_launch(const double* gathered, int world, int64_t n_slots, double* out, hipStream_t s);
bool bf_wave_launch(const BfArgs& a, const CovParams& P, int64_t n_blocks, hipStream_t s);
bool bf_group_launch(const BfArgs& a, const CovParams& P, int lanes, hipStream_t s);
bool bf_group_supported(int m, int lanes);
bool bf_pairb_launch(const BfArgs& a, const CovParams& P, hipStream_t s);
bool bf_pairb_supported(int m);
bool bf_pairb_blocks_launch(const BfArgs& a, hipStream_t s);  // NNGP_KIND_BLOCKS (bf_pairb.h)
// wave pair plans (pair_plan.h, pair_plan.hip)
bool bf_pairb_planned_supported(int m, int kind, int dim);
bool bf_pairb_planned_launch(const BfArgs& a, const CovParams& P, const PlanLaunch& pl, hipStream_t s);
hipError_t bf_launch_planned(const BfArgs& a, const PlanLaunch& pl, hipStream_t s);
size_t pair_plan_build_lds(int m);
hipError_t pair_plan_build_launch(const int32_t* nbr, const int32_t* order, int64_t n_rows, int m, int dim, int64_t i0,
                                  int64_t n_points, int64_t tq, int64_t trem, void* plan, hipStream_t s);
bool bf_pairb_blocks_supported(int m);
bool bf_group_blocks_launch(const BfArgs& a, hipStream_t s);  // NNGP_KIND_BLOCKS at m = 25..32 (bf_group.h)
bool bf_group_blocks_supported(int m);
hipError_t matern_table_launch(const CovParams& P, double* tab, hipStream_t s);  // matern_table.hip
bool matern_table_extent(double nu, int* e0, int* noct);  // false: more than NNGP_MT_MAX_OCT octaves
bool matern_table_params(double nu, CovParams* p);        // ... and the below-table series (mt_series, mt_A)
hipError_t matern_eval_launch(const double* u, int64_t n, double nu, double* out, hipStream_t s);
hipError_t joint_dist_launch(const double* coords, int64_t n_points, int dim, const double* qcoords,
                             const int32_t* nbr, const int32_t* order, int64_t n_rows, int m, int64_t i0, double* dist,
                             hipStream_t s);
// number of 256-thread blocks (= partial records) each kernel launches for n_rows
int64_t bf_group_blocks(int64_t n_rows, int lanes);
int64_t bf_lane_blocks(int64_t n_rows);
int64_t bf_wave_blocks(int64_t n_rows);

constexpr int kKnnMaxLevels = 16;
// one grid over the prefix s[0:np] of the points (level 0: all of them)
struct KnnLevel {
    int64_t np;       // points in the prefix
    int g;            // grid side (g^dim cells over the common bounding box)
    int64_t n_cells;  // g * g
    size_t off_idx_sorted, off_pts_sorted, off_cell_start;  // byte offsets into the workspace
};
struct KnnPlan {
    int64_t n_points;
    int dim;          // coordinate dimension (1..3)
    int g;            // level 0 grid side (g^dim cells)
    int64_t n_cells;  // level 0 cells
    int n_levels;
    KnnLevel lv[kKnnMaxLevels];
    size_t sort_temp_bytes;
    size_t total_bytes;
    // byte offsets into the workspace (level 0's arrays are lv[0].off_*)
    size_t off_bbox, off_key, off_key_sorted, off_sort_temp, off_idx, off_perm;
};

hipError_t knn_plan(int64_t n_points, int dim, KnnPlan* plan);
// prior mode: rows [q0, q1) of coords against coords[0:i]; query mode: query[q0:q1] against all coords
// rows: NULL, or (prior mode) the point index of each of the q1 - q0 query rows
hipError_t knn_launch(bool prior, const double* coords, int64_t n_points, int m, const double* query, int64_t q0,
                      int64_t q1, const int32_t* rows, int32_t* nbr, void* workspace, const KnnPlan& plan,
                      hipStream_t s);

// Gibbs sampler (gibbs.hip)
size_t reverse_workspace_bytes(int64_t n, int m);
hipError_t reverse_launch(const int32_t* nbr, int64_t n, int m, int32_t* off, int32_t* rev_j, int32_t* rev_k,
                          void* workspace, hipStream_t s);
int64_t color_moral_graph_host(const int32_t* nbr, const int32_t* off, const int32_t* rev_j, int64_t n, int m,
                               int32_t* color);
int64_t color_moral_graph_device(const int32_t* nbr, const int32_t* off, const int32_t* rev_j, int64_t n, int m,
                                 int32_t* color, void* workspace, hipStream_t s, hipError_t* err);
size_t gibbs_prep_bytes(int64_t n, int m);
hipError_t philox_normals_launch(int64_t n, uint64_t seed, uint64_t sweep, double* z, hipStream_t s);
hipError_t gibbs_prepare_launch(const double* B, const double* Ft, const int32_t* off, const int32_t* rev_j,
                                const int32_t* rev_k, const int32_t* order, int64_t n, int m, void* prep,
                                hipStream_t s);
hipError_t gibbs_prepare_range_launch(const double* B, const double* Ft, const int32_t* off, const int32_t* rev_j,
                                      const int32_t* rev_k, int64_t n, int m, int64_t row0, int64_t row1, void* prep,
                                      hipStream_t s);
hipError_t gibbs_w_color_launch(const int32_t* member_rows, int64_t n_members, const void* prep, int64_t n, int m,
                                double sigma2, double tau2, const double* yres, const double* noise_w, double* w,
                                double* r, const int32_t* rev_j, const double* z, uint64_t seed, uint64_t sweep,
                                double* w_out, const double* var, hipStream_t s);
hipError_t gibbs_w_apply_launch(const int32_t* rows, int64_t n_rows, const double* wsrc, const double* B, int m,
                                double* w, double* r, const int32_t* rev_j, const int32_t* rev_k, hipStream_t s);
hipError_t gibbs_member_rows_launch(const int32_t* members, int64_t n, const int32_t* off, int32_t* rows,
                                    hipStream_t s);
hipError_t gibbs_tile_sweep_launch(const int32_t* tiles, const int32_t* phase_off_host, const int32_t* phase_lds_host,
                                   int n_phases, const int32_t* tinfo, const int32_t* tstep, int ecap,
                                   const int32_t* tfp, const int32_t* off, const int32_t* rev_loc, const void* prep,
                                   int64_t n, int m, int64_t n_entries, double sigma2, double tau2,
                                   const double* yres, const double* noise_w, double* w, double* r, const double* z,
                                   hipStream_t s);
hipError_t gibbs_w_sweep_launch(const int32_t* member_rows, int n_colors, const int32_t* color_off_host,
                                const void* prep, int64_t n, int m, double sigma2, double tau2,
                                const double* yres, const double* noise_w, double* w, double* r,
                                const int32_t* rev_j, const double* z, uint64_t seed, uint64_t sweep, hipStream_t s);
hipError_t gibbs_w_sweep_chains_launch(const int32_t* member_rows, int n_colors, const int32_t* color_off_host,
                                       int chains, const void* const* preps, int64_t n, int m, const double* sigma2,
                                       const double* tau2, const double* const* yres, const double* noise_w,
                                       double* const* w, double* const* r, const int32_t* rev_j,
                                       const double* const* z, hipStream_t s, double* w_il = nullptr,
                                       double* r_il = nullptr);
size_t gibbs_stats_workspace_bytes(int64_t n, int p);
hipError_t gibbs_stats_launch(int64_t n, const double* r, const double* Ft, const double* yres, const double* y,
                              const double* X, int p, const double* w, const double* noise_w, double* out,
                              void* workspace, hipStream_t s);

// row-order plan (nngp_row_order): Morton-sorted local rows for cache locality
size_t row_order_workspace_bytes(int64_t n_rows);
hipError_t row_order_launch(const double* coords, int dim, int64_t i0, int64_t n_rows, int32_t* order,
                            const int32_t* nbr, int m, int32_t* nbr_sorted, void* workspace, size_t workspace_bytes,
                            hipStream_t s);

// Bijective XCD-aware block remap: blocks are dealt round-robin over the 8 XCDs
// (b % 8 shares an L2), so give each XCD a contiguous range of logical blocks;
// with Morton-ordered rows that keeps one XCD's gathers inside one spatial region
// (its own L2).  Speed only: any placement gives identical results.
__device__ __forceinline__ int64_t xcd_logical_block(int64_t b, int64_t nb) {
    const int64_t q = nb / 8, r = nb % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// ---------------------------------------------------------------- wave helpers
__device__ __forceinline__ double wave_bcast(double v, int lane) {
    const long long u = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(u & 0xffffffffll), lane);
    const int hi = __builtin_amdgcn_readlane((int)(u >> 32), lane);
    return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
    return v;
}

// Fixed-order reduction of one 256-thread block's (log F, r^2/F) sums and of its
// first bad-pivot / bad-index rows (INFINITY = none) into bpart[4 * block ..].
// Every thread of the block must call it (it synchronises the block).  No global
// atomics and no pre-initialised status words: bf_finalize folds the records.
__device__ __forceinline__ void block_partials_store(double lf, double q, double badp, double badi, double* bpart,
                                                     int64_t block) {
    __shared__ double sh[4][4];
    lf = wave_sum(lf);
    q = wave_sum(q);
    if (__any(badp != INFINITY || badi != INFINITY)) {  // wave-uniform; rare
        badp = wave_min(badp);
        badi = wave_min(badi);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sh[w][0] = lf;
        sh[w][1] = q;
        sh[w][2] = badp;
        sh[w][3] = badi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double a = 0.0, b = 0.0, c = INFINITY, d = INFINITY;
        for (int k = 0; k < (int)(blockDim.x >> 6); ++k) {
            a += sh[k][0];
            b += sh[k][1];
            c = fmin(c, sh[k][2]);
            d = fmin(d, sh[k][3]);
        }
        double* o = bpart + 4 * block;
        o[0] = a;
        o[1] = b;
        o[2] = c;
        o[3] = d;
    }
}

}  // namespace nngp
