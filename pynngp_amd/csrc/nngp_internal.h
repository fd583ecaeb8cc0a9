// Internal declarations shared by the HIP translation units of libnngp_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nngp_math.h"

namespace nngp {

// Invalid neighbour slots (index -1) are moved "infinitely" far away: slot a sits
// at (kFar * (a + 1), 0), so every covariance involving it is sigma2 * 2^-(huge) = 0
// (ldexp underflow) and its row/column of the joint block is a decoupled diagonal
// entry.  That keeps the pair loops free of per-entry selects; B is zeroed at the
// store.  (kFar * 64)^2 stays finite.
constexpr double kFar = 1e150;

constexpr int kAlgoAuto = 0;
constexpr int kAlgoLane = 1;
constexpr int kAlgoWave = 2;
constexpr int kLaneMaxM = 16;

struct BfArgs {
    const double* coords;  // (n_points, 2) row-major
    int64_t n_points;
    const int32_t* nbr;  // (n_rows, m), -1 padded; row r is location i0 + r
    int64_t n_rows;
    int64_t i0;
    int m;
    int kind;
    double sigma2, phi, tau2;
    const double* values;      // (n_points,) or null
    double* B;                 // (n_rows, m) or null
    double* F;                 // (n_rows,) or null
    double* partials;          // [4]
    double* wpart;             // 2 doubles per wave
    unsigned long long* status;  // [2], preset to ~0
};

hipError_t bf_launch(const BfArgs& a, int algo, hipStream_t s);
bool bf_wave_launch(const BfArgs& a, const CovParams& P, int64_t n_waves, hipStream_t s);
int64_t bf_lane_waves(int64_t n_rows);
int64_t bf_wave_waves(int64_t n_rows);

struct KnnPlan {
    int64_t n_points;
    int gx, gy;
    int64_t n_cells;
    size_t sort_temp_bytes;
    size_t total_bytes;
    // byte offsets into the workspace
    size_t off_bbox, off_key, off_key_sorted, off_idx_sorted, off_pts_sorted, off_cell_start, off_sort_temp, off_idx;
};

hipError_t knn_plan(int64_t n_points, KnnPlan* plan);
// prior mode: rows [q0, q1) of coords against coords[0:i]; query mode: query[q0:q1] against all coords
hipError_t knn_launch(bool prior, const double* coords, int64_t n_points, int m, const double* query, int64_t q0,
                      int64_t q1, int32_t* nbr, void* workspace, const KnnPlan& plan, hipStream_t s);

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

// Fixed-order wave reduction of (lf, q); lane 0 stores them at slot (thread >> 6).
__device__ __forceinline__ void wave_partials_store(double lf, double q, double* wpart, int64_t thread) {
    lf = wave_sum(lf);
    q = wave_sum(q);
    if ((threadIdx.x & 63) == 0) {
        const int64_t w = thread >> 6;
        wpart[2 * w] = lf;
        wpart[2 * w + 1] = q;
    }
}

}  // namespace nngp
