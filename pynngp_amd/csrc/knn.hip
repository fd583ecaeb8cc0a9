// Exact ordered prior-neighbour sets on gfx950, ordinates of dimension D = 1, 2, 3.
//
// Reference: NNGP._make_s_neighbor_sets, pyNNGP/nngp.py:49-62 -- for every i the
// k = min(m, i) nearest points among s[0:i], ascending distance, self excluded
// (a fresh sklearn KDTree over s[0:i] per i: O(N^2 log N); the KDTree takes
// ordinates of any dimension).  sklearn 1.7.2 orders by the fp64 reduced distance
// rdist = ((0 + t0*t0) + t1*t1) + ..., t = s_i - s_j, no FMA
// (sklearn/metrics/_dist_metrics.pxd:26-40); sort_results=True
// (sklearn/neighbors/_binary_tree.pxi.tp:1088,1188).  Here: the same key in the same
// order with contraction disabled, exact ties broken by lower index.
//
// Method: a uniform grid of g^D cells over the bounding box, points radix-sorted by
// (cell, index) so each cell's prior points j < i form a prefix.  One lane per
// query i scans Chebyshev shells of cells around its own cell, keeping the k best
// (rdist, j) in a register-resident sorted list, and stops when the k-th best
// rdist is below the squared distance to the unscanned region (minus a slack
// that covers cell-assignment rounding).  Levels: grid L covers only the prefix
// s[0:n/4^L] (2 points per cell of ITS prefix), and query i scans the grid of the
// smallest prefix holding all of s[0:i] -- its prior points fill >= 1/4 of that
// prefix, so a few dozen cells suffice at every i (one full-density grid made early,
// sparse-prior queries scan thousands of cells: 7.2 ms at N = 1e6, m = 15, all of it
// the slowest waves).  Queries with i < kBruteBelow scan s[0:i] directly.
// Query order (prior mode): lanes of a wave take queries sorted by (floor(log2 i),
// Morton code of the cell), so they have similar prior densities (similar ring counts,
// little divergence) AND neighbouring cells (shared cell-list and point lines in L1/L2);
// each query still writes its own output row.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <math.h>
#include <stdint.h>

#include "geom.h"
#include "nngp_internal.h"

namespace nngp {

constexpr double kPointsPerCell = 2.0;
constexpr int64_t kBruteBelow = 1024;      // prior queries i < this: brute force over s[0:i]
constexpr int64_t kLevelMinPoints = 4096;  // no grid level over fewer points than this

struct KnnLevels {  // kernel-argument view of the plan's grids
    int n;
    int64_t np[kKnnMaxLevels];
    int g[kKnnMaxLevels];
    const int32_t* cell_start[kKnnMaxLevels];
    const int32_t* idx_sorted[kKnnMaxLevels];
    const double* pts_sorted[kKnnMaxLevels];  // (np, D) in cell order
};

// g cells per axis over the bounding box (degenerate axes get unit width)
template <int D>
struct GridD {
    double lo[D], w[D], iv[D];
    int g;
};

template <int D>
__device__ __forceinline__ GridD<D> make_grid(const Bbox& b, int g) {
    GridD<D> G;
    G.g = g;
#pragma unroll
    for (int k = 0; k < D; ++k) {
        double r = b.hi[k] - b.lo[k];
        if (!(r > 0.0)) r = 1.0;
        G.lo[k] = b.lo[k];
        G.w[k] = r / g;
        G.iv[k] = g / r;
    }
    return G;
}

__device__ __forceinline__ int cell_coord(double v, double lo, double iv, int g) {
    double t = floor((v - lo) * iv);
    int c = (int)fmin(fmax(t, 0.0), (double)(g - 1));
    return c;
}

template <int D>
__device__ __forceinline__ int64_t cell_linear(const int (&c)[D], int g) {
    int64_t key = 0;
#pragma unroll
    for (int k = D - 1; k >= 0; --k) key = key * g + c[k];  // axis 0 fastest
    return key;
}

template <int D>
__global__ __launch_bounds__(256) void cell_keys(const double* __restrict__ p, int64_t n, const Bbox* __restrict__ box,
                                                 int g, uint32_t* __restrict__ key, int32_t* __restrict__ idx) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const GridD<D> G = make_grid<D>(*box, g);
    double x[D];
    load_point<D>(p + t * D, x);
    int c[D];
#pragma unroll
    for (int k = 0; k < D; ++k) c[k] = cell_coord(x[k], G.lo[k], G.iv[k], g);
    key[t] = (uint32_t)cell_linear<D>(c, g);
    idx[t] = (int32_t)t;
}

// cell_start[c] = first sorted position with key >= c, for c in [0, n_cells]
__global__ __launch_bounds__(256) void cell_bounds(const uint32_t* __restrict__ key_sorted, int64_t n, int64_t n_cells,
                                                   int32_t* __restrict__ cell_start) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c > n_cells) return;
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if ((int64_t)key_sorted[mid] < c)
            lo = mid + 1;
        else
            hi = mid;
    }
    cell_start[c] = (int32_t)lo;
}

template <int D>
__global__ __launch_bounds__(256) void gather_sorted(const double* __restrict__ p, const int32_t* __restrict__ idx_sorted,
                                                     int64_t n, double* __restrict__ pts_sorted) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const int64_t j = idx_sorted[t];
#pragma unroll
    for (int k = 0; k < D; ++k) pts_sorted[t * D + k] = p[j * D + k];
}

// sort key of query position t (prior mode): log2 band of the point index, then the
// Morton code of its cell coarsened by `shift` bits per axis (band in the top 5 bits)
template <int D>
__global__ __launch_bounds__(256) void query_keys(const double* __restrict__ p, int64_t q0, int64_t nq,
                                                  const int32_t* __restrict__ rows, const Bbox* __restrict__ box,
                                                  int g, int shift, uint32_t* __restrict__ key,
                                                  int32_t* __restrict__ pos) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nq) return;
    const int64_t i = rows != nullptr ? (int64_t)rows[t] : q0 + t;
    const GridD<D> G = make_grid<D>(*box, g);
    double x[D];
    load_point<D>(p + i * D, x);
    uint32_t c[D];
#pragma unroll
    for (int k = 0; k < D; ++k) c[k] = (uint32_t)cell_coord(x[k], G.lo[k], G.iv[k], g) >> shift;
    const uint32_t band = 31u - (uint32_t)__clz((unsigned)(i + 1));  // floor(log2(i + 1)) <= 31
    key[t] = (band << 27) | (morton<D>(c) & ((1u << 27) - 1));
    pos[t] = (int32_t)t;
}

// sklearn euclidean_rdist64 without contraction: d = 0; d += t_k * t_k, k = 0 .. D-1.  The
// pragma is what keeps it that way: hipcc's default -ffp-contract=fast-honor-pragmas turns
// t0*t0 + t1*t1 into one v_fmac_f64 (even through __dmul_rn / __dadd_rn, which are plain *
// and + in this ROCm's headers), and that rounds differently from sklearn's sum on
// near-ties (tests/test_gpu_knn.py::test_knn_fma_sensitive_ties).
template <int D>
__device__ __forceinline__ double rdist(const double (&q)[D], const double* __restrict__ p) {
#pragma clang fp contract(off)
    double d = 0.0;
#pragma unroll
    for (int k = 0; k < D; ++k) {
        const double t = q[k] - p[k];
        d = d + t * t;
    }
    return d;
}

__device__ __forceinline__ bool key_less(double da, int32_t ia, double db, int32_t ib) {
    return da < db || (da == db && ia < ib);
}

// Sorted list of the KMAX slots; real entries occupy [KMAX-k, KMAX), the slots
// below hold (-inf, -1) sentinels that never move, so the worst kept entry is
// always slot KMAX-1 (static register indexing throughout).
template <int KMAX>
struct TopK {
    double d[KMAX];
    int32_t j[KMAX];
    __device__ __forceinline__ void init(int k) {
#pragma unroll
        for (int s = 0; s < KMAX; ++s) {
            const bool real = s >= KMAX - k;
            d[s] = real ? INFINITY : -INFINITY;
            j[s] = real ? INT32_MAX : -1;
        }
    }
    __device__ __forceinline__ void push(double dc, int32_t jc) {
        if (!key_less(dc, jc, d[KMAX - 1], j[KMAX - 1])) return;
#pragma unroll
        for (int s = KMAX - 1; s > 0; --s) {
            const bool below = key_less(dc, jc, d[s - 1], j[s - 1]);
            const bool here = !below && key_less(dc, jc, d[s], j[s]);
            const double nd = below ? d[s - 1] : (here ? dc : d[s]);
            const int32_t nj = below ? j[s - 1] : (here ? jc : j[s]);
            d[s] = nd;
            j[s] = nj;
        }
        if (key_less(dc, jc, d[0], j[0])) {
            d[0] = dc;
            j[0] = jc;
        }
    }
};

// PRIOR: query row t is reference point i = q0 + t, candidates j < i, k = min(i, m).
// !PRIOR: query row t is query[t], every reference point is a candidate, k = min(m, n).
// Cells are scanned in Chebyshev shells r = 0, 1, ... around the query's cell (in D = 3 the
// shell's faces in the two outer axes are scanned whole, its inside rows only at x = +-r).
template <int KMAX, bool PRIOR, int D>
__global__ __launch_bounds__(256) void knn_query_kernel(const double* __restrict__ coords, int64_t n, int m,
                                                        const double* __restrict__ query, int64_t q0, int64_t q1,
                                                        const int32_t* __restrict__ rows,
                                                        const int32_t* __restrict__ perm,
                                                        int64_t brute_below, const Bbox* __restrict__ box,
                                                        const KnnLevels lv, int32_t* __restrict__ nbr) {
    const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q0 + u >= q1) return;
    const int64_t t = perm != nullptr ? (int64_t)perm[u] : u;       // query position (output row)
    const int64_t i = rows != nullptr ? (int64_t)rows[t] : q0 + t;  // PRIOR with a row list: query row t is point rows[t]
    const int64_t limit = PRIOR ? i : n;  // candidates are reference points j < limit
    const int k = (int)(limit < m ? limit : m);
    int32_t* out = nbr + t * m;
    if (k == 0) {
        for (int s = 0; s < m; ++s) out[s] = -1;
        return;
    }
    double q[D];
    load_point<D>((PRIOR ? coords : query) + i * D, q);
    TopK<KMAX> top;
    top.init(k);
    if (PRIOR && i < brute_below) {
        for (int64_t jj = 0; jj < i; ++jj) top.push(rdist<D>(q, coords + jj * D), (int32_t)jj);
    } else {
        // the smallest prefix grid holding every candidate (prior: s[0:i]; query mode: level 0)
        int L = 0;
        if (PRIOR) {
#pragma unroll 1
            for (int l = lv.n - 1; l > 0; --l)
                if (lv.np[l] >= i) {
                    L = l;
                    break;
                }
        }
        const int g = lv.g[L];
        const int32_t* __restrict__ cell_start = lv.cell_start[L];
        const int32_t* __restrict__ idx_sorted = lv.idx_sorted[L];
        const double* __restrict__ pts_sorted = lv.pts_sorted[L];
        const GridD<D> G = make_grid<D>(*box, g);
        int cq[D];
        double slack = 0.0;
#pragma unroll
        for (int a = 0; a < D; ++a) {
            cq[a] = cell_coord(q[a], G.lo[a], G.iv[a], g);
            slack += 1e-7 * G.w[a] + 1e-13 * (fabs(G.lo[a]) + fabs(G.lo[a] + g * G.w[a]));
        }
        int64_t found = 0;
        const int32_t lim = (int32_t)(limit < INT32_MAX ? limit : INT32_MAX);
        auto scan_cell = [&](int64_t c) {
            const int32_t e = cell_start[c + 1];
            for (int32_t pp = cell_start[c]; pp < e; ++pp) {
                const int32_t jj = idx_sorted[pp];
                if (PRIOR && jj >= lim) break;  // (cell, index) order: the rest are not prior
                top.push(rdist<D>(q, pts_sorted + (int64_t)pp * D), jj);
                ++found;
            }
        };
        // scan the x-run [x0, x1] of cells in the row whose outer coordinates are `outer`
        auto scan_run = [&](int64_t row_base, int x0, int x1, int step) {
            for (int xx = x0; xx <= x1; xx += step) {
                if (xx < 0 || xx >= g) continue;
                scan_cell(row_base + xx);
            }
        };
        for (int r = 0; r <= g; ++r) {
            const int cx = cq[0];
            if constexpr (D == 1) {
                scan_run(0, cx - r, cx + r, r == 0 ? 1 : 2 * r);
            } else if constexpr (D == 2) {
                const int cy = cq[1];
                const int y0 = cy - r, y1 = cy + r;
                for (int yy = (y0 < 0 ? 0 : y0); yy <= (y1 < g ? y1 : g - 1); ++yy) {
                    const bool face = (yy == y0) || (yy == y1);
                    scan_run((int64_t)yy * g, cx - r, cx + r, (face || r == 0) ? 1 : 2 * r);
                }
            } else {
                const int cy = cq[1], cz = cq[2];
                const int z0 = cz - r, z1 = cz + r, y0 = cy - r, y1 = cy + r;
                for (int zz = (z0 < 0 ? 0 : z0); zz <= (z1 < g ? z1 : g - 1); ++zz) {
                    for (int yy = (y0 < 0 ? 0 : y0); yy <= (y1 < g ? y1 : g - 1); ++yy) {
                        const bool face = zz == z0 || zz == z1 || yy == y0 || yy == y1;
                        scan_run(((int64_t)zz * g + yy) * g, cx - r, cx + r, (face || r == 0) ? 1 : 2 * r);
                    }
                }
            }
            // distance from q to the region outside the scanned box of cells
            double bnd = INFINITY;
#pragma unroll
            for (int a = 0; a < D; ++a) {
                if (cq[a] - r > 0) bnd = fmin(bnd, q[a] - (G.lo[a] + (cq[a] - r) * G.w[a]));
                if (cq[a] + r < g - 1) bnd = fmin(bnd, (G.lo[a] + (cq[a] + r + 1) * G.w[a]) - q[a]);
            }
            if (bnd == INFINITY) break;  // whole grid scanned
            if (found >= k) {
                const double b = bnd - slack;
                if (b > 0.0 && top.d[KMAX - 1] < b * b * (1.0 - 1e-12)) break;
            }
        }
    }
#pragma unroll
    for (int s = 0; s < KMAX; ++s) {
        const int o = s - (KMAX - k);
        if (o >= 0) out[o] = top.j[s];
    }
    for (int s = k; s < m; ++s) out[s] = -1;
}

// cells per axis for np points at ~kPointsPerCell points per cell, keeping g^D < 2^31
static int grid_side(int64_t n, int dim) {
    double g = ceil(pow((double)n / kPointsPerCell, 1.0 / dim));
    const double cap = dim == 1 ? 1073741824.0 : (dim == 2 ? 46340.0 : 1290.0);
    if (g < 1.0) g = 1.0;
    if (g > cap) g = cap;
    return (int)g;
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

hipError_t knn_plan(int64_t n_points, int dim, KnnPlan* plan) {
    if (dim < 1 || dim > kMaxDim) return hipErrorInvalidValue;
    KnnPlan p{};
    p.n_points = n_points;
    p.dim = dim;
    // levels: prefixes n, n/4, n/16, ... down to kLevelMinPoints
    p.n_levels = 0;
    for (int64_t np = n_points; p.n_levels < kKnnMaxLevels; np = (np + 3) / 4) {
        KnnLevel& L = p.lv[p.n_levels++];
        L.np = np;
        L.g = grid_side(np, dim);
        L.n_cells = 1;
        for (int k = 0; k < dim; ++k) L.n_cells *= L.g;
        if ((np + 3) / 4 < kLevelMinPoints) break;
    }
    p.g = p.lv[0].g;
    p.n_cells = p.lv[0].n_cells;
    unsigned bits = 1;
    while ((1ll << bits) < p.n_cells) ++bits;
    size_t tb = 0, tq = 0;
    hipError_t e = rocprim::radix_sort_pairs((void*)nullptr, tb, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                             (const int32_t*)nullptr, (int32_t*)nullptr, (size_t)n_points, 0u, bits);
    if (e != hipSuccess) return e;
    e = rocprim::radix_sort_pairs((void*)nullptr, tq, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                  (const int32_t*)nullptr, (int32_t*)nullptr, (size_t)n_points, 0u, 32u);
    if (e != hipSuccess) return e;
    if (tq > tb) tb = tq;
    p.sort_temp_bytes = tb;
    size_t off = 0;
    p.off_bbox = off;
    off += align256(sizeof(double) * (2 * kMaxDim * 256 + 2 * kMaxDim + 8));
    p.off_key = off;
    off += align256(sizeof(uint32_t) * n_points);
    p.off_key_sorted = off;
    off += align256(sizeof(uint32_t) * n_points);
    p.off_idx = off;
    off += align256(sizeof(int32_t) * n_points);
    for (int l = 0; l < p.n_levels; ++l) {
        KnnLevel& L = p.lv[l];
        L.off_idx_sorted = off;
        off += align256(sizeof(int32_t) * L.np);
        L.off_pts_sorted = off;
        off += align256(dim * sizeof(double) * L.np);
        L.off_cell_start = off;
        off += align256(sizeof(int32_t) * (L.n_cells + 1));
    }
    p.off_perm = off;
    off += align256(sizeof(int32_t) * n_points);
    p.off_sort_temp = off;
    off += align256(tb);
    p.total_bytes = off;
    *plan = p;
    return hipSuccess;
}

template <int KMAX, int D>
static void launch_query(bool prior, const double* coords, int64_t n, int m, const double* query, int64_t q0,
                         int64_t q1, const int32_t* rows, const int32_t* perm, int64_t brute_below, const Bbox* box,
                         const KnnLevels& lv, int32_t* nbr, hipStream_t s) {
    const dim3 grid((unsigned)((q1 - q0 + 255) / 256)), block(256);
    if (prior)
        hipLaunchKernelGGL((knn_query_kernel<KMAX, true, D>), grid, block, 0, s, coords, n, m, query, q0, q1, rows,
                           perm, brute_below, box, lv, nbr);
    else
        hipLaunchKernelGGL((knn_query_kernel<KMAX, false, D>), grid, block, 0, s, coords, n, m, query, q0, q1, rows,
                           perm, brute_below, box, lv, nbr);
}

template <int D>
static hipError_t knn_launch_d(bool prior, const double* coords, int64_t n, int m, const double* query, int64_t q0,
                               int64_t q1, const int32_t* rows, int32_t* nbr, void* workspace, const KnnPlan& pl,
                               hipStream_t s) {
    char* w = (char*)workspace;
    double* bpart = (double*)(w + pl.off_bbox);
    Bbox* box = (Bbox*)(bpart + 2 * kMaxDim * 256);
    uint32_t* key = (uint32_t*)(w + pl.off_key);
    uint32_t* key_sorted = (uint32_t*)(w + pl.off_key_sorted);
    int32_t* idx = (int32_t*)(w + pl.off_idx);
    void* temp = (void*)(w + pl.off_sort_temp);

    hipLaunchKernelGGL((bbox_partial<D>), dim3(256), dim3(256), 0, s, coords, n, bpart);
    hipLaunchKernelGGL((bbox_final<D>), dim3(1), dim3(64), 0, s, bpart, 256, box);
    // one grid per level over the prefix s[0:np] (query mode only needs level 0); every
    // level shares the bounding box and the key / key_sorted / idx scratch
    KnnLevels lv{};
    lv.n = prior ? pl.n_levels : 1;
    hipError_t e = hipSuccess;
    for (int l = 0; l < lv.n; ++l) {
        const KnnLevel& L = pl.lv[l];
        int32_t* idx_sorted = (int32_t*)(w + L.off_idx_sorted);
        double* pts_sorted = (double*)(w + L.off_pts_sorted);
        int32_t* cell_start = (int32_t*)(w + L.off_cell_start);
        const unsigned nb = (unsigned)((L.np + 255) / 256);
        hipLaunchKernelGGL((cell_keys<D>), dim3(nb), dim3(256), 0, s, coords, L.np, box, L.g, key, idx);
        unsigned bits = 1;
        while ((1ll << bits) < L.n_cells) ++bits;
        size_t tb = pl.sort_temp_bytes;
        e = rocprim::radix_sort_pairs(temp, tb, key, key_sorted, idx, idx_sorted, (size_t)L.np, 0u, bits, s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(cell_bounds, dim3((unsigned)((L.n_cells + 1 + 255) / 256)), dim3(256), 0, s, key_sorted,
                           L.np, L.n_cells, cell_start);
        hipLaunchKernelGGL((gather_sorted<D>), dim3(nb), dim3(256), 0, s, coords, idx_sorted, L.np, pts_sorted);
        lv.np[l] = L.np;
        lv.g[l] = L.g;
        lv.cell_start[l] = cell_start;
        lv.idx_sorted[l] = idx_sorted;
        lv.pts_sorted[l] = pts_sorted;
    }
    // brute force where scanning s[0:i] is cheaper than any grid
    int64_t brute_below = kBruteBelow > 8 * (int64_t)m ? kBruteBelow : 8 * (int64_t)m;
    // prior mode: visit the queries in (log2 band, cell Morton) order (speed only); the cell
    // sorts' key / key_sorted / idx scratch is free again
    const int32_t* perm = nullptr;
    const int64_t nq = q1 - q0;
    if (prior && nq > 1 && nq <= n) {
        int cb = 1;
        while ((1 << cb) < pl.g && cb < 30) ++cb;
        const int per_axis = 27 / D;  // 27 Morton bits + 5 band bits fit 32
        const int shift = cb > per_axis ? cb - per_axis : 0;
        int32_t* pos = (int32_t*)(w + pl.off_perm);
        hipLaunchKernelGGL((query_keys<D>), dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, s, coords, q0, nq, rows,
                           box, pl.g, shift, key, idx);
        size_t tq = pl.sort_temp_bytes;
        e = rocprim::radix_sort_pairs(temp, tq, key, key_sorted, idx, pos, (size_t)nq, 0u, 32u, s);
        if (e != hipSuccess) return e;
        perm = pos;
    }
#define NNGP_Q(KM) launch_query<KM, D>(prior, coords, n, m, query, q0, q1, rows, perm, brute_below, box, lv, nbr, s)
    if (m <= 8)
        NNGP_Q(8);
    else if (m <= 16)
        NNGP_Q(16);
    else if (m <= 24)
        NNGP_Q(24);
    else if (m <= 32)
        NNGP_Q(32);
    else if (m <= 64)
        NNGP_Q(64);
    else
        return hipErrorInvalidValue;
#undef NNGP_Q
    return hipGetLastError();
}

hipError_t knn_launch(bool prior, const double* coords, int64_t n, int m, const double* query, int64_t q0, int64_t q1,
                      const int32_t* rows, int32_t* nbr, void* workspace, const KnnPlan& pl, hipStream_t s) {
    switch (pl.dim) {
        case 1: return knn_launch_d<1>(prior, coords, n, m, query, q0, q1, rows, nbr, workspace, pl, s);
        case 2: return knn_launch_d<2>(prior, coords, n, m, query, q0, q1, rows, nbr, workspace, pl, s);
        case 3: return knn_launch_d<3>(prior, coords, n, m, query, q0, q1, rows, nbr, workspace, pl, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace nngp
