// Exact ordered prior-neighbour sets on gfx950.
//
// Reference: NNGP._make_s_neighbor_sets, pyNNGP/nngp.py:49-62 -- for every i the
// k = min(m, i) nearest points among s[0:i], ascending distance, self excluded
// (a fresh sklearn KDTree over s[0:i] per i: O(N^2 log N)).  sklearn 1.7.2 orders
// by the fp64 reduced distance rdist = (0 + t0*t0) + t1*t1, t = s_i - s_j, no
// FMA (sklearn/metrics/_dist_metrics.pxd:26-40); sort_results=True
// (sklearn/neighbors/_binary_tree.pxi.tp:1088,1188).  Here: same key, computed
// with __dmul_rn/__dadd_rn (no contraction), exact ties broken by lower index.
//
// Method: one uniform grid over the bounding box, points radix-sorted by
// (cell, index) so each cell's prior points j < i form a prefix.  One lane per
// query i scans square rings of cells around its own cell, keeping the k best
// (rdist, j) in a register-resident sorted list, and stops when the k-th best
// rdist is below the squared distance to the unscanned region (minus a slack
// that covers cell-assignment rounding).  Levels: grid L covers only the prefix
// s[0:n/4^L] (2 points per cell of ITS prefix), and query i scans the grid of the
// smallest prefix holding all of s[0:i] -- its prior points fill >= 1/4 of that
// prefix, so ~30 cells suffice at every i (one full-density grid made early, sparse-
// prior queries scan thousands of cells: 7.2 ms at N = 1e6, m = 15, all of it the
// slowest waves).  Queries with i < kBruteBelow scan s[0:i] directly.
// Query order (prior mode): lanes of a wave take queries sorted by (floor(log2 i),
// Morton code of the cell), so they have similar prior densities (similar ring counts,
// little divergence) AND neighbouring cells (shared cell-list and point lines in L1/L2);
// each query still writes its own output row.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <math.h>
#include <stdint.h>

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
    const double2* pts_sorted[kKnnMaxLevels];
};

struct Bbox {
    double minx, miny, maxx, maxy;
};

__global__ __launch_bounds__(256) void bbox_partial(const double2* __restrict__ p, int64_t n, double* __restrict__ out) {
    double a = INFINITY, b = INFINITY, c = -INFINITY, d = -INFINITY;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        const double2 v = p[k];
        a = fmin(a, v.x);
        b = fmin(b, v.y);
        c = fmax(c, v.x);
        d = fmax(d, v.y);
    }
    __shared__ double s[4][256];
    s[0][threadIdx.x] = a;
    s[1][threadIdx.x] = b;
    s[2][threadIdx.x] = c;
    s[3][threadIdx.x] = d;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            s[0][threadIdx.x] = fmin(s[0][threadIdx.x], s[0][threadIdx.x + o]);
            s[1][threadIdx.x] = fmin(s[1][threadIdx.x], s[1][threadIdx.x + o]);
            s[2][threadIdx.x] = fmax(s[2][threadIdx.x], s[2][threadIdx.x + o]);
            s[3][threadIdx.x] = fmax(s[3][threadIdx.x], s[3][threadIdx.x + o]);
        }
        __syncthreads();
    }
    if (threadIdx.x < 4) out[4 * blockIdx.x + threadIdx.x] = s[threadIdx.x][0];
}

__global__ __launch_bounds__(64) void bbox_final(const double* __restrict__ part, int nblk, Bbox* __restrict__ box) {
    if (threadIdx.x != 0) return;
    Bbox b{INFINITY, INFINITY, -INFINITY, -INFINITY};
    for (int k = 0; k < nblk; ++k) {
        b.minx = fmin(b.minx, part[4 * k]);
        b.miny = fmin(b.miny, part[4 * k + 1]);
        b.maxx = fmax(b.maxx, part[4 * k + 2]);
        b.maxy = fmax(b.maxy, part[4 * k + 3]);
    }
    *box = b;
}

struct Grid {
    double minx, miny, wx, wy, ivx, ivy;
    int gx, gy;
};

__device__ __forceinline__ Grid make_grid(const Bbox& b, int gx, int gy) {
    Grid g;
    g.gx = gx;
    g.gy = gy;
    g.minx = b.minx;
    g.miny = b.miny;
    double rx = b.maxx - b.minx, ry = b.maxy - b.miny;
    if (!(rx > 0.0)) rx = 1.0;
    if (!(ry > 0.0)) ry = 1.0;
    g.wx = rx / gx;
    g.wy = ry / gy;
    g.ivx = gx / rx;
    g.ivy = gy / ry;
    return g;
}

__device__ __forceinline__ int cell_coord(double v, double lo, double iv, int g) {
    double t = floor((v - lo) * iv);
    int c = (int)fmin(fmax(t, 0.0), (double)(g - 1));
    return c;
}

__global__ __launch_bounds__(256) void cell_keys(const double2* __restrict__ p, int64_t n, const Bbox* __restrict__ box,
                                                 int gx, int gy, uint32_t* __restrict__ key, int32_t* __restrict__ idx) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const Grid g = make_grid(*box, gx, gy);
    const double2 v = p[k];
    const int cx = cell_coord(v.x, g.minx, g.ivx, gx);
    const int cy = cell_coord(v.y, g.miny, g.ivy, gy);
    key[k] = (uint32_t)cy * (uint32_t)gx + (uint32_t)cx;
    idx[k] = (int32_t)k;
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

__global__ __launch_bounds__(256) void gather_sorted(const double2* __restrict__ p, const int32_t* __restrict__ idx_sorted,
                                                     int64_t n, double2* __restrict__ pts_sorted) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) pts_sorted[k] = p[idx_sorted[k]];
}

// bits of x spread to the even positions (x < 2^16)
__device__ __forceinline__ uint32_t spread_bits(uint32_t x) {
    x = (x | (x << 8)) & 0x00FF00FFu;
    x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u;
    x = (x | (x << 1)) & 0x55555555u;
    return x;
}

// sort key of query position t (prior mode): log2 band of the point index, then the
// Morton code of its cell coarsened to `cbits` bits per axis (band in the top 5 bits)
__global__ __launch_bounds__(256) void query_keys(const double2* __restrict__ p, int64_t q0, int64_t nq,
                                                  const int32_t* __restrict__ rows, const Bbox* __restrict__ box,
                                                  int gx, int gy, int shift, uint32_t* __restrict__ key,
                                                  int32_t* __restrict__ pos) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nq) return;
    const int64_t i = rows != nullptr ? (int64_t)rows[t] : q0 + t;
    const Grid g = make_grid(*box, gx, gy);
    const double2 v = p[i];
    const uint32_t cx = (uint32_t)cell_coord(v.x, g.minx, g.ivx, gx) >> shift;
    const uint32_t cy = (uint32_t)cell_coord(v.y, g.miny, g.ivy, gy) >> shift;
    const uint32_t band = 31u - (uint32_t)__clz((unsigned)(i + 1));  // floor(log2(i + 1)) <= 31
    key[t] = (band << 27) | ((spread_bits(cx) | (spread_bits(cy) << 1)) & ((1u << 27) - 1));
    pos[t] = (int32_t)t;
}

// sklearn euclidean_rdist64 without contraction.  The pragma is what keeps it that way:
// __dmul_rn / __dadd_rn are plain * and + in this ROCm's headers, and hipcc's default
// -ffp-contract=fast-honor-pragmas turned t0*t0 + t1*t1 into one v_fmac_f64, which
// rounds differently from sklearn's (0 + t0*t0) + t1*t1 on near-ties
// (tests/test_gpu_knn.py::test_knn_fma_sensitive_ties).
__device__ __forceinline__ double rdist(double qx, double qy, double px, double py) {
#pragma clang fp contract(off)
    const double t0 = qx - px;
    const double t1 = qy - py;
    return t0 * t0 + t1 * t1;
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
template <int KMAX, bool PRIOR>
__global__ __launch_bounds__(256) void knn_query_kernel(const double2* __restrict__ coords, int64_t n, int m,
                                                        const double2* __restrict__ query, int64_t q0, int64_t q1,
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
    const double2 q = PRIOR ? coords[i] : query[i];
    TopK<KMAX> top;
    top.init(k);
    if (PRIOR && i < brute_below) {
        for (int64_t jj = 0; jj < i; ++jj) {
            const double2 p = coords[jj];
            top.push(rdist(q.x, q.y, p.x, p.y), (int32_t)jj);
        }
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
        const int gx = lv.g[L], gy = lv.g[L];
        const int32_t* __restrict__ cell_start = lv.cell_start[L];
        const int32_t* __restrict__ idx_sorted = lv.idx_sorted[L];
        const double2* __restrict__ pts_sorted = lv.pts_sorted[L];
        const Grid g = make_grid(*box, gx, gy);
        const int cx = cell_coord(q.x, g.minx, g.ivx, gx);
        const int cy = cell_coord(q.y, g.miny, g.ivy, gy);
        const double slack = 1e-7 * (g.wx + g.wy) +
                             1e-13 * (fabs(g.minx) + fabs(g.miny) + fabs(g.minx + gx * g.wx) + fabs(g.miny + gy * g.wy));
        int64_t found = 0;
        const int rmax = gx > gy ? gx : gy;
        const int32_t lim = (int32_t)(limit < INT32_MAX ? limit : INT32_MAX);
        for (int r = 0; r <= rmax; ++r) {
            const int y0 = cy - r, y1 = cy + r;
            const int ya = y0 < 0 ? 0 : y0, yb = y1 < gy ? y1 : gy - 1;
            for (int yy = ya; yy <= yb; ++yy) {
                // cells at Chebyshev distance exactly r: whole span on rows cy +- r, two cells elsewhere
                const bool edge_row = (yy == y0) || (yy == y1);
                const int step = (edge_row || r == 0) ? 1 : 2 * r;
                for (int xx = cx - r; xx <= cx + r; xx += step) {
                    if (xx < 0 || xx >= gx) continue;
                    const int64_t c = (int64_t)yy * gx + xx;
                    const int32_t e = cell_start[c + 1];
                    for (int32_t pp = cell_start[c]; pp < e; ++pp) {
                        const int32_t jj = idx_sorted[pp];
                        if (PRIOR && jj >= lim) break;  // (cell, index) order: the rest are not prior
                        const double2 p = pts_sorted[pp];
                        top.push(rdist(q.x, q.y, p.x, p.y), jj);
                        ++found;
                    }
                }
            }
            // distance from q to the region outside the scanned square of cells
            const double bl = (cx - r > 0) ? q.x - (g.minx + (cx - r) * g.wx) : INFINITY;
            const double br = (cx + r < gx - 1) ? (g.minx + (cx + r + 1) * g.wx) - q.x : INFINITY;
            const double bb = (cy - r > 0) ? q.y - (g.miny + (cy - r) * g.wy) : INFINITY;
            const double bt = (cy + r < gy - 1) ? (g.miny + (cy + r + 1) * g.wy) - q.y : INFINITY;
            const double bnd = fmin(fmin(bl, br), fmin(bb, bt));
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

static int grid_side(int64_t n) {
    double g = ceil(sqrt((double)n / kPointsPerCell));
    if (g < 1.0) g = 1.0;
    if (g > 46340.0) g = 46340.0;  // n_cells < 2^31
    return (int)g;
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

hipError_t knn_plan(int64_t n_points, KnnPlan* plan) {
    KnnPlan p{};
    p.n_points = n_points;
    // levels: prefixes n, n/4, n/16, ... down to kLevelMinPoints
    p.n_levels = 0;
    for (int64_t np = n_points; p.n_levels < kKnnMaxLevels; np = (np + 3) / 4) {
        KnnLevel& L = p.lv[p.n_levels++];
        L.np = np;
        L.g = grid_side(np);
        L.n_cells = (int64_t)L.g * L.g;
        if ((np + 3) / 4 < kLevelMinPoints) break;
    }
    p.gx = p.gy = p.lv[0].g;
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
    off += align256(sizeof(double) * (4 * 256 + 8));
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
        off += align256(2 * sizeof(double) * L.np);
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

template <int KMAX>
static void launch_query(bool prior, const double* coords, int64_t n, int m, const double* query, int64_t q0,
                         int64_t q1, const int32_t* rows, const int32_t* perm, int64_t brute_below, const Bbox* box,
                         const KnnLevels& lv, int32_t* nbr, hipStream_t s) {
    const dim3 grid((unsigned)((q1 - q0 + 255) / 256)), block(256);
    if (prior)
        hipLaunchKernelGGL((knn_query_kernel<KMAX, true>), grid, block, 0, s, (const double2*)coords, n, m,
                           (const double2*)query, q0, q1, rows, perm, brute_below, box, lv, nbr);
    else
        hipLaunchKernelGGL((knn_query_kernel<KMAX, false>), grid, block, 0, s, (const double2*)coords, n, m,
                           (const double2*)query, q0, q1, rows, perm, brute_below, box, lv, nbr);
}

hipError_t knn_launch(bool prior, const double* coords, int64_t n, int m, const double* query, int64_t q0, int64_t q1,
                      const int32_t* rows, int32_t* nbr, void* workspace, const KnnPlan& pl, hipStream_t s) {
    char* w = (char*)workspace;
    double* bpart = (double*)(w + pl.off_bbox);
    Bbox* box = (Bbox*)(bpart + 4 * 256);
    uint32_t* key = (uint32_t*)(w + pl.off_key);
    uint32_t* key_sorted = (uint32_t*)(w + pl.off_key_sorted);
    int32_t* idx = (int32_t*)(w + pl.off_idx);
    void* temp = (void*)(w + pl.off_sort_temp);
    const double2* p = (const double2*)coords;

    hipLaunchKernelGGL(bbox_partial, dim3(256), dim3(256), 0, s, p, n, bpart);
    hipLaunchKernelGGL(bbox_final, dim3(1), dim3(64), 0, s, bpart, 256, box);
    // one grid per level over the prefix s[0:np] (query mode only needs level 0); every
    // level shares the bounding box and the key / key_sorted / idx scratch
    KnnLevels lv{};
    lv.n = prior ? pl.n_levels : 1;
    hipError_t e = hipSuccess;
    for (int l = 0; l < lv.n; ++l) {
        const KnnLevel& L = pl.lv[l];
        int32_t* idx_sorted = (int32_t*)(w + L.off_idx_sorted);
        double2* pts_sorted = (double2*)(w + L.off_pts_sorted);
        int32_t* cell_start = (int32_t*)(w + L.off_cell_start);
        const unsigned nb = (unsigned)((L.np + 255) / 256);
        hipLaunchKernelGGL(cell_keys, dim3(nb), dim3(256), 0, s, p, L.np, box, L.g, L.g, key, idx);
        unsigned bits = 1;
        while ((1ll << bits) < L.n_cells) ++bits;
        size_t tb = pl.sort_temp_bytes;
        e = rocprim::radix_sort_pairs(temp, tb, key, key_sorted, idx, idx_sorted, (size_t)L.np, 0u, bits, s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(cell_bounds, dim3((unsigned)((L.n_cells + 1 + 255) / 256)), dim3(256), 0, s, key_sorted,
                           L.np, L.n_cells, cell_start);
        hipLaunchKernelGGL(gather_sorted, dim3(nb), dim3(256), 0, s, p, idx_sorted, L.np, pts_sorted);
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
        while ((1 << cb) < (pl.gx > pl.gy ? pl.gx : pl.gy)) ++cb;
        const int shift = cb > 13 ? cb - 13 : 0;  // 2 * 13 Morton bits + 5 band bits fit 32
        int32_t* pos = (int32_t*)(w + pl.off_perm);
        hipLaunchKernelGGL(query_keys, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, s, p, q0, nq, rows, box,
                           pl.gx, pl.gy, shift, key, idx);
        size_t tq = pl.sort_temp_bytes;
        e = rocprim::radix_sort_pairs(temp, tq, key, key_sorted, idx, pos, (size_t)nq, 0u, 32u, s);
        if (e != hipSuccess) return e;
        perm = pos;
    }
#define NNGP_Q(KM) launch_query<KM>(prior, coords, n, m, query, q0, q1, rows, perm, brute_below, box, lv, nbr, s)
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

}  // namespace nngp
