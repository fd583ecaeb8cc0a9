// Processing order for the B/F sweep: the local rows of a shard sorted by the
// Morton (Z-order) code of their coordinates.
//
// The sweep's gathers (each location's m neighbour coordinates and values) are
// the latency it waits on.  In the reference's ordering (input order, nngp.py:51)
// consecutive locations are spatially unrelated, so a wave's neighbours are
// scattered over the whole coordinate array and are served from the Infinity
// Cache at best.  Visiting rows in Z-order instead makes the locations of one
// block -- and, with the kernels' XCD-aware block remap, of one XCD -- a compact
// patch whose neighbours stay in that XCD's L2.  Only the visiting order
// changes: every row's B, F and log-lik term are bit-identical; the fixed-order
// partial sums follow the (deterministic) order.  The neighbour rows are copied
// into the same order (nbr_sorted) so the sweep reads them coalesced; B and F
// are still written at their natural rows.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <math.h>
#include <stdint.h>

#include "nngp_internal.h"

namespace nngp {

__global__ __launch_bounds__(256) void order_bbox_partial(const double2* __restrict__ p, int64_t n,
                                                          double* __restrict__ out) {
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

__device__ __forceinline__ uint32_t spread_bits16(uint32_t v) {
    v &= 0xffffu;
    v = (v | (v << 8)) & 0x00ff00ffu;
    v = (v | (v << 4)) & 0x0f0f0f0fu;
    v = (v | (v << 2)) & 0x33333333u;
    v = (v | (v << 1)) & 0x55555555u;
    return v;
}

__global__ __launch_bounds__(256) void morton_keys(const double2* __restrict__ p, int64_t n,
                                                   const double* __restrict__ part, int nblk,
                                                   uint32_t* __restrict__ key, int32_t* __restrict__ val) {
    double minx = INFINITY, miny = INFINITY, maxx = -INFINITY, maxy = -INFINITY;
    for (int k = 0; k < nblk; ++k) {  // every thread folds the 256 block partials (tiny, cached)
        minx = fmin(minx, part[4 * k]);
        miny = fmin(miny, part[4 * k + 1]);
        maxx = fmax(maxx, part[4 * k + 2]);
        maxy = fmax(maxy, part[4 * k + 3]);
    }
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const double sx = maxx > minx ? 65535.0 / (maxx - minx) : 0.0;
    const double sy = maxy > miny ? 65535.0 / (maxy - miny) : 0.0;
    const double2 v = p[t];
    const uint32_t qx = (uint32_t)fmin(fmax((v.x - minx) * sx, 0.0), 65535.0);
    const uint32_t qy = (uint32_t)fmin(fmax((v.y - miny) * sy, 0.0), 65535.0);
    key[t] = spread_bits16(qx) | (spread_bits16(qy) << 1);
    val[t] = (int32_t)t;
}

__global__ __launch_bounds__(256) void permute_rows(const int32_t* __restrict__ nbr, const int32_t* __restrict__ order,
                                                    int64_t n_rows, int m, int32_t* __restrict__ nbr_sorted) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_rows * m) return;
    const int64_t t = k / m, s = k % m;
    nbr_sorted[k] = nbr[(int64_t)order[t] * m + s];
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

static size_t sort_temp_bytes(int64_t n) {
    size_t tb = 0;
    if (rocprim::radix_sort_pairs((void*)nullptr, tb, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                  (const int32_t*)nullptr, (int32_t*)nullptr, (size_t)n, 0u, 32u) != hipSuccess)
        return 0;
    return tb;
}

size_t row_order_workspace_bytes(int64_t n_rows) {
    if (n_rows < 1) return 256;
    const size_t tb = sort_temp_bytes(n_rows);
    if (tb == 0) return 0;
    return align256(4 * 256 * sizeof(double)) + 3 * align256((size_t)n_rows * 4) + align256(tb);
}

hipError_t row_order_launch(const double* coords, int64_t i0, int64_t n_rows, int32_t* order, const int32_t* nbr,
                            int m, int32_t* nbr_sorted, void* workspace, size_t workspace_bytes, hipStream_t s) {
    if (n_rows < 1) return hipSuccess;
    const size_t tb = sort_temp_bytes(n_rows);
    char* w = (char*)workspace;
    double* part = (double*)w;
    w += align256(4 * 256 * sizeof(double));
    uint32_t* key = (uint32_t*)w;
    w += align256((size_t)n_rows * 4);
    uint32_t* key_sorted = (uint32_t*)w;
    w += align256((size_t)n_rows * 4);
    int32_t* val = (int32_t*)w;
    w += align256((size_t)n_rows * 4);
    const double2* p = (const double2*)coords + i0;
    hipLaunchKernelGGL(order_bbox_partial, dim3(256), dim3(256), 0, s, p, n_rows, part);
    hipLaunchKernelGGL(morton_keys, dim3((unsigned)((n_rows + 255) / 256)), dim3(256), 0, s, p, n_rows, part, 256,
                       key, val);
    size_t t = tb;
    (void)workspace_bytes;
    hipError_t e = rocprim::radix_sort_pairs((void*)w, t, key, key_sorted, val, order, (size_t)n_rows, 0u, 32u, s);
    if (e != hipSuccess || nbr_sorted == nullptr || m == 0) return e;
    hipLaunchKernelGGL(permute_rows, dim3((unsigned)((n_rows * m + 255) / 256)), dim3(256), 0, s, nbr, order, n_rows,
                       m, nbr_sorted);
    return hipGetLastError();
}

}  // namespace nngp
