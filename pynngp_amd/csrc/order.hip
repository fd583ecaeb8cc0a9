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

#include "geom.h"
#include "nngp_internal.h"

namespace nngp {

// Morton code of each row's point, quantised to morton_bits<D>() bits per axis over the
// bounding box of the rows (folded from the per-block partials by every thread)
template <int D>
__global__ __launch_bounds__(256) void morton_keys(const double* __restrict__ p, int64_t n,
                                                   const double* __restrict__ part, int nblk,
                                                   uint32_t* __restrict__ key, int32_t* __restrict__ val) {
    const Bbox b = bbox_fold<D>(part, nblk);
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const double top = (double)((1ull << morton_bits<D>()) - 1);
    double x[D];
    load_point<D>(p + t * D, x);
    uint32_t c[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {
        const double sc = b.hi[k] > b.lo[k] ? top / (b.hi[k] - b.lo[k]) : 0.0;
        c[k] = (uint32_t)fmin(fmax((x[k] - b.lo[k]) * sc, 0.0), top);
    }
    key[t] = morton<D>(c);
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
    return align256(2 * kMaxDim * 256 * sizeof(double)) + 3 * align256((size_t)n_rows * 4) + align256(tb);
}

hipError_t row_order_launch(const double* coords, int dim, int64_t i0, int64_t n_rows, int32_t* order,
                            const int32_t* nbr, int m, int32_t* nbr_sorted, void* workspace, size_t workspace_bytes,
                            hipStream_t s) {
    if (n_rows < 1) return hipSuccess;
    const size_t tb = sort_temp_bytes(n_rows);
    char* w = (char*)workspace;
    double* part = (double*)w;
    w += align256(2 * kMaxDim * 256 * sizeof(double));
    uint32_t* key = (uint32_t*)w;
    w += align256((size_t)n_rows * 4);
    uint32_t* key_sorted = (uint32_t*)w;
    w += align256((size_t)n_rows * 4);
    int32_t* val = (int32_t*)w;
    w += align256((size_t)n_rows * 4);
    const double* p = coords + i0 * dim;
    const dim3 nb((unsigned)((n_rows + 255) / 256));
    switch (dim) {
        case 1:
            hipLaunchKernelGGL((bbox_partial<1>), dim3(256), dim3(256), 0, s, p, n_rows, part);
            hipLaunchKernelGGL((morton_keys<1>), nb, dim3(256), 0, s, p, n_rows, part, 256, key, val);
            break;
        case 2:
            hipLaunchKernelGGL((bbox_partial<2>), dim3(256), dim3(256), 0, s, p, n_rows, part);
            hipLaunchKernelGGL((morton_keys<2>), nb, dim3(256), 0, s, p, n_rows, part, 256, key, val);
            break;
        case 3:
            hipLaunchKernelGGL((bbox_partial<3>), dim3(256), dim3(256), 0, s, p, n_rows, part);
            hipLaunchKernelGGL((morton_keys<3>), nb, dim3(256), 0, s, p, n_rows, part, 256, key, val);
            break;
        default:
            return hipErrorInvalidValue;
    }
    size_t t = tb;
    (void)workspace_bytes;
    hipError_t e = rocprim::radix_sort_pairs((void*)w, t, key, key_sorted, val, order, (size_t)n_rows, 0u, 32u, s);
    if (e != hipSuccess || nbr_sorted == nullptr || m == 0) return e;
    hipLaunchKernelGGL(permute_rows, dim3((unsigned)((n_rows * m + 255) / 256)), dim3(256), 0, s, nbr, order, n_rows,
                       m, nbr_sorted);
    return hipGetLastError();
}

}  // namespace nngp
