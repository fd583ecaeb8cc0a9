// D-dimensional point helpers shared by the neighbour search (knn.hip) and the
// Z-order visiting order (order.hip): bounding boxes and Morton codes for points
// stored fp64 (n, D) row-major, D = 1, 2, 3 (the reference's ordinates may have any
// dimension, pyNNGP/nngp.py:55-61; 1-D series, 2-D fields, 3-D space or space-time).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "nngp_internal.h"

namespace nngp {

constexpr int kMaxDim = 3;

struct Bbox {
    double lo[kMaxDim], hi[kMaxDim];
};

// per-block partial bounding boxes: out[2 D b + k] = min of axis k, out[2 D b + D + k] = max
template <int D>
__global__ __launch_bounds__(256) void bbox_partial(const double* __restrict__ p, int64_t n, double* __restrict__ out) {
    double lo[D], hi[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {
        lo[k] = INFINITY;
        hi[k] = -INFINITY;
    }
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
        double x[D];
        load_point<D>(p + t * D, x);
#pragma unroll
        for (int k = 0; k < D; ++k) {
            lo[k] = fmin(lo[k], x[k]);
            hi[k] = fmax(hi[k], x[k]);
        }
    }
    __shared__ double s[2 * D][256];
#pragma unroll
    for (int k = 0; k < D; ++k) {
        s[k][threadIdx.x] = lo[k];
        s[D + k][threadIdx.x] = hi[k];
    }
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
#pragma unroll
            for (int k = 0; k < D; ++k) {
                s[k][threadIdx.x] = fmin(s[k][threadIdx.x], s[k][threadIdx.x + o]);
                s[D + k][threadIdx.x] = fmax(s[D + k][threadIdx.x], s[D + k][threadIdx.x + o]);
            }
        }
        __syncthreads();
    }
    if ((int)threadIdx.x < 2 * D) out[2 * D * blockIdx.x + threadIdx.x] = s[threadIdx.x][0];
}

// fold nblk partial boxes (every caller thread may do it: tiny and cached)
template <int D>
__device__ __forceinline__ Bbox bbox_fold(const double* __restrict__ part, int nblk) {
    Bbox b;
#pragma unroll
    for (int k = 0; k < kMaxDim; ++k) {
        b.lo[k] = k < D ? INFINITY : 0.0;
        b.hi[k] = k < D ? -INFINITY : 0.0;
    }
    for (int j = 0; j < nblk; ++j)
#pragma unroll
        for (int k = 0; k < D; ++k) {
            b.lo[k] = fmin(b.lo[k], part[2 * D * j + k]);
            b.hi[k] = fmax(b.hi[k], part[2 * D * j + D + k]);
        }
    return b;
}

template <int D>
__global__ __launch_bounds__(64) void bbox_final(const double* __restrict__ part, int nblk, Bbox* __restrict__ box) {
    if (threadIdx.x == 0) *box = bbox_fold<D>(part, nblk);
}

// bits of x spread to every 2nd (x < 2^16) / 3rd (x < 2^10) position
__device__ __forceinline__ uint32_t spread2(uint32_t x) {
    x &= 0xffffu;
    x = (x | (x << 8)) & 0x00FF00FFu;
    x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u;
    x = (x | (x << 1)) & 0x55555555u;
    return x;
}
__device__ __forceinline__ uint32_t spread3(uint32_t x) {
    x &= 0x3ffu;
    x = (x | (x << 16)) & 0x030000FFu;
    x = (x | (x << 8)) & 0x0300F00Fu;
    x = (x | (x << 4)) & 0x030C30C3u;
    x = (x | (x << 2)) & 0x09249249u;
    return x;
}

// Morton code of integer cell coordinates c[k] < 2^bits(D) (D = 1: 32, 2: 16, 3: 10 bits)
template <int D>
__device__ __forceinline__ uint32_t morton(const uint32_t (&c)[D]) {
    if constexpr (D == 1) return c[0];
    else if constexpr (D == 2) return spread2(c[0]) | (spread2(c[1]) << 1);
    else return spread3(c[0]) | (spread3(c[1]) << 1) | (spread3(c[2]) << 2);
}

template <int D>
constexpr int morton_bits() {
    return D == 1 ? 32 : (D == 2 ? 16 : 10);
}

}  // namespace nngp
