// Dispatch for the four-lanes-per-location sweep kernels at m = 25..32 (template in bf_group.h,
// instantiations in bf_quad_b.hip / bf_quad_c.hip: 2-D exponential and Matern-3/2, and one runtime-
// kind, runtime-dimension kernel per m for the rest).  The
// two-lane bf_group and the m <= 20 four-lane instantiations were comparison points of the
// blocked pair kernel (bf_pairb.h) and are no longer built into the library.
#include "bf_group.h"

namespace nngp {

bool bf_quad_launch_b(const BfArgs&, const CovParams&, hipStream_t);
bool bf_quad_launch_c(const BfArgs&, const CovParams&, hipStream_t);
bool bf_quad_matern_launch_b(const BfArgs&, const CovParams&, hipStream_t);
bool bf_quad_matern_launch_c(const BfArgs&, const CovParams&, hipStream_t);

int64_t bf_group_blocks(int64_t n_rows, int P) { return (n_rows * P + 255) / 256; }

bool bf_group_supported(int m, int P) {
    return P == 4 && m >= 25 && m <= 32;
}

bool bf_group_launch(const BfArgs& a, const CovParams& Pc, int P, hipStream_t s) {
    if (!bf_group_supported(a.m, P)) return false;
    if (a.kind == NNGP_KIND_MATERN)  // the launch's table in a.cblk
        return a.m <= 28 ? bf_quad_matern_launch_b(a, Pc, s) : bf_quad_matern_launch_c(a, Pc, s);
    return a.m <= 28 ? bf_quad_launch_b(a, Pc, s) : bf_quad_launch_c(a, Pc, s);
}

}  // namespace nngp
