// Dispatch for the P-lanes-per-location sweep kernels (template in bf_group.h,
// instantiations in bf_pair_*.hip / bf_quad.hip).
#include "bf_group.h"

namespace nngp {

bool bf_pair_launch_a(const BfArgs&, const CovParams&, hipStream_t);
bool bf_pair_launch_b(const BfArgs&, const CovParams&, hipStream_t);
bool bf_pair_launch_c(const BfArgs&, const CovParams&, hipStream_t);
bool bf_pair_launch_d(const BfArgs&, const CovParams&, hipStream_t);
bool bf_quad_launch(const BfArgs&, const CovParams&, hipStream_t);
bool bf_quad_launch_b(const BfArgs&, const CovParams&, hipStream_t);
bool bf_quad_launch_c(const BfArgs&, const CovParams&, hipStream_t);

int64_t bf_group_blocks(int64_t n_rows, int P) { return (n_rows * P + 255) / 256; }

bool bf_group_supported(int m, int P) {
    if (P == 2) return m >= 10 && m <= 20;
    if (P == 4) return m == 15 || m == 16 || m == 20 || (m >= 25 && m <= 32);
    return false;
}

bool bf_group_launch(const BfArgs& a, const CovParams& Pc, int P, hipStream_t s) {
    if (!bf_group_supported(a.m, P)) return false;
    if (P == 4) return a.m <= 20 ? bf_quad_launch(a, Pc, s) : a.m <= 28 ? bf_quad_launch_b(a, Pc, s)
                                                                          : bf_quad_launch_c(a, Pc, s);
    if (a.m <= 13) return bf_pair_launch_a(a, Pc, s);
    if (a.m <= 16) return bf_pair_launch_b(a, Pc, s);
    if (a.m <= 18) return bf_pair_launch_c(a, Pc, s);
    return bf_pair_launch_d(a, Pc, s);
}

}  // namespace nngp
