// Instantiations of bf_group (bf_group.h) with 4 lanes per location for the general-smoothness Matern kind
// (the launch's table in LDS) at m = 25..28.
#include "bf_group.h"

namespace nngp {

bool bf_quad_matern_launch_b(const BfArgs& a, const CovParams& Pc, hipStream_t s) {
    return launch_group_matern_if<25>(a, Pc, s) || launch_group_matern_if<26>(a, Pc, s) ||
           launch_group_matern_if<27>(a, Pc, s) || launch_group_matern_if<28>(a, Pc, s);
}

}  // namespace nngp
