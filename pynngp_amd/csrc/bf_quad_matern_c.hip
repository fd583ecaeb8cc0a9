// Instantiations of bf_group (bf_group.h) with 4 lanes per location for the general-smoothness Matern kind
// (the launch's table in LDS) at m = 29..32.
#include "bf_group.h"

namespace nngp {

bool bf_quad_matern_launch_c(const BfArgs& a, const CovParams& Pc, hipStream_t s) {
    return launch_group_matern_if<29>(a, Pc, s) || launch_group_matern_if<30>(a, Pc, s) ||
           launch_group_matern_if<31>(a, Pc, s) || launch_group_matern_if<32>(a, Pc, s);
}

}  // namespace nngp
