// Instantiations of bf_group (bf_group.h) with 4 lanes per location for m = 25..28
// (above bf_pairb's register budget; 2 waves per SIMD without spills at m = 28).
#include "bf_group.h"

namespace nngp {

bool bf_quad_launch_b(const BfArgs& a, const CovParams& Pc, hipStream_t s) {
    return launch_group_if<25, 4>(a, Pc, s) || launch_group_if<26, 4>(a, Pc, s) ||
           launch_group_if<27, 4>(a, Pc, s) || launch_group_if<28, 4>(a, Pc, s);
}

}  // namespace nngp
