// Instantiations of bf_group (bf_group.h) with 4 lanes per location for m = 29..32
// (one wave per SIMD; m = 32 spills ~90 VGPRs to scratch).
#include "bf_group.h"

namespace nngp {

bool bf_quad_launch_c(const BfArgs& a, const CovParams& Pc, hipStream_t s) {
    return launch_group_if<29, 4>(a, Pc, s) || launch_group_if<30, 4>(a, Pc, s) ||
           launch_group_if<31, 4>(a, Pc, s) || launch_group_if<32, 4>(a, Pc, s);
}

}  // namespace nngp
