// Instantiations of bf_pairb (bf_pairb.h) for m in 1..11 (split over translation units for parallel builds).
#include "bf_pairb.h"

namespace nngp {

bool bf_pairb_launch_a(const BfArgs& a, const CovParams& Pc, hipStream_t s) {
    return launch_pairb_if<1>(a, Pc, s) || launch_pairb_if<2>(a, Pc, s) || launch_pairb_if<3>(a, Pc, s) || launch_pairb_if<4>(a, Pc, s) ||
           launch_pairb_if<5>(a, Pc, s) || launch_pairb_if<6>(a, Pc, s) || launch_pairb_if<7>(a, Pc, s) ||
           launch_pairb_if<8>(a, Pc, s) || launch_pairb_if<9>(a, Pc, s) || launch_pairb_if<10>(a, Pc, s) ||
           launch_pairb_if<11>(a, Pc, s);
}

}  // namespace nngp
