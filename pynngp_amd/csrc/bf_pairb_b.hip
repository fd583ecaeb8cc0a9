// Instantiations of bf_pairb (bf_pairb.h) for m in 12..16.
#include "bf_pairb.h"

namespace nngp {

bool bf_pairb_launch_b(const BfArgs& a, const CovParams& Pc, hipStream_t s) {
    return launch_pairb_if<12>(a, Pc, s) || launch_pairb_if<13>(a, Pc, s) || launch_pairb_if<14>(a, Pc, s) ||
           launch_pairb_if<15>(a, Pc, s) || launch_pairb_if<16>(a, Pc, s);
}

}  // namespace nngp
