// Instantiations of bf_pairb (bf_pairb.h) for m in 17..20.
#include "bf_pairb.h"

namespace nngp {

bool bf_pairb_launch_c(const BfArgs& a, const CovParams& Pc, hipStream_t s) {
    return launch_pairb_if<17>(a, Pc, s) || launch_pairb_if<18>(a, Pc, s) || launch_pairb_if<19>(a, Pc, s) ||
           launch_pairb_if<20>(a, Pc, s);
}

}  // namespace nngp
