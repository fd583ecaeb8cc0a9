// Instantiation of the round-1 pair kernel for the A/B algo "pairb_r1" (m = 15, exponential, 2-D).
#include "bf_pairb_r1.h"

namespace nngp {

bool bf_pairb_r1_launch(const BfArgs& a, const CovParams& P, hipStream_t s) {
    if (a.m != 15 || a.kind != 0 || a.dim != 2) return false;
    r1::launch_pairb_mk<15, 0>(a, P, s);
    return true;
}

}  // namespace nngp
