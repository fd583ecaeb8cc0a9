// Instantiations of the round-1 pair kernel for the A/B algo "pairb_r1" (m = 15, exponential,
// 2-D); NNGP_R1_VAR (0..3, read once) selects the variant (bf_pairb_r1.h).
#include <stdlib.h>

#include "bf_pairb_r1.h"

namespace nngp {

int pairb_r1_variant() {
    static const int v = [] {
        const char* e = getenv("NNGP_R1_VAR");
        return e != nullptr ? (atoi(e) & 3) : 0;
    }();
    return v;
}

bool bf_pairb_r1_launch(const BfArgs& a, const CovParams& P, hipStream_t s) {
    if (a.m != 15 || a.kind != 0 || a.dim != 2) return false;
    switch (pairb_r1_variant()) {
        case 1: r1::launch_pairb_mk<15, 0, 1>(a, P, s); break;
        case 2: r1::launch_pairb_mk<15, 0, 2>(a, P, s); break;
        case 3: r1::launch_pairb_mk<15, 0, 3>(a, P, s); break;
        default: r1::launch_pairb_mk<15, 0, 0>(a, P, s); break;
    }
    return true;
}

}  // namespace nngp
