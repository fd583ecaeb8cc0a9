// Instantiations of bf_group (bf_group.h) with 2 lanes per location for m in {14, 15, 16}.
// Split into several translation units so the (large, fully unrolled) kernels compile in parallel.
#include "bf_group.h"

namespace nngp {

bool bf_pair_launch_b(const BfArgs& a, const CovParams& Pc, hipStream_t s) {
    return launch_group_if<14, 2>(a, Pc, s) ||
           launch_group_if<15, 2>(a, Pc, s) ||
           launch_group_if<16, 2>(a, Pc, s);
}

}  // namespace nngp
