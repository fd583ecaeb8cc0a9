// Instantiations of bf_group (bf_group.h) with 2 lanes per location for m in {19, 20}.
// Split into several translation units so the (large, fully unrolled) kernels compile in parallel.
#include "bf_group.h"

namespace nngp {

bool bf_pair_launch_d(const BfArgs& a, const CovParams& Pc, hipStream_t s) {
    return launch_group_if<19, 2>(a, Pc, s) ||
           launch_group_if<20, 2>(a, Pc, s);
}

}  // namespace nngp
