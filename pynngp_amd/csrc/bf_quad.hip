// Instantiations of bf_group (bf_group.h) with 4 lanes per location for m in {15, 16, 20}.
// Split into several translation units so the (large, fully unrolled) kernels compile in parallel.
#include "bf_group.h"

namespace nngp {

bool bf_quad_launch(const BfArgs& a, const CovParams& Pc, hipStream_t s) {
    return launch_group_if<15, 4>(a, Pc, s) ||
           launch_group_if<16, 4>(a, Pc, s) ||
           launch_group_if<20, 4>(a, Pc, s);
}

}  // namespace nngp
