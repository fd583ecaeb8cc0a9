// Instantiations of bf_group (bf_group.h) with 4 lanes per location reading the joint blocks'
// covariances from memory (NNGP_KIND_BLOCKS) for m = 25..32: nngp_bf_sweep_blocks above the
// blocked pair kernel's register budget (bf_pairb<M, NNGP_KIND_BLOCKS> serves 1..24), as the fused
// kinds' four-lane kernels do (bf_quad_b.hip, bf_quad_c.hip).
#include "bf_group.h"

namespace nngp {

bool bf_group_blocks_supported(int m) { return m >= 25 && m <= 32; }

bool bf_group_blocks_launch(const BfArgs& a, hipStream_t s) {
    return launch_group_blocks_if<25>(a, s) || launch_group_blocks_if<26>(a, s) || launch_group_blocks_if<27>(a, s) ||
           launch_group_blocks_if<28>(a, s) || launch_group_blocks_if<29>(a, s) || launch_group_blocks_if<30>(a, s) ||
           launch_group_blocks_if<31>(a, s) || launch_group_blocks_if<32>(a, s);
}

}  // namespace nngp
