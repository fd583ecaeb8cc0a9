// Instantiations of bf_pairb (bf_pairb.h) for m in 21..24 (one wave per SIMD: 370-512 registers
// with AGPRs; still ~10x the one-wavefront-per-location kernel).
#include "bf_pairb.h"

namespace nngp {

bool bf_pairb_launch_d(const BfArgs& a, const CovParams& Pc, hipStream_t s) {
    return launch_pairb_if<21>(a, Pc, s) || launch_pairb_if<22>(a, Pc, s) || launch_pairb_if<23>(a, Pc, s) ||
           launch_pairb_if<24>(a, Pc, s);
}

}  // namespace nngp
