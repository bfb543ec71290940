// Two-set split-MFMA kernel instantiations for K = 32 knots: one
// transformed dim only (two dims hold 2 x 95 spline parameters per lane
// beside the other set's layer: the register file spills; x4_eligible).
#include "zf_flow_x4_kernel.h"

namespace zf {

int launch_x4_k32(const X3Launch& a, bool inverse, int small_pieces, int ks0) {
  if (a.D / 2 != 1) return enotsup("two-set kernel: K = 32 with two transformed dims not instantiated");
  if (ks0 == 1) return launch_x4<32, true, 1>(a, inverse, small_pieces);
  if (ks0 == 2) return launch_x4<32, true, 2>(a, inverse, small_pieces);
  return enotsup("two-set kernel: Dense_0 k-steps not instantiated");
}

}  // namespace zf
