// Two-set split-MFMA kernel instantiations for K = 8 knots: one or two
// transformed dims (ONE), one or two Dense_0 k-steps (KS0), both directions.
#include "zf_flow_x4_kernel.h"

namespace zf {

int launch_x4_k8(const X3Launch& a, bool inverse, int small_pieces, int ks0) {
  const bool one = a.D / 2 == 1;
  if (ks0 == 1) return one ? launch_x4<8, true, 1>(a, inverse, small_pieces) : launch_x4<8, false, 1>(a, inverse, small_pieces);
  if (ks0 == 2) return one ? launch_x4<8, true, 2>(a, inverse, small_pieces) : launch_x4<8, false, 2>(a, inverse, small_pieces);
  return enotsup("two-set kernel: Dense_0 k-steps not instantiated");
}

}  // namespace zf
