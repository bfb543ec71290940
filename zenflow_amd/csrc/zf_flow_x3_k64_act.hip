// Split-MFMA fused flow kernel instantiations for K = 64 knots with
// NeuralSplineCoupling activations other than swish (f16x2 only; the full
// activation switch, no narrower sets at this knot count).
#include "zf_flow_x3_kernel.h"

namespace zf {

int launch_x3_k64_act(const X3Launch& a, bool inverse) {
  return a.NT == 2 ? launch_x3_k<2, 64, true>(a, inverse)
                   : enotsup("bf16x3 takes swish couplings only (x3_eligible)");
}

}  // namespace zf
