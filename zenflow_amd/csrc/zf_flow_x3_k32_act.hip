// Split-MFMA fused flow kernel instantiations for K = 32 knots with
// NeuralSplineCoupling activations other than swish (both schemes; own
// translation unit so the swish build is untouched and both compile in
// parallel).
#include "zf_flow_x3_kernel.h"

namespace zf {

int launch_x3_k32_act(const X3Launch& a, bool inverse) {
  return a.NT == 2 ? launch_x3_k<2, 32, true>(a, inverse) : launch_x3_k<3, 32, true>(a, inverse);
}

}  // namespace zf
