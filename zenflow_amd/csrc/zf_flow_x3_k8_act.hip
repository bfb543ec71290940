// Split-MFMA fused flow kernel instantiations for K = 8 knots with
// NeuralSplineCoupling activations other than swish (both schemes; own
// translation unit so the swish build is untouched and both compile in
// parallel).
#include "zf_flow_x3_kernel.h"

namespace zf {

int launch_x3_k8_act(const X3Launch& a, bool inverse) {
  return a.NT == 2 ? launch_x3_k<2, 8, true>(a, inverse) : launch_x3_k<3, 8, true>(a, inverse);
}

}  // namespace zf
