// Split-MFMA fused flow kernel instantiations for K = 8 knots with
// NeuralSplineCoupling activations other than swish (f16x2 only; own
// translation unit so the swish build is untouched and both compile in
// parallel).
#include "zf_flow_x3_kernel.h"

namespace zf {

int launch_x3_k8_act(const X3Launch& a, bool inverse) {
  if (a.NT != 2) return enotsup("split-MFMA kernel: other activations need the f16x2 scheme");
  return launch_x3_k<2, 8, true>(a, inverse);
}

}  // namespace zf
