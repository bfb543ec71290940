// Split-MFMA fused flow kernel instantiations for K = 8 knots with
// NeuralSplineCoupling activations other than swish (f16x2 only; own
// translation unit so the swish build is untouched and both compile in
// parallel).
#include "zf_flow_x3_kernel.h"

namespace zf {

int launch_x3_k8_act2(const X3Launch& a, bool inverse);

// f16x2 flows whose activations are all sigmoid / softplus (centred) get the
// narrower instantiation zf_flow_x3_k8_act2 (their activation inside the
// group steps: sigmoid 0.85 -> 1.03 G samples/s); every other activation runs
// the full switch here (a relu / tanh / gelu / elu / leaky_relu-only set
// measured 0.5-2% slower than this one and was retired in round 6:
// profiles/r06_aset_ab.txt).
int launch_x3_k8_act(const X3Launch& a, bool inverse) {
  if (a.NT == 2 && a.aset == 2) return launch_x3_k8_act2(a, inverse);
  return a.NT == 2 ? launch_x3_k<2, 8, true>(a, inverse)
                   : enotsup("bf16x3 takes swish couplings only (x3_eligible)");
}

}  // namespace zf
