// Split-MFMA fused flow kernel instantiations for K = 16 knots with
// NeuralSplineCoupling activations other than swish (both schemes; own
// translation unit so the swish build is untouched and both compile in
// parallel).
#include "zf_flow_x3_kernel.h"

namespace zf {

int launch_x3_k16_act1(const X3Launch& a, bool inverse);
int launch_x3_k16_act2(const X3Launch& a, bool inverse);

// f16x2 flows whose activations are all of one kind get the narrower
// instantiations (zf_flow_x3_k16_act1 / _act2: the other kind's code out of
// the register budget); mixed flows and bf16x3 take the full switch here.
int launch_x3_k16_act(const X3Launch& a, bool inverse) {
#ifndef ZF_X3_ASET_OFF  // tuning A/B only: every f16x2 flow on the full switch
  if (a.NT == 2 && a.aset == 1) return launch_x3_k16_act1(a, inverse);
  if (a.NT == 2 && a.aset == 2) return launch_x3_k16_act2(a, inverse);
#endif
  return a.NT == 2 ? launch_x3_k<2, 16, true>(a, inverse) : launch_x3_k<3, 16, true>(a, inverse);
}

}  // namespace zf
