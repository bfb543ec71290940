// Split-MFMA fused flow kernel instantiations for K = 8 knots (one
// translation unit per knot count, compiled in parallel).
#include "zf_flow_x3_kernel.h"

namespace zf {

int launch_x3_k8_act(const X3Launch& a, bool inverse);

int launch_x3_k8(const X3Launch& a, bool inverse) {
  if (a.oact) return launch_x3_k8_act(a, inverse);
  return a.NT == 2 ? launch_x3_k<2, 8>(a, inverse) : launch_x3_k<3, 8>(a, inverse);
}

}  // namespace zf
