// Split-MFMA fused flow kernel instantiations for K = 64 knots (couplings of
// 33..64 knots run padded to it, x3_padded_knots): 12 last-layer tiles and 191
// spline parameters per lane take one wave per SIMD (x3_occupancy).
#include "zf_flow_x3_kernel.h"

namespace zf {

int launch_x3_k64_act(const X3Launch& a, bool inverse);

int launch_x3_k64(const X3Launch& a, bool inverse) {
  if (a.oact) return launch_x3_k64_act(a, inverse);
  return a.NT == 2 ? launch_x3_k<2, 64>(a, inverse) : launch_x3_k<3, 64>(a, inverse);
}

}  // namespace zf
