// Split-MFMA fused flow kernel instantiations for K = 32 knots (one
// translation unit per knot count, compiled in parallel).
#include "zf_flow_x3_kernel.h"

namespace zf {

int launch_x3_k32(const X3Launch& a, bool inverse) {
  return a.NT == 2 ? launch_x3_k<2, 32>(a, inverse) : launch_x3_k<3, 32>(a, inverse);
}

}  // namespace zf
