// Split-MFMA fused flow kernel instantiations for K = 8 knots, f16x2, for
// flows whose couplings use only the centred sigmoid / softplus (and swish):
// the activation switch holds only those forms (ASET = 2, x3_act_tile).
#include "zf_flow_x3_kernel.h"

namespace zf {

int launch_x3_k8_act2(const X3Launch& a, bool inverse) { return launch_x3_k<2, 8, true, 2>(a, inverse); }

}  // namespace zf
