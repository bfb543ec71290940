// Split-MFMA fused flow kernel instantiations for K = 16 knots, f16x2, for
// flows whose couplings use only relu / tanh / gelu / elu / leaky_relu (and swish):
// the activation switch holds only those forms (ASET = 1, x3_act_tile).
#include "zf_flow_x3_kernel.h"

namespace zf {

int launch_x3_k16_act1(const X3Launch& a, bool inverse) { return launch_x3_k<2, 16, true, 1>(a, inverse); }

}  // namespace zf
