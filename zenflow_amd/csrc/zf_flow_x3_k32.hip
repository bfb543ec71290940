// Split-MFMA fused flow kernel instantiations for K = 32 knots (one
// translation unit per knot count, compiled in parallel).
#include "zf_flow_x3_kernel.h"

namespace zf {

int launch_x3_k32_act(const X3Launch& a, bool inverse);

int launch_x3_k32(const X3Launch& a, bool inverse) {
  if (a.oact) return launch_x3_k32_act(a, inverse);
  return a.NT == 2 ? launch_x3_k<2, 32>(a, inverse) : launch_x3_k<3, 32>(a, inverse);
}

}  // namespace zf

#ifdef ZF_X3_TRACE
// tuning build only: install the per-wave phase-trace buffer of the K = 32 kernels
extern "C" int zf_x3_trace_set_k32(void* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(zf::x3_trace_buf), &buf, sizeof(buf)) == hipSuccess ? 0 : 1;
}
#endif
