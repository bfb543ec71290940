// Host side of the two-set split-MFMA kernel (zf_flow_x4_kernel.h): LDS
// footprint and the dispatch to the per-knot-count translation units.
#include "zf_flow_x4_kernel.h"

namespace zf {

int launch_x4_k8(const X3Launch& a, bool inverse, int small_pieces, int ks0);
int launch_x4_k16(const X3Launch& a, bool inverse, int small_pieces, int ks0);
int launch_x4_k32(const X3Launch& a, bool inverse, int small_pieces, int ks0);

size_t x4_lds_bytes_host(int K, bool one, int D, int C, int small_pieces) {
  return x4_lds_bytes(K, one, D, C, small_pieces);
}

int launch_flow_x4(const X3Launch& a, bool inverse, int small_pieces, int ks0) {
  if (a.NT != 2 || a.T != 4) return einval("two-set kernel: f16x2 at hidden <= 128 only");
  if (a.K == 8) return launch_x4_k8(a, inverse, small_pieces, ks0);
  if (a.K == 16) return launch_x4_k16(a, inverse, small_pieces, ks0);
  if (a.K == 32) return launch_x4_k32(a, inverse, small_pieces, ks0);
  return enotsup("two-set kernel: knots not instantiated");
}

}  // namespace zf
