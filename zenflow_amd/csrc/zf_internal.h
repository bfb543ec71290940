// Internal helpers shared by the libzenflow_amd translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/zenflow_amd.h"

namespace zf {

void set_error(const char* fmt, ...);

// Returns 0 or the (positive) hipError_t, recording a message.
inline int hip_status(hipError_t e, const char* what) {
  if (e == hipSuccess) return ZF_OK;
  set_error("%s: %s (%d)", what, hipGetErrorString(e), (int)e);
  return (int)e;
}

inline int einval(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  set_error("%s", buf);
  return ZF_EINVAL;
}

inline int enotsup(const char* msg) {
  set_error("not supported: %s", msg);
  return ZF_ENOTSUP;
}

#define ZF_TRY_HIP(expr)                                   \
  do {                                                     \
    int _zf_rc = ::zf::hip_status((expr), #expr);          \
    if (_zf_rc != ZF_OK) return _zf_rc;                    \
  } while (0)

// Post-launch check: a bad launch configuration surfaces here.
#define ZF_CHECK_LAUNCH(name) ZF_TRY_HIP(hipGetLastError())

// Trainer pieces the layered eval path (zf_layered.hip) runs (zf_train.hip):
// C = A . W + bias (W row-major [K][N], a FLAX Dense kernel) and, when H is
// given, H = act(C) (the trainer's fused epilogue).  Mg: the batch that
// picks the tile shape.  rmax (optional): max |output row| as float bits
// per row (H when given, else C) for a following f16x2 layer (zf_layered.hip).
int dense_gemm(long long Mg, int M, int N, int K, const float* A, int lda, const float* W, int ldw, float* C,
               int ldc, float* H, hipStream_t st, const float* bias, int act, unsigned* rmax = nullptr);
// One coupling's RQ spline over B rows from raw conditioner outputs P
// [B][dt][3K-1] (normalize_spline_params + forward with log_det += into ld,
// or inverse), state columns rotated by rot.
int spline_rows(bool inverse, const float* s_in, float* s_out, const float* P, float* ld, int B, int D, int dt,
                int K, int rot, hipStream_t st);

}  // namespace zf
