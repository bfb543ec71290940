// Counter-based latent sampling on the device:
// Philox4x32-10 keyed by the 64-bit seed, counter = (row, dim, stream), so a
// sample depends only on (seed, row, dim) — not on the launch shape — and any
// kernel can draw the latent of the rows it owns in its prologue.
//
// Reference: Distribution.sample (src/zenflow/distributions.py:61-62 Normal,
// :75-78 TruncatedNormal, :106-112 Beta, :125-126 Uniform) draws with
// jax.random (threefry); those bits cannot be reproduced, so parity for
// sampling is statistical (tests/test_gpu_sampling.py) and sample paths are
// pinned on Chain.inverse of a given z.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/zenflow_amd.h"

namespace zf {

struct U32x4 {
  unsigned int v[4];
};

__device__ __forceinline__ U32x4 philox4x32_10(U32x4 c, unsigned int k0, unsigned int k1) {
  constexpr unsigned int M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  constexpr unsigned int W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned int hi0 = __umulhi(M0, c.v[0]), lo0 = M0 * c.v[0];
    const unsigned int hi1 = __umulhi(M1, c.v[2]), lo1 = M1 * c.v[2];
    U32x4 n;
    n.v[0] = hi1 ^ c.v[1] ^ k0;
    n.v[1] = lo1;
    n.v[2] = hi0 ^ c.v[3] ^ k1;
    n.v[3] = lo0;
    c = n;
    k0 += W0;
    k1 += W1;
  }
  return c;
}

__device__ __forceinline__ U32x4 philox_at(unsigned long long seed, long long row, int dim, unsigned int stream) {
  U32x4 c;
  c.v[0] = (unsigned int)row;
  c.v[1] = (unsigned int)((unsigned long long)row >> 32);
  c.v[2] = (unsigned int)dim;
  c.v[3] = stream;
  return philox4x32_10(c, (unsigned int)seed, (unsigned int)(seed >> 32));
}

// [0, 1) and (0, 1] from the top 24 bits.
__device__ __forceinline__ float u01_co(unsigned int b) { return (float)(b >> 8) * 5.9604644775390625e-8f; }
__device__ __forceinline__ float u01_oc(unsigned int b) { return (float)((b >> 8) + 1) * 5.9604644775390625e-8f; }

// Box-Muller standard normal from two words.
__device__ __forceinline__ float normal_of(unsigned int a, unsigned int b) {
  const float r = sqrtf(-2.0f * logf(u01_oc(a)));
  return r * cospif(2.0f * u01_co(b));
}

// Marsaglia-Tsang Gamma(alpha, 1), alpha >= 1 (Beta.peakness >= 1 is enforced,
// distributions.py:96-97).  Trial t uses stream base + 2t.
__device__ __forceinline__ float gamma_draw(unsigned long long seed, long long row, int dim, unsigned int base,
                                            float alpha) {
  const float d = alpha - (1.0f / 3.0f);
  const float cc = rsqrtf(9.0f * d);
  for (unsigned int t = 0; t < 64u; ++t) {
    const U32x4 r = philox_at(seed, row, dim, base + 2u * t);
    const float n = normal_of(r.v[0], r.v[1]);
    float v = 1.0f + cc * n;
    if (v <= 0.0f) continue;
    v = v * v * v;
    const float u = u01_oc(r.v[2]);
    if (logf(u) < 0.5f * n * n + d - d * v + d * logf(v)) return d * v;
  }
  return d;  // not reached in practice (acceptance > 95% per trial)
}

// One latent coordinate z[row, dim] of the flow's latent distribution.
__device__ __forceinline__ float latent_draw(int latent, float param, unsigned long long seed, long long row,
                                             int dim) {
  if (latent == ZF_LATENT_UNIFORM) return u01_co(philox_at(seed, row, dim, 0u).v[0]);
  if (latent == ZF_LATENT_BETA) {
    const float x = gamma_draw(seed, row, dim, 16u, param);
    const float y = gamma_draw(seed, row, dim, 17u, param);
    return x / (x + y);
  }
  // Normal(0.5, 0.1); TruncatedNormal rejects outside +-5 sigma.
  for (unsigned int t = 0; t < 64u; ++t) {
    const U32x4 r = philox_at(seed, row, dim, 1u + t);
    const float n = normal_of(r.v[0], r.v[1]);
    if (latent != ZF_LATENT_TRUNCNORM || fabsf(n) <= 5.0f) return 0.5f + 0.1f * n;
  }
  return 0.5f;
}

}  // namespace zf
