// Activations of the conditioner's hidden layers (NeuralSplineCoupling.act,
// bijectors.py:319; flax.linen / jax.nn definitions) and their derivatives
// (training).  The code is uniform per op (zf_op_desc.act).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/zenflow_amd.h"

namespace zf {

constexpr float kSqrt2OverPi = 0.7978845608028654f;  // jax.nn.gelu(approximate=True)
constexpr float kGeluC = 0.044715f;

// Every activation except swish (swish has its own tuned forms next to each
// kernel that uses it).
__device__ __forceinline__ float act_other(int code, float v) {
  switch (code) {
    case ZF_ACT_RELU: return fmaxf(v, 0.0f);                                   // jax.nn.relu
    case ZF_ACT_TANH: return tanhf(v);                                         // jnp.tanh
    case ZF_ACT_SIGMOID: return 1.0f / (1.0f + expf(-v));                      // jax.nn.sigmoid
    case ZF_ACT_GELU: {                                                        // jax.nn.gelu (tanh form)
      const float t = tanhf(kSqrt2OverPi * (v + kGeluC * v * v * v));
      return 0.5f * v * (1.0f + t);
    }
    case ZF_ACT_SOFTPLUS: return fmaxf(v, 0.0f) + log1pf(expf(-fabsf(v)));     // jnp.logaddexp(x, 0)
    case ZF_ACT_ELU: return v > 0.0f ? v : expm1f(v);                          // jax.nn.elu, alpha 1
    case ZF_ACT_LEAKY_RELU: return v >= 0.0f ? v : 0.01f * v;                  // jax.nn.leaky_relu
    default: return __builtin_nanf("");
  }
}

// d act / d v (jax.grad of the forms above; relu'(0) = 0 as jax's)
__device__ __forceinline__ float act_other_grad(int code, float v) {
  switch (code) {
    case ZF_ACT_RELU: return v > 0.0f ? 1.0f : 0.0f;
    case ZF_ACT_TANH: {
      const float t = tanhf(v);
      return 1.0f - t * t;
    }
    case ZF_ACT_SIGMOID: {
      const float s = 1.0f / (1.0f + expf(-v));
      return s * (1.0f - s);
    }
    case ZF_ACT_GELU: {
      const float u = kSqrt2OverPi * (v + kGeluC * v * v * v);
      const float t = tanhf(u);
      return 0.5f * (1.0f + t) + 0.5f * v * (1.0f - t * t) * kSqrt2OverPi * (1.0f + 3.0f * kGeluC * v * v);
    }
    case ZF_ACT_SOFTPLUS: return 1.0f / (1.0f + expf(-v));
    case ZF_ACT_ELU: return v > 0.0f ? 1.0f : expf(v);
    case ZF_ACT_LEAKY_RELU: return v >= 0.0f ? 1.0f : 0.01f;
    default: return __builtin_nanf("");
  }
}

}  // namespace zf
