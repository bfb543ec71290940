// Split-MFMA fused flow kernel (K3): the whole op chain of
// flow_kernel (zf_flow.hip) in one launch, with the conditioner's streamed
// Dense layers (hidden -> hidden and hidden -> spline parameters) on 16-bit
// MFMA using a split of both fp32 operands:
//   * f16x2 (default): x*2^k = hi + lo, two RNE fp16 terms of power-of-two
//     scaled operands, three v_mfma_f32_32x32x16_f16 products per k-step
//     (lo*hi + hi*lo + hi*hi), fp32 accumulate;
//   * bf16x3 (ZF_X3_SCHEME=bf16x3): x = hi + mid + lo, three RNE bf16 terms,
//     six v_mfma_f32_32x32x16_bf16 products per k-step, small terms first —
//     an fp32 dot product to ~1e-7 relative (tests/hip/mfma_bf16x3_layout.hip).
//
// Execution model:
//   * 4 waves x 32 samples = 128 samples per block; hidden 128 (T = 4): 3
//     blocks per CU (168 VGPRs), or 2 with a dim-pair loop / K = 32;
//     hidden 256 (T = 8): one block per CU (the 8 + 8 accumulator tiles take
//     a wave's whole VGPR + AGPR file).
//   * Weights are the MFMA A operand, pre-split on the host and packed in the
//     exact per-lane fragment order; each streamed layer is a sequence of
//     "groups" (one 32-row input tile x all output tiles x terms: 16 KiB for
//     128 -> 128 at f16x2) that the block DMAs global -> LDS
//     (global_load_lds_dwordx4, no VGPR staging) one group ahead into a
//     double buffer, so a weight byte crosses L2 -> CU once per block.
//   * The B operand is the previous layer's fp32 accumulator tile, split in
//     registers (accumulator-as-operand: k-step s of a tile uses accumulator
//     registers 8s..8s+7; A is packed with the same k order, no shuffles).
//   * The last layer's rows are permuted so that lane half h of every output
//     tile holds 16 consecutive spline parameters of transformed dim h
//     (ONE, dim 2-3: 32 parameters of the one dim per tile): the whole
//     normalize_spline_params + bin search + RQ spline runs from registers;
//     more than 2 transformed dims loop over dim pairs (PAIRS).
//   * Layer 0 (BatchNorm'd conditioning inputs, 1-2 k-steps, fp32 MFMA),
//     ShiftBounds, Roll and the latent epilogue are shared with flow_kernel
//     (zf_flow_dev.h).
// Eligibility (host, x3_eligible): hidden widths <= 256 (<= 128 padded to
// 128), one knot count in {8, 16, 32} for all couplings, dim <= 64.
// Everything else, and ZF_DISABLE_X3=1, runs flow_kernel.
#pragma once
#include "zf_flow_dev.h"

#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <utility>
#include <vector>

namespace zf {
namespace {

typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 halfx2 __attribute__((ext_vector_type(2)));
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));

// Split scheme (NT = terms per operand):
//   NT = 3 "bf16x3": x = hi + mid + lo (RNE bf16 each), six products per
//          k-step — an fp32 dot product to ~1e-7 relative;
//   NT = 2 "f16x2":  x*2^k = hi + lo (RNE fp16 each; 11-bit significands, so
//          the pair holds 22 bits) with hi*hi + hi*lo + lo*hi — three
//          products, each within ~2^-22 relative.  Operands are scaled by
//          powers of two into fp16's range: weights per layer on the host
//          (max |W| * 2^kw in [2^13, 2^14)), activations per sample in the
//          kernel (x3_act_scale); the accumulator is scaled back exactly.
template <int NT>
struct XT;
template <>
struct XT<3> {
  using E = bf16x8;
  static constexpr int kProd = 6;
};
template <>
struct XT<2> {
  using E = halfx8;
  static constexpr int kProd = 3;
};

// Hidden 256 (one wave per SIMD, nothing else to hide LDS latency or fill
// MFMA issue gaps): A fragments one output tile ahead, and each group's
// MFMAs interleaved with its VALU by sched_group_barrier, kWideSched VALU
// per MFMA (measured +4-5% at cfg5; at T = 4 both were neutral to -12%).
constexpr int kWideSched = 3;

#ifndef ZF_X3_WAVES
#define ZF_X3_WAVES 4
#endif
constexpr int kX3Waves = ZF_X3_WAVES;  // waves per block: 32 samples each
static_assert(kX3Waves % 4 == 0, "whole 128-row NLL partial slots per block");

// Tuning-only phase trace (a separate build with -DZF_X3_TRACE=1, never the
// shipped library): each wave sums s_memtime ticks per phase and writes them
// at exit (lane 0, vector stores) to the buffer zf_x3_trace_set_k* installs.
#ifndef ZF_X3_ABL
#define ZF_X3_ABL 0  // tuning-only ablations (wrong results), never set in the shipped build
#endif
#ifdef ZF_X3_TRACE
constexpr int kX3TraceSlots = 16;
__device__ unsigned long long* x3_trace_buf;
#define X3T_NOW() __builtin_amdgcn_s_memtime()
#endif
// Bytes of one weight group = one 32-row input tile: [s][out tile][part] x 1 KiB.
template <int NT>
constexpr int group_bytes(int NOUT) { return 2 * NOUT * NT * 1024; }


// Regs 8s..8s+7 of an accumulator tile -> hi / mid / lo bf16x8 (RNE each).
template <int S>
__device__ __forceinline__ void split8(const floatx16& v, bf16x8& bh, bf16x8& bm, bf16x8& bl) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const floatx2 x = {v[8 * S + 2 * i], v[8 * S + 2 * i + 1]};
    const bf16x2 h = __builtin_convertvector(x, bf16x2);
    const floatx2 r = x - __builtin_convertvector(h, floatx2);
    const bf16x2 m = __builtin_convertvector(r, bf16x2);
    const floatx2 r2 = r - __builtin_convertvector(m, floatx2);
    const bf16x2 l = __builtin_convertvector(r2, bf16x2);
    bh[2 * i] = h[0]; bh[2 * i + 1] = h[1];
    bm[2 * i] = m[0]; bm[2 * i + 1] = m[1];
    bl[2 * i] = l[0]; bl[2 * i + 1] = l[1];
  }
}

// Regs 8s..8s+7 of an (already scaled) activation tile -> hi / lo fp16x8
// (RNE each; the residual x - hi is exact).  The lo term by
// v_fma_mix{lo,hi}_f16 (x*1 - f32(hi) rounded to f16 in one instruction:
// 3 instead of 5 VALU per value pair, bit-identical to sub + cvt —
// tests/hip/f16_split_mix.hip).
template <int S>
__device__ __forceinline__ void split8h(const floatx16& v, halfx8& bh, halfx8& bl) {
  // One asm statement for all eight lo terms, ending in `s_nop 1`: hipcc
  // pads no hazard inside or after an asm statement, and its outputs feed an
  // MFMA operand, which needs two wait states after a VALU write (without
  // the pad a schedule that put the MFMA right behind the asm read stale
  // operands).
  uint32_t h[4], l[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const halfx2 hv = __builtin_convertvector(floatx2{v[8 * S + 2 * i], v[8 * S + 2 * i + 1]}, halfx2);
    __builtin_memcpy(&h[i], &hv, 4);
  }
  asm(
      "v_fma_mixlo_f16 %0, %4, 1.0, -%12 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %0, %5, 1.0, -%12 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixlo_f16 %1, %6, 1.0, -%13 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %1, %7, 1.0, -%13 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixlo_f16 %2, %8, 1.0, -%14 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %2, %9, 1.0, -%14 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixlo_f16 %3, %10, 1.0, -%15 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %3, %11, 1.0, -%15 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
      "s_nop 1"
      : "=&v"(l[0]), "=&v"(l[1]), "=&v"(l[2]), "=&v"(l[3])
      : "v"(v[8 * S + 0]), "v"(v[8 * S + 1]), "v"(v[8 * S + 2]), "v"(v[8 * S + 3]), "v"(v[8 * S + 4]),
        "v"(v[8 * S + 5]), "v"(v[8 * S + 6]), "v"(v[8 * S + 7]), "v"(h[0]), "v"(h[1]), "v"(h[2]), "v"(h[3]));
  __builtin_memcpy(&bh, h, 16);
  __builtin_memcpy(&bl, l, 16);
}

// split8h in two halves for the slot schedule: the hi terms (4 v_cvt_pk),
// then the lo terms (the asm block, one slot later, so it does not wait on
// the conversions' latency).
template <int S>
__device__ __forceinline__ void split8h_hi(const floatx16& v, uint32_t (&h)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const halfx2 hv = __builtin_convertvector(floatx2{v[8 * S + 2 * i], v[8 * S + 2 * i + 1]}, halfx2);
    __builtin_memcpy(&h[i], &hv, 4);
  }
}

template <int S>
__device__ __forceinline__ void split8h_lo(const floatx16& v, const uint32_t (&h)[4], halfx8& bh, halfx8& bl) {
  uint32_t l[4];
  asm("v_fma_mixlo_f16 %0, %4, 1.0, -%12 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %0, %5, 1.0, -%12 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixlo_f16 %1, %6, 1.0, -%13 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %1, %7, 1.0, -%13 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixlo_f16 %2, %8, 1.0, -%14 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %2, %9, 1.0, -%14 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixlo_f16 %3, %10, 1.0, -%15 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %3, %11, 1.0, -%15 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
      "s_nop 1"
      : "=&v"(l[0]), "=&v"(l[1]), "=&v"(l[2]), "=&v"(l[3])
      : "v"(v[8 * S + 0]), "v"(v[8 * S + 1]), "v"(v[8 * S + 2]), "v"(v[8 * S + 3]), "v"(v[8 * S + 4]),
        "v"(v[8 * S + 5]), "v"(v[8 * S + 6]), "v"(v[8 * S + 7]), "v"(h[0]), "v"(h[1]), "v"(h[2]), "v"(h[3]));
  __builtin_memcpy(&bh, h, 16);
  __builtin_memcpy(&bl, l, 16);
}

template <int NT, int S>
__device__ __forceinline__ void splitk(const floatx16& v, typename XT<NT>::E (&b)[NT]) {
  if constexpr (NT == 3) {
    split8<S>(v, b[0], b[1], b[2]);
  } else {
    split8h<S>(v, b[0], b[1]);
  }
}

// f16x2: every swished layer (Dense_0 .. Dense_{n_hidden-1}) is packed with
// its weights and bias multiplied by log2(e) (x3_pack), so its accumulator
// holds v' = v*log2(e) and the sigmoid's exponent needs no multiply.
constexpr float kSwishPrescale = 1.44269504088896341f;

// Layer-input activation: swish(v) (bf16x3), or f16x2's swish(v) * sc from
// the prescaled v' with c = isc*log2(e) (isc = 1/sc a power of two):
//   swish(v) * sc = v' / ((1 + 2^-v') * c)  — one fma, exp2, rcp, mul, so
// neither the exponent scale nor the activation scale costs an instruction.
template <int NT>
__device__ __forceinline__ float act_swish(float v, float c) {
  if constexpr (NT == 2) {
    const float e = __builtin_amdgcn_exp2f(-v);
    return v * __builtin_amdgcn_rcpf(__builtin_fmaf(e, c, c));
  }
  return swish(v);
}

// The layer-input activation of one accumulator tile.  OACT = false: every
// coupling is swish (act_swish, the tuned form).  OACT = true (f16x2 only):
// NeuralSplineCoupling.act per coupling (wave-uniform `act`, zf_act.h forms,
// one switch per tile); swish couplings keep act_swish and the log2(e)
// prescale, the others are packed unscaled and multiply their activation by
// the power-of-two scale c = sc of x3_act_scale.
template <int CODE>
__device__ __forceinline__ void act_tile_fixed(floatx16& t, float c) {
#pragma unroll
  for (int r = 0; r < 16; ++r) t[r] = act_other(CODE, t[r]) * c;
}

// f16x2 sigmoid / softplus, centred: their information
// sits in small deviations from 1/2 and log 2, which a per-sample scale of
// the raw value cannot resolve to fp32's precision.  The kernel feeds
// a(v) = act(v) - C to the split MFMA (C = 1/2, log 2; a(0) = 0 and
// |a(v)| <= |v|, so x3_act_scale's per-sample scale keeps a's relative
// precision), and x3_pack folds C * colsum(W) of the consuming layer into
// its bias.  act(v) is rounded to fp32 first, as the reference's
// jax.nn.sigmoid / softplus output is, so a = fl(act(v)) - C carries the
// reference's own rounding (the subtraction is exact for act(v) in [C/2, 2C]).
// Near v = 0 both are evaluated from their series (|v| < 1/4: truncation
// below 1e-9 of a), so a carries the deviation to fp32's relative precision
// instead of the 1-2 ulp of 1/2 or log 2 the rounded act(v) carries there
// (tiny pre-activations under large weights: the hardware log2 alone put
// softplus' mean error at 2.3x the fp32 oracle's).
constexpr float kLn2 = 0.693147180559945309f;
__device__ __forceinline__ float act_sigmoid_centered(float v) {
  // 1 / (1 + 2^(-v log2 e)) with a residual-corrected reciprocal (as the
  // bf16x3 form); 1 + e = inf (v < -88) gives 0.  |v| < 1/4: tanh(v/2)/2 =
  // v/4 - v^3/48 + v^5/480 - 17 v^7/80640.  (Round 6 measured a form with a
  // clamped exponent and no inf / NaN tests 3% SLOWER at cfg2's shape:
  // profiles/r06_act_ab.txt.)
  const float d = 1.0f + __builtin_amdgcn_exp2f(-v * kSwishPrescale);
  const float q = __builtin_amdgcn_rcpf(d);
  const float sg = __builtin_fmaf(q, __builtin_fmaf(-d, q, 1.0f), q);
  const float v2 = v * v;
  const float ser =
      v * __builtin_fmaf(v2, __builtin_fmaf(v2, __builtin_fmaf(v2, -17.0f / 80640.0f, 1.0f / 480.0f), -1.0f / 48.0f),
                         0.25f);
  return fabsf(v) < 0.25f ? ser : (d == __builtin_huge_valf() ? 0.0f : sg) - 0.5f;
}
// softplus (round 6; 7% faster at cfg2's shape,
// profiles/r06_act_ab.txt): the select tests |v| >= 1/4, false for NaN, so a
// NaN input takes the series branch and stays NaN without a compare of its
// own; log1p's small-t series is gone: a centred value a = softplus(v) -
// log 2 carries t = exp(-|v|) < 1/64 only at |v| > 4.2, where 1 + t's
// rounding (2^-24 absolute) is below a's own ulp.
__device__ __forceinline__ float act_softplus_centered(float v) {
  // logaddexp(v, 0) - log 2 = max(v, 0) + log1p(exp(-|v|)) - log 2, log1p
  // from the hardware log2 of 1 + t.
  // |v| < 1/4: softplus(v) - log 2 = v/2 + v^2/8 - v^4/192 + v^6/2880
  const float t = __builtin_amdgcn_exp2f(-fabsf(v) * kSwishPrescale);
  const float sp = __builtin_fmaf(__builtin_amdgcn_logf(1.0f + t), kLn2, fmaxf(v, 0.0f));
  const float v2 = v * v;
  const float ser = v * __builtin_fmaf(v, __builtin_fmaf(v2, __builtin_fmaf(v2, 1.0f / 2880.0f, -1.0f / 192.0f), 0.125f),
                                       0.5f);
  return fabsf(v) >= 0.25f ? sp - kLn2 : ser;
}

template <int CODE>
__device__ __forceinline__ void act_tile_centered(floatx16& t, float c) {
#pragma unroll
  for (int r = 0; r < 16; ++r)
    t[r] = (CODE == ZF_ACT_SIGMOID ? act_sigmoid_centered(t[r]) : act_softplus_centered(t[r])) * c;
}

template <int CODE>
__device__ __forceinline__ void act_tile_plain(floatx16& t) {
#pragma unroll
  for (int r = 0; r < 16; ++r) t[r] = act_other(CODE, t[r]);
}

// bf16x3 sigmoid: 1 / (1 + 2^(-v log2 e)) from the hardware exp2 and a
// residual-corrected reciprocal (8 VALU instead of expf + IEEE division);
// 1 + e = inf (v < -88) gives 0, as 1 / (1 + expf(-v)) does.
template <>
__device__ __forceinline__ void act_tile_plain<ZF_ACT_SIGMOID>(floatx16& t) {
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float d = 1.0f + __builtin_amdgcn_exp2f(-t[r] * kSwishPrescale);
    const float q = __builtin_amdgcn_rcpf(d);
    const float c = __builtin_fmaf(q, __builtin_fmaf(-d, q, 1.0f), q);
    t[r] = d == __builtin_huge_valf() ? 0.0f : c;  // NaN stays NaN
  }
}

// ASET (f16x2 OACT kernels): the activations one instantiation takes besides
// swish — 0: all of them (a flow mixing centred and plain activations),
// 1: relu / tanh / gelu / elu / leaky_relu, 2: sigmoid / softplus (centred).
// Narrower sets keep the other forms' code out of the register budget.
template <int NT, bool OACT, int ASET = 0>
__device__ __forceinline__ void x3_act_tile(floatx16& t, float c, int act) {
  if constexpr (!OACT) {
#pragma unroll
    for (int r = 0; r < 16; ++r) t[r] = act_swish<NT>(t[r], c);
  } else if constexpr (NT == 3) {
    // bf16x3: no scales; every activation, sigmoid and softplus included
    switch (act) {
      case ZF_ACT_RELU: act_tile_plain<ZF_ACT_RELU>(t); break;
      case ZF_ACT_TANH: act_tile_plain<ZF_ACT_TANH>(t); break;
      case ZF_ACT_SIGMOID: act_tile_plain<ZF_ACT_SIGMOID>(t); break;
      case ZF_ACT_GELU: act_tile_plain<ZF_ACT_GELU>(t); break;
      case ZF_ACT_SOFTPLUS: act_tile_plain<ZF_ACT_SOFTPLUS>(t); break;
      case ZF_ACT_ELU: act_tile_plain<ZF_ACT_ELU>(t); break;
      case ZF_ACT_LEAKY_RELU: act_tile_plain<ZF_ACT_LEAKY_RELU>(t); break;
      default:
#pragma unroll
        for (int r = 0; r < 16; ++r) t[r] = swish(t[r]);
    }
  } else {
    if constexpr (ASET == 2) {
      switch (act) {
        case ZF_ACT_SIGMOID: act_tile_centered<ZF_ACT_SIGMOID>(t, c); break;
        case ZF_ACT_SOFTPLUS: act_tile_centered<ZF_ACT_SOFTPLUS>(t, c); break;
        default:
#pragma unroll
          for (int r = 0; r < 16; ++r) t[r] = act_swish<NT>(t[r], c);
      }
    } else {
      switch (act) {
        case ZF_ACT_RELU: act_tile_fixed<ZF_ACT_RELU>(t, c); break;
        case ZF_ACT_TANH: act_tile_fixed<ZF_ACT_TANH>(t, c); break;
        case ZF_ACT_GELU: act_tile_fixed<ZF_ACT_GELU>(t, c); break;
        case ZF_ACT_ELU: act_tile_fixed<ZF_ACT_ELU>(t, c); break;
        case ZF_ACT_LEAKY_RELU: act_tile_fixed<ZF_ACT_LEAKY_RELU>(t, c); break;
        case ZF_ACT_SIGMOID:
          if constexpr (ASET == 0) act_tile_centered<ZF_ACT_SIGMOID>(t, c);
          break;
        case ZF_ACT_SOFTPLUS:
          if constexpr (ASET == 0) act_tile_centered<ZF_ACT_SOFTPLUS>(t, c);
          break;
        default:
#pragma unroll
          for (int r = 0; r < 16; ++r) t[r] = act_swish<NT>(t[r], c);
      }
    }
  }
}

__device__ __forceinline__ floatx16 mfma3(const bf16x8& ah, const bf16x8& am, const bf16x8& al,
                                          const bf16x8& bh, const bf16x8& bm, const bf16x8& bl,
                                          floatx16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
}

// One k-step of the split product, small terms first.
template <int NT>
__device__ __forceinline__ floatx16 mfma_split(const typename XT<NT>::E (&a)[NT], const typename XT<NT>::E (&b)[NT],
                                               floatx16 acc) {
  if constexpr (NT == 3) {
    return mfma3(a[0], a[1], a[2], b[0], b[1], b[2], acc);
  } else {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[1], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[1], acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[0], acc, 0, 0, 0);
  }
}

// A fragment (NT parts of 1 KiB; this lane's 16 bytes of each) from LDS.
template <int NT>
__device__ __forceinline__ void load_frag(const char* a, typename XT<NT>::E (&f)[NT]) {
  using E = typename XT<NT>::E;
  if constexpr (NT == 3) f[1] = *reinterpret_cast<const E*>(a + 1024);
  f[0] = *reinterpret_cast<const E*>(a);
  if constexpr (NT == 3) f[2] = *reinterpret_cast<const E*>(a + 2048);
  else f[1] = *reinterpret_cast<const E*>(a + 1024);
}

// f16x2: per-sample power-of-two scale sc = 1/isc of a layer input, from its
// raw (log2(e)-prescaled) pre-activations, so its largest |swish| lands below
// 2^14 (|swish(v)| <= |v| < |v'|), and the exact factor that undoes both
// scales on the accumulator: us = 2^-(e_act + kw) (ius = 1/us).  Returned
// in isc: the swish constant c = isc*log2(e) (act_swish).  Lanes l and l^32
// hold the same sample.
// The two wave halves' copies of x (lane l and lane l ^ 32 hold the same
// sample): .lo = the value of lane l & 31, .hi = that of lane l | 32, on
// every lane.  One v_permlane32_swap (VALU; gfx950) instead of the
// ds_bpermute an __shfl_xor(x, 32) lowers to (an LDS round trip, in the
// kernel's serial spline phase), and no select to pick the halves.
struct X3Halves {
  float lo, hi;
};
__device__ __forceinline__ X3Halves x3_halves(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_int(x), __float_as_int(x), false, false);
  return {__int_as_float(r[0]), __int_as_float(r[1])};
}

template <int T, bool OACT = false>
__device__ __forceinline__ void x3_act_scale(const floatx16 (&hb)[T], int kw, float& isc, float& us, float& ius,
                                             int act = ZF_ACT_SWISH) {
  float m = 0.f;
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) m = fmaxf(m, fabsf(hb[t][r]));
  {
    const X3Halves q = x3_halves(m);
    m = fmaxf(q.lo, q.hi);
  }
  // OACT: |act(v)| <= |v| for every activation the kernel takes (relu,
  // leaky_relu, tanh, gelu, elu, and sigmoid / softplus centred:
  // act_tile_centered), so the bound holds as for swish.
  // (e clamped: a layer input below 2^-60 keeps scale 2^74, so a bias
  // seeded as bias / us stays finite)
  const int e = max(__builtin_amdgcn_frexp_expf(m), -60);
  // swish: the act_swish constant c = 2^(e-14) log2(e); others: sc = 2^(14-e)
  isc = (OACT && act != ZF_ACT_SWISH) ? __builtin_amdgcn_ldexpf(1.0f, 14 - e)
                                      : __builtin_amdgcn_ldexpf(kSwishPrescale, e - 14);
  us = __builtin_amdgcn_ldexpf(1.0f, e - 14 - kw);
  ius = __builtin_amdgcn_ldexpf(1.0f, 14 + kw - e);
}

// Layer end: acc = acc * us + bias (f16x2: undo the scales) or acc + bias.
template <int NT>
__device__ __forceinline__ floatx16 x3_finish(const floatx16& acc, float us, const floatx16& b) {
  if constexpr (NT == 2) {
    floatx16 r;
#pragma unroll
    for (int i = 0; i < 16; ++i) r[i] = __builtin_fmaf(acc[i], us, b[i]);
    return r;
  } else {
    return acc + b;
  }
}

// One weight group from LDS: input tile Q (2 k-steps of 16) into NOUT
// output tiles.  Block (s, o, part) is 1 KiB at ((s*NOUT + o)*NT + part) KiB;
// lane l's 16 bytes at l*16.
template <int NT, int T, int NOUT, int Q>
__device__ __forceinline__ void x3_group(const char* buf, const floatx16 (&hb)[T], floatx16 (&acc)[NOUT],
                                         int lane) {
  using E = typename XT<NT>::E;
  const char* lb = buf + lane * 16;
if constexpr (T == 8) {
  // A fragments one output tile ahead (LDS latency off the MFMA chain).
  E c[NT];
  load_frag<NT>(lb, c);
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    E b[NT];
    if (s == 0) splitk<NT, 0>(hb[Q], b);
    else splitk<NT, 1>(hb[Q], b);
#pragma unroll
    for (int o = 0; o < NOUT; ++o) {
      const int t = s * NOUT + o;
      E n[NT];
      if (t + 1 < 2 * NOUT) load_frag<NT>(lb + (((t + 1) * NT) << 10), n);
      acc[o] = mfma_split<NT>(c, b, acc[o]);
      if (t + 1 < 2 * NOUT) {
#pragma unroll
        for (int i = 0; i < NT; ++i) c[i] = n[i];
      }
    }
  }
} else {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    E b[NT];
    if (s == 0) splitk<NT, 0>(hb[Q], b);
    else splitk<NT, 1>(hb[Q], b);
#pragma unroll
    for (int o = 0; o < NOUT; ++o) {
      E a[NT];
      load_frag<NT>(lb + (((s * NOUT + o) * NT) << 10), a);
      acc[o] = mfma_split<NT>(a, b, acc[o]);
    }
  }
}
}

// The group stream of the NSC being computed (byte offsets into the x3
// blob), set up at NSC entry from the op's scalar fields: the per-step
// prefetch then needs no memory access of its own (a scalar load there would
// make its lgkmcnt wait drain the step's LDS reads too).  Groups in order:
// hidden layers (T groups each), then the last layer (T groups per pair of
// transformed dims).
struct X3Span {
  long long base;       // group 0 of this NSC
  long long next_base;  // group 0 of the next NSC in execution order within range, or -1
  int G, nhid;          // groups in this NSC, hidden-layer groups among them
  int last_pieces;      // KiB pieces of one last-layer group
  int next_pieces;      // KiB pieces of the next NSC's group 0
};

template <int NT, int T>
__device__ __forceinline__ int first_pieces(const DevOp& op) {
  return (op.n_hidden > 1 ? group_bytes<NT>(T) : group_bytes<NT>(op.x3_tlast)) >> 10;
}

// Every scalar of one op the kernel uses, read at the top of the op loop for
// every op kind: one batch of independent scalar loads and one wait, instead
// of a chain of load -> wait -> branch -> load (each lgkmcnt(0) wait there
// also drains the wave's outstanding LDS reads).
struct X3Sc {
  int kind, shift, nh, act, dt, dc, DC, KS0, G, tlast, nxt, npieces, npar, kw1, kw_last, kreal;
  long long x3, nbase, nbn, bn, w0_rel, b_rel, blast_rel, sb;
};

template <bool INV>
__device__ __forceinline__ X3Sc x3_scalars(const DevOp& op) {
  constexpr int d = INV ? 1 : 0;
  X3Sc c;
  c.kind = op.kind; c.shift = op.shift; c.nh = op.n_hidden; c.act = op.act;
  c.dt = op.dt; c.dc = op.dc; c.DC = op.DC; c.KS0 = op.KS0;
  c.G = op.x3_groups; c.tlast = op.x3_tlast; c.nxt = op.x3_next[d];
  c.npieces = op.x3_npieces[d]; c.npar = op.x3_npar[d];
  c.kw1 = op.x3_kw[1];
  c.kreal = op.K;  // this coupling's knots (the kernel's K may be padded above them)
  c.kw_last = op.x3_kw[op.n_hidden & 15];
  c.x3 = op.x3; c.nbase = op.x3_nbase[d]; c.nbn = op.x3_nbn[d]; c.bn = op.bn;
  c.w0_rel = op.w[0] - op.bn; c.b_rel = op.b[0] - op.bn; c.blast_rel = op.x3_blast - op.bn;
  c.sb = op.sb;
  return c;
}

template <int NT, int T>
__device__ __forceinline__ X3Span make_span(const X3Sc& c, bool has_next) {
  X3Span sp;
  sp.base = c.x3;
  sp.G = c.G;
  sp.nhid = T * (c.nh - 1);
  sp.last_pieces = group_bytes<NT>(c.tlast) >> 10;
  sp.next_base = has_next ? c.nbase : -1;
  sp.next_pieces = has_next ? c.npieces : 0;
  return sp;
}

// Issue the DMA of one group into an LDS buffer: 1 KiB pieces (one
// global_load_lds_dwordx4 per wave: wave-uniform LDS base, lane*16 implied)
// spread over the block's waves.
__device__ __forceinline__ void x3_dma(const char* __restrict__ src, char* dst, int pieces, int wave, int lane) {
#if ZF_X3_ABL == 5  // tuning ablation 5: a quarter of the weight stream (wrong results)
  pieces = (pieces + 3) / 4;
#endif
  for (int p = wave; p < pieces; p += kX3Waves)
    __builtin_amdgcn_global_load_lds((const void*)(src + (p << 10) + lane * 16),
                                     (__attribute__((address_space(3))) void*)(dst + (p << 10)), 16, 0, 0);
}

// Block-wide weight-group pipeline state (every field wave-uniform).
struct X3Pipe {
  char* cur;    // LDS buffer holding the group this wave computes next
  char* nxt;    // the other buffer of the double buffer (the prefetch target)
  int g;        // index of that group within the current NSC
  X3Span span;  // current NSC's group stream
  int wave;
  // the next NSC's small parameters (DMA'd at step 0 of this NSC into the
  // other LDS parameter region; null at the last NSC of the range)
  const char* par_src;
  char* par_dst;
  int par_pieces;
#ifdef ZF_X3_TRACE
  unsigned long long tbar;  // ticks spent in the per-group DMA wait + barrier
  unsigned long long tdma;  // x3_step (plain steps: the dim-pair / hidden-256 last layers): DMA issue
  unsigned long long tgrp;  // x3_step: the group's MFMAs, fragment reads and split (x3_group) + finish
#endif
};

// DMA the group after group p.g (the next one of this NSC, or group 0 of
// the next NSC) into `dst`; nothing at the end of the stream.
template <int NT, int T>
__device__ __forceinline__ void x3_issue_next(const char* __restrict__ x3, const X3Pipe& p, char* dst, int lane) {
  constexpr int kHid = group_bytes<NT>(T);
  if (p.g == 0 && p.par_src != nullptr) x3_dma(p.par_src, p.par_dst, p.par_pieces, p.wave, lane);
  const int g = p.g + 1;
#if ZF_X3_ABL == 6  // tuning ablation 6: the stream stops after each NSC's first two groups (real weights stay; wrong results)
  if (g > 1 && g < p.span.G) return;
#endif
  long long off;
  int pieces;
  if (g < p.span.nhid) {
    off = p.span.base + (long long)g * kHid;
    pieces = kHid >> 10;
  } else if (g < p.span.G) {
    off = p.span.base + (long long)p.span.nhid * kHid + (long long)(g - p.span.nhid) * (p.span.last_pieces << 10);
    pieces = p.span.last_pieces;
  } else {
    if (p.span.next_base < 0) return;
    off = p.span.next_base;
    pieces = p.span.next_pieces;
  }
  x3_dma(x3 + off, dst, pieces, p.wave, lane);
}

// One pipeline step: wait for this wave's DMAs, block barrier (the group in
// buffer `buf` is complete and the other buffer is free), prefetch the next
// group into it, then this group's MFMAs.  `bias` (optional): bias tiles of
// a layer whose accumulators did not start from the bias, loaded here — in
// the layer's last step, when its earlier input tiles are dead — and joined
// after the MFMAs (x3_finish, which also undoes the f16x2 scales).
template <int NT, int T, int NOUT, int Q, bool SW, bool OACT>
__device__ __forceinline__ void x3_step(const char* __restrict__ x3, X3Pipe& p, floatx16 (&hb)[T],
                                        floatx16 (&acc)[NOUT], int lane, const float* __restrict__ bias,
                                        int hh, float isc, float us, int act) {
#ifdef ZF_X3_TRACE
  const unsigned long long tb0 = X3T_NOW();
#endif
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#ifdef ZF_X3_TRACE
  p.tbar += X3T_NOW() - tb0;
#endif
#ifdef ZF_X3_TRACE
  const unsigned long long td0 = X3T_NOW();
#endif
  x3_issue_next<NT, T>(x3, p, p.nxt, lane);
#ifdef ZF_X3_TRACE
  const unsigned long long td1 = X3T_NOW();
  p.tdma += td1 - td0;
#endif
  if (bias != nullptr) {
    floatx16 bt[NOUT];
#pragma unroll
    for (int o = 0; o < NOUT; ++o) bt[o] = bias_acc(bias + o * 32, hh);
    x3_group<NT, T, NOUT, Q>(p.cur, hb, acc, lane);
#pragma unroll
    for (int o = 0; o < NOUT; ++o) acc[o] = x3_finish<NT>(acc[o], us, bt[o]);
  } else {
    x3_group<NT, T, NOUT, Q>(p.cur, hb, acc, lane);
  }
#ifdef ZF_X3_TRACE
  {  // wait for the group's MFMA results (a stamp cannot see an MFMA in flight)
    float sink = acc[0][0];
    asm volatile("; use %0" : "+v"(sink));
    p.tgrp += X3T_NOW() - td1;
  }
#endif
  // SW: the layer input arrives as pre-activations except tile 0; the swish
  // of tile Q+1 goes here, in the same scheduling region as this group's
  // MFMAs, whose issue gaps it fills.
  if constexpr (SW && !OACT && Q + 1 < T) {
    x3_act_tile<NT, OACT>(hb[Q + 1], isc, act);
  }
  if constexpr (T == 8) {
    // the k-step-0 split first, then every MFMA followed by its share of LDS
    // reads and VALU (split of k-step 1, the deferred swish)
    constexpr int kP = XT<NT>::kProd;
    __builtin_amdgcn_sched_group_barrier(0x100, NT, 0);
    __builtin_amdgcn_sched_group_barrier(0x402, 20, 0);
#pragma unroll
    for (int i = 0; i < 2 * kP * NOUT; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      if ((NT == 3 && i % 2 == 0) || (NT == 2 && i % 3 != 2)) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x402, kWideSched, 0);
    }
  }
  char* const t = p.cur;
  p.cur = p.nxt;
  p.nxt = t;
  p.g += 1;
}

// k-step-level software pipeline (hidden 128, one pass per layer): group Q
// multiplies k-step (Q, 0) with the split carried in `cs`, and beside its
// MFMAs forms the split of (Q, 1), the swish of tile Q+1 and the split of
// (Q+1, 0) for the next group — so the bf16 split and the deferred swish sit
// in the MFMA issue gaps of the same wave (cross-wave they would not overlap:
// tests/hip/coexec_probe.hip modes 2 and 6).
template <int NT, int T, int NOUT, int Q, bool HASB, bool OACT, int AS = 0>
__device__ __forceinline__ void x3_step_pipe(const char* __restrict__ x3, X3Pipe& p, floatx16 (&hb)[T],
                                             floatx16 (&acc)[NOUT], int lane, const float* __restrict__ bias,
                                             int hh, typename XT<NT>::E (&cs)[NT], float isc, float us,
                                             int act) {
  using E = typename XT<NT>::E;
#ifdef ZF_X3_TRACE
  const unsigned long long tb0 = X3T_NOW();
#endif
#if ZF_X3_ABL != 3  // tuning ablation 3: no per-group DMA wait / barrier (wrong results)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#endif
#ifdef ZF_X3_TRACE
  p.tbar += X3T_NOW() - tb0;
#endif
  x3_issue_next<NT, T>(x3, p, p.nxt, lane);
  const char* lb = p.cur + lane * 16;
  E s1[NT];
  splitk<NT, 1>(hb[Q], s1);
#if ZF_X3_ABL == 1  // tuning ablation 1: one A fragment per step (no per-tile LDS reads; wrong results)
  E a1[NT];
  load_frag<NT>(lb, a1);
#endif
#pragma unroll
  for (int o = 0; o < NOUT; ++o) {
#if ZF_X3_ABL == 1
    acc[o] = mfma_split<NT>(a1, cs, acc[o]);
#else
    E a[NT];
    load_frag<NT>(lb + ((o * NT) << 10), a);
    acc[o] = mfma_split<NT>(a, cs, acc[o]);
#endif
  }
  if constexpr (Q + 1 < T) {
#if ZF_X3_ABL != 2  // tuning ablation 2: no swish inside the group steps (wrong results)
    // OACT with a narrowed activation set (AS, f16x2): tile Q+1's activation
    // here too, beside this group's MFMAs (not serially at the layer end)
    if constexpr (!OACT || (NT == 2 && AS != 0)) x3_act_tile<NT, OACT, AS>(hb[Q + 1], isc, act);
#endif
    splitk<NT, 0>(hb[Q + 1], cs);
  }
#pragma unroll
  for (int o = 0; o < NOUT; ++o) {
#if ZF_X3_ABL == 1
    acc[o] = mfma_split<NT>(a1, s1, acc[o]);
#else
    E a[NT];
    load_frag<NT>(lb + (((NOUT + o) * NT) << 10), a);
    acc[o] = mfma_split<NT>(a, s1, acc[o]);
#endif
  }
  if constexpr (HASB) {
    // the layer end, acc * us + bias; each bias tile read as it is used, after
    // the group's MFMAs (no 16 x NOUT registers held across them)
#pragma unroll
    for (int o = 0; o < NOUT; ++o) acc[o] = x3_finish<NT>(acc[o], us, bias_acc(bias + o * 32, hh));
  }
  char* const t = p.cur;
  p.cur = p.nxt;
  p.nxt = t;
  p.g += 1;
}


// One product term of a (k-step, tile) triple: j = 0: lo*hi, 1: hi*lo, 2: hi*hi
// (f16x2, small terms first as mfma_split).
__device__ __forceinline__ floatx16 mfma_term2(const halfx8 (&a)[2], const halfx8 (&b)[2], int j, floatx16 acc) {
  if (j == 0) return __builtin_amdgcn_mfma_f32_32x32x16_f16(a[1], b[0], acc, 0, 0, 0);
  if (j == 1) return __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[1], acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[0], acc, 0, 0, 0);
}

// VALU work items of slot m of x3_step_slots (a slot's items are independent
// of each other, so none waits on another's latency inside the slot):
//   slot 0: hi terms of the split of (Q, 1); slot 1: its lo terms;
//   swish of tile Q+1 as a 4-stage modulo pipeline, value i: exp at slot
//   i+1, fma at i+2, rcp at i+3, mul at i+4 (ring of 4 temporaries);
//   split of (Q+1, 0) (needs values 0..7, whose muls end at slot 11): hi at
//   slot max(12, 3 NOUT), lo one slot later — after the k-step-0 MFMAs that read cs.
// Slots past the group's last MFMA run after it, in the same order.
template <int T, int NOUT, int Q, int m>
__device__ __forceinline__ void x3_valu_slot(floatx16 (&hb)[T], halfx8 (&cs)[2], halfx8 (&s1)[2], float (&tq)[4],
                                             uint32_t (&s1h)[4], uint32_t (&csh)[4], float c) {
  // the split of (Q+1, 0) overwrites cs: not before the last k-step-0 MFMA (slot 3 NOUT - 1)
  constexpr int kCs = 3 * NOUT > 12 ? 3 * NOUT : 12;
  if constexpr (m == 0) split8h_hi<1>(hb[Q], s1h);
  if constexpr (m == 1) split8h_lo<1>(hb[Q], s1h, s1[0], s1[1]);
  if constexpr (Q + 1 < T) {
    constexpr int i0 = m - 1, i1 = m - 2, i2 = m - 3, i3 = m - 4;
    if constexpr (i3 >= 0 && i3 < 16) {
      hb[Q + 1][i3] = hb[Q + 1][i3] * tq[i3 & 3];
      // pin the value here: values 8..15 are only read by the next group's
      // split, and machine sinking would otherwise move their whole chain there
      asm volatile("" ::"v"(hb[Q + 1][i3]));
    }
    if constexpr (i2 >= 0 && i2 < 16) tq[i2 & 3] = __builtin_amdgcn_rcpf(tq[i2 & 3]);
    if constexpr (i1 >= 0 && i1 < 16) tq[i1 & 3] = __builtin_fmaf(tq[i1 & 3], c, c);
    if constexpr (i0 >= 0 && i0 < 16) tq[i0 & 3] = __builtin_amdgcn_exp2f(-hb[Q + 1][i0]);
    if constexpr (m == kCs) split8h_hi<0>(hb[Q + 1], csh);
    if constexpr (m == kCs + 1) split8h_lo<0>(hb[Q + 1], csh, cs[0], cs[1]);
  }
}

// Slot m: one MFMA term of triple m / 3 (the next triple's A fragments read
// at its first term), then the slot's VALU, then a scheduling barrier that
// keeps the compiler from regrouping the MFMAs.
template <int T, int NOUT, int Q, int m>
__device__ __forceinline__ void x3_slot(const char* lb, floatx16 (&hb)[T], floatx16 (&acc)[NOUT],
                                        halfx8 (&fr)[2][2], halfx8 (&cs)[2], halfx8 (&s1)[2], float (&tq)[4],
                                        uint32_t (&s1h)[4], uint32_t (&csh)[4], float c) {
  constexpr int t = m / 3, j = m % 3, ks = t / NOUT, o = t % NOUT;
  if constexpr (j == 0 && t + 1 < 2 * NOUT) load_frag<2>(lb + (((t + 1) * 2) << 10), fr[(t + 1) & 1]);
  if constexpr (ks == 0) acc[o] = mfma_term2(fr[t & 1], cs, j, acc[o]);
  else acc[o] = mfma_term2(fr[t & 1], s1, j, acc[o]);
  x3_valu_slot<T, NOUT, Q, m>(hb, cs, s1, tq, s1h, csh, c);
#if ZF_X3_ABL == 12 || ZF_X3_ABL == 13  // tuning: extra VALU in the group slots (12: v_add, 13: v_exp), 8 per group
  if constexpr (j == 0) {
    float dd;
    if (ZF_X3_ABL == 12) asm volatile("v_add_f32 %0, %1, %2" : "=v"(dd) : "v"(acc[o][0]), "v"(acc[o][1]));
    else asm volatile("v_exp_f32 %0, %1" : "=v"(dd) : "v"(acc[o][0]));
  }
#endif
  __builtin_amdgcn_sched_barrier(0);
}

template <int T, int NOUT, int Q, int... M>
__device__ __forceinline__ void x3_slots_all(std::integer_sequence<int, M...>, const char* lb, floatx16 (&hb)[T],
                                             floatx16 (&acc)[NOUT], halfx8 (&fr)[2][2], halfx8 (&cs)[2],
                                             halfx8 (&s1)[2], float (&tq)[4], uint32_t (&s1h)[4],
                                             uint32_t (&csh)[4], float c) {
  (x3_slot<T, NOUT, Q, M>(lb, hb, acc, fr, cs, s1, tq, s1h, csh, c), ...);
}

template <int T, int NOUT, int Q, int... M>
__device__ __forceinline__ void x3_valu_tail(std::integer_sequence<int, M...>, floatx16 (&hb)[T], halfx8 (&cs)[2],
                                             halfx8 (&s1)[2], float (&tq)[4], uint32_t (&s1h)[4],
                                             uint32_t (&csh)[4], float c) {
  (x3_valu_slot<T, NOUT, Q, 2 * NOUT * 3 + M>(hb, cs, s1, tq, s1h, csh, c), ...);
}

// f16x2, hidden 128, swish: the step as 2 x NOUT x 3 MFMA slots in a fixed
// order, each slot = one MFMA + its share of the step's VALU (the split of
// k-step (Q, 1), the swish of tile Q+1 one value per slot, the split of
// (Q+1, 0)), pinned by scheduling barriers, so the VALU issues between the
// MFMAs of the wave's own dependent triples instead of after them; the A
// fragments of the next triple are read one triple ahead.
template <int T, int NOUT, int Q, bool HASB>
__device__ __forceinline__ void x3_step_slots(const char* __restrict__ x3, X3Pipe& p, floatx16 (&hb)[T],
                                              floatx16 (&acc)[NOUT], int lane, const float* __restrict__ bias,
                                              int hh, halfx8 (&cs)[2], float isc, float us) {
  constexpr int NT = 2;
#ifdef ZF_X3_TRACE
  const unsigned long long tb0 = X3T_NOW();
#endif
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#ifdef ZF_X3_TRACE
  p.tbar += X3T_NOW() - tb0;
#endif
  x3_issue_next<NT, T>(x3, p, p.nxt, lane);
  const char* lb = p.cur + lane * 16;
  halfx8 fr[2][NT];
  load_frag<NT>(lb, fr[0]);
  halfx8 s1[NT];
  constexpr int kSlots = 2 * NOUT * 3;
  // VALU work items by slot (a slot's items are independent of each other,
  // so none waits on another's latency inside the slot):
  //   slot 0: hi terms of the split of (Q, 1); slot 1: its lo terms;
  //   swish of tile Q+1 as a 4-stage modulo pipeline, value i: exp at slot
  //   i+1, fma at i+2, rcp at i+3, mul at i+4 (ring of 4 temporaries);
  //   split of (Q+1, 0) (needs values 0..7: their muls end at slot 11):
  //   hi at slot 12, lo at slot 13 — after the k-step-0 MFMAs that read cs.
  // Stages that fall past the last slot run after it, in the same order.
  float tq[4];
  uint32_t s1h[4], csh[4];
  x3_slots_all<T, NOUT, Q>(std::make_integer_sequence<int, kSlots>{}, lb, hb, acc, fr, cs, s1, tq, s1h, csh, isc);
  // the stages that did not fit in the slots (small groups), in slot order
  x3_valu_tail<T, NOUT, Q>(std::make_integer_sequence<int, (kSlots < 20 ? 20 - kSlots : 0)>{}, hb, cs, s1, tq,
                           s1h, csh, isc);
  static_assert(kSlots >= 2, "at least one triple per k-step");
  if constexpr (HASB) {
    // the layer end, acc * us + bias, one fma per value; the bias tiles are
    // read here, when the layer's input tiles are dead (no registers held
    // across the group's MFMAs)
#pragma unroll
    for (int o = 0; o < NOUT; ++o) acc[o] = x3_finish<NT>(acc[o], us, bias_acc(bias + o * 32, hh));
  }
  char* const t = p.cur;
  p.cur = p.nxt;
  p.nxt = t;
  p.g += 1;
}

// Early per-sample scale (x3_early_scale, f16x2 swish at hidden 128): the
// scale of a layer input from a bound instead of the exact maximum of the
// previous layer's pre-activations, so it is known before that layer ends
// and the layer's last group step can finish its tiles and swish + split the
// next layer's tile 0 beside its own MFMAs (x3_step_slots_last) instead of
// after them.  With R, B of DevOp::x3_rb, every pre-activation of Dense_l
// obeys |v'_j| <= R_l * max_k |a_k| + B_l, and |swish(v)| <= |v| <= |v'|:
// U_0 = R_0 max|u| + B_0 (u the BatchNorm'd conditioner inputs), U_l =
// R_l U_{l-1} + B_l.  The scale is that of x3_act_scale with U in place of
// the maximum (U >= the maximum, so no split operand exceeds 2^14); the split
// terms of in-range values are the exact ones scaled by a power of two, so the
// MFMA sums are the same bits as with the exact scale unless the bound is so
// loose (> 2^13) that some residual terms fall below fp16's normal range.
__device__ __forceinline__ void x3_scale_from(float U, int kw, float& isc, float& us, float& ius) {
  // a bound that overflowed (R * max |a| + B > FLT_MAX while the values are
  // finite) would give frexp's exponent 0 for inf and a 2^14 scale: clamp it,
  // so the scale stays at or above every finite value's
  const int e = max(__builtin_amdgcn_frexp_expf(fminf(U, 3.40282347e38f)), -60);
  isc = __builtin_amdgcn_ldexpf(kSwishPrescale, e - 14);
  us = __builtin_amdgcn_ldexpf(1.0f, e - 14 - kw);
  ius = __builtin_amdgcn_ldexpf(1.0f, 14 + kw - e);
}

// The last group step of a layer (Q = T-1) in tile-major order: slot m
// multiplies (tile m / 6, k-step (m / 3) % 2, term m % 3), so tile o's sums
// are complete after slot 6o+5; its finish (acc * us + bias, the bias read
// two slots ahead) runs at slots 6o+7 / 6o+8, and NEXT: the next layer's
// tile 0 is swished with its scale constant cn (exp at slot 9+i, fma 10+i,
// rcp 11+i, mul 12+i for value i) and its k-step-0 split formed at slots
// 20 / 21 (into cs, after the last k-step-0 MFMA of this step read it at
// slot 20).  Stages past the last MFMA run after it in slot order.
template <bool CR>
__device__ __forceinline__ float x3_squareplus2_t(float x);

template <int T, int NOUT, bool NEXT, int SPT, int m>
__device__ __forceinline__ void x3_valu_slot_last(floatx16 (&hb)[T], floatx16 (&acc)[NOUT], halfx8 (&cs)[2],
                                                  halfx8 (&s1)[2], float (&tq)[4], uint32_t (&s1h)[4],
                                                  uint32_t (&csh)[4], floatx16& bt, const float* __restrict__ bias,
                                                  int hh, float us, float cn, float& mx) {
  constexpr int Q = T - 1;
  if constexpr (m == 0) split8h_hi<1>(hb[Q], s1h);
  if constexpr (m == 1) split8h_lo<1>(hb[Q], s1h, s1[0], s1[1]);
  constexpr int ob = (m - 4) / 6;  // bias of tile ob read at slot 6 ob + 4
  if constexpr (m >= 4 && (m - 4) % 6 == 0 && ob < NOUT) bt = bias_acc(bias + ob * 32, hh);
  constexpr int of = (m - 7) / 6;  // finish of tile of at slots 6 of + 7 (values 0-7) and 6 of + 8 (8-15)
  if constexpr (m >= 7 && of < NOUT && ((m - 7) % 6 == 0 || (m - 7) % 6 == 1)) {
    constexpr int r0 = (m - 7) % 6 == 0 ? 0 : 8;
#pragma unroll
    for (int r = r0; r < r0 + 8; ++r) acc[of][r] = __builtin_fmaf(acc[of][r], us, bt[r]);
  }
  // SPT (the last layer): tiles 0..SPT-1 hold spline width / height logits,
  // which the spline takes through 2 squareplus (x3_squareplus2): formed
  // here, two values per slot from slot 6o+9, beside the remaining MFMAs
#pragma unroll
  for (int o2 = 0; o2 < SPT && o2 < NOUT; ++o2) {
    const int rr = m - 9 - 6 * o2;  // compile-time after unrolling
    if (rr >= 0 && rr < 8) {
      acc[o2][2 * rr] = x3_squareplus2_t<false>(acc[o2][2 * rr]);
      acc[o2][2 * rr + 1] = x3_squareplus2_t<false>(acc[o2][2 * rr + 1]);
    }
  }
  // NEXT: the exact maximum |v'| of the finished values, one slot after their finish
  constexpr int oq = (m - 8) / 6;
  if constexpr (NEXT && m >= 8 && oq < NOUT && ((m - 8) % 6 == 0 || (m - 8) % 6 == 1)) {
    constexpr int r0 = (m - 8) % 6 == 0 ? 0 : 8;
#pragma unroll
    for (int r = r0; r < r0 + 8; r += 2)  // one v_max3 per two values (the compiler forms a max / max3 tree: 1.5x)
      asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(mx) : "v"(acc[oq][r]), "v"(acc[oq][r + 1]));
  }
  if constexpr (NEXT) {
    constexpr int i0 = m - 9, i1 = m - 10, i2 = m - 11, i3 = m - 12;
    if constexpr (i3 >= 0 && i3 < 16) {
      acc[0][i3] = acc[0][i3] * tq[i3 & 3];
      asm volatile("" ::"v"(acc[0][i3]));
    }
    if constexpr (i2 >= 0 && i2 < 16) tq[i2 & 3] = __builtin_amdgcn_rcpf(tq[i2 & 3]);
    if constexpr (i1 >= 0 && i1 < 16) tq[i1 & 3] = __builtin_fmaf(tq[i1 & 3], cn, cn);
    if constexpr (i0 >= 0 && i0 < 16) tq[i0 & 3] = __builtin_amdgcn_exp2f(-acc[0][i0]);
    if constexpr (m == 20) split8h_hi<0>(acc[0], csh);
    if constexpr (m == 21) split8h_lo<0>(acc[0], csh, cs[0], cs[1]);
  }
}

template <int T, int NOUT, bool NEXT, int SPT, int m>
__device__ __forceinline__ void x3_slot_last(const char* lb, floatx16 (&hb)[T], floatx16 (&acc)[NOUT],
                                             halfx8 (&fr)[2][2], halfx8 (&cs)[2], halfx8 (&s1)[2], float (&tq)[4],
                                             uint32_t (&s1h)[4], uint32_t (&csh)[4], floatx16& bt,
                                             const float* __restrict__ bias, int hh, float us, float cn, float& mx) {
  constexpr int t = m / 3, j = m % 3, o = t / 2, ks = t % 2;
  constexpr int tn = t + 1, on = tn / 2, ksn = tn % 2;
  if constexpr (j == 0 && tn < 2 * NOUT) load_frag<2>(lb + (((ksn * NOUT + on) * 2) << 10), fr[tn & 1]);
  if constexpr (ks == 0) acc[o] = mfma_term2(fr[t & 1], cs, j, acc[o]);
  else acc[o] = mfma_term2(fr[t & 1], s1, j, acc[o]);
  x3_valu_slot_last<T, NOUT, NEXT, SPT, m>(hb, acc, cs, s1, tq, s1h, csh, bt, bias, hh, us, cn, mx);
  __builtin_amdgcn_sched_barrier(0);
}

template <int T, int NOUT, bool NEXT, int SPT, int... M>
__device__ __forceinline__ void x3_slots_all_last(std::integer_sequence<int, M...>, const char* lb,
                                                  floatx16 (&hb)[T], floatx16 (&acc)[NOUT], halfx8 (&fr)[2][2],
                                                  halfx8 (&cs)[2], halfx8 (&s1)[2], float (&tq)[4],
                                                  uint32_t (&s1h)[4], uint32_t (&csh)[4], floatx16& bt,
                                                  const float* __restrict__ bias, int hh, float us, float cn,
                                                  float& mx) {
  (x3_slot_last<T, NOUT, NEXT, SPT, M>(lb, hb, acc, fr, cs, s1, tq, s1h, csh, bt, bias, hh, us, cn, mx), ...);
}

template <int T, int NOUT, bool NEXT, int SPT, int... M>
__device__ __forceinline__ void x3_valu_tail_last(std::integer_sequence<int, M...>, floatx16 (&hb)[T],
                                                  floatx16 (&acc)[NOUT], halfx8 (&cs)[2], halfx8 (&s1)[2],
                                                  float (&tq)[4], uint32_t (&s1h)[4], uint32_t (&csh)[4],
                                                  floatx16& bt, const float* __restrict__ bias, int hh, float us,
                                                  float cn, float& mx) {
  (x3_valu_slot_last<T, NOUT, NEXT, SPT, 6 * NOUT + M>(hb, acc, cs, s1, tq, s1h, csh, bt, bias, hh, us, cn, mx),
   ...);
}

// A layer's last group step (see x3_valu_slot_last).  On return acc holds the
// finished pre-activations acc * us + bias, and NEXT: tile 0 swished with the
// next layer's constant cn and cs its k-step-0 split (what the next layer's
// first x3_step_slots expects of hb[0] / cs).
template <int T, int NOUT, bool NEXT, int SPT = 0>
__device__ __forceinline__ void x3_step_slots_last(const char* __restrict__ x3, X3Pipe& p, floatx16 (&hb)[T],
                                                   floatx16 (&acc)[NOUT], int lane, const float* __restrict__ bias,
                                                   int hh, halfx8 (&cs)[2], float us, float cn, float& mx) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  x3_issue_next<2, T>(x3, p, p.nxt, lane);
  const char* lb = p.cur + lane * 16;
  halfx8 fr[2][2];
  load_frag<2>(lb, fr[0]);
  halfx8 s1[2];
  float tq[4];
  uint32_t s1h[4], csh[4];
  floatx16 bt;
  constexpr int kSlots = 6 * NOUT;
  constexpr int kEnd0 = NEXT ? (6 * NOUT > 28 ? 6 * NOUT : 28) : 6 * (NOUT - 1) + 9;
  constexpr int kEnd = SPT > 0 && 6 * (SPT - 1) + 17 > kEnd0 ? 6 * (SPT - 1) + 17 : kEnd0;
  mx = 0.f;
  x3_slots_all_last<T, NOUT, NEXT, SPT>(std::make_integer_sequence<int, kSlots>{}, lb, hb, acc, fr, cs, s1, tq, s1h,
                                        csh, bt, bias, hh, us, cn, mx);
  x3_valu_tail_last<T, NOUT, NEXT, SPT>(std::make_integer_sequence<int, (kEnd > kSlots ? kEnd - kSlots : 0)>{}, hb,
                                        acc, cs, s1, tq, s1h, csh, bt, bias, hh, us, cn, mx);
  char* const t = p.cur;
  p.cur = p.nxt;
  p.nxt = t;
  p.g += 1;
}

// Fused swish + split (ZF_X3_FUSED): the hi / lo fp16 terms of the exact
// product v' * r of act_swish (one rounding each, v_fma_mix{lo,hi}: hi =
// RN16(v' r), lo = RN16(v' r - hi)) instead of the fp32 product, a
// conversion and the residual: 2 VALU per value instead of 2.5.  Value 2p of
// a k-step goes to the low halves of h[p] / l[p], value 2p + 1 to the high
// halves.  Their consumers are MFMAs of the next group step (behind its
// barrier), so no hazard pad is needed here.
template <int ODD>
__device__ __forceinline__ void mix_hi(uint32_t& h, float v, float r) {
  if constexpr (ODD == 0) asm("v_fma_mixlo_f16 %0, %1, %2, 0" : "=v"(h) : "v"(v), "v"(r));
  else asm("v_fma_mixhi_f16 %0, %1, %2, 0" : "+v"(h) : "v"(v), "v"(r));
}
template <int ODD>
__device__ __forceinline__ void mix_lo(uint32_t& l, float v, float r, uint32_t h) {
  if constexpr (ODD == 0)
    asm("v_fma_mixlo_f16 %0, %1, %2, -%3 op_sel_hi:[0,0,1]" : "=v"(l) : "v"(v), "v"(r), "v"(h));
  else
    asm("v_fma_mixhi_f16 %0, %1, %2, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(l) : "v"(v), "v"(r), "v"(h));
}

// Slot m's VALU in the fused schedule: Q == 0 splits its k-step 1 at slots
// 0 / 1 (tile 0 arrives swished in fp32); tile Q+1 runs as a 5-stage modulo
// pipeline, value i: exp at slot i+1, fma at i+2, rcp at i+3, hi at i+4, lo
// at i+5, into nh / nl (pairs 0-3: k-step 0, 4-7: k-step 1).
template <int T, int NOUT, int Q, int m>
__device__ __forceinline__ void x3_valu_slot_f(floatx16 (&hb)[T], halfx8 (&s1)[2], uint32_t (&s1h)[4],
                                               float (&tq)[5], uint32_t (&nh)[8], uint32_t (&nl)[8], float c) {
  if constexpr (Q == 0 && m == 0) split8h_hi<1>(hb[0], s1h);
  if constexpr (Q == 0 && m == 1) split8h_lo<1>(hb[0], s1h, s1[0], s1[1]);
  if constexpr (Q + 1 < T) {
    constexpr int i0 = m - 1, i1 = m - 2, i2 = m - 3, i3 = m - 4, i4 = m - 5;
    if constexpr (i4 >= 0 && i4 < 16) mix_lo<i4 & 1>(nl[i4 >> 1], hb[Q + 1][i4], tq[i4 % 5], nh[i4 >> 1]);
    if constexpr (i3 >= 0 && i3 < 16) mix_hi<i3 & 1>(nh[i3 >> 1], hb[Q + 1][i3], tq[i3 % 5]);
    if constexpr (i2 >= 0 && i2 < 16) tq[i2 % 5] = __builtin_amdgcn_rcpf(tq[i2 % 5]);
    if constexpr (i1 >= 0 && i1 < 16) tq[i1 % 5] = __builtin_fmaf(tq[i1 % 5], c, c);
    if constexpr (i0 >= 0 && i0 < 16) tq[i0 % 5] = __builtin_amdgcn_exp2f(-hb[Q + 1][i0]);
  }
}

template <int T, int NOUT, int Q, int m>
__device__ __forceinline__ void x3_slot_f(const char* lb, floatx16 (&hb)[T], floatx16 (&acc)[NOUT],
                                          halfx8 (&fr)[2][2], halfx8 (&cs)[2], halfx8 (&s1)[2], uint32_t (&s1h)[4],
                                          float (&tq)[5], uint32_t (&nh)[8], uint32_t (&nl)[8], float c) {
  constexpr int t = m / 3, j = m % 3, ks = t / NOUT, o = t % NOUT;
  if constexpr (j == 0 && t + 1 < 2 * NOUT) load_frag<2>(lb + (((t + 1) * 2) << 10), fr[(t + 1) & 1]);
  if constexpr (ks == 0) acc[o] = mfma_term2(fr[t & 1], cs, j, acc[o]);
  else acc[o] = mfma_term2(fr[t & 1], s1, j, acc[o]);
  x3_valu_slot_f<T, NOUT, Q, m>(hb, s1, s1h, tq, nh, nl, c);
  __builtin_amdgcn_sched_barrier(0);
}

template <int T, int NOUT, int Q, int... M>
__device__ __forceinline__ void x3_slots_all_f(std::integer_sequence<int, M...>, const char* lb, floatx16 (&hb)[T],
                                               floatx16 (&acc)[NOUT], halfx8 (&fr)[2][2], halfx8 (&cs)[2],
                                               halfx8 (&s1)[2], uint32_t (&s1h)[4], float (&tq)[5],
                                               uint32_t (&nh)[8], uint32_t (&nl)[8], float c) {
  (x3_slot_f<T, NOUT, Q, M>(lb, hb, acc, fr, cs, s1, s1h, tq, nh, nl, c), ...);
}

template <int T, int NOUT, int Q, int... M>
__device__ __forceinline__ void x3_valu_tail_f(std::integer_sequence<int, M...>, floatx16 (&hb)[T], halfx8 (&s1)[2],
                                               uint32_t (&s1h)[4], float (&tq)[5], uint32_t (&nh)[8],
                                               uint32_t (&nl)[8], float c) {
  (x3_valu_slot_f<T, NOUT, Q, 2 * NOUT * 3 + M>(hb, s1, s1h, tq, nh, nl, c), ...);
}

// x3_step_slots with the fused swish + split: cs / s1 hold tile Q's k-step
// 0 / 1 terms (s1 formed here for Q == 0), and leave tile Q+1's.
template <int T, int NOUT, int Q, bool HASB>
__device__ __forceinline__ void x3_step_slots_f(const char* __restrict__ x3, X3Pipe& p, floatx16 (&hb)[T],
                                                floatx16 (&acc)[NOUT], int lane, const float* __restrict__ bias,
                                                int hh, halfx8 (&cs)[2], halfx8 (&s1)[2], float isc, float us) {
  constexpr int NT = 2;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  x3_issue_next<NT, T>(x3, p, p.nxt, lane);
  const char* lb = p.cur + lane * 16;
  halfx8 fr[2][NT];
  load_frag<NT>(lb, fr[0]);
  constexpr int kSlots = 2 * NOUT * 3;
  float tq[5];
  uint32_t s1h[4], nh[8], nl[8];
  x3_slots_all_f<T, NOUT, Q>(std::make_integer_sequence<int, kSlots>{}, lb, hb, acc, fr, cs, s1, s1h, tq, nh, nl,
                             isc);
  x3_valu_tail_f<T, NOUT, Q>(std::make_integer_sequence<int, (kSlots < 21 ? 21 - kSlots : 0)>{}, hb, s1, s1h, tq,
                             nh, nl, isc);
  if constexpr (HASB) {
#pragma unroll
    for (int o = 0; o < NOUT; ++o) acc[o] = x3_finish<NT>(acc[o], us, bias_acc(bias + o * 32, hh));
  }
  if constexpr (Q + 1 < T) {
    __builtin_memcpy(&cs[0], &nh[0], 16);
    __builtin_memcpy(&cs[1], &nl[0], 16);
    __builtin_memcpy(&s1[0], &nh[4], 16);
    __builtin_memcpy(&s1[1], &nl[4], 16);
  }
  char* const t = p.cur;
  p.cur = p.nxt;
  p.nxt = t;
  p.g += 1;
}

// Dim-pair last layer (PAIRS, f16x2): the layer input is split once, before
// the pair loop (sp[tile][k-step] = hi / lo), so each pair's group steps are
// MFMAs and fragment reads only (the plain steps re-split every tile per
// pair).  A fragments one (k-step, tile) ahead.
template <int T, int NOUT, int Q>
__device__ __forceinline__ void x3_step_pre(const char* __restrict__ x3, X3Pipe& p, const halfx8 (&sp)[T][2][2],
                                            floatx16 (&acc)[NOUT], int lane) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  x3_issue_next<2, T>(x3, p, p.nxt, lane);
  const char* lb = p.cur + lane * 16;
  halfx8 c[2];
  load_frag<2>(lb, c);
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int o = 0; o < NOUT; ++o) {
      const int t = s * NOUT + o;
      halfx8 n[2];
      if (t + 1 < 2 * NOUT) load_frag<2>(lb + (((t + 1) * 2) << 10), n);
      acc[o] = mfma_split<2>(c, sp[Q][s], acc[o]);
      if (t + 1 < 2 * NOUT) {
        c[0] = n[0];
        c[1] = n[1];
      }
    }
  char* const tb = p.cur;
  p.cur = p.nxt;
  p.nxt = tb;
  p.g += 1;
}

template <int T, int NOUT, int Q = 0>
__device__ __forceinline__ void x3_layer_pre(const char* __restrict__ x3, X3Pipe& p, const halfx8 (&sp)[T][2][2],
                                             floatx16 (&acc)[NOUT], int lane) {
  x3_step_pre<T, NOUT, Q>(x3, p, sp, acc, lane);
  if constexpr (Q + 1 < T) x3_layer_pre<T, NOUT, Q + 1>(x3, p, sp, acc, lane);
}

// A pipelined layer: hb[0] already swished, cs = split of (0, 0).
template <int NT, int T, int NOUT, bool HASB, bool OACT, int Q = 0, int AS = 0>
__device__ __forceinline__ void x3_layer_pipe(const char* __restrict__ x3, X3Pipe& p, floatx16 (&hb)[T],
                                              floatx16 (&acc)[NOUT], int lane, const float* bias_last, int hh,
                                              typename XT<NT>::E (&cs)[NT], float isc, float us, int act,
                                              halfx8 (&fused_s1)[2]) {
#ifndef ZF_X3_FUSED
#define ZF_X3_FUSED 0
#endif
  if constexpr (NT == 2 && !OACT && ZF_X3_FUSED) {  // the swish kernels, fused swish + split
    static_assert(sizeof(typename XT<NT>::E) == 16, "halfx8 terms");
    halfx8(&s1)[2] = fused_s1;
    if constexpr (Q + 1 < T) {
      x3_step_slots_f<T, NOUT, Q, false>(x3, p, hb, acc, lane, nullptr, hh, cs, s1, isc, us);
      x3_layer_pipe<NT, T, NOUT, HASB, OACT, Q + 1>(x3, p, hb, acc, lane, bias_last, hh, cs, isc, us, act, s1);
    } else {
      x3_step_slots_f<T, NOUT, Q, HASB>(x3, p, hb, acc, lane, bias_last, hh, cs, s1, isc, us);
    }
    return;
  }
  if constexpr (NT == 2 && !OACT) {  // the swish kernels: explicit MFMA slots (x3_step_slots)
    if constexpr (Q + 1 < T) {
      x3_step_slots<T, NOUT, Q, false>(x3, p, hb, acc, lane, nullptr, hh, cs, isc, us);
      x3_layer_pipe<NT, T, NOUT, HASB, OACT, Q + 1>(x3, p, hb, acc, lane, bias_last, hh, cs, isc, us, act,
                                                    fused_s1);
    } else {
      x3_step_slots<T, NOUT, Q, HASB>(x3, p, hb, acc, lane, bias_last, hh, cs, isc, us);
    }
    return;
  }
  if constexpr (Q + 1 < T) {
    x3_step_pipe<NT, T, NOUT, Q, false, OACT, AS>(x3, p, hb, acc, lane, nullptr, hh, cs, isc, us, act);
    x3_layer_pipe<NT, T, NOUT, HASB, OACT, Q + 1, AS>(x3, p, hb, acc, lane, bias_last, hh, cs, isc, us, act,
                                                      fused_s1);
  } else {
    x3_step_pipe<NT, T, NOUT, Q, HASB, OACT, AS>(x3, p, hb, acc, lane, bias_last, hh, cs, isc, us, act);
  }
}

// A layer of the early-scale path (f16x2 swish, hidden 128): steps 0..T-2 as
// x3_step_slots (the layer input's tiles 1..T-1 swished with c in their
// slots), then x3_step_slots_last (finish; NEXT: the next layer's tile 0
// swished with cn and split into cs).
template <int T, int NOUT, bool NEXT, int SPT = 0, int Q = 0>
__device__ __forceinline__ void x3_layer_early(const char* __restrict__ x3, X3Pipe& p, floatx16 (&hb)[T],
                                               floatx16 (&acc)[NOUT], int lane, const float* __restrict__ bias,
                                               int hh, halfx8 (&cs)[2], float c, float us, float cn, float& mx) {
  if constexpr (Q + 1 < T) {
    x3_step_slots<T, NOUT, Q, false>(x3, p, hb, acc, lane, nullptr, hh, cs, c, us);
    x3_layer_early<T, NOUT, NEXT, SPT, Q + 1>(x3, p, hb, acc, lane, bias, hh, cs, c, us, cn, mx);
  } else {
    x3_step_slots_last<T, NOUT, NEXT, SPT>(x3, p, hb, acc, lane, bias, hh, cs, us, cn, mx);
  }
}

// A whole streamed Dense layer: T groups (one per input tile).
template <int NT, int T, int NOUT, bool SW, bool OACT, int Q = 0>
__device__ __forceinline__ void x3_layer(const char* __restrict__ x3, X3Pipe& p, floatx16 (&hb)[T],
                                         floatx16 (&acc)[NOUT], int lane, const float* bias_last, int hh,
                                         float isc, float us, int act) {
  if constexpr (Q + 1 < T) {
    x3_step<NT, T, NOUT, Q, SW, OACT>(x3, p, hb, acc, lane, nullptr, hh, isc, us, act);
    x3_layer<NT, T, NOUT, SW, OACT, Q + 1>(x3, p, hb, acc, lane, bias_last, hh, isc, us, act);
  } else {
    x3_step<NT, T, NOUT, Q, SW, OACT>(x3, p, hb, acc, lane, bias_last, hh, isc, us, act);
  }
}

// Conditioner input + first Dense (bijectors.py:341-343) as zf_flow_dev.h's
// layer0, with this NSC's small parameters from its LDS region `par` (offsets
// relative to op.bn) and the conditions from the per-wave state (columns D..)
// — no global load on the per-coupling path, so no vmcnt wait there drains
// the weight-group DMA in flight.
template <int T, bool OACT>
__device__ __forceinline__ void x3_layer0(const X3Sc& c, const float* par, const float* xs, int rot, int D,
                                          int s, int hh, int lane, floatx16 (&hb)[T], int swish_tiles,
                                          float* umax = nullptr) {
  const int dt = c.dt, dc = c.dc, DC = c.DC, KS0 = c.KS0;
  const int DCp = 2 * KS0;
  const float* bn = par;
  const float* w0b = par + c.w0_rel;
  const float* b0 = par + c.b_rel;
#pragma unroll
  for (int o = 0; o < T; ++o) hb[o] = bias_acc(b0 + o * 32, hh);
  for (int ks = 0; ks < KS0; ++ks) {
    const int k = 2 * ks + hh;
    float v = 0.f;
    if (k < dc) v = xs[wrap(dt + k + rot, D) * 32 + s];
    else if (k < DC) v = xs[(D + k - dc) * 32 + s];
    const float u = (v - bn[k]) * bn[DCp + k] + bn[2 * DCp + k];
    if (umax != nullptr) *umax = fmaxf(*umax, fabsf(u));  // padding inputs are 0: bn rows give u = 0
    const float* w0 = w0b + ks * 64 + lane;
#pragma unroll
    for (int o = 0; o < T; ++o) hb[o] = __builtin_amdgcn_mfma_f32_32x32x2f32(w0[o * KS0 * 64], u, hb[o], 0, 0, 0);
  }
#pragma unroll
  for (int o = 0; o < T; ++o)
    if (o < swish_tiles) {  // bf16x3 only (f16x2 passes 0)
      if constexpr (OACT) {
        x3_act_tile<3, true>(hb[o], 1.f, c.act);
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) hb[o][r] = swish(hb[o][r]);
      }
    }
}

// Spline arithmetic of the split-MFMA kernel: the spline parameters already differ from the reference's in the last ulp
// (GEMM summation order), so the per-lane spline uses ~1-ulp hardware forms:
// squareplus from v_sqrt_f32 (no Newton step), quotients from a refined
// reciprocal, and the log-det as ONE log of the product of its three terms
// (2 log(sk+eps) + log(num2+eps) - 2 log(den+eps), utils.py:133-135).
// Parity is checked by the same per-sample tolerance as every other path.
__device__ __forceinline__ float x3_squareplus(float x) {
  return 0.5f * (x + __builtin_amdgcn_sqrtf(__builtin_fmaf(x, x, 4.0f)));
}

// 2*squareplus(x): the widths and heights are normalised by their sum, so the
// factor 1/2 cancels exactly (a power of two): bit-identical knots.
__device__ __forceinline__ float x3_squareplus2(float x) {
  return x + __builtin_amdgcn_sqrtf(__builtin_fmaf(x, x, 4.0f));
}

__device__ __forceinline__ void x3_forward_eval(float x, const RqsBin& b, float& y, float& ld) {
  const float rw = rcp_refined(b.w);
  const float sk = b.h * rw;
  const float zr = (x - b.xk) * rw;  // :122
  const float z = (zr != zr) ? zr : fminf(fmaxf(zr, kEps), kOneMinusEps);
  const float az = 1.0f - z;
  const float num = b.h * z * (sk * z + b.dk * az);                // :125
  const float den = sk + (b.dkp1 + b.dk - 2.0f * sk) * z * az;     // :126
  const float rd = rcp_refined(den + kEps);
  const float yv = b.yk + num * rd;                                // :127
  y = b.oob ? x : yv;                                              // :130
  const float num2 = z * (b.dkp1 * z + 2.0f * sk * az) + b.dk * (az * az);  // :133
  const float sq = (sk + kEps) * rd;
  const float l = __logf((num2 + kEps) * (sq * sq));
  ld = b.oob ? 0.0f : l;                                           // :138
}

// The activation-switch kernels (OACT: relu ... softplus) take squareplus
// with a correctly rounded square root (rsq + one residual step), as the
// reference's fp32 jnp.sqrt: unbounded activations under large weights
// (softplus, tiny-activation regime) drive the last layer's logits to
// -5e3, where x + sqrt(x^2 + 4) cancels to the square root's last bit and a
// 1-ulp hardware sqrt doubles the reference's rounding there (mean error
// 1.7x the fp32 oracle's; with this form the CPU emulation of the kernel's
// arithmetic gives 1.1x).  The swish kernels keep the hardware form (-4
// VALU per parameter; their bounded-magnitude tests are at the oracle's level).
__device__ __forceinline__ float x3_sqrt_cr(float a) {
  const float y = __builtin_amdgcn_rsqf(a);
  const float sq = a * y;
  const float r = __builtin_fmaf(__builtin_fmaf(-sq, sq, a), 0.5f * y, sq);
  return a == __builtin_huge_valf() ? a : r;  // x^2 + 4 = inf: sqrt = inf, as jnp.sqrt
}
template <bool CR>
__device__ __forceinline__ float x3_squareplus2_t(float x) {
  const float a = __builtin_fmaf(x, x, 4.0f);
  return x + (CR ? x3_sqrt_cr(a) : __builtin_amdgcn_sqrtf(a));
}
template <bool CR>
__device__ __forceinline__ float x3_squareplus_t(float x) {
  const float a = __builtin_fmaf(x, x, 4.0f);
  return 0.5f * (x + (CR ? x3_sqrt_cr(a) : __builtin_amdgcn_sqrtf(a)));
}

// Bin selection over a power-of-two number of bins N by halving (log2 N
// compares, each followed by selects of the upper or lower half): bins
// base..base+N-1 have left knots X / Y, raw widths Wd / heights Ht and knot
// slope logits S (N + 1: both ends of every bin).  For strictly increasing
// knots this is the last bin whose left knot is <= v (and bin 0 for v below
// knot 1, or NaN): the same bin as the linear sweep of rqs_bin_monotone, with
// 4 compares and 79 selects at K = 16 instead of 15 and 90.
template <bool FWD, int N, int MX>
__device__ __forceinline__ void x3_bsel(float v, const float (&X)[MX], const float (&Y)[MX], const float (&Wd)[N],
                                        const float (&Ht)[N], const float (&S)[N + 1], float (&out)[6]) {
  static_assert(MX >= N, "knot arrays cover the bins");
  if constexpr (N == 1) {
    out[0] = X[0]; out[1] = Y[0]; out[2] = Wd[0]; out[3] = Ht[0]; out[4] = S[0]; out[5] = S[1];
  } else {
    constexpr int H = N / 2;
    const bool c = (FWD ? X[H] : Y[H]) <= v;
    float X2[H], Y2[H], W2[H], H2[H], S2[H + 1];
#pragma unroll
    for (int i = 0; i < H; ++i) {
      X2[i] = c ? X[H + i] : X[i];
      Y2[i] = c ? Y[H + i] : Y[i];
      W2[i] = c ? Wd[H + i] : Wd[i];
      H2[i] = c ? Ht[H + i] : Ht[i];
    }
#pragma unroll
    for (int i = 0; i <= H; ++i) S2[i] = c ? S[H + i] : S[i];
    x3_bsel<FWD, H, H>(v, X2, Y2, W2, H2, S2, out);
  }
}

// softmax_with_threshold's constants for a compile-time knot count (the
// kernel's K equals the couplings' real K): c * rnorm * j as literals.
template <int K>
struct KnotLit {
  static constexpr double c64 = 1e-5 / (1.0 - (double)K * 1e-5);
  static constexpr float c = (float)c64;
  static constexpr float norm = (float)(1.0 + c64 * (double)K);
  static constexpr float rnorm = (float)(1.0 / (double)norm);
  static constexpr float bc = c * rnorm;
};

// normalize_spline_params (utils.py:37-62) + the bin gather of
// _compute_rqs_input (utils.py:205-232) for one (sample, dim) per lane, from
// the raw logits P (widths P[0..K), heights P[K..2K), inner slopes
// P[2K..3K-1)).  With s_j = 2 squareplus(logit_j) (the factor 1/2 cancels in
// the quotient) and S = sum s_j, the normalised width is w_j = s_j a + bc
// (a = rnorm / S, bc = c rnorm: one fma, as before) and knot j is
// X_j = W_j a + j bc, W_j = s_0 + ... + s_{j-1} the raw running sum, which
// the normalisation forms anyway (its last term is S): one fma per knot
// instead of a normalising fma plus a running add.  The knots round
// differently from the reference's cumsum of normalised widths in the last
// ulp (as the fma'd widths already did); the spline is continuous across
// knots.  KLIT: j bc as literals (the kernel's K is the couplings' K); else
// from the runtime constants (padded knot counts).  Bin: x3_bsel; v at or
// beyond the last knot gives the idx == K fill (NaN width, height and right
// slope, utils.py:224-230) as rqs_bin_monotone.
template <bool FWD, int K, bool CR, bool KLIT, int NPV>
__device__ __forceinline__ RqsBin x3_bin(float v, const float (&P)[NPV], const KnotConsts& kc) {
  float ws[K], hs[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    ws[j] = x3_squareplus2_t<CR>(P[j]);
    hs[j] = x3_squareplus2_t<CR>(P[K + j]);
  }
  float X[K + 1], Y[K + 1];  // raw running sums, then knots
  X[0] = 0.f;
  Y[0] = 0.f;
  X[1] = ws[0];
  Y[1] = hs[0];
#pragma unroll
  for (int j = 1; j < K; ++j) {
    X[j + 1] = X[j] + ws[j];
    Y[j + 1] = Y[j] + hs[j];
  }
  const float rn = KLIT ? KnotLit<K>::rnorm : kc.rnorm;
  const float bc = KLIT ? KnotLit<K>::bc : kc.c * kc.rnorm;
  const float ax = rcp_refined(X[K]) * rn, ay = rcp_refined(Y[K]) * rn;
#pragma unroll
  for (int j = 1; j <= K; ++j) {
    const float jb = KLIT ? (float)j * KnotLit<K>::bc : (float)j * bc;
    X[j] = __builtin_fmaf(X[j], ax, jb);
    Y[j] = __builtin_fmaf(Y[j], ay, jb);
  }
  float S[K + 1];
  S[0] = 0.f;  // the boundary derivative 1 as the logit 0 (squareplus(0) == 1)
  S[K] = 0.f;
#pragma unroll
  for (int j = 1; j < K; ++j) S[j] = P[2 * K + j - 1];
  float o[6];
  x3_bsel<FWD, K, K + 1>(v, X, Y, ws, hs, S, o);
  RqsBin b;
  const bool sliver = (FWD ? X[K] : Y[K]) <= v;
  b.xk = sliver ? X[K] : o[0];
  b.yk = sliver ? Y[K] : o[1];
  b.w = sliver ? qnan() : __builtin_fmaf(o[2], ax, bc);
  b.h = sliver ? qnan() : __builtin_fmaf(o[3], ay, bc);
  const float lo = sliver ? 0.f : o[4];
  const float hi = sliver ? qnan() : o[5];
  b.dk = lo == 0.f ? 1.f : x3_squareplus_t<CR>(lo);
  b.dkp1 = hi == 0.f ? 1.f : x3_squareplus_t<CR>(hi);
  b.sk = b.h / b.w;
  b.oob = (v < 0.f) || (v >= 1.f);
  return b;
}

// Block: 4 waves x 32 samples, one 32-row input tile per weight group,
// double-buffered in LDS.  Small parameters (BatchNorm, first Dense, biases,
// ShiftBounds rows) are read from global memory (L2-resident), so the LDS
// footprint is 2 groups + the state: 50 KiB at T = 4 (3 blocks = 3 waves per
// SIMD, <= 168 VGPRs), 104 KiB at T = 8 (hidden 256: one block per CU, the
// 8 + 8 accumulator tiles need one wave's whole register file).
// ONE (one transformed dim, dim 2 or 3): the last layer's rows carry that
// dim's parameters in both lane halves (tile o, half h, register r =
// parameter 32o + 16h + r), so it takes ceil((3K-1)/32) tiles instead of
// ceil((3K-1)/16) half-empty ones, and the halves swap theirs by a lane
// shuffle before the spline.
// Waves per SIMD: hidden 128 with one dim pair and K <= 16 fits 168 VGPRs (3);
// a dim-pair loop keeps the hidden activations live across the last layer,
// and K = 32 holds 95 spline parameters per lane: 256 VGPRs (2); hidden 256
// needs the whole register file (1).  OACT kernels apply the activation to
// all tiles before the layer's groups instead of tile by tile inside them
// (a switch inside the pipelined steps spilled 110-130 VGPRs at 3 waves).
template <int T, int K, bool PAIRS>
constexpr int x3_occupancy() { return (T == 8 || K > 32) ? 1 : (PAIRS || K > 16) ? 2 : 3; }

template <int NT, int K, int T, bool PAIRS, bool ONE, bool INV, bool OACT, int ASET = 0>
__global__ __launch_bounds__(kX3Waves * 64, (x3_occupancy<T, K, PAIRS>())) void flow_kernel_x3(
    const DevFlow* __restrict__ F, const float* __restrict__ blob, const char* __restrict__ x3,
    const float* __restrict__ xin, const float* __restrict__ cin, float* __restrict__ y_out,
    const float* __restrict__ ld_in, float* __restrict__ ld_out, float* __restrict__ lp_out,
    double* __restrict__ block_partial, long long nparts, int op_begin, int op_end, long long N,
    unsigned long long seed, int gen) {
  // last-layer tiles per dim pair: 16 parameters per lane half (ONE: 32 of one dim per tile)
  constexpr int TL = ONE ? (3 * K - 1 + 31) / 32 : (3 * K - 1 + 15) / 16;
  constexpr int NPV = ONE ? 32 * TL : 16 * TL;  // spline parameters held per lane
  constexpr int NW = kX3Waves;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int D = F->D;
  const int C = F->C;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: scalar cursor math
  const int lane = threadIdx.x & 63;
  const int s = lane & 31;
  const int hh = lane >> 5;
  // one LDS weight buffer holds a hidden-layer group (T output tiles) or a
  // last-layer group (TL tiles: more than T at K = 32, hidden 128)
  constexpr int kBuf = group_bytes<NT>(T > TL ? T : TL);
  const int PB = F->x3_par_bytes;
  const int DS = D + C;  // state columns: x (rotated by `rot`), then c
  // LDS: [2][kBuf] weight groups | [2][PB] small parameters (NSCs alternate) |
  //      [NW][DS][32] state | [NW] partials
  char* par_lds = lds + 2 * kBuf;
  float* xs = reinterpret_cast<float*>(par_lds + 2 * PB) + wave * (32 * DS);
  double* s_part = reinterpret_cast<double*>(reinterpret_cast<float*>(par_lds + 2 * PB) + NW * 32 * DS);
  const float* sp = blob;
  const long long row = ((long long)blockIdx.x * NW + wave) * kTile + s;
  const bool valid = row < N;

  X3Pipe pipe;
  pipe.cur = lds;
  pipe.nxt = lds + kBuf;
  pipe.g = 0;
  pipe.wave = wave;
  {  // group 0 and the small parameters of the first NSC in execution order go
     // out before the state loads, so the block waits for one memory latency,
     // not two in a row
    int first = -1;
    const int nq = op_end - op_begin;
    for (int q = 0; q < nq; ++q) {
      const int oi = INV ? (op_end - 1 - q) : (op_begin + q);
      if (F->ops[oi].kind == ZF_OP_NSC) { first = oi; break; }
    }
    if (first >= 0) {
      const DevOp& fo = F->ops[first];
      x3_dma(x3 + fo.x3, pipe.cur, first_pieces<NT, T>(fo), wave, lane);
      x3_dma(reinterpret_cast<const char*>(blob + fo.bn), par_lds, fo.x3_par_pieces, wave, lane);
    }
  }
  load_state(xs, xin, row, valid, D, s, hh, F, seed, INV ? gen : 0);
  for (int j = hh; j < C; j += 2) xs[(D + j) * 32 + s] = valid ? cin[row * C + j] : 0.f;
  float ld = (ld_in != nullptr && valid) ? ld_in[row] : 0.f;
  int rot = 0;
  wave_lds_sync();
#ifdef ZF_X3_TRACE
  // slots: 0 start->first NSC, 1 layer 0, 2 hidden layers, 3 hidden->last
  // transition, 4 last layer, 5 spline, 6 epilogue, 7 barrier waits (inside
  // 2 and 4), 8 total, 9 couplings, 10 other ops
  unsigned long long tacc[kX3TraceSlots] = {};
  pipe.tbar = 0;
  pipe.tdma = 0;
  pipe.tgrp = 0;
  const unsigned long long t_begin = X3T_NOW();
  unsigned long long t_last = t_begin;
#define X3T(k)                                   \
  {                                              \
    const unsigned long long t_ = X3T_NOW();     \
    tacc[k] += t_ - t_last;                      \
    t_last = t_;                                 \
  }
#elif defined(ZF_X3_MARK)
  // tuning only: phase markers in the .s for per-phase static instruction counts
#define X3T(k) asm volatile(";ZFMARK " #k)
#else
#define X3T(k)
#endif
#ifdef ZF_X3_MARK
#define X3M(k) asm volatile(";ZFMARK " #k)
#else
#define X3M(k)
#endif
  pipe.par_src = nullptr;
  pipe.par_dst = nullptr;
  pipe.par_pieces = 0;
  {  // the first NSC's layer 0 reads the parameters before any group step's wait
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  int nsc_i = 0;  // NSCs entered, in execution order: parameter region nsc_i & 1

  const int nq = op_end - op_begin;
  for (int q = 0; q < nq; ++q) {
    const int oi = INV ? (op_end - 1 - q) : (op_begin + q);
    const DevOp& op = F->ops[oi];
    const X3Sc opc = x3_scalars<INV>(op);
    const int kind = opc.kind;
    if (kind == ZF_OP_ROLL) {  // bijectors.py:291 / :296
      rot = pmod(INV ? rot + opc.shift : rot - opc.shift, D);
    } else if (kind == ZF_OP_SHIFT_BOUNDS) {
      shift_bounds_op<INV>(sp + opc.sb, xs, s, hh, rot, D, ld);
      X3T(10);
    } else {  // ZF_OP_NSC, bijectors.py:329-371
      X3T(0);
#ifdef ZF_X3_TRACE
      tacc[9] += 1;
#endif
      {  // the next NSC's stream and parameters from this op's own record
        const bool has_next = opc.nxt >= op_begin && opc.nxt < op_end;
        pipe.span = make_span<NT, T>(opc, has_next);
        pipe.par_src = has_next ? reinterpret_cast<const char*>(blob + opc.nbn) : nullptr;
        pipe.par_dst = par_lds + ((nsc_i + 1) & 1) * PB;
        pipe.par_pieces = has_next ? opc.npar : 0;
      }
      pipe.g = 0;
      const float* par = reinterpret_cast<const float*>(par_lds + (nsc_i & 1) * PB);
      ++nsc_i;
      const int nh = opc.nh, act = opc.act, dt = opc.dt, kw_last = opc.kw_last;
      // this coupling's knots: a chain may mix knot counts up to the kernel's K
      // (x3_padded_knots); K - 1 real knots put the idx == K sliver at the
      // padded knot (rqs_bin_monotone padlast)
      const KnotConsts kc(opc.kreal);
      const bool padlast = opc.kreal == K - 1;
#ifdef ZF_X3_MARK
      const bool klit = true;  // marker builds: count one x3_bin copy
#else
      const bool klit = opc.kreal == K;  // x3_bin: the knot constants as literals
#endif
      // hidden biases are consecutive T x 32 blocks after Dense_0's (zf_flow.hip: b[l] = b[0] + l T 32)
      const long long b_rel = opc.b_rel + T * 32, blast_rel = opc.blast_rel;
      floatx16 hb[T];
      // The swish of a layer's output is deferred tile by tile into the next
      // streamed layer (x3_step, SW) — except before a PAIRS last layer,
      // which passes over its input once per dim pair.
      constexpr bool kLastSW = !PAIRS;
      constexpr bool kPipe = T == 4 && !PAIRS;
      // f16x2: every layer leaves raw pre-activations; the next streamed
      // layer scales and swishes them (act_swish) as it goes.
      // bf16x3 OACT: every tile's activation at the layer end (no switch inside
      // the group steps)
#ifndef ZF_X3_EARLY
#define ZF_X3_EARLY 1
#endif
      // f16x2 swish at hidden 128 (one dim pair): scales from bounds (x3_early_scale)
      constexpr bool kEarly = ZF_X3_EARLY && NT == 2 && !OACT && kPipe;
      // kEarly: the last layer's width / height tiles leave its last group
      // step as 2 squareplus (x3_step_slots_last SPT): K / 8 tiles of 16 per
      // lane half (one dim per half); ONE at K = 16: tile 0 (widths on half 0,
      // heights on half 1, the kSplitWH layout)
#ifndef ZF_X3_PRESP
#define ZF_X3_PRESP 1
#endif
      constexpr int kPreSP = (!ZF_X3_PRESP || !kEarly) ? 0 : !ONE ? K / 8 : (K == 16 ? 1 : 0);
      float umax = 0.f;
      x3_layer0<T, OACT>(opc, par, xs, rot, D, s, hh, lane, hb, NT == 2 ? 0 : (!OACT && (nh > 1 || kLastSW)) ? 1 : T,
                         kEarly ? &umax : nullptr);
      float eU = 0.f, eisc = 1.f, eus = 1.f, eius = 1.f;  // kEarly: bound and scales of the current layer input
      halfx8 ecs[2];  // kEarly: k-step-0 split of the current layer input's tile 0
      if constexpr (kEarly) {
        const X3Halves uq = x3_halves(umax);
        umax = fmaxf(uq.lo, uq.hi);
        eU = __builtin_fmaf(op.x3_rb[0][0], umax, op.x3_rb[0][1]);
        x3_scale_from(eU, nh > 1 ? opc.kw1 : kw_last, eisc, eus, eius);
        x3_act_tile<NT, false>(hb[0], eisc, act);
        split8h<0>(hb[0], ecs[0], ecs[1]);
      }
      // Hidden layers 1..n_hidden-1 (:343-345), T groups each.  bf16x3: the
      // biases seed the accumulators.  f16x2: they seed them divided by the
      // unscale (exact: powers of two) and the accumulators are multiplied
      // by it afterwards (kSeedScaled).
#ifndef ZF_X3_SEEDSCALED
#define ZF_X3_SEEDSCALED 0
#endif
      // f16x2 at hidden 128 (the slot schedule): zero-seeded accumulators and
      // one fma per value at the layer end (acc * us + bias) instead of a
      // bias * ius seed and an acc * us unscale (two multiplies per value)
      // (OACT too since round 5: a seeded bias sets the magnitude every MFMA
      // accumulation rounds at; sigmoid / softplus fold C colsum(W) into it,
      // 1e3-1e4 in the tiny-activation regime, where the zero-seeded sums of
      // the small centred terms plus one finish fma round far less)
      constexpr bool kSeedScaled = NT == 2 && (ZF_X3_SEEDSCALED || !kPipe);
      // the hidden layers of a dim-pair flow (d8, d16: PAIRS, 2 waves per
      // SIMD) and of hidden-256 flows (cfg5: T = 8, one wave per SIMD) take
      // the f16x2 slot schedule too: only the last layer, which re-reads its
      // input once per pair, keeps the plain group steps (d8 -2.1%, cfg5
      // -3.4% kernel time)
#ifndef ZF_X3_WIDE_PIPE
#define ZF_X3_WIDE_PIPE 1
#endif
#ifndef ZF_X3_PAIRS_PIPE
#define ZF_X3_PAIRS_PIPE 1
#endif
      constexpr bool kPipeH = kPipe || (ZF_X3_PAIRS_PIPE && (T == 4 || ZF_X3_WIDE_PIPE) && NT == 2 && !OACT);
      // OACT with a narrowed activation set: the layer input's tiles 1..T-1
      // activated inside the group steps (x3_step_pipe AS), like the swish
#ifndef ZF_X3_ACTIN
#define ZF_X3_ACTIN 1
#endif
      // (the centred set only: the five-way plain set spills 40 VGPRs that way, -13% on relu)
      constexpr bool kActIn = ZF_X3_ACTIN && NT == 2 && ASET == 2 && kPipeH;
      constexpr bool kSeedScaledH = NT == 2 && (ZF_X3_SEEDSCALED || !kPipeH);
      // Three waves share a SIMD at hidden 128: the one streaming weight
      // groups (MFMAs) wins issue arbitration over one in its VALU-only
      // phases (layer 0, spline), so the matrix pipe idles less (+1.5% cfg2,
      // +1.2% d8; nothing to arbitrate at hidden 256, one wave per SIMD).
#if ZF_X3_ABL != 4  // tuning ablation 4: no issue priority
      if constexpr (T == 4) __builtin_amdgcn_s_setprio(2);
#endif
      X3T(1);
      if constexpr (kEarly) {
        float eM = eU;  // max |v'| of the current layer input's pre-activations (exact from layer 2 on)
        for (int l = 1; l < nh; ++l) {
          // the next layer's input bound and scales (its tile 0 is swished in this layer's last
          // step), from the exact maximum of this layer's input, so bounds never compound
          const float nU = __builtin_fmaf(op.x3_rb[l][0], eM, op.x3_rb[l][1]);
          float nisc, nus, nius;
          x3_scale_from(nU, l + 1 < nh ? op.x3_kw[l + 1] : kw_last, nisc, nus, nius);
          floatx16 acc[T];
#pragma unroll
          for (int o = 0; o < T; ++o) acc[o] = floatx16{0};
          float mx;
          x3_layer_early<T, T, true>(x3, pipe, hb, acc, lane, par + b_rel + (l - 1) * (T * 32), hh, ecs, eisc, eus,
                                     nisc, mx);
#pragma unroll
          for (int o = 0; o < T; ++o) hb[o] = acc[o];
          eU = nU; eisc = nisc; eus = nus; eius = nius;
          const X3Halves mq = x3_halves(mx);
          eM = fmaxf(mq.lo, mq.hi);
        }
      } else
      for (int l = 1; l < nh; ++l) {
        floatx16 acc[T];
        float isc = 1.f, us = 1.f, ius = 1.f;
        if constexpr (NT == 2) {
          x3_act_scale<T, OACT>(hb, l == 1 ? opc.kw1 : op.x3_kw[l], isc, us, ius, act);
          // OACT: every tile here, outside the MFMA stream (the switch there
          // would cost a third of the waves)
#pragma unroll
          for (int o = 0; o < (OACT && !kActIn ? T : 1); ++o) x3_act_tile<NT, OACT, ASET>(hb[o], isc, act);
        }
        const float* bl_l = par + b_rel + (l - 1) * (T * 32);
#pragma unroll
        for (int o = 0; o < T; ++o)
          acc[o] = NT == 3 ? bias_acc(bl_l + o * 32, hh)
                           : (kSeedScaledH ? bias_acc(bl_l + o * 32, hh) * ius : floatx16{0});
        const float* bh = (NT == 2 && !kSeedScaledH) ? bl_l : nullptr;
        if constexpr (kPipeH) {
          typename XT<NT>::E cs[NT];
          splitk<NT, 0>(hb[0], cs);
          halfx8 fs1[2];  // ZF_X3_FUSED: the k-step 1 terms carried between group steps
          x3_layer_pipe<NT, T, T, NT == 2 && !kSeedScaledH, OACT, 0, kActIn ? ASET : 0>(x3, pipe, hb, acc, lane, bh, hh,
                                                                                     cs, isc, us,
                                                                 act, fs1);
        } else {
          x3_layer<NT, T, T, true, OACT>(x3, pipe, hb, acc, lane, bh, hh, isc, us, act);
        }
        if constexpr (kSeedScaledH) {
#pragma unroll
          for (int o = 0; o < T; ++o) acc[o] *= us;
        }
        const int nsw = NT == 2 ? 0 : (!OACT && (l + 1 < nh || kLastSW)) ? 1 : T;
#pragma unroll
        for (int o = 0; o < T; ++o) {
          if (o < nsw) {
            if constexpr (OACT) {
              hb[o] = acc[o];
              x3_act_tile<3, true>(hb[o], 1.f, act);
            } else {
#pragma unroll
              for (int r = 0; r < 16; ++r) hb[o][r] = swish(acc[o][r]);
            }
          } else {
            hb[o] = acc[o];
          }
        }
      }
      X3T(2);
      // Last Dense (:346-347), one pair of transformed dims at a time: lane
      // half h, tile o, register r = parameter 16*o + r of dim 2*pair + h.
      float ldn = 0.f;  // this coupling's log-det, summed in dim order (utils.py:139)
      // PAIRS == false: one pair (dt <= 2), and the hidden activations are
      // dead once the last layer has consumed them.
      const int npair = PAIRS ? (dt + 1) / 2 : 1;
      float lisc = 1.f, lus = 1.f, lius = 1.f;  // f16x2 scales of the last layer's input (all pairs)
      if constexpr (kEarly) {
        lisc = eisc; lus = eus; lius = eius;  // tile 0 swished, ecs its split
      } else if constexpr (NT == 2) {
        x3_act_scale<T, OACT>(hb, kw_last, lisc, lus, lius, act);
        // PAIRS: the input is read once per dim pair, so swish it whole here
#pragma unroll
        for (int o = 0; o < T; ++o)
          if (o == 0 || !kLastSW || (OACT && !(kActIn && kPipe))) x3_act_tile<NT, OACT, ASET>(hb[o], lisc, act);
      }
#ifndef ZF_X3_PRESPLIT
#define ZF_X3_PRESPLIT 1
#endif
      // PAIRS at hidden 128 (f16x2): the last layer's input split once for
      // all pairs (d8 -1.0%; at hidden 256, one wave per SIMD, the per-pair
      // re-split hides in the MFMA gaps and the pre-split cost 5.6%)
      constexpr bool kPre = ZF_X3_PRESPLIT && PAIRS && T == 4 && NT == 2 && !OACT;
      halfx8 sp[kPre ? T : 1][2][2];
      if constexpr (kPre) {
#pragma unroll
        for (int q = 0; q < T; ++q) {
          split8h<0>(hb[q], sp[q][0][0], sp[q][0][1]);
          split8h<1>(hb[q], sp[q][1][0], sp[q][1][1]);
        }
      }
      for (int pr = 0; pr < npair; ++pr) {
        // The bias seeds the accumulators when the hidden activations stay
        // live across pairs anyway; otherwise it joins in the last step, when
        // the first input tiles are dead (fewer registers at the peak);
        // f16x2 always joins it at the end, with the unscale.
        const float* bl = par + blast_rel + pr * TL * 32;
        floatx16 pa[TL];
        constexpr bool kSeed = PAIRS && NT == 3;
#pragma unroll
        for (int o = 0; o < TL; ++o)
          pa[o] = kSeed ? bias_acc(bl + o * 32, hh) : (kSeedScaled ? bias_acc(bl + o * 32, hh) * lius : floatx16{0});
        X3T(3);
        if constexpr (kEarly) {
          float mx;
          x3_layer_early<T, TL, false, kPreSP>(x3, pipe, hb, pa, lane, bl, hh, ecs, lisc, lus, 0.f, mx);
        } else if constexpr (kPre) {
          x3_layer_pre<T, TL>(x3, pipe, sp, pa, lane);
        } else if constexpr (kPipe) {
          typename XT<NT>::E cs[NT];
          splitk<NT, 0>(hb[0], cs);
          halfx8 fs1[2];
          x3_layer_pipe<NT, T, TL, !kSeedScaled, OACT, 0, kActIn ? ASET : 0>(x3, pipe, hb, pa, lane, bl, hh, cs, lisc,
                                                                             lus, act, fs1);
        } else {
          x3_layer<NT, T, TL, kLastSW, OACT>(x3, pipe, hb, pa, lane, (kSeed || kSeedScaled) ? nullptr : bl, hh,
                                             lisc, lus, act);
        }
        if constexpr (kSeedScaled) {
#pragma unroll
          for (int o = 0; o < TL; ++o) pa[o] *= lus;
        }
        if constexpr (T == 4) __builtin_amdgcn_s_setprio(0);
        X3T(4);
        // ONE at K = 16: tile 0 holds the widths on lane half 0 and the
        // heights on half 1, so each half normalises its own 16 (squareplus,
        // sum in order, quotients: the same operations per value) and one
        // exchange per knot gives both halves both; tile 1's slopes (half 0)
        // go to both halves.  Other ONE shapes exchange the whole row first.
        constexpr bool kSplitWH = ONE && K == 16;
        float P[NPV];
#pragma unroll
        for (int o = 0; o < TL; ++o)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            if constexpr (kSplitWH) {
              if (o == 0) P[r] = pa[0][r];
              else  // slope r of half 0, on both halves
                P[2 * K + r] = x3_halves(pa[1][r]).lo;
            } else if constexpr (ONE) {  // both halves end up with all of the dim's parameters
              const X3Halves q = x3_halves(pa[o][r]);
              P[32 * o + r] = q.lo;
              P[32 * o + 16 + r] = q.hi;
            } else {
              P[16 * o + r] = pa[o][r];
            }
          }
        X3M(11);
#if ZF_X3_ABL == 10 || ZF_X3_ABL == 11  // tuning: 64 extra VALU (10: v_add, 11: v_exp) in the spline phase
#pragma unroll
        for (int q2 = 0; q2 < 64; ++q2) {
          float dd;
          if (ZF_X3_ABL == 10) asm volatile("v_add_f32 %0, %1, %2" : "=v"(dd) : "v"(pa[0][q2 & 15]), "v"(pa[1][q2 & 15]));
          else asm volatile("v_exp_f32 %0, %1" : "=v"(dd) : "v"(pa[0][q2 & 15]));
        }
#endif
        // normalize_spline_params (utils.py:37-62) + RQ spline (utils.py:65-250)
        const int d = 2 * pr + hh;
        const bool dact = d < dt;  // the upper half idles on an odd last dim
        float ldv = 0.f;
        {
          float* xp = xs + wrap((dact ? d : 0) + rot, D) * 32 + s;
          const float xv = *xp;
#ifndef ZF_X3_BSEARCH
#define ZF_X3_BSEARCH 0
#endif
          RqsBin bin;
          bool binned = false;
          if constexpr (ZF_X3_BSEARCH && !kSplitWH && !kPreSP && (K == 8 || K == 16 || K == 32 || K == 64)) {
            if (klit) {  // the halving search takes unpadded knots only, not yet squareplus'd ones
              bin = x3_bin<!INV, K, OACT, true>(xv, P, kc);
              binned = true;
            }
          }
          if (!binned) {
            float w[K], hg[K];
            const float bc = kc.c * kc.rnorm;
            if constexpr (kSplitWH) {
              float sw = 0.f;  // half 0: the widths' sum, half 1: the heights'
#pragma unroll
              for (int j = 0; j < K; ++j) {
                w[j] = kPreSP ? P[j] : x3_squareplus2_t<OACT>(P[j]);
                sw = sw + w[j];
              }
              const float a = rcp_refined(sw) * kc.rnorm;
#pragma unroll
              for (int j = 0; j < K; ++j) {
                const X3Halves q = x3_halves(__builtin_fmaf(w[j], a, bc));
                w[j] = q.lo;
                hg[j] = q.hi;
              }
            } else {
              float sx = 0.f, sy = 0.f;
#pragma unroll
              for (int j = 0; j < K; ++j) {  // squareplus + sums in order (utils.py:30-33)
                w[j] = kPreSP ? P[j] : x3_squareplus2_t<OACT>(P[j]);
                hg[j] = kPreSP ? P[K + j] : x3_squareplus2_t<OACT>(P[K + j]);
                sx = sx + w[j];
                sy = sy + hg[j];
              }
              // (v / sum + c) / (1 + c K) as one fma per knot (v and sum both
              // 2*squareplus: the same quotient bits): the parameters
              // themselves already differ from the reference's in the last ulp
              // (GEMM summation order), so correctly rounded divisions buy nothing.
              const float ax = rcp_refined(sx) * kc.rnorm, ay = rcp_refined(sy) * kc.rnorm;
#pragma unroll
              for (int j = 0; j < K; ++j) {
                w[j] = __builtin_fmaf(w[j], ax, bc);
                hg[j] = __builtin_fmaf(hg[j], ay, bc);
              }
            }
            X3M(12);
            float sl[K - 1];  // raw slope logits; the bin's two get squareplus'd
#pragma unroll
            for (int j = 0; j < K - 1; ++j) sl[j] = P[2 * K + j];
#ifndef ZF_X3_EXECBIN
#define ZF_X3_EXECBIN 1
#endif
            // the latch as exec-masked moves (rqs_bin_exec): -15% of the spline phase's VALU issue
            const auto spf = [](float v) { return v == 0.f ? 1.f : x3_squareplus_t<OACT>(v); };
            if constexpr (ZF_X3_EXECBIN && K % 8 == 0) bin = rqs_bin_exec<!INV, K>(xv, w, hg, sl, spf, padlast);
            else bin = rqs_bin_monotone<!INV, K>(xv, w, hg, sl, spf, padlast);
            X3M(13);
          }
          float yv;
          if (!INV) {
            float l;
            x3_forward_eval(xv, bin, yv, l);
            ldv = dact ? l : 0.f;
          } else {
            yv = rqs_inverse_eval(xv, bin);
          }
          if (dact) *xp = yv;
        }
        wave_lds_sync();
        if (!INV) {
          const X3Halves q = x3_halves(ldv);
          ldn = ldn + q.lo;
          if (2 * pr + 1 < dt) ldn = ldn + q.hi;
        }
      }
      if (!INV) ld = ld + ldn;  // Chain: log_det += ld (bijectors.py:110)
      X3T(5);
    }
  }

  flow_epilogue<NW>(F, xs, s, hh, lane, wave, rot, D, row, valid, ld, lp_out, block_partial, NW / 4, nparts, y_out,
                    ld_out, s_part);
#ifdef ZF_X3_TRACE
  X3T(6);
  tacc[7] = pipe.tbar;
  tacc[11] = pipe.tdma;
  tacc[12] = pipe.tgrp;
  tacc[8] = t_last - t_begin;
  if (lane == 0 && x3_trace_buf != nullptr) {
    unsigned long long* o = x3_trace_buf + ((long long)blockIdx.x * NW + wave) * kX3TraceSlots;
#pragma unroll
    for (int k = 0; k < kX3TraceSlots; ++k) o[k] = tacc[k];
  }
#endif
#undef X3T
#undef X3M
}

template <int NT, int K, int T, bool PAIRS, bool ONE, bool OACT, int ASET = 0>
int launch_x3(const X3Launch& a, bool inverse) {
  const long long rows = kX3Waves * kTile;
  const long long grid = (a.N + rows - 1) / rows;
  if (grid > 0x7fffffffLL) return einval("N too large");
  constexpr int TL = ONE ? (3 * K - 1 + 31) / 32 : (3 * K - 1 + 15) / 16;
  size_t lds = (size_t)2 * group_bytes<NT>(T > TL ? T : TL) + (size_t)2 * a.par_bytes +
               (size_t)kX3Waves * 32 * (a.D + a.C) * 4 + kX3Waves * sizeof(double);
#ifdef ZF_X3_TRACE
  if (const char* pad = std::getenv("ZF_X3_LDS_PAD")) lds += (size_t)std::atoi(pad) * 1024;  // occupancy probe
#endif
  if (lds > 160 * 1024) return enotsup("bf16x3 LDS footprint too large");
  if (inverse)
    hipLaunchKernelGGL((flow_kernel_x3<NT, K, T, PAIRS, ONE, true, OACT, ASET>), dim3((unsigned)grid), dim3(kX3Waves * 64), lds, a.stream,
                       a.desc, a.blob, (const char*)a.x3, a.x, a.c, a.y, a.ld_in, a.ld_out, a.lp, a.part,
                       a.nparts, a.op_begin, a.op_end, a.N, a.seed, a.gen);
  else
    hipLaunchKernelGGL((flow_kernel_x3<NT, K, T, PAIRS, ONE, false, OACT, ASET>), dim3((unsigned)grid), dim3(kX3Waves * 64), lds, a.stream,
                       a.desc, a.blob, (const char*)a.x3, a.x, a.c, a.y, a.ld_in, a.ld_out, a.lp, a.part,
                       a.nparts, a.op_begin, a.op_end, a.N, a.seed, a.gen);
  ZF_CHECK_LAUNCH("flow_kernel_x3");
  return ZF_OK;
}

// Instantiated shapes (x3_eligible): K in {8, 16, 32} at hidden 128 (T = 4)
// and hidden 256 (T = 8).  PAIRS (a loop over transformed-dim pairs in the
// last layer) whenever dt > 2, and always at T = 8 (its hidden activations
// are live across the last layer anyway); ONE when dt == 1.
// OACT: some coupling's activation is not swish (f16x2 only).
template <int NT, int K, bool OACT = false, int ASET = 0>
int launch_x3_k(const X3Launch& a, bool inverse) {
  const int dt = a.D / 2;
  const bool one = dt == 1;  // must match x3_pack's last-layer layout
  if (a.T == 4) {
    if (dt > 2) return launch_x3<NT, K, 4, true, false, OACT, ASET>(a, inverse);
    return one ? launch_x3<NT, K, 4, false, true, OACT, ASET>(a, inverse)
               : launch_x3<NT, K, 4, false, false, OACT, ASET>(a, inverse);
  }
  if (a.T == 8)
    return one ? launch_x3<NT, K, 8, true, true, OACT, ASET>(a, inverse)
               : launch_x3<NT, K, 8, true, false, OACT, ASET>(a, inverse);
  return enotsup("split-MFMA kernel: hidden tiles not instantiated");
}

}  // namespace
}  // namespace zf
