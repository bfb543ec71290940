// Device-side pieces shared by the two fused flow kernels (zf_flow.hip: fp32
// MFMA, any width; zf_flow_x3.hip: bf16x3 MFMA with LDS-shared weights): the
// device flow descriptor, the scalar numerics the reference fixes, and the
// op steps that do not touch the conditioner GEMMs (ShiftBounds, the
// BatchNorm + first Dense layer, the latent log_prob epilogue).
#pragma once
#include "zf_act.h"
#include "zf_internal.h"
#include "zf_random.h"
#include "zf_spline.h"

#include <cstdint>
#include <vector>

namespace zf {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kTile = 32;  // samples per wave (one MFMA column block)
constexpr int kMaxOps = 64;

struct DevOp {
  int kind, shift, K, S;
  int n_hidden, dt, dc, DC;
  int KS0, T_last, nslot_mask, act;
  long long w[17];
  long long b[17];
  long long bn;
  long long sb;
  long long first_chunk;  // blob offset of this NSC's first streamed weight chunk (fp32 kernel)
  // bf16x3 kernel: byte offset of this NSC's weight-group stream in the x3
  // blob, its group count, blob offset of the row-permuted last-layer bias,
  // and the next NSC op index in forward / inverse execution order (or -1).
  long long x3;
  long long x3_blast;
  int x3_groups, x3_tlast;
  int x3_next[2];
  int x3_kw[17];  // f16x2: power-of-two weight scale of streamed layer l (1..n_hidden)
  // f16x2 swish: per Dense_l (0..n_hidden-1, as packed: log2(e) prescale
  // included) R = max_j sum_k |W[k][j]| and B = max_j |b[j]|, so every
  // pre-activation |v_j| <= R * max_k |a_k| + B (x3_early_scale)
  float x3_rb[16][2];
  // split-MFMA kernel: this NSC's small parameters (BatchNorm, Dense_0,
  // biases, the permuted last bias) are the contiguous blob floats
  // [bn, bn + 256 * x3_par_pieces), DMA'd into LDS one NSC ahead
  int x3_par_pieces;
  // the next NSC in forward / inverse execution order (x3_next[d] >= 0):
  // its group-0 byte offset and pieces, its parameter block and pieces —
  // copied here so the kernel's per-NSC scalars are one batch of independent loads
  long long x3_nbase[2], x3_nbn[2];
  int x3_npieces[2], x3_npar[2];
};

struct DevFlow {
  int D, C, latent, n_ops;
  int HP, nslot, per_wave, x3_ok;
  int small_floats;  // packed blob [0, small_floats): per-op small parameters
  int x3_par_bytes;  // split-MFMA kernel: LDS bytes of one NSC's small-parameter region (max over NSCs)
  int kreal;  // split-MFMA kernels: the couplings' knot count (the kernel's K may be padded above it)
  int _pad;
  float lat_c0, lat_c1, lat_c2, lat_c3;
  DevOp ops[kMaxOps];
};

__device__ __forceinline__ void wave_lds_sync() {
  // LDS ops of one wave execute in order; this only stops the compiler from
  // moving LDS accesses across the exchange point.
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// flax.linen.swish = x * sigmoid(x) = x / (1 + exp(-x)) (bijectors.py:319):
// v * rcp(1 + 2^(-v*log2e)) (~|v|*6e-8 relative error; a compensated exp
// argument with a Newton reciprocal, and expf with IEEE division, gave the
// same mean log_prob error against the fp32 oracle, scripts/diag_parity.py).
__device__ __forceinline__ float swish(float v) {
  return v * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-v * 1.44269504f));
}

// 1/x to ~0.5 ulp: hardware reciprocal + one Newton step.
__device__ __forceinline__ float rcp_refined(float x) {
  float r = __builtin_amdgcn_rcpf(x);
  return __builtin_fmaf(__builtin_fmaf(-x, r, 1.0f), r, r);
}

// x / d given r = rcp_refined(d): one residual correction of the product
// makes the quotient correctly rounded for these (normal, non-overflowing)
// operands — the IEEE division the reference performs, at a third of the cost.
__device__ __forceinline__ float div_cr(float x, float d, float r) {
  const float q = x * r;
  return __builtin_fmaf(__builtin_fmaf(-q, d, x), r, q);
}

// squareplus (utils.py:18-20) with a residual-corrected hardware square root
// (x^2 + 4 >= 4: never denormal); matches the correctly rounded sqrtf.
__device__ __forceinline__ float squareplus_fast(float x) {
  const float a = x * x + 4.0f;
  float sq = __builtin_amdgcn_sqrtf(a);
  sq = __builtin_fmaf(__builtin_fmaf(-sq, sq, a), 0.5f * __builtin_amdgcn_rcpf(sq), sq);
  return 0.5f * (x + sq);
}

// Bias of one 32-row output tile for this lane's 16 accumulator rows (packed
// [2 lane halves][16]).  Callers issue it BEFORE a tile's weight stream:
// vmcnt retires in order, so a bias load issued after the prefetch of the
// next weight chunk would make its consumer drain that prefetch too.
__device__ __forceinline__ void bias_tile(const float* __restrict__ bt, int hh, floatx4 (&b)[4]) {
  const floatx4* p = reinterpret_cast<const floatx4*>(bt + hh * 16);
#pragma unroll
  for (int r4 = 0; r4 < 4; ++r4) b[r4] = p[r4];
}

// The same bias tile as an accumulator initialiser: a layer's MFMAs then
// accumulate onto its bias (no separate add, no zero fill).
__device__ __forceinline__ floatx16 bias_acc(const float* __restrict__ bt, int hh) {
#if defined(ZF_X3_ABL) && ZF_X3_ABL == 7  // tuning ablation 7: no small-parameter loads (wrong results)
  floatx16 z;
#pragma unroll
  for (int r = 0; r < 16; ++r) z[r] = 0.01f * (r + hh);
  return z;
#endif
  floatx4 b[4];
  bias_tile(bt, hh, b);
  floatx16 a;
#pragma unroll
  for (int r = 0; r < 16; ++r) a[r] = b[r >> 2][r & 3];
  return a;
}

__device__ __forceinline__ int pmod(int a, int m) {
  int r = a % m;
  return r < 0 ? r + m : r;
}

// a mod m for a in [0, 2m): stored-column index of logical dim j under a
// rotation rot in [0, m) (no integer division on the per-sample path).
__device__ __forceinline__ int wrap(int a, int m) { return a >= m ? a - m : a; }

// softmax_with_threshold constants (utils.py:32-34): c and 1 + c*n are Python
// floats (fp64), rounded to fp32 where they meet fp32 arrays.
struct KnotConsts {
  float c, norm, rnorm;
  __device__ __forceinline__ explicit KnotConsts(int K) {
    const double c64 = 1e-5 / (1.0 - (double)K * 1e-5);
    c = (float)c64;
    norm = (float)(1.0 + c64 * (double)K);
    rnorm = rcp_refined(norm);
  }
};

// Per-wave state: xs[D][32] (column p = stored dim, lane = sample), from x
// or — Flow.sample (flow.py:70-78) — drawn from the latent on the fly.
__device__ __forceinline__ void load_state(float* xs, const float* __restrict__ xin, long long row,
                                           bool valid, int D, int s, int hh, const DevFlow* __restrict__ F,
                                           unsigned long long seed, int gen) {
  for (int d = hh; d < D; d += 2) {
    float v = 0.f;
    if (valid) v = gen ? latent_draw(F->latent, F->lat_c3, seed, row, d) : xin[row * D + d];
    xs[d * 32 + s] = v;
  }
}

// ShiftBounds of one value of logical dim i (bijectors.py:181-208 forward,
// eval branch of :261-273; :210-240 inverse).  r = the packed row sb + 8 i:
// [mode, a, b, xmin, xmax, mul, log mul, 0].
__device__ __forceinline__ float sb_forward_elem(const float* __restrict__ r, float v, float& l) {
  const int mode = (int)r[0];
  const float a = r[1], b = r[2], xmin = r[3];
  const float mul = r[5], logmul = r[6];
  if (mode == ZF_SB_BOTH) {  // :187-192
    l = logmul;
    return (v - a) * mul;
  }
  float t = v;
  if (mode == ZF_SB_LOWER) t = logf((v - a) + 1.17549435e-38f);  // safe_log :430
  if (mode == ZF_SB_UPPER) t = logf((b - v) + 1.17549435e-38f);
  const float zr = (t - xmin) * mul;
  l = (mode == ZF_SB_NONE) ? logmul : logmul - t;    // :197, :202
  return (zr != zr) ? zr : fminf(fmaxf(zr, 0.f), 1.f);  // :272 clip
}

__device__ __forceinline__ float sb_inverse_elem(const float* __restrict__ r, float zv) {
  const int mode = (int)r[0];
  const float a = r[1], b = r[2];
  const float xmin = r[3], xmax = r[4];
  if (mode == ZF_SB_BOTH) return zv * b + (1.f - zv) * a;
  const float t = zv * xmax + (1.f - zv) * xmin;
  return (mode == ZF_SB_LOWER) ? expf(t) + a : (mode == ZF_SB_UPPER ? b - expf(t) : t);
}

// ShiftBounds on the per-wave state.  `sb` is the packed [D][8] row block.
template <bool INV>
__device__ __forceinline__ void shift_bounds_op(const float* __restrict__ sb, float* xs, int s, int hh,
                                                int rot, int D, float& ld) {
  if (!INV) {
    float ldsb = 0.f;
    for (int i = 0; i < D; ++i) {
      const int p = wrap(i + rot, D);
      float l;
      const float z = sb_forward_elem(sb + 8 * i, xs[p * 32 + s], l);
      ldsb = ldsb + l;
      if (hh == 0) xs[p * 32 + s] = z;
    }
    ld = ld + ldsb;
  } else {
    for (int i = 0; i < D; ++i) {
      const int p = wrap(i + rot, D);
      const float xv = sb_inverse_elem(sb + 8 * i, xs[p * 32 + s]);
      if (hh == 0) xs[p * 32 + s] = xv;
    }
  }
  wave_lds_sync();
}

// Conditioner input + first Dense (bijectors.py:341-343): u = BatchNorm(
// hstack(xc, c)), hb = swish(W0^T u + b0) on fp32 MFMA, one k-step per 2
// inputs.  hb: T accumulator tiles (unit rows in registers, sample on lane).
template <int T>
__device__ __forceinline__ void layer0(const DevOp& op, const float* __restrict__ blob, const float* xs,
                                       const float* __restrict__ cin, long long row, bool valid, int C,
                                       int rot, int D, int s, int hh, int lane, floatx16 (&hb)[T],
                                       int swish_tiles = T, int act = ZF_ACT_SWISH) {
  const int dt = op.dt, dc = op.dc, DC = op.DC, KS0 = op.KS0;
  const int DCp = 2 * KS0;
  const float* bn = blob + op.bn;
#pragma unroll
  for (int o = 0; o < T; ++o) hb[o] = bias_acc(blob + op.b[0] + o * 32, hh);
  for (int ks = 0; ks < KS0; ++ks) {
    const int k = 2 * ks + hh;
    float v = 0.f;
    if (k < dc) v = xs[wrap(dt + k + rot, D) * 32 + s];
    else if (k < DC) v = valid ? cin[row * C + (k - dc)] : 0.f;
#if defined(ZF_X3_ABL) && ZF_X3_ABL == 7
    const float u = (v - 0.1f) * 1.1f + 0.01f;
#pragma unroll
    for (int o = 0; o < T; ++o)
      hb[o] = __builtin_amdgcn_mfma_f32_32x32x2f32(0.01f * (o + lane), u, hb[o], 0, 0, 0);
#else
    const float u = (v - bn[k]) * bn[DCp + k] + bn[2 * DCp + k];
    const float* w0 = blob + op.w[0] + ks * 64 + lane;
#pragma unroll
    for (int o = 0; o < T; ++o)
      hb[o] = __builtin_amdgcn_mfma_f32_32x32x2f32(w0[o * KS0 * 64], u, hb[o], 0, 0, 0);
#endif
  }
  // swish of tiles [0, swish_tiles): the bf16x3 kernel defers the others into
  // the next layer's MFMA stream
  if (act != ZF_ACT_SWISH) {  // the fp32 kernel's other activations (act is wave-uniform)
#pragma unroll
    for (int o = 0; o < T; ++o)
#pragma unroll
      for (int r = 0; r < 16; ++r) hb[o][r] = act_other(act, hb[o][r]);
    return;
  }
#pragma unroll
  for (int o = 0; o < T; ++o)
    if (o < swish_tiles)
#pragma unroll
      for (int r = 0; r < 16; ++r) hb[o][r] = swish(hb[o][r]);
}

// One coordinate's latent log-density (distributions.py:16-126, the
// jax.scipy.stats forms) with the DevFlow latent constants.
__device__ __forceinline__ float latent_logpdf(int lt, float c0, float c1, float c2, float v) {
  float t;
  if (lt == ZF_LATENT_NORMAL || lt == ZF_LATENT_TRUNCNORM) {
    // jax.scipy.stats.norm.logpdf: (log(2 pi s^2) + (x-loc)^2/s^2) / -2
    const float dv = v - 0.5f;
    t = (c0 + (dv * dv) / c1) / -2.0f;
    if (lt == ZF_LATENT_TRUNCNORM) {  // - log mass; -inf outside [-5, 5] sigma
      t = t - c2;
      const float xsd = dv / 0.1f;
      if (xsd < -5.f || xsd > 5.f) t = -INFINITY;
    }
  } else if (lt == ZF_LATENT_BETA) {
    // -betaln(a,a) + xlogy(a-1, x) + xlog1py(a-1, -x); -inf outside [0, 1]
    const float l1 = (c1 == 0.f) ? 0.f : c1 * logf(v);
    const float l2 = (c1 == 0.f) ? 0.f : c1 * log1pf(-v);
    t = c0 + (l1 + l2);
    if (v > 1.f || v < 0.f) t = -INFINITY;
  } else {  // uniform
    t = (v > 1.f || v < 0.f) ? -INFINITY : 0.f;
  }
  return t;
}

// jnp.nan_to_num(lp, nan=-inf) (flow.py:47): JAX's sequential where chain,
// each mask taken from the running result — NaN -> -inf -> finfo.min,
// +inf -> finfo.max, -inf -> finfo.min.
__device__ __forceinline__ float nan_to_num_lp(float lp) {
  if (lp != lp) lp = -INFINITY;
  if (lp == INFINITY) lp = 3.40282347e38f;
  if (lp == -INFINITY) lp = -3.40282347e38f;
  return lp;
}

// latent.log_prob(z) + log_det, nan_to_num (flow.py:41-48;
// distributions.py:16-33), block partial of sum(log_prob) for the NLL, and
// the optional y / log_det outputs.  Partials: block b writes part[b*pstride]
// (and zero into the pstride-1 slots after it that are < nparts), or
// part[slot] when given, so every kernel shape leaves the same
// ceil(N/128)-entry workspace for reduce.
template <int NW>
__device__ __forceinline__ void flow_epilogue(const DevFlow* __restrict__ F, const float* xs, int s,
                                              int hh, int lane, int wave, int rot, int D, long long row,
                                              bool valid, float ld, float* __restrict__ lp_out,
                                              double* __restrict__ block_partial, int pstride,
                                              long long nparts, float* __restrict__ y_out,
                                              float* __restrict__ ld_out, double* s_part,
                                              long long slot = -1) {
  if (lp_out != nullptr) {
    float lat = 0.f;
    for (int j = 0; j < D; ++j)
      lat = lat + latent_logpdf(F->latent, F->lat_c0, F->lat_c1, F->lat_c2, xs[wrap(j + rot, D) * 32 + s]);
    const float lp = nan_to_num_lp(lat + ld);
    if (valid && hh == 0) lp_out[row] = lp;
    if (block_partial != nullptr) {
      double v = (valid && hh == 0) ? (double)lp : 0.0;
#pragma unroll
      for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
      if (lane == 0) s_part[wave] = v;
      __syncthreads();
      if (threadIdx.x == 0) {
        double acc = 0.0;
        for (int w = 0; w < NW; ++w) acc += s_part[w];
        // slot: the partial index of these rows when a block covers several
        // 128-row slots (the two-set kernel calls this once per set)
        const long long b0 = slot >= 0 ? slot : (long long)blockIdx.x * pstride;
        block_partial[b0] = acc;
        for (int k = 1; k < pstride; ++k)
          if (b0 + k < nparts) block_partial[b0 + k] = 0.0;
      }
    }
  }
  if (y_out != nullptr && valid) {
    for (int j = hh; j < D; j += 2) y_out[row * D + j] = xs[wrap(j + rot, D) * 32 + s];
  }
  if (ld_out != nullptr && valid && hh == 0) ld_out[row] = ld;
}

// Host-side entry of the bf16x3 kernel (zf_flow_x3.hip).
struct X3Launch {
  const DevFlow* desc;
  const float* blob;
  const void* x3;
  const float *x, *c;
  float* y;
  const float* ld_in;
  float *ld_out, *lp;
  double* part;
  long long nparts;
  int op_begin, op_end;
  long long N;
  unsigned long long seed;
  int gen;  // 1: draw the input rows from the latent (zf_flow_sample)
  int K, D, C, T;  // knots, dim, conditions, hidden tiles (4: width <= 128, 8: <= 256)
  int NT;       // split scheme: 3 = bf16x3, 2 = f16x2
  bool oact;    // some coupling's activation is not swish (f16x2 kernels with act switch)
  int aset;     // oact, f16x2: 2 = only sigmoid/softplus (the _act2 units), 1 = only relu/tanh/gelu/elu/leaky_relu, 0 = both kinds (1 and 0: the full switch)
  int par_bytes;  // DevFlow::x3_par_bytes
  hipStream_t stream;
};
int launch_flow_x3(const X3Launch& a, bool inverse);
bool x3_eligible(const zf_flow_desc& desc, int HP, int* K);
// Layered eval path (zf_layered.hip) for shapes the fused kernels cannot hold
// (a hidden width above 256): op by op over row chunks — BatchNorm, the Dense
// layers on the trainer's GEMMs, the per-(row, dim) spline kernels.
struct LayeredFlow;
int layered_create(const zf_flow_desc& desc, const float* natural, int64_t n, LayeredFlow** out);
void layered_destroy(LayeredFlow* L);
int layered_run(LayeredFlow* L, const DevFlow& F, const float* packed, bool inverse, int op_begin, int op_end,
                const float* x, const float* c, float* y, const float* ld_in, float* ld_out, float* lp, double* part,
                long long N, hipStream_t st, unsigned long long seed, int gen);
int x3_last_tiles(int K);
int x3_pairs(const zf_flow_desc& desc);
int x3_buf_tiles(const zf_flow_desc& desc, int T, int K);
size_t x3_lds_bytes(int TB, int D, int NT, int par_bytes);
int x3_scheme();
int x3_scheme_for(const zf_flow_desc& desc);
void x3_pack(const zf_flow_desc& desc, const float* nat, int T, int NT, int Kp, DevFlow& F, float* packed,
             std::vector<uint16_t>& stream);

}  // namespace zf
