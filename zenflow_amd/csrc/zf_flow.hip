// Fused flow kernel: one launch runs a whole zenflow bijector chain
// (ShiftBounds -> [NeuralSplineCoupling, Roll]* -> NeuralSplineCoupling) and
// the latent log_prob epilogue for a tile of samples, keeping every
// intermediate on chip.  Reference call stack:
//   Flow.__call__ (flow.py:22-48) -> Chain.__call__ (bijectors.py:103-111)
//   -> ShiftBounds (:163-273) / Roll (:288-297) / NeuralSplineCoupling (:359-371)
//   -> conditioner MLP (:329-357) + normalize_spline_params + RQ spline (utils.py).
//
// Execution model (DESIGN.md §Fused kernel):
//   * one wave64 owns a tile of 32 samples; a 256-thread block = 4 independent
//     waves = 128 samples (no inter-wave sync in the op loop);
//   * conditioner GEMMs on fp32 MFMA v_mfma_f32_32x32x2_f32 (exact f32 fma
//     chain): weights are the A operand (out-unit x in-unit), activations the B
//     operand (in-unit x sample).  A layer's accumulator tile (unit rows in
//     registers, sample on the lane) is directly the B operand of the next
//     layer -> hidden activations never leave registers;
//   * weights are pre-packed in MFMA fragment order and streamed from L2 with
//     one dwordx4 per lane per 4 MFMAs (every wave reads the same bytes);
//   * the last layer's 32-row output tiles go through a per-wave LDS ring
//     (lane = sample, conflict-free), where one lane per (sample, dim) runs
//     normalize_spline_params + bin search + RQ spline + log-det in registers;
//   * per-sample state (D floats) lives in LDS; Roll is an index rotation.
#include "zf_flow_dev.h"

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace zf {
namespace {

constexpr int kWaves = 4;  // waves per block
constexpr int kBlockRows = kWaves * kTile;

// One 32-row output tile of a Dense layer on MFMA: acc = W^T[tile] . H over
// the T input tiles (activations hb: unit rows in registers, sample on the
// lane).  The weight fragments of one input tile (4 dwordx4 per lane, 16
// MFMAs) are streamed with exactly one chunk in flight: `cur` holds this
// tile's first chunk on entry and the next tile's (pnext, may be null) on exit.
template <int T>
__device__ __forceinline__ floatx16 mfma_tile(const floatx4* __restrict__ p,
                                              const floatx4* __restrict__ pnext, floatx4 (&cur)[4],
                                              const floatx16 (&hb)[T]) {
  floatx16 acc = floatx16{0};
#pragma unroll
  for (int t = 0; t < T; ++t) {
    floatx4 nxt[4];
    const bool more = (t + 1 < T);
    const floatx4* src = more ? p + (t + 1) * 256 : pnext;
    const bool have = more || (pnext != nullptr);
    if (have) {
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        nxt[r4] = src[r4 * 64];
      }
    }
    asm volatile("" ::: "memory");  // keep the next chunk's loads here, not hoisted
#pragma unroll
    for (int r4 = 0; r4 < 4; ++r4)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[r4][e], hb[t][4 * r4 + e], acc, 0, 0, 0);
    if (have) {
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) cur[r4] = nxt[r4];
    }
  }
  return acc;
}

// Raw conditioner outputs of one (sample, transformed dim) in the LDS ring:
// row q of the last layer lives at slot (q>>5)&mask, row q&31, column s.
struct RingParams {
  const float* ring;  // wave ring base + s
  int base;           // d * S
  int K, mask;
  float sx, sy, rsx, rsy;  // sum(squareplus) and refined reciprocals
  float c, norm, rnorm;    // threshold c, 1 + c*K and its reciprocal
  // row q of the last layer lives at ring slot (q >> 5) & (nslot-1), row q & 31:
  // ((q>>5)&mask)*1024 + (q&31)*32 == (q & (32*nslot-1)) * 32
  __device__ __forceinline__ float at(int q) const { return ring[(q & mask) << 5]; }
  // softmax_with_threshold (utils.py:23-34): (x / xs + c) / (1 + c*n), both
  // divisions correctly rounded (div_cr); squareplus values were stored in place.
  __device__ __forceinline__ float w(int j) const {
    return div_cr(div_cr(at(base + j), sx, rsx) + c, norm, rnorm);
  }
  __device__ __forceinline__ float h(int j) const {
    return div_cr(div_cr(at(base + K + j), sy, rsy) + c, norm, rnorm);
  }
  __device__ __forceinline__ float d(int j) const { return squareplus_fast(at(base + 2 * K + j)); }
};

// One pair of transformed dims (next_d, next_d+1; lanes 0-31 / 32-63) of the
// coupling: normalize_spline_params on the raw conditioner rows in the ring
// (utils.py:37-62), bin search + gather + RQ spline (utils.py:65-250) on the
// state column, per-dim log-det combined in dim order (utils.py:139).
template <bool INV>
__device__ __forceinline__ void spline_pair(float* ring, float* xs, int s, int hh, int next_d, int end,
                                            int S, int K, int mask, float cth, float norm, float rnorm,
                                            int rot, int D, float& ldc) {
  const int d = next_d + hh;
  float ldv = 0.f;
  if (d < end) {
    RingParams p;
    p.ring = ring + s;
    p.base = d * S;
    p.K = K;
    p.mask = (mask << 5) | 31;
    p.c = cth;
    p.norm = norm;
    p.rnorm = rnorm;
    float* rp = ring + s;
    float sx = 0.f, sy = 0.f;
    for (int j = 0; j < K; ++j) {  // squareplus in place + sums (utils.py:30-33)
      const int qx = p.base + j, qy = p.base + K + j;
      float* ax = rp + ((qx & p.mask) << 5);
      float* ay = rp + ((qy & p.mask) << 5);
      const float vx = squareplus_fast(*ax), vy = squareplus_fast(*ay);
      *ax = vx;
      *ay = vy;
      sx = sx + vx;
      sy = sy + vy;
    }
    p.sx = sx;
    p.sy = sy;
    p.rsx = rcp_refined(sx);
    p.rsy = rcp_refined(sy);
    float* xp = xs + wrap(d + rot, D) * 32 + s;
    const float xv = *xp;
    const RqsBin bin = rqs_bin<!INV>(xv, K, p);
    if (!INV) {
      float yv, l;
      rqs_forward_eval(xv, bin, yv, l);
      *xp = yv;
      ldv = l;
    } else {
      *xp = rqs_inverse_eval(xv, bin);
    }
  }
  wave_lds_sync();
  if (!INV) {  // log_det.sum(axis=1) in dim order (utils.py:139)
    const float other = __shfl_xor(ldv, 32);
    const float first = hh == 0 ? ldv : other;
    const float second = hh == 0 ? other : ldv;
    ldc = ldc + first;
    if (end - next_d == 2) ldc = ldc + second;
  }
}

// 2 waves per SIMD (<= 256 VGPR+AGPR) up to 4 activation tiles; the 8-tile
// (hidden 256) variant needs the whole register file.
template <int HP, bool INV>
__global__ __launch_bounds__(kWaves * 64, (HP <= 128 ? 2 : 1)) void flow_kernel(
    const DevFlow* __restrict__ F, const float* __restrict__ blob, const float* __restrict__ xin,
    const float* __restrict__ cin, float* __restrict__ y_out, const float* __restrict__ ld_in,
    float* __restrict__ ld_out, float* __restrict__ lp_out, double* __restrict__ block_partial,
    int op_begin, int op_end, long long N, unsigned long long seed, int gen) {
  constexpr int T = HP / 32;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  __shared__ double s_part[kWaves];

  const int D = F->D;
  const int C = F->C;
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int s = lane & 31;
  const int hh = lane >> 5;
  float* xs = lds + wave * F->per_wave;  // state [D][32]
  float* ring = xs + 32 * D;            // [nslot][32 rows][32 samples]
  const long long row = ((long long)blockIdx.x * kWaves + wave) * kTile + s;
  const bool valid = row < N;

  load_state(xs, xin, row, valid, D, s, hh, F, seed, INV ? gen : 0);
  float ld = (ld_in != nullptr && valid) ? ld_in[row] : 0.f;
  int rot = 0;  // logical dim j is stored in column (j + rot) mod D
  wave_lds_sync();

  floatx4 wc[4];  // streamed weight chunk
  const int nq = op_end - op_begin;
  for (int q = 0; q < nq; ++q) {
    const int oi = INV ? (op_end - 1 - q) : (op_begin + q);
    const DevOp& op = F->ops[oi];
    const int kind = op.kind;
    if (kind == ZF_OP_ROLL) {  // bijectors.py:291 / :296
      rot = pmod(INV ? rot + op.shift : rot - op.shift, D);
    } else if (kind == ZF_OP_SHIFT_BOUNDS) {
      shift_bounds_op<INV>(blob + op.sb, xs, s, hh, rot, D, ld);
    } else {  // ZF_OP_NSC, bijectors.py:329-371
      const int dt = op.dt;
      {  // first streamed chunk flies while layer 0 runs
        const floatx4* f = reinterpret_cast<const floatx4*>(blob + op.first_chunk) + lane;
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4) wc[r4] = f[r4 * 64];
      }
      floatx16 hb[T];
      layer0<T>(op, blob, xs, cin, row, valid, C, rot, D, s, hh, lane, hb, T, op.act);
      // Hidden layers 1..n_hidden-1 (:343-345): HP x HP on MFMA.  The last
      // tile of each layer prefetches the next layer's first chunk.
      for (int l = 1; l < op.n_hidden; ++l) {
        const floatx4* wl = reinterpret_cast<const floatx4*>(blob + op.w[l]) + lane;
        const floatx4* wnext = reinterpret_cast<const floatx4*>(blob + op.w[l + 1]) + lane;
        floatx16 ho[T];
#pragma unroll
        for (int o = 0; o < T; ++o) {
          const floatx4* nx = (o + 1 < T) ? wl + (o + 1) * T * 256 : wnext;
          floatx4 bv[4];
          bias_tile(blob + op.b[l] + o * 32, hh, bv);
          floatx16 acc = mfma_tile<T>(wl + o * T * 256, nx, wc, hb);
          if (op.act == ZF_ACT_SWISH) {
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = swish(acc[r] + bv[r >> 2][r & 3]);
          } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = act_other(op.act, acc[r] + bv[r >> 2][r & 3]);
          }
          ho[o] = acc;
        }
#pragma unroll
        for (int o = 0; o < T; ++o) hb[o] = ho[o];
      }
      // Last Dense (:346) -> (N, dt, 3K-1) params (:347), tile by tile through the ring.
      const int K = op.K, S = op.S, mask = op.nslot_mask;
      const floatx4* wl = reinterpret_cast<const floatx4*>(blob + op.w[op.n_hidden]) + lane;
      const float* bl = blob + op.b[op.n_hidden];
      const KnotConsts kc(K);
      const float cth = kc.c, norm = kc.norm, rnorm = kc.rnorm;
      int next_d = 0;
      float ldc = 0.f;
      const int T_last = op.T_last;
      for (int o = 0; o < T_last; ++o) {
        const floatx4* nx = (o + 1 < T_last) ? wl + (o + 1) * T * 256 : nullptr;
        floatx4 bv[4];
        bias_tile(bl + o * 32, hh, bv);
        floatx16 acc = mfma_tile<T>(wl + o * T * 256, nx, wc, hb);
        float* slot = ring + ((o & mask) << 10) + s;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rr = (r & 3) + 8 * (r >> 2) + 4 * hh;
          slot[rr * 32] = acc[r] + bv[r >> 2][r & 3];
        }
        wave_lds_sync();
        // Run the spline for every pair of transformed dims whose 2*S parameter
        // rows are complete, except after the last tile: the pairs left then
        // run below, after the loop, when the hidden activations are dead.
        if (o + 1 < T_last) {
          while (next_d < dt) {
            const int end = (next_d + 2 < dt) ? next_d + 2 : dt;
            if (end * S > (o + 1) * 32) break;
            spline_pair<INV>(ring, xs, s, hh, next_d, end, S, K, mask, cth, norm, rnorm, rot, D, ldc);
            next_d += 2;
          }
        }
      }
      while (next_d < dt) {
        const int end = (next_d + 2 < dt) ? next_d + 2 : dt;
        spline_pair<INV>(ring, xs, s, hh, next_d, end, S, K, mask, cth, norm, rnorm, rot, D, ldc);
        next_d += 2;
      }
      if (!INV) ld = ld + ldc;  // Chain: log_det += ld (bijectors.py:110)
    }
  }

  flow_epilogue<kWaves>(F, xs, s, hh, lane, wave, rot, D, row, valid, ld, lp_out, block_partial, 1, 0,
                        y_out, ld_out, s_part);
}

// Distribution.sample on the device: one thread per (row, dim).
__global__ __launch_bounds__(256) void latent_sample_kernel(int latent, float param, unsigned long long seed,
                                                            float* __restrict__ z, long long n, int D) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const long long row = i / D;
  const int d = (int)(i - row * D);
  z[i] = latent_draw(latent, param, seed, row, d);
}

// Deterministic fixed-order sum of per-block partials -> out[0]: one block
// of 1024 threads, eight independent loads in flight per thread (the
// 2^20-row NLL has 8192 partials), then a fixed LDS tree.
constexpr int kReduceThreads = 1024;
__global__ __launch_bounds__(kReduceThreads) void reduce_partials(const double* __restrict__ part, long long n,
                                                                  double* __restrict__ out) {
  __shared__ double sm[kReduceThreads];
  const int t = threadIdx.x;
  double acc = 0.0;
  long long i = t;
  for (; i + 7 * kReduceThreads < n; i += 8 * kReduceThreads) {
    double v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = part[i + j * kReduceThreads];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += v[j];
  }
  for (; i < n; i += kReduceThreads) acc += part[i];
  sm[t] = acc;
  __syncthreads();
  for (int w = kReduceThreads / 2; w >= 1; w >>= 1) {
    if (t < w) sm[t] += sm[t + w];
    __syncthreads();
  }
  if (t == 0) out[0] = sm[0];
}

// ---------------------------------------------------------------------------
// Host side: planning, packing, launches.
// ---------------------------------------------------------------------------

int round_up(int a, int m) { return (a + m - 1) / m * m; }
int64_t round_up64(int64_t a, int64_t m) { return (a + m - 1) / m * m; }

int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

struct OpGeom {
  int dt, dc, DC, K, S, OUT, KS0, T_last, nslot;
};

OpGeom nsc_geom(const zf_flow_desc* desc, const zf_op_desc& op) {
  OpGeom g;
  const int D = desc->dim;
  g.dt = D / 2;
  g.dc = D - g.dt;
  g.DC = g.dc + desc->cond_dim;
  g.K = op.knots;
  g.S = 3 * g.K - 1;
  g.OUT = g.dt * g.S;
  g.KS0 = (g.DC + 1) / 2;
  g.T_last = (g.OUT + 31) / 32;
  const int span = (g.dt >= 2 ? 2 * g.S : g.S);
  int need = (span + 31) / 32 + 1;
  if (need > g.T_last) need = g.T_last;
  g.nslot = next_pow2(need);
  return g;
}

int hidden_pad_of(const zf_flow_desc* desc) {
  int hmax = 0;
  for (int i = 0; i < desc->n_ops; ++i) {
    const zf_op_desc& op = desc->ops[i];
    if (op.kind != ZF_OP_NSC) continue;
    for (int l = 0; l < op.n_hidden; ++l) hmax = op.hidden[l] > hmax ? op.hidden[l] : hmax;
  }
  if (hmax == 0) return 32;
  int hp = 32;
  while (hp < hmax) hp <<= 1;  // instantiated tile counts: 1, 2, 4, 8
  return hp;
}

// Widths up to 256 run in the fused kernels; wider ones on the layered path
// (zf_layered.hip), whose row chunks shrink as the width grows.
constexpr int kMaxFusedWidth = 256, kMaxLayeredWidth = 4096;
// knots: the fused kernels take up to 64, the layered path's per-(row, dim)
// spline kernels (one row's 3K - 1 parameters per thread in LDS) up to 200
constexpr int kMaxFusedKnots = 64, kMaxLayeredKnots = 200;

int validate(const zf_flow_desc* desc) {
  if (!desc) return einval("desc is NULL");
  if (desc->dim < 1 || desc->dim > 64) return einval("dim %d out of range [1, 64]", desc->dim);
  if (desc->cond_dim < 0 || desc->cond_dim > 64) return einval("cond_dim out of range");
  if (desc->n_ops < 0 || desc->n_ops > kMaxOps) return einval("n_ops out of range");
  if (desc->latent < ZF_LATENT_NONE || desc->latent > ZF_LATENT_UNIFORM) return einval("bad latent");
  for (int i = 0; i < desc->n_ops; ++i) {
    const zf_op_desc& op = desc->ops[i];
    if (op.kind == ZF_OP_NSC) {
      if (desc->dim < 2) return einval("NeuralSplineCoupling needs dim >= 2");
      if (op.knots < 1 || op.knots > kMaxLayeredKnots)
        return einval("knots %d out of range [1, %d]", op.knots, kMaxLayeredKnots);
      if (op.n_hidden < 1 || op.n_hidden > 16) return enotsup("n_hidden must be in [1, 16]");
      for (int l = 0; l < op.n_hidden; ++l)
        if (op.hidden[l] < 1 || op.hidden[l] > kMaxLayeredWidth)
          return enotsup("hidden width must be in [1, 4096]");
      if (op.act < 0 || op.act >= ZF_ACT_COUNT) return einval("op %d: unknown activation %d", i, op.act);
    } else if (op.kind != ZF_OP_ROLL && op.kind != ZF_OP_SHIFT_BOUNDS) {
      return einval("op %d: unknown kind %d", i, op.kind);
    }
  }
  return ZF_OK;
}

}  // namespace
}  // namespace zf

struct zf_flow {
  zf_flow_desc desc;
  zf::DevFlow host;           // device descriptor (host copy)
  std::vector<float> natural; // natural blob (host copy, for stat updates)
  std::vector<float> packed;  // device blob (host copy)
  zf::DevFlow* d_desc = nullptr;
  float* d_blob = nullptr;
  void* d_x3 = nullptr;       // bf16x3 weight-group stream (x3 kernel), or null
  int x3_K = 0;
  bool x3_oact = false;  // some coupling's activation is not swish
  int x3_aset = 0;       // X3Launch::aset: which non-swish activations the flow uses
  int device = 0;
  zf::LayeredFlow* lay = nullptr;  // layered eval path (a hidden width > 256), or null
};

namespace zf {
namespace {

// Fill the packed (device) blob from the natural blob.  Layouts: zf_flow.hip
// header + DESIGN.md §Data layout.
void pack_nsc_bn(const zf_flow_desc* desc, const zf_op_desc& op, const float* nat, float* dst) {
  const OpGeom g = nsc_geom(desc, op);
  const int DCp = 2 * g.KS0;
  const float* mean = nat + op.off_bn;
  const float* var = mean + g.DC;
  const float* scale = var + g.DC;
  const float* bias = scale + g.DC;
  for (int k = 0; k < DCp; ++k) {
    if (k < g.DC) {
      // flax BatchNorm: mul = rsqrt(var + eps) * scale
      const float mul = (1.0f / std::sqrt(var[k] + 1e-5f)) * scale[k];
      dst[k] = mean[k];
      dst[DCp + k] = mul;
      dst[2 * DCp + k] = bias[k];
    } else {
      dst[k] = dst[DCp + k] = dst[2 * DCp + k] = 0.f;
    }
  }
}

void pack_sb(const zf_flow_desc* desc, const zf_op_desc& op, const float* nat, float* dst) {
  for (int i = 0; i < desc->dim; ++i) {
    const float* r = nat + op.off_sb + 8 * i;
    const int mode = (int)r[0];
    const float a = r[1], b = r[2], xmin = r[3], xmax = r[4];
    float mul;
    if (mode == ZF_SB_BOTH) mul = (float)(1.0 / ((double)b - (double)a));  // :189 (Python floats)
    else mul = 1.0f / (xmax - xmin);                                        // :265
    float* o = dst + 8 * i;
    o[0] = (float)mode; o[1] = a; o[2] = b; o[3] = xmin; o[4] = xmax;
    o[5] = mul; o[6] = std::log(mul); o[7] = 0.f;
  }
}

}  // namespace
}  // namespace zf

extern "C" {

int zf_flow_plan(zf_flow_desc* desc, int64_t* blob_floats) {
  int rc = zf::validate(desc);
  if (rc) return rc;
  if (!blob_floats) return zf::einval("blob_floats is NULL");
  int64_t off = 0;
  for (int i = 0; i < desc->n_ops; ++i) {
    zf_op_desc& op = desc->ops[i];
    op.off_bn = op.off_sb = 0;
    for (int l = 0; l < 17; ++l) op.off_w[l] = op.off_b[l] = 0;
    if (op.kind == ZF_OP_NSC) {
      const zf::OpGeom g = zf::nsc_geom(desc, op);
      op.off_bn = off;
      off += 4 * g.DC;
      int in = g.DC;
      for (int l = 0; l <= op.n_hidden; ++l) {
        const int out = l < op.n_hidden ? op.hidden[l] : g.OUT;
        op.off_w[l] = off;
        off += (int64_t)in * out;
        op.off_b[l] = off;
        off += out;
        in = out;
      }
    } else if (op.kind == ZF_OP_SHIFT_BOUNDS) {
      op.off_sb = off;
      off += 8 * desc->dim;
    }
  }
  *blob_floats = off;
  return ZF_OK;
}

int zf_flow_create(const zf_flow_desc* desc_in, const float* blob_host, int64_t blob_floats,
                   zf_flow_t** handle) {
  if (!handle) return zf::einval("handle is NULL");
  *handle = nullptr;
  zf_flow_desc desc = *desc_in;
  int64_t need = 0;
  int rc = zf_flow_plan(&desc, &need);
  if (rc) return rc;
  if (blob_floats != need) return zf::einval("blob has %lld floats, plan needs %lld", (long long)blob_floats, (long long)need);
  if (need > 0 && !blob_host) return zf::einval("blob is NULL");

  zf_flow* h = new zf_flow();
  h->desc = desc;
  h->natural.assign(blob_host, blob_host + need);
  zf::DevFlow& F = h->host;
  std::memset(&F, 0, sizeof(F));
  F.D = desc.dim;
  F.C = desc.cond_dim;
  F.latent = desc.latent;
  F.n_ops = desc.n_ops;
  F.HP = zf::hidden_pad_of(&desc);
  // a conditioner wider than the fused kernels hold runs layer by layer
  // knots beyond the fused kernels' (64: the split-MFMA kernel's largest
  // instantiation, and the fp32 kernel's LDS ring) run on the layered path too
  int kmax_ops = 0;
  for (int i = 0; i < desc.n_ops; ++i)
    if (desc.ops[i].kind == ZF_OP_NSC && desc.ops[i].knots > kmax_ops) kmax_ops = desc.ops[i].knots;
  const bool layered = F.HP > zf::kMaxFusedWidth || kmax_ops > zf::kMaxFusedKnots;
  if (layered) F.HP = 32;  // the fused layouts below are then not built
  int x3K = 0;
  // the split-MFMA kernel runs hidden <= 128 padded to 128 (4 tiles)
  const bool x3 = !layered && zf::x3_eligible(desc, F.HP < 128 ? 128 : F.HP, &x3K);
  if (x3 && F.HP < 128) F.HP = 128;
  const int HP = F.HP, T = HP / 32;
  // Latent constants in fp32, as jax.scipy.stats computes them.
  {
    const float s2 = 0.1f * 0.1f;
    F.lat_c0 = std::log(6.28318530717958647692f * s2);
    F.lat_c1 = s2;
    if (desc.latent == ZF_LATENT_BETA) {
      const double a = desc.latent_param;
      F.lat_c0 = (float)(-(std::lgamma(a) + std::lgamma(a) - std::lgamma(2.0 * a)));
      F.lat_c1 = (float)a - 1.0f;
      F.lat_c3 = (float)a;  // peakness, for on-device sampling
    } else if (desc.latent == ZF_LATENT_TRUNCNORM) {
      // _log_gauss_mass(-5, 5) = log1p(-ndtr(-5) - ndtr(-5))
      const float nd = (float)(0.5 * std::erfc(5.0 / std::sqrt(2.0)));
      F.lat_c2 = std::log1p(-nd - nd);
    }
  }
  // Packed blob layout.
  int64_t off = 0;
  auto take = [&](int64_t n) { const int64_t o = off; off = zf::round_up64(off + n, 4); return o; };
  int nslot = 1;
  // Small per-op parameters (ShiftBounds rows, BatchNorm, first Dense,
  // biases) first, for all ops: the bf16x3 kernel stages [0, small_floats)
  // in LDS once per block.  The streamed fp32 weight fragments follow.
  for (int i = 0; i < desc.n_ops; ++i) {
    const zf_op_desc& op = desc.ops[i];
    zf::DevOp& d = F.ops[i];
    d.kind = op.kind;
    d.shift = op.shift;
    if (op.kind == ZF_OP_NSC) {
      const zf::OpGeom g = zf::nsc_geom(&desc, op);
      d.K = g.K; d.S = g.S; d.n_hidden = op.n_hidden; d.dt = g.dt; d.dc = g.dc; d.DC = g.DC;
      d.KS0 = g.KS0; d.T_last = g.T_last; d.nslot_mask = g.nslot - 1; d.act = op.act;
      nslot = g.nslot > nslot ? g.nslot : nslot;
      d.bn = take(3 * 2 * g.KS0);
      if (layered) continue;  // BatchNorm rows only: the layered path reads the natural weights
      d.w[0] = take((int64_t)T * g.KS0 * 64);
      for (int l = 0; l < op.n_hidden; ++l) d.b[l] = take((int64_t)T * 32);
      d.b[op.n_hidden] = take((int64_t)g.T_last * 32);
      d.x3 = -1;
      if (x3) d.x3_blast = take((int64_t)zf::x3_pairs(desc) * zf::x3_last_tiles(x3K) * 32);
    } else if (op.kind == ZF_OP_SHIFT_BOUNDS) {
      d.sb = take(8 * desc.dim);
    }
  }
  F.small_floats = (int)off;
  for (int i = 0; i < desc.n_ops; ++i) {
    const zf_op_desc& op = desc.ops[i];
    zf::DevOp& d = F.ops[i];
    if (op.kind != ZF_OP_NSC || layered) continue;
    const zf::OpGeom g = zf::nsc_geom(&desc, op);
    for (int l = 1; l < op.n_hidden; ++l) d.w[l] = take((int64_t)T * T * 1024);
    d.w[op.n_hidden] = take((int64_t)g.T_last * T * 1024);
    d.first_chunk = op.n_hidden > 1 ? d.w[1] : d.w[op.n_hidden];
  }
  F.nslot = nslot;
  F.per_wave = zf::round_up(32 * desc.dim, 4) + nslot * 1024;
  h->packed.assign((size_t)(off > 0 ? off : 4), 0.f);
  float* P = h->packed.data();
  const float* nat = h->natural.data();
  for (int i = 0; i < desc.n_ops; ++i) {
    const zf_op_desc& op = desc.ops[i];
    const zf::DevOp& d = F.ops[i];
    if (op.kind == ZF_OP_SHIFT_BOUNDS) {
      zf::pack_sb(&desc, op, nat, P + d.sb);
    } else if (op.kind == ZF_OP_NSC) {
      const zf::OpGeom g = zf::nsc_geom(&desc, op);
      zf::pack_nsc_bn(&desc, op, nat, P + d.bn);
      if (layered) continue;
      // layer 0: A fragment of (o, ks): lane l -> W0[k = 2ks + (l>>5)][i = 32o + (l&31)]
      {
        const int in = g.DC, out = op.hidden[0];
        const float* W = nat + op.off_w[0];
        const float* B = nat + op.off_b[0];
        for (int o = 0; o < T; ++o)
          for (int ks = 0; ks < g.KS0; ++ks)
            for (int l = 0; l < 64; ++l) {
              const int k = 2 * ks + (l >> 5), ii = 32 * o + (l & 31);
              P[d.w[0] + ((int64_t)o * g.KS0 + ks) * 64 + l] = (k < in && ii < out) ? W[(int64_t)k * out + ii] : 0.f;
            }
        for (int o = 0; o < T; ++o)
          for (int hh = 0; hh < 2; ++hh)
            for (int r = 0; r < 16; ++r) {
              const int ii = 32 * o + (r & 3) + 8 * (r >> 2) + 4 * hh;
              P[d.b[0] + (o * 2 + hh) * 16 + r] = ii < out ? B[ii] : 0.f;
            }
      }
      // layers 1..n_hidden: fragment (o, t, r4, lane, e) ->
      //   W[k = 32t + e + 8 r4 + 4 (lane>>5)][i = 32o + (lane&31)]
      for (int l = 1; l <= op.n_hidden; ++l) {
        const int in = op.hidden[l - 1];
        const int out = l < op.n_hidden ? op.hidden[l] : g.OUT;
        const int To = l < op.n_hidden ? T : g.T_last;
        const float* W = nat + op.off_w[l];
        const float* B = nat + op.off_b[l];
        float* Wp = P + d.w[l];
        for (int o = 0; o < To; ++o)
          for (int t = 0; t < T; ++t)
            for (int r4 = 0; r4 < 4; ++r4)
              for (int ln = 0; ln < 64; ++ln)
                for (int e = 0; e < 4; ++e) {
                  const int k = 32 * t + e + 8 * r4 + 4 * (ln >> 5);
                  const int ii = 32 * o + (ln & 31);
                  Wp[((((int64_t)o * T + t) * 4 + r4) * 64 + ln) * 4 + e] =
                      (k < in && ii < out) ? W[(int64_t)k * out + ii] : 0.f;
                }
        for (int o = 0; o < To; ++o)
          for (int hh = 0; hh < 2; ++hh)
            for (int r = 0; r < 16; ++r) {
              const int ii = 32 * o + (r & 3) + 8 * (r >> 2) + 4 * hh;
              P[d.b[l] + (o * 2 + hh) * 16 + r] = ii < out ? B[ii] : 0.f;
            }
      }
    }
  }
  std::vector<uint16_t> x3s;
  const int NT = zf::x3_scheme_for(desc);
  if (x3) {
    // each NSC's small parameters [bn, end of the permuted last bias) as whole
    // 1 KiB DMA pieces (the blob allocation carries 1 KiB of slack past its end)
    const int tl = desc.dim / 2 == 1 ? (3 * x3K - 1 + 31) / 32 : zf::x3_last_tiles(x3K);
    int maxp = 0;
    for (int i = 0; i < desc.n_ops; ++i) {
      if (desc.ops[i].kind != ZF_OP_NSC) continue;
      zf::DevOp& d = F.ops[i];
      const int64_t end = d.x3_blast + (int64_t)zf::x3_pairs(desc) * tl * 32;
      d.x3_par_pieces = (int)((end - d.bn) * 4 + 1023) / 1024;
      maxp = d.x3_par_pieces > maxp ? d.x3_par_pieces : maxp;
    }
    F.x3_par_bytes = maxp * 1024;
  }
  if (x3 && zf::x3_lds_bytes(zf::x3_buf_tiles(desc, T, x3K), desc.dim + desc.cond_dim, NT, F.x3_par_bytes) <=
                160 * 1024) {
    zf::x3_pack(desc, nat, T, NT, x3K, F, P, x3s);
    F.x3_ok = NT == 3 ? 1 : 2;
    h->x3_K = x3K;
    for (int i = 0; i < desc.n_ops; ++i)
      if (desc.ops[i].kind == ZF_OP_NSC) F.kreal = desc.ops[i].knots;
    for (int i = 0; i < desc.n_ops; ++i)
      if (desc.ops[i].kind == ZF_OP_NSC && desc.ops[i].act != ZF_ACT_SWISH) h->x3_oact = true;
    {
      bool centred = false, plain = false;
      for (int i = 0; i < desc.n_ops; ++i) {
        if (desc.ops[i].kind != ZF_OP_NSC || desc.ops[i].act == ZF_ACT_SWISH) continue;
        if (desc.ops[i].act == ZF_ACT_SIGMOID || desc.ops[i].act == ZF_ACT_SOFTPLUS) centred = true;
        else plain = true;
      }
      h->x3_aset = centred && plain ? 0 : centred ? 2 : 1;
    }
  }
  const bool use_x3 = F.x3_ok != 0;
  int rcd = ZF_OK;
  hipError_t e = hipGetDevice(&h->device);
  if (e == hipSuccess && layered) {
    rcd = zf::layered_create(desc, nat, need, &h->lay);
    if (rcd) {
      zf_flow_destroy(h);
      return rcd;
    }
  }
  if (e == hipSuccess && use_x3) e = hipMalloc(&h->d_x3, x3s.size() * sizeof(uint16_t));
  if (e == hipSuccess && use_x3)
    e = hipMemcpy(h->d_x3, x3s.data(), x3s.size() * sizeof(uint16_t), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMalloc(&h->d_desc, sizeof(zf::DevFlow));
  // + 1 KiB: the split-MFMA kernel DMAs whole 1 KiB pieces of small parameters
  if (e == hipSuccess) e = hipMalloc(&h->d_blob, h->packed.size() * sizeof(float) + 1024);
  if (e == hipSuccess) e = hipMemcpy(h->d_desc, &h->host, sizeof(zf::DevFlow), hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = hipMemcpy(h->d_blob, h->packed.data(), h->packed.size() * sizeof(float), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    rcd = zf::hip_status(e, "zf_flow_create");
    zf_flow_destroy(h);
    return rcd;
  }
  *handle = h;
  return ZF_OK;
}

int zf_flow_destroy(zf_flow_t* h) {
  if (!h) return ZF_OK;
  if (h->d_desc) (void)hipFree(h->d_desc);
  if (h->d_blob) (void)hipFree(h->d_blob);
  if (h->d_x3) (void)hipFree(h->d_x3);
  zf::layered_destroy(h->lay);
  delete h;
  return ZF_OK;
}

int zf_flow_kernel_variant(const zf_flow_t* h) {
  if (!h) return -1;
  if (h->lay) return ZF_KERNEL_LAYERED;
  return h->host.x3_ok == 2 ? ZF_KERNEL_F16X2 : h->host.x3_ok ? ZF_KERNEL_BF16X3 : ZF_KERNEL_FP32;
}

int64_t zf_flow_workspace_bytes(int64_t N) {
  const int64_t blocks = (N + zf::kBlockRows - 1) / zf::kBlockRows;
  return zf::round_up64(blocks * 8 + 64, 256);
}

}  // extern "C"

namespace zf {
namespace {

template <bool INV>
int launch_flow(zf_flow* h, int op_begin, int op_end, const float* x, const float* c, float* y,
                const float* ld_in, float* ld_out, float* lp, double* part, int64_t N,
                void* stream, unsigned long long seed = 0, int gen = 0) {
  if (!h) return einval("handle is NULL");
  if (N < 0) return einval("N < 0");
  if (op_begin < 0 || op_end > h->host.n_ops || op_begin > op_end) return einval("bad op range");
  if (N == 0) return ZF_OK;
  if (!x && !gen) return einval("x is NULL");
  if (h->host.C > 0 && !c) return einval("flow is conditional (C=%d) but c is NULL", h->host.C);
  if (h->lay)
    return layered_run(h->lay, h->host, h->d_blob, INV, op_begin, op_end, x, c, y, ld_in, ld_out, lp, part, N,
                       (hipStream_t)stream, seed, gen);
  if (h->host.x3_ok) {
    X3Launch a;
    a.desc = h->d_desc; a.blob = h->d_blob; a.x3 = h->d_x3;
    a.x = x; a.c = c; a.y = y; a.ld_in = ld_in; a.ld_out = ld_out; a.lp = lp; a.part = part;
    a.nparts = (N + kBlockRows - 1) / kBlockRows;
    a.op_begin = op_begin; a.op_end = op_end; a.N = N; a.K = h->x3_K; a.D = h->host.D; a.C = h->host.C; a.T = h->host.HP / 32;
    a.NT = h->host.x3_ok == 2 ? 2 : 3;
    a.oact = h->x3_oact;
    a.aset = h->x3_aset;
    a.par_bytes = h->host.x3_par_bytes;
    a.seed = seed;
    a.gen = gen;
    a.stream = (hipStream_t)stream;
    return launch_flow_x3(a, INV);
  }
  const int64_t grid = (N + kBlockRows - 1) / kBlockRows;
  if (grid > 0x7fffffffLL) return einval("N too large");
  const size_t lds = sizeof(float) * (size_t)kWaves * h->host.per_wave;
  if (lds > 160 * 1024 - 64) return enotsup("LDS footprint too large (dim/knots)");
  hipStream_t st = (hipStream_t)stream;
  const long long n = (long long)N;
#define ZF_LAUNCH(HPV)                                                                          \
  hipLaunchKernelGGL((flow_kernel<HPV, INV>), dim3((unsigned)grid), dim3(kWaves * 64), lds, st, \
                     h->d_desc, h->d_blob, x, c, y, ld_in, ld_out, lp, part, op_begin, op_end, n, seed, gen)
  switch (h->host.HP) {
    case 32: ZF_LAUNCH(32); break;
    case 64: ZF_LAUNCH(64); break;
    case 128: ZF_LAUNCH(128); break;
    case 256: ZF_LAUNCH(256); break;
    default: return enotsup("hidden width");
  }
#undef ZF_LAUNCH
  ZF_CHECK_LAUNCH("flow_kernel");
  return ZF_OK;
}

}  // namespace
}  // namespace zf

extern "C" {

int zf_flow_log_prob_segment(zf_flow_t* h, int op_begin, int op_end, const float* x,
                             const float* c, const float* log_det_in, float* log_prob,
                             double* nll_sum, void* workspace, int64_t N, void* stream) {
  if (!h) return zf::einval("handle is NULL");
  if (!log_prob) return zf::einval("log_prob is NULL");
  if (h->host.latent == ZF_LATENT_NONE) return zf::einval("flow has no latent distribution");
  if (nll_sum && !workspace) return zf::einval("nll_sum requires a workspace");
  if (N == 0) {
    if (nll_sum) ZF_TRY_HIP(hipMemsetAsync(nll_sum, 0, sizeof(double), (hipStream_t)stream));
    return ZF_OK;
  }
  double* part = (double*)workspace;  // per-block partials when a workspace is given
  int rc = zf::launch_flow<false>(h, op_begin, op_end, x, c, nullptr, log_det_in, nullptr,
                                  log_prob, part, N, stream);
  if (rc) return rc;
  if (nll_sum) return zf_flow_nll_reduce(workspace, N, nll_sum, stream);
  return ZF_OK;
}

int zf_flow_nll_reduce(const void* workspace, int64_t N, double* nll_sum, void* stream) {
  if (!workspace || !nll_sum) return zf::einval("NULL argument");
  if (N <= 0) {
    ZF_TRY_HIP(hipMemsetAsync(nll_sum, 0, sizeof(double), (hipStream_t)stream));
    return ZF_OK;
  }
  const long long blocks = (N + zf::kBlockRows - 1) / zf::kBlockRows;
  hipLaunchKernelGGL(zf::reduce_partials, dim3(1), dim3(zf::kReduceThreads), 0, (hipStream_t)stream,
                     (const double*)workspace, blocks, nll_sum);
  ZF_CHECK_LAUNCH("reduce_partials");
  return ZF_OK;
}

int zf_flow_log_prob(zf_flow_t* h, const float* x, const float* c, float* log_prob,
                     double* nll_sum, void* workspace, int64_t N, void* stream) {
  if (!h) return zf::einval("handle is NULL");
  return zf_flow_log_prob_segment(h, 0, h->host.n_ops, x, c, nullptr, log_prob, nll_sum,
                                  workspace, N, stream);
}

int zf_flow_forward(zf_flow_t* h, int op_begin, int op_end, const float* x, const float* c,
                    float* y, const float* log_det_in, float* log_det, int64_t N, void* stream) {
  return zf::launch_flow<false>(h, op_begin, op_end, x, c, y, log_det_in, log_det, nullptr,
                                nullptr, N, stream);
}

int zf_flow_inverse(zf_flow_t* h, int op_begin, int op_end, const float* z, const float* c,
                    float* x, int64_t N, void* stream) {
  if (!x && N > 0) return zf::einval("x is NULL");
  return zf::launch_flow<true>(h, op_begin, op_end, z, c, x, nullptr, nullptr, nullptr, nullptr,
                               N, stream);
}

int zf_flow_sample(zf_flow_t* h, uint64_t seed, const float* c, float* x, int64_t N, void* stream) {
  if (!h) return zf::einval("handle is NULL");
  if (!x && N > 0) return zf::einval("x is NULL");
  if (h->host.latent == ZF_LATENT_NONE) return zf::einval("flow has no latent distribution");
  return zf::launch_flow<true>(h, 0, h->host.n_ops, nullptr, c, x, nullptr, nullptr, nullptr, nullptr,
                               N, stream, (unsigned long long)seed, 1);
}

int zf_latent_sample(int latent, double param, uint64_t seed, float* z, int64_t N, int D, void* stream) {
  if (latent < ZF_LATENT_NORMAL || latent > ZF_LATENT_UNIFORM) return zf::einval("bad latent %d", latent);
  if (latent == ZF_LATENT_BETA && !(param >= 1.0)) return zf::einval("Beta peakness must be >= 1");
  if (N < 0 || D < 1) return zf::einval("bad shape");
  if (N == 0) return ZF_OK;
  if (!z) return zf::einval("z is NULL");
  const long long n = (long long)N * D;
  const long long grid = (n + 255) / 256;
  if (grid > 0x7fffffffLL) return zf::einval("N too large");
  hipLaunchKernelGGL(zf::latent_sample_kernel, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, latent,
                     (float)param, (unsigned long long)seed, z, n, D);
  ZF_CHECK_LAUNCH("latent_sample_kernel");
  return ZF_OK;
}

static int upload_region(zf_flow* h, int64_t off, int64_t n) {
  ZF_TRY_HIP(hipSetDevice(h->device));
  ZF_TRY_HIP(hipDeviceSynchronize());  // no kernel may still read the blob
  ZF_TRY_HIP(hipMemcpy(h->d_blob + off, h->packed.data() + off, n * sizeof(float),
                       hipMemcpyHostToDevice));
  return ZF_OK;
}

int zf_flow_set_bn_stats(zf_flow_t* h, int op, const float* mean, const float* var) {
  if (!h || !mean || !var) return zf::einval("NULL argument");
  if (op < 0 || op >= h->desc.n_ops || h->desc.ops[op].kind != ZF_OP_NSC) return zf::einval("op %d is not an NSC", op);
  const zf_op_desc& od = h->desc.ops[op];
  const zf::OpGeom g = zf::nsc_geom(&h->desc, od);
  float* nat = h->natural.data() + od.off_bn;
  for (int k = 0; k < g.DC; ++k) { nat[k] = mean[k]; nat[g.DC + k] = var[k]; }
  zf::pack_nsc_bn(&h->desc, od, h->natural.data(), h->packed.data() + h->host.ops[op].bn);
  return upload_region(h, h->host.ops[op].bn, 3 * 2 * g.KS0);
}

int zf_flow_set_sb_stats(zf_flow_t* h, int op, const float* xmin, const float* xmax) {
  if (!h || !xmin || !xmax) return zf::einval("NULL argument");
  if (op < 0 || op >= h->desc.n_ops || h->desc.ops[op].kind != ZF_OP_SHIFT_BOUNDS) return zf::einval("op %d is not a ShiftBounds", op);
  const zf_op_desc& od = h->desc.ops[op];
  for (int i = 0; i < h->desc.dim; ++i) {
    h->natural[od.off_sb + 8 * i + 3] = xmin[i];
    h->natural[od.off_sb + 8 * i + 4] = xmax[i];
  }
  zf::pack_sb(&h->desc, od, h->natural.data(), h->packed.data() + h->host.ops[op].sb);
  return upload_region(h, h->host.ops[op].sb, 8 * h->desc.dim);
}

}  // extern "C"
