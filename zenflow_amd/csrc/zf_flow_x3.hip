// Host side of the split-MFMA fused flow kernel (zf_flow_x3_kernel.h):
// eligibility, the group-stream packing of the conditioner weights into MFMA
// A-fragment order (bf16x3 / f16x2 terms), and the launch dispatch to the
// per-knot-count translation units zf_flow_x3_k{8,16,32}.hip.
#include "zf_flow_x3_kernel.h"

#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace zf {

int launch_x3_k8(const X3Launch& a, bool inverse);
int launch_x3_k16(const X3Launch& a, bool inverse);
int launch_x3_k32(const X3Launch& a, bool inverse);
int launch_x3_k64(const X3Launch& a, bool inverse);

namespace {

uint16_t bf16_rne(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

float bf16_f(uint16_t b) {
  const uint32_t u = (uint32_t)b << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

}  // namespace

int x3_padded_knots(int K);
int x3_param_of(int jp, int Kp, int K, float* fill);

// One knot count for all couplings and one of the instantiated shapes
// (launch_flow_x3).
bool x3_eligible(const zf_flow_desc& desc, int HP, int* K_out) {
  const char* env = std::getenv("ZF_DISABLE_X3");
  if (env && env[0] == '1') return false;
  int K = 0;
  for (int i = 0; i < desc.n_ops; ++i) {
    const zf_op_desc& op = desc.ops[i];
    if (op.kind != ZF_OP_NSC) continue;
    // relu, leaky_relu, tanh, gelu and elu (act(0) = 0, |act(v)| <= |v|: the
    // f16x2 per-sample power-of-two scale keeps every value's relative
    // precision) run on either scheme; sigmoid and softplus on f16x2 run
    // centred (act(v) - C, C = 1/2 / log 2 folded into the next bias:
    // act_tile_centered, x3_pack).  On bf16x3 (ZF_X3_SCHEME=bf16x3) sigmoid
    // runs uncentred and softplus stays on the fp32 kernel: in the
    // tiny-activation regime (deviations from log 2 under 1e4-scale weights,
    // a cancellation of 1e3-size products) bf16x3's mean error was 5x the
    // fp32 oracle's (profiles/r03_diag_acts.jsonl; held by
    // tests/test_gpu_flow.py::test_split_scaling_extremes_other_acts).
    if (op.act == ZF_ACT_SOFTPLUS && x3_scheme() == 3) return false;
    // bf16x3 (the scaling-free reference scheme) is instantiated for swish
    // couplings only: its activation-switch builds were 10 MB of the library
    // for an opt-in scheme, so other activations there run the fp32 kernel
    // 
    if (op.act != ZF_ACT_SWISH && x3_scheme() == 3) return false;
    // a chain may mix knot counts: all run at the largest one's
    // instantiation; a 1-knot coupling anywhere keeps the flow off it, as a
    // flow of 1-knot couplings is (that case is not pinned)
    if (op.knots < 2) return false;
    if (op.knots > K) K = op.knots;
  }
  // hidden <= 128 runs padded to 128 (the caller pads HP); any dim the
  // fp32 kernel takes (LDS is checked at create time)
  const int Kp = x3_padded_knots(K);
  if (HP > 256 || desc.dim > 64 || Kp == 0) return false;
  *K_out = Kp;
  return true;
}

// The instantiated knot count a flow of K knots runs at (0: none).  K < Kp
// runs as Kp knots whose extra ones are inert (x3_param_of): their widths /
// heights enter the sums as exact zeros (logit -2^40: squareplus = 0) and
// their slope logits are 0 at the last real knot (the boundary derivative
// 1) and NaN beyond, so the idx == K sliver still gives NaN (utils.py:
// 224-230).  K = Kp - 1 has no NaN slope: the kernel starts the sliver at
// knot K itself (rqs_bin_monotone's padlast, per coupling).  K in 33..64
// runs at 64 (one wave per SIMD: 12 last-layer tiles and 191 spline
// parameters per lane, x3_occupancy).
int x3_padded_knots(int K) {
  if (K < 2) return 0;
  if (K <= 8) return 8;
  if (K <= 16) return 16;
  if (K <= 32) return 32;
  if (K <= 64) return 64;
  return 0;
}

// Parameter jp (of 3 Kp - 1) of a padded (sample, dim) row -> the real
// parameter of 3 K - 1 (widths, heights, slopes), or -1 with the inert
// value in *fill.
int x3_param_of(int jp, int Kp, int K, float* fill) {
  if (jp < Kp) {
    *fill = -1099511627776.0f;  // -2^40: x + sqrt(x^2 + 4) = 0 exactly
    return jp < K ? jp : -1;
  }
  if (jp < 2 * Kp) {
    *fill = -1099511627776.0f;
    return jp - Kp < K ? K + (jp - Kp) : -1;
  }
  const int q = jp - 2 * Kp;
  *fill = q == K - 1 ? 0.0f : __builtin_nanf("");
  return q < K - 1 ? 2 * K + q : -1;
}

// Split scheme for new handles: ZF_X3_SCHEME=bf16x3 | f16x2 (default f16x2).
int x3_scheme() {
  const char* env = std::getenv("ZF_X3_SCHEME");
  if (env && std::strcmp(env, "bf16x3") == 0) return 3;
  return 2;
}

// The scheme of one flow: bf16x3 when asked for (ZF_X3_SCHEME=bf16x3),
// f16x2 otherwise (every activation; sigmoid / softplus centred).
int x3_scheme_for(const zf_flow_desc& desc) {
  (void)desc;
  return x3_scheme() == 3 ? 3 : 2;
}

int x3_last_tiles(int K) { return (3 * K - 1 + 15) / 16; }
// ONE layout (one transformed dim): 32 parameters per tile
int x3_last_tiles_one(int K) { return (3 * K - 1 + 31) / 32; }

int x3_pairs(const zf_flow_desc& desc) { return (desc.dim / 2 + 1) / 2; }

// Pack the group streams (bf16 hi/mid/lo A fragments) of every NSC and the
// row-permuted last-layer biases (into `packed` at F.ops[i].x3_blast, which
// the caller allocated with x3_pairs * x3_last_tiles(K) * 32 floats).
void x3_pack(const zf_flow_desc& desc, const float* nat, int T, int NT, int Kp, DevFlow& F, float* packed,
             std::vector<uint16_t>& stream) {
  stream.clear();
  int prev = -1;
  for (int i = 0; i < desc.n_ops; ++i) {
    F.ops[i].x3_next[0] = F.ops[i].x3_next[1] = -1;
    if (desc.ops[i].kind != ZF_OP_NSC) continue;
    if (prev >= 0) { F.ops[prev].x3_next[0] = i; F.ops[i].x3_next[1] = prev; }
    prev = i;
  }
  for (int i = 0; i < desc.n_ops; ++i) {
    const zf_op_desc& op = desc.ops[i];
    if (op.kind != ZF_OP_NSC) continue;
    DevOp& d = F.ops[i];
    // K: the coupling's knots; Kp: the instantiation's (x3_padded_knots)
    const int dt = desc.dim / 2, K = Kp, S = 3 * K - 1;  // every coupling at the flow's instantiation
    const int Kr = op.knots, Sr = 3 * Kr - 1;
    const bool one = dt == 1;
    const int TL = one ? x3_last_tiles_one(K) : x3_last_tiles(K), NP = x3_pairs(desc);
    d.x3 = (long long)stream.size() * 2;
    d.x3_tlast = TL;
    d.x3_groups = T * (op.n_hidden - 1) + T * NP;
    for (int l = 1; l <= op.n_hidden; ++l) {
      const bool last = (l == op.n_hidden);
      const int in = op.hidden[l - 1];
      const int out = last ? dt * Sr : op.hidden[l];
      const int NOUT = last ? TL : T;
      const float* W = nat + op.off_w[l];
      // f16x2: the inputs of swished layers' activations carry log2(e)
      const float pre = (NT == 2 && !last && op.act == ZF_ACT_SWISH) ? kSwishPrescale : 1.0f;
      // f16x2: the layer's power-of-two scale, max |W| * 2^kw in [2^13, 2^14)
      int kw = 0;
      if (NT == 2) {
        float mx = 0.f;
        for (int64_t i = 0; i < (int64_t)in * out; ++i)
          mx = std::fmax(mx, std::fabs(W[i] * pre));
        if (mx > 0.f && std::isfinite(mx)) {
          int e;
          std::frexp(mx, &e);
          kw = 14 - e;
        }
      }
      d.x3_kw[l] = kw;
      for (int pr = 0; pr < (last ? NP : 1); ++pr)
        for (int q = 0; q < T; ++q)
          for (int s = 0; s < 2; ++s)
            for (int o = 0; o < NOUT; ++o) {
              uint16_t part[3][64][8];  // [term][lane][element]
              for (int ln = 0; ln < 64; ++ln)
                for (int j = 0; j < 8; ++j) {
                  const int kstep = 2 * q + s;
                  const int k = 16 * kstep + 8 * (j >> 2) + 4 * (ln >> 5) + (j & 3);
                  const int rho = ln & 31;
                  int col;
                  if (!last) {
                    col = 32 * o + rho;
                    if (col >= out) col = -1;
                  } else {
                    const int h = (rho >> 2) & 1, r = (rho & 3) + 4 * (rho >> 3);
                    const int jp = one ? 32 * o + 16 * h + r : 16 * o + r;
                    const int dd = one ? 0 : 2 * pr + h;
                    float fill;
                    const int jr = jp < S ? x3_param_of(jp, K, Kr, &fill) : -1;
                    col = (dd < dt && jr >= 0) ? dd * Sr + jr : -1;
                  }
                  const float x = (k < in && col >= 0) ? W[(int64_t)k * out + col] : 0.f;
                  if (NT == 3) {
                    const uint16_t bh = bf16_rne(x);
                    const float r1 = x - bf16_f(bh);
                    const uint16_t bm = bf16_rne(r1);
                    const uint16_t bl = bf16_rne(r1 - bf16_f(bm));
                    part[0][ln][j] = bh;
                    part[1][ln][j] = bm;
                    part[2][ln][j] = bl;
                  } else {
                    const float xs = std::ldexp(x * pre, kw);
                    const _Float16 h = (_Float16)xs;  // RNE
                    const _Float16 lo = (_Float16)(xs - (float)h);
                    std::memcpy(&part[0][ln][j], &h, 2);
                    std::memcpy(&part[1][ln][j], &lo, 2);
                  }
                }
              const uint16_t* pp = &part[0][0][0];
              stream.insert(stream.end(), pp, pp + NT * 64 * 8);
            }
    }
    // f16x2 sigmoid / softplus: the kernel feeds act(v) - C to every layer
    // after Dense_0 (act_tile_centered), so each such layer's bias takes
    // C * sum_k W[k][j] (fp64 sums, rounded once); the last layer's fold goes
    // into the permuted last bias below
    std::vector<double> lastfold;
    if (NT == 2 && (op.act == ZF_ACT_SIGMOID || op.act == ZF_ACT_SOFTPLUS)) {
      const double C = op.act == ZF_ACT_SIGMOID ? 0.5 : 0.69314718055994530942;
      for (int l = 1; l <= op.n_hidden; ++l) {
        const bool last = l == op.n_hidden;
        const int in = op.hidden[l - 1];
        const int out = last ? dt * Sr : op.hidden[l];
        const float* W = nat + op.off_w[l];
        std::vector<double> cs(out, 0.0);
        for (int k = 0; k < in; ++k)
          for (int j = 0; j < out; ++j) cs[j] += (double)W[(int64_t)k * out + j];
        if (last) {
          for (double& v : cs) v *= C;
          lastfold.swap(cs);
          continue;
        }
        for (int o = 0; o < T; ++o)
          for (int hh = 0; hh < 2; ++hh)
            for (int r = 0; r < 16; ++r) {
              const int ii = 32 * o + (r & 3) + 8 * (r >> 2) + 4 * hh;
              if (ii < out) {
                float& b = packed[d.b[l] + (o * 2 + hh) * 16 + r];
                b = (float)((double)b + C * cs[ii]);
              }
            }
      }
    }
    // f16x2: Dense_0 (fp32 fragments, d.w[0]) and the hidden biases of the
    // swished layers join the log2(e) prescale (act_swish); other
    // activations take their pre-activations unscaled.
    if (NT == 2 && op.act == ZF_ACT_SWISH) {
      const int KS0 = d.KS0;
      for (int64_t i = 0; i < (int64_t)T * KS0 * 64; ++i) packed[d.w[0] + i] *= kSwishPrescale;
      for (int l = 0; l < op.n_hidden; ++l)
        for (int64_t i = 0; i < (int64_t)T * 32; ++i) packed[d.b[l] + i] *= kSwishPrescale;
    }
    // f16x2 swish: the per-layer pre-activation bounds of x3_early_scale
    // (the prescaled weights and biases as the kernel multiplies them; fp64
    // row sums rounded up by a relative 2^-20, so the float bound holds)
    for (int l = 0; l < 16; ++l) d.x3_rb[l][0] = d.x3_rb[l][1] = 0.f;
    if (NT == 2 && op.act == ZF_ACT_SWISH) {
      const double pre = kSwishPrescale;
      for (int l = 0; l < op.n_hidden && l < 16; ++l) {
        const int in = l == 0 ? desc.dim - dt + desc.cond_dim : op.hidden[l - 1];
        const int out = op.hidden[l];
        const float* W = nat + op.off_w[l];
        const float* Bv = nat + op.off_b[l];
        double R = 0.0, Bm = 0.0;
        for (int j = 0; j < out; ++j) {
          double rs = 0.0;
          for (int k = 0; k < in; ++k) rs += std::fabs((double)W[(int64_t)k * out + j]);
          R = std::fmax(R, rs * pre);
          Bm = std::fmax(Bm, std::fabs((double)Bv[j]) * pre);
        }
        d.x3_rb[l][0] = (float)(R * (1.0 + 0x1p-20));
        d.x3_rb[l][1] = (float)(Bm * (1.0 + 0x1p-20));
      }
    }
    // group-0 pieces of this NSC (hidden group, or a last-layer group when it has no hidden streamed layer)
    d.x3_npieces[0] = d.x3_npieces[1] = (2 * (op.n_hidden > 1 ? T : TL) * NT * 1024) >> 10;  // own; fixed below
    // permuted last bias: [pair][o][lane half h][r] = bias[(2 pair + h) S + 16o + r]
    const float* B = nat + op.off_b[op.n_hidden];
    for (int pr = 0; pr < NP; ++pr)
      for (int o = 0; o < TL; ++o)
        for (int h = 0; h < 2; ++h)
          for (int r = 0; r < 16; ++r) {
            const int jp = one ? 32 * o + 16 * h + r : 16 * o + r, dd = one ? 0 : 2 * pr + h;
            float fill = 0.f;
            const int jr = (dd < dt && jp < S) ? x3_param_of(jp, K, Kr, &fill) : -1;
            float b = 0.f;
            if (jr >= 0)
              b = lastfold.empty() ? B[dd * Sr + jr] : (float)((double)B[dd * Sr + jr] + lastfold[dd * Sr + jr]);
            else if (dd < dt && jp < S)
              b = fill;  // inert padding knot
            packed[d.x3_blast + ((pr * TL + o) * 2 + h) * 16 + r] = b;
          }
  }
  // next-NSC copies (x3_npieces above held each op's own group-0 pieces)
  std::vector<int> own(desc.n_ops, 0);
  for (int i = 0; i < desc.n_ops; ++i) own[i] = desc.ops[i].kind == ZF_OP_NSC ? F.ops[i].x3_npieces[0] : 0;
  for (int i = 0; i < desc.n_ops; ++i) {
    if (desc.ops[i].kind != ZF_OP_NSC) continue;
    DevOp& d = F.ops[i];
    for (int dir = 0; dir < 2; ++dir) {
      const int n = d.x3_next[dir];
      d.x3_nbase[dir] = n >= 0 ? F.ops[n].x3 : -1;
      d.x3_nbn[dir] = n >= 0 ? F.ops[n].bn : 0;
      d.x3_npieces[dir] = n >= 0 ? own[n] : 0;
      d.x3_npar[dir] = n >= 0 ? F.ops[n].x3_par_pieces : 0;
    }
  }
}

// Weight-buffer tiles: the larger of a hidden group (T) and a last-layer
// group (x3_last_tiles*, one pass of the last layer).
int x3_buf_tiles(const zf_flow_desc& desc, int T, int K) {
  const int TL = desc.dim / 2 == 1 ? x3_last_tiles_one(K) : x3_last_tiles(K);
  return T > TL ? T : TL;
}

// TB = x3_buf_tiles; D = dim + cond_dim (the per-wave state holds x and c);
// par_bytes = DevFlow::x3_par_bytes
size_t x3_lds_bytes(int TB, int D, int NT, int par_bytes) {
  return (size_t)2 * 2 * TB * NT * 1024 + (size_t)2 * par_bytes + (size_t)kX3Waves * 32 * D * 4 +
         kX3Waves * sizeof(double);
}

int launch_flow_x3(const X3Launch& a, bool inverse) {
  if (a.NT != 2 && a.NT != 3) return einval("split-MFMA kernel: scheme %d", a.NT);
  if (a.K == 8) return launch_x3_k8(a, inverse);
  if (a.K == 16) return launch_x3_k16(a, inverse);
  if (a.K == 32) return launch_x3_k32(a, inverse);
  if (a.K == 64) return launch_x3_k64(a, inverse);
  return enotsup("split-MFMA kernel: knots not instantiated");
}

}  // namespace zf
