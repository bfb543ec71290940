// Two-set split-MFMA fused flow kernel (K4): the f16x2 scheme
// of flow_kernel_x3 (zf_flow_x3_kernel.h) at ONE wave per SIMD, each wave
// carrying TWO independent sets of 32 samples, so that the VALU-only work of
// one set runs inside the MFMA stream of the other.
//
// Why: the f16x2 kernel is VALU-issue-bound (per wave-coupling ≈ 1,450 VALU,
// 296 of them 8-cycle transcendentals, against 172 MFMAs of 32 cycles), and
// at three waves per SIMD the hardware overlaps one wave's VALU-only phases
// (spline, layer 0, layer boundaries) with another wave's MFMA phases only
// partly: two waves in MFMA phases at once leave the vector issue idle
// (r03 counters: matrix pipe 49%, vector issue 71%, both at once 27%).  Here
// one instruction stream holds both sets and the work is placed by hand:
//
//   phase X_n: set A streams NSC n's conditioner weights (layer 1 and last
//              layer group steps: 168 MFMAs at cfg2), and in the issue gaps
//              beside every MFMA set B runs its VALU-only chunk — the finish
//              + normalize_spline_params + bin search + RQ spline of NSC n-1,
//              the Rolls, then NSC n's layer 0 (BatchNorm + Dense_0 on fp32
//              MFMA), the f16x2 scale and the swish + split of its first tile;
//   phase Y_n: the same with the roles swapped (B streams NSC n, A runs its
//              spline of NSC n and layer 0 of NSC n+1).
//
// Each MFMA "slot" (one v_mfma_f32_32x32x16_f16 of the streaming set) is
// followed by that set's own share of the step's VALU (the split / swish
// modulo pipeline of x3_step_slots) and by the other set's chunk stages that
// fall into the slot (x4_vstage, spread evenly over the phase's slots),
// pinned by a scheduling barrier.  Weights are streamed through the same LDS
// double buffer as K3 (each NSC's groups once per set: the same L2 -> LDS
// bytes per sample); all small parameters (BatchNorm, Dense_0, biases, the
// permuted last bias, ShiftBounds rows) stay in LDS for the whole launch.
//
// Shapes: f16x2, every coupling swish with two hidden layers of width <= 128
// (T = 4), at most 2 transformed dims (no dim-pair loop), knots 8 / 16 (32:
// one transformed dim), conditioner inputs <= 4 (KS0 <= 2), only Rolls
// between couplings — every
// BASELINE config at hidden 128 (cfg1-cfg4) and the reference defaults at
// dim 2-5 (x4_eligible, zf_flow_x3.hip).  Rows: block b holds rows
// [256 b, 256 b + 256): set S of wave w the 32 rows 256 b + 128 S + 32 w +
// lane, so set S's NLL partial is K3's 128-row slot 2 b + S.
#pragma once
#include "zf_flow_x3_kernel.h"

namespace zf {
namespace {

#ifndef X4_ABL
#define X4_ABL 0  // tuning-only ablations (wrong results), never set in the shipped build
#endif

constexpr int kX4Waves = 4;                    // one wave per SIMD
constexpr int kX4Rows = kX4Waves * 2 * kTile;  // 256 rows per block

// One 32-sample set's registers.
template <int TL>
struct X4Set {
  floatx16 hb[4];    // layer input: pre-activations, swished tile by tile
  floatx16 acc[4];   // hidden layer (Dense_1) accumulators
  floatx16 pa[TL];   // last layer (Dense_2) accumulators
  halfx8 cs[2];      // split of (tile 0, k-step 0) of the next streamed layer
  float isc, us;     // f16x2 scales of the layer-1 input (x3_act_scale)
  float lus;         // unscale of the last layer's accumulators
  float ld;          // running log-det (Chain, bijectors.py:110)
  int rot;           // Roll as an index rotation of the state columns
  float* xs;         // this set's LDS state [D + C][32]
};

// The V set's chunk: scalars of the finished NSC (spline) and the next one
// (layer 0), in LDS float offsets (the small parameters sit at their blob
// offsets).
struct X4VC {
  long long blast;  // permuted last bias of the finished NSC
  int rdelta;       // Roll rotation between the finished NSC and the next (mod D)
  int dt, dc, DC;   // next NSC's geometry
  long long bn, w0, b0;
  int kw1;          // next NSC's layer-1 weight scale
};

// The M set's NSC: its streamed groups and hidden-layer constants.
struct X4MC {
  long long base;     // byte offset of group 0 in the x3 stream
  long long b1;       // hidden bias of Dense_1 (LDS float offset)
  int kw_last;        // last layer's weight scale
  long long next_base;  // group 0 of the next phase's NSC (-1: none)
};

// Working registers of the VALU chunk (the spline of one (sample, dim) per
// lane; ONE: the one dim on both lane halves, as K3).
template <int K, int TL>
struct X4V {
  float P[32 * TL];  // ONE: both halves' parameters after the exchange
  float w[K], hg[K];
  float sx, sy, ax, ay, bc;
  float xv, sxk, syk, sw, sh, lo, hi, xk, yk;
  float dk, dkp1, rw, sk, z, az, num, den, rd, yv, l;
  float ia, ib, ic;  // inverse quadratic
  floatx4 bq[3];     // bias quads read ahead of the finish
  float* xp;
  // layer 0
  float u[2], uv[2], bnm[2], bns[2], bnb[2];
  float w0f[4][2];
  float m;           // running max |pre-activation| (scale)
  float tq;          // swish temporary
  uint32_t csh[4];   // hi terms of the (0, 0) split
};

// Pin a value at this point of the program: the chunk stages are pure
// arithmetic, which instruction selection would otherwise sink to their
// first use (past the slots' scheduling barriers, into one block at the end
// of the phase).  An empty asm that takes the value keeps its computation in
// this slot (never used on loaded values: the asm would wait for the load).
__device__ __forceinline__ void x4_pin(float x) { asm volatile("" ::"v"(x)); }
__device__ __forceinline__ void x4_pin(const halfx8& x) { asm volatile("" ::"v"(x)); }

__device__ __forceinline__ float x4_lanes_max(float m) {
  // lanes l and l ^ 32 hold the same sample: v_permlane32_swap gives each
  // half the other's value in one instruction; m >= 0 (a max of |v|), so
  // the larger bit pattern is the larger float (no NaN canonicalisation)
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
  return __uint_as_float(r[0] > r[1] ? r[0] : r[1]);
}

// x for the lower / upper lane half: {value of half 0, value of half 1} on
// every lane.
__device__ __forceinline__ void x4_halves(float x, float& h0, float& h1) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  h0 = __uint_as_float(r[0]);
  h1 = __uint_as_float(r[1]);
}

// ---------------------------------------------------------------------------
// The VALU chunk as numbered stages (each a few instructions; their order is
// the program order of the computation).  Stage counts by part:
template <int K, bool ONE, bool INV, int KS0, int TL, bool VSPL, bool VL0>
struct X4Stages {
  static constexpr int nFIN = VSPL ? 4 * TL : 0;  // finish: 4 values of one last-layer tile each
  static constexpr int nSPW = VSPL ? K : 0;       // squareplus of the widths (+ running sum)
  // ONE at K = 16: the widths sit on lane half 0 and the heights on half 1
  // (tile 0), so each half normalises its own 16 and one exchange per knot
  // gives both halves both (SPW covers both, no SPH)
  static constexpr bool kSplitWH = ONE && K == 16;
  static constexpr int nSPH = (VSPL && !kSplitWH) ? K : 0;  // heights
  static constexpr int nNR0 = VSPL ? 1 : 0;       // the two normalisers
  static constexpr int nNRM = VSPL ? K : 0;       // normalised widths / heights
  static constexpr int nBS0 = VSPL ? 1 : 0;       // bin-search start
  static constexpr int nBS = VSPL ? K - 1 : 0;    // one knot each
  static constexpr int nBSF = VSPL ? 1 : 0;       // the idx == K sliver
  static constexpr int nEV = VSPL ? 4 : 0;        // RQ forward / inverse
  static constexpr int nWR = VSPL ? 1 : 0;        // state write, log-det, Rolls
  static constexpr int nL0R = VL0 ? 1 : 0;        // layer-0 reads
  static constexpr int nL0B = VL0 ? 4 : 0;        // bias tiles into the accumulators
  static constexpr int nL0U = VL0 ? 1 : 0;        // BatchNorm'd inputs
  static constexpr int nL0M = VL0 ? 4 * KS0 : 0;  // fp32 MFMAs
  static constexpr int nSC = VL0 ? 8 : 0;         // max |v| over 8 values each
  static constexpr int nSCF = VL0 ? 1 : 0;        // the scales
  static constexpr int nSW = VL0 ? 16 : 0;        // swish of tile 0, one value each
  static constexpr int nSP = VL0 ? 2 : 0;         // split (0, 0): hi, lo
  static constexpr int oFIN = 0;
  static constexpr int oSPW = oFIN + nFIN;
  static constexpr int oSPH = oSPW + nSPW;
  static constexpr int oNR0 = oSPH + nSPH;
  static constexpr int oNRM = oNR0 + nNR0;
  static constexpr int oBS0 = oNRM + nNRM;
  static constexpr int oBS = oBS0 + nBS0;
  static constexpr int oBSF = oBS + nBS;
  static constexpr int oEV = oBSF + nBSF;
  static constexpr int oWR = oEV + nEV;
  static constexpr int oL0R = oWR + nWR;
  static constexpr int oL0B = oL0R + nL0R;
  static constexpr int oL0U = oL0B + nL0B;
  static constexpr int oL0M = oL0U + nL0U;
  static constexpr int oSC = oL0M + nL0M;
  static constexpr int oSCF = oSC + nSC;
  static constexpr int oSW = oSCF + nSCF;
  static constexpr int oSP = oSW + nSW;
  static constexpr int N = oSP + nSP;
};

struct X4Ctx {
  const float* par;  // LDS copy of the small parameters (blob floats [0, small_floats))
  int lane, s, hh, D, C;
  float rnorm, cnorm;  // softmax_with_threshold constants (KnotConsts)
};

// Parameter j of this lane's (sample, dim) row: the last-layer accumulators
// in place (two dims: lane half h holds dim h's 16 per tile), or the
// exchanged copy (ONE).
template <int K, bool ONE, int TL, int J>
__device__ __forceinline__ float x4_P(const X4Set<TL>& V, const X4V<K, TL>& v) {
  if constexpr (ONE) return v.P[J];
  else return V.pa[J / 16][J % 16];
}

template <int I, int K, bool ONE, bool INV, int KS0, int TL, bool VSPL, bool VL0>
__device__ __forceinline__ void x4_vstage(const X4Ctx& cx, X4Set<TL>& V, X4V<K, TL>& v, const X4VC& vc) {
  using St = X4Stages<K, ONE, INV, KS0, TL, VSPL, VL0>;
  constexpr bool FWD = !INV;
  constexpr int S3 = 3 * K - 1;
  (void)S3;
  if constexpr (I >= St::oFIN && I < St::oFIN + St::nFIN) {
    // finish of the last layer (acc * lus + bias, K3's x3_finish), four
    // values of tile o per stage; the bias quad is read two stages ahead
    constexpr int q = I - St::oFIN, o = q / 4, r4 = q % 4;
    const float* bl = cx.par + vc.blast + cx.hh * 16;
    if constexpr (q == 0) {
      v.bq[0] = *reinterpret_cast<const floatx4*>(bl);
      if constexpr (St::nFIN > 1) v.bq[1] = *reinterpret_cast<const floatx4*>(bl + 4);
    }
    if constexpr (q + 2 < St::nFIN) {
      constexpr int q2 = q + 2;
      v.bq[q2 % 3] = *reinterpret_cast<const floatx4*>(bl + (q2 / 4) * 32 + 4 * (q2 % 4));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float f = __builtin_fmaf(V.pa[o][4 * r4 + i], V.lus, v.bq[q % 3][i]);
      if constexpr (St::kSplitWH) {
        if constexpr (o == 0) {  // widths (half 0) / heights (half 1): normalised per half first
          V.pa[0][4 * r4 + i] = f;
          x4_pin(f);
        } else {  // slopes (half 0) to both halves
          float h1;
          x4_halves(f, v.P[32 + 4 * r4 + i], h1);
          x4_pin(v.P[32 + 4 * r4 + i]);
        }
      } else if constexpr (ONE) {
        // both halves get the whole row (tile o, half h, register r =
        // parameter 32 o + 16 h + r)
        x4_halves(f, v.P[32 * o + 4 * r4 + i], v.P[32 * o + 16 + 4 * r4 + i]);
        x4_pin(v.P[32 * o + 4 * r4 + i]);
        x4_pin(v.P[32 * o + 16 + 4 * r4 + i]);
      } else {
        V.pa[o][4 * r4 + i] = f;
        x4_pin(f);
      }
    }
  } else if constexpr (I >= St::oSPW && I < St::oSPW + St::nSPW && St::kSplitWH) {
    // half 0: width j, half 1: height j; the running sum is sx on half 0, sy on half 1
    constexpr int j = I - St::oSPW;
    v.w[j] = x3_squareplus2(V.pa[0][j]);
    v.sx = j == 0 ? v.w[0] : v.sx + v.w[j];
    x4_pin(v.w[j]);
    x4_pin(v.sx);
  } else if constexpr (I >= St::oSPW && I < St::oSPW + St::nSPW) {
    constexpr int j = I - St::oSPW;
    v.w[j] = x3_squareplus2(x4_P<K, ONE, TL, j>(V, v));
    v.sx = j == 0 ? v.w[0] : v.sx + v.w[j];
    x4_pin(v.w[j]);
    x4_pin(v.sx);
  } else if constexpr (I >= St::oSPH && I < St::oSPH + St::nSPH) {
    constexpr int j = I - St::oSPH;
    v.hg[j] = x3_squareplus2(x4_P<K, ONE, TL, K + j>(V, v));
    v.sy = j == 0 ? v.hg[0] : v.sy + v.hg[j];
    x4_pin(v.hg[j]);
    x4_pin(v.sy);
  } else if constexpr (I == St::oNR0 && VSPL) {
    v.ax = rcp_refined(v.sx) * cx.rnorm;
    if constexpr (!St::kSplitWH) v.ay = rcp_refined(v.sy) * cx.rnorm;
    v.bc = cx.cnorm * cx.rnorm;
    x4_pin(v.ax);
    if constexpr (!St::kSplitWH) x4_pin(v.ay);
    // this lane's x (two dims: dim hh; ONE: dim 0 on both halves)
    v.xp = V.xs + wrap((ONE ? 0 : cx.hh) + V.rot, cx.D) * 32 + cx.s;
    v.xv = *v.xp;
  } else if constexpr (I >= St::oNRM && I < St::oNRM + St::nNRM && St::kSplitWH) {
    // normalise on the owning half, then the exchange: width j and height j on both halves
    constexpr int j = I - St::oNRM;
    const float f = __builtin_fmaf(v.w[j], v.ax, v.bc);
    x4_halves(f, v.w[j], v.hg[j]);
    x4_pin(v.w[j]);
    x4_pin(v.hg[j]);
  } else if constexpr (I >= St::oNRM && I < St::oNRM + St::nNRM) {
    constexpr int j = I - St::oNRM;
    v.w[j] = __builtin_fmaf(v.w[j], v.ax, v.bc);
    v.hg[j] = __builtin_fmaf(v.hg[j], v.ay, v.bc);
    x4_pin(v.w[j]);
    x4_pin(v.hg[j]);
  } else if constexpr (I == St::oBS0 && VSPL) {
    // rqs_bin_monotone: knot 0 latched up front
    v.sxk = 0.f; v.syk = 0.f; v.sw = v.w[0]; v.sh = v.hg[0];
    v.lo = 0.f; v.hi = x4_P<K, ONE, TL, 2 * K>(V, v);
    v.xk = v.w[0]; v.yk = v.hg[0];
  } else if constexpr (I >= St::oBS && I < St::oBS + St::nBS) {
    constexpr int j = I - St::oBS + 1;
    const bool c = (FWD ? v.xk : v.yk) <= v.xv;
    v.sxk = c ? v.xk : v.sxk;
    v.syk = c ? v.yk : v.syk;
    v.sw = c ? v.w[j] : v.sw;
    v.sh = c ? v.hg[j] : v.sh;
    v.lo = c ? x4_P<K, ONE, TL, 2 * K + j - 1>(V, v) : v.lo;
    if constexpr (j + 1 < K) v.hi = c ? x4_P<K, ONE, TL, 2 * K + j>(V, v) : v.hi;
    else v.hi = c ? 0.f : v.hi;
    v.xk = v.xk + v.w[j];
    v.yk = v.yk + v.hg[j];
    x4_pin(v.sxk); x4_pin(v.syk); x4_pin(v.sw); x4_pin(v.sh);
    x4_pin(v.lo); x4_pin(v.hi); x4_pin(v.xk); x4_pin(v.yk);
  } else if constexpr (I == St::oBSF && VSPL) {
    const bool c = (FWD ? v.xk : v.yk) <= v.xv;
    v.sxk = c ? v.xk : v.sxk;
    v.syk = c ? v.yk : v.syk;
    v.sw = c ? qnan() : v.sw;
    v.sh = c ? qnan() : v.sh;
    v.lo = c ? 0.f : v.lo;
    v.hi = c ? qnan() : v.hi;
    x4_pin(v.sxk); x4_pin(v.syk); x4_pin(v.sw); x4_pin(v.sh); x4_pin(v.lo); x4_pin(v.hi);
  } else if constexpr (I >= St::oEV && I < St::oEV + St::nEV) {
    constexpr int e = I - St::oEV;
    if constexpr (FWD) {  // x3_forward_eval in four stages
      if constexpr (e == 0) {
        v.dk = v.lo == 0.f ? 1.f : x3_squareplus(v.lo);
        v.dkp1 = v.hi == 0.f ? 1.f : x3_squareplus(v.hi);
        v.rw = rcp_refined(v.sw);
        x4_pin(v.dk); x4_pin(v.dkp1); x4_pin(v.rw);
      } else if constexpr (e == 1) {
        v.sk = v.sh * v.rw;
        const float zr = (v.xv - v.sxk) * v.rw;  // utils.py:122
        v.z = (zr != zr) ? zr : fminf(fmaxf(zr, kEps), kOneMinusEps);
        v.az = 1.0f - v.z;
        x4_pin(v.sk); x4_pin(v.z); x4_pin(v.az);
      } else if constexpr (e == 2) {
        v.num = v.sh * v.z * (v.sk * v.z + v.dk * v.az);                 // :125
        v.den = v.sk + (v.dkp1 + v.dk - 2.0f * v.sk) * v.z * v.az;      // :126
        v.rd = rcp_refined(v.den + kEps);
        x4_pin(v.num); x4_pin(v.den); x4_pin(v.rd);
      } else {
        const bool oob = (v.xv < 0.f) || (v.xv >= 1.f);
        const float yv = v.syk + v.num * v.rd;                                    // :127
        v.yv = oob ? v.xv : yv;                                                   // :130
        const float num2 = v.z * (v.dkp1 * v.z + 2.0f * v.sk * v.az) + v.dk * (v.az * v.az);  // :133
        const float sq = (v.sk + kEps) * v.rd;
        const float l = __logf((num2 + kEps) * (sq * sq));
        v.l = oob ? 0.0f : l;                                                     // :138
        x4_pin(v.yv); x4_pin(v.l);
      }
    } else {  // rqs_inverse_eval (utils.py:191-201)
      if constexpr (e == 0) {
        v.dk = v.lo == 0.f ? 1.f : x3_squareplus(v.lo);
        v.dkp1 = v.hi == 0.f ? 1.f : x3_squareplus(v.hi);
        x4_pin(v.dk); x4_pin(v.dkp1);
      } else if constexpr (e == 1) {
        v.sk = v.sh / v.sw;
        x4_pin(v.sk);
      } else if constexpr (e == 2) {
        const float dy = v.xv - v.syk;
        const float t = v.dkp1 + v.dk - 2.0f * v.sk;
        v.ia = v.sh * (v.sk - v.dk) + dy * t;  // :193
        v.ib = v.sh * v.dk - dy * t;           // :194
        v.ic = -v.sk * dy;                     // :195
        x4_pin(v.ia); x4_pin(v.ib); x4_pin(v.ic);
      } else {
        const float zq = 2.0f * v.ic / (-v.ib - __builtin_sqrtf(v.ib * v.ib - 4.0f * v.ia * v.ic));  // :197
        const float xq = zq * v.sw + v.sxk;   // :198
        const bool oob = (v.xv < 0.f) || (v.xv >= 1.f);
        v.yv = oob ? v.xv : xq;               // :201
        x4_pin(v.yv);
      }
    }
  } else if constexpr (I == St::oWR && VSPL) {
    const bool dact = ONE ? cx.hh == 0 : true;  // ONE: the upper half idles
    if (dact) *v.xp = v.yv;
    if constexpr (FWD) {
      // this coupling's log-det in dim order (utils.py:139), then Chain's +=
      float d0, d1;
      x4_halves(dact ? v.l : 0.f, d0, d1);
      float ldn = 0.f + d0;
      if constexpr (!ONE) ldn = ldn + d1;
      V.ld = V.ld + ldn;
    }
    V.rot = pmod(V.rot + vc.rdelta, cx.D);
    if constexpr (FWD) x4_pin(V.ld);
  } else if constexpr (I == St::oL0R && VL0) {
    // Dense_0 fragments, BatchNorm rows and the raw inputs of this lane's k
    const int DCp = 2 * KS0;
    const float* bn = cx.par + vc.bn;
#pragma unroll
    for (int ks = 0; ks < KS0; ++ks) {
      const int k = 2 * ks + cx.hh;
      const int col = k < vc.dc ? wrap(vc.dt + k + V.rot, cx.D) : (k < vc.DC ? cx.D + k - vc.dc : 0);
      const float raw = V.xs[col * 32 + cx.s];
      v.uv[ks] = k < vc.DC ? raw : 0.f;
      v.bnm[ks] = bn[k];
      v.bns[ks] = bn[DCp + k];
      v.bnb[ks] = bn[2 * DCp + k];
#pragma unroll
      for (int o = 0; o < 4; ++o) v.w0f[o][ks] = cx.par[vc.w0 + (o * KS0 + ks) * 64 + cx.lane];
    }
  } else if constexpr (I >= St::oL0B && I < St::oL0B + St::nL0B) {
    constexpr int o = I - St::oL0B;
    V.hb[o] = bias_acc(cx.par + vc.b0 + o * 32, cx.hh);
  } else if constexpr (I == St::oL0U && VL0) {
#pragma unroll
    for (int ks = 0; ks < KS0; ++ks) {
      v.u[ks] = (v.uv[ks] - v.bnm[ks]) * v.bns[ks] + v.bnb[ks];
      x4_pin(v.u[ks]);
    }
  } else if constexpr (I >= St::oL0M && I < St::oL0M + St::nL0M) {
    constexpr int q = I - St::oL0M, ks = q / 4, o = q % 4;
    V.hb[o] = __builtin_amdgcn_mfma_f32_32x32x2f32(v.w0f[o][ks], v.u[ks], V.hb[o], 0, 0, 0);
  } else if constexpr (I >= St::oSC && I < St::oSC + St::nSC) {
    // x3_act_scale's max |v'| over the layer-1 input, 8 values per stage
    constexpr int q = I - St::oSC, o = q / 2, r0 = 8 * (q % 2);
    float m = q == 0 ? 0.f : v.m;
#pragma unroll
    for (int r = 0; r < 8; ++r) m = fmaxf(m, fabsf(V.hb[o][r0 + r]));
    v.m = m;
    x4_pin(m);
  } else if constexpr (I == St::oSCF && VL0) {
    const float m = x4_lanes_max(v.m);
    const int e = max(__builtin_amdgcn_frexp_expf(m), -60);
    V.isc = __builtin_amdgcn_ldexpf(kSwishPrescale, e - 14);
    V.us = __builtin_amdgcn_ldexpf(1.0f, e - 14 - vc.kw1);
    x4_pin(V.isc);
    x4_pin(V.us);
  } else if constexpr (I >= St::oSW && I < St::oSW + St::nSW) {
    constexpr int r = I - St::oSW;
    V.hb[0][r] = act_swish<2>(V.hb[0][r], V.isc);
    x4_pin(V.hb[0][r]);
  } else if constexpr (I == St::oSP && VL0) {
    split8h_hi<0>(V.hb[0], v.csh);
#pragma unroll
    for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(v.csh[i]));
  } else if constexpr (I == St::oSP + 1 && VL0) {
    split8h_lo<0>(V.hb[0], v.csh, V.cs[0], V.cs[1]);
    x4_pin(V.cs[0]);
    x4_pin(V.cs[1]);
  }
}

template <int K, bool ONE, bool INV, int KS0, int TL, bool VSPL, bool VL0, int... I>
__device__ __forceinline__ void x4_vstages(std::integer_sequence<int, I...>, const X4Ctx& cx, X4Set<TL>& V,
                                           X4V<K, TL>& v, const X4VC& vc, int base) {
  (x4_vstage<I, K, ONE, INV, KS0, TL, VSPL, VL0>(cx, V, v, vc), ...);
}

template <int B, int E, int K, bool ONE, bool INV, int KS0, int TL, bool VSPL, bool VL0>
__device__ __forceinline__ void x4_vrange(const X4Ctx& cx, X4Set<TL>& V, X4V<K, TL>& v, const X4VC& vc) {
  if constexpr (B < E) {
    x4_vstage<B, K, ONE, INV, KS0, TL, VSPL, VL0>(cx, V, v, vc);
    x4_vrange<B + 1, E, K, ONE, INV, KS0, TL, VSPL, VL0>(cx, V, v, vc);
  }
}

// ---------------------------------------------------------------------------
// The M set's group steps.

struct X4Pipe {
  char* cur;   // LDS buffer of the group computed next
  char* nxt;   // the other buffer (prefetch target)
  int wave, lane;
};

// DMA the group after group g of the M set's NSC (groups 0-3: Dense_1, 4-7:
// the last layer), or the next phase's group 0.
template <int TL>
__device__ __forceinline__ void x4_issue_next(const char* __restrict__ x3, const X4Pipe& p, const X4MC& mc, int g) {
  constexpr int kHid = group_bytes<2>(4), kLast = group_bytes<2>(TL);
  const int n = g + 1;
  long long off;
  int pieces;
  if (n < 4) {
    off = mc.base + (long long)n * kHid;
    pieces = kHid >> 10;
  } else if (n < 8) {
    off = mc.base + 4LL * kHid + (long long)(n - 4) * kLast;
    pieces = kLast >> 10;
  } else {
    if (mc.next_base < 0) return;
    off = mc.next_base;
    pieces = kHid >> 10;
  }
  for (int q = p.wave; q < pieces; q += kX4Waves)
    __builtin_amdgcn_global_load_lds((const void*)(x3 + off + (q << 10) + p.lane * 16),
                                     (__attribute__((address_space(3))) void*)(p.nxt + (q << 10)), 16, 0, 0);
}

// Slot m of group step Q (NOUT output tiles): one MFMA term of the M set
// (x3_slot), its own VALU share (x3_valu_slot: split of (Q, 1), the swish
// modulo pipeline of tile Q + 1, split of (Q + 1, 0)), then the V set's
// chunk stages [VB, VE), then a scheduling barrier.
template <int NOUT, int Q, int m, int VB, int VE, int K, bool ONE, bool INV, int KS0, int TL, bool VSPL, bool VL0>
__device__ __forceinline__ void x4_slot(const char* lb, floatx16 (&hb)[4], floatx16 (&acc)[NOUT], halfx8 (&fr)[2][2],
                                        halfx8 (&cs)[2], halfx8 (&s1)[2], float (&tq)[4], uint32_t (&s1h)[4],
                                        uint32_t (&csh)[4], float c, const X4Ctx& cx, X4Set<TL>& V, X4V<K, TL>& v,
                                        const X4VC& vc) {
  constexpr int t = m / 3, j = m % 3, ks = t / NOUT, o = t % NOUT;
#if X4_ABL != 3  // tuning ablation 3: one A fragment per group step (wrong results)
  if constexpr (j == 0 && t + 1 < 2 * NOUT) load_frag<2>(lb + (((t + 1) * 2) << 10), fr[(t + 1) & 1]);
#else
  if constexpr (j == 0 && t == 0) { fr[1][0] = fr[0][0]; fr[1][1] = fr[0][1]; }
#endif
  if constexpr (ks == 0) acc[o] = mfma_term2(fr[t & 1], cs, j, acc[o]);
  else acc[o] = mfma_term2(fr[t & 1], s1, j, acc[o]);
#if X4_ABL != 4  // tuning ablation 4: no M-set VALU in the slots (wrong results)
  x3_valu_slot<4, NOUT, Q, m>(hb, cs, s1, tq, s1h, csh, c);
#endif
#if X4_ABL != 1  // tuning ablation 1: no V chunk in the phases (wrong results)
  x4_vrange<VB, VE, K, ONE, INV, KS0, TL, VSPL, VL0>(cx, V, v, vc);
#endif
  __builtin_amdgcn_sched_barrier(0);
}

template <int NOUT, int Q, int G0, int NS, int K, bool ONE, bool INV, int KS0, int TL, bool VSPL, bool VL0, int... M>
__device__ __forceinline__ void x4_slots(std::integer_sequence<int, M...>, const char* lb, floatx16 (&hb)[4],
                                         floatx16 (&acc)[NOUT], halfx8 (&fr)[2][2], halfx8 (&cs)[2], halfx8 (&s1)[2],
                                         float (&tq)[4], uint32_t (&s1h)[4], uint32_t (&csh)[4], float c,
                                         const X4Ctx& cx, X4Set<TL>& V, X4V<K, TL>& v, const X4VC& vc) {
  using St = X4Stages<K, ONE, INV, KS0, TL, VSPL, VL0>;
  (x4_slot<NOUT, Q, M, (G0 + M) * St::N / NS, (G0 + M + 1) * St::N / NS, K, ONE, INV, KS0, TL, VSPL, VL0>(
       lb, hb, acc, fr, cs, s1, tq, s1h, csh, c, cx, V, v, vc),
   ...);
}

// One group step of the M set: wait for the group's DMA, block barrier,
// prefetch the next group, then 2 x NOUT x 3 slots.  G0 = index of the
// step's first slot in the phase (the V chunk is spread over NS slots).
template <int NOUT, int Q, int G0, int NS, int K, bool ONE, bool INV, int KS0, int TL, bool VSPL, bool VL0>
__device__ __forceinline__ void x4_step(const char* __restrict__ x3, X4Pipe& p, const X4MC& mc, int g,
                                        floatx16 (&hb)[4], floatx16 (&acc)[NOUT], halfx8 (&cs)[2], float c,
                                        const X4Ctx& cx, X4Set<TL>& V, X4V<K, TL>& v, const X4VC& vc) {
#if X4_ABL != 2  // tuning ablation 2: no per-group DMA wait / barrier (wrong results)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#endif
  x4_issue_next<TL>(x3, p, mc, g);
  const char* lb = p.cur + p.lane * 16;
  halfx8 fr[2][2];
  load_frag<2>(lb, fr[0]);
  halfx8 s1[2];
  float tq[4];
  uint32_t s1h[4], csh[4];
  constexpr int kSlots = 2 * NOUT * 3;
  x4_slots<NOUT, Q, G0, NS, K, ONE, INV, KS0, TL, VSPL, VL0>(std::make_integer_sequence<int, kSlots>{}, lb, hb, acc,
                                                              fr, cs, s1, tq, s1h, csh, c, cx, V, v, vc);
  // the M set's stages that did not fit in the slots (small groups)
  x3_valu_tail<4, NOUT, Q>(std::make_integer_sequence<int, (kSlots < 20 ? 20 - kSlots : 0)>{}, hb, cs, s1, tq, s1h,
                           csh, c);
  char* const t = p.cur;
  p.cur = p.nxt;
  p.nxt = t;
}

template <int NOUT, int Q, int GB, int NS, int K, bool ONE, bool INV, int KS0, int TL, bool VSPL, bool VL0>
__device__ __forceinline__ void x4_layer(const char* __restrict__ x3, X4Pipe& p, const X4MC& mc, int g0,
                                         floatx16 (&hb)[4], floatx16 (&acc)[NOUT], halfx8 (&cs)[2], float c,
                                         const X4Ctx& cx, X4Set<TL>& V, X4V<K, TL>& v, const X4VC& vc) {
  x4_step<NOUT, Q, GB + Q * 6 * NOUT, NS, K, ONE, INV, KS0, TL, VSPL, VL0>(x3, p, mc, g0 + Q, hb, acc, cs, c, cx, V,
                                                                          v, vc);
  if constexpr (Q + 1 < 4)
    x4_layer<NOUT, Q + 1, GB, NS, K, ONE, INV, KS0, TL, VSPL, VL0>(x3, p, mc, g0, hb, acc, cs, c, cx, V, v, vc);
}

// One phase: the M set streams its NSC (Dense_1 then the last layer), the V
// set runs its chunk in the slots.
template <int K, bool ONE, bool INV, int KS0, int TL, bool VSPL, bool VL0>
__device__ __forceinline__ void x4_phase(const char* __restrict__ x3, X4Pipe& p, const X4MC& mc, const X4Ctx& cx,
                                         X4Set<TL>& M, X4Set<TL>& V, X4V<K, TL>& v, const X4VC& vc) {
  constexpr int NS = 24 * 4 + 6 * TL * 4;  // MFMA slots of the phase
  // Dense_1: zero-seeded, one fma per value at the end (acc * us + bias)
#pragma unroll
  for (int o = 0; o < 4; ++o) M.acc[o] = floatx16{0};
  x4_layer<4, 0, 0, NS, K, ONE, INV, KS0, TL, VSPL, VL0>(x3, p, mc, 0, M.hb, M.acc, M.cs, M.isc, cx, V, v, vc);
  {
    const float* bl = cx.par + mc.b1;
    floatx16 bt = bias_acc(bl, cx.hh);
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      floatx16 bn;
      if (o + 1 < 4) bn = bias_acc(bl + (o + 1) * 32, cx.hh);
      M.hb[o] = x3_finish<2>(M.acc[o], M.us, bt);
      if (o + 1 < 4) bt = bn;
    }
  }
  // the last layer's input: scale, swish of tile 0, split (0, 0)
  float lisc, lius;
  x3_act_scale<4>(M.hb, mc.kw_last, lisc, M.lus, lius);
  x3_act_tile<2, false>(M.hb[0], lisc, ZF_ACT_SWISH);
  split8h<0>(M.hb[0], M.cs[0], M.cs[1]);
#pragma unroll
  for (int o = 0; o < TL; ++o) M.pa[o] = floatx16{0};
  x4_layer<TL, 0, 96, NS, K, ONE, INV, KS0, TL, VSPL, VL0>(x3, p, mc, 4, M.hb, M.pa, M.cs, lisc, cx, V, v, vc);
}

// A set's chunk with nothing to overlap (the first layer 0, the last spline).
template <int K, bool ONE, bool INV, int KS0, int TL, bool VSPL, bool VL0>
__device__ __forceinline__ void x4_chunk(const X4Ctx& cx, X4Set<TL>& V, X4V<K, TL>& v, const X4VC& vc) {
  using St = X4Stages<K, ONE, INV, KS0, TL, VSPL, VL0>;
  x4_vrange<0, St::N, K, ONE, INV, KS0, TL, VSPL, VL0>(cx, V, v, vc);
}

// The next NSC at or after exec position q, and the Roll rotation up to it
// (only Rolls may sit between NSCs: x4_eligible).  Returns its op index or -1.
template <bool INV>
__device__ __forceinline__ int x4_next_nsc(const DevFlow* __restrict__ F, int op_begin, int op_end, int& q, int D,
                                           int& rdelta) {
  const int nq = op_end - op_begin;
  rdelta = 0;
  for (; q < nq; ++q) {
    const int oi = INV ? (op_end - 1 - q) : (op_begin + q);
    const int kind = F->ops[oi].kind;
    if (kind == ZF_OP_NSC) return oi;
    if (kind == ZF_OP_ROLL) rdelta = pmod(INV ? rdelta + F->ops[oi].shift : rdelta - F->ops[oi].shift, D);
  }
  return -1;
}

template <bool INV>
__device__ __forceinline__ void x4_fill_vc(const DevOp& op, X4VC& vc) {
  vc.dt = op.dt; vc.dc = op.dc; vc.DC = op.DC;
  vc.bn = op.bn; vc.w0 = op.w[0]; vc.b0 = op.b[0];
  vc.kw1 = op.x3_kw[1];
}

template <int TL>
__device__ __forceinline__ void x4_fill_mc(const DevOp& op, X4MC& mc) {
  mc.base = op.x3;
  mc.b1 = op.b[1];
  mc.kw_last = op.x3_kw[2];
}

// Non-NSC ops outside the NSC pipeline (leading / trailing: ShiftBounds, Roll).
template <bool INV, int TL>
__device__ __forceinline__ void x4_plain_op(const DevOp& op, const float* sb_lds, X4Set<TL>& S, int s, int hh, int D) {
  if (op.kind == ZF_OP_ROLL) {
    S.rot = pmod(INV ? S.rot + op.shift : S.rot - op.shift, D);
  } else if (op.kind == ZF_OP_SHIFT_BOUNDS) {
    shift_bounds_op<INV>(sb_lds, S.xs, s, hh, S.rot, D, S.ld);
  }
}

template <int K, bool ONE, bool INV, int KS0>
__global__ __launch_bounds__(kX4Waves * 64, 1) void flow_kernel_x4(
    const DevFlow* __restrict__ F, const float* __restrict__ blob, const char* __restrict__ x3,
    const float* __restrict__ xin, const float* __restrict__ cin, float* __restrict__ y_out,
    const float* __restrict__ ld_in, float* __restrict__ ld_out, float* __restrict__ lp_out,
    double* __restrict__ block_partial, long long nparts, int op_begin, int op_end, long long N,
    unsigned long long seed, int gen, int small_pieces) {
  constexpr int TL = ONE ? (3 * K - 1 + 31) / 32 : (3 * K - 1 + 15) / 16;
  constexpr int kBuf = group_bytes<2>(4 > TL ? 4 : TL);
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int D = F->D;
  const int C = F->C;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int s = lane & 31;
  const int hh = lane >> 5;
  const int DS = D + C;
  // LDS: [2][kBuf] weight groups | small parameters | [2 sets][4 waves][DS][32] state | [2][4] partials
  char* par_lds = lds + 2 * kBuf;
  float* xs0 = reinterpret_cast<float*>(par_lds + (small_pieces << 10));
  double* s_part = reinterpret_cast<double*>(xs0 + 2 * kX4Waves * 32 * DS);

  X4Ctx cx;
  cx.par = reinterpret_cast<const float*>(par_lds);
  cx.lane = lane; cx.s = s; cx.hh = hh; cx.D = D; cx.C = C;
  {
    const KnotConsts kc(F->kreal);
    cx.rnorm = kc.rnorm;
    cx.cnorm = kc.c;
  }
  X4Set<TL> A, B;
  const long long rowA = (long long)blockIdx.x * kX4Rows + wave * kTile + s;
  const long long rowB = rowA + kX4Waves * kTile;
  const bool validA = rowA < N, validB = rowB < N;
  A.xs = xs0 + wave * (32 * DS);
  B.xs = xs0 + (kX4Waves + wave) * (32 * DS);
  load_state(A.xs, xin, rowA, validA, D, s, hh, F, seed, INV ? gen : 0);
  load_state(B.xs, xin, rowB, validB, D, s, hh, F, seed, INV ? gen : 0);
  for (int j = hh; j < C; j += 2) {
    A.xs[(D + j) * 32 + s] = validA ? cin[rowA * C + j] : 0.f;
    B.xs[(D + j) * 32 + s] = validB ? cin[rowB * C + j] : 0.f;
  }
  A.ld = (ld_in != nullptr && validA) ? ld_in[rowA] : 0.f;
  B.ld = (ld_in != nullptr && validB) ? ld_in[rowB] : 0.f;
  A.rot = 0;
  B.rot = 0;
  A.lus = B.lus = 1.f;
  A.isc = B.isc = A.us = B.us = 1.f;

  X4Pipe pipe;
  pipe.cur = lds;
  pipe.nxt = lds + kBuf;
  pipe.wave = wave;
  pipe.lane = lane;
  // every small parameter into LDS, and group 0 of the first NSC
  for (int q = wave; q < small_pieces; q += kX4Waves)
    __builtin_amdgcn_global_load_lds((const void*)(reinterpret_cast<const char*>(blob) + (q << 10) + lane * 16),
                                     (__attribute__((address_space(3))) void*)(par_lds + (q << 10)), 16, 0, 0);
  int q = 0;
  const int nq = op_end - op_begin;
  // leading non-NSC ops (ShiftBounds, Roll), on both sets
  int first;
  {
    int qq = 0;
    for (; qq < nq; ++qq) {
      const int oi = INV ? (op_end - 1 - qq) : (op_begin + qq);
      if (F->ops[oi].kind == ZF_OP_NSC) break;
    }
    first = qq < nq ? (INV ? (op_end - 1 - qq) : (op_begin + qq)) : -1;
    if (first >= 0) {
      const int pieces = group_bytes<2>(4) >> 10;
      for (int p = wave; p < pieces; p += kX4Waves)
        __builtin_amdgcn_global_load_lds((const void*)(x3 + F->ops[first].x3 + (p << 10) + lane * 16),
                                         (__attribute__((address_space(3))) void*)(pipe.cur + (p << 10)), 16, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (; q < nq; ++q) {
    const int oi = INV ? (op_end - 1 - q) : (op_begin + q);
    const DevOp& op = F->ops[oi];
    if (op.kind == ZF_OP_NSC) break;
    const float* sb = cx.par + op.sb;
    x4_plain_op<INV>(op, sb, A, s, hh, D);
    x4_plain_op<INV>(op, sb, B, s, hh, D);
  }
  X4V<K, TL> va, vb;
  if (first >= 0) {
    X4VC vc;
    x4_fill_vc<INV>(F->ops[first], vc);
    vc.blast = 0;
    vc.rdelta = 0;
    wave_lds_sync();
    // set A: layer 0 of the first NSC, nothing to overlap
    x4_chunk<K, ONE, INV, KS0, TL, false, true>(cx, A, va, vc);
    int n = first;
    ++q;  // past the first NSC
    bool has_prev = false;
    long long prev_blast = 0;
    int prev_rd = 0;
    for (;;) {
      int rd;
      const int n2 = x4_next_nsc<INV>(F, op_begin, op_end, q, D, rd);
      const DevOp& opn = F->ops[n];
      X4MC mc;
      x4_fill_mc<TL>(opn, mc);
      // phase X_n: A streams NSC n; B: spline of the previous NSC + layer 0 of NSC n
      {
        mc.next_base = opn.x3;  // Y_n streams the same NSC
        X4VC vc;
        x4_fill_vc<INV>(opn, vc);
        vc.blast = prev_blast;
        vc.rdelta = prev_rd;
        if (has_prev) x4_phase<K, ONE, INV, KS0, TL, true, true>(x3, pipe, mc, cx, A, B, vb, vc);
        else x4_phase<K, ONE, INV, KS0, TL, false, true>(x3, pipe, mc, cx, A, B, vb, vc);
      }
      // phase Y_n: B streams NSC n; A: spline of NSC n + layer 0 of NSC n2
      {
        mc.next_base = n2 >= 0 ? F->ops[n2].x3 : -1;
        X4VC vc;
        if (n2 >= 0) x4_fill_vc<INV>(F->ops[n2], vc);
        vc.blast = opn.x3_blast;
        vc.rdelta = rd;
        if (n2 >= 0) x4_phase<K, ONE, INV, KS0, TL, true, true>(x3, pipe, mc, cx, B, A, va, vc);
        else x4_phase<K, ONE, INV, KS0, TL, true, false>(x3, pipe, mc, cx, B, A, va, vc);
      }
      has_prev = true;
      prev_blast = opn.x3_blast;
      prev_rd = rd;
      if (n2 < 0) break;
      n = n2;
      ++q;
    }
    // set B: the spline of the last NSC, nothing to overlap
    {
      X4VC vc;
      vc.blast = prev_blast;
      vc.rdelta = prev_rd;
      x4_chunk<K, ONE, INV, KS0, TL, true, false>(cx, B, vb, vc);
    }
    wave_lds_sync();
  }
  // trailing ShiftBounds (exec order after the last NSC); Rolls there are
  // already applied through prev_rd (or, with no NSC at all, here)
  {
    int last_nsc = -1;
    for (int qq = 0; qq < nq; ++qq) {
      const int oi = INV ? (op_end - 1 - qq) : (op_begin + qq);
      if (F->ops[oi].kind == ZF_OP_NSC) last_nsc = qq;
    }
    if (last_nsc >= 0) {
      for (int qq = last_nsc + 1; qq < nq; ++qq) {
        const int oi = INV ? (op_end - 1 - qq) : (op_begin + qq);
        const DevOp& op = F->ops[oi];
        if (op.kind == ZF_OP_SHIFT_BOUNDS) {
          const float* sb = cx.par + op.sb;
          shift_bounds_op<INV>(sb, A.xs, s, hh, A.rot, D, A.ld);
          shift_bounds_op<INV>(sb, B.xs, s, hh, B.rot, D, B.ld);
        }
      }
    }
  }
  wave_lds_sync();
  flow_epilogue<kX4Waves>(F, A.xs, s, hh, lane, wave, A.rot, D, rowA, validA, A.ld, lp_out, block_partial, 1,
                          nparts, y_out, ld_out, s_part, 2LL * blockIdx.x);
  flow_epilogue<kX4Waves>(F, B.xs, s, hh, lane, wave, B.rot, D, rowB, validB, B.ld, lp_out, block_partial, 1,
                          nparts, y_out, ld_out, s_part + kX4Waves, 2LL * blockIdx.x + 1);
}

// LDS bytes of the two-set kernel.
inline size_t x4_lds_bytes(int K, bool one, int D, int C, int small_pieces) {
  const int TL = one ? (3 * K - 1 + 31) / 32 : (3 * K - 1 + 15) / 16;
  return (size_t)2 * group_bytes<2>(4 > TL ? 4 : TL) + ((size_t)small_pieces << 10) +
         (size_t)2 * kX4Waves * 32 * (D + C) * 4 + 2 * kX4Waves * sizeof(double);
}

template <int K, bool ONE, int KS0>
int launch_x4(const X3Launch& a, bool inverse, int small_pieces) {
  const long long grid = (a.N + kX4Rows - 1) / kX4Rows;
  if (grid > 0x7fffffffLL) return einval("N too large");
  const size_t lds = x4_lds_bytes(K, ONE, a.D, a.C, small_pieces);
  if (lds > 160 * 1024) return enotsup("two-set kernel: LDS footprint too large");
  if (inverse)
    hipLaunchKernelGGL((flow_kernel_x4<K, ONE, true, KS0>), dim3((unsigned)grid), dim3(kX4Waves * 64), lds, a.stream,
                       a.desc, a.blob, (const char*)a.x3, a.x, a.c, a.y, a.ld_in, a.ld_out, a.lp, a.part, a.nparts,
                       a.op_begin, a.op_end, a.N, a.seed, a.gen, small_pieces);
  else
    hipLaunchKernelGGL((flow_kernel_x4<K, ONE, false, KS0>), dim3((unsigned)grid), dim3(kX4Waves * 64), lds,
                       a.stream, a.desc, a.blob, (const char*)a.x3, a.x, a.c, a.y, a.ld_in, a.ld_out, a.lp, a.part,
                       a.nparts, a.op_begin, a.op_end, a.N, a.seed, a.gen, small_pieces);
  ZF_CHECK_LAUNCH("flow_kernel_x4");
  return ZF_OK;
}

}  // namespace
}  // namespace zf
