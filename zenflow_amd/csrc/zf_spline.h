// Rational-quadratic spline device math (Durkan et al. 2019), restating the
// reference semantics of src/zenflow/utils.py:65-250 exactly, including its
// numerically "impure" details (EPS inside logs/denominators, z clip, the
// out-of-bounds identity, the fill-mode gather at the idx == K sliver).
#pragma once
#include <hip/hip_runtime.h>

namespace zf {

constexpr float kEps = 1e-5f;            // utils.py:15
constexpr float kOneMinusEps = 0.99999f; // 1 - EPS, a Python float rounded to fp32 (utils.py:123)

__device__ __forceinline__ float qnan() { return __builtin_nanf(""); }

// utils.py:18-20  squareplus(x, b=4) = 0.5 * (x + sqrt(x^2 + b))
__device__ __forceinline__ float squareplus(float x) {
  return 0.5f * (x + __builtin_sqrtf(x * x + 4.0f));
}

// Bin parameters gathered at idx (utils.py:205-232 `_compute_rqs_input`).
struct RqsBin {
  float xk, yk, w, h, dk, dkp1, sk;
  bool oob;
};

// Bin search + gather (utils.py:220-232, `_index` :244-250, `_knots` :235-241).
//   P provides  w(j) = dx_j, h(j) = dy_j (0 <= j < K), d(j) = slope_j (0 <= j < K-1).
// Count semantics of `_index`: idx = clip(#{k : knot_k <= v} - 1, 0, K), with
// knots = [0, cumsum]. For the (usual) monotone knots this is the last bin
// whose left knot is <= v; a non-monotone parameter set (never produced by
// normalize_spline_params) falls back to re-summing the knots up to idx.
// jnp.take_along_axis defaults to mode="fill": an out-of-range gather gives NaN
// (idx == K => dx, dy, sk, dk[idx+1] are NaN).
template <bool FWD, class P>
__device__ __forceinline__ RqsBin rqs_bin(float v, int K, const P& p) {
  float xk = 0.f, yk = 0.f;
  float sxk = 0.f, syk = 0.f;
  int cnt = 0, sel = 0;
  for (int j = 0; j < K; ++j) {
    const float kk = FWD ? xk : yk;
    if (kk <= v) { ++cnt; sel = j; sxk = xk; syk = yk; }
    xk = xk + p.w(j);
    yk = yk + p.h(j);
  }
  {
    const float kk = FWD ? xk : yk;
    if (kk <= v) { ++cnt; sel = K; sxk = xk; syk = yk; }
  }
  int idx = cnt - 1;
  idx = idx < 0 ? 0 : (idx > K ? K : idx);
  if (idx != sel) {  // non-monotone knots: reproduce the gather at idx exactly
    xk = 0.f; yk = 0.f;
    for (int j = 0; j < idx; ++j) { xk = xk + p.w(j); yk = yk + p.h(j); }
    sxk = xk; syk = yk; sel = idx;
  }
  RqsBin b;
  b.xk = sxk;
  b.yk = syk;
  b.w = sel < K ? p.w(sel) : qnan();
  b.h = sel < K ? p.h(sel) : qnan();
  b.dk = (sel == 0 || sel == K) ? 1.0f : p.d(sel - 1);             // dk = [1, slope, 1]
  b.dkp1 = (sel + 1 < K) ? p.d(sel) : (sel + 1 == K ? 1.0f : qnan());
  b.sk = b.h / b.w;                                                 // sk = dy / dx
  b.oob = (v < 0.f) || (v >= 1.f);                                  // :245
  return b;
}

// Same bin search + gather over knots held in registers (compile-time K: every
// w[j] / h[j] index is static).  `slope(j)` returns the derivative at inner
// knot j+1; only the two the bin needs are requested.
template <bool FWD, int K, class SL>
__device__ __forceinline__ RqsBin rqs_bin_regs(float v, const float (&w)[K], const float (&h)[K],
                                               const SL& slope) {
  float xk = 0.f, yk = 0.f, sxk = 0.f, syk = 0.f, sw = w[0], sh = h[0];
  int cnt = 0, sel = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const float kk = FWD ? xk : yk;
    if (kk <= v) { ++cnt; sel = j; sxk = xk; syk = yk; sw = w[j]; sh = h[j]; }
    xk = xk + w[j];
    yk = yk + h[j];
  }
  {
    const float kk = FWD ? xk : yk;
    if (kk <= v) { ++cnt; sel = K; sxk = xk; syk = yk; sw = qnan(); sh = qnan(); }
  }
  int idx = cnt - 1;
  idx = idx < 0 ? 0 : (idx > K ? K : idx);
  if (idx != sel) {  // non-monotone knots (never from normalize_spline_params)
    xk = 0.f; yk = 0.f;
    sw = qnan(); sh = qnan();
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if (j == idx) { sw = w[j]; sh = h[j]; }
      if (j < idx) { xk = xk + w[j]; yk = yk + h[j]; }
    }
    sxk = xk; syk = yk; sel = idx;
  }
  RqsBin b;
  b.xk = sxk;
  b.yk = syk;
  b.w = sw;
  b.h = sh;
  b.dk = (sel == 0 || sel == K) ? 1.0f : slope(sel - 1);
  b.dkp1 = (sel + 1 < K) ? slope(sel) : (sel + 1 == K ? 1.0f : qnan());
  b.sk = b.h / b.w;
  b.oob = (v < 0.f) || (v >= 1.f);
  return b;
}

// rqs_bin_regs with the K-1 inner-knot slope inputs also in registers: the
// two the bin needs are picked by the same sweep (static register indices
// only: a dynamic index into a register array would go through scratch),
// then mapped by `tf` (squareplus for raw conditioner logits, identity for
// slopes).  Same count / fill-mode semantics as rqs_bin.
template <bool FWD, int K, class TF>
__device__ __forceinline__ RqsBin rqs_bin_regs_sl(float v, const float (&w)[K], const float (&h)[K],
                                                  const float (&sl)[K - 1], const TF& tf) {
  float xk = 0.f, yk = 0.f, sxk = 0.f, syk = 0.f, sw = w[0], sh = h[0];
  float lo = 0.f, hi = (K > 1) ? sl[0] : 0.f;  // raw slope inputs at knots sel, sel+1
  int cnt = 0, sel = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const float kk = FWD ? xk : yk;
    if (kk <= v) {
      ++cnt; sel = j; sxk = xk; syk = yk; sw = w[j]; sh = h[j];
      if (j >= 1) lo = sl[j - 1];
      if (j + 1 < K) hi = sl[j];
    }
    xk = xk + w[j];
    yk = yk + h[j];
  }
  {
    const float kk = FWD ? xk : yk;
    if (kk <= v) { ++cnt; sel = K; sxk = xk; syk = yk; sw = qnan(); sh = qnan(); }
  }
  int idx = cnt - 1;
  idx = idx < 0 ? 0 : (idx > K ? K : idx);
  if (idx != sel) {  // non-monotone knots (never from normalize_spline_params)
    xk = 0.f; yk = 0.f;
    sw = qnan(); sh = qnan();
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if (j == idx) {
        sw = w[j]; sh = h[j];
        if (j >= 1) lo = sl[j - 1];
        if (j + 1 < K) hi = sl[j];
      }
      if (j < idx) { xk = xk + w[j]; yk = yk + h[j]; }
    }
    sxk = xk; syk = yk; sel = idx;
  }
  RqsBin b;
  b.xk = sxk;
  b.yk = syk;
  b.w = sw;
  b.h = sh;
  b.dk = (sel == 0 || sel == K) ? 1.0f : tf(lo);
  b.dkp1 = (sel + 1 < K) ? tf(hi) : (sel + 1 == K ? 1.0f : qnan());
  b.sk = b.h / b.w;
  b.oob = (v < 0.f) || (v >= 1.f);
  return b;
}

// rqs_bin_regs_sl for knots known to be strictly increasing (every width and
// height > 0, as normalize_spline_params guarantees: each is >= c > 0) and
// raw slope logits mapped by squareplus: the bin is the last knot <= v, so
// the count / fallback bookkeeping of the general version drops out, and the
// boundary derivative 1 is carried as the logit 0 (squareplus(0) == 1
// exactly).  Results equal rqs_bin_regs_sl's for such inputs, including the
// NaN fill at idx == K (utils.py:224-230).
template <bool FWD, int K, class TF>
__device__ __forceinline__ RqsBin rqs_bin_monotone(float v, const float (&w)[K], const float (&h)[K],
                                                   const float (&sl)[K - 1], const TF& sp, bool padlast = false) {
  // knot 0 (at 0) latched up front: for v >= 0 it is the first knot <= v,
  // and for v < 0 (out of bounds: identity) or NaN the bin is unused
  float sxk = 0.f, syk = 0.f, sw = w[0], sh = h[0];
  float lo = 0.f, hi = (K > 1) ? sl[0] : 0.f;  // logits of dk, dk+1 at the current bin
  float xk = w[0], yk = h[0];
  float xkm = xk, ykm = yk;  // knot K-1 (padlast)
  // branch-free latch (selects, not exec-masked moves)
#pragma unroll
  for (int j = 1; j < K; ++j) {
    const bool c = (FWD ? xk : yk) <= v;
    sxk = c ? xk : sxk;
    syk = c ? yk : syk;
    sw = c ? w[j] : sw;
    sh = c ? h[j] : sh;
    lo = c ? sl[j - 1] : lo;
    hi = c ? ((j + 1 < K) ? sl[j] : 0.f) : hi;
    if (j == K - 1) { xkm = xk; ykm = yk; }
    xk = xk + w[j];
    yk = yk + h[j];
  }
  {
    // padlast: knot K-1 is the couplings' last real knot (the split-MFMA
    // kernels run K-1 knots padded with one inert knot, x3_padded_knots), so
    // the idx == K sliver starts there
    const float kk = padlast ? (FWD ? xkm : ykm) : (FWD ? xk : yk);
    if (kk <= v) {
      sxk = padlast ? xkm : xk;
      syk = padlast ? ykm : yk;
      sw = qnan(); sh = qnan(); lo = 0.f; hi = qnan();
    }
  }
  RqsBin b;
  b.xk = sxk;
  b.yk = syk;
  b.w = sw;
  b.h = sh;
  b.dk = sp(lo);
  b.dkp1 = sp(hi);
  b.sk = b.h / b.w;
  b.oob = (v < 0.f) || (v >= 1.f);
  return b;
}

// rqs_bin_monotone's latch with exec-masked moves instead of selects
// (split-MFMA kernels, monotone knots only).  The knots grow along j, so the
// lanes whose knot j is <= v are a subset of those whose knot j-1 is: each
// knot's v_cmpx narrows exec to them and the latch is plain v_mov / v_add
// under that exec (8 full-rate VALU per knot against a compare, six
// two-pass v_cndmask_b32_e64 and two adds).  The same adds in the same
// order as rqs_bin_monotone's running sums (knot j = knot j-1 + w[j-1]),
// so the latched values are bit-identical.  Eight knots per asm statement;
// the narrowed exec is carried between statements in an SGPR pair.  The
// latched values are early-clobber: an input equal in value to one of them
// (a zero slope logit and the zero lo seed) must not share its register.
#ifndef ZF_CMPX_NOP
#define ZF_CMPX_NOP 0
#endif
#if ZF_CMPX_NOP
#define ZF_CMPX_PAD "s_nop 4\n\t"
#else
#define ZF_CMPX_PAD ""
#endif
#define ZF_KNOT_F(i)                                                                                   \
  "v_add_f32 %[t], %[sx], %[sw]\n\tv_cmpx_le_f32 vcc, %[t], %[v]\n\t" ZF_CMPX_PAD "v_mov_b32 %[sx], %[t]\n\t"       \
  "v_add_f32 %[sy], %[sy], %[sh]\n\tv_mov_b32 %[sw], %[w" #i "]\n\tv_mov_b32 %[sh], %[h" #i "]\n\t" \
  "v_mov_b32 %[lo], %[hi]\n\tv_mov_b32 %[hi], %[s" #i "]\n\t"
#define ZF_KNOT_I(i)                                                                                   \
  "v_add_f32 %[t], %[sy], %[sh]\n\tv_cmpx_le_f32 vcc, %[t], %[v]\n\t" ZF_CMPX_PAD "v_mov_b32 %[sy], %[t]\n\t"       \
  "v_add_f32 %[sx], %[sx], %[sw]\n\tv_mov_b32 %[sw], %[w" #i "]\n\tv_mov_b32 %[sh], %[h" #i "]\n\t" \
  "v_mov_b32 %[lo], %[hi]\n\tv_mov_b32 %[hi], %[s" #i "]\n\t"
#define ZF_KNOT_OPS(i) [w##i] "v"(w[i]), [h##i] "v"(h[i]), [s##i] "v"(s[i])
#define ZF_KNOT_OUTS                                                                                 \
  [sx] "+&v"(sx), [sy] "+&v"(sy), [sw] "+&v"(sw), [sh] "+&v"(sh), [lo] "+&v"(lo), [hi] "+&v"(hi), [m] "+s"(m), \
      [t] "=&v"(t), [sv] "=&s"(sv)

template <bool FWD, int N>
__device__ __forceinline__ void knot_chunk(unsigned long long& m, float v, float& sx, float& sy, float& sw, float& sh,
                                           float& lo, float& hi, const float* w, const float* h, const float* s) {
  static_assert(N == 7 || N == 8, "knot chunks of 7 or 8");
  float t;
  unsigned long long sv;
#define ZF_CHUNK(KN, ...)                                                                                        \
  asm("s_mov_b64 %[sv], exec\n\ts_mov_b64 exec, %[m]\n\t" KN(0) KN(1) KN(2) KN(3) KN(4) KN(5) KN(6) __VA_ARGS__ \
      "s_mov_b64 %[m], exec\n\ts_mov_b64 exec, %[sv]"                                                           \
      : ZF_KNOT_OUTS                                                                                             \
      : [v] "v"(v), ZF_KNOT_OPS(0), ZF_KNOT_OPS(1), ZF_KNOT_OPS(2), ZF_KNOT_OPS(3), ZF_KNOT_OPS(4), ZF_KNOT_OPS(5), \
        ZF_KNOT_OPS(6)ZF_CHUNK_LAST                                                                             \
      : "vcc")
  if constexpr (N == 8) {
#define ZF_CHUNK_LAST , ZF_KNOT_OPS(7)
    if constexpr (FWD) ZF_CHUNK(ZF_KNOT_F, ZF_KNOT_F(7));
    else ZF_CHUNK(ZF_KNOT_I, ZF_KNOT_I(7));
#undef ZF_CHUNK_LAST
  } else {
#define ZF_CHUNK_LAST
    if constexpr (FWD) ZF_CHUNK(ZF_KNOT_F, );
    else ZF_CHUNK(ZF_KNOT_I, );
#undef ZF_CHUNK_LAST
  }
#undef ZF_CHUNK
}

template <bool FWD, int K, class TF>
__device__ __forceinline__ RqsBin rqs_bin_exec(float v, const float (&w)[K], const float (&h)[K],
                                               const float (&sl)[K - 1], const TF& sp, bool padlast) {
  static_assert(K % 8 == 0, "knot chunks of 8");
  float sx = 0.f, sy = 0.f, sw = w[0], sh = h[0], lo = 0.f, hi = sl[0];
  float s2[K];  // slope logit j for knot j's upper neighbour; 0 past the last inner knot
#pragma unroll
  for (int j = 0; j < K - 1; ++j) s2[j] = sl[j];
  s2[K - 1] = 0.f;
  unsigned long long m = __builtin_amdgcn_read_exec();
  knot_chunk<FWD, 7>(m, v, sx, sy, sw, sh, lo, hi, w + 1, h + 1, s2 + 1);
#pragma unroll
  for (int c = 8; c < K; c += 8) knot_chunk<FWD, 8>(m, v, sx, sy, sw, sh, lo, hi, w + c, h + c, s2 + c);
  // the idx == K sliver: past knot K (or past the last real knot K-1, padlast)
  {
    float t;
    unsigned long long sv;
    const float nan = qnan();
    if (padlast) {
      asm("s_mov_b64 %[sv], exec\n\ts_mov_b64 exec, %[m]\n\t"
          "v_mov_b32 %[sw], %[nan]\n\tv_mov_b32 %[sh], %[nan]\n\tv_mov_b32 %[lo], 0\n\tv_mov_b32 %[hi], %[nan]\n\t"
          "s_mov_b64 exec, %[sv]"
          : [sw] "+&v"(sw), [sh] "+&v"(sh), [lo] "+&v"(lo), [hi] "+&v"(hi), [sv] "=&s"(sv)
          : [m] "s"(m), [nan] "v"(nan));
      (void)t;
    } else {
      asm("s_mov_b64 %[sv], exec\n\ts_mov_b64 exec, %[m]\n\t"
          "v_add_f32 %[t], %[a], %[da]\n\tv_cmpx_le_f32 vcc, %[t], %[v]\n\t" ZF_CMPX_PAD "v_mov_b32 %[a], %[t]\n\t"
          "v_add_f32 %[b], %[b], %[db]\n\t"
          "v_mov_b32 %[sw], %[nan]\n\tv_mov_b32 %[sh], %[nan]\n\tv_mov_b32 %[lo], 0\n\tv_mov_b32 %[hi], %[nan]\n\t"
          "s_mov_b64 exec, %[sv]"
          : [a] "+&v"(FWD ? sx : sy), [b] "+&v"(FWD ? sy : sx), [sw] "+&v"(sw), [sh] "+&v"(sh), [lo] "+&v"(lo),
            [hi] "+&v"(hi), [t] "=&v"(t), [sv] "=&s"(sv)
          : [m] "s"(m), [nan] "v"(nan), [v] "v"(v), [da] "v"(FWD ? sw : sh), [db] "v"(FWD ? sh : sw)
          : "vcc");
    }
  }
  RqsBin b;
  b.xk = sx;
  b.yk = sy;
  b.w = sw;
  b.h = sh;
  b.dk = sp(lo);
  b.dkp1 = sp(hi);
  b.sk = b.h / b.w;
  b.oob = (v < 0.f) || (v >= 1.f);
  return b;
}
#undef ZF_KNOT_F
#undef ZF_KNOT_I
#undef ZF_KNOT_OPS
#undef ZF_KNOT_OUTS

// utils.py:121-139 — forward value and per-dim log|dy/dx|.
__device__ __forceinline__ void rqs_forward_eval(float x, const RqsBin& b, float& y, float& ld) {
  const float zr = (x - b.xk) / b.w;               // :122
  // :123 jnp.clip propagates NaN (fmaxf/fminf would drop it)
  const float z = (zr != zr) ? zr : fminf(fmaxf(zr, kEps), kOneMinusEps);
  const float az = 1.0f - z;
  const float num = b.h * z * (b.sk * z + b.dk * az);              // :125
  const float den = b.sk + (b.dkp1 + b.dk - 2.0f * b.sk) * z * az;  // :126
  const float yv = b.yk + num / (den + kEps);                       // :127
  y = b.oob ? x : yv;                                               // :130
  const float num2 = z * (b.dkp1 * z + 2.0f * b.sk * az) + b.dk * (az * az);  // :133
  const float l = 2.0f * logf(b.sk + kEps) + logf(num2 + kEps) - 2.0f * logf(den + kEps);
  ld = b.oob ? 0.0f : l;                                            // :138
}

// utils.py:191-201 — inverse via the quadratic root.
__device__ __forceinline__ float rqs_inverse_eval(float y, const RqsBin& b) {
  const float dy = y - b.yk;
  const float t = b.dkp1 + b.dk - 2.0f * b.sk;
  const float a = b.h * (b.sk - b.dk) + dy * t;  // :193
  const float bb = b.h * b.dk - dy * t;          // :194
  const float c = -b.sk * dy;                    // :195
  const float z = 2.0f * c / (-bb - __builtin_sqrtf(bb * bb - 4.0f * a * c));  // :197
  const float x = z * b.w + b.xk;                // :198
  return b.oob ? y : x;                          // :201
}

}  // namespace zf
