// Fused flow kernel, bf16x3 variant: the same op chain as flow_kernel
// (zf_flow.hip) with the conditioner's streamed Dense layers (hidden ->
// hidden and hidden -> spline parameters) on v_mfma_f32_32x32x16_bf16 using
// the three-term bf16 split of both operands (x = hi + mid + lo, each an RNE
// bf16 of the remaining residual) and six products per k-step,
//   mid*mid + hi*lo + lo*hi + hi*mid + mid*hi + hi*hi   (small terms first),
// which reproduces an fp32 dot product to ~1e-7 relative (verified on the
// GPU by tests/hip/mfma_bf16x3_layout.hip) at 16/6 = 2.7x the fp32-MFMA rate.
//
// Execution model (DESIGN.md §bf16x3 kernel):
//   * 8 waves x 32 samples = 256 samples per block, one block per CU (2 waves
//     per SIMD).  The weight fragments (pre-split hi/mid/lo bf16, packed in
//     exactly the per-lane order the MFMA A operand wants) are shared by the
//     8 waves through LDS: each Dense layer is a sequence of "groups" (half
//     of the layer's input rows for all output tiles; 48 KiB for a 128x128
//     layer) that the block DMAs global->LDS (global_load_lds_dwordx4) one
//     group ahead into a double buffer, so every weight byte crosses L2->CU
//     once per 256 samples instead of once per 32;
//   * the B operand is the previous layer's f32 accumulator tile, split to
//     bf16x3 in registers (accumulator-as-operand: k-step s of a tile uses
//     accumulator registers 8s..8s+7; A is packed with the same k order);
//   * the last layer's rows are permuted so that lane half h of every output
//     tile holds 16 consecutive spline parameters of transformed dim h: the
//     whole normalize_spline_params + bin search + RQ spline runs from
//     registers, no LDS ring;
//   * layer 0 (BatchNorm'd conditioning inputs, 1-2 k-steps), ShiftBounds,
//     Roll and the latent epilogue are the fp32 kernel's (zf_flow_dev.h).
// Eligibility (host, x3_eligible): hidden widths padded to 128, knots 8 or
// 16, at most 2 transformed dims (dim <= 5).  Everything else, and
// ZF_DISABLE_X3=1, runs flow_kernel.
#include "zf_flow_dev.h"

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace zf {
namespace {

typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kX3T = 4;  // hidden tiles (hidden padded to 128)
// Bytes of one weight group covering GT input tiles: [tl][s][o][part] x 1 KiB.
constexpr int group_bytes(int GT, int NOUT) { return GT * 2 * NOUT * 3 * 1024; }

#ifndef ZF_X3_TRACE
#define ZF_X3_TRACE 0
#endif
#if ZF_X3_TRACE
// Timing probe (tuning builds only): s_memtime stamps of every wave of 4
// blocks, [block][wave][256] (event id << 48 | time).
__device__ unsigned long long g_x3_trace[4][8][256];
__device__ int g_x3_trace_n[4][8];
__device__ __forceinline__ void x3_mark(int ev) {
  const int b = blockIdx.x;
  const int tb = b == 5 ? 0 : b == 1029 ? 1 : b == 2053 ? 2 : b == 3077 ? 3 : -1;
  if (tb < 0) return;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) {
    const int n = g_x3_trace_n[tb][w];
    if (n < 256) g_x3_trace[tb][w][n] = ((unsigned long long)ev << 48) | (t & 0xffffffffffffull);
    g_x3_trace_n[tb][w] = n + 1;
  }
}
#define X3_MARK(ev) x3_mark(ev)
#else
#define X3_MARK(ev) ((void)0)
#endif

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

// One weight group from LDS: input tiles GT*Q .. GT*Q+GT-1 (2 k-steps of 16
// each) into NOUT output tiles.  Block (tl, s, o, part) is 1 KiB at
// (((tl*2 + s)*NOUT + o)*3 + part) KiB; lane l's 16 bytes at l*16.
template <int NOUT, int GT, int Q>
__device__ __forceinline__ void x3_group(const char* buf, const floatx16 (&hb)[kX3T], floatx16 (&acc)[NOUT],
                                         int lane) {
  const char* lb = buf + lane * 16;
#pragma unroll
  for (int tl = 0; tl < GT; ++tl) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 bh, bm, bl;
      if (s == 0) split8<0>(hb[GT * Q + tl], bh, bm, bl);
      else split8<1>(hb[GT * Q + tl], bh, bm, bl);
#pragma unroll
      for (int o = 0; o < NOUT; ++o) {
        const char* a = lb + ((((tl * 2 + s) * NOUT + o) * 3) << 10);
        const bf16x8 ah = *reinterpret_cast<const bf16x8*>(a);
        const bf16x8 am = *reinterpret_cast<const bf16x8*>(a + 1024);
        const bf16x8 al = *reinterpret_cast<const bf16x8*>(a + 2048);
        acc[o] = mfma3(ah, am, al, bh, bm, bl, acc[o]);
      }
    }
  }
}

// The group stream of the NSC being computed (byte offsets into the x3
// blob), set up at NSC entry from the op's scalar fields: the per-step
// prefetch then needs no memory access of its own (a scalar load there would
// make its lgkmcnt wait drain the step's LDS reads too).
struct X3Span {
  long long base;       // group 0 of this NSC
  long long next_base;  // group 0 of the next NSC in execution order within range, or -1
  int G, nhid;          // groups in this NSC, hidden-layer groups among them
  int last_pieces;      // KiB pieces of one last-layer group
  int next_pieces;      // KiB pieces of the next NSC's group 0
};

template <int GT>
__device__ __forceinline__ int first_pieces(const DevOp& op) {
  return (op.n_hidden > 1 ? group_bytes(GT, kX3T) : group_bytes(GT, op.x3_tlast)) >> 10;
}

template <int GT, bool INV>
__device__ __forceinline__ X3Span make_span(const DevFlow* __restrict__ F, int oi, int op_begin, int op_end) {
  const DevOp& op = F->ops[oi];
  X3Span sp;
  sp.base = op.x3;
  sp.G = op.x3_groups;
  sp.nhid = (kX3T / GT) * (op.n_hidden - 1);
  sp.last_pieces = group_bytes(GT, op.x3_tlast) >> 10;
  const int n = op.x3_next[INV ? 1 : 0];
  if (n >= op_begin && n < op_end) {
    sp.next_base = F->ops[n].x3;
    sp.next_pieces = first_pieces<GT>(F->ops[n]);
  } else {
    sp.next_base = -1;
    sp.next_pieces = 0;
  }
  return sp;
}

// Issue the DMA of one group into an LDS buffer: 1 KiB pieces (one
// global_load_lds_dwordx4 per wave: wave-uniform LDS base, lane*16 implied)
// spread over the block's waves.
template <int NW>
__device__ __forceinline__ void x3_dma(const char* __restrict__ src, char* dst, int pieces, int wave,
                                       int lane) {
  for (int p = wave; p < pieces; p += NW)
    __builtin_amdgcn_global_load_lds((const void*)(src + (p << 10) + lane * 16),
                                     (__attribute__((address_space(3))) void*)(dst + (p << 10)), 16, 0, 0);
}

// Block-wide weight-group pipeline state (every field wave-uniform).
struct X3Pipe {
  char* wbuf;   // [NBUF][group bytes] LDS ring
  int buf;      // ring slot holding the group this wave computes next
  int g;        // index of that group within the current NSC
  X3Span span;  // current NSC's group stream
  int lead;     // index of this wave among the NL DMA-issuing waves, or -1
};

// DMA the group after group p.g (the next one of this NSC, or group 0 of
// the next NSC) into `dst`; nothing at the end of the stream.
template <int NL, int GT>
__device__ __forceinline__ void x3_issue_next(const char* __restrict__ x3, const X3Pipe& p, char* dst, int lane) {
  constexpr int kHid = group_bytes(GT, kX3T);
  const int g = p.g + 1;
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
  x3_dma<NL>(x3 + off, dst, pieces, p.lead, lane);
}

// One pipeline step: wait for this wave's DMAs, block barrier (the group in
// slot `buf` is complete and the slot after it is free), the issuing waves
// prefetch the next group into the next slot, then this group's MFMAs.
template <int NL, int GT, int NBUF, int NOUT, int Q>
__device__ __forceinline__ void x3_step(const char* __restrict__ x3, X3Pipe& p, const floatx16 (&hb)[kX3T],
                                        floatx16 (&acc)[NOUT], int lane, const float* __restrict__ bias,
                                        int hh) {
  constexpr int kBuf = group_bytes(GT, kX3T);
  X3_MARK(1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  X3_MARK(2);
  if constexpr (NBUF == 3) {
    // Offset half-blocks: the wave whose step ends in a VALU tail (the
    // layer's last group -> epilogue / spline) issues its MFMAs first, so
    // that tail overlaps the partner wave's MFMAs on the same SIMD.
    if constexpr (Q + 1 == kX3T / GT) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
  }
  const int nb = (p.buf + 1 == NBUF) ? 0 : p.buf + 1;
  if (p.lead >= 0) x3_issue_next<NL, GT>(x3, p, p.wbuf + nb * kBuf, lane);
  if (bias != nullptr) {
    // Bias of a layer that started from zero: loaded here, in the layer's last
    // step (its earlier input tiles are dead by now), added after the MFMAs.
    floatx16 bt[NOUT];
#pragma unroll
    for (int o = 0; o < NOUT; ++o) bt[o] = bias_acc(bias + o * 32, hh);
    x3_group<NOUT, GT, Q>(p.wbuf + p.buf * kBuf, hb, acc, lane);
#pragma unroll
    for (int o = 0; o < NOUT; ++o) acc[o] += bt[o];
  } else {
    x3_group<NOUT, GT, Q>(p.wbuf + p.buf * kBuf, hb, acc, lane);
  }
  p.buf = nb;
  p.g += 1;
}

// A whole streamed Dense layer: kX3T / GT groups.
// `bias_last`: bias tiles added after the last step (nullptr: acc already
// holds the bias).
template <int NL, int GT, int NBUF, int NOUT, int Q = 0>
__device__ __forceinline__ void x3_layer(const char* __restrict__ x3, X3Pipe& p, const floatx16 (&hb)[kX3T],
                                         floatx16 (&acc)[NOUT], int lane, const float* bias_last = nullptr,
                                         int hh = 0) {
  if constexpr (Q + 1 < kX3T / GT) {
    x3_step<NL, GT, NBUF, NOUT, Q>(x3, p, hb, acc, lane, nullptr, hh);
    x3_layer<NL, GT, NBUF, NOUT, Q + 1>(x3, p, hb, acc, lane, bias_last, hh);
  } else {
    x3_step<NL, GT, NBUF, NOUT, Q>(x3, p, hb, acc, lane, bias_last, hh);
  }
}

// squareplus with a Newton-corrected reciprocal square root (one
// transcendental instead of sqrt + rcp): ~0.5 ulp, like sqrtf.
__device__ __forceinline__ float squareplus_rsq(float x) {
  const float a = x * x + 4.0f;
  const float r = __builtin_amdgcn_rsqf(a);
  float sq = a * r;
  sq = __builtin_fmaf(__builtin_fmaf(-sq, sq, a), 0.5f * r, sq);
  return 0.5f * (x + sq);
}

// PIPE 0: every wave issues DMA pieces and all waves step in lockstep
// (NBUF = 2).  PIPE 1: the block runs as two half-blocks offset by one
// group — waves [0, NW/2) issue every DMA and compute group t while waves
// [NW/2, NW) compute group t-1 (NBUF = 3) — so one half's VALU phases
// (spline, swish epilogues, layer 0) overlap the other half's MFMAs on the
// same SIMD.  PIPE 2: lockstep, small parameters read from global memory
// (L2-resident) instead of LDS, so that three 4-wave blocks fit a CU's LDS
// (3 waves per SIMD, <= 168 VGPRs).
template <int K, int NW, int GT, int PIPE, bool INV>
__global__ __launch_bounds__(NW * 64, PIPE == 2 ? 3 : 8 / NW) void flow_kernel_x3(
    const DevFlow* __restrict__ F, const float* __restrict__ blob, const char* __restrict__ x3,
    const float* __restrict__ xin, const float* __restrict__ cin, float* __restrict__ y_out,
    const float* __restrict__ ld_in, float* __restrict__ ld_out, float* __restrict__ lp_out,
    double* __restrict__ block_partial, long long nparts, int op_begin, int op_end, long long N,
    unsigned long long seed, int gen) {
  constexpr int TL = (3 * K - 1 + 15) / 16;  // last-layer tiles: 16 parameters per lane half
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int D = F->D;
  const int C = F->C;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: scalar cursor math
  const int lane = threadIdx.x & 63;
  const int s = lane & 31;
  const int hh = lane >> 5;
  constexpr int kBuf = group_bytes(GT, kX3T);
  constexpr int NBUF = PIPE == 1 ? 3 : 2;
  constexpr int NL = PIPE == 1 ? NW / 2 : NW;  // DMA-issuing waves
  constexpr bool kSmallLds = PIPE != 2;
  // LDS: [NBUF][kBuf] weight ring | small parameters | [NW][D][32] state | [NW] partials
  const int small4 = kSmallLds ? (F->small_floats + 3) & ~3 : 0;
  float* lsm = reinterpret_cast<float*>(lds + NBUF * kBuf);
  const float* sp = kSmallLds ? lsm : blob;
  float* xs = lsm + small4 + wave * (32 * D);
  double* s_part = reinterpret_cast<double*>(lsm + small4 + NW * 32 * D);
  const long long row = ((long long)blockIdx.x * NW + wave) * kTile + s;
  const bool valid = row < N;

  X3_MARK(0);
  {  // small parameters -> LDS (before any DMA is in flight)
    const floatx4* src = reinterpret_cast<const floatx4*>(blob);
    floatx4* dst = reinterpret_cast<floatx4*>(lsm);
    for (int i = threadIdx.x; i < small4 / 4; i += NW * 64) dst[i] = src[i];
  }
  load_state(xs, xin, row, valid, D, s, hh, F, seed, INV ? gen : 0);
  float ld = (ld_in != nullptr && valid) ? ld_in[row] : 0.f;
  int rot = 0;
  __syncthreads();

  X3Pipe pipe;
  pipe.wbuf = lds;
  pipe.buf = 0;
  pipe.g = 0;
  pipe.lead = wave < NL ? wave : -1;
  {  // group 0 of the first NSC in execution order goes out now
    int first = -1;
    const int nq = op_end - op_begin;
    for (int q = 0; q < nq; ++q) {
      const int oi = INV ? (op_end - 1 - q) : (op_begin + q);
      if (F->ops[oi].kind == ZF_OP_NSC) { first = oi; break; }
    }
    if (first >= 0 && pipe.lead >= 0)
      x3_dma<NL>(x3 + F->ops[first].x3, pipe.wbuf, first_pieces<GT>(F->ops[first]), pipe.lead, lane);
  }
  if (PIPE == 1 && pipe.lead < 0) __syncthreads();  // trailing half starts one step late

  const KnotConsts kc(K);
  const int nq = op_end - op_begin;
  for (int q = 0; q < nq; ++q) {
    const int oi = INV ? (op_end - 1 - q) : (op_begin + q);
    const DevOp& op = F->ops[oi];
    const int kind = op.kind;
    if (kind == ZF_OP_ROLL) {  // bijectors.py:291 / :296
      rot = pmod(INV ? rot + op.shift : rot - op.shift, D);
    } else if (kind == ZF_OP_SHIFT_BOUNDS) {
      shift_bounds_op<INV>(sp + op.sb, xs, s, hh, rot, D, ld);
    } else {  // ZF_OP_NSC, bijectors.py:329-371
      pipe.span = make_span<GT, INV>(F, oi, op_begin, op_end);
      pipe.g = 0;
      floatx16 hb[kX3T];
      X3_MARK(3);
      layer0<kX3T>(op, sp, xs, cin, row, valid, C, rot, D, s, hh, lane, hb);
      X3_MARK(4);
      // Hidden layers 1..n_hidden-1 (:343-345), kX3T / GT groups each.
      auto hidden = [&](int l) {
        floatx16 acc[kX3T];
#pragma unroll
        for (int o = 0; o < kX3T; ++o) acc[o] = bias_acc(sp + op.b[l] + o * 32, hh);
        x3_layer<NL, GT, NBUF, kX3T>(x3, pipe, hb, acc, lane);
        X3_MARK(5);
#pragma unroll
        for (int o = 0; o < kX3T; ++o)
#pragma unroll
          for (int r = 0; r < 16; ++r) hb[o][r] = swish(acc[o][r]);
      };
      for (int l = 1; l < op.n_hidden; ++l) hidden(l);
      // Last Dense (:346-347): lane half h, tile o, register r = parameter
      // 16*o + r of transformed dim h.
      floatx16 pa[TL];
#pragma unroll
      for (int o = 0; o < TL; ++o) pa[o] = floatx16{0};
      X3_MARK(6);
      x3_layer<NL, GT, NBUF, TL>(x3, pipe, hb, pa, lane, sp + op.x3_blast, hh);
      X3_MARK(7);
      float P[TL * 16];
#pragma unroll
      for (int o = 0; o < TL; ++o)
#pragma unroll
        for (int r = 0; r < 16; ++r) P[16 * o + r] = pa[o][r];
      // normalize_spline_params (utils.py:37-62) + RQ spline (utils.py:65-250)
      const int dt = op.dt;
      float ldv = 0.f;
      const bool act = hh < dt;  // lane half h transforms dim h (idle half when dt == 1)
      {
        float w[K], hg[K];
        float sx = 0.f, sy = 0.f;
#pragma unroll
        for (int j = 0; j < K; ++j) {  // squareplus + sums in order (utils.py:30-33)
          w[j] = squareplus_rsq(P[j]);
          hg[j] = squareplus_rsq(P[K + j]);
          sx = sx + w[j];
          sy = sy + hg[j];
        }
        // (v / sum + c) / (1 + c K) as one fma per knot: the parameters
        // themselves already differ from the reference's in the last ulp
        // (GEMM summation order), so correctly rounded divisions buy nothing.
        const float ax = rcp_refined(sx) * kc.rnorm, ay = rcp_refined(sy) * kc.rnorm;
        const float bc = kc.c * kc.rnorm;
#pragma unroll
        for (int j = 0; j < K; ++j) {
          w[j] = __builtin_fmaf(w[j], ax, bc);
          hg[j] = __builtin_fmaf(hg[j], ay, bc);
        }
        float sl[K - 1];  // raw slope logits; the bin's two get squareplus'd
#pragma unroll
        for (int j = 0; j < K - 1; ++j) sl[j] = P[2 * K + j];
        float* xp = xs + pmod(hh + rot, D) * 32 + s;
        const float xv = *xp;
        const RqsBin bin = rqs_bin_monotone<!INV, K>(xv, w, hg, sl, [](float v) { return v == 0.f ? 1.f : squareplus_rsq(v); });
        float yv;
        if (!INV) {
          float l;
          rqs_forward_eval(xv, bin, yv, l);
          ldv = act ? l : 0.f;
        } else {
          yv = rqs_inverse_eval(xv, bin);
        }
        if (act) *xp = yv;
      }
      wave_lds_sync();
      X3_MARK(8);
      if (!INV) {  // log_det.sum(axis=1) in dim order (utils.py:139), Chain += (bijectors.py:110)
        const float other = __shfl_xor(ldv, 32);
        float ldc = hh == 0 ? ldv : other;
        if (dt == 2) ldc = ldc + (hh == 0 ? other : ldv);
        ld = ld + ldc;
      }
    }
  }

  if (PIPE == 1 && pipe.lead >= 0) __syncthreads();  // leading half: matching trailing step
  X3_MARK(9);
  flow_epilogue<NW>(F, xs, s, hh, lane, wave, rot, D, row, valid, ld, lp_out, block_partial,
                    NW * kTile / 128, nparts, y_out, ld_out, s_part);
  X3_MARK(10);
}

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

// hidden widths padded to 128, one knot count in {8, 16}, <= 2 transformed dims.
bool x3_eligible(const zf_flow_desc& desc, int HP, int* K_out) {
  const char* env = std::getenv("ZF_DISABLE_X3");
  if (env && env[0] == '1') return false;
  if (HP != 128) return false;
  int K = 0;
  for (int i = 0; i < desc.n_ops; ++i) {
    const zf_op_desc& op = desc.ops[i];
    if (op.kind != ZF_OP_NSC) continue;
    if (K == 0) K = op.knots;
    if (op.knots != K) return false;
  }
  if (K != 8 && K != 16) return false;
  if (desc.dim / 2 > 2) return false;
  *K_out = K;
  return true;
}

int x3_last_tiles(int K) { return (3 * K - 1 + 15) / 16; }

// Pack the group streams (bf16 hi/mid/lo A fragments) of every NSC and the
// row-permuted last-layer biases (into `packed` at F.ops[i].x3_blast, which
// the caller allocated with x3_last_tiles(K)*32 floats).
void x3_pack(const zf_flow_desc& desc, const float* nat, int GT, DevFlow& F, float* packed,
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
    const int dt = desc.dim / 2, K = op.knots, S = 3 * K - 1;
    const int TL = x3_last_tiles(K);
    d.x3 = (long long)stream.size() * 2;
    d.x3_tlast = TL;
    d.x3_groups = (kX3T / GT) * op.n_hidden;
    for (int l = 1; l <= op.n_hidden; ++l) {
      const bool last = (l == op.n_hidden);
      const int in = op.hidden[l - 1];
      const int out = last ? dt * S : op.hidden[l];
      const int NOUT = last ? TL : kX3T;
      const float* W = nat + op.off_w[l];
      for (int q = 0; q < kX3T / GT; ++q)
        for (int tl = 0; tl < GT; ++tl)
          for (int s = 0; s < 2; ++s)
            for (int o = 0; o < NOUT; ++o) {
              uint16_t part[3][64][8];
              for (int ln = 0; ln < 64; ++ln)
                for (int j = 0; j < 8; ++j) {
                  const int kstep = 2 * (GT * q + tl) + s;
                  const int k = 16 * kstep + 8 * (j >> 2) + 4 * (ln >> 5) + (j & 3);
                  const int rho = ln & 31;
                  int col;
                  if (!last) {
                    col = 32 * o + rho;
                    if (col >= out) col = -1;
                  } else {
                    const int h = (rho >> 2) & 1, r = (rho & 3) + 4 * (rho >> 3), jp = 16 * o + r;
                    col = (h < dt && jp < S) ? h * S + jp : -1;
                  }
                  const float x = (k < in && col >= 0) ? W[(int64_t)k * out + col] : 0.f;
                  const uint16_t bh = bf16_rne(x);
                  const float r1 = x - bf16_f(bh);
                  const uint16_t bm = bf16_rne(r1);
                  const uint16_t bl = bf16_rne(r1 - bf16_f(bm));
                  part[0][ln][j] = bh;
                  part[1][ln][j] = bm;
                  part[2][ln][j] = bl;
                }
              const uint16_t* pp = &part[0][0][0];
              stream.insert(stream.end(), pp, pp + 3 * 64 * 8);
            }
    }
    // permuted last bias: [o][lane half h][r] = bias[h*S + 16o + r]
    const float* B = nat + op.off_b[op.n_hidden];
    for (int o = 0; o < TL; ++o)
      for (int h = 0; h < 2; ++h)
        for (int r = 0; r < 16; ++r) {
          const int jp = 16 * o + r;
          packed[d.x3_blast + (o * 2 + h) * 16 + r] = (h < dt && jp < S) ? B[h * S + jp] : 0.f;
        }
  }
}

template <int NW, int GT, int PIPE>
size_t lds_bytes(int small_floats, int D) {
  return (size_t)(PIPE == 1 ? 3 : 2) * group_bytes(GT, kX3T) + (size_t)(PIPE == 2 ? 0 : (small_floats + 3) & ~3) * 4 +
         (size_t)NW * 32 * D * 4 + NW * sizeof(double);
}

template <int K, int NW, int GT, int PIPE>
int launch_x3(const X3Launch& a, bool inverse) {
  const long long rows = NW * kTile;
  const long long grid = (a.N + rows - 1) / rows;
  if (grid > 0x7fffffffLL) return einval("N too large");
  const size_t lds = lds_bytes<NW, GT, PIPE>(a.small_floats, a.D);
  if (lds > 160 * 1024) return enotsup("bf16x3 LDS footprint too large");
  if (inverse)
    hipLaunchKernelGGL((flow_kernel_x3<K, NW, GT, PIPE, true>), dim3((unsigned)grid), dim3(NW * 64), lds, a.stream,
                       a.desc, a.blob, (const char*)a.x3, a.x, a.c, a.y, a.ld_in, a.ld_out, a.lp, a.part,
                       a.nparts, a.op_begin, a.op_end, a.N, a.seed, a.gen);
  else
    hipLaunchKernelGGL((flow_kernel_x3<K, NW, GT, PIPE, false>), dim3((unsigned)grid), dim3(NW * 64), lds, a.stream,
                       a.desc, a.blob, (const char*)a.x3, a.x, a.c, a.y, a.ld_in, a.ld_out, a.lp, a.part,
                       a.nparts, a.op_begin, a.op_end, a.N, a.seed, a.gen);
  ZF_CHECK_LAUNCH("flow_kernel_x3");
  return ZF_OK;
}

template <int K>
int launch_x3_k(const X3Launch& a, bool inverse) {
  switch (a.variant) {
    case 1: return launch_x3<K, 4, 1, 0>(a, inverse);  // 4 waves, 1-tile groups, 2 blocks per CU
    case 2: return launch_x3<K, 8, 2, 1>(a, inverse);  // 8 waves, half-blocks offset by one group
    case 3: return launch_x3<K, 8, 1, 1>(a, inverse);  // same with 1-tile groups
    case 4: return launch_x3<K, 4, 1, 2>(a, inverse);  // 4 waves, 3 blocks per CU
    default: return launch_x3<K, 8, 2, 0>(a, inverse); // 8 waves in lockstep
  }
}

int launch_flow_x3(const X3Launch& a, bool inverse) {
  if (a.K == 16) return launch_x3_k<16>(a, inverse);
  if (a.K == 8) return launch_x3_k<8>(a, inverse);
  return enotsup("bf16x3 kernel: knots must be 8 or 16");
}

#if ZF_X3_TRACE
extern "C" int zf_debug_x3_trace(unsigned long long* out, int* counts) {
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_x3_trace), sizeof(g_x3_trace));
  (void)hipMemcpyFromSymbol(counts, HIP_SYMBOL(g_x3_trace_n), sizeof(g_x3_trace_n));
  int z[32] = {0};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_x3_trace_n), z, sizeof(z));
  return 0;
}
#endif

size_t x3_lds_bytes(int variant, int small_floats, int D) {
  switch (variant) {
    case 1: return lds_bytes<4, 1, 0>(small_floats, D);
    case 2: return lds_bytes<8, 2, 1>(small_floats, D);
    case 3: return lds_bytes<8, 1, 1>(small_floats, D);
    case 4: return lds_bytes<4, 1, 2>(small_floats, D);
    default: return lds_bytes<8, 2, 0>(small_floats, D);
  }
}

int x3_group_tiles(int variant) { return (variant == 1 || variant == 3 || variant == 4) ? 1 : 2; }

}  // namespace zf
