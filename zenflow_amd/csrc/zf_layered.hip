// Layered eval path: Chain.__call__ / Chain.inverse / Flow.log_prob /
// Flow.sample (bijectors.py:103-116, flow.py:22-78) for flows whose
// conditioner the fused kernels cannot hold in registers and LDS — a hidden
// width above 256 (layer_utils.rect/tri build any width,
// layer_utils.py:6-18; NeuralSplineCoupling.layers, bijectors.py:318).
//
// Op by op over chunks of rows, every intermediate in HBM:
//   ShiftBounds        lay_sb_kernel       (zf_flow_dev.h sb_*_elem, the fused kernels' math)
//   NSC conditioner    lay_bn_kernel       hstack(xc, c) -> BatchNorm (eval: running stats)
//                      dense_gemm          Dense_0 + activation: the trainer's GEMMs (K <= 8: one
//                                          thread per 4 outputs), leaving the row maxima of its output
//                      dense_gemm_h2       Dense_l (l >= 1) + activation on f16x2 split MFMA with
//                                          per-row scales (gemm_h2_kernel below; K % 8 != 0 or
//                                          ZF_LAYERED_H2=0: the trainer's bf16x3 / fp32 GEMMs)
//                      dense_gemm_h2       last Dense -> raw spline parameters P [rows][dt][3K-1]
//   NSC spline         spline_rows         normalize_spline_params + RQ forward (log_det) / inverse
//   Roll               a rotation of the column index, no data movement
//   latent             lay_latent_kernel   log_prob + nan_to_num + the 128-row NLL partials
// Each Dense layer is a GEMM over the chunk's rows, so the weights are read
// once per 128 x 128 tile instead of once per 32-sample wave; the hidden
// activations cost 2 x 4 B x width per row and layer of HBM traffic, which
// the GEMMs' arithmetic intensity (2 x width flops per byte) covers.
//
// A handle's workspace is its own: calls on one handle are serialised by the
// caller (as every zf_flow_* call on one stream is).
#include "zf_flow_dev.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

namespace zf {

struct LayeredFlow {
  zf_flow_desc desc;     // with zf_flow_plan's natural offsets
  float* d_nat = nullptr;  // natural blob (FLAX layouts: Dense kernels [in][out])
  long long rows = 0;    // workspace capacity (rows)
  float *s0 = nullptr, *s1 = nullptr, *ld = nullptr, *U = nullptr, *Z = nullptr, *H0 = nullptr, *H1 = nullptr,
        *P = nullptr;
  unsigned *r0 = nullptr, *r1 = nullptr;  // max |row| of H0 / H1 (float bits) for dense_gemm_h2
  void* block = nullptr;  // one allocation holding the buffers above
  int hmax = 1, dcmax = 1, outmax = 1;
  // Dense layers l >= 1 on f16x2 split MFMA: per op, per layer, the packed
  // weights (pack_w_h2) and their scale exponent; d == nullptr: the layer
  // runs on dense_gemm (first layer, K % 8 != 0, or ZF_LAYERED_H2=0)
  struct H2W {
    void* d = nullptr;
    int kw = 0;
  };
  std::vector<std::vector<H2W>> h2;
  // One call at a time per handle: layered_run may grow (free + reallocate)
  // the workspace above, and every launch of a call reads its pointers, so
  // a second host thread on the same handle waits until the first has
  // enqueued all its launches (hipFree then waits for them on the device).
  std::mutex mu;
};

namespace {

constexpr long long kChunkFloats = 1ll << 26;  // per hidden-activation buffer (256 MiB)

__global__ void lay_sb_kernel(const float* __restrict__ x, float* __restrict__ y, float* __restrict__ ld,
                              const float* __restrict__ sb, int B, int D, int rot, int inverse) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float lsum = 0.f;
  for (int i = 0; i < D; ++i) {
    const int p = wrap(i + rot, D);
    const float v = x[(long long)b * D + p];
    if (inverse) {
      y[(long long)b * D + p] = sb_inverse_elem(sb + 8 * i, v);
    } else {
      float l;
      y[(long long)b * D + p] = sb_forward_elem(sb + 8 * i, v, l);
      lsum = lsum + l;
    }
  }
  if (!inverse) ld[b] = ld[b] + lsum;
}

// u = BatchNorm(hstack(xc, c)) with the packed [mean | mul | bias] rows of
// pack_nsc_bn (mul = rsqrt(var + eps) * scale), as the fused kernels' layer0.
__global__ void lay_bn_kernel(const float* __restrict__ s, const float* __restrict__ c, float* __restrict__ U,
                              const float* __restrict__ bn, int DCp, int B, int D, int C, int dt, int dc, int rot) {
  const int DC = dc + C;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)B * DC) return;
  const long long b = i / DC;
  const int k = (int)(i - b * DC);
  const float v = k < dc ? s[b * D + wrap(dt + k + rot, D)] : c[b * C + (k - dc)];
  U[i] = (v - bn[k]) * bn[DCp + k] + bn[2 * DCp + k];
}

// log_prob per row, and the sum of each 128-row block's log_prob in a fixed
// pairwise order into part[pbase + block] (zf_flow_nll_reduce's layout).
__global__ __launch_bounds__(128) void lay_latent_kernel(const float* __restrict__ s, const float* __restrict__ ld,
                                                         float* __restrict__ lp_out, double* __restrict__ part,
                                                         long long pbase, int B, int D, int rot, int lt, float c0,
                                                         float c1, float c2) {
  __shared__ double red[128];
  const int b = blockIdx.x * 128 + threadIdx.x;
  double v = 0.0;
  if (b < B) {
    float lat = 0.f;
    for (int j = 0; j < D; ++j) lat = lat + latent_logpdf(lt, c0, c1, c2, s[(long long)b * D + wrap(j + rot, D)]);
    const float lp = nan_to_num_lp(lat + ld[b]);
    if (lp_out) lp_out[b] = lp;
    v = (double)lp;
  }
  if (!part) return;
  red[threadIdx.x] = v;
  __syncthreads();
  for (int w = 64; w >= 1; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[pbase + blockIdx.x] = red[0];
}

// y[b][j] = state column of logical dim j (undoes the rotation)
__global__ void lay_out_kernel(const float* __restrict__ s, float* __restrict__ y, int B, int D, int rot) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)B * D) return;
  const long long b = i / D;
  const int j = (int)(i - b * D);
  y[i] = s[b * D + wrap(j + rot, D)];
}

// Flow.sample's latent draws: the generator and counters of zf_flow_sample
// (row = global row index), so both paths draw the same z.
__global__ void lay_draw_kernel(float* __restrict__ s, int B, long long row0, int D, int lt, float param,
                                unsigned long long seed) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)B * D) return;
  const long long b = i / D;
  const int d = (int)(i - b * D);
  s[i] = latent_draw(lt, param, seed, row0 + b, d);
}

// gemm_x3_kernel's tile geometry (zf_train.hip) and its XCD-aware tile order
constexpr int kX3BM = 128, kX3BN = 128, kX3BK = 32;
constexpr int kX3RS = 40;              // halfs per LDS row (32 k + 8 pad = 80 B)
// gemm_h2_kernel's LDS: ZF_H2_DB (default) double-buffers the k-tile stage
// (one barrier per k-tile instead of two) in 64-B rows whose 16-B chunks are
// XOR-swizzled by row bits 2-3 (16 lanes of a fragment read or a stage store
// hit 16 distinct 4-bank groups; the 80-B padded rows of one buffer would
// not leave room for two blocks per CU)
#ifndef ZF_H2_DB
#define ZF_H2_DB 1
#endif
constexpr bool kH2DB = ZF_H2_DB != 0;
// resident blocks per CU the kernel is built and launched for (tuning: 3
// needs the single-buffer stage's LDS and spills a few VGPRs)
#ifndef ZF_H2_OCC
#define ZF_H2_OCC 2
#endif
constexpr int kH2RS = kH2DB ? 32 : kX3RS;  // halfs per LDS row
constexpr int kH2Pl = 128 * kH2RS;         // halfs per plane
constexpr int kH2Buf = 4 * kH2Pl;          // one stage: A hi, A lo, B hi, B lo
__device__ __forceinline__ int h2_off(int row, int chunk) {
  return kH2DB ? row * 32 + 8 * (chunk ^ ((row >> 2) & 3)) : row * kX3RS + 8 * chunk;
}
typedef float tfloatx2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float sigmoidf(float z) { return 1.0f / (1.0f + expf(-z)); }

__device__ __forceinline__ int x3_tile(int ti, int ntiles) {
  const int b = blockIdx.x, G = gridDim.x;
  if ((G & 7) == 0 && ntiles % G == 0) return ti * G + (b & 7) * (G >> 3) + (b >> 3);
  return b + ti * G;
}

// ---- Eval-only Dense layers on f16x2 split MFMA (the layered path) ----------
// C / H = act(A . W + bias) for the layered eval path's Dense layers after
// the first, in the fused kernels' f16x2 scheme (zf_flow_x3_kernel.h) on a
// GEMM: row m of A is scaled by 2^(14 - e_m), e_m the frexp exponent of
// max |A[m][:]| (rin[m], float bits, left by A's producer), so its largest
// value lies in [2^13, 2^14); W was scaled by 2^kw and split once, on the
// host (layered_create: pack_w_h2); every operand is an RNE f16 hi + lo,
// three v_mfma_f32_32x32x16_f16 per k-step (lo.hi, hi.lo, hi.hi; lo.lo is
// below 2^-22 of the product) and the sum scaled back by 2^(e_m - 14 - kw),
// exactly.  Against gemm_x3_kernel: half the MFMAs, two LDS planes per
// operand instead of three, no weight split in the loop (the packed k-tile
// of W is one 16-KiB block copied to LDS).  Same tiles, waves, persistent
// two-deep staging and epilogue as gemm_x3_kernel; the epilogue also leaves
// max |output row| in rout (atomicMax of float bits, zeroed by the caller)
// for the next layer.  Eval only: training keeps bf16x3 (its gradients
// have no per-row scales to follow).
typedef _Float16 thalf8 __attribute__((ext_vector_type(8)));
typedef _Float16 thalf2 __attribute__((ext_vector_type(2)));
constexpr int kH2Tile = 2 * 128 * kX3BK;  // halfs per packed (n-tile, k-tile) block of W

// frexp exponent of a row max (float bits, non-negative): max in [2^(e-1), 2^e)
__device__ __forceinline__ int h2_row_exp(unsigned bits) {
  const int E = (int)((bits >> 23) & 0xff);
  return E == 0 ? -100 : E - 126;  // zero / subnormal rows: any scale keeps them exact enough
}

__device__ __forceinline__ void split2_store(const float (&x)[8], int sh, _Float16* p) {
  thalf8 hv, lv;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const tfloatx2 v = {ldexpf(x[2 * i], sh), ldexpf(x[2 * i + 1], sh)};
    const thalf2 vh = __builtin_convertvector(v, thalf2);
    const thalf2 vl = __builtin_convertvector(v - __builtin_convertvector(vh, tfloatx2), thalf2);
    hv[2 * i] = vh[0]; hv[2 * i + 1] = vh[1];
    lv[2 * i] = vl[0]; lv[2 * i + 1] = vl[1];
  }
  *reinterpret_cast<thalf8*>(p) = hv;
  *reinterpret_cast<thalf8*>(p + kH2Pl) = lv;
}

// max of x over each 16-lane DPP row (every lane of the row gets it)
__device__ __forceinline__ float h2_max16(float x) {
  auto step = [](float v, int ctrl) {
    const int o = ctrl == 0xB1   ? __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false)
                  : ctrl == 0x4E ? __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false)
                  : ctrl == 0x141 ? __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false)
                                  : __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false);
    return fmaxf(v, __int_as_float(o));
  };
  x = step(x, 0xB1);   // quad_perm [1, 0, 3, 2]
  x = step(x, 0x4E);   // quad_perm [2, 3, 0, 1]
  x = step(x, 0x141);  // row_half_mirror
  return step(x, 0x140);  // row_mirror
}

// The epilogue's activation.  SW: swish only — the act switch of every other
// activation, unrolled over the epilogue's 16 row pieces, made the kernel
// ~300 KB of code, fetched cold at every tile's epilogue.
// Swish with the hardware exp and reciprocal (~1 ulp each) instead of the
// IEEE divide: ~8 fewer VALU per value, a third of the epilogue (its error,
// a few 1e-7, is that of the f16x2 split the next layer applies anyway).
template <bool SW>
__device__ __forceinline__ float h2_act(int act, float v) {
  return SW || act == ZF_ACT_SWISH ? v * __builtin_amdgcn_rcpf(1.0f + __expf(-v)) : act_other(act, v);
}

template <bool WIDE, bool SW>
__global__ __launch_bounds__(256, ZF_H2_OCC) void gemm_h2_kernel(int M, int N, int K, const float* __restrict__ A, int lda,
                                                      const _Float16* __restrict__ Wp, const unsigned* __restrict__ rin,
                                                      int kw, float* __restrict__ C, int ldc,
                                                      const float* __restrict__ bias, float* __restrict__ H,
                                                      unsigned* __restrict__ rout, int act) {
  __shared__ __attribute__((aligned(16))) _Float16 lds[(kH2DB ? 2 : 1) * kH2Buf];
  __shared__ unsigned rowx[kX3BM];  // the tile's A-row maxima (float bits)
  __shared__ __attribute__((aligned(16))) float biasl[kX3BN];    // the tile's bias
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm0 = (wave >> 1) * 64, wn0 = (wave & 1) * 64;
  int m0 = 0, n0 = 0;
  const int r = lane & 31, h = lane >> 5;
  // One k-tile in registers, loaded two k-tiles ahead.  Every load is
  // unconditional (clamped addresses) and nothing is computed from a loaded
  // value until the stage is stored: a value used right after its load
  // (a select against zero, a scale from the row max) makes the compiler
  // wait for vmcnt(0) there — every older load too, the prefetch included.
  struct Stage {
    float4 ra[4];
    uint4 rb[4];
    unsigned rr[2];
    float bs;
  };
  const int tiles_n = (N + kX3BN - 1) / kX3BN;
  const int ntiles = tiles_n * ((M + kX3BM - 1) / kX3BM);
  // k-tiles per output tile, rounded up to even (pack_w_h2 zero-fills the
  // extra W block; its A k are past K and zeroed): the tile loop below runs
  // them as (S0, S1) pairs, so the epilogue is emitted once
  const int kt = ((K + kX3BK - 1) / kX3BK + 1) & ~1;
  const int mine = ntiles > (int)blockIdx.x ? (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x : 0;
  const int total = mine * kt;
  // A: thread -> rows (e >> 2) for e = tid, tid + 256, 8 k at 8 (e & 3) (rows past M
  // read row M - 1: their outputs are not stored; k past K are zeroed when stored),
  // with the rows' maxima; W: the packed block's 16 KiB as 4 dwordx4 per thread
  auto load = [&](int it, Stage& st) __attribute__((always_inline)) {
    const int ti = it / kt, kk = it - ti * kt, k0 = kk * kX3BK;
    const int tile = x3_tile(ti, ntiles);
    const int tmi = tile / tiles_n, tni = tile - tmi * tiles_n;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + 256 * i, row = min(tmi * kX3BM + (e >> 2), M - 1);
      const float* src = A + (long long)row * lda + min(k0 + 8 * (e & 3), K - 8);
      st.ra[2 * i] = *reinterpret_cast<const float4*>(src);
      st.ra[2 * i + 1] = *reinterpret_cast<const float4*>(src + 4);
      st.rr[i] = rin[row];
    }
    st.bs = bias[min(tni * kX3BN + (tid & 127), N - 1)];
    const uint4* wsrc = reinterpret_cast<const uint4*>(Wp + (long long)(tni * kt + kk) * kH2Tile);
#pragma unroll
    for (int q = 0; q < 4; ++q) st.rb[q] = wsrc[tid + 256 * q];
  };
  if (total == 0) return;
  // Straight-line staging: both stages loaded before the loop, the k-loop
  // body two k-steps (S0 then S1) with the refill unconditional.  Any path
  // that skips a refill (an `if` around a load or around the second k-step)
  // leaves the compiler's wait counting unsure which stage is newest, and it
  // then waits for all loads (vmcnt(0)) at every stage store: a one-deep
  // prefetch.
  Stage S0, S1;
  load(0, S0);
  load(min(1, total - 1), S1);
  floatx16 acc[2][2];
  auto epilogue = [&]() __attribute__((always_inline)) {
    if (WIDE) {
      float* T = reinterpret_cast<float*>(lds) + wave * (32 * 68);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int g = 0; g < 4; ++g)
            *reinterpret_cast<float4*>(T + r * 68 + 32 * j + 8 * g + 4 * h) =
                float4{acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const int row = 4 * t + (lane >> 4), c4 = lane & 15;
          const float4 v = *reinterpret_cast<const float4*>(T + row * 68 + 4 * c4);
          const int lr = wm0 + 32 * i + row, m = m0 + lr, n = n0 + wn0 + 4 * c4;
          const int us = h2_row_exp(rowx[lr]) - 14 - kw;
          const float4 b4 = *reinterpret_cast<const float4*>(biasl + wn0 + 4 * c4);
          float x[4] = {ldexpf(v.x, us) + b4.x, ldexpf(v.y, us) + b4.y, ldexpf(v.z, us) + b4.z,
                        ldexpf(v.w, us) + b4.w};
          float mx = 0.f;
          if (m < M && n < N) {
            const long long o = (long long)m * ldc + n;
            if (C) *reinterpret_cast<float4*>(C + o) = float4{x[0], x[1], x[2], x[3]};
            if (H) {
#pragma unroll
              for (int u = 0; u < 4; ++u) x[u] = h2_act<SW>(act, x[u]);
              *reinterpret_cast<float4*>(H + o) = float4{x[0], x[1], x[2], x[3]};
            }
            mx = fmaxf(fmaxf(fabsf(x[0]), fabsf(x[1])), fmaxf(fabsf(x[2]), fabsf(x[3])));
          }
          if (rout) {
            // max over the 16 lanes of one row piece (64 columns) by DPP within
            // the 16-lane row (quad xor 1, quad xor 2, half-row mirror, row
            // mirror: four VALU, no LDS permute), then one atomic per row and wave
            mx = h2_max16(mx);
            if (c4 == 0 && m < M) atomicMax(rout + m, __float_as_uint(mx));
          }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
      }
    } else {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int lr = wm0 + 32 * i + (q & 3) + 8 * (q >> 2) + 4 * h, m = m0 + lr;
          if (m >= M) continue;
          const int us = h2_row_exp(rowx[lr]) - 14 - kw;
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int n = n0 + wn0 + 32 * j + r;
            if (n >= N) continue;
            float v = ldexpf(acc[i][j][q], us) + biasl[wn0 + 32 * j + r];
            const long long o = (long long)m * ldc + n;
            if (C) C[o] = v;
            if (H) H[o] = v = h2_act<SW>(act, v);
            if (rout) atomicMax(rout + m, __float_as_uint(fabsf(v)));
          }
        }
    }
    __syncthreads();
  };
  auto kstep = [&](int it, int kk, Stage& S) __attribute__((always_inline)) {
    const int k0 = kk * kX3BK;
    _Float16* const Ap = lds + (kH2DB ? (it & 1) * kH2Buf : 0);  // this k-tile's stage buffer
    _Float16* const Bp = Ap + 2 * kH2Pl;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + 256 * i;
      const bool kok = k0 + 8 * (e & 3) < K;
      const float4 u = kok ? S.ra[2 * i] : float4{0.f, 0.f, 0.f, 0.f};
      const float4 w = kok ? S.ra[2 * i + 1] : float4{0.f, 0.f, 0.f, 0.f};
      const float x[8] = {u.x, u.y, u.z, u.w, w.x, w.y, w.z, w.w};
      split2_store(x, 14 - h2_row_exp(S.rr[i]), Ap + h2_off(e >> 2, e & 3));
      if ((e & 3) == 0) rowx[e >> 2] = S.rr[i];  // (every k-tile of the tile: the same values)
    }
    if (tid < kX3BN) biasl[tid] = S.bs;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      // packed block [plane][n 0..127][k 0..31]: dwordx4 f = tid + 256 q -> plane f >> 9,
      // row (f >> 2) & 127, k 8 (f & 3)
      const int f = tid + 256 * q;
      *reinterpret_cast<uint4*>(Bp + (f >> 9) * kH2Pl + h2_off((f >> 2) & 127, f & 3)) = S.rb[q];
    }
    __syncthreads();
    load(min(it + 2, total - 1), S);  // (the last two refills repeat a k-tile, unused)
#pragma unroll
    for (int s = 0; s < kX3BK / 16; ++s) {
      thalf8 af[2][2], bf[2][2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          af[i][t] = *reinterpret_cast<const thalf8*>(Ap + t * kH2Pl + h2_off(wm0 + 32 * i + r, 2 * s + h));
          bf[i][t] = *reinterpret_cast<const thalf8*>(Bp + t * kH2Pl + h2_off(wn0 + 32 * i + r, 2 * s + h));
        }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          auto mf = [&](int ta, int tb, const floatx16& c) {
            return WIDE ? __builtin_amdgcn_mfma_f32_32x32x16_f16(bf[j][tb], af[i][ta], c, 0, 0, 0)
                        : __builtin_amdgcn_mfma_f32_32x32x16_f16(af[i][ta], bf[j][tb], c, 0, 0, 0);
          };
          floatx16 c = mf(1, 0, acc[i][j]);  // (A term, B term): lo hi, hi lo, hi hi
          c = mf(0, 1, c);
          acc[i][j] = mf(0, 0, c);
        }
    }
    // single buffer: the next store overwrites this stage; double buffer: the
    // next store goes to the other one, which every wave finished reading
    // before passing this k-tile's barrier
    if (!kH2DB) __syncthreads();
  };
  int it = 0;
  for (int ti = 0; ti < mine; ++ti) {
    const int tile = x3_tile(ti, ntiles);
    m0 = (tile / tiles_n) * kX3BM;
    n0 = (tile - (tile / tiles_n) * tiles_n) * kX3BN;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = floatx16{0};
    for (int kk = 0; kk < kt; kk += 2, it += 2) {
      kstep(it, kk, S0);
      kstep(it + 1, kk + 1, S1);
    }
    if (kH2DB) __syncthreads();  // the epilogue's LDS transpose spans both stage buffers
    epilogue();
  }
}

int dense_gemm_h2(int M, int N, int K, const float* A, int lda, const void* Wp, const unsigned* rin, int kw,
                  float* C, int ldc, float* H, unsigned* rout, hipStream_t st, const float* bias, int act) {
  if (M <= 0 || N <= 0) return ZF_OK;
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (K % 8 != 0 || lda % 4 != 0 || !al16(A) || !al16(Wp) || !bias)
    return einval("dense_gemm_h2: K %% 8, 16-B aligned A rows and packed W, and a bias are required");
  if (rout) ZF_TRY_HIP(hipMemsetAsync(rout, 0, (size_t)M * sizeof(unsigned), st));
  const long long ntiles = (long long)((N + kX3BN - 1) / kX3BN) * ((M + kX3BM - 1) / kX3BM);
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const dim3 grid((unsigned)std::min<long long>(ntiles, (long long)ZF_H2_OCC * ncu));
  const bool wide = N % 4 == 0 && ldc % 4 == 0 && (!C || al16(C)) && (!H || al16(H));
  const _Float16* W = static_cast<const _Float16*>(Wp);
  const bool sw = act == ZF_ACT_SWISH || !H;  // no activation stored: the swish-only form
#define ZF_H2_LAUNCH(W_, S_)                                                                                    \
  hipLaunchKernelGGL((gemm_h2_kernel<W_, S_>), grid, dim3(256), 0, st, M, N, K, A, lda, W, rin, kw, C, ldc, bias, \
                     H, rout, act)
  if (wide) {
    if (sw) ZF_H2_LAUNCH(true, true);
    else ZF_H2_LAUNCH(true, false);
  } else {
    if (sw) ZF_H2_LAUNCH(false, true);
    else ZF_H2_LAUNCH(false, false);
  }
#undef ZF_H2_LAUNCH
  ZF_CHECK_LAUNCH("gemm_h2_kernel");
  return ZF_OK;
}

void pack_w_h2(const float* W, int K, int N, std::vector<uint16_t>& out, int& kw) {
  float mx = 0.f;
  for (long long i = 0; i < (long long)K * N; ++i) mx = std::max(mx, std::fabs(W[i]));
  int e = 0;
  (void)std::frexp(mx, &e);  // mx in [2^(e-1), 2^e)
  kw = (mx > 0.f && std::isfinite(mx)) ? 14 - e : 0;
  const int tn = (N + 127) / 128, tk = ((K + kX3BK - 1) / kX3BK + 1) & ~1;  // even (gemm_h2_kernel)
  out.assign((size_t)tn * tk * kH2Tile, 0);
  for (int a = 0; a < tn; ++a)
    for (int b = 0; b < tk; ++b) {
      uint16_t* blk = out.data() + ((size_t)a * tk + b) * kH2Tile;
      for (int n = 0; n < 128; ++n)
        for (int k = 0; k < kX3BK; ++k) {
          const int gn = a * 128 + n, gk = b * kX3BK + k;
          if (gn >= N || gk >= K) continue;
          const float v = std::ldexp(W[(long long)gk * N + gn], kw);
          const _Float16 hi = (_Float16)v;
          const _Float16 lo = (_Float16)(v - (float)hi);
          std::memcpy(blk + n * kX3BK + k, &hi, 2);
          std::memcpy(blk + 128 * kX3BK + n * kX3BK + k, &lo, 2);
        }
    }
}


inline unsigned nblocks(long long n, int t) { return (unsigned)((n + t - 1) / t); }

int ensure_rows(LayeredFlow* L, long long rows) {
  if (rows <= L->rows) return ZF_OK;
  if (L->block) (void)hipFree(L->block);
  L->block = nullptr;
  L->rows = 0;
  const int D = L->desc.dim;
  const long long per = 2ll * D + 1 + L->dcmax + 3ll * L->hmax + L->outmax + 2;  // floats per row
  ZF_TRY_HIP(hipMalloc(&L->block, (size_t)(per * rows) * sizeof(float)));
  float* p = static_cast<float*>(L->block);
  auto take = [&](long long n) { float* q = p; p += n * rows; return q; };
  L->s0 = take(D);
  L->s1 = take(D);
  L->ld = take(1);
  L->U = take(L->dcmax);
  L->Z = take(L->hmax);
  L->H0 = take(L->hmax);
  L->H1 = take(L->hmax);
  L->P = take(L->outmax);
  L->r0 = reinterpret_cast<unsigned*>(take(1));
  L->r1 = reinterpret_cast<unsigned*>(take(1));
  L->rows = rows;
  return ZF_OK;
}

}  // namespace

int layered_create(const zf_flow_desc& desc, const float* natural, int64_t n, LayeredFlow** out) {
  *out = nullptr;
  LayeredFlow* L = new LayeredFlow();
  L->desc = desc;
  for (int i = 0; i < desc.n_ops; ++i) {
    const zf_op_desc& op = desc.ops[i];
    if (op.kind != ZF_OP_NSC) continue;
    const int dt = desc.dim / 2, dc = desc.dim - dt;
    L->dcmax = std::max(L->dcmax, dc + desc.cond_dim);
    L->outmax = std::max(L->outmax, dt * (3 * op.knots - 1));
    for (int l = 0; l < op.n_hidden; ++l) L->hmax = std::max(L->hmax, op.hidden[l]);
  }
  hipError_t e = hipMalloc(&L->d_nat, (size_t)std::max<int64_t>(n, 1) * sizeof(float));
  if (e == hipSuccess && n > 0) e = hipMemcpy(L->d_nat, natural, (size_t)n * sizeof(float), hipMemcpyHostToDevice);
  static const bool h2_on = [] {
    const char* v = std::getenv("ZF_LAYERED_H2");
    return !(v && v[0] == '0');
  }();
  L->h2.resize(desc.n_ops);
  for (int i = 0; i < desc.n_ops && e == hipSuccess && h2_on; ++i) {
    const zf_op_desc& op = desc.ops[i];
    if (op.kind != ZF_OP_NSC) continue;
    const int dt = desc.dim / 2;
    L->h2[i].resize(op.n_hidden + 1);
    for (int l = 1; l <= op.n_hidden && e == hipSuccess; ++l) {
      const int K = op.hidden[l - 1], N = l == op.n_hidden ? dt * (3 * op.knots - 1) : op.hidden[l];
      if (K % 8 != 0) continue;
      std::vector<uint16_t> pk;
      pack_w_h2(natural + op.off_w[l], K, N, pk, L->h2[i][l].kw);
      e = hipMalloc(&L->h2[i][l].d, pk.size() * sizeof(uint16_t));
      if (e == hipSuccess) e = hipMemcpy(L->h2[i][l].d, pk.data(), pk.size() * sizeof(uint16_t), hipMemcpyHostToDevice);
    }
  }
  if (e != hipSuccess) {
    layered_destroy(L);
    return hip_status(e, "layered_create");
  }
  *out = L;
  return ZF_OK;
}

void layered_destroy(LayeredFlow* L) {
  if (!L) return;
  if (L->d_nat) (void)hipFree(L->d_nat);
  if (L->block) (void)hipFree(L->block);
  for (auto& v : L->h2)
    for (auto& w : v)
      if (w.d) (void)hipFree(w.d);
  delete L;
}

int layered_run(LayeredFlow* L, const DevFlow& F, const float* packed, bool inverse, int op_begin, int op_end,
                const float* x, const float* c, float* y, const float* ld_in, float* ld_out, float* lp, double* part,
                long long N, hipStream_t st, unsigned long long seed, int gen) {
  const zf_flow_desc& desc = L->desc;
  const int D = desc.dim, C = desc.cond_dim;
  std::lock_guard<std::mutex> lock(L->mu);
  // rows per chunk: a multiple of the 128-row NLL partial, every buffer of
  // the workspace (hidden activations, the conditioner input U, the spline
  // parameters P) within kChunkFloats, so each GEMM's M * N stays below 2^26
  const long long wmax = std::max<long long>({L->hmax, L->outmax, L->dcmax});
  long long R = std::max(128ll, (kChunkFloats / wmax) / 128 * 128);
  R = std::min(R, (N + 127) / 128 * 128);
  int rc = ensure_rows(L, R);
  if (rc) return rc;
  for (long long row0 = 0; row0 < N; row0 += R) {
    const int n = (int)std::min(R, N - row0);
    const float* cur;
    if (gen) {
      hipLaunchKernelGGL(lay_draw_kernel, dim3(nblocks((long long)n * D, 256)), dim3(256), 0, st, L->s1, n, row0, D,
                         F.latent, F.lat_c3, seed);
      ZF_CHECK_LAUNCH("lay_draw_kernel");
      cur = L->s1;
    } else {
      cur = x + row0 * D;
    }
    const float* cc = C > 0 ? c + row0 * C : nullptr;
    if (!inverse) {
      if (ld_in) ZF_TRY_HIP(hipMemcpyAsync(L->ld, ld_in + row0, n * sizeof(float), hipMemcpyDeviceToDevice, st));
      else ZF_TRY_HIP(hipMemsetAsync(L->ld, 0, n * sizeof(float), st));
    }
    int rot = 0;
    const int cnt = op_end - op_begin;
    for (int t = 0; t < cnt; ++t) {
      const int i = inverse ? op_end - 1 - t : op_begin + t;
      const zf_op_desc& op = desc.ops[i];
      const DevOp& d = F.ops[i];
      float* out = cur == L->s0 ? L->s1 : L->s0;
      if (op.kind == ZF_OP_ROLL) {
        rot = ((inverse ? rot + op.shift : rot - op.shift) % D + D) % D;
        continue;
      }
      if (op.kind == ZF_OP_SHIFT_BOUNDS) {
        hipLaunchKernelGGL(lay_sb_kernel, dim3(nblocks(n, 256)), dim3(256), 0, st, cur, out, L->ld, packed + d.sb, n,
                           D, rot, inverse ? 1 : 0);
        ZF_CHECK_LAUNCH("lay_sb_kernel");
        cur = out;
        continue;
      }
      // NeuralSplineCoupling (bijectors.py:321-371)
      const int DC = d.DC;
      hipLaunchKernelGGL(lay_bn_kernel, dim3(nblocks((long long)n * DC, 256)), dim3(256), 0, st, cur, cc, L->U,
                         packed + d.bn, 2 * d.KS0, n, D, C, d.dt, d.dc, rot);
      ZF_CHECK_LAUNCH("lay_bn_kernel");
      const float* in = L->U;
      int in_w = DC;
      auto h2w = [&](int l) -> const LayeredFlow::H2W* {
        return l < (int)L->h2[i].size() && L->h2[i][l].d ? &L->h2[i][l] : nullptr;
      };
      for (int l = 0; l <= op.n_hidden; ++l) {
        const bool last = l == op.n_hidden;
        const int out_w = last ? d.dt * d.S : op.hidden[l];
        float* H = (l & 1) ? L->H1 : L->H0;
        // the row maxima of H when the next layer runs on f16x2 (layer l writes
        // r0 / r1 by its parity, layer l reads those of layer l - 1)
        unsigned* rout = !last && h2w(l + 1) ? ((l & 1) ? L->r1 : L->r0) : nullptr;
        const unsigned* rin = (l & 1) ? L->r0 : L->r1;
        // hidden layers keep only the activation H (no pre-activation store: eval has no backward)
        if (const LayeredFlow::H2W* w = h2w(l))
          rc = dense_gemm_h2(n, out_w, in_w, in, in_w, w->d, rin, w->kw, last ? L->P : nullptr, out_w,
                             last ? nullptr : H, rout, st, L->d_nat + op.off_b[l], op.act);
        else
          rc = dense_gemm(n, n, out_w, in_w, in, in_w, L->d_nat + op.off_w[l], out_w, last ? L->P : nullptr, out_w,
                          last ? nullptr : H, st, L->d_nat + op.off_b[l], op.act, rout);
        if (rc) return rc;
        in = H;
        in_w = out_w;
      }
      rc = spline_rows(inverse, cur, out, L->P, L->ld, n, D, d.dt, op.knots, rot, st);
      if (rc) return rc;
      cur = out;
    }
    if (y) {
      hipLaunchKernelGGL(lay_out_kernel, dim3(nblocks((long long)n * D, 256)), dim3(256), 0, st, cur, y + row0 * D, n,
                         D, rot);
      ZF_CHECK_LAUNCH("lay_out_kernel");
    }
    if (!inverse && ld_out)
      ZF_TRY_HIP(hipMemcpyAsync(ld_out + row0, L->ld, n * sizeof(float), hipMemcpyDeviceToDevice, st));
    if (!inverse && (lp || part)) {
      hipLaunchKernelGGL(lay_latent_kernel, dim3(nblocks(n, 128)), dim3(128), 0, st, cur, L->ld,
                         lp ? lp + row0 : nullptr, part, row0 / 128, n, D, rot, F.latent, F.lat_c0, F.lat_c1,
                         F.lat_c2);
      ZF_CHECK_LAUNCH("lay_latent_kernel");
    }
  }
  return ZF_OK;
}

}  // namespace zf
