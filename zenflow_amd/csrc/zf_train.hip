// Training: train-mode forward with stored activations, the reverse pass
// (RQ spline, conditioner MLP, BatchNorm with batch statistics) and the
// optimiser update, for zenflow.train (src/zenflow/train.py:18-138):
//   loss_fn  (train.py:64-72): -mean(Flow.__call__(x, c, train=True))
//   step     (train.py:80-86): jax.grad -> optax (n)adamw update
// The path is op by op and unfused (a training batch is 10^3-10^5 rows; the
// weights change every step, so the fused inference kernels' packed weight
// layouts would have to be rebuilt each step).  GEMMs are an LDS-tiled fp32
// kernel; everything else is per-row elementwise / per-column reductions.
// All parameters and gradients live in the natural FLAX blob layout of
// zf_flow_plan on the device.
#include "zf_act.h"
#include "zf_internal.h"
#include "zf_spline.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <cstdlib>
#include <map>
#include <vector>

namespace zf {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr float kBnEps = 1e-5f;     // flax.linen.BatchNorm epsilon
constexpr float kBnMomentum = 0.99f; // flax.linen.BatchNorm momentum
constexpr float kEpsT = 1e-5f;       // utils.py:15

__host__ __device__ __forceinline__ int pmodi(int a, int m) {
  int r = a % m;
  return r < 0 ? r + m : r;
}

// ---- GEMM on fp32 MFMA: C[M,N] = op(A)[M,K] . op(B)[K,N], row-major ----------
// v_mfma_f32_32x32x2_f32 is a k-ordered f32 fma chain (exact f32, the same
// numerics as a scalar fmaf loop).  Block tile BM x BN x 32 staged through LDS
// (k-major, +1 padding: the transposing stores are conflict-free), 4 waves in
// 2 x 2, each (BM/2) x (BN/2) as 32 x 32 MFMA tiles; the next k-tile's global
// loads are in flight in registers while the current one is multiplied.
// Epilogues fused into the store:
//   kEpiNone   C = acc
//   kEpiBias   z = acc + bias[n]; C = z; H = act(z) if H (flax.linen.swish, or
//              the op's other activation, zf_act.h)
//   kEpiDSwish C = acc * act'(Z[m, n])  (gradient through the activation)
// WG (weight gradients, split-K over the batch): block z multiplies rows
// [z*KC, (z+1)*KC) into part[z][M+1][N]; row M is the bias gradient, the
// column sums of the B tile (op(B) = layer-output gradient), which blocks with
// blockIdx.y == 0 form on the VALU beside the MFMAs.
constexpr int MBK = 32;
enum { kEpiNone = 0, kEpiBias = 1, kEpiDSwish = 2 };

__device__ __forceinline__ float sigmoidf(float z) { return 1.0f / (1.0f + expf(-z)); }

// The fused store of one output element (both GEMM forms below).
__device__ __forceinline__ void gemm_epilogue(float v, int n, long long o, float* __restrict__ C, int epi,
                                              const float* __restrict__ bias, float* __restrict__ H,
                                              const float* __restrict__ Z, int act) {
  if (epi == kEpiBias) {
    v = v + bias[n];
    if (H) H[o] = act == ZF_ACT_SWISH ? v * sigmoidf(v) : act_other(act, v);
  } else if (epi == kEpiDSwish) {
    const float z = Z[o];
    if (act == ZF_ACT_SWISH) {
      const float sg = sigmoidf(z);
      v = v * (sg + z * sg * (1.0f - sg));
    } else {
      v = v * act_other_grad(act, z);
    }
  }
  if (C) C[o] = v;  // null: the eval path keeps only the activation H
}

// The same for four consecutive columns n..n+3 (n % 4 == 0 < N, N % 4 == 0,
// 16-B aligned rows): one dwordx4 per array instead of four dword stores.
__device__ __forceinline__ void gemm_epilogue4(float4 v, int n, long long o, float* __restrict__ C, int epi,
                                               const float* __restrict__ bias, float* __restrict__ H,
                                               const float* __restrict__ Z, int act) {
  float x[4] = {v.x, v.y, v.z, v.w};
  if (epi == kEpiBias) {
    // four scalar loads: a Dense bias inside the natural blob need not be
    // 16-B aligned (the layered path's biases alternate), and the WIDE
    // epilogue should not depend on it
    x[0] = x[0] + bias[n];
    x[1] = x[1] + bias[n + 1];
    x[2] = x[2] + bias[n + 2];
    x[3] = x[3] + bias[n + 3];
    if (H) {
      float y[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) y[t] = act == ZF_ACT_SWISH ? x[t] * sigmoidf(x[t]) : act_other(act, x[t]);
      *reinterpret_cast<float4*>(H + o) = float4{y[0], y[1], y[2], y[3]};
    }
  } else if (epi == kEpiDSwish) {
    const float4 z4 = *reinterpret_cast<const float4*>(Z + o);
    const float z[4] = {z4.x, z4.y, z4.z, z4.w};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (act == ZF_ACT_SWISH) {
        const float sg = sigmoidf(z[t]);
        x[t] = x[t] * (sg + z[t] * sg * (1.0f - sg));
      } else {
        x[t] = x[t] * act_other_grad(act, z[t]);
      }
    }
  }
  if (C) *reinterpret_cast<float4*>(C + o) = float4{x[0], x[1], x[2], x[3]};
}

// SPLITQ: block z = q of a 64 x 64 tile multiplies only the k-pairs
// p = q (mod 4) — exactly accumulator set q of the NACC = 4 kernel, in the
// same order (trailing all-zero pairs aside, which only turn -0 into +0) —
// into part[q][M][N]; gemm_combine_kernel then forms
// (P0 + P1) + (P2 + P3) and the epilogue: the same bits from four times the
// blocks (small batches: 1024 rows give 32 tiles for 256 CUs).
// The block body, with the block's coordinates passed in (mgemm_kernel: its
// blockIdx; wgrad_group_kernel: decoded from one launch over several GEMMs).
// SW: no activation but swish in the epilogue (its code only; the generic
// form's act switch made the 128 x 128 kernel ~255 KB, fetched cold at
// every epilogue)
template <int BM, int BN, bool TA, bool TB, bool WG, bool SPLITQ, bool SW = false>
__device__ __forceinline__ void mgemm_body(const uint3 bid, int M, int N, int K, const float* __restrict__ A, int lda,
                                           const float* __restrict__ B, int ldb, float* __restrict__ C, int ldc,
                                           int epi, const float* __restrict__ bias, float* __restrict__ H,
                                           const float* __restrict__ Z, int KC, int act) {
  constexpr int NA = BM * MBK / 256, NB = BN * MBK / 256;  // tile elements per thread
  constexpr int TM = BM / 64, TN = BN / 64;                // 32x32 tiles per wave
  __shared__ float As[MBK][BM + 1];
  __shared__ float Bs[MBK][BN + 1];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm0 = (wave >> 1) * (BM / 2), wn0 = (wave & 1) * (BN / 2);
  const int m0 = bid.y * BM, n0 = bid.x * BN;
  const int kbeg = WG ? bid.z * KC : 0;
  // SPLITQ: block q runs a virtual k range holding only its k-pairs
  // p = q, q + 4, q + 8, ... (virtual pair v = real pair 4 v + q), so one
  // k-tile of loads serves 16 of its pairs instead of 4
  const int q4 = SPLITQ ? (int)bid.z : 0;
  const int kend = WG ? min(K, kbeg + KC) : SPLITQ ? 2 * max(0, ((K + 1) / 2 - q4 + 3) / 4) : K;
  auto real_k = [&](int k) { return SPLITQ ? 2 * (4 * (k >> 1) + q4) + (k & 1) : k; };
  const int kmax = SPLITQ ? K : kend;
  float ra[NA], rb[NB];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int e = tid + 256 * i;
      const int mm = TA ? (e % BM) : (e / MBK), kk = TA ? (e / BM) : (e % MBK);
      const int m = m0 + mm, k = real_k(k0 + kk);
      ra[i] = (m < M && k0 + kk < kend && k < kmax) ? (TA ? A[(long long)k * lda + m] : A[(long long)m * lda + k])
                                                    : 0.f;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int e = tid + 256 * i;
      const int nn = TB ? (e / MBK) : (e % BN), kk = TB ? (e % MBK) : (e / BN);
      const int n = n0 + nn, k = real_k(k0 + kk);
      rb[i] = (n < N && k0 + kk < kend && k < kmax) ? (TB ? B[(long long)n * ldb + k] : B[(long long)k * ldb + n])
                                                    : 0.f;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int e = tid + 256 * i;
      As[TA ? (e / BM) : (e % MBK)][TA ? (e % BM) : (e / MBK)] = ra[i];
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int e = tid + 256 * i;
      Bs[TB ? (e % MBK) : (e / BN)][TB ? (e / MBK) : (e % BN)] = rb[i];
    }
  };
  // NACC interleaved accumulator sets (k-pair s goes to set s % NACC),
  // summed pairwise at the end: a 256-long fp32 fma chain becomes four
  // 64-long ones (the input-gradient and forward GEMMs run K up to 256;
  // the weight-gradient chunks are 32 rows).
  constexpr int NACC = (WG || SPLITQ || TM * TN > 1) ? 1 : 4;  // 128-wide tiles: registers for one set only
  floatx16 acc[NACC][TM][TN];
#pragma unroll
  for (int q = 0; q < NACC; ++q)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[q][i][j] = floatx16{0};
  // bias-gradient column sums (WG, bid.y == 0): column cc, k-quarter cq
  constexpr int CQ = 256 / BN, CK = MBK / CQ;
  const int cc = tid % BN, cq = tid / BN;
  float csum = 0.f;
  const bool do_cs = WG && bid.y == 0;
  const int r = lane & 31, h = lane >> 5;
  if (kbeg < kend) load(kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += MBK) {
    store();
    __syncthreads();
    if (k0 + MBK < kend) load(k0 + MBK);
#pragma unroll
    for (int kb = 0; kb < MBK; kb += 2) {
      float a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = As[kb + h][wm0 + 32 * i + r];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = Bs[kb + h][wn0 + 32 * j + r];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[(kb / 2) % NACC][i][j] =
              __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[(kb / 2) % NACC][i][j], 0, 0, 0);
    }
    if (do_cs) {
#pragma unroll
      for (int kk = 0; kk < CK; ++kk) csum += Bs[cq * CK + kk][cc];
    }
    __syncthreads();
  }
  if constexpr (NACC > 1) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[0][i][j] = NACC == 4 ? (acc[0][i][j] + acc[1][i][j]) + (acc[2][i][j] + acc[3][i][j])
                                 : acc[0][i][j] + acc[1][i][j];
  }
  if (SPLITQ) {
    float* P = C + (long long)bid.z * M * N;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int m = m0 + wm0 + (q & 3) + 8 * (q >> 2) + 4 * h, n = n0 + wn0 + r;
      if (m < M && n < N) P[(long long)m * N + n] = acc[0][0][0][q];
    }
    return;
  }
  if (WG) {
    float* P = C + (long long)bid.z * (M + 1) * N;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int m = m0 + wm0 + 32 * i + (q & 3) + 8 * (q >> 2) + 4 * h, n = n0 + wn0 + 32 * j + r;
          if (m < M && n < N) P[(long long)m * N + n] = acc[0][i][j][q];
        }
    if (do_cs) {
      float* red = &As[0][0];  // free after the loop's last barrier
      red[cq * BN + cc] = csum;
      __syncthreads();
      if (cq == 0 && n0 + cc < N) {
        float v = red[cc];
        for (int q = 1; q < CQ; ++q) v = v + red[q * BN + cc];
        P[(long long)M * N + n0 + cc] = v;
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int m = m0 + wm0 + 32 * i + (q & 3) + 8 * (q >> 2) + 4 * h, n = n0 + wn0 + 32 * j + r;
        if (m < M && n < N)
          gemm_epilogue(acc[0][i][j][q], n, (long long)m * ldc + n, C, epi, bias, H, Z, SW ? ZF_ACT_SWISH : act);
      }
}


template <int BM, int BN, bool TA, bool TB, bool WG, bool SPLITQ = false, bool SW = false>
__global__ __launch_bounds__(256) void mgemm_kernel(int M, int N, int K, const float* __restrict__ A, int lda,
                                                    const float* __restrict__ B, int ldb, float* __restrict__ C,
                                                    int ldc, int epi, const float* __restrict__ bias,
                                                    float* __restrict__ H, const float* __restrict__ Z, int KC,
                                                    int act) {
  mgemm_body<BM, BN, TA, TB, WG, SPLITQ, SW>(uint3{blockIdx.x, blockIdx.y, blockIdx.z}, M, N, K, A, lda, B, ldb, C,
                                             ldc, epi, bias, H, Z, KC, act);
}

__global__ void gemm_combine_kernel(int M, int N, const float* __restrict__ P, float* __restrict__ C, int ldc,
                                    int epi, const float* __restrict__ bias, float* __restrict__ H,
                                    const float* __restrict__ Z, int act) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long MN = (long long)M * N;
  if (i >= MN) return;
  const int m = (int)(i / N), n = (int)(i - (long long)m * N);
  const float v = (P[i] + P[MN + i]) + (P[2 * MN + i] + P[3 * MN + i]);
  gemm_epilogue(v, n, (long long)m * ldc + n, C, epi, bias, H, Z, act);
}

// C = A . B for K <= 8 (the first Dense of a coupling: K = dc + C inputs),
// one thread per output, with the arithmetic of the 64 x 64 interleaved
// MFMA kernel: k-pair p into set p mod 4 as fma(a1, b1, fma(a0, b0, s)) (the
// f32 MFMA's k-ordered fma chain), the tile's all-zero pairs as s + 0 (they
// only turn -0 into +0), then (s0 + s1) + (s2 + s3) and the same epilogue.
// The MFMA kernel would run 32 blocks of one mostly empty k-tile.
__global__ void gemm_small_k_kernel(int M, int N, int K, const float* __restrict__ A, int lda,
                                    const float* __restrict__ B, int ldb, float* __restrict__ C, int ldc, int epi,
                                    const float* __restrict__ bias, float* __restrict__ H,
                                    const float* __restrict__ Z, int act) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)M * N) return;
  const int m = (int)(i / N), n = (int)(i - (long long)m * N);
  float sq[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int k = 2 * p;
    if (k < K) {
      const float a0 = A[(long long)m * lda + k], b0 = B[(long long)k * ldb + n];
      const float a1 = k + 1 < K ? A[(long long)m * lda + k + 1] : 0.f;
      const float b1 = k + 1 < K ? B[(long long)(k + 1) * ldb + n] : 0.f;
      sq[p] = __builtin_fmaf(a1, b1, __builtin_fmaf(a0, b0, sq[p]));
    }
  }
  const float v = (__fadd_rn(sq[0], 0.f) + __fadd_rn(sq[1], 0.f)) + (__fadd_rn(sq[2], 0.f) + __fadd_rn(sq[3], 0.f));
  gemm_epilogue(v, n, (long long)m * ldc + n, C, epi, bias, H, Z, act);
}

// gemm_small_k_kernel with four consecutive outputs of kSk4Rows rows per
// thread (N % 4 == 0, 16-B aligned C / H rows): the same fma order per
// output (the same bits), the B columns and bias read once for all rows,
// and one dwordx4 store per array and row.  Grid (ceil(N / 256),
// ceil(M / (4 kSk4Rows))), block (64, 4): no per-thread division.
constexpr int kSk4Rows = 8;
__global__ __launch_bounds__(256) void gemm_small_k4_kernel(int M, int N, int K, const float* __restrict__ A, int lda,
                                     const float* __restrict__ B, int ldb, float* __restrict__ C, int ldc, int epi,
                                     const float* __restrict__ bias, float* __restrict__ H, int act,
                                     unsigned* __restrict__ rmax) {
  const int m0 = (blockIdx.y * 4 + threadIdx.y) * kSk4Rows;
  const int n = 4 * (blockIdx.x * 64 + threadIdx.x);
  if (m0 >= M) return;  // uniform per wave (a wave is one threadIdx.y)
  const bool nok = n < N;
  if (!nok && !rmax) return;
  float b[8][4], bs[4];
#pragma unroll
  for (int k = 0; k < 8; ++k)
#pragma unroll
    for (int t = 0; t < 4; ++t) b[k][t] = nok && k < K ? B[(long long)k * ldb + n + t] : 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t) bs[t] = nok && epi == kEpiBias ? bias[n + t] : 0.f;
  for (int r = 0; r < kSk4Rows; ++r) {
    const int m = m0 + r;
    if (m >= M) break;
    // (a lane past the last column, kept for the row max, multiplies zeros and stores nothing)
    float a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = k < K ? A[(long long)m * lda + k] : 0.f;
    float out[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float sq[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int k = 2 * p;
        if (k < K) sq[p] = __builtin_fmaf(a[k + 1], b[k + 1][t], __builtin_fmaf(a[k], b[k][t], sq[p]));
      }
      float v = (__fadd_rn(sq[0], 0.f) + __fadd_rn(sq[1], 0.f)) + (__fadd_rn(sq[2], 0.f) + __fadd_rn(sq[3], 0.f));
      if (epi == kEpiBias) v = v + bs[t];
      out[t] = v;
    }
    const long long o = (long long)m * ldc + n;
    float mx = 0.f;
    if (epi == kEpiBias && H) {
      float y[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) y[t] = act == ZF_ACT_SWISH ? out[t] * sigmoidf(out[t]) : act_other(act, out[t]);
      if (nok) *reinterpret_cast<float4*>(H + o) = float4{y[0], y[1], y[2], y[3]};
      if (rmax && nok) mx = fmaxf(fmaxf(fabsf(y[0]), fabsf(y[1])), fmaxf(fabsf(y[2]), fabsf(y[3])));
    } else if (rmax && nok) {
      mx = fmaxf(fmaxf(fabsf(out[0]), fabsf(out[1])), fmaxf(fabsf(out[2]), fabsf(out[3])));
    }
    if (C && nok) *reinterpret_cast<float4*>(C + o) = float4{out[0], out[1], out[2], out[3]};
    if (rmax) {
      // max |row piece| over the wave's 256 columns by DPP (within each
      // 16-lane row, then row_bcast:15 / row_bcast:31 into lane 63: VALU
      // only, no LDS permutes), one atomic per row and wave
#define ZF_DMAX(CTRL, ROWS) \
  mx = fmaxf(mx, __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(mx), __float_as_int(mx), CTRL, ROWS, 0xF, false)))
      ZF_DMAX(0xB1, 0xF);   // quad_perm [1, 0, 3, 2]
      ZF_DMAX(0x4E, 0xF);   // quad_perm [2, 3, 0, 1]
      ZF_DMAX(0x141, 0xF);  // row_half_mirror
      ZF_DMAX(0x140, 0xF);  // row_mirror: every lane has its 16-lane row's max
      ZF_DMAX(0x142, 0xA);  // row_bcast:15 into rows 1 and 3
      ZF_DMAX(0x143, 0xC);  // row_bcast:31 into rows 2 and 3: lane 63 has the wave's max
#undef ZF_DMAX
      if (threadIdx.x == 63) atomicMax(rmax + m, __float_as_uint(mx));
    }
  }
}

// ---- Large-batch GEMMs on bf16x3 split MFMA ----------------------------------
// C = A . op(B) (A row-major [M][K]; B row-major [K][N], or [N][K] when TB)
// with every fp32 operand split into three RNE bf16 terms (x = hi + mid + lo)
// and six v_mfma_f32_32x32x16_bf16 products per k-step, small terms first —
// an fp32 dot product to ~1e-7 relative (the inference kernels' bf16x3
// scheme, zf_flow_x3_kernel.h), at 419 TFLOP/s fp32-equivalent peak against
// the fp32 MFMA's 157.  Block tile 128 x 128 x 32, 4 waves in 2 x 2, each
// 64 x 64 as 2 x 2 MFMA tiles.  The split is done once per element, when a
// k-tile is stored to LDS: LDS holds three bf16 planes of A ([m][k]) and of
// B ([n][k]), rows of 32 k padded to 80 B (the 16 rows of a ds_read_b128
// lane group land on 16 distinct 4-bank slots), so the inner loop is
// fragment reads and MFMAs only.  The next k-tile's global loads are in
// flight in registers while the current one is multiplied; 60 KiB of LDS ->
// 2 blocks per CU.  K % 8 == 0 (a ragged last k-tile is zero-filled).
// Epilogue: when N and the output rows allow it (WIDE), B is the MFMA's
// first operand, so a lane holds one output row's 4 consecutive columns per
// register group (same products, same sums, same bits); the tile goes
// through LDS and leaves as row-contiguous dwordx4 stores, whole 128-B lines.
// The MFMA layout's 64 dword stores per lane were store-issue-bound: cfg5's
// hidden layer 111 us with them, 70 us with dwordx4 row pieces
// (tests/hip/gemm_probe.hip).  Same epilogues as mgemm_kernel.  Used when
// the GLOBAL batch gives >= 512 such blocks; ZF_TRAIN_X3=0 keeps the fp32
// kernel.
typedef __bf16 tbf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 tbf16x2 __attribute__((ext_vector_type(2)));
typedef float tfloatx2 __attribute__((ext_vector_type(2)));
constexpr int kX3BM = 128, kX3BN = 128, kX3BK = 32;
constexpr int kX3RS = 40;                       // bf16 per LDS row (32 k + 8 pad = 80 B)
constexpr int kX3Plane = 128 * kX3RS;           // bf16 per plane

// three RNE bf16 terms of 8 fp32 values, stored to the three planes at p
__device__ __forceinline__ void split3_store(const float (&x)[8], __bf16* p) {
  tbf16x8 h, m, l;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const tfloatx2 v = {x[2 * i], x[2 * i + 1]};
    const tbf16x2 vh = __builtin_convertvector(v, tbf16x2);
    const tfloatx2 r = v - __builtin_convertvector(vh, tfloatx2);
    const tbf16x2 vm = __builtin_convertvector(r, tbf16x2);
    const tfloatx2 r2 = r - __builtin_convertvector(vm, tfloatx2);
    const tbf16x2 vl = __builtin_convertvector(r2, tbf16x2);
    h[2 * i] = vh[0]; h[2 * i + 1] = vh[1];
    m[2 * i] = vm[0]; m[2 * i + 1] = vm[1];
    l[2 * i] = vl[0]; l[2 * i + 1] = vl[1];
  }
  *reinterpret_cast<tbf16x8*>(p) = h;
  *reinterpret_cast<tbf16x8*>(p + kX3Plane) = m;
  *reinterpret_cast<tbf16x8*>(p + 2 * kX3Plane) = l;
}

// The output tile of a persistent block's ti-th round.  Blocks go to the 8
// XCDs round-robin (block b -> XCD b % 8), each XCD with its own L2; when
// every round is full (gridDim % 8 == 0, ntiles % gridDim == 0) a round's
// tiles are dealt in runs of gridDim / 8 consecutive tiles per XCD, so the
// N-tiles of one row band (the same A rows) share an L2 instead of fetching
// the rows once per XCD.  Which block computes a tile changes nothing else.
__device__ __forceinline__ int x3_tile(int ti, int ntiles) {
  const int b = blockIdx.x, G = gridDim.x;
  if ((G & 7) == 0 && ntiles % G == 0) return ti * G + (b & 7) * (G >> 3) + (b >> 3);
  return b + ti * G;
}

template <bool TB, bool WIDE, bool SW>
__global__ __launch_bounds__(256, 2) void gemm_x3_kernel(int M, int N, int K, const float* __restrict__ A, int lda,
                                                      const float* __restrict__ B, int ldb, float* __restrict__ C,
                                                      int ldc, int epi, const float* __restrict__ bias,
                                                      float* __restrict__ H, const float* __restrict__ Z, int act) {
  __shared__ __attribute__((aligned(16))) __bf16 lds[6 * kX3Plane];
  __bf16* const Ap = lds;
  __bf16* const Bp = lds + 3 * kX3Plane;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm0 = (wave >> 1) * 64, wn0 = (wave & 1) * 64;
  int m0 = 0, n0 = 0;  // the current output tile (the loop below)
  const int r = lane & 31, h = lane >> 5;
  // Register staging of one k-tile: A rows (and B rows when TB) as float4s,
  // B columns as scalars (!TB).  Two sets, filled two k-tiles ahead of the
  // MFMAs that consume them — across output-tile boundaries too, so neither
  // a tile's first k-tile nor any other waits on a full memory latency
  // (one set, one k-tile ahead: Dense 512 x 512 at 0.31 of the MFMA rate).
  struct Stage {
    float4 ra[4], rb[4];
    float rbs[16];
  };
  // Every load is unconditional, from a clamped address, and nothing is
  // computed from a loaded value until its stage is stored: a select right
  // after a load (`ok ? x : 0`) makes the compiler wait for vmcnt(0) there,
  // for the prefetch too.  Rows past M / columns past N read the last one
  // (their outputs are not stored); k past K are zeroed when stored.
  // row-major [rows][K] tiles (A; B when TB): thread -> row e >> 2 (e = tid,
  // tid + 256), 8 consecutive k at 8 (e & 3) as two float4s
  auto load_rows = [&](const float* P, int ld, int r0, int R, int k0, float4 (&v)[4]) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + 256 * i, row = min(r0 + (e >> 2), R - 1);
      const float* src = P + (long long)row * ld + min(k0 + 8 * (e & 3), K - 8);
      v[2 * i] = *reinterpret_cast<const float4*>(src);
      v[2 * i + 1] = *reinterpret_cast<const float4*>(src + 4);
    }
  };
  auto store_rows = [&](__bf16* P, const float4 (&v)[4], int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + 256 * i;
      const bool kok = k0 + 8 * (e & 3) < K;
      const float4 u = kok ? v[2 * i] : float4{0.f, 0.f, 0.f, 0.f};
      const float4 w = kok ? v[2 * i + 1] : float4{0.f, 0.f, 0.f, 0.f};
      const float x[8] = {u.x, u.y, u.z, u.w, w.x, w.y, w.z, w.w};
      split3_store(x, P + (e >> 2) * kX3RS + 8 * (e & 3));
    }
  };
  // B row-major [K][N] (!TB): thread -> column n0 + (tid & 127), k 16 (tid >> 7) .. +15
  auto load_cols = [&](int tn0, int k0, float (&v)[16]) {
    const int n = min(tn0 + (tid & 127), N - 1);
    const int kb = k0 + 16 * (tid >> 7);
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = B[(long long)min(kb + j, K - 1) * ldb + n];
  };
  auto store_cols = [&](const float (&v)[16], int k0) {
    __bf16* P = Bp + (tid & 127) * kX3RS + 16 * (tid >> 7);
    const int kb = k0 + 16 * (tid >> 7);
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      float x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = kb + 8 * g + u < K ? v[8 * g + u] : 0.f;
      split3_store(x, P + 8 * g);
    }
  };
  // persistent blocks: a block takes output tiles blockIdx.x, + gridDim.x,
  // ...; a tile's epilogue stores drain while the next tile's loads and
  // MFMAs run (one launch round of blocks had every block storing at once).
  // The block's k-tiles in order: iteration it = tile ti (the ti-th of this
  // block) x kt k-tiles + k-tile kk.
  const int tiles_n = (N + kX3BN - 1) / kX3BN;
  const int ntiles = tiles_n * ((M + kX3BM - 1) / kX3BM);
  // k-tiles per output tile, rounded up to even (an odd K / 32's extra
  // k-tile is past K: zeroed when stored) so the tile loop below runs them
  // as (S0, S1) pairs and the epilogue is emitted once (three inlined
  // copies of the generic epilogue made the kernel too big for the
  // instruction cache; SW, swish couplings, leaves out the other
  // activations' code)
  const int kt = ((K + kX3BK - 1) / kX3BK + 1) & ~1;
  const int mine = ntiles > (int)blockIdx.x ? (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x : 0;
  const int total = mine * kt;
  auto load = [&](int it, Stage& st) __attribute__((always_inline)) {
    const int ti = it / kt, k0 = (it - ti * kt) * kX3BK;
    const int tile = x3_tile(ti, ntiles);
    const int tm0 = (tile / tiles_n) * kX3BM, tn0 = (tile - (tile / tiles_n) * tiles_n) * kX3BN;
    load_rows(A, lda, tm0, M, k0, st.ra);
    if (TB) load_rows(B, ldb, tn0, N, k0, st.rb);
    else load_cols(tn0, k0, st.rbs);
  };
  if (total == 0) return;
  // Straight-line staging (gemm_h2_kernel, zf_layered.hip): both stages
  // loaded before the loop, two k-steps per iteration with unconditional
  // refills, an odd last k-step after it — a skipped refill on any path
  // leaves the compiler unsure which stage is newest, and it then waits for
  // every load at each stage store (Dense 512 x 512 eval: 1.4x faster).
  Stage S0, S1;
  load(0, S0);
  load(min(1, total - 1), S1);
  floatx16 acc[2][2];
  auto epilogue = [&]() __attribute__((always_inline)) {
    if (WIDE) {
      // through LDS (free after the loop's last barrier), per wave and per
      // 32-row half: ds_write_b128 of each lane's row pieces (row pitch 68
      // floats: conflict-free), then row-contiguous float4s — each store
      // instruction writes 4 rows x 256 B, whole 128-B lines
      float* T = reinterpret_cast<float*>(lds) + wave * (32 * 68);
  #pragma unroll
      for (int i = 0; i < 2; ++i) {
  #pragma unroll
        for (int j = 0; j < 2; ++j)
  #pragma unroll
          for (int g = 0; g < 4; ++g)
            *reinterpret_cast<float4*>(T + r * 68 + 32 * j + 8 * g + 4 * h) =
                float4{acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's own LDS writes
        __builtin_amdgcn_wave_barrier();
  #pragma unroll
        for (int t = 0; t < 8; ++t) {
          const int row = 4 * t + (lane >> 4), c4 = lane & 15;
          const float4 v = *reinterpret_cast<const float4*>(T + row * 68 + 4 * c4);
          const int m = m0 + wm0 + 32 * i + row, n = n0 + wn0 + 4 * c4;
          if (m < M && n < N) gemm_epilogue4(v, n, (long long)m * ldc + n, C, epi, bias, H, Z, SW ? ZF_ACT_SWISH : act);
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
      }
    } else {
  #pragma unroll
      for (int i = 0; i < 2; ++i)
  #pragma unroll
        for (int j = 0; j < 2; ++j)
  #pragma unroll
          for (int q = 0; q < 16; ++q) {
            const int m = m0 + wm0 + 32 * i + (q & 3) + 8 * (q >> 2) + 4 * h, n = n0 + wn0 + 32 * j + r;
            if (m < M && n < N)
              gemm_epilogue(acc[i][j][q], n, (long long)m * ldc + n, C, epi, bias, H, Z, SW ? ZF_ACT_SWISH : act);
          }
    }
    __syncthreads();  // the next tile's planes overwrite the epilogue's LDS
  };
  // one k-iteration from stage S (refilled with iteration it + 2 once stored)
  auto kstep = [&](int it, int kk, Stage& S) __attribute__((always_inline)) {
    store_rows(Ap, S.ra, kk * kX3BK);
    if (TB) store_rows(Bp, S.rb, kk * kX3BK);
    else store_cols(S.rbs, kk * kX3BK);
    __syncthreads();
    load(min(it + 2, total - 1), S);  // (the last two refills repeat a k-tile, unused)
#pragma unroll
    for (int s = 0; s < kX3BK / 16; ++s) {
      tbf16x8 af[2][3], bf[2][3];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          af[i][t] = *reinterpret_cast<const tbf16x8*>(Ap + t * kX3Plane + (wm0 + 32 * i + r) * kX3RS + 16 * s + 8 * h);
          bf[i][t] = *reinterpret_cast<const tbf16x8*>(Bp + t * kX3Plane + (wn0 + 32 * i + r) * kX3RS + 16 * s + 8 * h);
        }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          // WIDE: B as the MFMA's first operand, so D = C^T: lane = row m and
          // each group of 4 registers = 4 consecutive columns (one dwordx4
          // store; the same products and sums, the same bits)
          auto mf = [&](int ta, int tb, const floatx16& c) {
            return WIDE ? __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf[j][tb], af[i][ta], c, 0, 0, 0)
                        : __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][ta], bf[j][tb], c, 0, 0, 0);
          };
          floatx16 c = mf(1, 1, acc[i][j]);  // (A term, B term): m m, h l, l h, h m, m h, h h
          c = mf(0, 2, c);
          c = mf(2, 0, c);
          c = mf(0, 1, c);
          c = mf(1, 0, c);
          acc[i][j] = mf(0, 0, c);
        }
    }
    __syncthreads();
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
    epilogue();
  }
}

// max |H[m][0..N)| as float bits into r[m] (a producer without the fused row max)
__global__ __launch_bounds__(256) void row_absmax_kernel(int M, int N, const float* __restrict__ H, int ldh,
                                                         unsigned* __restrict__ r) {
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (m >= M) return;
  float mx = 0.f;
  for (int n = lane; n < N; n += 64) mx = fmaxf(mx, fabsf(H[(long long)m * ldh + n]));
#pragma unroll
  for (int w = 1; w < 64; w <<= 1) mx = fmaxf(mx, __shfl_xor(mx, w));
  if (lane == 0) r[m] = __float_as_uint(mx);
}

template <int T>
void gemm_launch(bool tb, int M, int N, int K, const float* A, int lda, const float* B, int ldb, float* C, int ldc,
                 hipStream_t st, int epi, const float* bias, float* H, const float* Z, int act) {
  const dim3 grid((N + T - 1) / T, (M + T - 1) / T);
  const bool sw = act == ZF_ACT_SWISH || epi == kEpiNone || (epi == kEpiBias && !H);
#define ZF_MG_LAUNCH(TB_, SW_)                                                                                \
  hipLaunchKernelGGL((mgemm_kernel<T, T, false, TB_, false, false, SW_>), grid, dim3(256), 0, st, M, N, K, A, lda, \
                     B, ldb, C, ldc, epi, bias, H, Z, 0, act)
  if (!tb) {
    if (sw) ZF_MG_LAUNCH(false, true);
    else ZF_MG_LAUNCH(false, false);
  } else {
    if (sw) ZF_MG_LAUNCH(true, true);
    else ZF_MG_LAUNCH(true, false);
  }
#undef ZF_MG_LAUNCH
}

// C = A . op(B) with A row-major [M][K]; 128 x 128 tiles when they give at
// least 512 blocks over the GLOBAL batch's Mg rows, 64 x 64 otherwise.  The
// two tiles accumulate differently (one chain vs four interleaved), so the
// choice follows the global batch: every data-parallel shard then runs the
// kernel, and gets the bits, of the one-device step.  64 x 64 tiles that
// would leave most CUs idle (< 256 blocks, K >= 64) run as the four split
// sets + combine (SPLITQ; same bits) when a workspace of 4 M N floats is
// given (`split`, the trainer's split-K buffer), and K <= 8 as one thread
// per output (gemm_small_k_kernel; same bits); ZF_TRAIN_SPLITQ=0: neither.
int gemm(bool tb, long long Mg, int M, int N, int K, const float* A, int lda, const float* B, int ldb, float* C,
         int ldc, hipStream_t st, int epi = kEpiNone, const float* bias = nullptr, float* H = nullptr,
         const float* Z = nullptr, int act = ZF_ACT_SWISH, float* split = nullptr, long long split_cap = 0,
         unsigned* rmax = nullptr, bool* rmax_done = nullptr) {
  if (M <= 0 || N <= 0) return ZF_OK;
  const long long big = (long long)((N + 127) / 128) * ((Mg + 127) / 128);
  const long long tiles64 = (long long)((N + 63) / 64) * ((M + 63) / 64);
  static const bool x3_ok = [] {
    const char* e = std::getenv("ZF_TRAIN_X3");
    return !(e && e[0] == '0');
  }();
  const bool a_ok = lda % 4 == 0 && (reinterpret_cast<uintptr_t>(A) & 15) == 0;
  const bool b_ok = !tb || (ldb % 4 == 0 && (reinterpret_cast<uintptr_t>(B) & 15) == 0);
  if (big >= 512 && !tb && K <= 8) {
    // the first Dense (K = dc + C <= 8) at large batches too: one thread per
    // output is bound by its Z / H stores, the MFMA tiles would multiply a
    // 32-deep k-tile of zeros (the choice follows the global batch, as below;
    // not a split-set form, so ZF_TRAIN_SPLITQ=0 keeps it)
    const long long MN = (long long)M * N;
    auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    if (N % 4 == 0 && ldc % 4 == 0 && al16(C) && al16(H) && (epi == kEpiBias || epi == kEpiNone)) {
      hipLaunchKernelGGL(gemm_small_k4_kernel, dim3((unsigned)((N + 255) / 256), (unsigned)((M + 4 * kSk4Rows - 1) / (4 * kSk4Rows))),
                         dim3(64, 4), 0, st, M, N, K, A, lda, B, ldb, C, ldc, epi, bias, H, act, rmax);
      ZF_CHECK_LAUNCH("gemm_small_k4_kernel");
      if (rmax_done) *rmax_done = rmax != nullptr;
      return ZF_OK;
    }
    hipLaunchKernelGGL(gemm_small_k_kernel, dim3((unsigned)((MN + 255) / 256)), dim3(256), 0, st, M, N, K, A, lda, B,
                       ldb, C, ldc, epi, bias, H, Z, act);
    ZF_CHECK_LAUNCH("gemm_small_k_kernel");
    return ZF_OK;
  }
  if (big >= 512 && x3_ok && K % 8 == 0 && a_ok && b_ok) {
    // two resident blocks per CU (60 KiB of LDS each), persistent over the tiles
    const long long ntiles = (long long)((N + kX3BN - 1) / kX3BN) * ((M + kX3BM - 1) / kX3BM);
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const dim3 grid((unsigned)std::min<long long>(ntiles, 2ll * ncu));
    auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    const bool wide = N % 4 == 0 && ldc % 4 == 0 && al16(C) && (!H || al16(H)) && (!Z || al16(Z));
    // the swish-only epilogue whenever no other activation is applied
    const bool sw = act == ZF_ACT_SWISH || epi == kEpiNone || (epi == kEpiBias && !H);
#define ZF_X3_LAUNCH(TB_, W_, S_)                                                                                    \
  hipLaunchKernelGGL((gemm_x3_kernel<TB_, W_, S_>), grid, dim3(256), 0, st, M, N, K, A, lda, B, ldb, C, ldc, epi, \
                     bias, H, Z, act)
#define ZF_X3_LAUNCH_SW(TB_, W_) \
  if (sw) ZF_X3_LAUNCH(TB_, W_, true); else ZF_X3_LAUNCH(TB_, W_, false)
    if (tb) {
      if (wide) ZF_X3_LAUNCH_SW(true, true);
      else ZF_X3_LAUNCH_SW(true, false);
    } else {
      if (wide) ZF_X3_LAUNCH_SW(false, true);
      else ZF_X3_LAUNCH_SW(false, false);
    }
#undef ZF_X3_LAUNCH_SW
#undef ZF_X3_LAUNCH
    ZF_CHECK_LAUNCH("gemm_x3_kernel");
    return ZF_OK;
  }
  if (big >= 512) {
    gemm_launch<128>(tb, M, N, K, A, lda, B, ldb, C, ldc, st, epi, bias, H, Z, act);
  } else if (split != nullptr && !tb && K <= 8) {
    const long long MN = (long long)M * N;
    hipLaunchKernelGGL(gemm_small_k_kernel, dim3((unsigned)((MN + 255) / 256)), dim3(256), 0, st, M, N, K, A, lda, B,
                       ldb, C, ldc, epi, bias, H, Z, act);
  } else if (split != nullptr && tiles64 < 256 && K >= 64 && 4ll * M * N <= split_cap) {
    const dim3 grid((N + 63) / 64, (M + 63) / 64, 4);
    if (!tb)
      hipLaunchKernelGGL((mgemm_kernel<64, 64, false, false, false, true>), grid, dim3(256), 0, st, M, N, K, A, lda, B,
                         ldb, split, N, kEpiNone, nullptr, nullptr, nullptr, 0, act);
    else
      hipLaunchKernelGGL((mgemm_kernel<64, 64, false, true, false, true>), grid, dim3(256), 0, st, M, N, K, A, lda, B,
                         ldb, split, N, kEpiNone, nullptr, nullptr, nullptr, 0, act);
    ZF_CHECK_LAUNCH("mgemm_kernel<splitq>");
    const long long MN = (long long)M * N;
    hipLaunchKernelGGL(gemm_combine_kernel, dim3((unsigned)((MN + 255) / 256)), dim3(256), 0, st, M, N, split, C, ldc,
                       epi, bias, H, Z, act);
  } else {
    gemm_launch<64>(tb, M, N, K, A, lda, B, ldb, C, ldc, st, epi, bias, H, Z, act);
  }
  ZF_CHECK_LAUNCH("mgemm_kernel");
  return ZF_OK;
}

inline unsigned blocks_for(long long n, int t = 256) { return (unsigned)((n + t - 1) / t); }

// Split-K workspace (floats) shared by the batch reductions below.
constexpr int64_t kWsFloats = 32ll << 20;
// The split-set GEMMs' partials (4 M N floats, M N < 256 tiles of 64 x 64).
constexpr int64_t kSplitFloats = 4ll << 20;

// ---- batch reductions: row leaves + one fixed pairwise tree ----------------
// Every sum over the batch rows (weight and bias gradients, BatchNorm sums
// forward and reverse, the loss) is formed the same way: the rows are cut
// into n contiguous leaves of `rows` rows, each leaf is summed in row order,
// and the leaves are combined in fp64 by the pairwise tree
// ((l0 + l1) + (l2 + l3)) + ... (tree_n).  The global leaf count is a power of
// two that depends on the GLOBAL batch size only (leaves_for); under data
// parallelism rank r holds leaves [r n, (r+1) n) of it, reduces that subtree,
// and the ranks' subtree roots are all-gathered and combined by the top of
// the same tree.  So every rank gets the same bits, and R ranks reproduce
// one rank's bits on the same global batch (R a power of two dividing the
// leaf count, shards of B/R rows, B a multiple of the leaf count).
constexpr int kMaxLeaves = 64;        // one tree level (registers)
constexpr int kLeafCap = kMaxLeaves * kMaxLeaves;  // two levels: up to 4096 leaves

inline int pow2floor(long long v) {
  int p = 1;
  while ((long long)p * 2 <= v && p < (1 << 30)) p *= 2;
  return p;
}

struct Leaves {
  int n;     // this rank's leaves (a power of two)
  int rows;  // rows per leaf (the last one may be short or empty)
};

// ~32 rows per leaf, at most `cap` (a power of two) leaves in the whole batch.
inline Leaves leaves_for(long long B_loc, long long Bg, int world, int cap) {
  const long long want = std::max<long long>(1, std::min<long long>(Bg / 32, cap));
  Leaves l;
  l.n = std::max(1, pow2floor(want / std::max(1, world)));
  l.rows = (int)((B_loc + l.n - 1) / l.n);
  return l;
}

// Pairwise tree over p[0], p[stride], ..., p[(n-1) stride] (n <= NMAX <= 64)
// in fp64: level s adds element i + s into i for i a multiple of 2s (the
// perfect tree for a power of two; a shorter tail just joins later).  NMAX
// only sizes the register array: every NMAX >= n gives the same bits.
template <int NMAX, typename TI>
__device__ __forceinline__ double tree_n(const TI* __restrict__ p, long long stride, int n) {
  double v[NMAX];
#pragma unroll
  for (int i = 0; i < NMAX; ++i) v[i] = i < n ? (double)p[i * stride] : 0.0;
#pragma unroll
  for (int s = 1; s < NMAX; s *= 2)
#pragma unroll
    for (int i = 0; i < NMAX; i += 2 * s)
      if (i + s < n) v[i] = v[i] + v[i + s];
  return v[0];
}

// The same tree in place over LDS columns (leaf i of column k at
// p[i * stride + k]), all threads of the block taking part, one barrier per
// level: the same pairings and operand order as tree_n.  Result in p[k].
__device__ __forceinline__ void lds_tree(double* p, int n, int ncols, int stride) {
  for (int s = 1; s < n; s *= 2) {
    const int pairs = (n + 2 * s - 1) / (2 * s);
    for (int t = threadIdx.x; t < pairs * ncols; t += blockDim.x) {
      const int j = t / ncols, k = t - j * ncols, i = 2 * s * j;
      if (i + s < n) p[i * stride + k] = p[i * stride + k] + p[(i + s) * stride + k];
    }
    __syncthreads();
  }
}

// Two such trees (same shapes) level by level under one barrier per level:
// each tree's pairwise sums are unchanged.
__device__ __forceinline__ void lds_tree2(double* p, double* q, int n, int ncols, int stride) {
  for (int s = 1; s < n; s *= 2) {
    const int pairs = (n + 2 * s - 1) / (2 * s);
    for (int t = threadIdx.x; t < pairs * ncols; t += blockDim.x) {
      const int j = t / ncols, k = t - j * ncols, i = 2 * s * j;
      if (i + s < n) {
        p[i * stride + k] = p[i * stride + k] + p[(i + s) * stride + k];
        q[i * stride + k] = q[i * stride + k] + q[(i + s) * stride + k];
      }
    }
    __syncthreads();
  }
}

// Launch KERNEL<..., NMAX> with the smallest register tree that holds n leaves.
#define ZF_NMAX_DISPATCH(n, LAUNCH) \
  do {                              \
    if ((n) <= 8) LAUNCH(8);        \
    else if ((n) <= 16) LAUNCH(16); \
    else if ((n) <= 32) LAUNCH(32); \
    else LAUNCH(64);                \
  } while (0)

// out[k] = tree over n leaves of part[leaf * N + k]
template <typename TI, int NMAX>
__global__ void tree_cols_kernel(const TI* __restrict__ part, int n, long long N, double* __restrict__ out) {
  const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < N) out[k] = tree_n<NMAX>(part + k, N, n);
}

// First level of a two-level tree: out[g * N + k] = tree over the 64 leaves
// [64 g, 64 g + 64) of part (a perfect subtree of the power-of-two leaf tree,
// so the second level over the group roots completes the same tree).
template <typename TI>
__global__ void tree_groups_kernel(const TI* __restrict__ part, int groups, long long N, double* __restrict__ out) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)groups * N) return;
  const long long g = t / N, k = t - g * N;
  out[t] = tree_n<kMaxLeaves>(part + g * kMaxLeaves * N + k, N, kMaxLeaves);
}

// same, then the final fp32 rounding (the gradient handed to the optimiser)
template <int NMAX>
__global__ void tree_cols_cast_kernel(const double* __restrict__ part, int n, long long N, float* __restrict__ out) {
  const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < N) out[k] = (float)tree_n<NMAX>(part + k, N, n);
}

// dW/db from the split-K partials part[leaf][M+1][N] (fp32 leaf GEMMs, or
// their fp64 group roots), combined by the leaf tree into the fp64 gradient
// accumulator.
// dW / db from the n (a power of two) leaf partials of each element: the
// four waves of a block each reduce a perfect subtree of n / 4 consecutive
// leaves for 64 elements (n < 4: one wave per leaf), joined as the top two
// levels of the same tree — four times the waves of a thread-per-element tree
// for the same bits.
template <typename TI, int NMAX>
__global__ __launch_bounds__(256) void wgrad_tree(int M, int N, int n, const TI* __restrict__ part,
                                                  double* __restrict__ dW, double* __restrict__ db) {
  __shared__ double r[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int P = n < 4 ? n : 4, m = n / P;
  const long long idx = (long long)blockIdx.x * 64 + lane;
  const long long MN1 = (long long)(M + 1) * N;
  if (w < P && idx < MN1) r[w][lane] = tree_n<NMAX>(part + (long long)w * m * MN1 + idx, MN1, m);
  __syncthreads();
  if (w != 0 || idx >= MN1) return;
  double v = r[0][lane];
  if (P == 2) v = v + r[1][lane];
  else if (P == 4) v = (v + r[1][lane]) + (r[2][lane] + r[3][lane]);
  if (idx < (long long)M * N) dW[idx] = v;
  else db[idx - (long long)M * N] = v;
}

// dW[M,N] = A^T . G and db[N] = colsum(G), A row-major [B][M] (layer input),
// G row-major [B][N] (gradient of the layer output): one split-K block per
// leaf (rows [z lv.rows, (z+1) lv.rows)), then wgrad_tree.
int wgrad(int M, int N, int B, const Leaves& lv, const float* A, const float* G, double* dW, double* db, float* ws,
          double* ws2, hipStream_t st) {
  constexpr int T = 64;
  const int64_t MN1 = (int64_t)(M + 1) * N;
  if ((int64_t)lv.n * MN1 > kWsFloats) return enotsup("training: weight-gradient workspace");
  hipLaunchKernelGGL((mgemm_kernel<T, T, true, false, true>), dim3((N + T - 1) / T, (M + T - 1) / T, lv.n),
                     dim3(256), 0, st, M, N, B, A, M, G, N, ws, N, kEpiNone, nullptr, nullptr, nullptr, lv.rows,
                     (int)ZF_ACT_SWISH);
  ZF_CHECK_LAUNCH("mgemm_kernel<wgrad>");
  if (lv.n <= kMaxLeaves) {
#define ZF_L(NM) hipLaunchKernelGGL((wgrad_tree<float, NM>), dim3(blocks_for(MN1, 64)), dim3(256), 0, st, M, N, lv.n, ws, dW, db)
    ZF_NMAX_DISPATCH(lv.n < 4 ? 1 : lv.n / 4, ZF_L);
#undef ZF_L
  } else {  // two levels: groups of 64 leaves, then their roots
    const int groups = lv.n / kMaxLeaves;
    hipLaunchKernelGGL(tree_groups_kernel<float>, dim3(blocks_for((int64_t)groups * MN1)), dim3(256), 0, st, ws,
                       groups, MN1, ws2);
    ZF_CHECK_LAUNCH("tree_groups_kernel");
#define ZF_L(NM) hipLaunchKernelGGL((wgrad_tree<double, NM>), dim3(blocks_for(MN1, 64)), dim3(256), 0, st, M, N, groups, ws2, dW, db)
    ZF_NMAX_DISPATCH(groups < 4 ? 1 : groups / 4, ZF_L);
#undef ZF_L
  }
  ZF_CHECK_LAUNCH("wgrad_tree");
  return ZF_OK;
}

// Weight-gradient trees of several layers in one launch: the backward pass
// writes each layer's leaf partials to its own slice of the split-K
// workspace and the trees of all of them run at the end (or when the
// workspace or the item list is full) — one launch instead of one per layer,
// the same per-element trees (wgrad_tree's), so the same bits.
constexpr int kTreeItems = 24;
struct TreeItem {
  const float* part;
  double* dW;
  double* db;
  int M, N, n, blocks;  // blocks of 64 elements
};
struct TreeBatch {
  int count;
  TreeItem it[kTreeItems];
};

template <int NMAX>
__global__ __launch_bounds__(256) void wgrad_tree_batch(TreeBatch tb) {
  __shared__ double r[4][64];
  int b = blockIdx.x, i = 0;
  while (i + 1 < tb.count && b >= tb.it[i].blocks) b -= tb.it[i++].blocks;
  const TreeItem& t = tb.it[i];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int P = t.n < 4 ? t.n : 4, m = t.n / P;
  const long long idx = (long long)b * 64 + lane;
  const long long MN1 = (long long)(t.M + 1) * t.N;
  if (w < P && idx < MN1) r[w][lane] = tree_n<NMAX>(t.part + (long long)w * m * MN1 + idx, MN1, m);
  __syncthreads();
  if (w != 0 || idx >= MN1) return;
  double v = r[0][lane];
  if (P == 2) v = v + r[1][lane];
  else if (P == 4) v = (v + r[1][lane]) + (r[2][lane] + r[3][lane]);
  if (idx < (long long)t.M * t.N) t.dW[idx] = v;
  else t.db[idx - (long long)t.M * t.N] = v;
}

// Weight-gradient GEMMs deferred into one launch: each problem is the
// mgemm_kernel<64, 64, TA, !TB, WG> grid it would have launched on its own
// (the same blocks, the same bits), laid end to end.
struct WgGemm {
  const float *A, *G;
  float* part;
  int M, N, B, rows, tx, ty, block0;
};
constexpr int kWgGroup = 8;
struct WgGroup {
  int count;
  WgGemm g[kWgGroup];
};

__global__ __launch_bounds__(256) void wgrad_group_kernel(WgGroup grp) {
  int i = 0;
  while (i + 1 < grp.count && (int)blockIdx.x >= grp.g[i + 1].block0) ++i;
  const WgGemm& g = grp.g[i];
  int r = (int)blockIdx.x - g.block0;
  const unsigned bx = r % g.tx;
  r /= g.tx;
  const unsigned by = r % g.ty, bz = r / g.ty;
  mgemm_body<64, 64, true, false, true, false>(uint3{bx, by, bz}, g.M, g.N, g.B, g.A, g.M, g.G, g.N, g.part, g.N,
                                               kEpiNone, nullptr, nullptr, nullptr, g.rows, (int)ZF_ACT_SWISH);
}

struct WgradQueue {
  TreeBatch tb;
  WgGroup gq;        // GEMMs not launched yet
  int gblocks = 0;   // their blocks
  int64_t used = 0;  // workspace floats holding pending partials
  int nmax = 1;
};

int wgrad_launch_gemms(WgradQueue& q, hipStream_t st) {
  if (q.gq.count == 0) return ZF_OK;
  hipLaunchKernelGGL(wgrad_group_kernel, dim3(q.gblocks), dim3(256), 0, st, q.gq);
  ZF_CHECK_LAUNCH("wgrad_group_kernel");
  q.gq.count = 0;
  q.gblocks = 0;
  return ZF_OK;
}

// Launch the deferred GEMMs before `p` (a buffer one of them reads) is
// overwritten.
int wgrad_before_write(WgradQueue& q, const float* p, hipStream_t st) {
  for (int i = 0; i < q.gq.count; ++i)
    if (q.gq.g[i].A == p || q.gq.g[i].G == p) return wgrad_launch_gemms(q, st);
  return ZF_OK;
}

int wgrad_flush(WgradQueue& q, hipStream_t st) {
  int rc = wgrad_launch_gemms(q, st);
  if (rc) return rc;
  if (q.tb.count == 0) return ZF_OK;
  int blocks = 0;
  for (int i = 0; i < q.tb.count; ++i) blocks += q.tb.it[i].blocks;
  const int nm = q.nmax < 4 ? 1 : q.nmax / 4;
#define ZF_L(NM) hipLaunchKernelGGL((wgrad_tree_batch<NM>), dim3(blocks), dim3(256), 0, st, q.tb)
  ZF_NMAX_DISPATCH(nm, ZF_L);
#undef ZF_L
  ZF_CHECK_LAUNCH("wgrad_tree_batch");
  q.tb.count = 0;
  q.used = 0;
  q.nmax = 1;
  return ZF_OK;
}

// wgrad with the tree deferred into `q` (one level of leaves: n <= 64);
// more leaves run wgrad's two-level form at once, after the queue.
int wgrad_deferred(WgradQueue& q, int M, int N, int B, const Leaves& lv, const float* A, const float* G, double* dW,
                   double* db, float* ws, double* ws2, hipStream_t st) {
  const int64_t MN1 = (int64_t)(M + 1) * N, need = (int64_t)lv.n * MN1;
  int rc;
  if (lv.n > kMaxLeaves) {
    if ((rc = wgrad_flush(q, st))) return rc;
    return wgrad(M, N, B, lv, A, G, dW, db, ws, ws2, st);
  }
  if (need > kWsFloats) return enotsup("training: weight-gradient workspace");
  if (q.used + need > kWsFloats || q.tb.count == kTreeItems)
    if ((rc = wgrad_flush(q, st))) return rc;
  float* part = ws + q.used;
  if (q.gq.count == kWgGroup && (rc = wgrad_launch_gemms(q, st))) return rc;
  WgGemm& g = q.gq.g[q.gq.count++];
  g.A = A;
  g.G = G;
  g.part = part;
  g.M = M;
  g.N = N;
  g.B = B;
  g.rows = lv.rows;
  g.tx = (N + 63) / 64;
  g.ty = (M + 63) / 64;
  g.block0 = q.gblocks;
  q.gblocks += g.tx * g.ty * lv.n;
  TreeItem& it = q.tb.it[q.tb.count++];
  it.part = part;
  it.dW = dW;
  it.db = db;
  it.M = M;
  it.N = N;
  it.n = lv.n;
  it.blocks = (int)blocks_for(MN1, 64);
  q.used += need;
  q.nmax = std::max(q.nmax, lv.n);
  return ZF_OK;
}

// Leaf sums of two per-column sums over rows [b0, b1), in row order, fp64:
// s1 = sum x, s2 = sum x * y (y = x: the sum of squares).
constexpr int kLeafInflight = 32;
template <class FX, class FY>
__device__ __forceinline__ void leaf_sums2(FX x_at, FY y_at, int b0, int b1, double& s1, double& s2) {
  double a = 0.0, q = 0.0;
  int b = b0;
  // kLeafInflight rows' loads in flight before their (in-order) sums: the
  // leaf is a chain of dependent adds, its loads are not (the one-block
  // BatchNorm kernels expose every serial round trip: 32 rows, a whole leaf
  // at the default batch, in one)
  constexpr int R = kLeafInflight;
  for (; b + R <= b1; b += R) {
    float xv[R], yv[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      xv[j] = x_at(b + j);
      yv[j] = y_at(b + j);
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      a += (double)xv[j];
      q += (double)xv[j] * (double)yv[j];
    }
  }
  for (; b < b1; ++b) {
    const double xv = (double)x_at(b), yv = (double)y_at(b);
    a += xv;
    q += xv * yv;
  }
  s1 = a;
  s2 = q;
}

// One thread per (leaf z, column k): p[z][k] = sum x, p[z][N + k] = sum x*y
// over the leaf's rows of X, Y row-major [B][N] (Y NULL: Y = X).
__global__ void leaf_colsums_kernel(const float* __restrict__ X, const float* __restrict__ Y, int B, int N, int rows,
                                    int n, double* __restrict__ p) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * N) return;
  const int z = t / N, k = t - z * N;
  const int b0 = min(B, z * rows), b1 = min(B, b0 + rows);
  const float* Yp = Y ? Y : X;
  leaf_sums2([&](int b) { return X[(long long)b * N + k]; }, [&](int b) { return Yp[(long long)b * N + k]; }, b0, b1,
             p[(long long)z * 2 * N + k], p[(long long)z * 2 * N + N + k]);
}

// Leaf sums of one column vector (the per-row loss), fp64 in row order.
__global__ void leaf_sum_kernel(const double* __restrict__ x, int B, int rows, int n, double* __restrict__ p) {
  const int z = blockIdx.x * blockDim.x + threadIdx.x;
  if (z >= n) return;
  const int b0 = min(B, z * rows), b1 = min(B, b0 + rows);
  double a = 0.0;
  for (int b = b0; b < b1; ++b) a += x[b];
  p[z] = a;
}

// out[k] = tree over n leaves (a power of two up to kLeafCap, or any n <= 64)
// of part[leaf * N + k]; tmp: (n / 64) * N doubles for the two-level case.
inline int launch_tree_cols(const double* part, int n, long long N, double* out, hipStream_t st,
                            double* tmp = nullptr) {
  if (n > kMaxLeaves) {
    if (!tmp) return einval("tree over %d leaves needs a workspace", n);
    const int groups = n / kMaxLeaves;
    hipLaunchKernelGGL(tree_groups_kernel<double>, dim3(blocks_for((long long)groups * N)), dim3(256), 0, st, part,
                       groups, N, tmp);
    ZF_CHECK_LAUNCH("tree_groups_kernel");
    part = tmp;
    n = groups;
  }
#define ZF_L(NM) hipLaunchKernelGGL((tree_cols_kernel<double, NM>), dim3(blocks_for(N)), dim3(256), 0, st, part, n, N, out)
  ZF_NMAX_DISPATCH(n, ZF_L);
#undef ZF_L
  ZF_CHECK_LAUNCH("tree_cols_kernel");
  return ZF_OK;
}

// ---- ShiftBounds (train mode; bijectors.py:163-273) -------------------------
// Natural row per dim: [mode, a, b, xmin, xmax, margin, -, -].  Batch min/max
// of the (safe_log-transformed) column -> running xmin/xmax (:250-259).
// This batch's min / max widened by the margin and merged with the running
// values, then the affine map, clip and log-det.  Every thread forms the
// statistics from the column min / max itself (a handful of scalars: no
// separate statistics launch); thread 0 also writes the running values when
// update is set — the one write another block can observe, and re-forming
// the statistics from it gives the same values (min / max are idempotent).
// first: this op starts the chain, so ld (not yet written this step) is set
// instead of accumulated.
__global__ void sb_forward_kernel(const float* __restrict__ x, float* __restrict__ y, float* __restrict__ ld,
                                  float* __restrict__ sb, int B, int D, int rot, const float* __restrict__ cmin,
                                  const float* __restrict__ cmax, int update, int first) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float lds = 0.f;
  for (int i = 0; i < D; ++i) {
    const int p = pmodi(i + rot, D);
    const float v = x[(long long)b * D + p];
    float* r = sb + 8 * i;
    const int mode = (int)r[0];
    const float a = r[1], bb = r[2];
    float z, l;
    if (mode == ZF_SB_BOTH) {
      const float mul = (float)(1.0 / ((double)bb - (double)a));
      z = (v - a) * mul;
      l = logf(mul);
    } else {
      const float margin = r[5];
      float xmin = cmin[i], xmax = cmax[i];
      const float delta = 0.5f * (xmax - xmin) * margin;
      xmin = xmin - delta;
      xmax = xmax + delta;
      xmin = fminf(r[3], xmin);  // jnp.minimum(ra_min, xmin); NaN from the batch propagates below
      xmax = fmaxf(r[4], xmax);
      if (cmin[i] != cmin[i]) xmin = cmin[i];
      if (cmax[i] != cmax[i]) xmax = cmax[i];
      if (update && b == 0) {
        r[3] = xmin;
        r[4] = xmax;
      }
      const float mul = 1.0f / (xmax - xmin);
      float t = v;
      if (mode == ZF_SB_LOWER) t = logf((v - a) + 1.17549435e-38f);
      if (mode == ZF_SB_UPPER) t = logf((bb - v) + 1.17549435e-38f);
      const float zr = (t - xmin) * mul;
      z = (zr != zr) ? zr : fminf(fmaxf(zr, 0.f), 1.f);
      l = (mode == ZF_SB_NONE) ? logf(mul) : logf(mul) - t;
    }
    lds = lds + l;
    y[(long long)b * D + p] = z;
  }
  ld[b] = (first ? 0.f : ld[b]) + lds;
}

// ---- NeuralSplineCoupling pieces --------------------------------------------
// U = hstack(xc, c): logical conditioning dim k is column pmod(dt + k + rot, D).
__global__ void gather_u_kernel(const float* __restrict__ s, const float* __restrict__ c, float* __restrict__ U,
                                int B, int D, int C, int dt, int dc, int rot) {
  const int DC = dc + C;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)B * DC) return;
  const long long b = i / DC;
  const int k = (int)(i - b * DC);
  U[i] = k < dc ? s[b * D + pmodi(dt + k + rot, D)] : c[b * C + (k - dc)];
}

// BatchNorm with batch statistics (flax, use_running_average=False):
// mean, var = max(0, E[u^2] - E[u]^2); u_hat = (u - mean) * rsqrt(var + eps);
// u_bn = u_hat * scale + bias.  Also the running-average update (momentum 0.99).
// sum / sumsq: fp64 column sums over the global batch of Bg rows.
__device__ __forceinline__ void bn_stats_one(double sum, double sumsq, long long Bg, int k, int DC,
                                             float* __restrict__ nat_bn, float& mean, float& rstd, int update) {
#pragma clang fp contract(off)
  // every operation separately rounded: the same bits in every kernel that inlines this
  mean = (float)(sum / Bg);
  const float mean2 = (float)(sumsq / Bg);
  const float var = fmaxf(0.f, mean2 - mean * mean);
  rstd = 1.0f / sqrtf(var + kBnEps);
  if (update) {
    nat_bn[k] = kBnMomentum * nat_bn[k] + (1.0f - kBnMomentum) * mean;
    nat_bn[DC + k] = kBnMomentum * nat_bn[DC + k] + (1.0f - kBnMomentum) * var;
  }
}

__global__ void bn_stats_kernel(const double* __restrict__ csum, const double* __restrict__ csq, long long Bg, int DC,
                                float* __restrict__ nat_bn, float* __restrict__ mean_out,
                                float* __restrict__ rstd_out, int update) {
  const int k = threadIdx.x;
  if (k >= DC) return;
  float mean, rstd;
  bn_stats_one(csum[k], csq[k], Bg, k, DC, nat_bn, mean, rstd, update);
  mean_out[k] = mean;
  rstd_out[k] = rstd;
}

// Per-element BatchNorm arithmetic shared by the single-block and the
// multi-launch paths, every operation separately rounded (fp contraction off:
// HIP's __f*_rn are plain operators that the compiler may still fuse, and it
// fuses differently in different kernels): both paths give the same bits.
__device__ __forceinline__ float bn_hat(float u, float mean, float rstd) {
#pragma clang fp contract(off)
  return (u - mean) * rstd;
}
__device__ __forceinline__ float bn_out(float uh, float scale, float bias) {
#pragma clang fp contract(off)
  return uh * scale + bias;
}
// reverse: the mean terms scale * sum / Bg, then
// dL/dU = rstd * (gUbn * scale - mg - Uhat * mgu)
__device__ __forceinline__ float bn_mean_term(float scale, double sum, long long Bg) {
#pragma clang fp contract(off)
  return scale * (float)sum / (float)Bg;
}
__device__ __forceinline__ float bn_grad_in(float gubn, float uh, float scale, float rstd, float mg, float mgu) {
#pragma clang fp contract(off)
  return rstd * (gubn * scale - mg - uh * mgu);
}
__device__ __forceinline__ float add_rn(float a, float b) {
#pragma clang fp contract(off)
  return a + b;
}

__global__ void bn_apply_kernel(const float* __restrict__ U, const float* __restrict__ mean,
                                const float* __restrict__ rstd, const float* __restrict__ scale,
                                const float* __restrict__ bias, float* __restrict__ Uhat, float* __restrict__ Ubn,
                                int B, int DC) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)B * DC) return;
  const int k = (int)(i % DC);
  const float uh = bn_hat(U[i], mean[k], rstd[k]);
  Uhat[i] = uh;
  Ubn[i] = bn_out(uh, scale[k], bias[k]);
}

// Spline-path arithmetic at a third of the IEEE expansions' instructions (the
// per-thread spline kernels are issue-latency bound: one wave per (row block),
// thousands of dependent VALU): a hardware reciprocal / square root with one
// Newton or residual step, and quotients by a loop-invariant divisor as one
// residual correction of x * rcp(d) — the correctly rounded result for these
// normal operands, as zf_flow_dev.h's div_cr in the inference kernels.
__device__ __forceinline__ float t_rcp(float x) {
  const float r = __builtin_amdgcn_rcpf(x);
  return __builtin_fmaf(__builtin_fmaf(-x, r, 1.0f), r, r);
}
__device__ __forceinline__ float t_div(float x, float d, float r) {
  const float q = x * r;
  return __builtin_fmaf(__builtin_fmaf(-q, d, x), r, q);
}
// sqrt(x^2 + 4) (>= 2: never denormal), residual-corrected hardware root
__device__ __forceinline__ float t_sq4(float x) {
  const float a = x * x + 4.0f;
  const float sq = __builtin_amdgcn_sqrtf(a);
  return __builtin_fmaf(__builtin_fmaf(-sq, sq, a), 0.5f * __builtin_amdgcn_rcpf(sq), sq);
}
__device__ __forceinline__ float sp_f(float x) { return 0.5f * (x + t_sq4(x)); }
__device__ __forceinline__ float sp_grad(float x) {
  const float sq = t_sq4(x);
  return 0.5f * (1.0f + t_div(x, sq, t_rcp(sq)));
}

constexpr int kMaxK = 64;

// One (row, transformed dim): normalize_spline_params (utils.py:37-62) of the
// raw conditioner outputs p[0..3K-1), bin, RQ spline forward (utils.py:65-141).
// With grads: reverse pass for gy (dL/dy) and gl (dL/dlog_det): dL/dx and dL/dp.
// No per-thread arrays (they would live in scratch): the normalised widths and
// heights are recomputed from p where needed, in the same float order.
// gp may alias p (in-place reverse): every p[j] is read before gp[j] is written.
// KT > 0: the knot count at compile time (8, 16, 32: every loop unrolled, so
// the per-knot squareplus / divisions of different knots overlap instead of
// running as one long dependent chain).  The same operations in the same
// order as KT = 0 (the runtime-K form for other counts), but not always the
// same bits: fp contraction may pair a multiply with a different add once
// the loops are unrolled.  Every rank runs the same form, so the
// data-parallel bit-identity holds.
template <bool GRAD, int KT = 0>
__device__ __forceinline__ void spline_one(const float* p, int Kr, float x, float& y, float& ld, float gy, float gl,
                                           float* gx, float* gp) {
  constexpr int U = KT > 0 ? KT + 1 : 1;  // unroll counts (1: as written)
  const int K = KT > 0 ? KT : Kr;
  const double c64 = 1e-5 / (1.0 - (double)K * 1e-5);  // utils.py:32-34, Python floats
  const float cc = (float)c64, norm = (float)(1.0 + c64 * (double)K);
  float Sa = 0.f, Sb = 0.f;
#pragma unroll U
  for (int j = 0; j < K; ++j) {
    Sa = Sa + sp_f(p[j]);
    Sb = Sb + sp_f(p[K + j]);
  }
  // bin: count semantics of _index (utils.py:244-250); the knots t_j are
  // non-decreasing, so the last knot <= x is knot cnt - 1 and its prefix sums
  // are the bin's left edge (xk, yk)
  float xk = 0.f, yk = 0.f;
  int cnt = 0;
  const float rSa = t_rcp(Sa), rSb = t_rcp(Sb), rnorm = t_rcp(norm);
  {
    float tx = 0.f, ty = 0.f;
#pragma unroll U
    for (int j = 0; j <= K; ++j) {
      if (tx <= x) {
        ++cnt;
        xk = tx;
        yk = ty;
      }
      if (j < K) {
        tx = tx + t_div(t_div(sp_f(p[j]), Sa, rSa) + cc, norm, rnorm);
        ty = ty + t_div(t_div(sp_f(p[K + j]), Sb, rSb) + cc, norm, rnorm);
      }
    }
  }
  int idx = cnt - 1;
  idx = idx < 0 ? 0 : (idx > K ? K : idx);
  if (cnt == 0) xk = yk = 0.f;
  const bool oob = (x < 0.f) || (x >= 1.f);
  if (idx == K || oob) {
    // idx == K: the reference's fill-mode gather gives NaN (utils.py:224-230);
    // oob rows are the identity with log_det 0 (:130, :138).
    y = oob ? x : __builtin_nanf("");
    ld = oob ? 0.f : __builtin_nanf("");
    if (GRAD) {
      *gx = oob ? gy : __builtin_nanf("");
#pragma unroll U
      for (int j = 0; j < 3 * K - 1; ++j) gp[j] = 0.f;
    }
    return;
  }
  const float wk = t_div(t_div(sp_f(p[idx]), Sa, rSa) + cc, norm, rnorm);
  const float hk = t_div(t_div(sp_f(p[K + idx]), Sb, rSb) + cc, norm, rnorm);
  const float dk = (idx == 0) ? 1.f : sp_f(p[2 * K + idx - 1]);
  const float dk1 = (idx + 1 == K) ? 1.f : sp_f(p[2 * K + idx]);
  const float rwk = t_rcp(wk);
  const float sk = t_div(hk, wk, rwk);
  const float zr = t_div(x - xk, wk, rwk);
  const float z = fminf(fmaxf(zr, kEpsT), 0.99999f);
  const float az = 1.0f - z;
  const float num = hk * z * (sk * z + dk * az);
  const float den = sk + (dk1 + dk - 2.0f * sk) * z * az;
  const float dE = den + kEpsT, rdE = t_rcp(dE);
  y = yk + t_div(num, dE, rdE);
  const float q = z * (dk1 * z + 2.0f * sk * az) + dk * (az * az);
  ld = 2.0f * logf(sk + kEpsT) + logf(q + kEpsT) - 2.0f * logf(den + kEpsT);
  if (!GRAD) return;
  // ---- reverse pass ----
  float g_yk = gy;
  const float g_num = t_div(gy, dE, rdE);
  const float dE2 = dE * dE, skE = sk + kEpsT, qE = q + kEpsT;
  float g_den = t_div(-gy * num, dE2, t_rcp(dE2)) - t_div(2.0f * gl, dE, rdE);
  float g_sk = t_div(2.0f * gl, skE, t_rcp(skE));
  const float g_q = t_div(gl, qE, t_rcp(qE));
  float g_hk = g_num * (sk * z * z + dk * z * az);
  g_sk += g_num * hk * z * z;
  float g_dk = g_num * hk * z * az;
  float g_z = g_num * hk * (2.0f * sk * z + dk * (az - z));
  g_sk += g_den * (1.0f - 2.0f * z * az);
  float g_dk1 = g_den * z * az;
  g_dk += g_den * z * az;
  g_z += g_den * (dk1 + dk - 2.0f * sk) * (az - z);
  g_dk1 += g_q * z * z;
  g_sk += g_q * 2.0f * z * az;
  g_dk += g_q * az * az;
  g_z += g_q * (2.0f * dk1 * z + 2.0f * sk * (az - z) - 2.0f * dk * az);
  const float g_zr = (zr > kEpsT && zr < 0.99999f) ? g_z : 0.f;  // jnp.clip passes inside only
  *gx = t_div(g_zr, wk, rwk);
  const float g_xk = t_div(-g_zr, wk, rwk);
  float g_wk = t_div(-g_zr * zr, wk, rwk);
  g_hk += t_div(g_sk, wk, rwk);
  const float wk2 = wk * wk;
  g_wk += t_div(-g_sk * hk, wk2, t_rcp(wk2));
  // gradient w.r.t. widths / heights: xk = sum_{j<idx} w_j (likewise yk), plus
  // the bin's own w_idx, h_idx; then through w_j = (sa_j / Sa + c) / norm
  auto gw = [&](int j) { return j < idx ? g_xk : (j == idx ? g_wk : 0.f); };
  auto gh = [&](int j) { return j < idx ? g_yk : (j == idx ? g_hk : 0.f); };
  float tw = 0.f, th = 0.f;
#pragma unroll U
  for (int j = 0; j < K; ++j) {
    tw += gw(j) * sp_f(p[j]);
    th += gh(j) * sp_f(p[K + j]);
  }
  const float gd0 = idx >= 1 ? g_dk * sp_grad(p[2 * K + idx - 1]) : 0.f;
  const float gd1 = idx + 1 < K ? g_dk1 * sp_grad(p[2 * K + idx]) : 0.f;
  const float Sa2 = Sa * Sa, Sb2 = Sb * Sb;
  const float twq = t_div(tw, Sa2, t_rcp(Sa2)), thq = t_div(th, Sb2, t_rcp(Sb2));
#pragma unroll U
  for (int j = 0; j < K; ++j) {
    const float gsa = t_div(t_div(gw(j), Sa, rSa) - twq, norm, rnorm);
    const float gsb = t_div(t_div(gh(j), Sb, rSb) - thq, norm, rnorm);
    gp[j] = gsa * sp_grad(p[j]);
    gp[K + j] = gsb * sp_grad(p[K + j]);
  }
#pragma unroll U
  for (int j = 0; j < K - 1; ++j) gp[2 * K + j] = 0.f;
  if (idx >= 1) gp[2 * K + idx - 1] = 0.f + gd0;
  if (idx + 1 < K) gp[2 * K + idx] = 0.f + gd1;
}

// Thread per (row, transformed dim): one-wave blocks of rpb = 64 / dt rows.
// The block's conditioner outputs P[b0 .. b0+rpb)[dt][S] are contiguous: they
// are staged through LDS with coalesced loads (thread-major [64][S], S odd for
// even K so the per-thread rows spread over the banks).  Logical dim d < dt is
// column pmod(d + rot, D); thread d also carries the conditioning columns
// dt + d, dt + d + dt, ... through unchanged.
constexpr int kSplThreads = 64;

// Launch LAUNCH(KT) with the compile-time knot count where instantiated.
#define ZF_KNOT_DISPATCH(K, LAUNCH) \
  do {                              \
    if ((K) == 8) LAUNCH(8);        \
    else if ((K) == 16) LAUNCH(16); \
    else if ((K) == 32) LAUNCH(32); \
    else LAUNCH(0);                 \
  } while (0)

// Global <-> LDS copies of n floats, kStageInflight loads in flight per lane
// (the per-thread spline kernels run one wave per block: every serial HBM
// round trip here is exposed — 48 in flight stage K = 16's 47 floats per
// lane in one round instead of six).
constexpr int kStageInflight = 48;
__device__ __forceinline__ void stage_rows(float* sp, const float* __restrict__ src, long long n) {
  for (long long e0 = threadIdx.x; e0 < n; e0 += kStageInflight * kSplThreads) {
    float v[kStageInflight];
#pragma unroll
    for (int u = 0; u < kStageInflight; ++u) {
      const long long e = e0 + u * kSplThreads;
      v[u] = e < n ? src[e] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kStageInflight; ++u) {
      const long long e = e0 + u * kSplThreads;
      if (e < n) sp[e] = v[u];
    }
  }
}

__device__ __forceinline__ void unstage_rows(float* __restrict__ dst, const float* sp, long long n) {
  for (long long e0 = threadIdx.x; e0 < n; e0 += 8 * kSplThreads) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const long long e = e0 + u * kSplThreads;
      if (e < n) dst[e] = sp[e];
    }
  }
}

// Forward: log-det summed per row in dim order through LDS.
template <int KT>
__global__ __launch_bounds__(kSplThreads) void spline_fwd_kernel(const float* __restrict__ s_in,
                                                                 float* __restrict__ s_out,
                                                                 const float* __restrict__ P, float* __restrict__ ld,
                                                                 int B, int D, int dt, int K, int rot) {
  extern __shared__ float sp[];
  __shared__ float lds[kSplThreads];
  const int S = 3 * K - 1, rpb = kSplThreads / dt;
  const int lr = threadIdx.x / dt, d = threadIdx.x - lr * dt;
  const long long b0 = (long long)blockIdx.x * rpb, b = b0 + lr;
  const int nrows = (int)(B - b0 < rpb ? B - b0 : rpb);
  const bool ok = lr < nrows;
  const int col = pmodi(d + rot, D);
  const float xv = ok ? s_in[b * D + col] : 0.f;  // in flight with the staging loads
  stage_rows(sp, P + b0 * dt * S, (long long)nrows * dt * S);
  __syncthreads();
  if (ok) {
    for (int j = dt + d; j < D; j += dt) {
      const int cj = pmodi(j + rot, D);
      s_out[b * D + cj] = s_in[b * D + cj];
    }
    float y, ldv;
    spline_one<false, KT>(sp + threadIdx.x * S, K, xv, y, ldv, 0.f, 0.f, nullptr, nullptr);
    s_out[b * D + col] = y;
    lds[threadIdx.x] = ldv;
  }
  __syncthreads();
  if (ok && d == 0) {
    float l = 0.f;
    for (int k = 0; k < dt; ++k) l = l + lds[threadIdx.x + k];
    ld[b] = ld[b] + l;
  }
}

// Inverse (the layered eval path's Chain.inverse; utils.py:144-202): the same
// per-(row, dim) layout and staging; knots normalized as spline_one forms
// them, bin search and quadratic root as the fused kernels (zf_spline.h).
struct RawKnots {
  const float* p;
  int K;
  float Sa, Sb, rSa, rSb, cc, norm, rnorm;
  __device__ float w(int j) const { return t_div(t_div(sp_f(p[j]), Sa, rSa) + cc, norm, rnorm); }
  __device__ float h(int j) const { return t_div(t_div(sp_f(p[K + j]), Sb, rSb) + cc, norm, rnorm); }
  __device__ float d(int j) const { return sp_f(p[2 * K + j]); }
};

__device__ __forceinline__ float spline_inv_one(const float* p, int K, float y) {
  RawKnots q;
  q.p = p;
  q.K = K;
  const double c64 = 1e-5 / (1.0 - (double)K * 1e-5);  // utils.py:32-34, Python floats
  q.cc = (float)c64;
  q.norm = (float)(1.0 + c64 * (double)K);
  float Sa = 0.f, Sb = 0.f;
  for (int j = 0; j < K; ++j) {
    Sa = Sa + sp_f(p[j]);
    Sb = Sb + sp_f(p[K + j]);
  }
  q.Sa = Sa;
  q.Sb = Sb;
  q.rSa = t_rcp(Sa);
  q.rSb = t_rcp(Sb);
  q.rnorm = t_rcp(q.norm);
  const RqsBin b = rqs_bin<false>(y, K, q);
  return rqs_inverse_eval(y, b);
}

__global__ __launch_bounds__(kSplThreads) void spline_inv_kernel(const float* __restrict__ s_in,
                                                                 float* __restrict__ s_out,
                                                                 const float* __restrict__ P, int B, int D, int dt,
                                                                 int K, int rot) {
  extern __shared__ float sp[];
  const int S = 3 * K - 1, rpb = kSplThreads / dt;
  const int lr = threadIdx.x / dt, d = threadIdx.x - lr * dt;
  const long long b0 = (long long)blockIdx.x * rpb, b = b0 + lr;
  const int nrows = (int)(B - b0 < rpb ? B - b0 : rpb);
  const bool ok = lr < nrows;
  const int col = pmodi(d + rot, D);
  const float yv = ok ? s_in[b * D + col] : 0.f;
  stage_rows(sp, P + b0 * dt * S, (long long)nrows * dt * S);
  __syncthreads();
  if (!ok) return;
  for (int j = dt + d; j < D; j += dt) {
    const int cj = pmodi(j + rot, D);
    s_out[b * D + cj] = s_in[b * D + cj];
  }
  s_out[b * D + col] = spline_inv_one(sp + threadIdx.x * S, K, yv);
}

// Reverse: g_in = dL/d(state_in) from g_out = dL/d(state_out) and gl per row;
// conditioning columns pass g_out through (their MLP share is added later).
// dL/dP is formed in place in the staged rows and written back coalesced.
template <int KT>
__global__ __launch_bounds__(kSplThreads) void spline_bwd_kernel(const float* __restrict__ s_in,
                                                                 const float* __restrict__ P,
                                                                 const float* __restrict__ g_out, float gl,
                                                                 float* __restrict__ g_in, float* __restrict__ gP,
                                                                 int B, int D, int dt, int K, int rot) {
  extern __shared__ float sp[];
  const int S = 3 * K - 1, rpb = kSplThreads / dt;
  const int lr = threadIdx.x / dt, d = threadIdx.x - lr * dt;
  const long long b0 = (long long)blockIdx.x * rpb, b = b0 + lr;
  const int nrows = (int)(B - b0 < rpb ? B - b0 : rpb);
  const long long n = (long long)nrows * dt * S;
  const bool ok = lr < nrows;
  const int col = pmodi(d + rot, D);
  const float xv = ok ? s_in[b * D + col] : 0.f, gv = ok ? g_out[b * D + col] : 0.f;  // in flight with the staging
  stage_rows(sp, P + b0 * dt * S, n);
  __syncthreads();
  if (ok) {
    for (int j = dt + d; j < D; j += dt) {
      const int cj = pmodi(j + rot, D);
      g_in[b * D + cj] = g_out[b * D + cj];
    }
    float y, ldv, gx;
    float* row = sp + threadIdx.x * S;
    spline_one<true, KT>(row, K, xv, y, ldv, gv, gl, &gx, row);
    g_in[b * D + col] = gx;
  }
  __syncthreads();
  unstage_rows(gP + b0 * dt * S, sp, n);
}

// BatchNorm reverse with batch statistics:
// gU = rstd * (gUhat - mean(gUhat) - u_hat * mean(gUhat * u_hat)), gUhat = gUbn * scale.
__global__ void bn_bwd_kernel(const float* __restrict__ gUbn, const float* __restrict__ Uhat,
                              const float* __restrict__ scale, const float* __restrict__ rstd,
                              const double* __restrict__ sum_g, const double* __restrict__ sum_gu,
                              float* __restrict__ gU, int B, long long Bg, int DC) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)B * DC) return;
  const int k = (int)(i % DC);
  // sum_g / sum_gu: global sums of gUbn and gUbn*Uhat; scaled into gUhat terms
  const float mg = bn_mean_term(scale[k], sum_g[k], Bg), mgu = bn_mean_term(scale[k], sum_gu[k], Bg);
  gU[i] = bn_grad_in(gUbn[i], Uhat[i], scale[k], rstd[k], mg, mgu);
}

// ---- small batches: BatchNorm forward / reverse in one single-block launch --
// (B * DC <= kBnSmall, one device).  The same arithmetic as the multi-launch
// path (gather_u + leaf_colsums + tree + bn_stats + bn_apply forward;
// leaf_colsums + tree + bn_bwd + scatter reverse): the same leaf_sums2 per
// (leaf, column) and the same tree_n over the leaves, here through LDS.
constexpr long long kBnSmall = 1ll << 14;
constexpr int kBnLeafCap = kLeafCap;  // leaves of a BatchNorm sum (both paths)

__global__ __launch_bounds__(1024) void bn_fwd_small(const float* __restrict__ s, const float* __restrict__ c,
                                                     float* __restrict__ Uhat, float* __restrict__ Ubn,
                                                     float* __restrict__ nat_bn, float* __restrict__ mean_out,
                                                     float* __restrict__ rstd_out, int B, int D, int C, int dt, int dc,
                                                     int rot, int n, int rows, int update) {
  __shared__ double p1[kMaxLeaves * 64], p2[kMaxLeaves * 64];
  __shared__ float smean[64], srstd[64];
  const int DC = dc + C, tid = threadIdx.x;
  auto u_at = [&](long long b, int kk) { return kk < dc ? s[b * D + pmodi(dt + kk + rot, D)] : c[b * C + (kk - dc)]; };
  for (int t = tid; t < n * DC; t += 1024) {
    const int z = t / DC, k = t - z * DC;
    const int b0 = min(B, z * rows), b1 = min(B, b0 + rows);
    leaf_sums2([&](int b) { return u_at(b, k); }, [&](int b) { return u_at(b, k); }, b0, b1, p1[t], p2[t]);
  }
  __syncthreads();
  lds_tree2(p1, p2, n, DC, DC);
  if (tid < DC) {
    float mean, rstd;
    bn_stats_one(p1[tid], p2[tid], B, tid, DC, nat_bn, mean, rstd, update);
    smean[tid] = mean;
    srstd[tid] = rstd;
    mean_out[tid] = mean;
    rstd_out[tid] = rstd;
  }
  __syncthreads();
  const float* scale = nat_bn + 2 * DC;
  const float* bias = nat_bn + 3 * DC;
  for (long long i = tid; i < (long long)B * DC; i += 1024) {
    const long long b = i / DC;
    const int kk = (int)(i - b * DC);
    const float uh = bn_hat(u_at(b, kk), smean[kk], srstd[kk]);
    Uhat[i] = uh;
    Ubn[i] = bn_out(uh, scale[kk], bias[kk]);
  }
}

// gUbn = dL/dUbn -> BatchNorm scale / bias gradients (fp64 accumulator) and
// dL/dU; the conditioning columns' share is added to g (dL/d state) in place.
__global__ __launch_bounds__(1024) void bn_bwd_small(const float* __restrict__ gUbn, const float* __restrict__ Uhat,
                                                     const float* __restrict__ scale, const float* __restrict__ rstd,
                                                     double* __restrict__ g_scale, double* __restrict__ g_bias,
                                                     float* __restrict__ g, int B, int D, int C, int dt, int dc,
                                                     int rot, int n, int rows) {
  __shared__ double p1[kMaxLeaves * 64], p2[kMaxLeaves * 64];
  __shared__ float mg_s[64], mgu_s[64];
  const int DC = dc + C, tid = threadIdx.x;
  for (int t = tid; t < n * DC; t += 1024) {
    const int z = t / DC, k = t - z * DC;
    const int b0 = min(B, z * rows), b1 = min(B, b0 + rows);
    leaf_sums2([&](int b) { return gUbn[(long long)b * DC + k]; }, [&](int b) { return Uhat[(long long)b * DC + k]; },
               b0, b1, p1[t], p2[t]);
  }
  __syncthreads();
  lds_tree2(p1, p2, n, DC, DC);
  if (tid < DC) {
    const double sg = p1[tid], sgu = p2[tid];
    g_scale[tid] = sgu;
    g_bias[tid] = sg;
    mg_s[tid] = bn_mean_term(scale[tid], sg, B);
    mgu_s[tid] = bn_mean_term(scale[tid], sgu, B);
  }
  __syncthreads();
  for (long long i = tid; i < (long long)B * dc; i += 1024) {
    const long long b = i / dc;
    const int kk = (int)(i - b * dc);
    const long long e = b * DC + kk;
    const float gu = bn_grad_in(gUbn[e], Uhat[e], scale[kk], rstd[kk], mg_s[kk], mgu_s[kk]);
    // a separately rounded add (no fma with the product above), as the
    // multi-launch path's scatter_gu_kernel adds a stored gU
    float* gp = g + b * D + pmodi(dt + kk + rot, D);
    *gp = add_rn(*gp, gu);
  }
}

__global__ void scatter_gu_kernel(const float* __restrict__ gU, float* __restrict__ g, int B, int D, int C, int dt,
                                  int dc, int rot) {
  const int DC = dc + C;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)B * dc) return;
  const long long b = i / dc;
  const int k = (int)(i - b * dc);
  float* gp = g + b * D + pmodi(dt + k + rot, D);
  *gp = add_rn(*gp, gU[b * DC + k]);
}

// ---- latent + loss ------------------------------------------------------------
// lp = latent.log_prob(z) + log_det, nan_to_num (flow.py:45-47); per-row
// loss terms -lp/Bg (fp64, summed by the leaf tree); gz = -(1/Bg) d latent_lp
// / dz (zero where lp is not finite).  Bg: the global batch size.
// leaf_rows > 0 (a divisor of the 256-row block): the block also forms the
// loss leaf sums of its rows in row order, as leaf_sum_kernel does, into
// leaf[block's leaves], the last block zeroing leaves past the last row
// (one launch fewer per step).
__global__ __launch_bounds__(256) void latent_loss_kernel(const float* __restrict__ z, const float* __restrict__ ld,
                                                          int B, long long Bg, int D, int rot, int latent, float a,
                                                          float betac, float tnmass, float* __restrict__ gz,
                                                          double* __restrict__ row_loss, int leaf_rows,
                                                          int leaf_n, double* __restrict__ leaf) {
  __shared__ double rl[256];
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) {
    float lat = 0.f;
    for (int j = 0; j < D; ++j) {
      const float v = z[(long long)b * D + pmodi(j + rot, D)];
      float t;
      if (latent == ZF_LATENT_NORMAL || latent == ZF_LATENT_TRUNCNORM) {
        const float dv = v - 0.5f;
        t = (logf(6.28318530717958647692f * 0.01f) + (dv * dv) / 0.01f) / -2.0f;
        if (latent == ZF_LATENT_TRUNCNORM) {
          t = t - tnmass;
          if (dv / 0.1f < -5.f || dv / 0.1f > 5.f) t = -INFINITY;
        }
      } else if (latent == ZF_LATENT_BETA) {
        const float am1 = a - 1.0f;
        t = betac + (am1 == 0.f ? 0.f : am1 * logf(v)) + (am1 == 0.f ? 0.f : am1 * log1pf(-v));
        if (v > 1.f || v < 0.f) t = -INFINITY;
      } else {
        t = (v > 1.f || v < 0.f) ? -INFINITY : 0.f;
      }
      lat = lat + t;
    }
    float lp = lat + ld[b];
    const bool fin = (lp == lp) && lp != INFINITY && lp != -INFINITY;
    if (lp != lp) lp = -INFINITY;
    if (lp == INFINITY) lp = 3.40282347e38f;
    if (lp == -INFINITY) lp = -3.40282347e38f;
    row_loss[b] = -(double)lp / (double)Bg;
    const float s = -1.0f / (float)Bg;
    for (int j = 0; j < D; ++j) {
      const int col = pmodi(j + rot, D);
      const float v = z[(long long)b * D + col];
      float g = 0.f;
      if (fin) {
        if (latent == ZF_LATENT_NORMAL || latent == ZF_LATENT_TRUNCNORM) g = -(v - 0.5f) / 0.01f;
        else if (latent == ZF_LATENT_BETA) g = (a - 1.0f) / v - (a - 1.0f) / (1.0f - v);
      }
      gz[(long long)b * D + col] = s * g;
    }
    rl[threadIdx.x] = -(double)lp / (double)Bg;
  }
  if (leaf_rows <= 0) return;
  __syncthreads();
  const int per = 256 / leaf_rows, z0 = blockIdx.x * 256;
  if ((int)threadIdx.x < per) {
    const int r0 = z0 + threadIdx.x * leaf_rows;
    if (r0 < B) {
      const int r1 = min(B, r0 + leaf_rows);
      double acc = 0.0;
      for (int r = r0; r < r1; ++r) acc += rl[r - z0];
      leaf[r0 / leaf_rows] = acc;
    }
  }
  if (blockIdx.x == gridDim.x - 1)  // the leaves past the last row are empty (0, as leaf_sum_kernel)
    for (int zl = (B + leaf_rows - 1) / leaf_rows + (int)threadIdx.x; zl < leaf_n; zl += 256) leaf[zl] = 0.0;
}

// ShiftBounds batch min / max of every rank (all-gathered [world][2][64]:
// min row, max row) -> the global min / max (a NaN anywhere stays NaN).
__global__ void minmax_ranks_kernel(const float* __restrict__ gath, int world, int D, float* __restrict__ cmin,
                                    float* __restrict__ cmax) {
  const int i = threadIdx.x;
  if (i >= D) return;
  float lo = gath[i], hi = gath[64 + i];
  for (int r = 1; r < world; ++r) {
    const float a = gath[r * 128 + i], b = gath[r * 128 + 64 + i];
    lo = (lo != lo || a != a) ? __builtin_nanf("") : fminf(lo, a);
    hi = (hi != hi || b != b) ? __builtin_nanf("") : fmaxf(hi, b);
  }
  cmin[i] = lo;
  cmax[i] = hi;
}

__device__ __forceinline__ void step_update(float* __restrict__ bc, float b1, float b2);

// bc != NULL: thread 0 also advances the optimiser's step counter (the step
// graph's launch before adam_kernel; step_kernel otherwise).
__global__ void cast_f64_f32_kernel(const double* __restrict__ x, long long n, float* __restrict__ y,
                                    float* __restrict__ bc = nullptr, float b1 = 0.f, float b2 = 0.f) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = (float)x[i];
  if (bc && i == 0) step_update(bc, b1, b2);
}

// ---- optimiser: optax adamw / nadamw ---------------------------------------
// scale_by_adam(b1, b2, eps, nesterov) -> add_decayed_weights(wd) -> scale(-lr)
// (optax/_src/transform.py, alias.py), masked to the parameter entries.
// Step count and bias corrections on the device (so a captured step graph
// replays correctly): bc[0] = step t (as float bits of an int), bc[1] =
// 1 - b1^t, bc[2] = 1 - b1^(t+1), bc[3] = 1 - b2^t.
__device__ __forceinline__ void step_update(float* __restrict__ bc, float b1, float b2) {
  int* cnt = reinterpret_cast<int*>(bc);
  const int t = *cnt + 1;
  *cnt = t;
  bc[1] = (float)(1.0 - pow((double)b1, (double)t));
  bc[2] = (float)(1.0 - pow((double)b1, (double)t + 1.0));
  bc[3] = (float)(1.0 - pow((double)b2, (double)t));
}

__global__ void step_kernel(float* __restrict__ bc, float b1, float b2) { step_update(bc, b1, b2); }

__global__ void adam_kernel(float* __restrict__ prm, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, const unsigned char* __restrict__ mask, long long n, float lr,
                            float b1, float b2, float eps, float wd, int nesterov, const float* __restrict__ bc) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !mask[i]) return;
  const float bc1 = bc[1], bc1n = bc[2], bc2 = bc[3];
  const float gi = g[i];
  const float mi = b1 * m[i] + (1.0f - b1) * gi;
  const float vi = b2 * v[i] + (1.0f - b2) * gi * gi;
  m[i] = mi;
  v[i] = vi;
  // bias corrections: bc1 = 1 - b1^t, bc1n = 1 - b1^(t+1), bc2 = 1 - b2^t
  const float mhat = nesterov ? b1 * (mi / bc1n) + (1.0f - b1) * (gi / bc1) : mi / bc1;
  const float vhat = vi / bc2;
  const float upd = mhat / (sqrtf(vhat) + eps) + wd * prm[i];
  prm[i] = prm[i] - lr * upd;
}

}  // namespace
}  // namespace zf

// ============================================================================
struct zf_trainer {
  zf_flow_desc desc;
  int D = 0, C = 0, n_ops = 0;
  int64_t nat_floats = 0;
  int64_t bmax = 0;
  zf_optim_desc opt;
  long long t = 0;  // optimiser step count (host mirror of d_step)
  std::vector<float> sb_modes, sb_prm;  // ShiftBounds pre-transform per dim (colstats)
  float* d_nat = nullptr;
  float* d_grad = nullptr;
  float* d_m = nullptr;
  float* d_v = nullptr;
  unsigned char* d_mask = nullptr;
  // arena: per-op saved activations + scratch
  std::vector<float*> bufs;
  std::vector<int64_t> sizes;
  float* d_state = nullptr;   // [n_ops + 1][bmax][D] states before each op
  float* d_c = nullptr;       // [bmax][C] conditioning inputs of the batch
  float* d_bc = nullptr;      // optimiser step count + bias corrections (step_kernel)
  // zf_trainer_step as one hipGraph per batch size (the body reads only the
  // trainer's own buffers: x and c are copied in before the launch)
  hipStream_t cap = nullptr;
  std::map<int64_t, hipGraphExec_t> graphs;
  bool use_graph = true;
  bool bn_small = true;  // ZF_TRAIN_BN_SMALL=0: always the multi-launch BatchNorm path
  bool splitq = true;    // ZF_TRAIN_SPLITQ=0: never the split-set GEMM (same bits either way)
  float* d_ld = nullptr;      // [bmax]
  float* d_g0 = nullptr;      // [bmax][D]
  float* d_g1 = nullptr;
  float* d_small = nullptr;   // per-column scratch (ShiftBounds min / max)
  double* d_leaf = nullptr;   // leaf partials of the BatchNorm sums / loss [kLeafCap][128]
  double* d_leaf2 = nullptr;  // first-level tree roots [kLeafCap / 64][128]
  double* d_ws2 = nullptr;    // first-level roots of the split-K partials
  double* d_roots = nullptr;  // [0,128): tree roots of one reduction; [128]: the loss
  double* d_rowloss = nullptr;  // [bmax] per-row loss terms
  double* d_g64 = nullptr;    // fp64 gradient accumulator (blob layout)
  // data parallelism: the communicator and its all-gather landing buffer
  zf_comm_desc comm{0, 1, nullptr, nullptr};
  void* d_gath = nullptr;
  int64_t gath_bytes = 0;
  void* d_colws = nullptr;
  float* d_ws = nullptr;      // split-K partials (kWsFloats)
  float* d_split = nullptr;   // split-set GEMM partials (kSplitFloats)
  int64_t colws_bytes = 0;
  struct NscBufs {
    float *U, *Uhat, *Ubn, *P, *gP, *gU, *gA, *gB;
    std::vector<float*> Z, H;
    float *mean, *rstd;
  };
  std::vector<NscBufs> nsc;
};

namespace zf {
namespace {

float* dmalloc(zf_trainer* t, int64_t n, int& rc) {
  if (rc) return nullptr;
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, (size_t)(n > 0 ? n : 1) * sizeof(float));
  if (e != hipSuccess) {
    rc = hip_status(e, "zf_trainer alloc");
    return nullptr;
  }
  t->bufs.push_back((float*)p);
  return (float*)p;
}

int nsc_dims(const zf_trainer* t, const zf_op_desc& op, int& dt, int& dc, int& DC, int& S) {
  dt = t->D / 2;
  dc = t->D - dt;
  DC = dc + t->C;
  S = 3 * op.knots - 1;
  return ZF_OK;
}

}  // namespace
}  // namespace zf

extern "C" {

int zf_trainer_create(const zf_flow_desc* desc_in, const float* blob_host, int64_t blob_floats,
                      const unsigned char* param_mask, int64_t batch_max, const zf_optim_desc* opt,
                      zf_trainer_t** out) {
  if (!desc_in || !blob_host || !param_mask || !opt || !out) return zf::einval("NULL argument");
  *out = nullptr;
  zf_flow_desc desc = *desc_in;
  int64_t need = 0;
  int rc = zf_flow_plan(&desc, &need);
  if (rc) return rc;
  if (need != blob_floats) return zf::einval("blob has %lld floats, plan needs %lld", (long long)blob_floats, (long long)need);
  if (batch_max < 1 || batch_max > (1 << 24)) return zf::einval("batch_max outside [1, 2^24]");
  for (int i = 0; i < desc.n_ops; ++i) {
    const zf_op_desc& op = desc.ops[i];
    if (op.kind == ZF_OP_SHIFT_BOUNDS && i != 0)
      return zf::enotsup("training: ShiftBounds is supported only as the first bijector");
    if (op.kind == ZF_OP_NSC && op.knots > zf::kMaxK) return zf::enotsup("training: knots > 64");
    if (op.kind == ZF_OP_NSC && desc.dim - desc.dim / 2 + desc.cond_dim > 64)
      return zf::enotsup("training: more than 64 conditioner inputs");
  }
  zf_trainer* t = new zf_trainer();
  t->desc = desc;
  t->D = desc.dim;
  t->C = desc.cond_dim;
  t->n_ops = desc.n_ops;
  t->nat_floats = need;
  t->bmax = batch_max;
  t->opt = *opt;
  const int64_t B = batch_max, D = desc.dim;
  if (desc.n_ops > 0 && desc.ops[0].kind == ZF_OP_SHIFT_BOUNDS) {
    const float* row = blob_host + desc.ops[0].off_sb;
    for (int j = 0; j < D; ++j) {
      const int mode = (int)row[8 * j];
      t->sb_modes.push_back((float)mode);
      t->sb_prm.push_back(mode == ZF_SB_LOWER ? row[8 * j + 1] : row[8 * j + 2]);
    }
  }
  rc = ZF_OK;
  t->d_nat = zf::dmalloc(t, need, rc);
  t->d_grad = zf::dmalloc(t, need, rc);
  t->d_m = zf::dmalloc(t, need, rc);
  t->d_v = zf::dmalloc(t, need, rc);
  t->d_mask = (unsigned char*)zf::dmalloc(t, (need + 3) / 4, rc);
  t->d_state = zf::dmalloc(t, (int64_t)(desc.n_ops + 1) * B * D, rc);
  t->d_ld = zf::dmalloc(t, B, rc);
  t->d_g0 = zf::dmalloc(t, B * D, rc);
  t->d_g1 = zf::dmalloc(t, B * D, rc);
  t->d_small = zf::dmalloc(t, 8 * 256, rc);
  t->d_leaf = (double*)zf::dmalloc(t, 2 * zf::kLeafCap * 128, rc);
  t->d_leaf2 = (double*)zf::dmalloc(t, 2 * (zf::kLeafCap / zf::kMaxLeaves) * 128, rc);
  t->d_ws2 = (double*)zf::dmalloc(t, 2 * (zf::kWsFloats / zf::kMaxLeaves), rc);
  t->d_roots = (double*)zf::dmalloc(t, 2 * 256, rc);
  t->d_rowloss = (double*)zf::dmalloc(t, 2 * B, rc);
  t->d_g64 = (double*)zf::dmalloc(t, 2 * need, rc);
  if (!rc) {
    const hipError_t e = hipMemset(t->d_g64, 0, (size_t)need * sizeof(double));  // 2 need floats
    if (e != hipSuccess) rc = zf::hip_status(e, "zf_trainer_create gradient");
  }
  t->d_ws = zf::dmalloc(t, zf::kWsFloats, rc);
  t->d_split = zf::dmalloc(t, zf::kSplitFloats, rc);
  t->d_c = zf::dmalloc(t, B * (desc.cond_dim > 0 ? desc.cond_dim : 1), rc);
  t->d_bc = zf::dmalloc(t, 4, rc);
  {
    const char* g = std::getenv("ZF_TRAIN_GRAPH");
    t->use_graph = !(g && g[0] == '0');
    const char* bs = std::getenv("ZF_TRAIN_BN_SMALL");
    t->bn_small = !(bs && bs[0] == '0');
    const char* sq = std::getenv("ZF_TRAIN_SPLITQ");
    t->splitq = !(sq && sq[0] == '0');
  }
  if (!rc) {
    hipError_t e = hipStreamCreateWithFlags(&t->cap, hipStreamNonBlocking);
    if (e != hipSuccess) rc = zf::hip_status(e, "zf_trainer_create stream");
  }
  t->colws_bytes = zf_colstats_workspace_bytes(B, 64);
  t->d_colws = zf::dmalloc(t, t->colws_bytes / 4 + 1, rc);
  t->nsc.resize(desc.n_ops);
  for (int i = 0; i < desc.n_ops && !rc; ++i) {
    const zf_op_desc& op = desc.ops[i];
    if (op.kind != ZF_OP_NSC) continue;
    int dt, dc, DC, S;
    zf::nsc_dims(t, op, dt, dc, DC, S);
    zf_trainer::NscBufs& nb = t->nsc[i];
    nb.U = zf::dmalloc(t, B * DC, rc);
    nb.Uhat = zf::dmalloc(t, B * DC, rc);
    nb.Ubn = zf::dmalloc(t, B * DC, rc);
    nb.gU = zf::dmalloc(t, B * DC, rc);
    nb.P = zf::dmalloc(t, B * dt * S, rc);
    nb.gP = zf::dmalloc(t, B * dt * S, rc);
    int hmax = 0;
    for (int l = 0; l < op.n_hidden; ++l) {
      nb.Z.push_back(zf::dmalloc(t, B * op.hidden[l], rc));
      nb.H.push_back(zf::dmalloc(t, B * op.hidden[l], rc));
      hmax = op.hidden[l] > hmax ? op.hidden[l] : hmax;
    }
    nb.gA = zf::dmalloc(t, B * hmax, rc);
    nb.gB = zf::dmalloc(t, B * hmax, rc);
    nb.mean = zf::dmalloc(t, DC, rc);
    nb.rstd = zf::dmalloc(t, DC, rc);
  }
  hipError_t e = hipSuccess;
  if (!rc) e = hipMemcpy(t->d_nat, blob_host, need * sizeof(float), hipMemcpyHostToDevice);
  if (!rc && e == hipSuccess) e = hipMemcpy(t->d_mask, param_mask, need, hipMemcpyHostToDevice);
  if (!rc && e == hipSuccess) e = hipMemset(t->d_m, 0, need * sizeof(float));
  if (!rc && e == hipSuccess) e = hipMemset(t->d_v, 0, need * sizeof(float));
  if (!rc && e == hipSuccess) e = hipMemset(t->d_bc, 0, 4 * sizeof(float));
  if (!rc && e != hipSuccess) rc = zf::hip_status(e, "zf_trainer_create");
  if (rc) {
    zf_trainer_destroy(t);
    return rc;
  }
  *out = t;
  return ZF_OK;
}

int zf_trainer_destroy(zf_trainer_t* t) {
  if (!t) return ZF_OK;
  (void)hipDeviceSynchronize();
  for (auto& kv : t->graphs) (void)hipGraphExecDestroy(kv.second);
  if (t->cap) (void)hipStreamDestroy(t->cap);
  for (float* p : t->bufs) (void)hipFree(p);
  if (t->d_gath) (void)hipFree(t->d_gath);
  delete t;
  return ZF_OK;
}

int zf_trainer_set_comm(zf_trainer_t* t, const zf_comm_desc* comm) {
  if (!t) return zf::einval("trainer is NULL");
  zf_comm_desc c{0, 1, nullptr, nullptr};
  if (comm) c = *comm;
  if (c.world < 1 || c.rank < 0 || c.rank >= c.world) return zf::einval("bad rank %d / world %d", c.rank, c.world);
  if (c.world > zf::kMaxLeaves) return zf::enotsup("training: more than 64 ranks");
  if (c.world > 1 && !c.allgather) return zf::einval("communicator without allgather");
  // the gather buffer only grows (largest exchange: the fp64 gradient of
  // every rank), and stays allocated while the communicator is cleared for a
  // one-device step (train(): a batch with fewer rows than ranks, once per
  // epoch), so clearing / restoring it costs no device sync or allocation
  const int64_t need =
      c.world > 1 ? std::max<int64_t>(t->nat_floats, 256) * (int64_t)sizeof(double) * c.world : 0;
  if (need > t->gath_bytes) {
    ZF_TRY_HIP(hipDeviceSynchronize());
    if (t->d_gath) (void)hipFree(t->d_gath);
    t->d_gath = nullptr;
    t->gath_bytes = 0;
    ZF_TRY_HIP(hipMalloc(&t->d_gath, (size_t)need));
    t->gath_bytes = need;
  }
  t->comm = c;
  return ZF_OK;
}

}  // extern "C"

namespace zf {
namespace {

// Copy the batch into the trainer's buffers (state 0, d_c).
int trainer_stage(zf_trainer_t* t, const float* x, const float* c, int64_t B64, hipStream_t st) {
  if (!t) return einval("trainer is NULL");
  if (B64 < 1 || B64 > t->bmax) return einval("batch %lld outside [1, %lld]", (long long)B64, (long long)t->bmax);
  if (!x) return einval("x is NULL");
  if (t->C > 0 && !c) return einval("flow is conditional but c is NULL");
  ZF_TRY_HIP(hipMemcpyAsync(t->d_state, x, (size_t)B64 * t->D * sizeof(float), hipMemcpyDeviceToDevice, st));
  if (t->C > 0)
    ZF_TRY_HIP(hipMemcpyAsync(t->d_c, c, (size_t)B64 * t->C * sizeof(float), hipMemcpyDeviceToDevice, st));
  return ZF_OK;
}

inline double* loss_slot(zf_trainer_t* t) { return t->d_roots + 128; }

// Data parallelism: this rank's tree roots (n doubles, in place) -> the
// global ones: all-gather every rank's roots, combine them by the top of the
// leaf tree (tree_n over ranks).  Nothing to do on one device.
int dp_combine(zf_trainer_t* t, double* roots, long long n, hipStream_t st) {
  const int W = t->comm.world;
  if (W <= 1) return ZF_OK;
  if ((int64_t)n * (int64_t)sizeof(double) * W > t->gath_bytes) return einval("all-gather buffer too small");
  const int rc = t->comm.allgather(t->comm.ctx, roots, t->d_gath, (size_t)n * sizeof(double), st);
  if (rc) return rc;
  return launch_tree_cols((const double*)t->d_gath, W, n, roots, st);
}

// Train-mode forward + loss + reverse pass from the staged batch of B rows
// (this rank's shard of a global batch of Bg rows); the loss lands in
// loss_slot(t), the gradient in G (natural blob layout, fp32).
// step_in_cast: an optimiser update follows; the one-device gradient cast
// advances its step counter (trainer_update then skips step_kernel).
int trainer_body(zf_trainer_t* t, int B, long long Bg, int update_stats, float* G, hipStream_t st,
                 bool* step_in_cast = nullptr) {
  const int D = t->D, C = t->C, W = t->comm.world;
  const float* c = t->d_c;
  const zf_flow_desc& desc = t->desc;
  float* nat = t->d_nat;
  double* G64 = t->d_g64;
  // state before op i; Roll is an index rotation, so it aliases its input
  std::vector<float*> sp(desc.n_ops + 1);
  sp[0] = t->d_state;
  for (int i = 0; i < desc.n_ops; ++i)
    sp[i + 1] = desc.ops[i].kind == ZF_OP_ROLL ? sp[i] : t->d_state + (int64_t)(i + 1) * t->bmax * D;
  auto state = [&](int i) { return sp[i]; };
  // a leading ShiftBounds sets ld itself (sb_forward_kernel, first)
  if (desc.n_ops == 0 || desc.ops[0].kind != ZF_OP_SHIFT_BOUNDS)
    ZF_TRY_HIP(hipMemsetAsync(t->d_ld, 0, (size_t)B * sizeof(float), st));
  const Leaves lbn = leaves_for(B, Bg, W, kBnLeafCap);
  // the single-block BatchNorm kernels have no exchange point (one device only)
  const bool small_ok = W == 1 && t->bn_small;
  int rc;
  // ---- forward (train mode) ----
  int rot = 0;
  std::vector<int> rots(desc.n_ops + 1, 0);
  for (int i = 0; i < desc.n_ops; ++i) {
    const zf_op_desc& op = desc.ops[i];
    rots[i] = rot;
    float* sin = state(i);
    float* sout = state(i + 1);
    if (op.kind == ZF_OP_ROLL) {
      rot = zf::pmodi(rot - op.shift, D);
    } else if (op.kind == ZF_OP_SHIFT_BOUNDS) {
      float* sb = nat + op.off_sb;
      // batch min / max of the (safe_log-transformed) columns (first op: rot == 0)
      rc = zf_colstats(sin, B, D, D, 0, t->sb_modes.data(), t->sb_prm.data(), t->d_small, t->d_small + 64,
                       nullptr, nullptr, t->d_colws, st);
      if (rc) return rc;
      if (W > 1) {  // min / max over all ranks (exact in any order)
        rc = t->comm.allgather(t->comm.ctx, t->d_small, t->d_gath, 128 * sizeof(float), st);
        if (rc) return rc;
        hipLaunchKernelGGL(minmax_ranks_kernel, dim3(1), dim3(64), 0, st, (const float*)t->d_gath, W, D,
                           t->d_small, t->d_small + 64);
        ZF_CHECK_LAUNCH("minmax_ranks_kernel");
      }
      hipLaunchKernelGGL(zf::sb_forward_kernel, dim3(zf::blocks_for(B)), dim3(256), 0, st, sin, sout, t->d_ld, sb, B,
                         D, rot, (const float*)t->d_small, (const float*)(t->d_small + 64), update_stats,
                         i == 0 ? 1 : 0);
      ZF_CHECK_LAUNCH("sb_forward_kernel");
    } else if (op.kind == ZF_OP_NSC) {
      int dt, dc, DC, S;
      zf::nsc_dims(t, op, dt, dc, DC, S);
      zf_trainer::NscBufs& nb = t->nsc[i];
      float* bn = nat + op.off_bn;  // [mean, var, scale, bias]
      if (small_ok && (long long)B * DC <= zf::kBnSmall) {
        hipLaunchKernelGGL(zf::bn_fwd_small, dim3(1), dim3(1024), 0, st, sin, c, nb.Uhat, nb.Ubn, bn, nb.mean,
                           nb.rstd, B, D, C, dt, dc, rot, lbn.n, lbn.rows, update_stats);
        ZF_CHECK_LAUNCH("bn_fwd_small");
      } else {
        hipLaunchKernelGGL(zf::gather_u_kernel, dim3(zf::blocks_for((int64_t)B * DC)), dim3(256), 0, st, sin, c,
                           nb.U, B, D, C, dt, dc, rot);
        ZF_CHECK_LAUNCH("gather_u_kernel");
        // column sums / sums of squares: leaves -> tree -> (ranks) -> statistics
        hipLaunchKernelGGL(leaf_colsums_kernel, dim3(blocks_for((int64_t)lbn.n * DC)), dim3(256), 0, st, nb.U,
                           nullptr, B, DC, lbn.rows, lbn.n, t->d_leaf);
        ZF_CHECK_LAUNCH("leaf_colsums_kernel");
        if ((rc = launch_tree_cols(t->d_leaf, lbn.n, 2 * DC, t->d_roots, st, t->d_leaf2))) return rc;
        if ((rc = dp_combine(t, t->d_roots, 2 * DC, st))) return rc;
        hipLaunchKernelGGL(zf::bn_stats_kernel, dim3(1), dim3(64), 0, st, t->d_roots, t->d_roots + DC, Bg, DC, bn,
                           nb.mean, nb.rstd, update_stats);
        ZF_CHECK_LAUNCH("bn_stats_kernel");
        hipLaunchKernelGGL(zf::bn_apply_kernel, dim3(zf::blocks_for((int64_t)B * DC)), dim3(256), 0, st, nb.U,
                           nb.mean, nb.rstd, bn + 2 * DC, bn + 3 * DC, nb.Uhat, nb.Ubn, B, DC);
        ZF_CHECK_LAUNCH("bn_apply_kernel");
      }
      const float* in = nb.Ubn;
      int in_w = DC;
      for (int l = 0; l <= op.n_hidden; ++l) {
        const bool last = (l == op.n_hidden);
        const int out_w = last ? dt * S : op.hidden[l];
        float* Z = last ? nb.P : nb.Z[l];
        rc = zf::gemm(false, Bg, B, out_w, in_w, in, in_w, nat + op.off_w[l], out_w, Z, out_w, st, zf::kEpiBias,
                      nat + op.off_b[l], last ? nullptr : nb.H[l], nullptr, op.act, t->splitq ? t->d_split : nullptr,
                      zf::kSplitFloats);
        if (rc) return rc;
        if (!last) {
          in = nb.H[l];
          in_w = out_w;
        }
      }
      const int rpb = zf::kSplThreads / dt;
#define ZF_SPL(KTV) hipLaunchKernelGGL((zf::spline_fwd_kernel<KTV>), dim3(zf::blocks_for(B, rpb)), dim3(zf::kSplThreads),\
                         (size_t)zf::kSplThreads * S * sizeof(float), st, sin, sout, nb.P,\
                         t->d_ld, B, D, dt, op.knots, rot)
      ZF_KNOT_DISPATCH(op.knots, ZF_SPL);
#undef ZF_SPL
      ZF_CHECK_LAUNCH("spline_fwd_kernel");
    } else {
      return zf::einval("op %d: unknown kind", i);
    }
  }
  rots[desc.n_ops] = rot;
  // ---- latent + loss ----
  const int lt = desc.latent;
  const float a = (float)desc.latent_param;
  const float betac = lt == ZF_LATENT_BETA
                          ? (float)(-(std::lgamma(desc.latent_param) * 2.0 - std::lgamma(2.0 * desc.latent_param)))
                          : 0.f;
  const float tnm = (float)std::log1p(-2.0 * 0.5 * std::erfc(5.0 / std::sqrt(2.0)));
  float* g = t->d_g0;
  float* g_prev = t->d_g1;
  {
    const Leaves ll = leaves_for(B, Bg, W, kLeafCap);
    // leaves that tile the 256-row blocks are summed inside the loss kernel
    const bool fused = ll.rows > 0 && ll.rows <= 256 && 256 % ll.rows == 0;
    hipLaunchKernelGGL(zf::latent_loss_kernel, dim3(zf::blocks_for(B)), dim3(256), 0, st, state(desc.n_ops),
                       t->d_ld, B, Bg, D, rot, lt, a, betac, tnm, g, t->d_rowloss, fused ? ll.rows : 0, ll.n,
                       t->d_leaf);
    ZF_CHECK_LAUNCH("latent_loss_kernel");
    if (!fused) {
      hipLaunchKernelGGL(leaf_sum_kernel, dim3(blocks_for(ll.n, 64)), dim3(64), 0, st, t->d_rowloss, B, ll.rows,
                         ll.n, t->d_leaf);
      ZF_CHECK_LAUNCH("leaf_sum_kernel");
    }
    if ((rc = launch_tree_cols(t->d_leaf, ll.n, 1, loss_slot(t), st, t->d_leaf2))) return rc;
    if ((rc = dp_combine(t, loss_slot(t), 1, st))) return rc;
  }
  // ---- reverse ----
  // G64 needs no clearing per step: every parameter entry is assigned below
  // (the weight-gradient trees, the BatchNorm scale / bias gradients) and the
  // non-parameter entries (batch statistics, ShiftBounds rows) stay at the
  // zeros written once at zf_trainer_create
  const float gl = -1.0f / (float)Bg;  // d loss / d log_det of every op and row
  zf::WgradQueue wq;
  wq.tb.count = 0;
  wq.gq.count = 0;
  for (int i = desc.n_ops - 1; i >= 0; --i) {
    const zf_op_desc& op = desc.ops[i];
    if (op.kind == ZF_OP_ROLL || op.kind == ZF_OP_SHIFT_BOUNDS) continue;  // Roll: index map; SB: first op
    int dt, dc, DC, S;
    zf::nsc_dims(t, op, dt, dc, DC, S);
    zf_trainer::NscBufs& nb = t->nsc[i];
    const int r = rots[i];
    // spline: g -> g_prev (transformed columns), gP
    const int rpb = zf::kSplThreads / dt;
#define ZF_SPL(KTV) hipLaunchKernelGGL((zf::spline_bwd_kernel<KTV>), dim3(zf::blocks_for(B, rpb)), dim3(zf::kSplThreads),\
                       (size_t)zf::kSplThreads * S * sizeof(float), st, state(i), nb.P, g, gl,\
                       g_prev, nb.gP, B, D, dt, op.knots, r)
    ZF_KNOT_DISPATCH(op.knots, ZF_SPL);
#undef ZF_SPL
    ZF_CHECK_LAUNCH("spline_bwd_kernel");
    // MLP reverse
    const float* gout = nb.gP;
    int out_w = dt * S;
    float* gbufs[2] = {nb.gA, nb.gB};
    int which = 0;
    for (int l = op.n_hidden; l >= 0; --l) {
      const int in_w = l == 0 ? DC : op.hidden[l - 1];
      const float* hin = l == 0 ? nb.Ubn : nb.H[l - 1];
      // dW_l = hin^T . gout ; db_l = colsum(gout): leaves capped by the
      // split-K workspace (a power of two, the same on every rank)
      const int cap = pow2floor(std::min<int64_t>(kLeafCap, std::max<int64_t>(1, kWsFloats / ((int64_t)(in_w + 1) * out_w))));
      rc = zf::wgrad_deferred(wq, in_w, out_w, B, leaves_for(B, Bg, W, cap), hin, gout, G64 + op.off_w[l],
                              G64 + op.off_b[l], t->d_ws, t->d_ws2, st);
      if (rc) return rc;
      // g_in = gout . W_l^T
      float* gin = l == 0 ? nb.gU : gbufs[which];
      if ((rc = zf::wgrad_before_write(wq, gin, st))) return rc;  // a deferred dW GEMM still reads it
      // (through swish of layer l-1 when l > 0)
      rc = zf::gemm(true, Bg, B, in_w, out_w, gout, out_w, nat + op.off_w[l], out_w, gin, in_w, st,
                    l > 0 ? zf::kEpiDSwish : zf::kEpiNone, nullptr, nullptr, l > 0 ? nb.Z[l - 1] : nullptr, op.act,
                    t->splitq ? t->d_split : nullptr, zf::kSplitFloats);
      if (rc) return rc;
      if (l > 0) {
        gout = gin;
        out_w = in_w;
        which ^= 1;
      }
    }
    // BatchNorm: gU holds d loss / d Ubn
    float* bn = nat + op.off_bn;
    double* gbn = G64 + op.off_bn;
    if (small_ok && (long long)B * DC <= zf::kBnSmall) {
      hipLaunchKernelGGL(zf::bn_bwd_small, dim3(1), dim3(1024), 0, st, nb.gU, nb.Uhat, bn + 2 * DC, nb.rstd,
                         gbn + 2 * DC, gbn + 3 * DC, g_prev, B, D, C, dt, dc, r, lbn.n, lbn.rows);
      ZF_CHECK_LAUNCH("bn_bwd_small");
    } else {
      // sums of gUbn and gUbn * Uhat: leaves -> tree (this rank's share of the
      // scale / bias gradient) -> (ranks) -> the reverse formula's global sums
      hipLaunchKernelGGL(leaf_colsums_kernel, dim3(blocks_for((int64_t)lbn.n * DC)), dim3(256), 0, st, nb.gU,
                         nb.Uhat, B, DC, lbn.rows, lbn.n, t->d_leaf);
      ZF_CHECK_LAUNCH("leaf_colsums_kernel");
      if ((rc = launch_tree_cols(t->d_leaf, lbn.n, 2 * DC, t->d_roots, st, t->d_leaf2))) return rc;
      ZF_TRY_HIP(hipMemcpyAsync(gbn + 3 * DC, t->d_roots, DC * sizeof(double), hipMemcpyDeviceToDevice, st));
      ZF_TRY_HIP(hipMemcpyAsync(gbn + 2 * DC, t->d_roots + DC, DC * sizeof(double), hipMemcpyDeviceToDevice, st));
      if ((rc = dp_combine(t, t->d_roots, 2 * DC, st))) return rc;
      // gU := d loss / d U, in place (reads each element before writing it)
      hipLaunchKernelGGL(zf::bn_bwd_kernel, dim3(zf::blocks_for((int64_t)B * DC)), dim3(256), 0, st, nb.gU,
                         nb.Uhat, bn + 2 * DC, nb.rstd, t->d_roots, t->d_roots + DC, nb.gU, B, Bg, DC);
      ZF_CHECK_LAUNCH("bn_bwd_kernel");
      hipLaunchKernelGGL(zf::scatter_gu_kernel, dim3(zf::blocks_for((int64_t)B * dc)), dim3(256), 0, st, nb.gU,
                         g_prev, B, D, C, dt, dc, r);
      ZF_CHECK_LAUNCH("scatter_gu_kernel");
    }
    float* tmp = g;
    g = g_prev;
    g_prev = tmp;
  }
  if ((rc = zf::wgrad_flush(wq, st))) return rc;
  // ---- the gradient: (all ranks' fp64 shares, tree over ranks) -> fp32 ----
  if (W > 1) {
    rc = t->comm.allgather(t->comm.ctx, G64, t->d_gath, (size_t)t->nat_floats * sizeof(double), st);
    if (rc) return rc;
#define ZF_L(NM) hipLaunchKernelGGL((tree_cols_cast_kernel<NM>), dim3(blocks_for(t->nat_floats)), dim3(256), 0, st, \
                                    (const double*)t->d_gath, W, (long long)t->nat_floats, G)
    ZF_NMAX_DISPATCH(W, ZF_L);
#undef ZF_L
    ZF_CHECK_LAUNCH("tree_cols_cast_kernel");
  } else {
    hipLaunchKernelGGL(cast_f64_f32_kernel, dim3(blocks_for(t->nat_floats)), dim3(256), 0, st, G64,
                       (long long)t->nat_floats, G, step_in_cast ? t->d_bc : nullptr, t->opt.b1, t->opt.b2);
    ZF_CHECK_LAUNCH("cast_f64_f32_kernel");
    if (step_in_cast) *step_in_cast = true;
  }
  return ZF_OK;
}

int trainer_update(zf_trainer_t* t, hipStream_t st, bool step_done = false) {
  const zf_optim_desc& o = t->opt;
  if (!step_done) {
    hipLaunchKernelGGL(step_kernel, dim3(1), dim3(1), 0, st, t->d_bc, o.b1, o.b2);
    ZF_CHECK_LAUNCH("step_kernel");
  }
  hipLaunchKernelGGL(adam_kernel, dim3(blocks_for(t->nat_floats)), dim3(256), 0, st, t->d_nat, t->d_grad, t->d_m,
                     t->d_v, t->d_mask, (long long)t->nat_floats, o.learning_rate, o.b1, o.b2, o.eps, o.weight_decay,
                     o.nesterov, t->d_bc);
  ZF_CHECK_LAUNCH("adam_kernel");
  return ZF_OK;
}

// The whole step (body + optimiser) captured once per batch size.
int step_graph(zf_trainer_t* t, int B, hipGraphExec_t* out) {
  auto it = t->graphs.find(B);
  if (it != t->graphs.end()) {
    *out = it->second;
    return ZF_OK;
  }
  if (t->graphs.size() >= 8) {  // bound the cache (batch sizes rarely vary)
    ZF_TRY_HIP(hipStreamSynchronize(t->cap));
    ZF_TRY_HIP(hipDeviceSynchronize());
    for (auto& kv : t->graphs) (void)hipGraphExecDestroy(kv.second);
    t->graphs.clear();
  }
  ZF_TRY_HIP(hipStreamBeginCapture(t->cap, hipStreamCaptureModeThreadLocal));
  bool stepped = false;
  int rc = trainer_body(t, B, B, 1, t->d_grad, t->cap, &stepped);
  if (!rc) rc = trainer_update(t, t->cap, stepped);
  hipGraph_t g = nullptr;
  const hipError_t e = hipStreamEndCapture(t->cap, &g);
  if (!rc && e != hipSuccess) rc = hip_status(e, "hipStreamEndCapture");
  hipGraphExec_t exec = nullptr;
  if (!rc) {
    const hipError_t ei = hipGraphInstantiate(&exec, g, nullptr, nullptr, 0);
    if (ei != hipSuccess) rc = hip_status(ei, "hipGraphInstantiate");
  }
  if (g) (void)hipGraphDestroy(g);
  if (rc) return rc;
  t->graphs[B] = exec;
  *out = exec;
  return ZF_OK;
}

}  // namespace
}  // namespace zf

extern "C" {

int zf_trainer_loss_grad_shard(zf_trainer_t* t, const float* x, const float* c, int64_t rows, int64_t global_rows,
                               int update_stats, double* loss, float* grad, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  int rc = zf::trainer_stage(t, x, c, rows, st);
  if (rc) return rc;
  if (global_rows < rows || (t->comm.world == 1 && global_rows != rows))
    return zf::einval("global_rows %lld vs rows %lld (world %d)", (long long)global_rows, (long long)rows, t->comm.world);
  rc = zf::trainer_body(t, (int)rows, global_rows, update_stats, grad ? grad : t->d_grad, st);
  if (rc) return rc;
  if (loss) ZF_TRY_HIP(hipMemcpyAsync(loss, zf::loss_slot(t), sizeof(double), hipMemcpyDeviceToDevice, st));
  return ZF_OK;
}

int zf_trainer_loss_grad(zf_trainer_t* t, const float* x, const float* c, int64_t B, int update_stats,
                         double* loss, float* grad, void* stream) {
  if (!t) return zf::einval("trainer is NULL");
  return zf_trainer_loss_grad_shard(t, x, c, B, B * t->comm.world, update_stats, loss, grad, stream);
}

int zf_trainer_step_shard(zf_trainer_t* t, const float* x, const float* c, int64_t rows, int64_t global_rows,
                          double* loss, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  int rc = zf::trainer_stage(t, x, c, rows, st);
  if (rc) return rc;
  if (global_rows < rows || (t->comm.world == 1 && global_rows != rows))
    return zf::einval("global_rows %lld vs rows %lld (world %d)", (long long)global_rows, (long long)rows, t->comm.world);
  if (t->use_graph && t->comm.world == 1) {  // collectives are issued eagerly
    hipGraphExec_t exec = nullptr;
    rc = zf::step_graph(t, (int)rows, &exec);
    if (rc) return rc;
    ZF_TRY_HIP(hipGraphLaunch(exec, st));
  } else {
    bool stepped = false;
    rc = zf::trainer_body(t, (int)rows, global_rows, 1, t->d_grad, st, &stepped);
    if (!rc) rc = zf::trainer_update(t, st, stepped);
    if (rc) return rc;
  }
  t->t += 1;
  if (loss) ZF_TRY_HIP(hipMemcpyAsync(loss, zf::loss_slot(t), sizeof(double), hipMemcpyDeviceToDevice, st));
  return ZF_OK;
}

int zf_trainer_step(zf_trainer_t* t, const float* x, const float* c, int64_t B, double* loss, void* stream) {
  if (!t) return zf::einval("trainer is NULL");
  return zf_trainer_step_shard(t, x, c, B, B * t->comm.world, loss, stream);
}

int zf_trainer_get_blob(zf_trainer_t* t, float* blob_host) {
  if (!t || !blob_host) return zf::einval("NULL argument");
  ZF_TRY_HIP(hipDeviceSynchronize());
  ZF_TRY_HIP(hipMemcpy(blob_host, t->d_nat, t->nat_floats * sizeof(float), hipMemcpyDeviceToHost));
  return ZF_OK;
}

int zf_trainer_set_blob(zf_trainer_t* t, const float* blob_host) {
  if (!t || !blob_host) return zf::einval("NULL argument");
  ZF_TRY_HIP(hipDeviceSynchronize());
  ZF_TRY_HIP(hipMemcpy(t->d_nat, blob_host, t->nat_floats * sizeof(float), hipMemcpyHostToDevice));
  return ZF_OK;
}

}  // extern "C"

// ---- Entry points of the layered eval path (zf_layered.hip) -----------------
namespace zf {

int dense_gemm(long long Mg, int M, int N, int K, const float* A, int lda, const float* W, int ldw, float* C,
               int ldc, float* H, hipStream_t st, const float* bias, int act, unsigned* rmax) {
  if (rmax && M > 0) ZF_TRY_HIP(hipMemsetAsync(rmax, 0, (size_t)M * sizeof(unsigned), st));
  bool done = false;
  const int rc = gemm(false, Mg, M, N, K, A, lda, W, ldw, C, ldc, st, bias ? kEpiBias : kEpiNone, bias, H, nullptr,
                      act, nullptr, 0, rmax, &done);
  if (rc || !rmax || done || M <= 0) return rc;
  hipLaunchKernelGGL(row_absmax_kernel, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, st, M, N, H ? H : C, ldc, rmax);
  ZF_CHECK_LAUNCH("row_absmax_kernel");
  return ZF_OK;
}

int spline_rows(bool inverse, const float* s_in, float* s_out, const float* P, float* ld, int B, int D, int dt,
                int K, int rot, hipStream_t st) {
  if (B <= 0) return ZF_OK;
  // the layered eval path takes up to 200 knots (the block's rows of 3K - 1
  // parameters staged in LDS: 64 x 599 floats); training stays at kMaxK
  if (dt < 1 || dt > kSplThreads || K < 1 || K > 200) return enotsup("spline rows: transformed dims or knots out of range");
  const int S = 3 * K - 1, rpb = kSplThreads / dt;
  const size_t lds = (size_t)kSplThreads * S * sizeof(float);
  if (inverse) {
    hipLaunchKernelGGL(spline_inv_kernel, dim3(blocks_for(B, rpb)), dim3(kSplThreads), lds, st, s_in, s_out, P, B,
                       D, dt, K, rot);
    ZF_CHECK_LAUNCH("spline_inv_kernel");
    return ZF_OK;
  }
#define ZF_SPL(KTV)                                                                                          \
  hipLaunchKernelGGL((spline_fwd_kernel<KTV>), dim3(blocks_for(B, rpb)), dim3(kSplThreads), lds, st, s_in, \
                     s_out, P, ld, B, D, dt, K, rot)
  ZF_KNOT_DISPATCH(K, ZF_SPL);
#undef ZF_SPL
  ZF_CHECK_LAUNCH("spline_fwd_kernel");
  return ZF_OK;
}

}  // namespace zf
