// K1 — standalone rational-quadratic spline kernels at the `zenflow.utils`
// boundary (utils.rational_quadratic_spline_forward/inverse, utils.py:65-202;
// normalize_spline_params, utils.py:37-62).
//
// HBM-bound: per (row, dim) item the kernel reads x + dx[K] + dy[K] + slope[K-1]
// and writes y (+ one log_det per row): 4*(3K+1) bytes per item + 4 per row.
// K % 4 == 0 (4/8/16/32, 16-B aligned params): rqs_kernel_direct, one thread
// per item streaming its own dx/dy rows as dwordx4 straight to registers
// (no LDS staging or barrier between a wave's loads and its math: measured
// 2x the LDS-staged variant; 5.7-5.8 TB/s at K=16).  Other K: rqs_kernel,
// rows staged through LDS with an odd stride.  The row log-det is summed in
// dim order (utils.py:139), by lane shuffles where a row's items share a wave.
#include "zf_internal.h"
#include "zf_spline.h"

#include <cstdlib>

namespace zf {
namespace {

constexpr int kK1Threads = 256;
constexpr int kK1LdsBudgetFloats = 12288;  // 48 KiB per block

struct LdsParams {
  const float* dx;  // item stride K+1
  const float* dy;
  const float* sl;  // item stride K+1 (K-1 used)
  int ks;
  __device__ float w(int j) const { return dx[j]; }
  __device__ float h(int j) const { return dy[j]; }
  __device__ float d(int j) const { return sl[j]; }
};

// Copy `n` contiguous floats src[0..n) into LDS rows of `KX` values with
// stride `ks` (dst[(f/KX)*ks + f%KX]): dwordx4 loads (coalesced, 16 B/lane)
// where the source is 16-B aligned.  KX > 0 is a compile-time item width
// (constant-divisor index split); KX == 0 takes the runtime width `kx`.
template <int KX>
__device__ __forceinline__ void stage_rows(float* dst, const float* __restrict__ src, int64_t n,
                                           int kx, int ks) {
  const int K = KX > 0 ? KX : kx;
  const int tid = threadIdx.x;
  const uintptr_t addr = reinterpret_cast<uintptr_t>(src);
  int64_t head = 0;
  if (addr & 15) head = (16 - (addr & 15)) / 4;
  if (head > n) head = n;
  for (int64_t f = tid; f < head; f += blockDim.x) {
    const int it = (int)(f / K), j = (int)(f - (int64_t)it * K);
    dst[it * ks + j] = src[f];
  }
  const int nv = (int)((n - head) / 4);
  const float4* src4 = reinterpret_cast<const float4*>(src + head);
  const int h = (int)head;
  for (int q = tid; q < nv; q += blockDim.x) {
    const float4 v = src4[q];
    const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const unsigned f = (unsigned)(h + 4 * q + e);
      const unsigned it = f / (unsigned)K, j = f - it * (unsigned)K;
      dst[it * ks + j] = vv[e];
    }
  }
  for (int64_t f = head + 4 * (int64_t)nv + tid; f < n; f += blockDim.x) {
    const int it = (int)(f / K), j = (int)(f - (int64_t)it * K);
    dst[it * ks + j] = src[f];
  }
}

template <bool FWD, int KT>
__global__ __launch_bounds__(kK1Threads) void rqs_kernel(
    const float* __restrict__ xin, const float* __restrict__ dx, const float* __restrict__ dy,
    const float* __restrict__ slope, float* __restrict__ out, float* __restrict__ log_det,
    int64_t M, int N, int Kr, int R) {
  const int K = KT > 0 ? KT : Kr;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int ks = (K % 2 == 0) ? K + 1 : K + 2;  // odd LDS row stride: conflict-free
  const int64_t r0 = (int64_t)blockIdx.x * R;
  if (r0 >= M) return;
  const int rows = (int)((M - r0) < R ? (M - r0) : R);
  const int items = rows * N;
  const int64_t item0 = r0 * N;
  float* s_dx = lds;
  float* s_dy = s_dx + (size_t)R * N * ks;
  float* s_sl = s_dy + (size_t)R * N * ks;
  float* s_ld = s_sl + (size_t)R * N * ks;

  stage_rows<KT>(s_dx, dx + item0 * K, (int64_t)items * K, K, ks);
  stage_rows<KT>(s_dy, dy + item0 * K, (int64_t)items * K, K, ks);
  if (K > 1)
    stage_rows<(KT > 1 ? KT - 1 : 0)>(s_sl, slope + item0 * (K - 1), (int64_t)items * (K - 1), K - 1, ks);
  __syncthreads();

  const int i = threadIdx.x;
  if (i < items) {
    const float v = xin[item0 + i];
    LdsParams p{s_dx + i * ks, s_dy + i * ks, s_sl + i * ks, ks};
    const RqsBin b = rqs_bin<FWD>(v, K, p);
    if (FWD) {
      float y, ld;
      rqs_forward_eval(v, b, y, ld);
      if (out) out[item0 + i] = y;
      s_ld[i] = ld;
    } else {
      out[item0 + i] = rqs_inverse_eval(v, b);
    }
  }
  if (FWD && log_det) {
    __syncthreads();
    if (i < rows) {
      float acc = 0.f;  // log_det.sum(axis=1), dim order
      for (int n = 0; n < N; ++n) acc = acc + s_ld[i * N + n];
      log_det[r0 + i] = acc;
    }
  }
}

// Direct (no-LDS) path for K % 4 == 0: one thread per (row, dim) item reads
// its own dx/dy rows as K/4 dwordx4 each (a 64-B row per array at K=16; the
// thread consumes every byte it fetches) and keeps the knots in registers.
// Slopes (SM): 0 = gather only the two the bin needs, after the search;
// 1 = load the whole slope row with the knots and pick the two in the search
// sweep (no dependent second memory round trip).  Measured (bench_rqs, same
// box): SM 1 +5% at K = 16 (forward 0.667 -> 0.70 of HBM, inverse 0.69 ->
// 0.715), -12% at K = 32 (register pressure), even at K = 8; the aligned-
// float4 window form of SM 1 lost at every K.  Nothing is staged, no barrier
// sits between a wave's loads and its math, so every wave streams
// independently.  The row log-det (sum over N dims, dim order) goes by lane
// shuffles (N a power of two) or through a tiny LDS array.
template <bool FWD, int K, int SM>
__global__ __launch_bounds__(kK1Threads) void rqs_kernel_direct(
    const float* __restrict__ xin, const float* __restrict__ dx, const float* __restrict__ dy,
    const float* __restrict__ slope, float* __restrict__ out, float* __restrict__ log_det,
    int64_t M, int N, int R) {
  constexpr int Q = K / 4;
  __shared__ float s_ld[kK1Threads];
  const int64_t r0 = (int64_t)blockIdx.x * R;
  const int64_t left = M - r0;
  const int rows = (int)(left < R ? left : R);
  const int items = rows * N;
  const int tid = threadIdx.x;
  const int64_t item = r0 * N + min(tid, items - 1);  // clamped: loads stay unconditional
  const float4* rw = reinterpret_cast<const float4*>(dx + item * K);
  const float4* rh = reinterpret_cast<const float4*>(dy + item * K);
  float w[K], h[K];
#pragma unroll
  for (int c = 0; c < Q; ++c) {
    const float4 a = rw[c];
    const float4 b = rh[c];
    w[4 * c] = a.x; w[4 * c + 1] = a.y; w[4 * c + 2] = a.z; w[4 * c + 3] = a.w;
    h[4 * c] = b.x; h[4 * c + 1] = b.y; h[4 * c + 2] = b.z; h[4 * c + 3] = b.w;
  }
  const float v = xin[item];
  const float* slp = slope + item * (K - 1);
  RqsBin bn;
  if constexpr (SM == 0) {
    bn = rqs_bin_regs<FWD, K>(v, w, h, [&](int j) { return slp[j]; });
  } else {
    float sl[K - 1];
#pragma unroll
    for (int j = 0; j < K - 1; ++j) sl[j] = slp[j];
    bn = rqs_bin_regs_sl<FWD, K>(v, w, h, sl, [](float s) { return s; });
  }
  if (FWD) {
    float y, l;
    rqs_forward_eval(v, bn, y, l);
    if (tid < items && out) out[item] = y;
    if (log_det) {
      if (N <= 64 && (N & (N - 1)) == 0) {
        // a row's N items sit on N consecutive lanes of one wave: gather
        // them by lane shuffles and sum in dim order (utils.py:139), no LDS
        // round trip or block barrier
        const int lane = tid & 63, base = lane & ~(N - 1);
        float acc = 0.f;
        for (int n = 0; n < N; ++n) acc = acc + __shfl(l, base + n);
        if (lane == base && tid < items) log_det[r0 + tid / N] = acc;
      } else {
        if (tid < items) s_ld[tid] = l;
        __syncthreads();
        if (tid < rows) {
          float acc = 0.f;  // log_det.sum(axis=1), dim order
          for (int n = 0; n < N; ++n) acc = acc + s_ld[tid * N + n];
          log_det[r0 + tid] = acc;
        }
      }
    }
  } else if (tid < items) {
    out[item] = rqs_inverse_eval(v, bn);
  }
}

// Two lanes per (row, dim) item (K = 32): lane p of a pair loads knots
// 16p..16p+15 (the pair reads one contiguous 128-B row per array, half the
// registers of the one-lane form, so twice the waves stream), and sweeps
// them from the partner's prefix: lane 0 sums its 16 widths / heights in
// order and lane 1 continues the same sequential sums from there (the knots
// carry the one-lane form's bits).  The bin comes from lane 1 when any of its
// knots (16..32) is <= v, else from lane 0; non-monotone knots fall back to
// the generic search (rqs_bin).  Both lanes evaluate, lane 0 stores.
struct GlobalParams {
  const float* dx;
  const float* dy;
  const float* sl;
  __device__ float w(int j) const { return dx[j]; }
  __device__ float h(int j) const { return dy[j]; }
  __device__ float d(int j) const { return sl[j]; }
};

template <bool FWD, int K>
__global__ __launch_bounds__(kK1Threads) void rqs_kernel_pair(
    const float* __restrict__ xin, const float* __restrict__ dx, const float* __restrict__ dy,
    const float* __restrict__ slope, float* __restrict__ out, float* __restrict__ log_det,
    int64_t M, int N, int R) {
  constexpr int KH = K / 2, Q = KH / 4;
  __shared__ float s_ld[kK1Threads / 2];
  const int64_t r0 = (int64_t)blockIdx.x * R;
  const int64_t left = M - r0;
  const int rows = (int)(left < R ? left : R);
  const int items = rows * N;
  const int tid = threadIdx.x;
  const int it = tid >> 1, p = tid & 1;
  const int64_t item = r0 * N + min(it, items - 1);  // clamped: loads stay unconditional
  const float4* rw = reinterpret_cast<const float4*>(dx + item * K + KH * p);
  const float4* rh = reinterpret_cast<const float4*>(dy + item * K + KH * p);
  float w[KH], h[KH];
#pragma unroll
  for (int c = 0; c < Q; ++c) {
    const float4 a = rw[c];
    const float4 b = rh[c];
    w[4 * c] = a.x; w[4 * c + 1] = a.y; w[4 * c + 2] = a.z; w[4 * c + 3] = a.w;
    h[4 * c] = b.x; h[4 * c + 1] = b.y; h[4 * c + 2] = b.z; h[4 * c + 3] = b.w;
  }
  const float v = xin[item];
  // lane 0's knot 16 = its in-order sums; lane 1 starts from them
  float ex = 0.f, ey = 0.f;
#pragma unroll
  for (int j = 0; j < KH; ++j) { ex = ex + w[j]; ey = ey + h[j]; }
  const float px = __shfl_xor(ex, 1), py = __shfl_xor(ey, 1);
  float xk = p ? px : 0.f, yk = p ? py : 0.f;
  float sxk = 0.f, syk = 0.f, sw = w[0], sh = h[0];
  int cnt = 0, sel = 0;
#pragma unroll
  for (int j = 0; j < KH; ++j) {
    const float kk = FWD ? xk : yk;
    if (kk <= v) { ++cnt; sel = KH * p + j; sxk = xk; syk = yk; sw = w[j]; sh = h[j]; }
    xk = xk + w[j];
    yk = yk + h[j];
  }
  if (p) {  // the last knot (K)
    const float kk = FWD ? xk : yk;
    if (kk <= v) { ++cnt; sel = K; sxk = xk; syk = yk; sw = qnan(); sh = qnan(); }
  }
  // lane 1's data where it has a hit, else lane 0's
  const int ocnt = __shfl_xor(cnt, 1), osel = __shfl_xor(sel, 1);
  const float oxk = __shfl_xor(sxk, 1), oyk = __shfl_xor(syk, 1), ow = __shfl_xor(sw, 1), oh = __shfl_xor(sh, 1);
  const int c1 = p ? cnt : ocnt;
  const bool own = p ? (c1 > 0) : (c1 == 0);
  RqsBin b;
  const int bsel = own ? sel : osel;
  b.xk = own ? sxk : oxk;
  b.yk = own ? syk : oyk;
  b.w = own ? sw : ow;
  b.h = own ? sh : oh;
  const int tot = cnt + ocnt;
  int idx = tot - 1;
  idx = idx < 0 ? 0 : (idx > K ? K : idx);
  const float* slp = slope + item * (K - 1);
  if (idx != bsel) {  // non-monotone knots (never from normalize_spline_params)
    b = rqs_bin<FWD>(v, K, GlobalParams{dx + item * K, dy + item * K, slp});
  } else {
    b.dk = (bsel == 0 || bsel == K) ? 1.0f : slp[bsel - 1];
    b.dkp1 = (bsel + 1 < K) ? slp[bsel] : (bsel + 1 == K ? 1.0f : qnan());
    b.sk = b.h / b.w;
    b.oob = (v < 0.f) || (v >= 1.f);
  }
  if (FWD) {
    float y, l;
    rqs_forward_eval(v, b, y, l);
    if (p == 0 && it < items && out) out[item] = y;
    if (log_det) {
      if (N <= 32 && (N & (N - 1)) == 0) {
        // a row's N items sit on 2N consecutive lanes: sum in dim order
        const int lane = tid & 63, base = lane & ~(2 * N - 1);
        float acc = 0.f;
        for (int n = 0; n < N; ++n) acc = acc + __shfl(l, base + 2 * n);
        if (lane == base && it < items) log_det[r0 + it / N] = acc;
      } else {
        if (p == 0 && it < items) s_ld[it] = l;
        __syncthreads();
        if (tid < rows) {
          float acc = 0.f;  // log_det.sum(axis=1), dim order
          for (int n = 0; n < N; ++n) acc = acc + s_ld[tid * N + n];
          log_det[r0 + tid] = acc;
        }
      }
    }
  } else if (p == 0 && it < items) {
    out[item] = rqs_inverse_eval(v, b);
  }
}

// Row-wise utils kernels (thresholded softmax, normalize_spline_params):
// one thread per row, but the block's rows (contiguous in HBM) are staged
// through LDS with coalesced loads and stores (odd row stride) — a thread
// walking its own row in global memory would touch a new cache line per
// element and re-read each row once per pass.
constexpr int kRowThreads = 256;
constexpr int kRowLdsFloats = 12288;  // 48 KiB budget per block (dynamic, sized to the rows)

__host__ __device__ inline int row_stride(int K) { return K | 1; }
inline int rows_per_block(int K) {
  const int r = kRowLdsFloats / row_stride(K);
  return r < kRowThreads ? r : kRowThreads;
}

__device__ __forceinline__ void rows_in(float* lds, const float* __restrict__ src, int rows, int K) {
  const int ks = row_stride(K), n = rows * K;
  for (int e = threadIdx.x; e < n; e += kRowThreads) {
    const int r = e / K;
    lds[r * ks + (e - r * K)] = src[e];
  }
}

__device__ __forceinline__ void rows_out(float* __restrict__ dst, const float* lds, int rows, int K) {
  const int ks = row_stride(K), n = rows * K;
  for (int e = threadIdx.x; e < n; e += kRowThreads) {
    const int r = e / K;
    dst[e] = lds[r * ks + (e - r * K)];
  }
}

// (squareplus(v) / sum + c) / norm over a row in LDS (utils.py:23-34).
__device__ __forceinline__ void softmax_row(float* r, int K, float c, float norm) {
  float xs = 0.f;
  for (int j = 0; j < K; ++j) {
    const float v = squareplus(r[j]);
    r[j] = v;
    xs = xs + v;
  }
  for (int j = 0; j < K; ++j) r[j] = (r[j] / xs + c) / norm;
}

// utils.py:37-62: dx, dy rows through softmax_with_threshold, slopes through
// squareplus (elementwise over the block's contiguous slope rows).
__global__ __launch_bounds__(kRowThreads) void normalize_kernel(float* __restrict__ dx, float* __restrict__ dy,
                                                                float* __restrict__ sl, int64_t M, int K, int R) {
  extern __shared__ float lds[];  // [2][R][row_stride(K)]: dx and dy rows together
  const int64_t r0 = (int64_t)blockIdx.x * R;
  const int rows = (int)(M - r0 < R ? M - r0 : R);
  const double c64 = 1e-5 / (1.0 - (double)K * 1e-5);  // Python floats (utils.py:32)
  const float c = (float)c64;
  const float norm = (float)(1.0 + c64 * (double)K);
  float* ly = lds + R * row_stride(K);
  rows_in(lds, dx + r0 * K, rows, K);
  rows_in(ly, dy + r0 * K, rows, K);
  __syncthreads();
  if ((int)threadIdx.x < rows) {
    softmax_row(lds + threadIdx.x * row_stride(K), K, c, norm);
    softmax_row(ly + threadIdx.x * row_stride(K), K, c, norm);
  }
  __syncthreads();
  rows_out(dx + r0 * K, lds, rows, K);
  rows_out(dy + r0 * K, ly, rows, K);
  if (K > 1) {
    float* s = sl + r0 * (K - 1);
    const int n = rows * (K - 1);
    for (int e = threadIdx.x; e < n; e += kRowThreads) s[e] = squareplus(s[e]);
  }
}

// normalize_spline_params fast path (K in {4, 8, 16, 32}, 16-B aligned
// arrays): a pure stream, so every lane moves float4s (1 KiB per
// wave-instruction, four in flight per lane) and the row of K knots lives on
// G = K/4 consecutive lanes: lane partial sums (sequential over its four)
// combined by xor-shuffles.  Quotients by a reciprocal and one fma
// correction (the correctly rounded quotient but for ties at the last
// bit; the sum order already makes the result differ from the reference's
// sequential sum by an ulp).  Blocks [0, B) stream dx, [B, 2B) dy, the rest
// the slope logits through squareplus.
constexpr int kNormU = 4;  // float4s per lane
typedef float nf4 __attribute__((ext_vector_type(4)));

// squareplus with a Newton-corrected hardware rsqrt (x^2 + 4 >= 4: no
// denormal scaling, unlike sqrtf's expansion): ~0.5 ulp.
__device__ __forceinline__ float squareplus_stream(float x) {
  const float a = x * x + 4.0f;
  const float r = __builtin_amdgcn_rsqf(a);
  const float sq = a * r;
  return 0.5f * (x + __builtin_fmaf(__builtin_fmaf(-sq, sq, a), 0.5f * r, sq));
}

__device__ __forceinline__ float div_corr(float a, float b, float rb) {
  const float q = a * rb;
  return __builtin_fmaf(__builtin_fmaf(-q, b, a), rb, q);
}

template <int K>
__global__ __launch_bounds__(256) void normalize_vec_kernel(float* __restrict__ dx, float* __restrict__ dy,
                                                            float* __restrict__ sl, int64_t n4, int64_t nsl,
                                                            int64_t bxy, float c, float norm, float rnorm) {
  constexpr int G = K / 4;
  const int64_t b = blockIdx.x;
  if (b < 2 * bxy) {
    nf4* p = reinterpret_cast<nf4*>(b < bxy ? dx : dy);
    const int64_t i0 = (b < bxy ? b : b - bxy) * (256 * kNormU) + threadIdx.x;
    nf4 v[kNormU];
#pragma unroll
    for (int u = 0; u < kNormU; ++u) {
      const int64_t i = i0 + u * 256;
      v[u] = i < n4 ? __builtin_nontemporal_load(p + i) : nf4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < kNormU; ++u) {
      nf4 w = v[u];
      w.x = squareplus_stream(w.x); w.y = squareplus_stream(w.y); w.z = squareplus_stream(w.z); w.w = squareplus_stream(w.w);
      float sum = ((w.x + w.y) + w.z) + w.w;  // utils.py:32 (jnp.sum over the row)
#pragma unroll
      for (int m = 1; m < G; m <<= 1) sum += __shfl_xor(sum, m);
      const float rs = 1.0f / sum;
      w.x = div_corr(div_corr(w.x, sum, rs) + c, norm, rnorm);  // utils.py:33
      w.y = div_corr(div_corr(w.y, sum, rs) + c, norm, rnorm);
      w.z = div_corr(div_corr(w.z, sum, rs) + c, norm, rnorm);
      w.w = div_corr(div_corr(w.w, sum, rs) + c, norm, rnorm);
      const int64_t i = i0 + u * 256;
      if (i < n4) __builtin_nontemporal_store(w, p + i);
    }
  } else {
    nf4* p = reinterpret_cast<nf4*>(sl);
    const int64_t n = nsl >> 2;
    const int64_t i0 = (b - 2 * bxy) * (256 * kNormU) + threadIdx.x;
    nf4 v[kNormU];
#pragma unroll
    for (int u = 0; u < kNormU; ++u) {
      const int64_t i = i0 + u * 256;
      v[u] = i < n ? __builtin_nontemporal_load(p + i) : nf4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < kNormU; ++u) {
      const int64_t i = i0 + u * 256;
      nf4 w = v[u];
      w.x = squareplus_stream(w.x); w.y = squareplus_stream(w.y); w.z = squareplus_stream(w.z); w.w = squareplus_stream(w.w);
      if (i < n) __builtin_nontemporal_store(w, p + i);
    }
    if (i0 == 0)  // the < 4 trailing slope logits
      for (int64_t e = n * 4; e < nsl; ++e) sl[e] = squareplus(sl[e]);
  }
}

// utils.py:18-20 elementwise; b is the reference's `b` argument.
__global__ void squareplus_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n,
                                  float b) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { const float v = x[i]; y[i] = 0.5f * (v + __builtin_sqrtf(v * v + b)); }
}

// utils.py:23-34 over rows of K; c and 1 + c*n are float64 Python scalars.
__global__ __launch_bounds__(kRowThreads) void softmax_threshold_kernel(const float* __restrict__ x,
                                                                        float* __restrict__ y, int64_t M, int K,
                                                                        int R, float c, float norm) {
  extern __shared__ float lds[];  // [R][row_stride(K)]
  const int64_t r0 = (int64_t)blockIdx.x * R;
  const int rows = (int)(M - r0 < R ? M - r0 : R);
  rows_in(lds, x + r0 * K, rows, K);
  __syncthreads();
  if ((int)threadIdx.x < rows) softmax_row(lds + threadIdx.x * row_stride(K), K, c, norm);
  __syncthreads();
  rows_out(y + r0 * K, lds, rows, K);
}

template <bool FWD>
int launch_rqs(const float* x, const float* dx, const float* dy, const float* slope, float* out,
               float* log_det, int64_t M, int N, int K, void* stream) {
  if (M < 0 || N <= 0 || K < 1 || K > 256) return einval("bad shape M=%lld N=%d K=%d", (long long)M, N, K);
  if (M == 0) return ZF_OK;
  if (!x || !dx || !dy || (K > 1 && !slope)) return einval("NULL input");
  if (!FWD && !out) return einval("NULL output");
  hipStream_t st = (hipStream_t)stream;
  const bool aligned = ((reinterpret_cast<uintptr_t>(dx) | reinterpret_cast<uintptr_t>(dy)) & 15) == 0;
  if (aligned && K == 32 && N <= kK1Threads / 2 && std::getenv("ZF_K1_ONE_LANE") == nullptr) {
    const int R = (kK1Threads / 2) / N;
    const int64_t grid = (M + R - 1) / R;
    if (grid > 0x7fffffffLL) return einval("M too large");
    hipLaunchKernelGGL((rqs_kernel_pair<FWD, 32>), dim3((unsigned)grid), dim3(kK1Threads), 0, st, x, dx, dy, slope,
                       out, log_det, M, N, R);
    ZF_CHECK_LAUNCH("rqs_kernel_pair");
    return ZF_OK;
  }
  if (aligned && (K == 4 || K == 8 || K == 16 || K == 32) && N <= kK1Threads) {
    const int R = kK1Threads / N;
    const int64_t grid = (M + R - 1) / R;
    if (grid > 0x7fffffffLL) return einval("M too large");
#define ZF_RQSD(KV)                                                                                   \
  hipLaunchKernelGGL((rqs_kernel_direct<FWD, KV, KV == 16>), dim3((unsigned)grid), dim3(kK1Threads), 0, \
                     st, x, dx, dy, slope, out, log_det, M, N, R)
    switch (K) {
      case 4: ZF_RQSD(4); break;
      case 8: ZF_RQSD(8); break;
      case 16: ZF_RQSD(16); break;
      default: ZF_RQSD(32); break;
    }
#undef ZF_RQSD
    ZF_CHECK_LAUNCH("rqs_kernel_direct");
    return ZF_OK;
  }
  const int ks = (K % 2 == 0) ? K + 1 : K + 2;
  const int per_item = 3 * ks + 1;
  int R = kK1LdsBudgetFloats / (per_item * N);
  if (R > kK1Threads / N) R = kK1Threads / N;
  if (R < 1) return enotsup("N*(3K+4) too large for one block (N > 256 or K too large)");
  const size_t lds = sizeof(float) * (size_t)R * N * per_item;
  const int64_t grid = (M + R - 1) / R;
  if (grid > 0x7fffffffLL) return einval("M too large");
#define ZF_RQS(KV)                                                                              \
  hipLaunchKernelGGL((rqs_kernel<FWD, KV>), dim3((unsigned)grid), dim3(kK1Threads), lds, st, x, \
                     dx, dy, slope, out, log_det, M, N, K, R)
  switch (K) {
    case 4: ZF_RQS(4); break;
    case 8: ZF_RQS(8); break;
    case 16: ZF_RQS(16); break;
    case 32: ZF_RQS(32); break;
    default: ZF_RQS(0); break;
  }
#undef ZF_RQS
  ZF_CHECK_LAUNCH("rqs_kernel");
  return ZF_OK;
}

}  // namespace
}  // namespace zf

extern "C" {

int zf_rqs_forward(const float* x, const float* dx, const float* dy, const float* slope,
                   float* y, float* log_det, int64_t M, int N, int K, void* stream) {
  return zf::launch_rqs<true>(x, dx, dy, slope, y, log_det, M, N, K, stream);
}

int zf_rqs_inverse(const float* y, const float* dx, const float* dy, const float* slope,
                   float* x, int64_t M, int N, int K, void* stream) {
  return zf::launch_rqs<false>(y, dx, dy, slope, x, nullptr, M, N, K, stream);
}

int zf_squareplus(const float* x, float* y, int64_t n, float b, void* stream) {
  if (n < 0) return zf::einval("n < 0");
  if (n == 0) return ZF_OK;
  if (!x || !y) return zf::einval("NULL argument");
  const int64_t grid = (n + 255) / 256;
  hipLaunchKernelGGL(zf::squareplus_kernel, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream,
                     x, y, n, b);
  ZF_CHECK_LAUNCH("squareplus_kernel");
  return ZF_OK;
}

int zf_softmax_with_threshold(const float* x, float* y, int64_t M, int K, double threshold,
                              void* stream) {
  if (M < 0 || K < 1) return zf::einval("bad shape");
  if (M == 0) return ZF_OK;
  if (!x || !y) return zf::einval("NULL argument");
  if (K > zf::kRowLdsFloats / 2) return zf::einval("K too large");
  const double c64 = threshold / (1.0 - (double)K * threshold);
  const int R = zf::rows_per_block(K);
  const int64_t grid = (M + R - 1) / R;
  if (grid > 0x7fffffffLL) return zf::einval("M too large");
  hipLaunchKernelGGL(zf::softmax_threshold_kernel, dim3((unsigned)grid), dim3(zf::kRowThreads),
                     (size_t)R * zf::row_stride(K) * sizeof(float),
                     (hipStream_t)stream, x, y, M, K, R, (float)c64, (float)(1.0 + c64 * (double)K));
  ZF_CHECK_LAUNCH("softmax_threshold_kernel");
  return ZF_OK;
}

int zf_normalize_spline_params(float* dx, float* dy, float* slope, int64_t M, int K,
                               void* stream) {
  if (M < 0 || K < 1) return zf::einval("bad shape");
  if (M == 0) return ZF_OK;
  if (!dx || !dy || (K > 1 && !slope)) return zf::einval("NULL input");
  if (K > zf::kRowLdsFloats / 2) return zf::einval("K too large");
  const bool aligned = ((reinterpret_cast<uintptr_t>(dx) | reinterpret_cast<uintptr_t>(dy) |
                         reinterpret_cast<uintptr_t>(slope)) & 15) == 0;
  if (aligned && (K == 4 || K == 8 || K == 16 || K == 32) && std::getenv("ZF_NORM_ROWS") == nullptr) {
    const double c64 = 1e-5 / (1.0 - (double)K * 1e-5);  // utils.py:32 (Python floats)
    const float norm = (float)(1.0 + c64 * (double)K);
    const int64_t n4 = M * K / 4, nsl = M * (K - 1);
    const int64_t per = 256 * zf::kNormU;
    const int64_t bxy = (n4 + per - 1) / per;
    int64_t bs = (nsl / 4 + per - 1) / per;
    if (bs == 0 && nsl > 0) bs = 1;  // tail-only slopes
    const int64_t grid = 2 * bxy + bs;
    if (grid > 0x7fffffffLL) return zf::einval("M too large");
#define ZF_NORMV(KV)                                                                                          \
  hipLaunchKernelGGL(zf::normalize_vec_kernel<KV>, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, dx, \
                     dy, slope, n4, nsl, bxy, (float)c64, norm, (float)(1.0 / (double)norm))
    switch (K) {
      case 4: ZF_NORMV(4); break;
      case 8: ZF_NORMV(8); break;
      case 16: ZF_NORMV(16); break;
      default: ZF_NORMV(32); break;
    }
#undef ZF_NORMV
    ZF_CHECK_LAUNCH("normalize_vec_kernel");
    return ZF_OK;
  }
  const int R = zf::rows_per_block(2 * K + 1);  // dx and dy rows share the LDS budget
  const int64_t grid = (M + R - 1) / R;
  if (grid > 0x7fffffffLL) return zf::einval("M too large");
  hipLaunchKernelGGL(zf::normalize_kernel, dim3((unsigned)grid), dim3(zf::kRowThreads),
                     (size_t)2 * R * zf::row_stride(K) * sizeof(float),
                     (hipStream_t)stream, dx, dy, slope, M, K, R);
  ZF_CHECK_LAUNCH("normalize_kernel");
  return ZF_OK;
}

}  // extern "C"
