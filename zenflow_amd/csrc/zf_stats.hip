// Train-mode batch statistics: per-column min / max (fp32) and sum / sum of
// squares (fp64) over the batch axis.  Used for ShiftBounds' batch min/max
// (bijectors.py:250-257, with the safe_log pre-transform of one-sided bounds,
// :193-202) and flax BatchNorm's batch mean / variance (bijectors.py:342 with
// use_running_average=False).  Two deterministic passes: per-block partials,
// then a fixed-order combine.
#include "zf_internal.h"

#include <cfloat>
#include <cmath>

namespace zf {
namespace {

constexpr int kStatThreads = 256;
constexpr int kStatMaxCols = 64;

struct ColPre {
  int mode[kStatMaxCols];  // ZF_SB_LOWER / ZF_SB_UPPER apply safe_log, else identity
  float a[kStatMaxCols];
};

__device__ __forceinline__ float pre_transform(float v, int mode, float a) {
  if (mode == ZF_SB_LOWER) return logf((v - a) + 1.17549435e-38f);
  if (mode == ZF_SB_UPPER) return logf((a - v) + 1.17549435e-38f);
  return v;
}

// Block b reduces rows [b*rows_per_block, ...) for every column; thread t
// handles column t % ncols, rows t / ncols + k * (256 / ncols).
__global__ __launch_bounds__(kStatThreads) void colstats_partial(
    const float* __restrict__ x, long long N, int ncols, long long ld, int col_offset, ColPre pre,
    long long rows_per_block, float* __restrict__ pmin, float* __restrict__ pmax,
    double* __restrict__ psum, double* __restrict__ psq) {
  __shared__ float smin[kStatThreads], smax[kStatThreads];
  __shared__ double ssum[kStatThreads], ssq[kStatThreads];
  const int t = threadIdx.x;
  const int lanes_per_col = kStatThreads / ncols;
  const int col = t % ncols;
  const int sub = t / ncols;
  float mn = INFINITY, mx = -INFINITY;
  double sm = 0.0, sq = 0.0;
  if (sub < lanes_per_col) {
    const long long r0 = (long long)blockIdx.x * rows_per_block;
    long long r1 = r0 + rows_per_block;
    if (r1 > N) r1 = N;
    const int mode = pre.mode[col];
    const float a = pre.a[col];
    auto acc = [&](float raw) {
      const float v = pre_transform(raw, mode, a);
      // jnp.min/max propagate NaN
      if (v != v) { mn = v; mx = v; }
      else if (mn == mn) { mn = fminf(mn, v); mx = fmaxf(mx, v); }
      sm += (double)v;
      sq += (double)v * (double)v;
    };
    // kU rows' loads in flight ahead of the in-order accumulation (a small
    // batch is one block: every serial round trip would be exposed)
    constexpr int kU = 8;
    long long r = r0 + sub;
    for (; r + (kU - 1) * (long long)lanes_per_col < r1; r += kU * (long long)lanes_per_col) {
      float vv[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) vv[u] = x[(r + u * (long long)lanes_per_col) * ld + col_offset + col];
#pragma unroll
      for (int u = 0; u < kU; ++u) acc(vv[u]);
    }
    for (; r < r1; r += lanes_per_col) acc(x[r * ld + col_offset + col]);
  }
  smin[t] = mn; smax[t] = mx; ssum[t] = sm; ssq[t] = sq;
  __syncthreads();
  if (t < ncols) {
    float m0 = INFINITY, m1 = -INFINITY;
    double a0 = 0.0, a1 = 0.0;
    auto comb = [&](float lo, float hi, double s1, double s2) {
      if (lo != lo || m0 != m0) { m0 = m0 != m0 ? m0 : lo; m1 = m0; }
      else { m0 = fminf(m0, lo); m1 = fmaxf(m1, hi); }
      a0 += s1;
      a1 += s2;
    };
    int k = 0;
    for (; k + 8 <= lanes_per_col; k += 8) {  // eight entries' LDS reads ahead of the in-order combine
      float lo[8], hi[8];
      double s1[8], s2[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = (k + u) * ncols + t;
        lo[u] = smin[i]; hi[u] = smax[i]; s1[u] = ssum[i]; s2[u] = ssq[i];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) comb(lo[u], hi[u], s1[u], s2[u]);
    }
    for (; k < lanes_per_col; ++k) {
      const int i = k * ncols + t;
      comb(smin[i], smax[i], ssum[i], ssq[i]);
    }
    const size_t o = (size_t)blockIdx.x * ncols + t;
    pmin[o] = m0; pmax[o] = m1; psum[o] = a0; psq[o] = a1;
  }
}

__global__ void colstats_final(const float* __restrict__ pmin, const float* __restrict__ pmax,
                               const double* __restrict__ psum, const double* __restrict__ psq,
                               int nblocks, int ncols, float* cmin, float* cmax, double* csum,
                               double* csq) {
  const int c = threadIdx.x;
  if (c >= ncols) return;
  float m0 = INFINITY, m1 = -INFINITY;
  double a0 = 0.0, a1 = 0.0;
  for (int b = 0; b < nblocks; ++b) {
    const size_t i = (size_t)b * ncols + c;
    if (pmin[i] != pmin[i] || m0 != m0) { m0 = m0 != m0 ? m0 : pmin[i]; m1 = m0; }
    else { m0 = fminf(m0, pmin[i]); m1 = fmaxf(m1, pmax[i]); }
    a0 += psum[i];
    a1 += psq[i];
  }
  if (cmin) cmin[c] = m0;
  if (cmax) cmax[c] = m1;
  if (csum) csum[c] = a0;
  if (csq) csq[c] = a1;
}

int stat_blocks(int64_t N) {
  int64_t b = (N + 4095) / 4096;
  if (b < 1) b = 1;
  if (b > 2048) b = 2048;
  return (int)b;
}

}  // namespace
}  // namespace zf

extern "C" {

int64_t zf_colstats_workspace_bytes(int64_t N, int ncols) {
  const int64_t nb = zf::stat_blocks(N);
  return nb * ncols * (4 + 4 + 8 + 8) + 256;
}

int zf_colstats(const float* x, int64_t N, int ncols, int64_t ld, int col_offset,
                const float* pre_modes, const float* pre_params, float* cmin, float* cmax,
                double* csum, double* csumsq, void* workspace, void* stream) {
  if (ncols < 1 || ncols > zf::kStatMaxCols) return zf::einval("ncols must be in [1, 64]");
  if (N < 0 || ld < ncols + col_offset || col_offset < 0) return zf::einval("bad shape");
  if (!workspace) return zf::einval("workspace is NULL");
  if (N > 0 && !x) return zf::einval("x is NULL");
  zf::ColPre pre;
  for (int c = 0; c < zf::kStatMaxCols; ++c) {
    pre.mode[c] = (pre_modes && c < ncols) ? (int)pre_modes[c] : ZF_SB_NONE;
    pre.a[c] = (pre_params && c < ncols) ? pre_params[c] : 0.f;
  }
  const int nb = zf::stat_blocks(N);
  const long long rpb = N > 0 ? (N + nb - 1) / nb : 1;
  char* ws = (char*)workspace;
  float* pmin = (float*)ws;
  float* pmax = pmin + (size_t)nb * ncols;
  double* psum = (double*)(((uintptr_t)(pmax + (size_t)nb * ncols) + 7) & ~(uintptr_t)7);
  double* psq = psum + (size_t)nb * ncols;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(zf::colstats_partial, dim3(nb), dim3(zf::kStatThreads), 0, st, x,
                     (long long)N, ncols, (long long)ld, col_offset, pre, rpb, pmin, pmax, psum, psq);
  ZF_CHECK_LAUNCH("colstats_partial");
  hipLaunchKernelGGL(zf::colstats_final, dim3(1), dim3(64), 0, st, pmin, pmax, psum, psq, nb, ncols,
                     cmin, cmax, csum, csumsq);
  ZF_CHECK_LAUNCH("colstats_final");
  return ZF_OK;
}

}  // extern "C"
