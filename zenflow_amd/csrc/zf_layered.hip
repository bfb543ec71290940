// Layered eval path: Chain.__call__ / Chain.inverse / Flow.log_prob /
// Flow.sample (bijectors.py:103-116, flow.py:22-78) for flows whose
// conditioner the fused kernels cannot hold in registers and LDS — a hidden
// width above 256 (layer_utils.rect/tri build any width,
// layer_utils.py:6-18; NeuralSplineCoupling.layers, bijectors.py:318).
//
// Op by op over chunks of rows, every intermediate in HBM:
//   ShiftBounds        lay_sb_kernel       (zf_flow_dev.h sb_*_elem, the fused kernels' math)
//   NSC conditioner    lay_bn_kernel       hstack(xc, c) -> BatchNorm (eval: running stats)
//                      dense_gemm          Dense_l + activation: the trainer's GEMMs
//                                          (bf16x3 split MFMA at >= 512 128x128 tiles, else fp32 MFMA)
//                      dense_gemm          last Dense -> raw spline parameters P [rows][dt][3K-1]
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
#include <mutex>
#include <vector>

namespace zf {

struct LayeredFlow {
  zf_flow_desc desc;     // with zf_flow_plan's natural offsets
  float* d_nat = nullptr;  // natural blob (FLAX layouts: Dense kernels [in][out])
  long long rows = 0;    // workspace capacity (rows)
  float *s0 = nullptr, *s1 = nullptr, *ld = nullptr, *U = nullptr, *Z = nullptr, *H0 = nullptr, *H1 = nullptr,
        *P = nullptr;
  void* block = nullptr;  // one allocation holding the buffers above
  int hmax = 1, dcmax = 1, outmax = 1;
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

inline unsigned nblocks(long long n, int t) { return (unsigned)((n + t - 1) / t); }

int ensure_rows(LayeredFlow* L, long long rows) {
  if (rows <= L->rows) return ZF_OK;
  if (L->block) (void)hipFree(L->block);
  L->block = nullptr;
  L->rows = 0;
  const int D = L->desc.dim;
  const long long per = 2ll * D + 1 + L->dcmax + 3ll * L->hmax + L->outmax;  // floats per row
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
      for (int l = 0; l <= op.n_hidden; ++l) {
        const bool last = l == op.n_hidden;
        const int out_w = last ? d.dt * d.S : op.hidden[l];
        float* H = (l & 1) ? L->H1 : L->H0;
        // hidden layers keep only the activation H (no pre-activation store: eval has no backward)
        rc = dense_gemm(n, n, out_w, in_w, in, in_w, L->d_nat + op.off_w[l], out_w, last ? L->P : nullptr, out_w,
                        last ? nullptr : H, st, L->d_nat + op.off_b[l], op.act);
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
