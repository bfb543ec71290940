// Timing probe for the trainer's large-batch forward GEMMs (zf_train.hip):
// gemm_x3_kernel (bf16x3 split MFMA) vs mgemm_kernel<128> (fp32 MFMA), with
// and without the bias + activation epilogue, at the cfg5 x 65536 shapes.
// Built against the trainer source itself (included) and the library:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I zenflow_amd/csrc \
//     tests/hip/gemm_probe.hip -Lzenflow_amd -lzenflow_amd -o build/gemm_probe
#include "../../zenflow_amd/csrc/zf_train.hip"

#include <algorithm>
#include <type_traits>
#include <cmath>
#include <cstdio>
#include <vector>

namespace {

__global__ void fill_kernel(float* p, long long n, unsigned seed) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    p[i] = ((h & 0xffffff) / 16777216.0f - 0.5f) * 0.2f;
  }
}

__global__ void write_kernel(float* __restrict__ C, float* __restrict__ H, long long n) {
  const long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i < n) {
    *reinterpret_cast<float4*>(C + i) = float4{1.f, 2.f, 3.f, 4.f};
    if (H) *reinterpret_cast<float4*>(H + i) = float4{1.f, 2.f, 3.f, 4.f};
  }
}

template <class F>
float time_it(F f, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) f();
  (void)hipEventRecord(a, 0);
  for (int i = 0; i < reps; ++i) f();
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms * 1e3f / reps;
}

__device__ __forceinline__ float fast_swish(float v) {
  return v * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * v));
}
// the fused store of four consecutive columns (n % 4 == 0, N % 4 == 0)
template <bool FAST = false>
__device__ __forceinline__ void gemm_epilogue4(float4 v, int n, long long o, float* __restrict__ C, int epi,
                                               const float* __restrict__ bias, float* __restrict__ H,
                                               const float* __restrict__ Z, int act) {
  using namespace zf;
  float x[4] = {v.x, v.y, v.z, v.w};
  if (epi == kEpiBias) {
    const float4 b = *reinterpret_cast<const float4*>(bias + n);
    x[0] += b.x; x[1] += b.y; x[2] += b.z; x[3] += b.w;
    if (H) {
      float y[4];
#pragma unroll
      for (int t = 0; t < 4; ++t)
        y[t] = act == ZF_ACT_SWISH ? (FAST ? fast_swish(x[t]) : x[t] * sigmoidf(x[t])) : act_other(act, x[t]);
      *reinterpret_cast<float4*>(H + o) = float4{y[0], y[1], y[2], y[3]};
    }
  } else if (epi == kEpiDSwish) {
    const float4 z4 = *reinterpret_cast<const float4*>(Z + o);
    const float z[4] = {z4.x, z4.y, z4.z, z4.w};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (act == ZF_ACT_SWISH) {
        const float sg = FAST ? __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * z[t]))
                              : sigmoidf(z[t]);
        x[t] = x[t] * (sg + z[t] * sg * (1.0f - sg));
      } else {
        x[t] = x[t] * act_other_grad(act, z[t]);
      }
    }
  }
  *reinterpret_cast<float4*>(C + o) = float4{x[0], x[1], x[2], x[3]};
}

// Experimental variants of gemm_x3_kernel (this probe only): STAGES k-tiles
// of global loads in flight in registers; ABL ablations (results wrong by
// construction): 1 = no epilogue stores, 2 = no global loads after the
// first k-tile, 4 = no MFMA.
template <bool TB, int STAGES, int ABL, bool WIDE = false, bool FAST = false>
__global__ __launch_bounds__(256) void x3v(int M, int N, int K, const float* __restrict__ A, int lda,
                                           const float* __restrict__ B, int ldb, float* __restrict__ C, int ldc,
                                           int epi, const float* __restrict__ bias, float* __restrict__ H,
                                           const float* __restrict__ Z, int act) {
  using namespace zf;
  __shared__ __attribute__((aligned(16))) __bf16 lds[6 * kX3Plane];
  __bf16* const Ap = lds;
  __bf16* const Bp = lds + 3 * kX3Plane;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm0 = (wave >> 1) * 64, wn0 = (wave & 1) * 64;
  const int m0 = blockIdx.y * kX3BM, n0 = blockIdx.x * kX3BN;
  const int r = lane & 31, h = lane >> 5;
  float4 ra[STAGES][4], rb[STAGES][4];
  float rbs[STAGES][16];
  auto load_rows = [&](const float* P, int ld, int r0, int R, int k0, float4 (&v)[4]) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + 256 * i, row = r0 + (e >> 2);
      const float* src = P + (long long)row * ld + k0 + 8 * (e & 3);
      v[2 * i] = row < R ? *reinterpret_cast<const float4*>(src) : float4{0.f, 0.f, 0.f, 0.f};
      v[2 * i + 1] = row < R ? *reinterpret_cast<const float4*>(src + 4) : float4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto store_rows = [&](__bf16* P, const float4 (&v)[4]) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + 256 * i;
      const float x[8] = {v[2 * i].x, v[2 * i].y, v[2 * i].z, v[2 * i].w,
                          v[2 * i + 1].x, v[2 * i + 1].y, v[2 * i + 1].z, v[2 * i + 1].w};
      split3_store(x, P + (e >> 2) * kX3RS + 8 * (e & 3));
    }
  };
  auto load_cols = [&](int k0, float (&v)[16]) {
    const int n = n0 + (tid & 127);
    const float* src = B + (long long)(k0 + 16 * (tid >> 7)) * ldb + n;
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = n < N ? src[(long long)j * ldb] : 0.f;
  };
  auto store_cols = [&](const float (&v)[16]) {
    __bf16* P = Bp + (tid & 127) * kX3RS + 16 * (tid >> 7);
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const float x[8] = {v[8 * g], v[8 * g + 1], v[8 * g + 2], v[8 * g + 3],
                          v[8 * g + 4], v[8 * g + 5], v[8 * g + 6], v[8 * g + 7]};
      split3_store(x, P + 8 * g);
    }
  };
  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = floatx16{0};
  auto load = [&](int k0, auto bc) {
    constexpr int b = decltype(bc)::value;
    load_rows(A, lda, m0, M, k0, ra[b]);
    if (TB) load_rows(B, ldb, n0, N, k0, rb[b]);
    else load_cols(k0, rbs[b]);
  };
  auto iter = [&](int k0, auto bc) {
    constexpr int b = decltype(bc)::value;
    store_rows(Ap, ra[b]);
    if (TB) store_rows(Bp, rb[b]);
    else store_cols(rbs[b]);
    __syncthreads();
    if (!(ABL & 2) && k0 + STAGES * kX3BK < K) load(k0 + STAGES * kX3BK, bc);
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
          if (ABL & 4) {
            acc[i][j][0] += (float)af[i][0][0] + (float)bf[j][0][1] + (float)af[i][1][2] + (float)bf[j][1][3] +
                            (float)af[i][2][4] + (float)bf[j][2][5];
          } else {
            floatx16 c = acc[i][j];
            if (WIDE) {  // D[n][m]: lane = row m, registers = 4 consecutive columns per group
              c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf[j][1], af[i][1], c, 0, 0, 0);
              c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf[j][2], af[i][0], c, 0, 0, 0);
              c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf[j][0], af[i][2], c, 0, 0, 0);
              c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf[j][1], af[i][0], c, 0, 0, 0);
              c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf[j][0], af[i][1], c, 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf[j][0], af[i][0], c, 0, 0, 0);
            } else {
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][1], bf[j][1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][0], bf[j][2], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][2], bf[j][0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][0], bf[j][1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][1], bf[j][0], c, 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][0], bf[j][0], c, 0, 0, 0);
            }
          }
        }
    }
    __syncthreads();
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, STAGES - 1>;
  load(0, I0{});
  if (STAGES == 2 && kX3BK < K) load(kX3BK, I1{});
  for (int k0 = 0; k0 < K; k0 += STAGES * kX3BK) {
    iter(k0, I0{});
    if (STAGES == 2 && k0 + kX3BK < K) iter(k0 + kX3BK, I1{});
  }
  if (WIDE) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int m = m0 + wm0 + 32 * i + r, n = n0 + wn0 + 32 * j + 8 * g + 4 * h;
          float4 v = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
          if ((ABL & 1) && v.x != 12345.678f) continue;
          if (m < M && n < N) gemm_epilogue4<FAST>(v, n, (long long)m * ldc + n, C, epi, bias, H, Z, act);
        }
    return;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int m = m0 + wm0 + 32 * i + (q & 3) + 8 * (q >> 2) + 4 * h, n = n0 + wn0 + 32 * j + r;
        if ((ABL & 1) && acc[i][j][q] != 12345.678f) continue;
        if (m < M && n < N) gemm_epilogue(acc[i][j][q], n, (long long)m * ldc + n, C, epi, bias, H, Z, act);
      }
}

// the shipped kernel's persistent grid: min(tiles, 2 blocks per CU)
inline dim3 x3grid(dim3 g) { return dim3(std::min(g.x * g.y, 512u)); }

}  // namespace

int main() {
  const int M = 65536, K = 256;
  const int Ns[2] = {256, 760};
  float *A, *B, *C, *H, *bias;
  (void)hipMalloc(&A, sizeof(float) * M * K);
  (void)hipMalloc(&B, sizeof(float) * K * 1024);
  (void)hipMalloc(&C, sizeof(float) * (long long)M * 1024);
  (void)hipMalloc(&H, sizeof(float) * (long long)M * 1024);
  (void)hipMalloc(&bias, sizeof(float) * 1024);
  hipLaunchKernelGGL(fill_kernel, dim3((M * K + 255) / 256), dim3(256), 0, 0, A, (long long)M * K, 1u);
  hipLaunchKernelGGL(fill_kernel, dim3((K * 1024 + 255) / 256), dim3(256), 0, 0, B, (long long)K * 1024, 2u);
  hipLaunchKernelGGL(fill_kernel, dim3(4), dim3(256), 0, 0, bias, 1024ll, 3u);
  (void)hipDeviceSynchronize();
  for (int N : Ns) {
    const double gf = 2.0 * M * N * K / 1e9;
    {
      const dim3 g3((N + 127) / 128, M / 128);
#define ZF_V(TB, ST, AB, W, F, EPI, HH)                                                                        \
  {                                                                                                             \
    const float t = time_it(                                                                                    \
        [&] {                                                                                                   \
          hipLaunchKernelGGL((x3v<TB, ST, AB, W, F>), g3, dim3(256), 0, 0, M, N, K, A, K, B, N, C, N, EPI, bias,  \
                             HH, nullptr, ZF_ACT_SWISH);                                                        \
        },                                                                                                      \
        20);                                                                                                    \
    std::printf("N=%d variant abl=%d fast=%d epi=%d H=%d: %8.1f us (%6.1f TF/s)\n", N, AB, (int)F, EPI,        \
                HH != nullptr, t, gf / t * 1e3);                                                                \
  }
      ZF_V(false, 1, 0, true, false, 1, H) ZF_V(false, 1, 0, true, true, 1, H) ZF_V(false, 1, 0, true, false, 1, nullptr)
      ZF_V(false, 1, 0, true, false, 0, nullptr)
#undef ZF_V
    }
    for (int withH = 0; withH < 2; ++withH) {
      float* h = withH ? H : nullptr;
      for (int epi : {(int)zf::kEpiNone, (int)zf::kEpiBias}) {
        const dim3 g3((N + 127) / 128, M / 128);
        const float tx3 = time_it(
            [&] {
              hipLaunchKernelGGL((zf::gemm_x3_kernel<false, true>), x3grid(g3), dim3(256), 0, 0, M, N, K, A, K, B, N, C, N, epi,
                                 bias, h, nullptr, ZF_ACT_SWISH);
            },
            20);
        const float tmg = time_it(
            [&] {
              hipLaunchKernelGGL((zf::mgemm_kernel<128, 128, false, false, false>), g3, dim3(256), 0, 0, M, N, K, A,
                                 K, B, N, C, N, epi, bias, h, nullptr, 0, ZF_ACT_SWISH);
            },
            20);
        std::printf("N=%d epi=%d H=%d  x3 %8.1f us (%6.1f TF/s)  mgemm128 %8.1f us (%6.1f TF/s)\n", N, epi, withH,
                    tx3, gf / tx3 * 1e3, tmg, gf / tmg * 1e3);
      }
    }
    // x3 vs fp32 MFMA on the same operands (epi none), and the transposed-B
    // form (B read as [N][K]: the input-gradient GEMMs) with the DSwish epilogue
    {
      const long long n = (long long)M * N;
      float *C1, *C2;
      (void)hipMalloc(&C1, sizeof(float) * n);
      (void)hipMalloc(&C2, sizeof(float) * n);
      const dim3 g3((N + 127) / 128, M / 128);
      hipLaunchKernelGGL((zf::gemm_x3_kernel<false, true>), x3grid(g3), dim3(256), 0, 0, M, N, K, A, K, B, N, C1, N,
                         (int)zf::kEpiNone, bias, nullptr, nullptr, ZF_ACT_SWISH);
      hipLaunchKernelGGL((zf::mgemm_kernel<128, 128, false, false, false>), g3, dim3(256), 0, 0, M, N, K, A, K, B, N,
                         C2, N, (int)zf::kEpiNone, bias, nullptr, nullptr, 0, ZF_ACT_SWISH);
      std::vector<float> h1(n), h2(n);
      (void)hipMemcpy(h1.data(), C1, sizeof(float) * n, hipMemcpyDeviceToHost);
      (void)hipMemcpy(h2.data(), C2, sizeof(float) * n, hipMemcpyDeviceToHost);
      double md = 0, mx = 0;
      for (long long i = 0; i < n; ++i) {
        md = std::max(md, (double)std::fabs(h1[i] - h2[i]));
        mx = std::max(mx, (double)std::fabs(h2[i]));
      }
      std::printf("N=%d  x3 vs fp32 MFMA: max |diff| / max |C| = %.3g\n", N, md / mx);
      hipLaunchKernelGGL((x3v<false, 1, 0, true>), g3, dim3(256), 0, 0, M, N, K, A, K, B, N, C2, N,
                         (int)zf::kEpiBias, bias, C, nullptr, ZF_ACT_SWISH);
      hipLaunchKernelGGL((zf::gemm_x3_kernel<false, true>), x3grid(g3), dim3(256), 0, 0, M, N, K, A, K, B, N, C1, N,
                         (int)zf::kEpiBias, bias, H, nullptr, ZF_ACT_SWISH);
      {
        std::vector<float> w1(n), w2(n), q1(n), q2(n);
        (void)hipMemcpy(w1.data(), C1, sizeof(float) * n, hipMemcpyDeviceToHost);
        (void)hipMemcpy(w2.data(), C2, sizeof(float) * n, hipMemcpyDeviceToHost);
        (void)hipMemcpy(q1.data(), H, sizeof(float) * n, hipMemcpyDeviceToHost);
        (void)hipMemcpy(q2.data(), C, sizeof(float) * n, hipMemcpyDeviceToHost);
        long long d1 = 0, d2 = 0;
        for (long long i = 0; i < n; ++i) { d1 += w1[i] != w2[i]; d2 += q1[i] != q2[i]; }
        std::printf("N=%d  wide-store variant vs shipped kernel (bias+swish): %lld / %lld z, %lld h elements differ\n", N, d1, n, d2);
      }
      // transposed B: Bt[n][k] = B[k][n] (K x N -> N x K), C = A . Bt^T must equal C1
      float* Bt;
      (void)hipMalloc(&Bt, sizeof(float) * N * K);
      std::vector<float> hb((size_t)K * N), hbt((size_t)K * N);
      (void)hipMemcpy(hb.data(), B, sizeof(float) * K * N, hipMemcpyDeviceToHost);
      for (int k = 0; k < K; ++k)
        for (int j = 0; j < N; ++j) hbt[(size_t)j * K + k] = hb[(size_t)k * N + j];
      (void)hipMemcpy(Bt, hbt.data(), sizeof(float) * K * N, hipMemcpyHostToDevice);
      hipLaunchKernelGGL((zf::gemm_x3_kernel<true, true>), x3grid(g3), dim3(256), 0, 0, M, N, K, A, K, Bt, K, C2, N,
                         (int)zf::kEpiNone, bias, nullptr, nullptr, ZF_ACT_SWISH);
      (void)hipMemcpy(h2.data(), C2, sizeof(float) * n, hipMemcpyDeviceToHost);
      long long neq = 0;
      for (long long i = 0; i < n; ++i) neq += h1[i] != h2[i];
      std::printf("N=%d  x3 transposed-B form: %lld of %lld elements differ from the row-major form\n", N, neq, n);
      const float ttb = time_it(
          [&] {
            hipLaunchKernelGGL((zf::gemm_x3_kernel<true, true>), x3grid(g3), dim3(256), 0, 0, M, N, K, A, K, Bt, K, C2, N,
                               (int)zf::kEpiDSwish, bias, nullptr, C1, ZF_ACT_SWISH);
          },
          20);
      const float tmtb = time_it(
          [&] {
            hipLaunchKernelGGL((zf::mgemm_kernel<128, 128, false, true, false>), g3, dim3(256), 0, 0, M, N, K, A, K,
                               Bt, K, C2, N, (int)zf::kEpiDSwish, bias, nullptr, C1, 0, ZF_ACT_SWISH);
          },
          20);
      std::printf("N=%d  transposed B + dswish: x3 %8.1f us (%6.1f TF/s)  mgemm128 %8.1f us (%6.1f TF/s)\n", N, ttb,
                  gf / ttb * 1e3, tmtb, gf / tmtb * 1e3);
      (void)hipFree(C1);
      (void)hipFree(C2);
      (void)hipFree(Bt);
    }
    const long long n = (long long)M * N;
    const float tw = time_it(
        [&] { hipLaunchKernelGGL(write_kernel, dim3((unsigned)((n / 4 + 255) / 256)), dim3(256), 0, 0, C, H, n); }, 20);
    std::printf("N=%d  plain float4 write of C and H: %8.1f us (%.2f TB/s)\n", N, tw, 8.0 * n / tw * 1e-6);
  }
  {  // the last layer's input gradient: K = 760 (not a multiple of the 32-wide k-tile), transposed B
    const int N = 256, K2 = 760;
    const double gf = 2.0 * M * N * K2 / 1e9;
    float *G, *W;
    (void)hipMalloc(&G, sizeof(float) * (long long)M * K2);
    (void)hipMalloc(&W, sizeof(float) * N * K2);
    hipLaunchKernelGGL(fill_kernel, dim3((unsigned)(((long long)M * K2 + 255) / 256)), dim3(256), 0, 0, G,
                       (long long)M * K2, 5u);
    hipLaunchKernelGGL(fill_kernel, dim3((N * K2 + 255) / 256), dim3(256), 0, 0, W, (long long)N * K2, 6u);
    const dim3 g3(N / 128, M / 128);
    const float tx = time_it(
        [&] {
          hipLaunchKernelGGL((zf::gemm_x3_kernel<true, true>), x3grid(g3), dim3(256), 0, 0, M, N, K2, G, K2, W, K2, C, N,
                             (int)zf::kEpiDSwish, bias, nullptr, H, ZF_ACT_SWISH);
        },
        20);
    const float tm = time_it(
        [&] {
          hipLaunchKernelGGL((zf::mgemm_kernel<128, 128, false, true, false>), g3, dim3(256), 0, 0, M, N, K2, G, K2,
                             W, K2, C + (long long)M * N, N, (int)zf::kEpiDSwish, bias, nullptr, H, 0, ZF_ACT_SWISH);
        },
        20);
    const long long n = (long long)M * N;
    std::vector<float> h1(n), h2(n);
    (void)hipMemcpy(h1.data(), C, sizeof(float) * n, hipMemcpyDeviceToHost);
    (void)hipMemcpy(h2.data(), C + n, sizeof(float) * n, hipMemcpyDeviceToHost);
    double md = 0, mx = 0;
    for (long long i = 0; i < n; ++i) {
      md = std::max(md, (double)std::fabs(h1[i] - h2[i]));
      mx = std::max(mx, (double)std::fabs(h2[i]));
    }
    std::printf("K=760 transposed B + dswish: x3 %8.1f us (%6.1f TF/s)  mgemm128 %8.1f us (%6.1f TF/s)  max|diff|/max %.3g\n",
                tx, gf / tx * 1e3, tm, gf / tm * 1e3, md / mx);
  }
  (void)hipDeviceSynchronize();
  return 0;
}
