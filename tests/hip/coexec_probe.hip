// Probe (GPU box, tuning only): do bf16 MFMAs of one wave and plain VALU of
// another wave on the same SIMD execute concurrently, and does it matter
// whether the MFMA accumulator lives in VGPRs or AGPRs?
//   waves 0-3: M MFMA (32x32x16 bf16) chains;  waves 4-7: VALU fma chains.
// mode 0: MFMA waves only, 1: VALU waves only, 2: both (VGPR acc),
// 3: MFMA only (AGPR acc), 4: both (AGPR acc), 5: both, the VALU wave also
//    doing v_exp/v_rcp (transcendental mix like swish),
// 6: the MFMA waves themselves interleave the VALU waves' work (same total
//    VALU: 8 fma per MFMA), VALU waves idle.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int MODE>
__global__ __launch_bounds__(512, 1) void probe(float* out, int iters) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  float sink = 0.f;
  const bool mfma_wave = wave < 4;
  if (mfma_wave && MODE != 1 && MODE != 6) {
    bf16x8 a, b;
    for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(0.001f * (lane + i)); b[i] = (__bf16)(0.002f * (lane - i)); }
    floatx16 acc0 = {0}, acc1 = {0}, acc2 = {0}, acc3 = {0};
    if (MODE == 3 || MODE == 4) {
      for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc0) : "v"(a), "v"(b));
          asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc1) : "v"(a), "v"(b));
          asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc2) : "v"(a), "v"(b));
          asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc3) : "v"(a), "v"(b));
        }
      }
    } else {
      for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc1, 0, 0, 0);
          acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc2, 0, 0, 0);
          acc3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc3, 0, 0, 0);
        }
      }
    }
    for (int r = 0; r < 16; ++r) sink += acc0[r] + acc1[r] + acc2[r] + acc3[r];
  }
  if (mfma_wave && MODE == 6) {
    bf16x8 a, b;
    for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(0.001f * (lane + i)); b[i] = (__bf16)(0.002f * (lane - i)); }
    floatx16 acc0 = {0}, acc1 = {0}, acc2 = {0}, acc3 = {0};
    float v[16];
    for (int i = 0; i < 16; ++i) v[i] = 0.001f * (lane + i);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc0, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = __builtin_fmaf(v[i], 0.999f, 0.0001f);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc1, 0, 0, 0);
#pragma unroll
        for (int i = 8; i < 16; ++i) v[i] = __builtin_fmaf(v[i], 0.999f, 0.0001f);
        acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc2, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = __builtin_fmaf(v[i], 0.999f, 0.0001f);
        acc3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc3, 0, 0, 0);
#pragma unroll
        for (int i = 8; i < 16; ++i) v[i] = __builtin_fmaf(v[i], 0.999f, 0.0001f);
      }
    }
    for (int r = 0; r < 16; ++r) sink += acc0[r] + acc1[r] + acc2[r] + acc3[r];
    for (int i = 0; i < 16; ++i) sink += v[i];
  }
  if (!mfma_wave && MODE != 0 && MODE != 3 && MODE != 6) {
    float v[16];
    for (int i = 0; i < 16; ++i) v[i] = 0.001f * (lane + i);
    // 16 MFMAs of the other wave = 512 cycles; 128 independent fma per iter (4 cyc each = 512)
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < 8; ++k)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          if (MODE == 5 && (i & 7) == 0) v[i] = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(v[i]));
          else v[i] = __builtin_fmaf(v[i], 0.999f, 0.0001f);
        }
    }
    for (int i = 0; i < 16; ++i) sink += v[i];
  }
  out[blockIdx.x * 512 + threadIdx.x] = sink;
}

template <int MODE>
float run(float* d, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(probe<MODE>, dim3(256), dim3(512), 0, 0, d, iters);
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(probe<MODE>, dim3(256), dim3(512), 0, 0, d, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

int main() {
  float* d;
  (void)hipMalloc(&d, 256 * 512 * 4);
  const int it = 2000;
  printf("mode0 mfma-only(vgpr)  %.3f ms\n", run<0>(d, it));
  printf("mode1 valu-only        %.3f ms\n", run<1>(d, it));
  printf("mode2 both(vgpr acc)   %.3f ms\n", run<2>(d, it));
  printf("mode3 mfma-only(agpr)  %.3f ms\n", run<3>(d, it));
  printf("mode4 both(agpr acc)   %.3f ms\n", run<4>(d, it));
  printf("mode5 both+trans(vgpr) %.3f ms\n", run<5>(d, it));
  printf("mode6 in-wave fillers  %.3f ms\n", run<6>(d, it));
  return 0;
}
