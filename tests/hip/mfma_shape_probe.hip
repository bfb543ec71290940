// MFMA tile shape under VALU load ("16x16x32 MFMA"): the same
// fp16 flops as v_mfma_f32_32x32x16_f16 (one per step) or as
// v_mfma_f32_16x16x32_f16 (two per step), each step followed by V
// independent VALU fmas (the split kernel issues ~9.5 VALU per 32x32x16
// MFMA), at W waves per SIMD.  Prints TFLOP/s (fp16, dense) per
// configuration.  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tests/hip/mfma_shape_probe.hip -o tune/mfma_shape_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kSteps = 2048;  // unrolled by the compiler; accumulators rotate (4 big, 8 small)

template <bool BIG, int V>
__global__ __launch_bounds__(256) void probe(float* out, float seed) {
  const int lane = threadIdx.x & 63;
  half8 a, b;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = (_Float16)(seed * (lane + i));
    b[i] = (_Float16)(seed * (lane - i));
  }
  floatx16 c16[4] = {floatx16{0}, floatx16{0}, floatx16{0}, floatx16{0}};
  floatx4 c4[8] = {floatx4{0}, floatx4{0}, floatx4{0}, floatx4{0}, floatx4{0}, floatx4{0}, floatx4{0}, floatx4{0}};
  float vx[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) vx[i] = seed * (i + lane);
  for (int s = 0; s < kSteps; s += 4) {  // four 32x32x16-equivalents, static accumulators
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (BIG) {
        c16[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c16[u], 0, 0, 0);
      } else {
        c4[2 * u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c4[2 * u], 0, 0, 0);
        c4[2 * u + 1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c4[2 * u + 1], 0, 0, 0);
      }
#pragma unroll
      for (int v = 0; v < V; ++v) vx[(u * V + v) & 15] = __builtin_fmaf(vx[(u * V + v) & 15], 1.0001f, 0.5f);
    }
  }
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc += vx[i] + c16[0][i] + c16[1][i] + c16[2][i] + c16[3][i];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    acc += c4[0][i] + c4[1][i] + c4[2][i] + c4[3][i] + c4[4][i] + c4[5][i] + c4[6][i] + c4[7][i];
  if (acc == 12345.f) out[blockIdx.x * blockDim.x + threadIdx.x] = acc;  // keep the work
}

template <bool BIG, int V>
void run(int waves_per_simd, float* out) {
  int ncu = 256;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = ncu * waves_per_simd;  // 4 waves per block: one per SIMD
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL((probe<BIG, V>), dim3(blocks), dim3(256), 0, 0, out, 1e-3f);
  (void)hipEventRecord(e0, 0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((probe<BIG, V>), dim3(blocks), dim3(256), 0, 0, out, 1e-3f);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double flops = 5.0 * blocks * 4 * (double)kSteps * 32768.0;
  std::printf("%s V=%2d waves/SIMD=%d: %8.1f TFLOP/s fp16 (%.3f ms per launch)\n",
              BIG ? "32x32x16      " : "2 x 16x16x32  ", V, waves_per_simd, flops / (ms * 1e-3) * 1e-12, ms / 5);
}

int main() {
  float* out;
  (void)hipMalloc(&out, 1 << 24);
  for (int w : {1, 3}) {
    run<true, 0>(w, out);
    run<false, 0>(w, out);
    run<true, 8>(w, out);
    run<false, 8>(w, out);
    run<true, 12>(w, out);
    run<false, 12>(w, out);
  }
  (void)hipDeviceSynchronize();
  return 0;
}
