// Probe (GPU box, tuning only): a synthetic model of the split-MFMA flow
// kernel's per-coupling instruction stream, to price schedules before
// writing them.  One "set-coupling" = an MFMA phase (168
// v_mfma_f32_32x32x16_f16, each followed by its own filler: one
// transcendental + two v_fma_f32, like the deferred swish + split) and a
// VALU-only phase (the spline / layer 0: 672 v_fma_f32 + 48 transcendentals
// in 16 independent chains).
//   single: each wave runs [MFMA phase][VALU phase] per iteration (1 set);
//   dual  : each wave runs two sets, B's VALU phase spread over A's MFMA gaps
//           (4 fma + 2/7 transcendental extra per gap), then A's over B's —
//           two set-couplings per iteration.
// Reported: cycles per set-coupling per wave (s_memtime), and wall time per
// set-coupling per SIMD.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));

#define MF(acc) asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b))
#define FMA(x) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(c1), "v"(c2))
#define EXP(x) asm volatile("v_exp_f32 %0, %0" : "+v"(x))

constexpr int kMfma = 168;

template <bool DUAL, int FILL_FMA>
__device__ __forceinline__ void mfma_phase(floatx16 (&acc)[4], float (&va)[8], float (&vb)[16], const halfx8& a,
                                           const halfx8& b, float c1, float c2) {
#pragma unroll
  for (int m = 0; m < kMfma; ++m) {
    MF(acc[m & 3]);
    EXP(va[m & 7]);
#pragma unroll
    for (int f = 0; f < FILL_FMA; ++f) FMA(va[(m + 1 + f) & 7]);
    if constexpr (DUAL) {  // the other set's VALU phase: 672 fma + 48 trans over 168 gaps
      FMA(vb[(4 * m) & 15]);
      FMA(vb[(4 * m + 1) & 15]);
      FMA(vb[(4 * m + 2) & 15]);
      FMA(vb[(4 * m + 3) & 15]);
      if (m % 7 == 3 || m % 7 == 6) EXP(vb[(m + 5) & 15]);
    }
  }
}

__device__ __forceinline__ void valu_phase(float (&v)[16], float c1, float c2) {
#pragma unroll
  for (int i = 0; i < 42; ++i) {
#pragma unroll
    for (int j = 0; j < 16; ++j) FMA(v[j]);
    if (i % 7 == 0)
#pragma unroll
      for (int j = 0; j < 8; ++j) EXP(v[2 * j]);
  }
}

template <int MODE>  // 0: single, 1: dual, 2: single with 3 fma fillers, 3: dual with 3
__global__ __launch_bounds__(768, 1) void probe(int iters, int nw, float* out, unsigned long long* cyc) {
  extern __shared__ char lds[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (threadIdx.x == 0) lds[0] = 0;
  __syncthreads();
  halfx8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (_Float16)(0.001f * (lane + i)); b[i] = (_Float16)(0.002f * (lane - i)); }
  floatx16 accA[4] = {}, accB[4] = {};
  float vaA[8], vaB[8], vA[16], vB[16];
  for (int i = 0; i < 16; ++i) { vA[i] = 0.001f * (lane + i); vB[i] = 0.002f * (lane + i); }
  for (int i = 0; i < 8; ++i) { vaA[i] = 0.003f * (lane + i); vaB[i] = 0.004f * (lane + i); }
  const float c1 = 0.999f, c2 = 1e-4f;
  constexpr int FF = (MODE & 2) ? 3 : 2;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE & 1) {
      mfma_phase<true, FF>(accA, vaA, vB, a, b, c1, c2);
      mfma_phase<true, FF>(accB, vaB, vA, a, b, c1, c2);
    } else {
      mfma_phase<false, FF>(accA, vaA, vB, a, b, c1, c2);
      valu_phase(vA, c1, c2);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float sink = 0.f;
  for (int r = 0; r < 16; ++r) sink += accA[0][r] + accA[1][r] + accA[2][r] + accA[3][r] + accB[0][r] + accB[3][r];
  for (int i = 0; i < 16; ++i) sink += vA[i] + vB[i];
  for (int i = 0; i < 8; ++i) sink += vaA[i] + vaB[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = sink;
  if (lane == 0) cyc[blockIdx.x * 12 + w] = t1 - t0;
}

template <int MODE>
void run(const char* name, int nw, int iters, float* d_out, unsigned long long* d_cyc) {
  const int blocks = 256;
  hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(nw * 64), 150 * 1024, 0, iters, nw, d_out, d_cyc);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(nw * 64), 150 * 1024, 0, iters, nw, d_out, d_cyc);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> cyc(blocks * 12);
  (void)hipMemcpy(cyc.data(), d_cyc, cyc.size() * 8, hipMemcpyDeviceToHost);
  std::vector<double> v;
  const int sets = (MODE & 1) ? 2 : 1;
  for (int bk = 0; bk < blocks; ++bk)
    for (int q = 0; q < nw; ++q) v.push_back((double)cyc[bk * 12 + q] / (iters * sets));
  std::sort(v.begin(), v.end());
  const int per_simd = nw / 4;
  // wall-clock ns per set-coupling per SIMD
  const double ns = ms * 1e6 / ((double)iters * sets * per_simd);
  printf("%-22s waves/SIMD %d: %8.1f cyc per set-coupling per wave (median), wall %.3f ms = %7.1f ns per "
         "set-coupling per SIMD\n", name, per_simd, v[v.size() / 2], ms, ns);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 40;
  float* d_out;
  unsigned long long* d_cyc;
  (void)hipMalloc(&d_out, 256 * 768 * 4);
  (void)hipMalloc(&d_cyc, 256 * 12 * 8);
  for (int nw : {4, 8, 12}) {
    run<0>("single (exp+2fma)", nw, iters, d_out, d_cyc);
    run<1>("dual (exp+2fma)", nw, iters, d_out, d_cyc);
    run<2>("single (exp+3fma)", nw, iters, d_out, d_cyc);
    run<3>("dual (exp+3fma)", nw, iters, d_out, d_cyc);
  }
  return 0;
}
