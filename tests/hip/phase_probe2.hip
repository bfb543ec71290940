// Probe (GPU box, tuning only): the synthetic per-coupling stream of
// phase_probe.hip (168 MFMAs with exp+2fma fillers, then a VALU phase) with
// the split-MFMA kernel's structure added piece by piece, to find which one
// keeps three waves per SIMD from overlapping:
//   DEP  : the MFMAs as dependent triples on one accumulator (the split
//          product lo*hi + hi*lo + hi*hi) instead of round-robin over 4
//   LDS  : each triple's A fragment read from LDS (2 x ds_read_b128) right
//          before it, waited with lgkmcnt(0)
//   BAR  : a workgroup barrier every 24 MFMAs (4-wave blocks, 3 per CU)
//   CHAIN: the VALU phase as 16 serially dependent steps per chain (a bin
//          search) on 2 chains instead of 16 independent chains
// Grid: 768 blocks x 256 threads, ~50 KiB LDS each (3 blocks per CU).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));

#define FMA(x) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(c1), "v"(c2))
#define EXP(x) asm volatile("v_exp_f32 %0, %0" : "+v"(x))

template <int F>
__global__ __launch_bounds__(256, 3) void probe(int iters, float* out, unsigned long long* cyc) {
  constexpr bool DEP = F & 1, LDS = F & 2, BAR = F & 4, CHAIN = F & 8;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 4096; i += 256) reinterpret_cast<float*>(lds)[i] = 0.001f * (i & 255);
  __syncthreads();
  halfx8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (_Float16)(0.001f * (lane + i)); b[i] = (_Float16)(0.002f * (lane - i)); }
  floatx16 acc[4] = {};
  float va[8], v[16];
  for (int i = 0; i < 16; ++i) v[i] = 0.001f * (lane + i);
  for (int i = 0; i < 8; ++i) va[i] = 0.003f * (lane + i);
  const float c1 = 0.999f, c2 = 1e-4f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    // MFMA phase: 56 triples = 168 MFMAs
#pragma unroll
    for (int t = 0; t < 56; ++t) {
      if constexpr (BAR) {
        if (t % 8 == 0) __syncthreads();
      }
      halfx8 a0 = a, a1 = a;
      if constexpr (LDS) {
        const char* p = lds + ((t * 2048 + lane * 16) & 16383);
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:1024\n\ts_waitcnt lgkmcnt(0)"
                     : "=v"(a0), "=v"(a1)
                     : "v"((unsigned)(size_t)p));
      }
#pragma unroll
      for (int m = 0; m < 3; ++m) {
        floatx16& c = DEP ? acc[t & 3] : acc[(3 * t + m) & 3];
        if (m == 1) asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(c) : "v"(a1), "v"(b));
        else asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(c) : "v"(a0), "v"(b));
        EXP(va[(3 * t + m) & 7]);
        FMA(va[(3 * t + m + 1) & 7]);
        FMA(va[(3 * t + m + 2) & 7]);
      }
    }
    // VALU phase: 672 fma + 48 exp
    if constexpr (CHAIN) {
#pragma unroll
      for (int i = 0; i < 336; ++i) {
        FMA(v[0]);
        FMA(v[1]);
        if (i % 14 == 0) {
          EXP(v[0]);
          EXP(v[1]);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < 42; ++i) {
#pragma unroll
        for (int j = 0; j < 16; ++j) FMA(v[j]);
        if (i % 7 == 0)
#pragma unroll
          for (int j = 0; j < 8; ++j) EXP(v[2 * j]);
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float sink = 0.f;
  for (int r = 0; r < 16; ++r) sink += acc[0][r] + acc[1][r] + acc[2][r] + acc[3][r];
  for (int i = 0; i < 16; ++i) sink += v[i];
  for (int i = 0; i < 8; ++i) sink += va[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = sink;
  if (lane == 0) cyc[blockIdx.x * 4 + w] = t1 - t0;
}

template <int F>
void run(int iters, float* d_out, unsigned long long* d_cyc, int per_cu) {
  const int blocks = 768;
  const size_t lds = per_cu == 3 ? 50 * 1024 : per_cu == 2 ? 76 * 1024 : 150 * 1024;
  hipLaunchKernelGGL(probe<F>, dim3(blocks), dim3(256), lds, 0, iters, d_out, d_cyc);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(probe<F>, dim3(blocks), dim3(256), lds, 0, iters, d_out, d_cyc);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> cyc(blocks * 4);
  (void)hipMemcpy(cyc.data(), d_cyc, cyc.size() * 8, hipMemcpyDeviceToHost);
  std::vector<double> v;
  for (auto c : cyc) v.push_back((double)c / iters);
  std::sort(v.begin(), v.end());
  // per SIMD: 3 waves (3 blocks x 4 waves over 4 SIMDs) each doing `iters` set-couplings
  printf("waves/SIMD %d F=%2d DEP %d LDS %d BAR %d CHAIN %d: %8.1f cyc per set-coupling per wave (median) -> %7.1f per SIMD; wall %.3f ms\n",
         per_cu, F, F & 1, (F >> 1) & 1, (F >> 2) & 1, (F >> 3) & 1, v[v.size() / 2], v[v.size() / 2] / per_cu, ms);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20;
  float* d_out;
  unsigned long long* d_cyc;
  (void)hipMalloc(&d_out, 768 * 256 * 4);
  (void)hipMalloc(&d_cyc, 768 * 4 * 8);
  for (int pc : {1, 3}) {
    run<0>(iters, d_out, d_cyc, pc);
    run<1>(iters, d_out, d_cyc, pc);
    run<2>(iters, d_out, d_cyc, pc);
    run<3>(iters, d_out, d_cyc, pc);
    run<15>(iters, d_out, d_cyc, pc);
  }
  return 0;
}
