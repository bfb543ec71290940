// Probe (GPU box, tuning only): how fast can ONE SIMD run
// the instruction mix of flow_kernel_x3's cfg2 wave-coupling when nothing
// waits on anything — no data dependencies, no LDS, no barriers — and does
// splitting the work into MFMA waves and VALU waves (producer / consumer)
// beat running it uniformly?  The mix per wave-coupling is the static budget
// of profiles/r05_x3_valu_budget.txt: 172 v_mfma_f32_32x32x16_f16, 297
// transcendentals, 128 v_fma_mix, 122 two-pass VALU (v_cvt_pk / max3 /
// cndmask) and ~800 full-rate fp32 VALU.  One "unit" = 4 MFMAs + 4 v_exp +
// 3 v_rcp + 3 v_fma_mixlo + 3 v_cvt_pk + 18 v_fma (43 units = one
// wave-coupling), every VALU on its own register chain (16 chains per kind).
// Layouts (12 waves per CU, one block per CU, LDS-pinned; wave w runs on
// SIMD w % 4):
//   0 uniform:     every wave issues U units, VALU of a unit between its MFMAs;
//   1 specialised: waves 0-3 issue the SIMD's 3U units of MFMAs only, waves
//                  4-11 the VALU of 1.5U units each (two VALU waves per SIMD);
//   2 MFMA only (3 waves x U units), 3 VALU only (3 waves x U units);
//   4 specialised + in-wave share: the MFMA waves also carry 1/3 of the VALU
//                  of their units, the VALU waves 1/3 each.
// Prints SIMD cycles (s_memtime of the slowest wave) per wave-coupling
// (3 waves x U units / 43 per SIMD), to set against the kernel's measured
// 11,455 cycles per wave-coupling (GRBM_GUI_ACTIVE, r05_x3_stall_counters).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));

#define EXP(r) asm volatile("v_exp_f32 %0, %0" : "+v"(r))
#define RCP(r) asm volatile("v_rcp_f32 %0, %0" : "+v"(r))
#define MIX(r, b) asm volatile("v_fma_mixlo_f16 %0, %1, 1.0, -%0 op_sel_hi:[0,0,1]" : "+v"(r) : "v"(b))
#define CVT(r, b) asm volatile("v_cvt_pk_f16_f32 %0, %1, %0" : "+v"(r) : "v"(b))
#define FMA(r, b) asm volatile("v_fma_f32 %0, %1, %1, %0" : "+v"(r) : "v"(b))

struct Regs {
  float e[16], f[16], m[8], c[8];
};

// The VALU of one unit, share s of n (n = 1: all of it; the instructions are
// dealt round-robin so every share has the same mix); i0 rotates the chains.
template <int N, int S>
__device__ __forceinline__ void valu_unit(Regs& r, float b, int i0) {
  int k = 0;
#define DEAL(stmt) do { if (k % N == S) { stmt; } ++k; } while (0)
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    DEAL(EXP(r.e[(q) & 15]));
    DEAL(FMA(r.f[(4 * q) & 15], b));
    DEAL(FMA(r.f[(4 * q + 1) & 15], b));
    if (q < 3) DEAL(RCP(r.e[(8 + q) & 15]));
    DEAL(FMA(r.f[(4 * q + 2) & 15], b));
    if (q < 3) DEAL(MIX(r.m[(q) & 7], b));
    DEAL(FMA(r.f[(4 * q + 3) & 15], b));
    if (q < 3) DEAL(CVT(r.c[(q) & 7], b));
    if (q < 2) DEAL(FMA(r.f[(9 + q) & 15], b));
  }
#undef DEAL
}

template <int MODE>
__global__ __launch_bounds__(768, 1) void probe(unsigned long long* out, int units, float seed) {
  extern __shared__ char pin[];
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  if (seed > 1e30f) pin[threadIdx.x] = 0;  // keep the LDS allocation: one block per CU
  Regs r;
#pragma unroll
  for (int i = 0; i < 16; ++i) { r.e[i] = 1e-3f * (lane + i) + seed; r.f[i] = 1.0f + r.e[i]; }
#pragma unroll
  for (int i = 0; i < 8; ++i) { r.m[i] = r.e[i]; r.c[i] = r.f[i]; }
  const float b = 0.999f + seed;
  halfx8 x, y;
#pragma unroll
  for (int i = 0; i < 8; ++i) { x[i] = (_Float16)(0.01f * (lane + i)); y[i] = (_Float16)(0.02f * (lane - i)); }
  floatx16 a0 = {0}, a1 = {0}, a2 = {0}, a3 = {0};
  const bool mw = wave < 4;
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#define MF4(V0, V1, V2, V3)                                   \
  a0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(x, y, a0, 0, 0, 0); V0; \
  __builtin_amdgcn_sched_barrier(0);                          \
  a1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(x, y, a1, 0, 0, 0); V1; \
  __builtin_amdgcn_sched_barrier(0);                          \
  a2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(x, y, a2, 0, 0, 0); V2; \
  __builtin_amdgcn_sched_barrier(0);                          \
  a3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(x, y, a3, 0, 0, 0); V3; \
  __builtin_amdgcn_sched_barrier(0);
  if (MODE == 0 || (MODE == 2)) {
    for (int u = 0; u < units; ++u) {
      if (MODE == 0) {
        MF4((valu_unit<4, 0>(r, b, u)), (valu_unit<4, 1>(r, b, u)), (valu_unit<4, 2>(r, b, u)), (valu_unit<4, 3>(r, b, u)))
      } else {
        MF4((void)0, (void)0, (void)0, (void)0)
      }
    }
  } else if (MODE == 3) {
    for (int u = 0; u < units; ++u) valu_unit<1, 0>(r, b, u);
  } else if (MODE == 1) {
    if (mw) {
      for (int u = 0; u < 3 * units; ++u) { MF4((void)0, (void)0, (void)0, (void)0) }
    } else {
      for (int u = 0; u < 3 * units / 2; ++u) valu_unit<1, 0>(r, b, u);
    }
  } else if (MODE == 4) {
    if (mw) {
      for (int u = 0; u < 3 * units; ++u) {
        MF4((valu_unit<12, 0>(r, b, u)), (valu_unit<12, 1>(r, b, u)), (valu_unit<12, 2>(r, b, u)), (valu_unit<12, 3>(r, b, u)))
      }
    } else {
      // two thirds of the SIMD's VALU over its two VALU waves
      for (int u = 0; u < 3 * units / 2; ++u) {
        valu_unit<3, 1>(r, b, u);
        valu_unit<3, 2>(r, b, u);
      }
    }
  }
#undef MF4
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += r.e[i] + r.f[i] + a0[i] + a1[i] + a2[i] + a3[i];
#pragma unroll
  for (int i = 0; i < 8; ++i) s += r.m[i] + r.c[i];
  if (lane == 0) out[blockIdx.x * 16 + wave] = (t1 - t0) | (s == 12345.f ? 1ull : 0ull);
}

template <int MODE>
double run(unsigned long long* d, unsigned long long* h, int units) {
  const size_t lds = 100 * 1024;
  for (int rep = 0; rep < 2; ++rep)
    hipLaunchKernelGGL((probe<MODE>), dim3(256), dim3(768), lds, 0, d, units, 0.f);
  hipDeviceSynchronize();
  hipMemcpy(h, d, 256 * 16 * 8, hipMemcpyDeviceToHost);
  unsigned long long mx = 0;
  for (int i = 0; i < 256; ++i)
    for (int w = 0; w < 12; ++w) mx = h[i * 16 + w] > mx ? h[i * 16 + w] : mx;
  // SIMD cycles per wave-coupling: 3 waves x units / 43 wave-couplings per SIMD
  return (double)mx / (3.0 * units / 43.0);
}

int main() {
  unsigned long long *d, *h;
  hipMalloc(&d, 256 * 16 * 8);
  h = (unsigned long long*)malloc(256 * 16 * 8);
  const int units = 43 * 40;  // 40 wave-couplings per wave
  const char* names[] = {"uniform (3 waves x mix)", "specialised (1 MFMA + 2 VALU waves)", "MFMA only", "VALU only",
                         "specialised, 1/3 VALU in the MFMA wave"};
  const double t[5] = {run<0>(d, h, units), run<1>(d, h, units), run<2>(d, h, units), run<3>(d, h, units),
                       run<4>(d, h, units)};
  for (int m = 0; m < 5; ++m)
    printf("%-40s %8.0f SIMD cycles per wave-coupling (kernel: 11455; frac ceiling at the kernel's clock %.3f)\n",
           names[m], t[m], 0.349 * 11455.0 / t[m]);
  return 0;
}
