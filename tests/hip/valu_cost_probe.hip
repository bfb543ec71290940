// Probe (GPU box, tuning only): SIMD cycles per wave64 instruction on gfx950
// for the instruction kinds of the split-MFMA flow kernel, at NW waves per
// SIMD (one 256*NW-thread block per CU, LDS-pinned), each wave issuing 16
// independent chains; and the same instructions as in-wave fillers between
// v_mfma_f32_32x32x16_f16 of the issuing wave (F per MFMA), with the other
// waves of the SIMD idle or issuing the same filler stream (cross-wave).
// Prints cycles per instruction per SIMD (s_memtime ticks of the slowest wave).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));

enum { OP_FMA, OP_MUL, OP_EXP, OP_RCP, OP_SQRT, OP_MIX, OP_CVTPK, OP_MAX3, OP_CND, OP_PKFMA, OP_CVTF16, OP_CVTF16HI, OP_AND, OP_PKMUL, OP_LDEXP, OP_LOG, OP_MAX, OP_CNDS, OP_MOV, OP_PKMOV, OP_PKADD, OP_CMPX, OP_EXP3FMA, OP_EXPMIX, OP_EXPCVT, OP_EXPRCP2FMA, OP_NONE };
static const char* kNames[] = {"v_fma_f32", "v_mul_f32", "v_exp_f32", "v_rcp_f32", "v_sqrt_f32", "v_fma_mixlo_f16",
                               "v_cvt_pk_f16_f32", "v_max3_f32", "v_cndmask_b32", "v_pk_fma_f32", "v_cvt_f32_f16", "v_cvt_f32_f16 sdwa", "v_and_b32", "v_pk_mul_f32", "v_ldexp_f32", "v_log_f32", "v_max_f32", "v_cndmask s[]", "v_mov_b32", "v_pk_mov_b32", "v_pk_add_f32", "v_cmpx(all true)", "exp+3fma (/4)", "exp+mix (/2)", "exp+cvt_pk (/2)", "exp,rcp+2fma (/4)", "none"};

typedef float floatx2 __attribute__((ext_vector_type(2)));
template <int OP>
__device__ __forceinline__ void op1(float& a, float b, float c);
template <int OP>
__device__ __forceinline__ void op1(float& a, float b, float c) {
  if constexpr (OP == OP_FMA) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a) : "v"(b), "v"(c));
  if constexpr (OP == OP_MUL) asm volatile("v_mul_f32 %0, %1, %0" : "+v"(a) : "v"(b));
  if constexpr (OP == OP_EXP) asm volatile("v_exp_f32 %0, %0" : "+v"(a));
  if constexpr (OP == OP_RCP) asm volatile("v_rcp_f32 %0, %0" : "+v"(a));
  if constexpr (OP == OP_SQRT) asm volatile("v_sqrt_f32 %0, %0" : "+v"(a));
  if constexpr (OP == OP_MIX) asm volatile("v_fma_mixlo_f16 %0, %1, %2, -%0 op_sel_hi:[0,0,1]" : "+v"(a) : "v"(b), "v"(c));
  if constexpr (OP == OP_CVTPK) asm volatile("v_cvt_pk_f16_f32 %0, %1, %0" : "+v"(a) : "v"(b));
  if constexpr (OP == OP_MAX3) asm volatile("v_max3_f32 %0, %1, %2, %0" : "+v"(a) : "v"(b), "v"(c));
  if constexpr (OP == OP_CND) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a) : "v"(b));
  if constexpr (OP == OP_CVTF16) asm volatile("v_cvt_f32_f16 %0, %0" : "+v"(a));
  if constexpr (OP == OP_CVTF16HI) asm volatile("v_cvt_f32_f16_sdwa %0, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1" : "+v"(a));
  if constexpr (OP == OP_AND) asm volatile("v_and_b32 %0, %1, %0" : "+v"(a) : "v"(b));
  if constexpr (OP == OP_LDEXP) asm volatile("v_ldexp_f32 %0, %0, %1" : "+v"(a) : "v"(b));
  if constexpr (OP == OP_LOG) asm volatile("v_log_f32 %0, %0" : "+v"(a));
  if constexpr (OP == OP_MAX) asm volatile("v_max_f32 %0, %1, %0" : "+v"(a) : "v"(b));
  if constexpr (OP == OP_MOV) asm volatile("v_mov_b32 %0, %1" : "=v"(a) : "v"(b));
  if constexpr (OP == OP_PKMOV) {
    floatx2 x2 = {a, b};
    asm volatile("v_pk_mov_b32 %0, %0, %0 op_sel:[1,0]" : "+v"(x2));
    a = x2[0];
  }
  if constexpr (OP == OP_PKADD) {
    floatx2 x2 = {a, b};
    asm volatile("v_pk_add_f32 %0, %0, %0" : "+v"(x2));
    a = x2[0];
  }
  if constexpr (OP == OP_CMPX) asm volatile("v_cmpx_le_f32 vcc, %0, %1" : : "v"(b), "v"(a) : "vcc");  // b <= a: exec stays
  if constexpr (OP == OP_PKFMA) {
    floatx2 x2 = {a, b};
    asm volatile("v_pk_fma_f32 %0, %0, %0, %0" : "+v"(x2));
    a = x2[0];
  }
  if constexpr (OP == OP_EXP3FMA)
  {
    float t1, t2, t3;  // independent fmas beside the exp chain
    asm volatile("v_exp_f32 %0, %0\n\tv_fma_f32 %1, %4, %4, %4\n\tv_fma_f32 %2, %4, %4, %4\n\tv_fma_f32 %3, %4, %4, %4"
                 : "+v"(a), "=&v"(t1), "=&v"(t2), "=&v"(t3) : "v"(c));
  }
  if constexpr (OP == OP_EXPMIX)
  {
    float t1;
    asm volatile("v_exp_f32 %0, %0\n\tv_fma_mixlo_f16 %1, %2, 1.0, -%2 op_sel_hi:[0,0,1]" : "+v"(a), "=&v"(t1) : "v"(c));
  }
  if constexpr (OP == OP_EXPCVT) {
    float t1;
    asm volatile("v_exp_f32 %0, %0\n\tv_cvt_pk_f16_f32 %1, %2, %2" : "+v"(a), "=&v"(t1) : "v"(c));
  }
  if constexpr (OP == OP_EXPRCP2FMA)
  {
    float t1, t2;
    asm volatile("v_exp_f32 %0, %0\n\tv_fma_f32 %1, %3, %3, %3\n\tv_rcp_f32 %0, %0\n\tv_fma_f32 %2, %3, %3, %3"
                 : "+v"(a), "=&v"(t1), "=&v"(t2) : "v"(c));
  }
  if constexpr (OP == OP_CNDS) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[40:41]" : "+v"(a) : "v"(b) : "s40", "s41");
}

// MODE 0: every wave issues ITERS x 128 filler instructions (16 chains).
// MODE 1: wave w of SIMD (w < 1... ) — wave 0 of each SIMD issues MFMAs with F
//         fillers each, the others idle.
// MODE 2: wave 0 of each SIMD issues MFMAs with F fillers each, the others
//         issue the filler stream only (F * MFMA count each).
template <int OP, int MODE, int F>
__global__ __launch_bounds__(1024, 1) void probe(unsigned long long* out, int iters, float seed) {
  extern __shared__ char pin[];
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  if (seed > 1e30f) pin[threadIdx.x] = 0;  // keep the LDS allocation
  float a[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) a[i] = 1.0f + 1e-3f * (lane + i) + seed;
  const float b = 0.999f + seed, c = 1e-4f;
  const bool mfma_wave = (MODE == 3) || ((MODE != 0) && (wave < 4));
  if (MODE == 4 && mfma_wave) __builtin_amdgcn_s_setprio(3);  // waves 0-3 land on the 4 SIMDs
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (MODE == 0) {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < 8; ++k)
#pragma unroll
        for (int i = 0; i < 16; ++i) op1<OP>(a[i], b, c);
    }
  } else if (mfma_wave) {
    halfx8 x, y;
#pragma unroll
    for (int i = 0; i < 8; ++i) { x[i] = (_Float16)(0.01f * (lane + i)); y[i] = (_Float16)(0.02f * (lane - i)); }
    floatx16 acc0 = {0}, acc1 = {0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(x, y, acc0, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < F; ++i) op1<OP>(a[i], b, c);
        __builtin_amdgcn_sched_barrier(0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(x, y, acc1, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < F; ++i) op1<OP>(a[8 + i], b, c);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) a[r] += acc0[r] + acc1[r];
  } else if (MODE == 2 || MODE == 4) {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < 8; ++k)
#pragma unroll
        for (int i = 0; i < 2 * F; ++i) op1<OP>(a[i], b, c);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += a[i];
  if (lane == 0) out[blockIdx.x * 16 + wave] = (t1 - t0) | (s == 12345.f ? 1ull : 0ull);
}

template <int OP, int MODE, int F>
double run(int nw, unsigned long long* d, unsigned long long* h, int iters) {
  const int threads = 256 * nw;
  const size_t lds = 100 * 1024;  // one block per CU
  hipLaunchKernelGGL((probe<OP, MODE, F>), dim3(256), dim3(threads), lds, 0, d, iters, 0.f);
  hipLaunchKernelGGL((probe<OP, MODE, F>), dim3(256), dim3(threads), lds, 0, d, iters, 0.f);
  hipDeviceSynchronize();
  hipMemcpy(h, d, 256 * 16 * 8, hipMemcpyDeviceToHost);
  unsigned long long mx = 0;
  for (int i = 0; i < 256; ++i)
    for (int w = 0; w < 4 * nw; ++w) mx = h[i * 16 + w] > mx ? h[i * 16 + w] : mx;
  return (double)mx;
}

template <int OP>
void row(unsigned long long* d, unsigned long long* h) {
  const int it = 400;
  printf("%-18s", kNames[OP]);
  for (int nw = 1; nw <= 4; ++nw) {  // cycles per instruction per SIMD
    const double t = run<OP, 0, 4>(nw, d, h, it);
    printf("  nw%d %5.2f", nw, t / (double(nw) * it * 128));
  }
  // MFMA stream with F fillers (16 MFMA per iteration); cycles per MFMA
  const double m0 = run<OP_NONE, 1, 0>(1, d, h, it) / (it * 16.0);
  const double m4 = run<OP, 1, 4>(1, d, h, it) / (it * 16.0);
  const double m8 = run<OP, 1, 8>(1, d, h, it) / (it * 16.0);
  const double m4x3 = run<OP, 1, 4>(3, d, h, it) / (it * 16.0);
  const double c4x3 = run<OP, 2, 4>(3, d, h, it) / (it * 16.0);
  const double a3 = run<OP, 3, 4>(3, d, h, it) / (it * 16.0 * 3);
  const double a3_0 = run<OP_NONE, 3, 0>(3, d, h, it) / (it * 16.0 * 3);
  const double p4x3 = run<OP, 4, 4>(3, d, h, it) / (it * 16.0);
  printf("  | mfma %.1f +4in %.1f +8in %.1f (1w) +4in,3w-idle %.1f +4in,2w x8 cross %.1f prio %.1f | 3w all mfma %.1f +4in %.1f\n", m0, m4, m8, m4x3, c4x3, p4x3, a3_0, a3);
}

int main() {
  unsigned long long *d, *h;
  hipMalloc(&d, 256 * 16 * 8);
  h = (unsigned long long*)malloc(256 * 16 * 8);
  row<OP_FMA>(d, h);
  row<OP_EXP>(d, h);
  row<OP_EXP3FMA>(d, h);
  row<OP_EXPRCP2FMA>(d, h);
  row<OP_EXPMIX>(d, h);
  row<OP_EXPCVT>(d, h);
  row<OP_CND>(d, h);
  row<OP_CNDS>(d, h);
  row<OP_MOV>(d, h);
  row<OP_PKMOV>(d, h);
  row<OP_PKADD>(d, h);
  row<OP_PKFMA>(d, h);
  row<OP_CMPX>(d, h);
  row<OP_CVTPK>(d, h);
  row<OP_AND>(d, h);
  return 0;
}
