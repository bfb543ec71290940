// Probe (GPU box, tuning only): how VALU, transcendental and MFMA issue of
// one or more waves share a SIMD.  One block per CU (large LDS), waves w,
// w+4, w+8 on one SIMD; each wave runs a role for `iters` iterations and
// records its s_memtime cycles.  Per iteration:
//   M : 16 v_mfma_f32_32x32x16_f16 (4 independent accumulators) = 512 matrix cycles
//   V : 128 independent-chain v_fma_f32 (one wave alone: 512 issue cycles)
//   T : 64 transcendentals (v_exp / v_rcp alternating)
//   Fk: 16 MFMAs, each followed by k v_fma_f32 (in-wave fillers)
//   S : 16 MFMAs, each followed by a swish-like filler (exp, fma, rcp, mul)
//   I : idle (exits at once)
// usage: issue_probe [iters]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));

enum Role { R_I = 0, R_M, R_V, R_T, R_F2, R_F4, R_F6, R_F8, R_S, R_S2 };

#define MF(acc) asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b))
#define FMA(x) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(c1), "v"(c2))
#define EXP(x) asm volatile("v_exp_f32 %0, %0" : "+v"(x))
#define RCP(x) asm volatile("v_rcp_f32 %0, %0" : "+v"(x))
#define MUL(x, y) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x) : "v"(y))

__device__ __forceinline__ void run_role(int role, int iters, float& sink, int lane) {
  halfx8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (_Float16)(0.001f * (lane + i)); b[i] = (_Float16)(0.002f * (lane - i)); }
  floatx16 acc0 = {0}, acc1 = {0}, acc2 = {0}, acc3 = {0};
  float v[16];
  for (int i = 0; i < 16; ++i) v[i] = 0.001f * (lane + i);
  const float c1 = 0.999f, c2 = 0.0001f;
  if (role == R_M) {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < 4; ++k) { MF(acc0); MF(acc1); MF(acc2); MF(acc3); }
    }
  } else if (role == R_V) {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
#pragma unroll
        for (int i = 0; i < 16; ++i) FMA(v[i]);
      }
    }
  } else if (role == R_T) {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
#pragma unroll
        for (int i = 0; i < 16; ++i) { if (i & 1) RCP(v[i]); else EXP(v[i]); }
      }
    }
  } else if (role >= R_F2 && role <= R_F8) {
    const int kf = 2 * (role - R_F2 + 1);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
#define FILL(base) \
  if (kf >= 2) { FMA(v[(base) + 0]); FMA(v[(base) + 1]); } \
  if (kf >= 4) { FMA(v[(base) + 2]); FMA(v[(base) + 3]); } \
  if (kf >= 6) { FMA(v[(base) + 4]); FMA(v[(base) + 5]); } \
  if (kf >= 8) { FMA(v[(base) + 6]); FMA(v[(base) + 7]); }
        MF(acc0); FILL(0); MF(acc1); FILL(8); MF(acc2); FILL(0); MF(acc3); FILL(8);
#undef FILL
      }
    }
  } else if (role == R_S || role == R_S2) {
    // swish-like filler per MFMA: exp, fma, rcp, mul (24 issue cycles for one wave);
    // R_S2: two of them per MFMA (48)
    const int reps = role == R_S ? 1 : 2;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
#define SW(x, y) { EXP(x); FMA(x); RCP(x); MUL(x, y); }
        MF(acc0); SW(v[0], v[1]); if (reps > 1) SW(v[2], v[3]);
        MF(acc1); SW(v[4], v[5]); if (reps > 1) SW(v[6], v[7]);
        MF(acc2); SW(v[8], v[9]); if (reps > 1) SW(v[10], v[11]);
        MF(acc3); SW(v[12], v[13]); if (reps > 1) SW(v[14], v[15]);
#undef SW
      }
    }
  }
  for (int r = 0; r < 16; ++r) sink += acc0[r] + acc1[r] + acc2[r] + acc3[r];
  for (int i = 0; i < 16; ++i) sink += v[i];
}

struct Roles { int r[12]; };

__global__ __launch_bounds__(768, 1) void probe(Roles roles, int iters, float* out, unsigned long long* cyc,
                                                unsigned* hwid) {
  extern __shared__ char lds[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (threadIdx.x == 0) lds[0] = 0;
  __syncthreads();
  const int role = roles.r[w];
  float sink = 0.f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  run_role(role, iters, sink, lane);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = sink;
  if (lane == 0) {
    cyc[blockIdx.x * 12 + w] = t1 - t0;
    hwid[blockIdx.x * 12 + w] = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));
  }
}

static const char* rname(int r) {
  static const char* n[] = {"I", "M", "V", "T", "F2", "F4", "F6", "F8", "S", "S2"};
  return n[r];
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 400;
  const int blocks = 256;
  float* d_out;
  unsigned long long* d_cyc;
  unsigned* d_hw;
  (void)hipMalloc(&d_out, blocks * 768 * 4);
  (void)hipMalloc(&d_cyc, blocks * 12 * 8);
  (void)hipMalloc(&d_hw, blocks * 12 * 4);
  // configs: per SIMD slot list (slot 0 = waves 0-3, slot 1 = 4-7, slot 2 = 8-11)
  struct Cfg { const char* name; int s[3]; };
  const Cfg cfgs[] = {
      {"M", {R_M, -1, -1}},           {"V", {R_V, -1, -1}},           {"T", {R_T, -1, -1}},
      {"V+V", {R_V, R_V, -1}},        {"V+V+V", {R_V, R_V, R_V}},     {"T+T", {R_T, R_T, -1}},
      {"M+M", {R_M, R_M, -1}},        {"M+V", {R_M, R_V, -1}},        {"V+M", {R_V, R_M, -1}},
      {"M+T", {R_M, R_T, -1}},        {"M+V+V", {R_M, R_V, R_V}},     {"F2", {R_F2, -1, -1}},
      {"F4", {R_F4, -1, -1}},         {"F6", {R_F6, -1, -1}},         {"F8", {R_F8, -1, -1}},
      {"S", {R_S, -1, -1}},           {"S2", {R_S2, -1, -1}},         {"F4+F4", {R_F4, R_F4, -1}},
      {"S+S", {R_S, R_S, -1}},        {"M+S", {R_M, R_S, -1}},        {"F4+V", {R_F4, R_V, -1}},
      {"S+T", {R_S, R_T, -1}},        {"S+S+S", {R_S, R_S, R_S}},     {"F6+F6", {R_F6, R_F6, -1}},
  };
  for (const Cfg& c : cfgs) {
    int nw = 0;
    Roles roles;
    for (int s = 0; s < 3; ++s)
      if (c.s[s] >= 0) nw = 4 * (s + 1);
    for (int w = 0; w < 12; ++w) roles.r[w] = (w < nw && c.s[w / 4] >= 0) ? c.s[w / 4] : R_I;
    hipLaunchKernelGGL(probe, dim3(blocks), dim3(nw * 64), 150 * 1024, 0, roles, iters, d_out, d_cyc, d_hw);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 3; ++r)
      hipLaunchKernelGGL(probe, dim3(blocks), dim3(nw * 64), 150 * 1024, 0, roles, iters, d_out, d_cyc, d_hw);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> cyc(blocks * 12);
    std::vector<unsigned> hw(blocks * 12);
    (void)hipMemcpy(cyc.data(), d_cyc, cyc.size() * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hw.data(), d_hw, hw.size() * 4, hipMemcpyDeviceToHost);
    // median over blocks of each slot's wave-0 cycles per iteration
    printf("%-7s wall %.3f ms |", c.name, ms / 3);
    for (int s = 0; s < 3; ++s) {
      if (c.s[s] < 0) continue;
      std::vector<double> v;
      for (int b = 0; b < blocks; ++b)
        for (int q = 0; q < 4; ++q) v.push_back((double)cyc[b * 12 + s * 4 + q] / iters);
      std::sort(v.begin(), v.end());
      printf(" slot%d %-3s %7.1f cyc/it", s, rname(c.s[s]), v[v.size() / 2]);
    }
    // SIMD check: waves w and w+4 of block 0 on one SIMD
    int same = 1;
    for (int w = 0; w + 4 < nw; ++w) same &= ((hw[w] >> 4) & 3) == ((hw[w + 4] >> 4) & 3);
    printf(" | pairs-same-simd %d\n", same);
  }
  return 0;
}
