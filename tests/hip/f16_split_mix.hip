// Probe (run on the GPU box): the f16x2 split via v_cvt_pk_f16_f32 + v_fma_mix{lo,hi}_f16
// (lo = f16(x - f32(hi)) in one instruction) must equal the host RNE split bit for bit.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef _Float16 halfx2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split2(float x0, float x1, uint32_t& h, uint32_t& l) {
  const halfx2 hv = __builtin_convertvector(floatx2{x0, x1}, halfx2);
  __builtin_memcpy(&h, &hv, 4);
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(l) : "v"(x0), "v"(h));
  asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(l) : "v"(x1), "v"(h));
}
__global__ void k(const float* x, uint32_t* h, uint32_t* l, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 < n) split2(x[2 * i], x[2 * i + 1], h[i], l[i]);
}
int main() {
  const int n = 1 << 20;
  float* hx = (float*)malloc(n * 4);
  uint32_t s = 12345;
  for (int i = 0; i < n; ++i) { s = s * 1664525u + 1013904223u; int e = (s >> 24) % 28; s = s * 1664525u + 1013904223u;
    hx[i] = ((s >> 8) * (1.0f / 16777216.0f) - 0.5f) * ldexpf(1.f, e - 13); }
  float* dx; uint32_t *dh, *dl;
  hipMalloc(&dx, n * 4); hipMalloc(&dh, n * 2); hipMalloc(&dl, n * 2);
  hipMemcpy(dx, hx, n * 4, hipMemcpyHostToDevice);
  k<<<n / 2 / 256, 256>>>(dx, dh, dl, n);
  uint16_t* hh = (uint16_t*)malloc(n * 2); uint16_t* hl = (uint16_t*)malloc(n * 2);
  hipMemcpy(hh, dh, n * 2, hipMemcpyDeviceToHost); hipMemcpy(hl, dl, n * 2, hipMemcpyDeviceToHost);
  long bad = 0; double maxrel = 0;
  for (int i = 0; i < n; ++i) {
    _Float16 a, b; memcpy(&a, &hh[i], 2); memcpy(&b, &hl[i], 2);
    _Float16 ea = (_Float16)hx[i]; _Float16 eb = (_Float16)(hx[i] - (float)ea);
    if (memcmp(&a, &ea, 2) || memcmp(&b, &eb, 2)) ++bad;
    double rel = fabs((double)(float)a + (double)(float)b - hx[i]) / fabs(hx[i]);
    if (hx[i] != 0 && rel > maxrel) maxrel = rel;
  }
  printf("fma_mix split: %ld mismatches vs host RNE split of %d, max rel err %.3g (2^-22 = %.3g)\n", bad, n, maxrel, ldexp(1, -22));
  return bad != 0;
}
