// Probe (run on the GPU box): which SIMD each wave of a 512-thread block
// with a large LDS footprint (one block per CU) lands on.  HW_ID bits [5:4].
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(512, 1) void probe(unsigned* out) {
  extern __shared__ char lds[];
  lds[threadIdx.x] = 0;
  if ((threadIdx.x & 63) == 0) {
    unsigned id = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));
    out[blockIdx.x * 8 + (threadIdx.x >> 6)] = id;
  }
}
int main() {
  unsigned* d;
  const int blocks = 64;
  hipMalloc(&d, blocks * 8 * 4);
  hipLaunchKernelGGL(probe, dim3(blocks), dim3(512), 150 * 1024, 0, d);
  unsigned h[blocks * 8];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int b = 0; b < 8; ++b) {
    printf("block %d:", b);
    for (int w = 0; w < 8; ++w) {
      unsigned v = h[b * 8 + w];
      printf(" w%d->simd%u(cu%u,slot%u)", w, (v >> 4) & 3, (v >> 8) & 15, v & 15);
    }
    printf("\n");
  }
  return 0;
}
