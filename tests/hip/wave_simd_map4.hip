// Probe (GPU box): SIMD placement of the waves of 256-thread blocks at the
// split-MFMA kernel's footprint (34 KiB LDS, 3 blocks per CU, 8192 blocks):
// how many blocks have exactly one wave per SIMD.  HW_ID bits [5:4] = SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(256, 3) void probe(unsigned* out) {
  extern __shared__ char lds[];
  lds[threadIdx.x] = 0;
  if ((threadIdx.x & 63) == 0) {
    unsigned id = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));
    out[blockIdx.x * 4 + (threadIdx.x >> 6)] = id;
  }
  // some work so blocks overlap in time
  float a = threadIdx.x;
  for (int i = 0; i < 20000; ++i) a = a * 0.999f + 0.5f;
  if (a == 1.2345f) out[0] = 0;
}
int main() {
  unsigned* d;
  const int blocks = 8192;
  hipMalloc(&d, blocks * 4 * 4);
  hipLaunchKernelGGL(probe, dim3(blocks), dim3(256), 34 * 1024, 0, d);
  static unsigned h[blocks * 4];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int good = 0, hist[5] = {0};
  for (int b = 0; b < blocks; ++b) {
    int cnt[4] = {0};
    for (int w = 0; w < 4; ++w) cnt[(h[b * 4 + w] >> 4) & 3]++;
    bool ok = cnt[0] == 1 && cnt[1] == 1 && cnt[2] == 1 && cnt[3] == 1;
    good += ok;
    hist[cnt[3]]++;
  }
  printf("blocks with one wave per SIMD: %d of %d; waves on SIMD 3 per block: 0:%d 1:%d 2:%d 3:%d 4:%d\n", good, blocks,
         hist[0], hist[1], hist[2], hist[3], hist[4]);
  for (int b = 0; b < 6; ++b) {
    printf("block %d:", b);
    for (int w = 0; w < 4; ++w) printf(" w%d->simd%u", w, (h[b * 4 + w] >> 4) & 3);
    printf("\n");
  }
  return 0;
}
