// Layout check for the bf16x3 conditioner GEMM (run on the GPU box):
// Y^T (32 out x 32 samples) = W^T . X^T with X^T an f32 accumulator tile of a
// previous MFMA (rows in registers, sample on the lane), computed two ways:
// (a) v_mfma_f32_32x32x2_f32 (reference), (b) 6 x v_mfma_f32_32x32x16_bf16
// with hi/mid/lo splits, X converted in-register (accumulator-as-operand).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ inline void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)x;
  const float r = x - (float)h;
  m = (__bf16)r;
  l = (__bf16)(r - (float)m);
}

// W: [32 in][32 out] row-major f32; Xin: [32 rows][32 samples]; out f32/bf16 Y: [32 out][32 samples]
__global__ void k(const float* W, const float* X, float* Yf, float* Yb) {
  const int lane = threadIdx.x, h = lane >> 5, c = lane & 31;
  // accumulator-layout tile of X: reg r -> row (r&3) + 8(r>>2) + 4h, col c
  floatx16 xt;
  for (int r = 0; r < 16; ++r) xt[r] = X[((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + c];
  // (a) f32 path: A frag for reg r: W^T[i=c][k=row(r,h)]
  floatx16 acc = {0};
  for (int r = 0; r < 16; ++r) {
    const int kk = (r & 3) + 8 * (r >> 2) + 4 * h;
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(W[kk * 32 + c], xt[r], acc, 0, 0, 0);
  }
  // (b) bf16x3 path: k-step s uses regs 8s..8s+7; element j <-> row 16s + 8(j>>2) + 4h + (j&3)
  floatx16 acc2 = {0};
  for (int s = 0; s < 2; ++s) {
    bf16x8 bh, bm, bl, ah, am, al;
    for (int j = 0; j < 8; ++j) {
      __bf16 a, b, d;
      split3(xt[8 * s + j], a, b, d);
      bh[j] = a; bm[j] = b; bl[j] = d;
      const int kk = 16 * s + 8 * (j >> 2) + 4 * h + (j & 3);
      split3(W[kk * 32 + c], a, b, d);
      ah[j] = a; am[j] = b; al[j] = d;
    }
    acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, acc2, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc2, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc2, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, acc2, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, acc2, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc2, 0, 0, 0);
  }
  for (int r = 0; r < 16; ++r) {
    const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
    Yf[row * 32 + c] = acc[r];
    Yb[row * 32 + c] = acc2[r];
  }
}

int main() {
  std::vector<float> W(1024), X(1024), Yf(1024), Yb(1024);
  srand(1);
  for (auto& v : W) v = (rand() / (float)RAND_MAX - 0.5f) * 0.3f;
  for (auto& v : X) v = (rand() / (float)RAND_MAX - 0.5f) * 3.f;
  float *dW, *dX, *dYf, *dYb;
  hipMalloc(&dW, 4096); hipMalloc(&dX, 4096); hipMalloc(&dYf, 4096); hipMalloc(&dYb, 4096);
  hipMemcpy(dW, W.data(), 4096, hipMemcpyHostToDevice);
  hipMemcpy(dX, X.data(), 4096, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dW, dX, dYf, dYb);
  hipMemcpy(Yf.data(), dYf, 4096, hipMemcpyDeviceToHost);
  hipMemcpy(Yb.data(), dYb, 4096, hipMemcpyDeviceToHost);
  double emf = 0, emb = 0, scale = 0;
  for (int o = 0; o < 32; ++o)
    for (int s = 0; s < 32; ++s) {
      double ref = 0, mag = 0;
      for (int i = 0; i < 32; ++i) { ref += (double)W[i * 32 + o] * X[i * 32 + s]; mag += fabs((double)W[i * 32 + o] * X[i * 32 + s]); }
      emf = fmax(emf, fabs(Yf[o * 32 + s] - ref) / mag);
      emb = fmax(emb, fabs(Yb[o * 32 + s] - ref) / mag);
    }
  printf("f32 mfma max rel err %.3g | bf16x3 max rel err %.3g\n", emf, emb);
  return (emf < 1e-6 && emb < 1e-6) ? 0 : 1;
}
