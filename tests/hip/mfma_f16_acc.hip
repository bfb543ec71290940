// Probe (GPU box, tuning only): how exactly does v_mfma_f32_32x32x16_f16 sum
// its 16 fp16 x fp16 products into the fp32 accumulator?  Compares the MFMA
// result with the exact sum (fp64 on the host) on random operands with a
// spread of exponents, C = 0 and C = random fp32, and reports the error in
// ulps of the correctly rounded result and relative to sum |a b| + |c|.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));

// A: [32 rows][16 k] , B: [16 k][32 cols], C/D: [32][32]; element j of lane
// (r + 32h) <-> k = 8h + j for both operands (any consistent map sums the
// same 16 products).  Accumulator register q of lane (c + 32h) <-> row
// (q & 3) + 8 (q >> 2) + 4h.
__global__ void k(const _Float16* A, const _Float16* B, const float* Cm, float* D, int chain) {
  const int lane = threadIdx.x, h = lane >> 5, c = lane & 31;
  halfx8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = A[c * 16 + 8 * h + j];
    b[j] = B[(8 * h + j) * 32 + c];
  }
  floatx16 acc;
  for (int q = 0; q < 16; ++q) acc[q] = Cm[((q & 3) + 8 * (q >> 2) + 4 * h) * 32 + c];
  for (int i = 0; i < chain; ++i) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
  for (int q = 0; q < 16; ++q) D[((q & 3) + 8 * (q >> 2) + 4 * h) * 32 + c] = acc[q];
}

int main() {
  std::mt19937 g(7);
  std::normal_distribution<double> nd(0, 1);
  std::uniform_real_distribution<double> ud(-12, 4);
  _Float16 *dA, *dB;
  float *dC, *dD;
  (void)hipMalloc(&dA, 32 * 16 * 2);
  (void)hipMalloc(&dB, 16 * 32 * 2);
  (void)hipMalloc(&dC, 32 * 32 * 4);
  (void)hipMalloc(&dD, 32 * 32 * 4);
  const char* names[] = {"C=0, unit-scale", "C=0, exponent spread", "C=random, spread", "cancel (C=-sum)",
                         "C=0 spread, 8-deep chain"};
  for (int mode = 0; mode < 5; ++mode) {
    double max_ulp = 0, max_rel = 0, sum_ulp = 0;
    long n = 0;
    for (int trial = 0; trial < 200; ++trial) {
      std::vector<_Float16> A(32 * 16), B(16 * 32);
      std::vector<float> C(32 * 32, 0.f), Dh(32 * 32);
      for (auto& v : A) v = (_Float16)(nd(g) * (mode == 0 ? 1.0 : std::exp2(ud(g))));
      for (auto& v : B) v = (_Float16)(nd(g) * (mode == 0 ? 1.0 : std::exp2(ud(g))));
      std::vector<double> ex(32 * 32), mag(32 * 32);
      for (int r = 0; r < 32; ++r)
        for (int cc = 0; cc < 32; ++cc) {
          double s = 0, m = 0;
          for (int kk = 0; kk < 16; ++kk) {
            const double p = (double)A[r * 16 + kk] * (double)B[kk * 32 + cc];
            s += p;  // exact: 22-bit products, 16 terms, exponents within fp64 range
            m += std::fabs(p);
          }
          if (mode == 2) C[r * 32 + cc] = (float)(nd(g) * std::exp2(ud(g)));
          if (mode == 3) C[r * 32 + cc] = -(float)s;
          ex[r * 32 + cc] = s;
          mag[r * 32 + cc] = m;
        }
      const int chain = mode == 4 ? 8 : 1;
      (void)hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
      (void)hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
      (void)hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice);
      hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD, chain);
      (void)hipMemcpy(Dh.data(), dD, Dh.size() * 4, hipMemcpyDeviceToHost);
      for (int i = 0; i < 32 * 32; ++i) {
        double exact;
        if (chain == 1) {
          exact = ex[i] + (double)C[i];
        } else {  // reference: fp32 rounding after each MFMA's exact sum
          float accf = C[i];
          for (int t = 0; t < chain; ++t) accf = (float)((double)accf + ex[i]);
          exact = accf;
        }
        const float cr = (float)exact;
        const double ulp = std::ldexp(1.0, std::ilogb(cr == 0.f ? 1e-30f : cr) - 23);
        const double e = std::fabs((double)Dh[i] - exact);
        max_ulp = std::max(max_ulp, e / ulp);
        sum_ulp += e / ulp;
        max_rel = std::max(max_rel, e / (mag[i] * chain + std::fabs((double)C[i]) + 1e-300));
        ++n;
      }
    }
    printf("%-28s max err %8.2f ulp of result, mean %6.3f ulp, max err / (sum|ab|+|c|) %.3e\n", names[mode],
           max_ulp, sum_ulp / n, max_rel);
  }
  return 0;
}
