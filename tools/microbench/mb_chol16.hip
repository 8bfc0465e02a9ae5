// Cycles of the 16×16 diagonal-tile factor (chol16_factor, omb_linalg.hip) in one wave, alone on a CU, for the
// variants of its column update (tools only).  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/microbench/mb_chol16 tools/microbench/mb_chol16.hip
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../optimobo_amd/csrc/omb_linalg.hip"
#include "../../optimobo_amd/csrc/omb_wide.hip"
#include "../../optimobo_amd/csrc/omb_gemm.hip"

using namespace omb;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)

// Round 4 measured VAR 0 (the compiler's v_mov_b64_dpp + 2 fma, kept in omb_linalg.hip) against an inline-asm
// v_fmac_f64_dpp form (3,188 vs 3,784 cycles, profiles/r04_f_mb_chol16.txt); the asm form was removed from the library.
template <int VAR>
__global__ __launch_bounds__(64) void f16_kernel(const double* __restrict__ D, double* __restrict__ out, int reps,
                                                 unsigned long long* cyc) {
  const int c = threadIdx.x & 15;
  double a[16], x[16];
  for (int q = 0; q < 16; ++q) a[q] = D[c * 16 + q];
  unsigned long long t0 = 0, t1 = 0;
  int bad = 0;
  for (int r = 0; r < reps; ++r) {
#pragma unroll
    for (int q = 0; q < 16; ++q) x[q] = (q == c) ? 1.0 : 0.0;
    double b[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) b[q] = a[q];
    __builtin_amdgcn_s_waitcnt(0);
    if (r == reps - 1) t0 = __builtin_readcyclecounter();
    bad += chol16_factor(b, x);
#pragma unroll
    for (int q = 0; q < 16; ++q) asm volatile("" : "+v"(b[q]), "+v"(x[q]));
    if (r == reps - 1) t1 = __builtin_readcyclecounter();
    if (r == reps - 1)
      for (int q = 0; q < 16; ++q) {
        out[c * 16 + q] = b[q];
        out[256 + q * 16 + c] = x[q];
      }
  }
  if (threadIdx.x == 0) {
    cyc[0] = t1 - t0;
    cyc[1] = bad;
  }
}

int main() {
  const int n = 16;
  std::vector<double> h(n * n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) h[i * n + j] = (i == j) ? n : 1.0 / (1.0 + std::abs((double)(i - j)));
  double *D, *out;
  unsigned long long* cyc;
  CK(hipMalloc(&D, n * n * 8));
  CK(hipMalloc(&out, 2 * n * n * 8));
  CK(hipMalloc(&cyc, 16));
  CK(hipMemcpy(D, h.data(), n * n * 8, hipMemcpyHostToDevice));
  const char* names[1] = {"chol16_factor (DPP mov + 2 fma)"};
  for (int rep = 0; rep < 2; ++rep)
    for (int v = 0; v < 1; ++v) {
      hipLaunchKernelGGL(f16_kernel<0>, dim3(1), dim3(64), 0, 0, D, out, 20, cyc);
      CK(hipDeviceSynchronize());
      unsigned long long c[2];
      CK(hipMemcpy(c, cyc, 16, hipMemcpyDeviceToHost));
      std::vector<double> o(2 * n * n);
      CK(hipMemcpy(o.data(), out, o.size() * 8, hipMemcpyDeviceToHost));
      // residual of L·Lᵀ = D and L·W = I
      double e1 = 0, e2 = 0;
      for (int i = 0; i < n; ++i)
        for (int j = 0; j <= i; ++j) {
          double s = 0, w = 0;
          for (int k = 0; k <= j; ++k) s += o[i * n + k] * o[j * n + k];
          for (int k = j; k <= i; ++k) w += o[i * n + k] * o[n * n + k * n + j];
          e1 = std::max(e1, std::abs(s - h[i * n + j]));
          e2 = std::max(e2, std::abs(w - (i == j ? 1.0 : 0.0)));
        }
      if (rep == 1)
        printf("%-30s %6llu cycles per 16x16 factor + inverse (%.0f per column)  |LLt-D| %.1e  |LW-I| %.1e  bad %llu\n",
               names[v], c[0], c[0] / 16.0, e1, e2, c[1]);
    }
  return 0;
}
