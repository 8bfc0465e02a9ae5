// Dependent-issue latency of the ops on the Cholesky pivot chain (gfx950, one wave per SIMD, s_memtime
// cycles): v_fma_f64 chains, v_rsq_f64 chains, v_readlane → VALU round trips, and the pivot-step
// pattern (rsq + two Newton steps + mul + fma) — per dependent op, averaged over long chains.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/microbench/mb_latency tools/microbench/mb_latency.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)

constexpr int kIters = 4096;

__device__ __forceinline__ double readlane_f64(double v, int l) {
  const long long b = __builtin_bit_cast(long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(b & 0xffffffffll), l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(b >> 32), l);
  return __builtin_bit_cast(double, (long long)(((unsigned long long)hi << 32) | lo));
}

template <int MODE>
__global__ void kern(double* out, unsigned long long* cyc, double seed) {
  double x = seed + 1e-9 * threadIdx.x;
  const double c = 0.999999, d = 1e-7;
  const unsigned long long t0 = __builtin_readcyclecounter();
#pragma unroll 16
  for (int i = 0; i < kIters; ++i) {
    if constexpr (MODE == 0) {                 // 1 dependent fma
      x = fma(x, c, d);
    } else if constexpr (MODE == 1) {          // 1 dependent rsq (+ fma to keep it bounded)
      x = __builtin_amdgcn_rsq(x);
    } else if constexpr (MODE == 2) {          // readlane → fma (scalar operand) round trip
      x = fma(readlane_f64(x, 5), c, d);
    } else if constexpr (MODE == 3) {          // the pivot step: rsq + 2 Newton + mul + fma (9 dependent ops)
      const double y0 = __builtin_amdgcn_rsq(x);
      const double hd = 0.5 * x;
      const double y1 = fma(y0, fma(-hd * y0, y0, 0.5), y0);
      const double inv = fma(y1, fma(-hd * y1, y1, 0.5), y1);
      const double s = 0.3 * inv;
      x = fma(-s, s, 1.0 + 1e-3 * x);
    } else if constexpr (MODE == 4) {          // pivot step with one Newton step (6 dependent ops)
      const double y0 = __builtin_amdgcn_rsq(x);
      const double hd = 0.5 * x;
      const double inv = fma(y0, fma(-hd * y0, y0, 0.5), y0);
      const double s = 0.3 * inv;
      x = fma(-s, s, 1.0 + 1e-3 * x);
    } else {                                   // 1 dependent mul
      x = x * c;
    }
  }
  const unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
void run(const char* name, int ops_per_iter, double* out, unsigned long long* cyc) {
  hipLaunchKernelGGL((kern<MODE>), dim3(1), dim3(64), 0, 0, out, cyc, 0.7);
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL((kern<MODE>), dim3(1), dim3(64), 0, 0, out, cyc, 0.7);
  CK(hipDeviceSynchronize());
  unsigned long long c;
  CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
  printf("%-44s %8.2f cycles per iteration, %6.2f per dependent op\n", name, (double)c / kIters,
         (double)c / kIters / ops_per_iter);
}

int main() {
  double* out;
  unsigned long long* cyc;
  CK(hipMalloc(&out, 64 * 8));
  CK(hipMalloc(&cyc, 64));
  run<0>("v_fma_f64 chain", 1, out, cyc);
  run<5>("v_mul_f64 chain", 1, out, cyc);
  run<1>("v_rsq_f64 chain", 1, out, cyc);
  run<2>("v_readlane x2 -> v_fma_f64 (SGPR operand)", 3, out, cyc);
  run<3>("pivot step: rsq + 2 Newton + mul + fma", 9, out, cyc);
  run<4>("pivot step: rsq + 1 Newton + mul + fma", 6, out, cyc);
  return 0;
}
