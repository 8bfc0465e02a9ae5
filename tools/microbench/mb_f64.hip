// Microbenchmark: FP64 MFMA vs FP64 VALU FMA throughput on gfx950, and their overlap.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef double d4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while(0)

template <int MODE>  // 0 = mfma only, 1 = valu only, 2 = waves 0-3 mfma / 4-7 valu, 3 = exp
__global__ __launch_bounds__(512) void kern(double* out, int iters, double seed) {
  int lane = threadIdx.x & 63;
  int wave = threadIdx.x >> 6;
  double a = seed + lane * 1e-3, b = seed - lane * 1e-3;
  bool do_mfma = (MODE == 0) || (MODE == 2 && wave < 4);
  bool do_valu = (MODE == 1) || (MODE == 2 && wave >= 4);
  double acc = 0.0;
  if (do_mfma) {
    d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    for (int i = 0; i < iters; ++i) {
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
    }
    acc += c0[0] + c1[1] + c2[2] + c3[3];
  }
  if (do_valu) {
    double x0 = a, x1 = b, x2 = a + 1, x3 = b + 1, x4 = a + 2, x5 = b + 2, x6 = a + 3, x7 = b + 3;
    for (int i = 0; i < iters * 16; ++i) {  // 16 x 8 FMAs per iter ~ match flops? set per-iter flop count below
      x0 = __builtin_fma(x0, a, b); x1 = __builtin_fma(x1, a, b);
      x2 = __builtin_fma(x2, a, b); x3 = __builtin_fma(x3, a, b);
      x4 = __builtin_fma(x4, a, b); x5 = __builtin_fma(x5, a, b);
      x6 = __builtin_fma(x6, a, b); x7 = __builtin_fma(x7, a, b);
    }
    acc += x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
  }
  if (MODE == 3) {
    double x0 = a * 1e-3, x1 = b * 1e-3, x2 = x0 + 0.1, x3 = x1 + 0.1;
    for (int i = 0; i < iters; ++i) {
      x0 = exp(-x0); x1 = exp(-x1); x2 = exp(-x2); x3 = exp(-x3);
    }
    acc += x0 + x1 + x2 + x3;
  }
  if (MODE == 4) {
    double x0 = a * 1e-3, x1 = b * 1e-3, x2 = x0 + 0.1, x3 = x1 + 0.1;
    for (int i = 0; i < iters; ++i) {
      x0 = erfc(x0); x1 = erfc(x1); x2 = erfc(x2); x3 = erfc(x3);
    }
    acc += x0 + x1 + x2 + x3;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int MODE>
float run(int blocks, int iters, double* d) {
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern<MODE>, dim3(blocks), dim3(512), 0, 0, d, iters, 0.5);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(kern<MODE>, dim3(blocks), dim3(512), 0, 0, d, iters, 0.5);
  CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
  float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
  return ms;
}

int main() {
  int blocks = 256 * 2;  // 2 blocks of 512 threads per CU = 16 waves/CU
  int iters = 4096;
  double* d; CHECK(hipMalloc(&d, sizeof(double) * blocks * 512));
  double waves = blocks * 8.0;
  float ms0 = run<0>(blocks, iters, d);
  double fl0 = waves * iters * 4 * (16.0 * 16 * 4 * 2);
  printf("MFMA f64 16x16x4: %.3f ms, %.2f TFLOP/s, cycles/MFMA/SIMD @2.4GHz ~ %.1f\n", ms0, fl0 / ms0 / 1e9,
         (ms0 * 1e-3 * 2.4e9) / (waves * iters * 4 / (256.0 * 4)));
  float ms1 = run<1>(blocks, iters, d);
  double fl1 = waves * 64 * iters * 16 * 8 * 2.0;
  printf("VALU f64 fma: %.3f ms, %.2f TFLOP/s\n", ms1, fl1 / ms1 / 1e9);
  float ms2 = run<2>(blocks, iters, d);
  printf("mixed (half waves mfma, half valu): %.3f ms  (mfma-only part would be %.3f, valu-only part %.3f)\n", ms2, ms0 / 2, ms1 / 2);
  float ms3 = run<3>(blocks, iters / 4, d);
  double ex = waves * 64 * (iters / 4) * 4.0;
  printf("exp f64: %.3f ms, %.2f Gexp/s\n", ms3, ex / ms3 / 1e6);
  float ms4 = run<4>(blocks, iters / 4, d);
  printf("erfc f64: %.3f ms, %.2f Gerfc/s\n", ms4, ex / ms4 / 1e6);
  CHECK(hipFree(d));
  return 0;
}
