// VALU rate of the Matern-5/2 transform (matern_r2_tab256_x2) on gfx950, in isolation and next to the
// r² MFMA of the generation step: elements per second per CU from registers only, with the 256-entry
// exp table in LDS, for 4 / 8 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/microbench/mb_matern tools/microbench/mb_matern.hip
#include <cstdio>
#include <cstdlib>

#include "../../optimobo_amd/csrc/omb_internal.h"

using namespace omb;
typedef double d4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)

// MODE 0: transform only (inputs from registers); MODE 1: r² MFMA (2 k-steps) + transform of its 4
// outputs per lane, as the posterior's generation step; MODE 2: MODE 1 + μ fma + LDS write per element.
template <int MODE>
__global__ __launch_bounds__(512) void kern(double* out, int iters, ExpCoef ec) {
  __shared__ double tab[256];
  __shared__ double sink[512 * 4];
  if (threadIdx.x < 256) tab[threadIdx.x] = kExp2Tab256[threadIdx.x];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const double pm[3] = {1.3, kSqrt5 * 1.3, kFiveThirds * 1.3};
  double acc = 0.0, r2 = 0.3 + 1e-3 * lane, r2b = 1.7 - 1e-3 * lane;
  const double a0 = 0.1 + 1e-3 * lane, a1 = 0.2 - 1e-4 * lane, b0 = 0.5, b1 = 0.25;
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 0) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        double v0, v1;
        matern_r2_tab256_x2(r2 + e, r2b + e, pm, ec, tab, v0, v1);
        acc += v0 + v1;
      }
      r2 += 1e-7;
      r2b += 1e-7;
    } else {
      d4 cr = d4{r2, r2b, r2 + 1, r2b + 1};
      cr = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, cr, 0, 0, 0);
      cr = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, cr, 0, 0, 0);
#pragma unroll
      for (int e = 0; e < 4; e += 2) {
        double v0, v1;
        matern_r2_tab256_x2(fabs(cr[e]), fabs(cr[e + 1]), pm, ec, tab, v0, v1);
        if constexpr (MODE == 2) {
          acc = fma(a0, v0, acc);
          acc = fma(a1, v1, acc);
          sink[(threadIdx.x * 4 + e) & 2047] = v0;
          sink[(threadIdx.x * 4 + e + 1) & 2047] = v1;
        } else {
          acc += v0 + v1;
        }
      }
      r2 += 1e-7;
      r2b += 1e-7;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc + sink[threadIdx.x];
}

template <int MODE>
void run(int blocks_per_cu, double* d) {
  const int blocks = 256 * blocks_per_cu, iters = 2048;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((kern<MODE>), dim3(blocks), dim3(512), 0, 0, d, iters, exp_coef());
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL((kern<MODE>), dim3(blocks), dim3(512), 0, 0, d, iters, exp_coef());
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double elems = (double)blocks * 512 * iters * 4;
  const double per_simd_cycles = ms * 1e-3 * 2.4e9 / ((elems / 64) / 1024);   // cycles per 64-element wave-op
  printf("mode %d (%s), %d waves/SIMD: %.3f ms, %.2f Gelem/s, %.2f cycles @2.4GHz per element per SIMD\n", MODE,
         MODE == 0 ? "transform only" : (MODE == 1 ? "MFMA r2 + transform" : "MFMA r2 + transform + mu + LDS"),
         2 * blocks_per_cu, ms, elems / ms / 1e6, per_simd_cycles / 64);
}

int main() {
  double* d;
  CK(hipMalloc(&d, sizeof(double) * 256 * 4 * 512));
  for (int b : {1, 2, 4}) {
    run<0>(b, d);
    run<1>(b, d);
    run<2>(b, d);
  }
  return 0;
}
