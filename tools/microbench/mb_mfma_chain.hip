// FP64 MFMA issue behaviour on gfx950 (v_mfma_f64_16x16x4_f64): throughput per SIMD as a function of
// independent accumulator chains per wave (1, 2, 4, 8) and waves per SIMD (1, 2, 4), with the B operand
// in registers or read from LDS per MFMA (ds_read_b64, the posterior kernels' pattern).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench/mb_mfma_chain tools/microbench/mb_mfma_chain.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double d4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)

template <int CH, bool LDSB>
__global__ void kern(double* out, int iters) {
  __shared__ double buf[4096];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 4096; i += blockDim.x) buf[i] = 1e-3 * i;
  __syncthreads();
  double a = 1.0 + 1e-3 * lane, b = 0.5 - 1e-4 * lane;
  d4 acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = d4{0, 0, 0, 0};
  int off = (threadIdx.x >> 6) * 64 + lane;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const double bb = LDSB ? buf[(off + 128 * c) & 4095] : b;
      acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bb, acc[c], 0, 0, 0);
    }
    off += 512;
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += acc[c][0] + acc[c][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int CH, bool LDSB>
void run(int waves_per_simd, double* d) {
  const int threads = 256 * waves_per_simd;        // 4 SIMDs
  const int blocks = 256;                          // one workgroup per CU
  const int total_mfma = 1 << 14;                  // per wave-chain-set: keep the work per SIMD fixed
  const int iters = total_mfma / (CH * waves_per_simd);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((kern<CH, LDSB>), dim3(blocks), dim3(threads), 0, 0, d, iters);
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL((kern<CH, LDSB>), dim3(blocks), dim3(threads), 0, 0, d, iters);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double mfma_per_simd = (double)iters * CH * waves_per_simd;
  const double flops = mfma_per_simd * 1024.0 * 2048.0;
  printf("chains/wave %d  waves/SIMD %d  B from %-4s : %.3f ms  %.1f TFLOP/s  %.1f ns per MFMA per SIMD\n", CH,
         waves_per_simd, LDSB ? "LDS" : "regs", ms, flops / (ms * 1e-3) / 1e12, ms * 1e6 / mfma_per_simd);
}

int main() {
  double* d;
  CK(hipMalloc(&d, sizeof(double) * 256 * 1024));
  for (int w : {1, 2, 4}) {
    run<1, false>(w, d); run<2, false>(w, d); run<4, false>(w, d); run<8, false>(w, d);
    run<1, true>(w, d); run<2, true>(w, d); run<4, true>(w, d); run<8, true>(w, d);
  }
  return 0;
}
