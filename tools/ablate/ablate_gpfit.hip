// Phase costs of the one-workgroup GP-fit evaluation (gp_lml_small_batch_kernel, 2 problems, d = 2) at
// several n: full, without the block sweep, without the gradient sums, without the kernel evaluations of
// the K build (tools only).  Variants interleaved.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/ablate/ablate_gpfit tools/ablate/ablate_gpfit.hip
#include <cstdio>
#include <cstdlib>
#include <vector>

// per-step phase timestamps (100 MHz constant clock) of waves 0 and 1 of workgroup 0, first attempt
__device__ unsigned long long g_ftrace[2][8][8];
#define OMB_FIT_TRACE(p, id)                                                                     \
  do {                                                                                           \
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0 && threadIdx.x < 128 && t < 0 && (p) < 8)     \
      g_ftrace[threadIdx.x >> 6][p][id] = __builtin_amdgcn_s_memrealtime();                       \
  } while (0)

#include "../../optimobo_amd/csrc/omb_posterior.hip"
#include "../../optimobo_amd/csrc/omb_linalg.hip"
#include "../../optimobo_amd/csrc/omb_wide.hip"
#include "../../optimobo_amd/csrc/omb_gemm.hip"

using namespace omb;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)

template <int ABL>
float run(const double* X, int n, const FitBatch& b, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((gp_lml_small_batch_kernel<2, OMB_KERNEL_MATERN52, ABL>), dim3(2), dim3(kSmallFitThreads), 0, 0, X,
                     2, n, b, 1e-8);
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((gp_lml_small_batch_kernel<2, OMB_KERNEL_MATERN52, ABL>), dim3(2), dim3(kSmallFitThreads), 0, 0,
                       X, 2, n, b, 1e-8);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps * 1000.f;
}

int main() {
  const int ns[] = {20, 40, 64, 96, 119, 128};
  for (int n : ns) {
    std::vector<double> hX(n * 2), hy(2 * n);
    srand(n);
    for (auto& v : hX) v = 4.0 * rand() / RAND_MAX - 2.0;
    for (int i = 0; i < n; ++i) {
      hy[i] = 100.0 * (hX[2 * i] * hX[2 * i] + hX[2 * i + 1] * hX[2 * i + 1]);
      hy[n + i] = (hX[2 * i] - 1) * (hX[2 * i] - 1) + hX[2 * i + 1] * hX[2 * i + 1];
    }
    double *X, *y, *out;
    CK(hipMalloc(&X, n * 2 * 8)); CK(hipMalloc(&y, 2 * n * 8)); CK(hipMalloc(&out, 2 * 16 * 8));
    CK(hipMemcpy(X, hX.data(), n * 2 * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(y, hy.data(), 2 * n * 8, hipMemcpyHostToDevice));
    FitBatch b{};
    for (int p = 0; p < 2; ++p) {
      b.y[p] = y + p * n;
      b.out[p] = out + p * 16;
      b.variance[p] = p ? 3.0 : 1e5;
      for (int j = 0; j < 8; ++j) b.ls[p][j] = p ? 0.9 : 1.7;
    }
    float t[4] = {0, 0, 0, 0};
    for (int r = 0; r < 3; ++r) {
      t[0] += run<0>(X, n, b, 20);
      t[1] += run<1>(X, n, b, 20);
      t[2] += run<2>(X, n, b, 20);
      t[3] += run<4 | 2>(X, n, b, 20);
    }
    std::vector<double> ho(32);
    run<0>(X, n, b, 1);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(ho.data(), out, 32 * 8, hipMemcpyDeviceToHost));
    {
      std::vector<unsigned long long> tr(2 * 8 * 8);
      CK(hipMemcpyFromSymbol(tr.data(), HIP_SYMBOL(g_ftrace), tr.size() * 8));
      const int NB = (n + 15) / 16;
      for (int p = 0; p < NB && p < 8; ++p) {
        const unsigned long long* w0 = &tr[(0 * 8 + p) * 8];
        const unsigned long long* w1 = &tr[(1 * 8 + p) * 8];
        printf("   step %d (us): w0 chol %.2f inv %.2f | bar1 w0 %.2f w1 %.2f | B w1 %.2f | bar2 w1 %.2f | C w1 %.2f | bar3 w1 %.2f\n", p,
               (w0[1] - w0[0]) / 100.0, (w0[2] - w0[1]) / 100.0, (w0[3] - w0[2]) / 100.0, (w1[3] - w1[2]) / 100.0,
               (w1[4] - w1[3]) / 100.0, (w1[5] - w1[4]) / 100.0, (w1[6] - w1[5]) / 100.0, (w1[7] - w1[6]) / 100.0);
      }
    }
    printf("n=%3d  full %7.1f us  no sweep %7.1f  no gradient %7.1f  no K evals, no gradient %7.1f   jitter %g/%g info %g/%g\n",
           n, t[0] / 3, t[1] / 3, t[2] / 3, t[3] / 3, ho[2 + 3], ho[16 + 2 + 3], ho[2 + 4], ho[16 + 2 + 4]);
    CK(hipFree(X)); CK(hipFree(y)); CK(hipFree(out));
  }
  return 0;
}
