// Timing of the blocked Cholesky (launch_cholesky: chol_diag / chol_trsm / chol_update kernels) on an
// SPD matrix (tools only; not part of the library).  Correctness is tests/test_gpu_turbo.py.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/ablate/ablate_chol tools/ablate/ablate_chol.hip
// Run on the GPU box: ./tools/ablate/ablate_chol [N ...]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../optimobo_amd/csrc/omb_linalg.hip"

using namespace omb;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)

int main(int argc, char** argv) {
  std::vector<int64_t> sizes;
  for (int i = 1; i < argc; ++i) sizes.push_back(atoll(argv[i]));
  if (sizes.empty()) sizes = {512, 1024, 3000};
  for (int64_t N : sizes) {
    std::vector<double> h(N * N);
    for (int64_t i = 0; i < N; ++i)
      for (int64_t j = 0; j < N; ++j) h[i * N + j] = (i == j) ? N : 1.0 / (1.0 + std::abs((double)(i - j)));
    double *A0, *A, *ws;
    int* info;
    CK(hipMalloc(&A0, N * N * 8));
    CK(hipMalloc(&A, N * N * 8));
    CK(hipMalloc(&ws, kCholWsDoubles * 8));
    CK(hipMalloc(&info, 64));
    CK(hipMemcpy(A0, h.data(), N * N * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e30f, sum = 0.f;
    const int reps = 10;
    for (int r = 0; r < reps + 1; ++r) {
      CK(hipMemcpy(A, A0, N * N * 8, hipMemcpyDeviceToDevice));
      CK(hipMemset(info, 0, 4));
      CK(hipEventRecord(e0));
      CK(launch_cholesky(0, A, N, N, info, ws));
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0) {
        best = ms < best ? ms : best;
        sum += ms;
      }
    }
    int hinfo = -1;
    CK(hipMemcpy(&hinfo, info, 4, hipMemcpyDeviceToHost));
    // residual spot check on a few entries: (L Lᵀ)[i][j] vs A[i][j]
    std::vector<double> L(N * N);
    CK(hipMemcpy(L.data(), A, N * N * 8, hipMemcpyDeviceToHost));
    double worst = 0.0;
    for (int t = 0; t < 200; ++t) {
      const int64_t i = (t * 7919) % N, j = (t * 104729) % (i + 1);
      double s = 0.0;
      for (int64_t k = 0; k <= j; ++k) s += L[i * N + k] * L[j * N + k];
      worst = std::max(worst, std::abs(s - h[i * N + j]) / std::abs(h[i * N + i]));
    }
    printf("N=%lld  Cholesky %.3f ms (best %.3f, %d steps = %.1f us/step)  info %d  max |LLt - A|/A_ii %.2e\n",
           (long long)N, sum / reps, best, (int)((N + 63) / 64), best * 1e3 / ((N + 63) / 64), hinfo, worst);
    CK(hipFree(A0)); CK(hipFree(A)); CK(hipFree(ws)); CK(hipFree(info));
  }
  return 0;
}
