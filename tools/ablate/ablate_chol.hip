// Ablation timing of one Cholesky panel step (tools only; not part of the library).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/ablate/ablate_chol tools/ablate/ablate_chol.hip
// Run on the GPU box: ./tools/ablate/ablate_chol [N]
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../optimobo_amd/csrc/omb_linalg.hip"

using namespace omb;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)

template <int ABL, bool VEC = false>
float step_ms(double* A, int64_t N, int* ctr, int reps) {
  const unsigned blocks = (unsigned)((N - 64 + 255) / 256);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipMemset(ctr, 0, 8 * 1024));
  hipLaunchKernelGGL((chol_panel_kernel<ABL, VEC>), dim3(blocks), dim3(256), 0, 0, A, N, N, 0, ctr, ctr + 1);
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((chol_panel_kernel<ABL, VEC>), dim3(blocks), dim3(256), 0, 0, A, N, N, 1 + i, ctr, ctr + 1);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int64_t N = argc > 1 ? atoll(argv[1]) : 3000;
  std::vector<double> h(N * N);
  for (int64_t i = 0; i < N; ++i)
    for (int64_t j = 0; j < N; ++j) h[i * N + j] = (i == j) ? N : 1.0 / (1.0 + std::abs((double)(i - j)));
  double* A;
  int* ctr;
  CK(hipMalloc(&A, N * N * 8));
  CK(hipMalloc(&ctr, 8 * 1024));
  CK(hipMemcpy(A, h.data(), N * N * 8, hipMemcpyHostToDevice));
  // steps 1.. (the matrix stays positive definite: diagonally dominant); timed over 20 steps each
  float full = 0, nodiag = 0, nopanel = 0, none = 0, vec = 0;
  for (int r = 0; r < 3; ++r) {
    full += step_ms<0>(A, N, ctr, 20);
    vec += step_ms<0, true>(A, N, ctr, 20);
    nodiag += step_ms<1>(A, N, ctr, 20);
    nopanel += step_ms<2>(A, N, ctr, 20);
    none += step_ms<3>(A, N, ctr, 20);
  }
  printf("N=%lld  full %.1f us  16B rows %.1f us  no-diag %.1f us  no-panel %.1f us  neither %.1f us\n",
         (long long)N, full / 3 * 1e3, vec / 3 * 1e3, nodiag / 3 * 1e3, nopanel / 3 * 1e3, none / 3 * 1e3);
  return 0;
}
