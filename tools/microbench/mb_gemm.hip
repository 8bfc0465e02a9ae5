// Latency of the trailing-update GEMM shapes of the blocked Cholesky (tools only).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/microbench/mb_gemm tools/microbench/mb_gemm.hip
// Run on the GPU box: ./tools/microbench/mb_gemm [N]
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../optimobo_amd/csrc/omb_linalg.hip"
#include "../../optimobo_amd/csrc/omb_wide.hip"

using namespace omb;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)

template <typename F>
float time_us(F&& f, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  f();
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / reps;
}

int main(int argc, char** argv) {
  const int64_t N = argc > 1 ? atoll(argv[1]) : 3000;
  std::vector<double> h(N * N);
  for (auto& v : h) v = rand() / (double)RAND_MAX;
  double* A;
  CK(hipMalloc(&A, N * N * 8));
  CK(hipMemcpy(A, h.data(), N * N * 8, hipMemcpyHostToDevice));
  const int64_t rest = N - 128;
  double* L21 = A + 64 * N;
  double* C = A + 64 * N + 64;
  const int reps = 50;
  float t_small = time_us([&] { gemm<false, true, false, true>(0, rest, 64, 64, -1.0, L21, N, L21, N, 1.0, C, N, nullptr); }, reps);
  float t_small0 = time_us([&] { gemm<false, true, false, true>(0, rest, 64, 64, -1.0, L21, N, L21, N, 0.0, C, N, nullptr); }, reps);
  float t_full = time_us([&] { gemm<false, true, false, true>(0, rest, rest, 64, -1.0, L21, N, L21, N, 1.0, C, N, nullptr); }, reps);
  float t_half = time_us([&] { gemm<false, true, false, true>(0, rest / 2, rest / 2, 64, -1.0, L21, N, L21, N, 1.0, C, N, nullptr); }, reps);
  float t_tiny = time_us([&] { gemm<false, true, false, true>(0, 64, 64, 64, -1.0, L21, N, L21, N, 1.0, C, N, nullptr); }, reps);
  float t_empty = time_us([&] { hipLaunchKernelGGL(add_diag_kernel, dim3(1), dim3(64), 0, 0, C, 1, N, 0.0); }, reps);
  printf("N=%lld rest=%lld  small(rest x 64, k64) %.1f us  beta0 %.1f us  full lower (rest^2, k64) %.1f us  "
         "half %.1f us  64x64 %.1f us  empty kernel %.1f us\n",
         (long long)N, (long long)rest, t_small, t_small0, t_full, t_half, t_tiny, t_empty);
  return 0;
}
