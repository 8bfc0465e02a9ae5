// Timing of the blocked Cholesky (launch_cholesky: chol_diag / chol_panel / chol_update kernels) on an
// SPD matrix (tools only; not part of the library).  Correctness is tests/test_gpu_turbo.py.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/ablate/ablate_chol tools/ablate/ablate_chol.hip
// Run on the GPU box: ./tools/ablate/ablate_chol [N ...]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

// phase timestamps of chol_diag_kernel: shader clock (s_memtime) and the 100 MHz constant clock
__device__ unsigned long long g_trace[2][32];
#define OMB_CHOL_TRACE(id, cond)                                  \
  do {                                                            \
    if (cond) {                                                   \
      g_trace[0][id] = __builtin_readcyclecounter();              \
      g_trace[1][id] = __builtin_amdgcn_s_memrealtime();          \
    }                                                             \
  } while (0)

__device__ unsigned long long g_col[4][64];
#define OMB_CHOL_COL(w, j, cond)                                  \
  do {                                                            \
    if (cond) g_col[w][j] = __builtin_readcyclecounter();         \
  } while (0)

#define OMB_TOOLS_KNOBS
#include "../../optimobo_amd/csrc/omb_linalg.hip"
#include "../../optimobo_amd/csrc/omb_gemm.hip"

using namespace omb;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)

static void trace_diag() {
  const int N = 64;
  std::vector<double> h(N * N);
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) h[i * N + j] = (i == j) ? N : 1.0 / (1.0 + std::abs((double)(i - j)));
  double *A, *ws;
  int* info;
  CK(hipMalloc(&A, N * N * 8));
  CK(hipMalloc(&ws, chol_ws_doubles(N) * 8));
  CK(hipMalloc(&info, 64));
  const char* names[17] = {"start", "loaded", "b0 begin", "b0 factored", "b1 begin", "b1 factored", "b2 begin",
                           "b2 factored", "b3 begin", "b3 factored", "w0 L + W_00", "w1 L + W_11", "w2 L + W_22",
                           "w3 L + W_33", "(unused)", "barrier", "W done"};
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipMemcpy(A, h.data(), N * N * 8, hipMemcpyHostToDevice));
    CK(hipMemset(info, 0, 4));
    hipLaunchKernelGGL(chol_diag_kernel, dim3(1), dim3(256), 0, 0, A, (int64_t)N, (int64_t)N, ws, info,
                       reinterpret_cast<int*>(ws + kCholWsDoubles), 0);
    CK(hipDeviceSynchronize());
    unsigned long long t[2][32];
    CK(hipMemcpyFromSymbol(t, HIP_SYMBOL(g_trace), sizeof(t)));
    if (rep < 2) continue;
    printf("chol_diag_kernel phases (cycles of s_memtime from start; us from the 100 MHz clock)\n");
    for (int i = 0; i < 17; ++i)
      printf("  %-12s %8lld cyc  %7.2f us\n", names[i], (long long)(t[0][i] - t[0][0]), (t[1][i] - t[1][0]) / 100.0);
    unsigned long long c[4][64];
    CK(hipMemcpyFromSymbol(c, HIP_SYMBOL(g_col), sizeof(c)));
    printf("per column j: cycle (from start) at which wave w has applied (j < 16w) or factored (16w <= j < 16w+16) "
           "column j\n");
    for (int j = 0; j < 64; ++j) {
      printf("  col %2d:", j);
      for (int w = 0; w < 4; ++w) {
        if (j < 16 * w + 16) printf(" w%d %7lld", w, (long long)(c[w][j] - t[0][0]));
      }
      printf("\n");
    }
  }
  CK(hipFree(A)); CK(hipFree(ws)); CK(hipFree(info));
}

int main(int argc, char** argv) {
  trace_diag();
  // extra dynamic LDS per update workgroup: 0 (3 workgroups per CU by VGPRs), 16 KB (2), 48 KB (1)
  const size_t extra[3] = {0, 16 << 10, 48 << 10};
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
    CK(hipMalloc(&ws, chol_ws_doubles(N) * 8));
    CK(hipMalloc(&info, 64));
    CK(hipMemcpy(A0, h.data(), N * N * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // the two launch schedules interleaved: kCholTwoLaunch (panel + update per step, round 2) and
    // kCholFused (the update launch forms the next panel; round 3)
    float best = 1e30f, sum = 0.f, best2 = 1e30f, sum2 = 0.f;
    const int reps = 10;
    for (int r = 0; r < reps + 1; ++r) {
      for (int mode = 0; mode < 2; ++mode) {
        CK(hipMemcpy(A, A0, N * N * 8, hipMemcpyDeviceToDevice));
        CK(hipMemset(info, 0, 4));
        CK(hipEventRecord(e0));
        CK(launch_cholesky_mode(0, A, N, N, info, ws, mode == 0 ? kCholTwoLaunch : kCholFused));
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r > 0 && mode == 1) {
          best = ms < best ? ms : best;
          sum += ms;
        } else if (r > 0) {
          best2 = ms < best2 ? ms : best2;
          sum2 += ms;
        }
      }
    }
    printf("N=%lld  two launches per step %.3f ms (best %.3f)\n", (long long)N, sum2 / reps, best2);
    {
      float sx[3] = {0.f, 0.f, 0.f};
      for (int r = 0; r < reps + 1; ++r)
        for (int v = 0; v < 3; ++v) {
          set_chol_update_lds(extra[v]);
          CK(hipMemcpy(A, A0, N * N * 8, hipMemcpyDeviceToDevice));
          CK(hipEventRecord(e0));
          CK(launch_cholesky(0, A, N, N, info, ws));
          CK(hipEventRecord(e1));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          if (r > 0) sx[v] += ms;
        }
      set_chol_update_lds(0);
      printf("N=%lld  fused, extra LDS per update workgroup 0 / 16 KB / 48 KB: %.3f / %.3f / %.3f ms\n", (long long)N,
             sx[0] / reps, sx[1] / reps, sx[2] / reps);
    }
    // the same launch sequence captured once into a hipGraph and replayed (launch-gap ablation)
    float gbest = 1e30f, gsum = 0.f;
    {
      hipStream_t s;
      CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      hipGraph_t graph;
      hipGraphExec_t exec;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      CK(launch_cholesky(s, A, N, N, info, ws));
      CK(hipStreamEndCapture(s, &graph));
      CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
      for (int r = 0; r < reps + 1; ++r) {
        CK(hipMemcpyAsync(A, A0, N * N * 8, hipMemcpyDeviceToDevice, s));
        CK(hipMemsetAsync(info, 0, 4, s));
        CK(hipEventRecord(e0, s));
        CK(hipGraphLaunch(exec, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r > 0) {
          gbest = ms < gbest ? ms : gbest;
          gsum += ms;
        }
      }
      CK(hipStreamSynchronize(s));
      CK(hipGraphExecDestroy(exec));
      CK(hipGraphDestroy(graph));
      CK(hipStreamDestroy(s));
    }
    printf("N=%lld  hipGraph replay %.3f ms (best %.3f)\n", (long long)N, gsum / reps, gbest);
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
    printf("N=%lld  Cholesky (fused) %.3f ms (best %.3f, %d steps = %.1f us/step)  info %d  max |LLt - A|/A_ii %.2e\n",
           (long long)N, sum / reps, best, (int)((N + 63) / 64), best * 1e3 / ((N + 63) / 64), hinfo, worst);
    CK(hipFree(A0)); CK(hipFree(A)); CK(hipFree(ws)); CK(hipFree(info));
  }
  return 0;
}
