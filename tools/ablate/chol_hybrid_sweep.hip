// Per-step launches for the first k0 steps, then the persistent launch (launch_cholesky_persist's k0): time and
// factor against the per-step launches alone, for a list of k0 (tools only).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/ablate/chol_hybrid_sweep tools/ablate/chol_hybrid_sweep.hip
// Run:   ./tools/ablate/chol_hybrid_sweep N [N ...]   (k0 list from CHOL_K0S, default 0,4,8,12,16,24,32; the
//        persistent launch's lookahead L list from CHOL_LS, default 3 — 0 = round 4's step-major task order; the
//        far tiles' update batching from CHOL_BW, "batch:window" pairs, default the library's — 1:0 = round 5's table)
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define OMB_TOOLS_KNOBS
#include "../../optimobo_amd/csrc/omb_linalg.hip"
#include "../../optimobo_amd/csrc/omb_wide.hip"
#include "../../optimobo_amd/csrc/omb_gemm.hip"

using namespace omb;

// ≈ us microseconds of GPU time ahead of the timed launches, so the host has queued them all before the GPU reaches
// them (the per-step launches then run back to back, as in the config-6 pipeline behind its GEMMs)
__global__ void busy_kernel(int us) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)us * 100ull) __builtin_amdgcn_s_sleep(8);
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  std::vector<int> k0s = {0, 4, 8, 12, 16, 24, 32};
  if (const char* e = getenv("CHOL_K0S")) {
    k0s.clear();
    std::string s(e);
    size_t p = 0;
    while (p < s.size()) {
      size_t q = s.find(',', p);
      if (q == std::string::npos) q = s.size();
      k0s.push_back(atoi(s.substr(p, q - p).c_str()));
      p = q + 1;
    }
  }
  std::vector<int> Ls = {3};
  if (const char* e = getenv("CHOL_LS")) {
    Ls.clear();
    std::string s(e);
    size_t p = 0;
    while (p < s.size()) {
      size_t q = s.find(',', p);
      if (q == std::string::npos) q = s.size();
      Ls.push_back(atoi(s.substr(p, q - p).c_str()));
      p = q + 1;
    }
  }
  std::vector<std::pair<int, int>> bws = {{-1, -1}};
  if (const char* e = getenv("CHOL_BW")) {
    bws.clear();
    std::string s(e);
    size_t p = 0;
    while (p < s.size()) {
      size_t q = s.find(',', p);
      if (q == std::string::npos) q = s.size();
      const std::string item = s.substr(p, q - p);
      const size_t c = item.find(':');
      bws.push_back({atoi(item.substr(0, c).c_str()), c == std::string::npos ? 0 : atoi(item.substr(c + 1).c_str())});
      p = q + 1;
    }
  }
  std::vector<int64_t> sizes;
  for (int i = 1; i < argc; ++i) sizes.push_back(atoll(argv[i]));
  if (sizes.empty()) sizes = {3000};
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
    std::vector<double> R(N * N), L(N * N);
    auto run = [&](int mode, int k0, float& best) {
      set_chol_hybrid_k0(k0);
      best = 1e30f;
      for (int r = 0; r < 6; ++r) {
        CK(hipMemcpy(A, A0, N * N * 8, hipMemcpyDeviceToDevice));
        CK(hipDeviceSynchronize());
        hipLaunchKernelGGL(busy_kernel, dim3(1), dim3(64), 0, 0, 3000);
        CK(hipEventRecord(e0));
        CK(launch_cholesky_mode(0, A, N, N, info, ws, mode));
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r > 0) best = std::min(best, ms);
      }
      int hinfo = -1;
      CK(hipMemcpy(&hinfo, info, 4, hipMemcpyDeviceToHost));
      return hinfo;
    };
    float tb;
    int ib = run(kCholBlocked, -1, tb);
    CK(hipMemcpy(R.data(), A, N * N * 8, hipMemcpyDeviceToHost));
    printf("N=%lld per-step launches %.3f ms info %d\n", (long long)N, tb, ib);
    std::vector<double> L1(N * N);
    for (int la : Ls)
    for (int k0 : k0s) {
      for (size_t v = 0; v < bws.size(); ++v) {
        set_chol_lookahead(la);
        set_chol_batch(bws[v].first, bws[v].second);
        float tp;
        const int ip = run(kCholPersistent, k0, tp);
        CK(hipMemcpy(L.data(), A, N * N * 8, hipMemcpyDeviceToHost));
        double md = 0.0;
        for (int64_t i = 0; i < N; ++i)
          for (int64_t j = 0; j <= i; ++j) md = std::max(md, std::abs(L[i * N + j] - R[i * N + j]) / std::sqrt(h[i * N + i]));
        // batches are bitwise the single-step tasks: every variant against the first of this (L, k0)
        long long ndiff = 0;
        if (v == 0) L1 = L;
        else
          for (int64_t i = 0; i < N; ++i)
            for (int64_t j = 0; j <= i; ++j) ndiff += L[i * N + j] != L1[i * N + j];
        printf("N=%lld L=%d k0=%d batch=%d window=%d: %.3f ms info %d max |L - L_steps|/sqrt(A_ii) %.2e  bits != first %lld\n",
               (long long)N, la, k0, bws[v].first, bws[v].second, tp, ip, md, ndiff);
      }
    }
    set_chol_lookahead(-1);
    set_chol_batch(-1, -1);
    set_chol_hybrid_k0(-1);
    CK(hipFree(A0)); CK(hipFree(A)); CK(hipFree(ws)); CK(hipFree(info));
  }
  return 0;
}
