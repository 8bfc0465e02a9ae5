// K block at n_var > 8 (BASELINE config 5: n = 1024, d = 30, N = 2^19), variants of the library's
// kernel_block_pipe_kernel on the same data, interleaved (tools only): one or two row tiles per loop
// iteration, without stores (compute alone) and without compute (stores alone).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/ablate/ablate_kblock3 tools/ablate/ablate_kblock3.hip
// Run on the GPU box: ./tools/ablate/ablate_kblock3 [n] [N] [d]   (d = 6 or 30)
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <vector>
#include <algorithm>

#include "../../optimobo_amd/csrc/omb_posterior.hip"
#include "../../optimobo_amd/csrc/omb_wide.hip"

using namespace omb;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)

template <typename F>
float time_ms(F&& f, int reps) {
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
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms / reps;
}

template <int DP>
void bench(int n, int64_t N, int d) {
  const int R = (n + 15) / 16, Q = (R + 3) / 4, n_pad = 64 * Q;
  std::vector<double> hX((size_t)n * d), hls(d, 1.0), ha(n, 0.1), hXc((size_t)N * d);
  srand(3);
  for (auto& v : hX) v = rand() / (double)RAND_MAX;
  for (auto& v : hXc) v = rand() / (double)RAND_MAX;
  for (auto& v : hls) v = 0.5 + rand() / (double)RAND_MAX;
  double *X, *al, *Xs, *xsq, *alp, *lsp, *Xf, *Xc, *K1, *K2;
  CK(hipMalloc(&X, hX.size() * 8)); CK(hipMalloc(&al, n * 8)); CK(hipMalloc(&Xs, (size_t)n_pad * DP * 8));
  CK(hipMalloc(&xsq, n_pad * 8)); CK(hipMalloc(&alp, n_pad * 8 + DP * 8)); CK(hipMalloc(&Xf, packed_X_size(n_pad, DP) * 8));
  CK(hipMalloc(&Xc, hXc.size() * 8)); CK(hipMalloc(&K1, (size_t)n * N * 8)); CK(hipMalloc(&K2, (size_t)n * N * 8));
  CK(hipMemcpy(X, hX.data(), hX.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(al, ha.data(), n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(Xc, hXc.data(), hXc.size() * 8, hipMemcpyHostToDevice));
  lsp = alp + n_pad;
  CK(launch_pack_gp(0, n, d, DP, X, hls.data(), al, nullptr, Xs, xsq, alp, nullptr, 0, n_pad));
  CK(launch_pack_x(0, d, DP, n_pad, Xs, xsq, Xf));
  GPDev g{Xs, xsq, alp, nullptr, lsp, 1.3, n, R, 0, 0, Xf};
  const ExpCoef ec = exp_coef();
  dim3 g3((unsigned)((N + 127) / 128), (unsigned)((n + kblock_rows(DP) - 1) / kblock_rows(DP)));
  struct V { const char* name; void (*launch)(dim3, GPDev, int, const double*, int64_t, double*, ExpCoef); bool full; };
#define L(...) [](dim3 gr, GPDev gg, int dd, const double* xc, int64_t nn, double* k, ExpCoef e) { \
    hipLaunchKernelGGL((kernel_block_pipe_kernel<__VA_ARGS__>), gr, dim3(512), 0, 0, gg, dd, xc, nn, k, e); }
  const V vs[] = {
      {"library: 1 row tile / iteration", L(DP, 0, true, false, false, 1, 0), true},
      {"1 row tile, no stores", L(DP, 0, true, false, false, 1, 1), false},
      {"1 row tile, stores only", L(DP, 0, true, false, false, 1, 2), false},
  };
#undef L
#define P(CB, RCP, ROLL) [](dim3 gr, GPDev gg, int dd, const double* xc, int64_t nn, double* k, ExpCoef e) { \
    dim3 g2((unsigned)((nn + 128 * CB - 1) / (128 * CB)), gr.y);                                     \
    hipLaunchKernelGGL((kernel_block_persist_kernel<DP, 0, CB, RCP, ROLL>), g2, dim3(512), 0, 0, gg, dd, xc, nn, k, e); }
#define PA(CB, RCP, ROLL) [](dim3 gr, GPDev gg, int dd, const double* xc, int64_t nn, double* k, ExpCoef e) { \
    dim3 g2((unsigned)((nn + 128 * CB - 1) / (128 * CB)), gr.y);                                     \
    hipLaunchKernelGGL((kernel_block_persist_kernel<DP, 0, CB, RCP, ROLL, (DP > 8)>), g2, dim3(512), 0, 0, gg, dd, xc, nn, k, e); }
  const V ps[] = {
      {"(warm-up) persistent CB=8, 1/l, rolled", P(8, true, true), true},
      {"persistent CB=8, 1/l, rolled, aug r2", PA(8, true, true), true},
      {"persistent CB=8, 1/l, rolled", P(8, true, true), true},
      {"persistent CB=8, 1/l, aug r2", PA(8, true, false), true},
      {"persistent CB=8, 1/l", P(8, true, false), true},
      {"persistent CB=16, 1/l, rolled, aug r2", PA(16, true, true), true},
      {"persistent CB=4, 1/l, rolled, aug r2", PA(4, true, true), true},
      {"persistent CB=8, 1/l, rolled, aug r2 (again)", PA(8, true, true), true},
      {"persistent CB=8, 1/l, rolled (again)", P(8, true, true), true},
  };
#undef P
#undef PA
  std::vector<V> all(vs, vs + sizeof(vs) / sizeof(vs[0]));
  all.insert(all.end(), ps, ps + sizeof(ps) / sizeof(ps[0]));
  const int NV = (int)all.size();
  std::vector<float> t(NV, 0.f);
  for (int r = 0; r < 3; ++r)
    for (int i = 0; i < NV; ++i) t[i] += time_ms([&] { all[i].launch(g3, g, d, Xc, N, K1, ec); }, 5);
  const double bytes = 8.0 * (n + d) * N + 8.0 * n * (d + 1);
  for (int i = 0; i < NV; ++i) {
    const double ms = t[i] / 3;
    printf("n=%d N=%lld d=%d  %-36s %.3f ms  %5.0f GB/s  (%.3f of 8 TB/s)\n", n, (long long)N, d, all[i].name, ms,
           bytes / (ms * 1e-3) / 1e9, bytes / (ms * 1e-3) / 1e9 / 8000.0);
  }
  // outputs of the full variants against the library's
  std::vector<double> a((size_t)n * N), b((size_t)n * N);
  all[0].launch(g3, g, d, Xc, N, K1, ec);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(a.data(), K1, a.size() * 8, hipMemcpyDeviceToHost));
  for (int i = 1; i < NV; ++i) {
    if (!all[i].full) continue;
    CK(hipMemset(K2, 0xff, (size_t)n * N * 8));
    all[i].launch(g3, g, d, Xc, N, K2, ec);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(b.data(), K2, b.size() * 8, hipMemcpyDeviceToHost));
    size_t diff = 0;
    double mx = 0.0;
    for (size_t j = 0; j < a.size(); ++j) {
      diff += (a[j] != b[j]);
      mx = std::max(mx, std::fabs(a[j] - b[j]) / std::max(std::fabs(a[j]), 1e-300));
    }
    printf("%s vs library: %zu of %zu elements differ, max rel %.2e\n", all[i].name, diff, a.size(), mx);
  }
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 1024;
  const int64_t N = argc > 2 ? atoll(argv[2]) : (1 << 19);
  const int d = argc > 3 ? atoi(argv[3]) : 30;
  if (d == 6) bench<6>(n, N, d);
  else if (d == 30) bench<32>(n, N, d);
  else { printf("d must be 6 or 30\n"); return 1; }
  return 0;
}
