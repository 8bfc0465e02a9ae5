// Ablation timing of the covariance SYRK (Σ = K(X*, X*) − VᵀV, config 6's shape: n_train 512, N 3000, d 30): the
// register-staged gemm_kernel<…, KSS> against syrk_glds_kernel<STAGES, SR> variants, interleaved in one process, each
// checked bitwise against the register path (tools only).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form -o tools/ablate/ablate_syrk \
//          tools/ablate/ablate_syrk.hip
// Run:   ./tools/ablate/ablate_syrk [N] [K] [kp]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../optimobo_amd/csrc/omb_gemm.hip"

using namespace omb;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  const int64_t N = argc > 1 ? atoll(argv[1]) : 3000, K = argc > 2 ? atoll(argv[2]) : 512;
  const int kp = argc > 3 ? atoi(argv[3]) : 32;
  std::vector<double> hv(K * N), hx(N * kp), hq(N);
  srand(7);
  for (auto& v : hv) v = (rand() / (double)RAND_MAX - 0.5) * 0.2;
  for (int64_t i = 0; i < N; ++i) {
    double q = 0;
    for (int j = 0; j < kp; ++j) {
      const double v = j < 30 ? (rand() / (double)RAND_MAX) : 0.0;
      hx[i * kp + j] = v;
      q += v * v;
    }
    hq[i] = q;
  }
  double *V, *xs, *xq, *S0, *S1;
  CK(hipMalloc(&V, K * N * 8));
  CK(hipMalloc(&xs, N * kp * 8));
  CK(hipMalloc(&xq, N * 8));
  CK(hipMalloc(&S0, N * N * 8));
  CK(hipMalloc(&S1, N * N * 8));
  CK(hipMemcpy(V, hv.data(), K * N * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(xs, hx.data(), N * kp * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(xq, hq.data(), N * 8, hipMemcpyHostToDevice));
  CK(hipMemset(S0, 0, N * N * 8));
  CK(hipMemset(S1, 0, N * N * 8));
  const CovEpi ce{xs, xq, kp, OMB_KERNEL_MATERN52, 0.5, 1e-9};
  const int T = (int)((N + kGT - 1) / kGT);
  int g1 = 0;
  const int* tmap = xcd_tile_map(kMapSyrk, T, T, &g1);
  const dim3 grid = dim3((unsigned)g1);
  struct Variant {
    const char* name;
    void (*fn)(dim3, const double*, double*, int64_t, int64_t, CovEpi, const int*);
  };
#define GLDS(ST, SR, MB)                                                                                            \
  [](dim3 g, const double* V, double* S, int64_t N, int64_t K, CovEpi ce, const int* tm) {                         \
    hipLaunchKernelGGL((syrk_glds_kernel<ST, SR, MB>), g, dim3(256), 0, 0, N, K, -1.0, V, N, S, N, ce, tm);      \
  }
  const Variant vs[] = {
      {"register 2-slab (gemm_kernel)",
       [](dim3 g, const double* V, double* S, int64_t N, int64_t K, CovEpi ce, const int* tm) {
         hipLaunchKernelGGL((gemm_kernel<true, false, false, true, false, true>), g, dim3(256), 0, 0, N, N, K, -1.0, V,
                            N, V, N, 0.0, S, N, (const double*)nullptr, (int64_t)0, (int64_t)0, ce, tm);
       }},
      {"glds 3 x 16 (library)", GLDS(3, 16, 1)},
      {"glds 2 x 16, 5 wg/CU bound", GLDS(2, 16, 5)},
      {"glds 3 x 8, 5 wg/CU bound", GLDS(3, 8, 5)},
      {"glds 3 x 8, 6 wg/CU bound", GLDS(3, 8, 6)},
      {"glds 4 x 8, 4 wg/CU bound", GLDS(4, 8, 4)},
      {"glds 2 x 32", GLDS(2, 32, 1)},
      {"glds 3 x 16 again", GLDS(3, 16, 1)},
  };
#undef GLDS
  const int NV = sizeof(vs) / sizeof(vs[0]);
  auto launch = [&](const Variant& v, double* S) { v.fn(grid, V, S, N, K, ce, tmap); };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> t(NV, 0.f);
  const int reps = 20;
  for (int round = 0; round < 3; ++round)
    for (int i = 0; i < NV; ++i) {
      launch(vs[i], S1);
      CK(hipEventRecord(e0));
      for (int r = 0; r < reps; ++r) launch(vs[i], S1);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[i] += ms / reps;
    }
  std::vector<double> a(N * N), b(N * N);
  launch(vs[0], S0);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(a.data(), S0, N * N * 8, hipMemcpyDeviceToHost));
  const double flops = (double)N * (N + 1) * K;   // the lower triangle's multiply-adds × 2
  for (int i = 0; i < NV; ++i) {
    CK(hipMemset(S1, 0, N * N * 8));
    launch(vs[i], S1);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(b.data(), S1, N * N * 8, hipMemcpyDeviceToHost));
    long long diff = 0;
    for (int64_t r = 0; r < N; ++r)
      for (int64_t c = 0; c <= r; ++c) diff += memcmp(&a[r * N + c], &b[r * N + c], 8) != 0;
    printf("%-30s %8.2f us  %6.1f TFLOP/s  lower-triangle entries != register path: %lld\n", vs[i].name,
           1e3 * t[i] / 3, flops / (t[i] / 3 * 1e-3) / 1e12, diff);
  }
  return 0;
}
