// Ablation timing of posterior_kernel variants (tools only; not part of the library).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/ablate/ablate_posterior tools/ablate/ablate_posterior.hip
// Run on the GPU box: ./tools/ablate/ablate_posterior [n] [N]
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../optimobo_amd/csrc/omb_posterior.hip"

using namespace omb;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)

template <int RT, int NW, int ABL>
float run(const GPArgs& a, const double* Xc, int64_t N, double* mu, double* var, int reps) {
  dim3 grid((unsigned)((N + 63) / 64), 2);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((posterior_kernel<RT, 4, 6, 0, NW, ABL>), grid, dim3(64 * NW), 0, 0, a, Xc, N, mu, var);
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((posterior_kernel<RT, 4, 6, 0, NW, ABL>), grid, dim3(64 * NW), 0, 0, a, Xc, N, mu, var);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

template <int RT, int CT, int NW, int ABL>
float run2p(const GPArgs& a, const double* Xc, int64_t N, double* mu, double* var, int reps) {
  dim3 grid((unsigned)((N + 16 * CT - 1) / (16 * CT)), 2);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((posterior2p_kernel<RT, CT, 6, 0, NW, ABL>), grid, dim3(64 * NW), 0, 0, a, Xc, N, mu, var);
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((posterior2p_kernel<RT, CT, 6, 0, NW, ABL>), grid, dim3(64 * NW), 0, 0, a, Xc, N, mu, var);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main(int argc, char** argv) {
  int n = argc > 1 ? atoi(argv[1]) : 512;
  int64_t N = argc > 2 ? atoll(argv[2]) : (1 << 20);
  const int d = 6, DP = 6;
  int R = (n + 15) / 16, Q = (R + 3) / 4, n_pad = 64 * Q;
  std::vector<double> hXs(n_pad * DP), hxsq(n_pad), ha(n_pad), hL(packed_L_size(R)), hls(DP, 1.0), hXc(N * d);
  srand(1);
  for (auto& v : hXs) v = rand() / (double)RAND_MAX;
  for (int k = 0; k < n_pad; ++k) {
    double s = 0;
    for (int j = 0; j < DP; ++j) s += hXs[k * DP + j] * hXs[k * DP + j];
    hxsq[k] = s;
    ha[k] = rand() / (double)RAND_MAX - 0.5;
  }
  for (auto& v : hL) v = (rand() / (double)RAND_MAX - 0.5) * 0.1;
  for (auto& v : hXc) v = rand() / (double)RAND_MAX;
  double *Xs, *xsq, *al, *Lp, *ls, *Xc, *mu, *var;
  CK(hipMalloc(&Xs, hXs.size() * 8)); CK(hipMalloc(&xsq, n_pad * 8)); CK(hipMalloc(&al, n_pad * 8));
  CK(hipMalloc(&Lp, hL.size() * 8)); CK(hipMalloc(&ls, DP * 8)); CK(hipMalloc(&Xc, hXc.size() * 8));
  CK(hipMalloc(&mu, 2 * N * 8)); CK(hipMalloc(&var, 2 * N * 8));
  CK(hipMemcpy(Xs, hXs.data(), hXs.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(xsq, hxsq.data(), n_pad * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(al, ha.data(), n_pad * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(Lp, hL.data(), hL.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(ls, hls.data(), DP * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(Xc, hXc.data(), hXc.size() * 8, hipMemcpyHostToDevice));
  GPArgs a{};
  for (int o = 0; o < 2; ++o) a.gp[o] = GPDev{Xs, xsq, al, Lp, ls, 1.0, n, R, 0, 0};
  a.d = d;
  a.DP = DP;
  const char* names[] = {"8w full", "8w no-matern(1)", "8w no-mfma(2)", "8w constA(4)", "8w nobarrier(8)",
                         "16w full", "16w no-matern(1)", "16w no-mfma(2)", "16w constA(4)", "16w nobarrier(8)",
                         "8w libm-math(16)", "16w libm-math(16)",
                         "2p 16w bn32", "2p 16w bn32 no-mfma", "2p 16w bn32 constA", "2p 8w bn32",
                         "8w barrier(32)", "16w barrier(32)", "8w counters+constA(4)"};
  const int NV = 19;
  float t[NV] = {0};
  for (int round = 0; round < 3; ++round) {
    t[16] += run<4, 8, 32>(a, Xc, N, mu, var, 5);
    t[17] += run<2, 16, 32>(a, Xc, N, mu, var, 5);
    t[18] += run<4, 8, 4>(a, Xc, N, mu, var, 5);
    t[12] += run2p<2, 2, 16, 0>(a, Xc, N, mu, var, 5);
    t[13] += run2p<2, 2, 16, 2>(a, Xc, N, mu, var, 5);
    t[14] += run2p<2, 2, 16, 4>(a, Xc, N, mu, var, 5);
    t[15] += run2p<4, 2, 8, 0>(a, Xc, N, mu, var, 5);
    t[10] += run<4, 8, 16>(a, Xc, N, mu, var, 5);
    t[11] += run<2, 16, 16>(a, Xc, N, mu, var, 5);
    t[0] += run<4, 8, 0>(a, Xc, N, mu, var, 5);
    t[1] += run<4, 8, 1>(a, Xc, N, mu, var, 5);
    t[2] += run<4, 8, 2>(a, Xc, N, mu, var, 5);
    t[3] += run<4, 8, 4>(a, Xc, N, mu, var, 5);
    t[4] += run<4, 8, 8>(a, Xc, N, mu, var, 5);
    t[5] += run<2, 16, 0>(a, Xc, N, mu, var, 5);
    t[6] += run<2, 16, 1>(a, Xc, N, mu, var, 5);
    t[7] += run<2, 16, 2>(a, Xc, N, mu, var, 5);
    t[8] += run<2, 16, 4>(a, Xc, N, mu, var, 5);
    t[9] += run<2, 16, 8>(a, Xc, N, mu, var, 5);
  }
  double flops = 2.0 * N * ((double)n * (n + 1) + 2 * n + 2 * n + n * (2 * d + 2) + 10 * n);
  for (int i = 0; i < NV; ++i)
    printf("%-22s %8.3f ms  %6.1f TFLOP/s-equiv\n", names[i], t[i] / 3, flops / (t[i] / 3 * 1e-3) / 1e12);
  return 0;
}
