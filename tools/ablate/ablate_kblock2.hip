// K block: VALU dot products (kernel_block_kernel) vs r² on MFMA (kernel_block_mfma_kernel), same
// data, interleaved (tools only).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/ablate/ablate_kblock2 tools/ablate/ablate_kblock2.hip
// Run on the GPU box: ./tools/ablate/ablate_kblock2 [n] [N] [d]   (d = 6 or 30)
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../optimobo_amd/csrc/omb_posterior.hip"

using namespace omb;

// The previous library kernel (VALU dot products), kept here as the baseline: each thread owns two
// adjacent candidates (16-byte non-temporal stores), each block 256 training rows.
template <int DP, int KIND>
__global__ __launch_bounds__(256) void kernel_block_kernel(GPDev g, int d, const double* __restrict__ Xc,
                                                           int64_t N, double* __restrict__ K, ExpCoef ec) {
  constexpr int kRows = kKBlockRows;
  const int64_t c = 2 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (c >= N) return;
  const bool two = (c + 1) < N;
  double b0[DP], b1[DP];
  double s0 = 0.0, s1 = 0.0;
#pragma unroll
  for (int j = 0; j < DP; ++j) {
    b0[j] = (j < d) ? Xc[c * d + j] / g.ls[j] : 0.0;
    b1[j] = (j < d && two) ? Xc[(c + 1) * d + j] / g.ls[j] : 0.0;
    s0 += b0[j] * b0[j];
    s1 += b1[j] * b1[j];
  }
  const int k0 = blockIdx.y * kRows;
  const int k1 = min(g.n, k0 + kRows);
  for (int k = k0; k < k1; ++k) {
    const double* xr = g.Xs + (int64_t)k * DP;
    double dot0 = 0.0, dot1 = 0.0;
#pragma unroll
    for (int j = 0; j < DP; ++j) {
      dot0 = fma(xr[j], b0[j], dot0);
      dot1 = fma(xr[j], b1[j], dot1);
    }
    const double xk = g.xsq[k];
    double v0, v1;
    kernel_of_r2_k_x2<KIND>(fma(-2.0, dot0, xk + s0), fma(-2.0, dot1, xk + s1), g.variance, ec, v0, v1);
    double* dst = K + (int64_t)k * N + c;
    if (two && ((N & 1) == 0)) {
      __builtin_nontemporal_store(d2{v0, v1}, reinterpret_cast<d2*>(dst));
    } else {
      __builtin_nontemporal_store(v0, dst);
      if (two) __builtin_nontemporal_store(v1, dst + 1);
    }
  }
}


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
  dim3 g1((unsigned)((N + 511) / 512), (unsigned)((n + kKBlockRows - 1) / kKBlockRows));
  dim3 g2((unsigned)((N + 63) / 64), (unsigned)((n + kKBlockRows - 1) / kKBlockRows));
  auto old_k = [&] { hipLaunchKernelGGL((kernel_block_kernel<DP, 0>), g1, dim3(256), 0, 0, g, d, Xc, N, K1, ec); };
  auto new_k = [&] { hipLaunchKernelGGL((kernel_block_mfma_kernel<DP, 0>), g2, dim3(256), 0, 0, g, d, Xc, N, K2, ec); };
  auto plain_k = [&] {
    hipLaunchKernelGGL((kernel_block_mfma_kernel<DP, 0, false>), g2, dim3(256), 0, 0, g, d, Xc, N, K2, ec);
  };
  float t1 = 0, t2 = 0, t3 = 0;
  for (int r = 0; r < 3; ++r) {
    t1 += time_ms(old_k, 5);
    t2 += time_ms(new_k, 5);
    t3 += time_ms(plain_k, 5);
  }
  printf("MFMA r2 with plain stores %.3f ms (%.0f GB/s)\n", t3 / 3, 8.0 * (n + d) * N / (t3 / 3 * 1e6));
  std::vector<double> h1((size_t)n * N), h2((size_t)n * N);
  CK(hipMemcpy(h1.data(), K1, h1.size() * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(h2.data(), K2, h2.size() * 8, hipMemcpyDeviceToHost));
  double md = 0;
  for (size_t i = 0; i < h1.size(); ++i) md = std::max(md, std::abs(h1[i] - h2[i]) / (std::abs(h1[i]) + 1e-300));
  const double bytes = 8.0 * (n + d) * N;
  printf("n=%d N=%lld d=%d  VALU dots %.3f ms (%.0f GB/s)  MFMA r2 %.3f ms (%.0f GB/s)  max rel diff %.2e\n", n,
         (long long)N, d, t1 / 3, bytes / (t1 / 3 * 1e6), t2 / 3, bytes / (t2 / 3 * 1e6), md);
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 512;
  const int64_t N = argc > 2 ? atoll(argv[2]) : (1 << 20);
  const int d = argc > 3 ? atoi(argv[3]) : 6;
  if (d == 6) bench<6>(n, N, d);
  else if (d == 30) bench<32>(n, N, d);
  else printf("d must be 6 or 30\n");
  return 0;
}
