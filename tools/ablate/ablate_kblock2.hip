// K block variants on the same data, interleaved (tools only): VALU dot products (kernel_block_kernel,
// the r01 baseline), r² on MFMA with 4 × 128-B store segments (kernel_block_mfma_kernel) and with the
// permlane16 swap to 2 × 256-B segments (kernel_block_swap_kernel), non-temporal and plain stores.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/ablate/ablate_kblock2 tools/ablate/ablate_kblock2.hip
// Run on the GPU box: ./tools/ablate/ablate_kblock2 [n] [N] [d]   (d = 6 or 30)
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "../../optimobo_amd/csrc/omb_posterior.hip"
#include "../../optimobo_amd/csrc/omb_wide.hip"

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
  auto mfma_nt = [&] { hipLaunchKernelGGL((kernel_block_mfma_kernel<DP, 0>), g2, dim3(256), 0, 0, g, d, Xc, N, K2, ec); };
  auto mfma_pl = [&] { hipLaunchKernelGGL((kernel_block_mfma_kernel<DP, 0, false>), g2, dim3(256), 0, 0, g, d, Xc, N, K2, ec); };
  dim3 g3((unsigned)((N + 127) / 128), (unsigned)((n + kblock_rows(DP) - 1) / kblock_rows(DP)));
  auto pipe_nt = [&] { hipLaunchKernelGGL((kernel_block_pipe_kernel<DP, 0>), g3, dim3(512), 0, 0, g, d, Xc, N, K1, ec); };
  auto pipe_pl = [&] { hipLaunchKernelGGL((kernel_block_pipe_kernel<DP, 0, false>), g3, dim3(512), 0, 0, g, d, Xc, N, K1, ec); };
  auto swap_nt = [&] { hipLaunchKernelGGL((kernel_block_pipe_kernel<DP, 0, true, true>), g3, dim3(512), 0, 0, g, d, Xc, N, K1, ec); };
  auto swap_pl = [&] { hipLaunchKernelGGL((kernel_block_pipe_kernel<DP, 0, false, true>), g3, dim3(512), 0, 0, g, d, Xc, N, K1, ec); };
  auto trans_nt = [&] { hipLaunchKernelGGL((kernel_block_pipe_kernel<DP, 0, true, false, true>), g3, dim3(512), 0, 0, g, d, Xc, N, K1, ec); };
  auto trans_pl = [&] { hipLaunchKernelGGL((kernel_block_pipe_kernel<DP, 0, false, false, true>), g3, dim3(512), 0, 0, g, d, Xc, N, K1, ec); };
  float t[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int r = 0; r < 3; ++r) {
    t[0] += time_ms(old_k, 5);
    t[1] += time_ms(mfma_nt, 5);
    t[2] += time_ms(mfma_pl, 5);
    t[3] += time_ms(swap_nt, 5);
    t[4] += time_ms(swap_pl, 5);
    t[5] += time_ms(pipe_nt, 5);
    t[6] += time_ms(pipe_pl, 5);
    t[7] += time_ms(trans_nt, 5);
    t[8] += time_ms(trans_pl, 5);
  }
  const char* names[9] = {"VALU dots (r01 baseline)", "MFMA r2, 4x128-B rows, nt (r01 library)", "MFMA r2, 4x128-B rows, plain",
                          "LDS-staged + permlane16 swap, 2x256-B rows, nt", "LDS-staged + permlane16 swap, 2x256-B rows, plain",
                          "Xf staged in LDS + base-pointer stores, nt", "Xf staged in LDS + base-pointer stores, plain",
                          "LDS transpose, 1-KB row stores (b128), nt", "LDS transpose, 1-KB row stores (b128), plain"};
  const double bytes = 8.0 * (n + d) * N + 8.0 * n * (d + 1);
  for (int i = 0; i < 9; ++i)
    printf("n=%d N=%lld d=%d  %-48s %.3f ms  %.0f GB/s  (%.3f of 8 TB/s)\n", n, (long long)N, d, names[i], t[i] / 3,
           bytes / (t[i] / 3 * 1e6), bytes / (t[i] / 3 * 1e6) / 8000.0);
  std::vector<double> h1((size_t)n * N), h2((size_t)n * N);
  mfma_nt();
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(h2.data(), K2, h2.size() * 8, hipMemcpyDeviceToHost));
  for (int v = 0; v < 3; ++v) {
    CK(hipMemset(K1, 0, h1.size() * 8));
    if (v == 0) swap_nt(); else if (v == 1) pipe_nt(); else trans_nt();
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h1.data(), K1, h1.size() * 8, hipMemcpyDeviceToHost));
    size_t ndiff = 0;
    double emax = 0.0;
    for (size_t i = 0; i < h1.size(); ++i) {
      ndiff += (h1[i] != h2[i]);
      emax = fmax(emax, fabs(h1[i] - h2[i]) / fmax(fabs(h2[i]), 1e-300));
    }
    // d ≤ 8: same arithmetic (must be 0); d > 8 the pipe kernel sums ‖x*/ℓ‖² by lane groups (last bits)
    printf("%s vs r01 kernel: %zu of %zu elements differ, max rel %.2e\n", v == 2 ? "trans" : (v ? "pipe" : "swap"), ndiff,
           h1.size(), emax);
  }
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 512;
  const int64_t N = argc > 2 ? atoll(argv[2]) : (1 << 20);
  const int d = argc > 3 ? atoi(argv[3]) : 6;
  if (d == 6) bench<6>(n, N, d);
  else if (d == 30) bench<32>(n, N, d);
  else if (d == 2) bench<2>(n, N, d);
  else printf("d must be 2, 6 or 30\n");
  return 0;
}
