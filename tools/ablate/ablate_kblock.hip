// K-block (omb_kernel_block) layout variants, timed on the same data (tools only).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/ablate/ablate_kblock tools/ablate/ablate_kblock.hip
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../optimobo_amd/csrc/omb_posterior.hip"
#include "../../optimobo_amd/csrc/omb_wide.hip"

using namespace omb;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)

// CPT candidates per thread (2 or 4), ROWS rows per block, NT = nontemporal stores.
template <int DP, int CPT, int ROWS, bool NTS>
__global__ __launch_bounds__(256) void kb_variant(GPDev g, int d, const double* __restrict__ Xc, int64_t N,
                                                  double* __restrict__ K) {
  const int64_t c = CPT * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (c + CPT > N) return;
  double b[CPT][DP], s[CPT];
#pragma unroll
  for (int q = 0; q < CPT; ++q) {
    s[q] = 0.0;
#pragma unroll
    for (int j = 0; j < DP; ++j) {
      b[q][j] = (j < d) ? Xc[(c + q) * d + j] / g.ls[j] : 0.0;
      s[q] += b[q][j] * b[q][j];
    }
  }
  const int k0 = blockIdx.y * ROWS;
  const int k1 = min(g.n, k0 + ROWS);
  for (int k = k0; k < k1; ++k) {
    const double* xr = g.Xs + (int64_t)k * DP;
    double v[CPT];
#pragma unroll
    for (int q = 0; q < CPT; ++q) {
      double dot = 0.0;
#pragma unroll
      for (int j = 0; j < DP; ++j) dot = fma(xr[j], b[q][j], dot);
      v[q] = kernel_of_r2<OMB_KERNEL_MATERN52>(fma(-2.0, dot, g.xsq[k] + s[q]), g.variance);
    }
    double* dst = K + (int64_t)k * N + c;
#pragma unroll
    for (int q = 0; q < CPT; q += 2) {
      d2 w = d2{v[q], v[q + 1]};
      if constexpr (NTS)
        __builtin_nontemporal_store(w, reinterpret_cast<d2*>(dst + q));
      else
        *reinterpret_cast<d2*>(dst + q) = w;
    }
  }
}

template <int CPT, int ROWS, bool NTS>
float run(const GPDev& g, const double* Xc, int64_t N, double* K, int n) {
  dim3 grid((unsigned)(N / (256 * CPT)), (unsigned)((n + ROWS - 1) / ROWS));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((kb_variant<6, CPT, ROWS, NTS>), grid, dim3(256), 0, 0, g, 6, Xc, N, K);
  CK(hipEventRecord(e0));
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((kb_variant<6, CPT, ROWS, NTS>), grid, dim3(256), 0, 0, g, 6, Xc, N, K);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / 5;
}

int main() {
  const int n = 512, DP = 6;
  const int64_t N = 1 << 20;
  std::vector<double> hXs(n * DP), hxsq(n), hls(DP, 1.0), hXc(N * 6);
  srand(2);
  for (auto& v : hXs) v = rand() / (double)RAND_MAX;
  for (int k = 0; k < n; ++k) {
    double s = 0;
    for (int j = 0; j < DP; ++j) s += hXs[k * DP + j] * hXs[k * DP + j];
    hxsq[k] = s;
  }
  for (auto& v : hXc) v = rand() / (double)RAND_MAX;
  double *Xs, *xsq, *ls, *Xc, *K;
  CK(hipMalloc(&Xs, hXs.size() * 8)); CK(hipMalloc(&xsq, n * 8)); CK(hipMalloc(&ls, DP * 8));
  CK(hipMalloc(&Xc, hXc.size() * 8)); CK(hipMalloc(&K, (size_t)n * N * 8));
  CK(hipMemcpy(Xs, hXs.data(), hXs.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(xsq, hxsq.data(), n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(ls, hls.data(), DP * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(Xc, hXc.data(), hXc.size() * 8, hipMemcpyHostToDevice));
  GPDev g{Xs, xsq, nullptr, nullptr, ls, 1.0, n, n / 16, 0, 0};
  const double bytes = 8.0 * (n + 6) * N;
  const char* names[] = {"cpt2 rows64", "cpt2 rows64 nt", "cpt2 rows128 nt", "cpt2 rows256 nt", "cpt2 rows512 nt",
                         "cpt2 rows32 nt", "cpt2 rows16 nt"};
  float t[7] = {0};
  for (int r = 0; r < 3; ++r) {
    t[0] += run<2, 64, false>(g, Xc, N, K, n);
    t[1] += run<2, 64, true>(g, Xc, N, K, n);
    t[2] += run<2, 128, true>(g, Xc, N, K, n);
    t[3] += run<2, 256, true>(g, Xc, N, K, n);
    t[4] += run<2, 512, true>(g, Xc, N, K, n);
    t[5] += run<2, 32, true>(g, Xc, N, K, n);
    t[6] += run<2, 16, true>(g, Xc, N, K, n);
  }
  for (int i = 0; i < 7; ++i) printf("%-18s %7.3f ms  %7.1f GB/s\n", names[i], t[i] / 3, bytes / (t[i] / 3 * 1e-3) / 1e9);
  return 0;
}
