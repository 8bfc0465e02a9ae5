// Ablation of the Thompson-step GEMM shapes (tools only; not part of the library): the library's
// gemm_kernel against tile variants and rocBLAS as an achievable-rate reference.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/ablate/ablate_gemm tools/ablate/ablate_gemm.hip -lrocblas
// Run on the GPU box: ./tools/ablate/ablate_gemm [N] [n]
//   SYRK   S (N×N, lower) −= VᵀV, V (n×N) row-major        (omb_posterior_samples: Σ = K** − VᵀV)
//   NN     V (n×N) = L⁻¹ (n×n) · K* (n×N)                   (V = L⁻¹K*)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#include <rocblas/rocblas.h>

#include "../../optimobo_amd/csrc/omb_gemm.hip"

using namespace omb;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)
#define RB(x) do { rocblas_status s_ = (x); if (s_ != rocblas_status_success) { printf("%s: %d\n", #x, (int)s_); exit(1);} } while (0)

// C (tile BM×BN per workgroup) = β·C + α·op(A)·op(B), waves of WM×WN, k-slabs of BK double-buffered in LDS.
template <int BM, int BN, int BK, int WM, int WN, bool TA, bool TB, bool LOWER>
__global__ __launch_bounds__((BM / WM) * (BN / WN) * 64) void gemmv_kernel(
    int64_t M, int64_t Nc, int64_t K, double alpha, const double* __restrict__ A, int64_t lda,
    const double* __restrict__ B, int64_t ldb, double beta, double* __restrict__ C, int64_t ldc) {
  constexpr int NWM = BM / WM, NWN = BN / WN, NT = NWM * NWN * 64;
  constexpr int FM = WM / 16, FN = WN / 16;
  constexpr int PA = BM + 2, PB = BN + 2;
  constexpr int LA = BM * BK / NT, LB = BN * BK / NT;
  static_assert(LA * NT == BM * BK && LB * NT == BN * BK, "slab loads");
  const int64_t m0 = (int64_t)blockIdx.y * BM, n0 = (int64_t)blockIdx.x * BN;
  if (LOWER && n0 >= m0 + BM) return;
  __shared__ double As[2][BK][PA];
  __shared__ double Bs[2][BK][PB];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / NWN, wn = wave % NWN;
  double ra[LA], rb[LB];
  auto fetch = [&](int64_t k0) {
#pragma unroll
    for (int e = 0; e < LA; ++e) {
      const int idx = tid + NT * e;
      const int am = TA ? (idx % BM) : (idx / BK), ak = TA ? (idx / BM) : (idx % BK);
      const int64_t gm = m0 + am, gk = k0 + ak;
      ra[e] = (gm < M && gk < K) ? (TA ? A[gk * lda + gm] : A[gm * lda + gk]) : 0.0;
    }
#pragma unroll
    for (int e = 0; e < LB; ++e) {
      const int idx = tid + NT * e;
      const int bn = TB ? (idx / BK) : (idx % BN), bk = TB ? (idx % BK) : (idx / BN);
      const int64_t gn = n0 + bn, gk = k0 + bk;
      rb[e] = (gn < Nc && gk < K) ? (TB ? B[gn * ldb + gk] : B[gk * ldb + gn]) : 0.0;
    }
  };
  auto stash = [&](int buf) {
#pragma unroll
    for (int e = 0; e < LA; ++e) {
      const int idx = tid + NT * e;
      As[buf][TA ? (idx / BM) : (idx % BK)][TA ? (idx % BM) : (idx / BK)] = ra[e];
    }
#pragma unroll
    for (int e = 0; e < LB; ++e) {
      const int idx = tid + NT * e;
      Bs[buf][TB ? (idx % BK) : (idx / BN)][TB ? (idx / BK) : (idx % BN)] = rb[e];
    }
  };
  d4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};
  fetch(0);
  stash(0);
  __syncthreads();
  int buf = 0;
  for (int64_t k0 = 0; k0 < K; k0 += BK) {
    const bool more = k0 + BK < K;
    if (more) fetch(k0 + BK);
#pragma unroll
    for (int ks = 0; ks < BK / 4; ++ks) {
      const int kk = 4 * ks + (lane >> 4);
      double a[FM], b[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) a[i] = As[buf][kk][WM * wm + 16 * i + (lane & 15)];
#pragma unroll
      for (int j = 0; j < FN; ++j) b[j] = Bs[buf][kk][WN * wn + 16 * j + (lane & 15)];
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (more) stash(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t row = m0 + WM * wm + 16 * i + (lane >> 4) + 4 * e;
        const int64_t col = n0 + WN * wn + 16 * j + (lane & 15);
        if (row < M && col < Nc && (!LOWER || col <= row)) {
          double v = alpha * acc[i][j][e];
          if (beta != 0.0) v = fma(beta, C[row * ldc + col], v);
          C[row * ldc + col] = v;
        }
      }
}

template <int BM, int BN, int BK, int WM, int WN, bool TA, bool TB, bool LOWER>
void gemmv(int64_t M, int64_t Nc, int64_t K, double alpha, const double* A, int64_t lda, const double* B, int64_t ldb,
           double beta, double* C, int64_t ldc) {
  dim3 grid((unsigned)((Nc + BN - 1) / BN), (unsigned)((M + BM - 1) / BM));
  hipLaunchKernelGGL((gemmv_kernel<BM, BN, BK, WM, WN, TA, TB, LOWER>), grid, dim3((BM / WM) * (BN / WN) * 64), 0, 0,
                     M, Nc, K, alpha, A, lda, B, ldb, beta, C, ldc);
}

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
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms * 1e3f / reps;
}

static double maxdiff_lower(const std::vector<double>& a, const std::vector<double>& b, int64_t N, bool lower) {
  double m = 0.0;
  for (int64_t i = 0; i < N; ++i)
    for (int64_t j = 0; j <= (lower ? i : N - 1); ++j) m = std::max(m, std::abs(a[i * N + j] - b[i * N + j]));
  return m;
}

int main(int argc, char** argv) {
  const int64_t N = argc > 1 ? atoll(argv[1]) : 3000;
  const int64_t n = argc > 2 ? atoll(argv[2]) : 512;
  std::vector<double> hV(n * N), hS(N * N), hL(n * n);
  srand(7);
  for (auto& v : hV) v = rand() / (double)RAND_MAX - 0.5;
  for (auto& v : hS) v = rand() / (double)RAND_MAX;
  for (auto& v : hL) v = rand() / (double)RAND_MAX - 0.5;
  double *V, *S, *S0, *L, *O;
  CK(hipMalloc(&V, n * N * 8));
  CK(hipMalloc(&S, N * N * 8));
  CK(hipMalloc(&S0, N * N * 8));
  CK(hipMalloc(&L, n * n * 8));
  CK(hipMalloc(&O, n * N * 8));
  CK(hipMemcpy(V, hV.data(), n * N * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(S0, hS.data(), N * N * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(L, hL.data(), n * n * 8, hipMemcpyHostToDevice));
  rocblas_handle h;
  RB(rocblas_create_handle(&h));
  const int reps = 10;
  const double syrk_flops = (double)N * (N + 1) * n;        // lower triangle
  const double nn_flops = 2.0 * n * n * N;

  struct V_ { const char* name; std::function<void()> f; bool lower_rowmajor; };
  const double m1 = -1.0, p1 = 1.0, z0 = 0.0;
  std::vector<V_> syrk = {
      {"library gemm_kernel 64x64 K16", [&] { CK(launch_gemm_tn_lower(0, N, n, -1.0, V, N, 1.0, S, N)); }, true},
      {"64x64 K32 (2x2 waves of 32x32)", [&] { gemmv<64, 64, 32, 32, 32, true, false, true>(N, N, n, -1.0, V, N, V, N, 1.0, S, N); }, true},
      {"128x128 K16 (2x2 waves of 64x64)", [&] { gemmv<128, 128, 16, 64, 64, true, false, true>(N, N, n, -1.0, V, N, V, N, 1.0, S, N); }, true},
      {"128x64 K16 (2x2 waves of 64x32)", [&] { gemmv<128, 64, 16, 64, 32, true, false, true>(N, N, n, -1.0, V, N, V, N, 1.0, S, N); }, true},
      {"64x64 K16 (1x1 wave 64x64)", [&] { gemmv<64, 64, 16, 64, 64, true, false, true>(N, N, n, -1.0, V, N, V, N, 1.0, S, N); }, true},
      {"128x128 K16 (4x2 waves of 32x64)", [&] { gemmv<128, 128, 16, 32, 64, true, false, true>(N, N, n, -1.0, V, N, V, N, 1.0, S, N); }, true},
      // rocBLAS, column-major view: S row-major lower = column-major upper; V row-major n×N = column-major N×n
      {"rocblas_dsyrk", [&] { RB(rocblas_dsyrk(h, rocblas_fill_upper, rocblas_operation_none, N, n, &m1, V, N, &p1, S, N)); }, true},
      {"rocblas_dgemm (full square)", [&] { RB(rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_transpose, N, N, n, &m1, V, N, V, N, &p1, S, N)); }, false},
  };
  std::vector<double> ref(N * N), got(N * N);
  for (size_t i = 0; i < syrk.size(); ++i) {
    CK(hipMemcpy(S, S0, N * N * 8, hipMemcpyDeviceToDevice));
    syrk[i].f();
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(i == 0 ? ref.data() : got.data(), S, N * N * 8, hipMemcpyDeviceToHost));
    double err = i == 0 ? 0.0 : maxdiff_lower(ref, got, N, true);
    float us = 0.f;
    for (int r = 0; r < 3; ++r) us += time_us(syrk[i].f, reps) / 3;
    printf("SYRK N=%lld n=%lld  %-36s %8.1f us  %6.1f TFLOP/s (lower-triangle flops)  max|diff| vs library %.2e\n",
           (long long)N, (long long)n, syrk[i].name, us, syrk_flops / (us * 1e-6) / 1e12, err);
  }
  std::vector<V_> nn = {
      {"library gemm_kernel 64x64 K16", [&] { CK(launch_gemm_nn(0, n, N, n, 1.0, L, n, V, N, 0.0, O, N)); }, false},
      {"64x64 K32", [&] { gemmv<64, 64, 32, 32, 32, false, false, false>(n, N, n, 1.0, L, n, V, N, 0.0, O, N); }, false},
      {"128x64 K16 (2x2 waves of 64x32)", [&] { gemmv<128, 64, 16, 64, 32, false, false, false>(n, N, n, 1.0, L, n, V, N, 0.0, O, N); }, false},
      {"64x128 K16 (2x2 waves of 32x64)", [&] { gemmv<64, 128, 16, 32, 64, false, false, false>(n, N, n, 1.0, L, n, V, N, 0.0, O, N); }, false},
      // row-major O = L·V  ⇔  column-major Oᵀ = Vᵀ·Lᵀ
      {"rocblas_dgemm", [&] { RB(rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_none, N, n, n, &p1, V, N, L, n, &z0, O, N)); }, false},
  };
  std::vector<double> oref(n * N), ogot(n * N);
  for (size_t i = 0; i < nn.size(); ++i) {
    nn[i].f();
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(i == 0 ? oref.data() : ogot.data(), O, n * N * 8, hipMemcpyDeviceToHost));
    double err = 0.0;
    if (i) for (int64_t j = 0; j < n * N; ++j) err = std::max(err, std::abs(oref[j] - ogot[j]));
    float us = 0.f;
    for (int r = 0; r < 3; ++r) us += time_us(nn[i].f, reps) / 3;
    printf("NN   n=%lld N=%lld  %-36s %8.1f us  %6.1f TFLOP/s  max|diff| vs library %.2e\n", (long long)n, (long long)N,
           nn[i].name, us, nn_flops / (us * 1e-6) / 1e12, err);
  }
  RB(rocblas_destroy_handle(h));
  return 0;
}
