// Ablation timing of posterior_kernel variants (tools only; not part of the library).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/ablate/ablate_posterior tools/ablate/ablate_posterior.hip
// Run on the GPU box: ./tools/ablate/ablate_posterior [n] [N] [d] [n_obj]
//   d = 6: config 3 variants (RT 4, CT 4); d = 30: config 5 variants (RT 8, CT 2, candidates in LDS)
// Variants are timed interleaved in one process (cdna_hip_programming.md §5.4 rule 24).
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>

// phase timestamps (100 MHz constant clock) and hardware id of every workgroup of posterior_tile_kernel
__device__ unsigned long long g_ptrace[4096][8];
#define OMB_POST_TRACE(id)                                                              \
  do {                                                                                  \
    if (threadIdx.x == 0) {                                                             \
      const unsigned wg_ = blockIdx.y * gridDim.x + blockIdx.x;                         \
      if (wg_ < 4096) {                                                                 \
        g_ptrace[wg_][id] = __builtin_amdgcn_s_memrealtime();                           \
        if ((id) == 0) {                                                                \
          unsigned hw_, xcc_;                                                           \
          asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_));             \
          asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_));           \
          g_ptrace[wg_][7] = ((unsigned long long)xcc_ << 32) | hw_;                    \
        }                                                                               \
      }                                                                                 \
    }                                                                                   \
  } while (0)

#include "../../optimobo_amd/csrc/omb_posterior.hip"
#include "../../optimobo_amd/csrc/omb_wide.hip"

using namespace omb;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)

struct Bench {
  GPArgs a;
  const double* Xc;
  int64_t N;
  int n_obj;
  double *mu, *var;
};

template <int RT, int CT, int NW, int ABL, int DP = 6, int WPE = NW / 4>
float run(const Bench& b, int reps) {
  dim3 grid((unsigned)((b.N + 16 * CT - 1) / (16 * CT)), b.n_obj);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((posterior_kernel<RT, CT, DP, 0, NW, ABL, WPE>), grid, dim3(64 * NW), 0, 0, b.a, b.Xc, b.N, b.mu,
                     b.var);
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((posterior_kernel<RT, CT, DP, 0, NW, ABL, WPE>), grid, dim3(64 * NW), 0, 0, b.a, b.Xc, b.N, b.mu,
                       b.var);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms / reps;
}


template <int RMAX, int CT, int ABL, int DP = 6>
float run_tile(const Bench& b, int reps) {
  dim3 grid((unsigned)((b.N + 16 * CT - 1) / (16 * CT)), b.n_obj);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((posterior_tile_kernel<RMAX, CT, DP, 0, ABL>), grid, dim3(512), 0, 0, b.a, b.Xc, b.N, b.mu, b.var);
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((posterior_tile_kernel<RMAX, CT, DP, 0, ABL>), grid, dim3(512), 0, 0, b.a, b.Xc, b.N, b.mu,
                       b.var);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms / reps;
}

template <int ABL, int NW = 8, bool XL = false, int DP = 6>
float run_reg(const Bench& b, int reps) {
  const dim3 grid = reg_grid(b.N, b.n_obj, NW, NW == 8 ? 2 : 1);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((posterior_reg_kernel<8, DP, 0, NW, XL, ABL>), grid, dim3(64 * NW), 0, 0, b.a, b.Xc, b.N, b.mu, b.var);
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((posterior_reg_kernel<8, DP, 0, NW, XL, ABL>), grid, dim3(64 * NW), 0, 0, b.a, b.Xc, b.N, b.mu, b.var);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms / reps;
}

// Accuracy of the table-driven Matern transforms against a long-double host reference.
__global__ void matern_acc_kernel(const double* r2, int M, ExpCoef ec, double* out) {
  __shared__ double t64[64], t256[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) {
    t256[i] = kExp2Tab256[i];
    if (i < 64) t64[i] = kExp2Tab64[i];
  }
  __syncthreads();
  const double pm[3] = {1.0, kSqrt5, kFiveThirds};
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; 2 * i + 1 < M; i += gridDim.x * blockDim.x) {
    double a, b;
    kernel_of_r2_tab_x2<0>(r2[2 * i], r2[2 * i + 1], pm, ec, t64, a, b);
    out[2 * i] = a; out[2 * i + 1] = b;
    matern_r2_tab256_x2<false>(r2[2 * i], r2[2 * i + 1], pm, ec, t256, a, b);
    out[M + 2 * i] = a; out[M + 2 * i + 1] = b;
    matern_r2_tab256_x2<true>(r2[2 * i], r2[2 * i + 1], pm, ec, t256, a, b);
    out[2 * M + 2 * i] = a; out[2 * M + 2 * i + 1] = b;
  }
}

void matern_accuracy() {
  const int M = 1 << 20;
  std::vector<double> r2(M), out(3 * M);
  for (int i = 0; i < M; ++i) {
    // half log-uniform over [1e-20, 1e4], half uniform over [0, 40]
    r2[i] = (i & 1) ? 40.0 * (i >> 1) / (M / 2) : pow(10.0, -20.0 + 24.0 * (i >> 1) / (M / 2));
  }
  r2[0] = 0.0;
  double *dr2, *dout;
  CK(hipMalloc(&dr2, M * 8)); CK(hipMalloc(&dout, 3 * M * 8));
  CK(hipMemcpy(dr2, r2.data(), M * 8, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(matern_acc_kernel, dim3(1024), dim3(256), 0, 0, dr2, M, exp_coef(), dout);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(out.data(), dout, 3 * M * 8, hipMemcpyDeviceToHost));
  const char* names[3] = {"tab64 (library default)", "tab256", "tab256 short sqrt"};
  for (int v = 0; v < 3; ++v) {
    double worst = 0, worst_r2 = 0, sum = 0;
    for (int i = 0; i < M; ++i) {
      long double r = sqrtl((long double)r2[i]);
      long double ref = (1.0L + sqrtl(5.0L) * r + 5.0L / 3.0L * r * r) * expl(-sqrtl(5.0L) * r);
      if (ref < 1e-300L) continue;
      double e = (double)fabsl(((long double)out[v * M + i] - ref) / ref);
      sum += e;
      if (e > worst) { worst = e; worst_r2 = r2[i]; }
    }
    printf("accuracy %-24s max rel err %.3e (%.2f ulp) at r2 = %.3e, mean %.3e\n", names[v], worst,
           worst / 1.1102230246251565e-16, worst_r2, sum / M);
  }
  CK(hipFree(dr2)); CK(hipFree(dout));
}

// Phase timeline of the library's n ≤ 128 tile kernel: per-workgroup durations of prologue, generation,
// barrier wait, multiply and reduction, and how many workgroups are resident per CU over time.
void trace_tile(const Bench& b) {
  dim3 grid((unsigned)((b.N + 63) / 64), b.n_obj);
  const unsigned nwg = grid.x * grid.y;
  if (nwg > 4096) { printf("trace: too many workgroups\n"); return; }
  for (int rep = 0; rep < 3; ++rep)
    hipLaunchKernelGGL((posterior_tile_kernel<8, 4, 6, 0, 0>), grid, dim3(512), 0, 0, b.a, b.Xc, b.N, b.mu, b.var);
  CK(hipDeviceSynchronize());
  std::vector<unsigned long long> t(4096 * 8);
  CK(hipMemcpyFromSymbol(t.data(), HIP_SYMBOL(g_ptrace), t.size() * 8));
  unsigned long long t0 = ~0ull, t1 = 0;
  for (unsigned w = 0; w < nwg; ++w) { t0 = std::min(t0, t[w * 8]); t1 = std::max(t1, t[w * 8 + 5]); }
  const char* ph[5] = {"prologue (etab, candidates)", "generation", "barrier wait", "multiply", "reduction + store"};
  printf("tile kernel trace: %u workgroups, span %.2f us (first start to last end)\n", nwg, (t1 - t0) / 100.0);
  for (int p = 0; p < 5; ++p) {
    std::vector<double> d;
    for (unsigned w = 0; w < nwg; ++w) d.push_back((t[w * 8 + p + 1] - t[w * 8 + p]) / 100.0);
    std::sort(d.begin(), d.end());
    double s = 0; for (double x : d) s += x;
    printf("  %-28s mean %6.2f us  p10 %6.2f  p50 %6.2f  p90 %6.2f\n", ph[p], s / d.size(), d[d.size() / 10], d[d.size() / 2],
           d[d.size() * 9 / 10]);
  }
  std::vector<double> life;
  for (unsigned w = 0; w < nwg; ++w) life.push_back((t[w * 8 + 5] - t[w * 8]) / 100.0);
  std::sort(life.begin(), life.end());
  printf("  workgroup lifetime p50 %.2f us; sum of lifetimes / span = %.1f workgroups resident on average\n",
         life[life.size() / 2], [&] { double s = 0; for (double x : life) s += x; return s; }() / ((t1 - t0) / 100.0));
  // start-time histogram in 2-us bins
  printf("  starts per 2-us bin:");
  for (unsigned long long s = t0; s < t1; s += 200) {
    int c = 0;
    for (unsigned w = 0; w < nwg; ++w) c += (t[w * 8] >= s && t[w * 8] < s + 200);
    printf(" %d", c);
  }
  printf("\n");
}

// Phase timeline of the library's counter-ring kernel (n > 256): prologue, chunk pipeline, final
// barrier, reduction; gaps between consecutive workgroups on the same CU (XCC + SE/SH/CU id).
template <int RT, int CT>
void trace_ring(const Bench& b) {
  dim3 grid((unsigned)((b.N + 16 * CT - 1) / (16 * CT)), b.n_obj);
  const unsigned nwg = grid.x * grid.y;
  if (nwg > 4096) { printf("trace: too many workgroups (%u)\n", nwg); return; }
  for (int rep = 0; rep < 3; ++rep)
    hipLaunchKernelGGL((posterior_kernel<RT, CT, 6, 0, 8, 0>), grid, dim3(512), 0, 0, b.a, b.Xc, b.N, b.mu, b.var);
  CK(hipDeviceSynchronize());
  std::vector<unsigned long long> t(4096 * 8);
  CK(hipMemcpyFromSymbol(t.data(), HIP_SYMBOL(g_ptrace), t.size() * 8));
  unsigned long long t0 = ~0ull, t1 = 0;
  for (unsigned w = 0; w < nwg; ++w) { t0 = std::min(t0, t[w * 8]); t1 = std::max(t1, t[w * 8 + 4]); }
  const char* ph[4] = {"prologue (table, candidates, counters)", "chunk pipeline", "final barrier", "reduction + store"};
  printf("ring kernel RT%d CT%d trace: %u workgroups, span %.2f us\n", RT, CT, nwg, (t1 - t0) / 100.0);
  for (int p = 0; p < 4; ++p) {
    std::vector<double> d;
    for (unsigned w = 0; w < nwg; ++w) d.push_back((t[w * 8 + p + 1] - t[w * 8 + p]) / 100.0);
    std::sort(d.begin(), d.end());
    double s = 0; for (double x : d) s += x;
    printf("  %-40s mean %7.2f us  p10 %7.2f  p50 %7.2f  p90 %7.2f\n", ph[p], s / d.size(), d[d.size() / 10],
           d[d.size() / 2], d[d.size() * 9 / 10]);
  }
  // per CU: sort its workgroups by start, gap = next start − previous end
  std::vector<std::pair<unsigned long long, unsigned>> byc;
  for (unsigned w = 0; w < nwg; ++w) {
    const unsigned long long hw = t[w * 8 + 7];
    const unsigned cu = (unsigned)((hw >> 8) & 0xf), sh = (unsigned)((hw >> 12) & 1), se = (unsigned)((hw >> 13) & 7);
    const unsigned xcc = (unsigned)(hw >> 32) & 0xf;
    byc.push_back({((unsigned long long)((xcc << 8) | (se << 5) | (sh << 4) | cu) << 40) | (t[w * 8] - t0), w});
  }
  std::sort(byc.begin(), byc.end());
  std::vector<double> gaps;
  unsigned ncu = 0;
  for (size_t i = 0; i < byc.size(); ++i) {
    if (i == 0 || (byc[i].first >> 40) != (byc[i - 1].first >> 40)) { ++ncu; continue; }
    const unsigned prev = byc[i - 1].second, cur = byc[i].second;
    gaps.push_back(((double)t[cur * 8] - (double)t[prev * 8 + 4]) / 100.0);
  }
  std::sort(gaps.begin(), gaps.end());
  double s = 0; for (double x : gaps) s += x;
  if (!gaps.empty())
    printf("  %u CUs seen; start of next minus end of previous workgroup on a CU: mean %.2f us p10 %.2f p50 %.2f p90 %.2f\n",
           ncu, s / gaps.size(), gaps[gaps.size() / 10], gaps[gaps.size() / 2], gaps[gaps.size() * 9 / 10]);
}

struct Variant {
  const char* name;
  float (*fn)(const Bench&, int);
};

int main(int argc, char** argv) {
  int n = argc > 1 ? atoi(argv[1]) : 512;
  int64_t N = argc > 2 ? atoll(argv[2]) : (1 << 20);
  const int d = argc > 3 ? atoi(argv[3]) : 6;
  const int n_obj = argc > 4 ? atoi(argv[4]) : 2;
  if (d != 6 && d != 30) { printf("d must be 6 or 30\n"); return 1; }
  const int DP = d == 6 ? 6 : 32;
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
  CK(hipMalloc(&mu, 3 * N * 8)); CK(hipMalloc(&var, 3 * N * 8));
  if (n_obj < 1 || n_obj > 3) { printf("n_obj must be 1..3\n"); return 1; }
  CK(hipMemcpy(Xs, hXs.data(), hXs.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(xsq, hxsq.data(), n_pad * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(al, ha.data(), n_pad * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(Lp, hL.data(), hL.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(ls, hls.data(), DP * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(Xc, hXc.data(), hXc.size() * 8, hipMemcpyHostToDevice));
  Bench b{};
  double* Xf;
  CK(hipMalloc(&Xf, packed_X_size(n_pad, DP) * 8));
  CK(launch_pack_x(0, d, DP, n_pad, Xs, xsq, Xf));
  for (int o = 0; o < 3; ++o) b.a.gp[o] = GPDev{Xs, xsq, al, Lp, ls, 1.0, n, R, 0, 0, Xf};
  b.a.d = d;
  b.a.DP = DP;
  b.a.ec = exp_coef();
  b.a.spin_limit = kDefaultSpinLimit;
  b.Xc = Xc;
  b.N = N;
  b.n_obj = n_obj;
  b.mu = mu;
  b.var = var;
  const Variant wide[] = {
      {"default RT8 CT2 (MFMA gen)", run<8, 2, 8, 0, 32>},
      {"16 waves RT4 CT2 (4 waves/SIMD)", run<4, 2, 16, 0, 32>},
      {"RT8 CT1, 4 waves/SIMD bound", run<8, 1, 8, 0, 32, 4>},
      {"default 2", run<8, 2, 8, 0, 32>},
      {"16 waves RT4 CT2 2", run<4, 2, 16, 0, 32>},
      {"RT8 CT1, 4 waves/SIMD bound 2", run<8, 1, 8, 0, 32, 4>},
      {"default 3", run<8, 2, 8, 0, 32>},
      {"16 waves RT4 CT2 3", run<4, 2, 16, 0, 32>},
      {"default 4", run<8, 2, 8, 0, 32>},
  };
  const Variant narrow[] = {
      {"RT4 CT2 4 waves/SIMD (library)", run<4, 2, 8, 0, 6, 4>},
      {"RT4 CT2 library, IEXP", run<4, 2, 8, 524288, 6, 4>},
      {"RT4 CT2 library 1b", run<4, 2, 8, 0, 6, 4>},
      {"RT4 CT2 library, IEXP 2", run<4, 2, 8, 524288, 6, 4>},
      {"16 waves RT2 CT4 (1 wg/CU, 4 waves/SIMD)", run<2, 4, 16, 0>},
      {"RT4 CT2 library 2", run<4, 2, 8, 0, 6, 4>},
      {"16 waves RT2 CT4 2", run<2, 4, 16, 0>},
      {"RT4 CT2 library 3", run<4, 2, 8, 0, 6, 4>},
      {"16 waves RT2 CT4 3", run<2, 4, 16, 0>},
      {"RT4 CT2 library 4", run<4, 2, 8, 0, 6, 4>},
  };
  // n ≤ 256 (configs 2 and 4): the library launches RT = 2 (n ≤ 256) or 1 (n ≤ 128), CT = 4, barrier pipeline
  const Variant small128[] = {
      {"reg16 library (warm-up slot)", run_reg<0, 16, true>},
      {"reg16 library", run_reg<0, 16, true>},
      {"ring RT1 CT4, 4 waves/SIMD (2 wg/CU)", run<1, 4, 8, 0, 6, 4>},
      {"ring RT1 CT2, 6 waves/SIMD (3 wg/CU)", run<1, 2, 8, 0, 6, 6>},
      {"ring RT1 CT2, 8 waves/SIMD (4 wg/CU)", run<1, 2, 8, 0, 6, 8>},
      {"reg16 library 2", run_reg<0, 16, true>},
      {"ring RT1 CT4, 4 waves/SIMD 2", run<1, 4, 8, 0, 6, 4>},
      {"ring RT1 CT2, 6 waves/SIMD 2", run<1, 2, 8, 0, 6, 6>},
      {"ring RT1 CT2, 8 waves/SIMD 2", run<1, 2, 8, 0, 6, 8>},
      {"reg16 library 3", run_reg<0, 16, true>},
      {"tile RMAX8 CT4", run_tile<8, 4, 0>},
  };
  const Variant small256[] = {
      {"(warm-up) library", run<2, 2, 8, 0, 6, 6>},
      {"RT2 CT2 6 waves/SIMD (library)", run<2, 2, 8, 0, 6, 6>},
      {"RT2 CT2 6w, IEXP", run<2, 2, 8, 524288, 6, 6>},
      {"RT2 CT2 6w library 1b", run<2, 2, 8, 0, 6, 6>},
      {"RT2 CT2 6w, IEXP 2", run<2, 2, 8, 524288, 6, 6>},
      {"RT2 CT2 6w, tab64 exp (16384)", run<2, 2, 8, 16384, 6, 6>},
      {"RT2 CT1, 8 waves/SIMD bound", run<2, 1, 8, 0, 6, 8>},
      {"RT2 CT1, 6 waves/SIMD bound", run<2, 1, 8, 0, 6, 6>},
      {"RT2 CT2 6w library 2", run<2, 2, 8, 0, 6, 6>},
      {"RT2 CT1, 6 waves/SIMD bound 2", run<2, 1, 8, 0, 6, 6>},
      {"RT2 CT1, 8 waves/SIMD bound 2", run<2, 1, 8, 0, 6, 8>},
      {"RT2 CT2 6w, tab64 exp 2", run<2, 2, 8, 16384, 6, 6>},
      {"RT2 CT2 6w library 3", run<2, 2, 8, 0, 6, 6>},
  };



  const Variant small[] = {
      {"RT2 CT4 barrier (library n<=256)", run<2, 4, 8, 32>},
      {"RT2 CT4 counter ring", run<2, 4, 8, 0>},
      {"RT2 CT2 barrier", run<2, 2, 8, 32>},
      {"RT2 CT2 counter ring", run<2, 2, 8, 0>},
      {"RT1 CT4 16 waves barrier", run<1, 4, 16, 32>},
      {"RT1 CT2 16 waves ring", run<1, 2, 16, 0>},
      {"RT4 CT4 counter ring", run<4, 4, 8, 0>},
      {"RT1 CT4 barrier (library n<=128)", run<1, 4, 8, 32>},
      {"RT1 CT2 counter ring", run<1, 2, 8, 0>},
      {"RT1 CT2 barrier", run<1, 2, 8, 32>},
  };
  matern_accuracy();
  if (d == 6 && n <= 128) trace_tile(b);
  if (d == 6 && n > 256) trace_ring<4, 4>(b);
  if (d == 6 && n > 128 && n <= 256) trace_ring<2, 2>(b);
  const bool is_small = d == 6 && n <= 256;
  (void)small;
  const Variant* vs = is_small ? (n <= 128 ? small128 : small256) : (d == 6 ? narrow : wide);
  const int NV = is_small ? (n <= 128 ? (int)(sizeof(small128) / sizeof(small128[0]))
                                      : (int)(sizeof(small256) / sizeof(small256[0])))
                          : (d == 6 ? (int)(sizeof(narrow) / sizeof(narrow[0])) : (int)(sizeof(wide) / sizeof(wide[0])));
  std::vector<float> t(NV, 0.f);
  for (int round = 0; round < 3; ++round)
    for (int i = 0; i < NV; ++i) t[i] += vs[i].fn(b, 5);
  // outputs of every full variant against the default variant (max relative difference, μ and σ²)
  {
    std::vector<double> m0(n_obj * N), v0(n_obj * N), m1(n_obj * N), v1(n_obj * N);
    vs[0].fn(b, 1);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(m0.data(), mu, n_obj * N * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(v0.data(), var, n_obj * N * 8, hipMemcpyDeviceToHost));
    for (int i = 1; i < NV; ++i) {
      if (strstr(vs[i].name, "only") || strstr(vs[i].name, "const") || strstr(vs[i].name, "no ")) continue;
      vs[i].fn(b, 1);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(m1.data(), mu, n_obj * N * 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(v1.data(), var, n_obj * N * 8, hipMemcpyDeviceToHost));
      double em = 0, ev = 0;
      for (int64_t j = 0; j < n_obj * N; ++j) {
        em = fmax(em, fabs(m1[j] - m0[j]) / fmax(fabs(m0[j]), 1e-300));
        ev = fmax(ev, fabs(v1[j] - v0[j]) / fmax(fabs(v0[j]), 1e-300));
      }
      printf("vs default: %-26s mu max rel %.2e  var max rel %.2e\n", vs[i].name, em, ev);
      if (em > 1e-10 || ev > 1e-10) {       // where a variant disagrees: first cases, counts by lane slot
        int64_t bad = 0, shown = 0, by16[16] = {0};
        for (int64_t j = 0; j < n_obj * N; ++j) {
          const bool w = fabs(m1[j] - m0[j]) > 1e-10 * fmax(fabs(m0[j]), 1e-300) ||
                         fabs(v1[j] - v0[j]) > 1e-10 * fmax(fabs(v0[j]), 1e-300);
          if (!w) continue;
          ++bad;
          ++by16[(j % N) % 16];
          if (shown++ < 6)
            printf("    obj %lld cand %lld (tile %lld): mu %.6e vs %.6e  var %.6e vs %.6e\n", (long long)(j / N),
                   (long long)(j % N), (long long)((j % N) / 16), m1[j], m0[j], v1[j], v0[j]);
        }
        printf("    %lld of %lld disagree; by candidate %% 16:", (long long)bad, (long long)(n_obj * N));
        for (int q = 0; q < 16; ++q) printf(" %lld", (long long)by16[q]);
        printf("\n");
      }
    }
  }
  double flops = (double)n_obj * N * ((double)n * (n + 1) + 2 * n + 2 * n + n * (2 * d + 2) + 10 * n);
  for (int i = 0; i < NV; ++i)
    printf("%-26s %8.3f ms  %6.1f TFLOP/s-equiv\n", vs[i].name, t[i] / 3, flops / (t[i] / 3 * 1e-3) / 1e12);
  return 0;
}
