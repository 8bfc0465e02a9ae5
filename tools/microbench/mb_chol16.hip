// Cycles of the 16×16 diagonal-tile factor (chol16_factor, omb_linalg.hip) in one wave, alone on a CU, for the
// variants of its column update (tools only).  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/microbench/mb_chol16 tools/microbench/mb_chol16.hip
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../optimobo_amd/csrc/omb_linalg.hip"
#include "../../optimobo_amd/csrc/omb_wide.hip"
#include "../../optimobo_amd/csrc/omb_gemm.hip"

using namespace omb;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)

// Round 4 measured VAR 0 (the compiler's v_mov_b64_dpp + 2 fma, kept in omb_linalg.hip) against an inline-asm
// v_fmac_f64_dpp form (3,188 vs 3,784 cycles, profiles/r04_f_mb_chol16.txt); the asm form was removed from the library.
// Round 5 variants (where the cycles go; profiles/r05_k_mb_chol16.txt).  Variant 1 alone is 11% faster here, but put
// into the library it made the persistent launch 1.5-2% slower (interleaved A/B, profiles/r05_n_chol16_ab.txt), so
// the library keeps variant 0:
//   1  the pivot test off the chain (rsq of dj as is; a non-positive pivot gives NaNs, flagged as before)
//   2  1 + the next pivot from 1/d_j (v_rcp + 2 Newton steps) instead of from 1/sqrt(d_j) (bits change)
//   3  no x (inverse) updates: the factor's share of the issue (output W wrong)
//   4  no updates past the two rows the pivot chain reads (output wrong): the chain alone
template <int VAR>
__device__ __forceinline__ int chol16_var(double (&a)[16], double (&x)[16]) {
  if constexpr (VAR == 0) {
    return chol16_factor(a, x);
  } else {
    int bad = 0;
    double dj = readlane_f64(a[0], 0);
    static_for<0, 16>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      double a1 = 0.0, ap = 0.0;
      if constexpr (j < 15) {
        a1 = readlane_f64(a[j], j + 1);
        ap = readlane_f64(a[j + 1], j + 1);
      }
      if (!(dj > 0.0) && bad == 0) bad = j + 1;
      const double y0 = __builtin_amdgcn_rsq(dj);
      const double hd = 0.5 * dj;
      const double y1 = fma(y0, fma(-hd * y0, y0, 0.5), y0);
      const double inv = fma(y1, fma(-hd * y1, y1, 0.5), y1);
      if constexpr (j < 15) {
        if constexpr (VAR == 2) {
          const double r0 = __builtin_amdgcn_rcp(dj);
          const double r1 = fma(r0, fma(-dj, r0, 1.0), r0);
          const double r2 = fma(r1, fma(-dj, r1, 1.0), r1);
          dj = fma(-(a1 * a1), r2, ap);
        } else {
          const double s1 = a1 * inv;
          dj = fma(-s1, s1, ap);
        }
      }
      const double l = a[j] * inv;
      a[j] = l;
      const double xj = x[j] * inv;
      x[j] = xj;
      const double nl = -l, nx = -xj;
      static_for<j + 1, 16>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        if (VAR == 4 && k > j + 2) return;
        const double lk = __builtin_amdgcn_mov_dpp(l, 0x150 + k, 0xf, 0xf, true);
        a[k] = fma(nl, lk, a[k]);
        if (VAR != 3 && VAR != 4) x[k] = fma(nx, lk, x[k]);
      });
    });
#pragma unroll
    for (int q = 0; q < 16; ++q) asm volatile("" : "+v"(a[q]), "+v"(x[q]));
    return bad;
  }
}

// 5  1 + the inverse on the other half-wave: lanes 0-31 hold the factor's rows (y = a), lanes 32-63 W's columns
//    (y = x); the column is moved to the upper half once per column (v_permlane32_swap of a register with itself
//    copies lanes 0-31 up), then one DPP broadcast + one fma per entry serves both (bitwise variant 1's values)
__device__ __forceinline__ double half_up_f64(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const unsigned lo = (unsigned)(b & 0xffffffffll), hi = (unsigned)(b >> 32);
  const auto rl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto rh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return __builtin_bit_cast(double, (long long)(((unsigned long long)rh[0] << 32) | rl[0]));
}
// 6 / 7: variant 1 / 5 with the next two rows' entries from wave-uniform values (L[j+1][j] = a1·inv is the chain's s1,
//    L[j+2][j] a readlane taken with it): the next column's readlanes no longer wait for a broadcast
template <bool SPLIT, bool UNI>
__device__ __forceinline__ int chol16_split(double (&y)[16], double (&x)[16]) {
  int bad = 0;
  double dj = readlane_f64(y[0], 0);
  static_for<0, 16>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    double a1 = 0.0, ap = 0.0, a2 = 0.0;
    if constexpr (j < 15) {
      a1 = readlane_f64(y[j], j + 1);
      ap = readlane_f64(y[j + 1], j + 1);
    }
    if constexpr (UNI && j < 14) a2 = readlane_f64(y[j], j + 2);
    if (!(dj > 0.0) && bad == 0) bad = j + 1;
    const double y0 = __builtin_amdgcn_rsq(dj);
    const double hd = 0.5 * dj;
    const double y1 = fma(y0, fma(-hd * y0, y0, 0.5), y0);
    const double inv = fma(y1, fma(-hd * y1, y1, 0.5), y1);
    double s1 = 0.0, s2 = 0.0;
    if constexpr (j < 15) {
      s1 = a1 * inv;
      dj = fma(-s1, s1, ap);
    }
    if constexpr (UNI && j < 14) s2 = a2 * inv;
    const double yj = y[j] * inv;
    y[j] = yj;
    double xj = 0.0;
    if constexpr (!SPLIT) {
      xj = x[j] * inv;
      x[j] = xj;
    }
    if constexpr (j < 15) {
      const double ny = -yj, nx = -xj;
      if constexpr (UNI) {
        y[j + 1] = fma(ny, s1, y[j + 1]);
        if constexpr (!SPLIT) x[j + 1] = fma(nx, s1, x[j + 1]);
        if constexpr (j < 14) {
          y[j + 2] = fma(ny, s2, y[j + 2]);
          if constexpr (!SPLIT) x[j + 2] = fma(nx, s2, x[j + 2]);
        }
      }
      const double lcol = SPLIT ? half_up_f64(yj) : yj;
      static_for<j + 1, 16>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        if (UNI && k <= j + 2) return;
        const double lk = __builtin_amdgcn_mov_dpp(lcol, 0x150 + k, 0xf, 0xf, true);
        y[k] = fma(ny, lk, y[k]);
        if constexpr (!SPLIT) x[k] = fma(nx, lk, x[k]);
      });
    }
  });
#pragma unroll
  for (int q = 0; q < 16; ++q) asm volatile("" : "+v"(y[q]), "+v"(x[q]));
  return bad;
}

// 8  software-pipelined: column j+1's pivot chain (rsq + two Newton steps) is issued between column j's broadcast
//    updates, in an order pinned by sched_barrier (the compiler put the chain after the updates: the wave issues in
//    order, so each of the chain's dependent ops stalled it); the next pivot's inputs come from wave-uniform values
//    (the two entries right below the diagonal updated with the uniform s1, s2) — bitwise variant 1's values
__device__ __forceinline__ double rsq_nr2(double d) {
  const double y0 = __builtin_amdgcn_rsq(d);
  const double hd = 0.5 * d;
  const double y1 = fma(y0, fma(-hd * y0, y0, 0.5), y0);
  return fma(y1, fma(-hd * y1, y1, 0.5), y1);
}
__device__ __forceinline__ int chol16_pipe(double (&a)[16], double (&x)[16]) {
  int badm = 0;
  double dj = readlane_f64(a[0], 0);
  double a1 = readlane_f64(a[0], 1), ap = readlane_f64(a[1], 1), a2 = readlane_f64(a[0], 2);
  badm |= (dj > 0.0) ? 0 : 1;
  double inv = rsq_nr2(dj);
  static_for<0, 16>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    double s1 = 0.0, s2 = 0.0, dn = 0.0;
    if constexpr (j < 15) s1 = a1 * inv;
    if constexpr (j < 14) s2 = a2 * inv;
    const double l = a[j] * inv;
    const double xj = x[j] * inv;
    a[j] = l;
    x[j] = xj;
    const double nl = -l, nx = -xj;
    if constexpr (j < 15) {
      dn = fma(-s1, s1, ap);
      a[j + 1] = fma(nl, s1, a[j + 1]);
      x[j + 1] = fma(nx, s1, x[j + 1]);
    }
    if constexpr (j < 14) {
      a[j + 2] = fma(nl, s2, a[j + 2]);
      x[j + 2] = fma(nx, s2, x[j + 2]);
    }
    // the next column's chain inputs (entries updated above)
    if constexpr (j < 14) {
      a1 = readlane_f64(a[j + 1], j + 2);
      ap = readlane_f64(a[j + 2], j + 2);
    }
    if constexpr (j < 13) a2 = readlane_f64(a[j + 1], j + 3);
    __builtin_amdgcn_sched_barrier(0);
    // chain ops interleaved with the broadcast updates k = j+3 .. 15
    double y0 = 0.0, hd = 0.0, t = 0.0, y1 = 0.0;
    auto chain = [&](auto sc) {
      constexpr int st = decltype(sc)::value;
      if constexpr (j < 15) {
        if constexpr (st == 0) { y0 = __builtin_amdgcn_rsq(dn); hd = 0.5 * dn; badm |= (dn > 0.0) ? 0 : (2 << j); }
        if constexpr (st == 1) t = fma(-hd * y0, y0, 0.5);
        if constexpr (st == 2) y1 = fma(y0, t, y0);
        if constexpr (st == 3) t = fma(-hd * y1, y1, 0.5);
        if constexpr (st == 4) inv = fma(y1, t, y1);
      }
    };
    auto upd = [&](auto kc) {
      constexpr int k = decltype(kc)::value;
      if constexpr (k < 16) {
        const double lk = __builtin_amdgcn_mov_dpp(l, 0x150 + k, 0xf, 0xf, true);
        a[k] = fma(nl, lk, a[k]);
        x[k] = fma(nx, lk, x[k]);
      }
    };
    static_for<0, 5>([&](auto sc) {
      constexpr int st = decltype(sc)::value;
      chain(sc);
      __builtin_amdgcn_sched_barrier(0);
      upd(std::integral_constant<int, j + 3 + 2 * st>{});
      upd(std::integral_constant<int, j + 4 + 2 * st>{});
      __builtin_amdgcn_sched_barrier(0);
    });
    static_for<j + 13, 16>([&](auto kc) { upd(kc); });
    __builtin_amdgcn_sched_barrier(0);
  });
#pragma unroll
  for (int q = 0; q < 16; ++q) asm volatile("" : "+v"(a[q]), "+v"(x[q]));
  return badm ? __builtin_ffs(badm) : 0;
}

template <int VAR>
__global__ __launch_bounds__(64) void f16_kernel(const double* __restrict__ D, double* __restrict__ out, int reps,
                                                 unsigned long long* cyc) {
  const int c = threadIdx.x & 15;
  double a[16], x[16];
  for (int q = 0; q < 16; ++q) a[q] = D[c * 16 + q];
  unsigned long long t0 = 0, t1 = 0;
  int bad = 0;
  for (int r = 0; r < reps; ++r) {
#pragma unroll
    for (int q = 0; q < 16; ++q) x[q] = (q == c) ? 1.0 : 0.0;
    double b[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) b[q] = a[q];
    if constexpr (VAR == 5 || VAR == 7) {
#pragma unroll
      for (int q = 0; q < 16; ++q) b[q] = threadIdx.x < 32 ? a[q] : x[q];
    }
    __builtin_amdgcn_s_waitcnt(0);
    if (r == reps - 1) t0 = __builtin_readcyclecounter();
    if constexpr (VAR == 5)
      bad += chol16_split<true, false>(b, x);
    else if constexpr (VAR == 6)
      bad += chol16_split<false, true>(b, x);
    else if constexpr (VAR == 7)
      bad += chol16_split<true, true>(b, x);
    else if constexpr (VAR == 8)
      bad += chol16_pipe(b, x);
    else
      bad += chol16_var<VAR>(b, x);
#pragma unroll
    for (int q = 0; q < 16; ++q) asm volatile("" : "+v"(b[q]), "+v"(x[q]));
    if (r == reps - 1) t1 = __builtin_readcyclecounter();
    if (r == reps - 1)
      for (int q = 0; q < 16; ++q) {
        constexpr bool sp = VAR == 5 || VAR == 7;
        if (!sp || threadIdx.x < 16) out[c * 16 + q] = b[q];
        if (!sp) out[256 + q * 16 + c] = x[q];
        else if (threadIdx.x >= 32 && threadIdx.x < 48) out[256 + q * 16 + c] = b[q];
      }
  }
  if (threadIdx.x == 0) {
    cyc[0] = t1 - t0;
    cyc[1] = bad;
  }
}

int main() {
  const int n = 16;
  std::vector<double> h(n * n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) h[i * n + j] = (i == j) ? n : 1.0 / (1.0 + std::abs((double)(i - j)));
  double *D, *out;
  unsigned long long* cyc;
  CK(hipMalloc(&D, n * n * 8));
  CK(hipMalloc(&out, 2 * n * n * 8));
  CK(hipMalloc(&cyc, 16));
  CK(hipMemcpy(D, h.data(), n * n * 8, hipMemcpyHostToDevice));
  const char* names[9] = {"chol16_factor (library)", "pivot test off the chain", "pivot from 1/d (rcp)",
                          "no x updates (W wrong)", "chain only (output wrong)", "1 + W on the upper half-wave",
                          "1 + next two rows uniform", "5 + next two rows uniform", "pipelined chain"};
  void (*kern[9])(const double*, double*, int, unsigned long long*) = {f16_kernel<0>, f16_kernel<1>, f16_kernel<2>,
                                                                       f16_kernel<3>, f16_kernel<4>, f16_kernel<5>,
                                                                       f16_kernel<6>, f16_kernel<7>, f16_kernel<8>};
  std::vector<double> ref;
  for (int rep = 0; rep < 2; ++rep)
    for (int v = 0; v < 9; ++v) {
      hipLaunchKernelGGL(kern[v], dim3(1), dim3(64), 0, 0, D, out, 20, cyc);
      CK(hipDeviceSynchronize());
      unsigned long long c[2];
      CK(hipMemcpy(c, cyc, 16, hipMemcpyDeviceToHost));
      std::vector<double> o(2 * n * n);
      CK(hipMemcpy(o.data(), out, o.size() * 8, hipMemcpyDeviceToHost));
      // residual of L·Lᵀ = D and L·W = I
      double e1 = 0, e2 = 0;
      for (int i = 0; i < n; ++i)
        for (int j = 0; j <= i; ++j) {
          double s = 0, w = 0;
          for (int k = 0; k <= j; ++k) s += o[i * n + k] * o[j * n + k];
          for (int k = j; k <= i; ++k) w += o[i * n + k] * o[n * n + k * n + j];
          e1 = std::max(e1, std::abs(s - h[i * n + j]));
          e2 = std::max(e2, std::abs(w - (i == j ? 1.0 : 0.0)));
        }
      if (v == 0) ref = o;
      bool same = true;
      for (int i = 0; i < n; ++i)
        for (int j = 0; j <= i; ++j) same = same && o[i * n + j] == ref[i * n + j] && o[n * n + i * n + j] == ref[n * n + i * n + j];
      if (rep == 1) printf("%s ", same ? "[bitwise = library]" : "[differs]          ");
      if (rep == 1)
        printf("%-30s %6llu cycles per 16x16 factor + inverse (%.0f per column)  |LLt-D| %.1e  |LW-I| %.1e  bad %llu\n",
               names[v], c[0], c[0] / 16.0, e1, e2, c[1]);
    }
  return 0;
}
