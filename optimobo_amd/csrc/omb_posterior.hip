// GP posterior on gfx950: the K(X, X*) block and the fused posterior kernel.
//
// Replaces GPy's PosteriorExact._raw_predict as reached through model.predict(x[None,:]) at
// optimobo/util_functions.py:155-158 (and emo.py:203-205, optimisers.py:336, parego.py:137):
//     K*  = σ_f² (1 + √5 r + 5/3 r²) exp(−√5 r),  r² = ‖x/ℓ‖² + ‖x*/ℓ‖² − 2 (x/ℓ)·(x*/ℓ)
//     μ   = K*ᵀ α
//     σ²  = σ_f² − Σ_rows (L⁻¹ K*)²
// All arithmetic is fp64 (fp32 fails parity by orders of magnitude).
//
// Fused posterior kernel (one workgroup = 512 threads = 8 waves, BN candidates):
//   * K* is generated 64 training rows at a time ("chunk") as 16×16 tiles: r² (or, for d > 8, the
//     cross term) of a tile is a few FP64 MFMA k-steps against fragment-packed training rows,
//     then the Matern transform runs in VALU (table-driven exp).  The values land in a 3-buffer
//     LDS ring in the B-operand fragment order of v_mfma_f64_16x16x4_f64, so each wave reads a
//     fragment as 64 consecutive doubles; waves synchronise per chunk through LDS counters.
//   * The triangular product V = L⁻¹ K* runs on FP64 MFMA: the A operand (L⁻¹) is read from a
//     packed, fragment-ordered copy (zero blocks above the diagonal are never stored or read);
//     it is L2-resident (1.06 MiB per objective at n = 512) and shared by every workgroup.
//   * Row tiles (16 rows) are dealt to waves so that, for every chunk, the four SIMD pairs
//     (waves w and w+4 share a SIMD) get equal MFMA work: tile r = 4q + ((pair + q) mod 4)
//     of quad q, quads split between the two waves of a pair in Gray-code order.
//   * μ accumulates in VALU during generation; σ² is a wave reduction of the squared MFMA
//     accumulators followed by a fixed-order cross-wave LDS reduction (deterministic).
#include <algorithm>

#include "omb_internal.h"
#include "omb_math.h"

namespace omb {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));

// ----------------------------------------------------------------------------- packing
struct LsArg {
  double v[OMB_MAX_DIM];
};

// Xs = X / ℓ (GPy Stationary._scaled_dist divides), xsq = Σ Xs², α padded, ℓ padded with 1.
__global__ void pack_rows_kernel(int n, int d, int DP, int n_pad, const double* __restrict__ X, LsArg ls,
                                 const double* __restrict__ alpha, double* __restrict__ Xs,
                                 double* __restrict__ xsq, double* __restrict__ alpha_p, double* __restrict__ ls_p) {
  int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < DP && blockIdx.x == 0) ls_p[k] = (k < d) ? ls.v[k] : 1.0;
  if (k >= n_pad) return;
  double s = 0.0;
  for (int j = 0; j < DP; ++j) {
    double v = 0.0;
    if (k < n && j < d) v = X[(int64_t)k * d + j] / ls.v[j];
    Xs[(int64_t)k * DP + j] = v;
    s += v * v;
  }
  xsq[k] = s;
  alpha_p[k] = (k < n) ? alpha[k] : 0.0;
}

// Packed L⁻¹: tile r (rows 16r..16r+15) holds k-steps S = 0 .. 4(r+1)-1 (columns 4S..4S+3);
// k-steps are stored in pairs so a lane loads both of its A values with one 16-byte load:
//     Lp[128 r (r+1) + 128 (S/2) + 2 lane + (S&1)] = L⁻¹[16r + (lane&15)][4S + (lane>>4)]
// (A-operand map of v_mfma_f64_16x16x4_f64: lane l holds A[l&15][l>>4]).
__global__ void pack_L_kernel(int n, const double* __restrict__ Linv, double* __restrict__ Lp) {
  const int r = blockIdx.y;
  const int per_tile = 256 * (r + 1);
  double* dst = Lp + 128ll * r * (r + 1);
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < per_tile; t += gridDim.x * blockDim.x) {
    int P = t >> 7, lane = (t & 127) >> 1, h = t & 1;
    int S = 2 * P + h;
    int row = 16 * r + (lane & 15), col = 4 * S + (lane >> 4);
    double v = 0.0;
    if (row < n && col < n && col <= row) v = Linv[(int64_t)row * n + col];
    dst[t] = v;
  }
}

hipError_t launch_pack_gp(hipStream_t stream, int n, int d, int DP, const double* X, const double* ls_host,
                          const double* alpha, const double* Linv, double* Xs, double* xsq, double* alpha_p,
                          double* Lp, int R, int n_pad) {
  LsArg ls{};
  for (int j = 0; j < d; ++j) ls.v[j] = ls_host[j];
  // ls_p lives right after alpha_p (see omb_set_gp's buffer carving).
  double* ls_p = alpha_p + n_pad;
  hipLaunchKernelGGL(pack_rows_kernel, dim3((n_pad + 255) / 256), dim3(256), 0, stream, n, d, DP, n_pad, X, ls,
                     alpha, Xs, xsq, alpha_p, ls_p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (R == 0) return hipSuccess;   // n_train above OMB_MAX_TRAIN: the dense path reads L^-1 unpacked
  hipLaunchKernelGGL(pack_L_kernel, dim3(4, R), dim3(256), 0, stream, n, Linv, Lp);
  return hipGetLastError();
}
// Xf: the training rows as the A operand of the r²-MFMA (posterior_kernel, kMfmaGen), augmented
// with two columns so that one dot product gives r² (the B side holds [−2·x*/ℓ, 1, ‖x*/ℓ‖²]):
//     A[k][j] = Xs[k][j] (j < d),  ‖Xs[k]‖² (j = d),  1 (j = d+1),  0 beyond.
// Row tile T (rows 16T..16T+15), k-step s = 2P + h (dims 4s..4s+3), pairs P < packed_X_pairs(DP):
//     Xf[(T·pairs + P)·128 + 2·lane + h] = A[16T + (lane&15)][4s + (lane>>4)]
// so a lane loads the A values of two k-steps with one 16-byte load, a wave 1 KiB contiguous.
__global__ void pack_X_kernel(int d, int DP, int pairs, int64_t total, const double* __restrict__ Xs,
                              const double* __restrict__ xsq, double* __restrict__ Xf) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t T = t / (128 * pairs);
    const int rem = (int)(t % (128 * pairs));
    const int P = rem >> 7, lane = (rem & 127) >> 1, h = rem & 1;
    const int j = 4 * (2 * P + h) + (lane >> 4);
    const int64_t row = 16 * T + (lane & 15);
    Xf[t] = (j < d) ? Xs[row * DP + j] : (j == d ? xsq[row] : (j == d + 1 ? 1.0 : 0.0));
  }
}

hipError_t launch_pack_x(hipStream_t stream, int d, int DP, int n_pad, const double* Xs, const double* xsq,
                         double* Xf) {
  const int64_t total = packed_X_size(n_pad, DP);
  const unsigned blocks = (unsigned)std::min<int64_t>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(pack_X_kernel, dim3(blocks), dim3(256), 0, stream, d, DP, packed_X_pairs(DP), total, Xs, xsq,
                     Xf);
  return hipGetLastError();
}

// ----------------------------------------------------------------------------- K block
// Standalone K(X_train, X*) (n, N) row-major — the HBM-bound kernel of the north star.
// K block with r² on MFMA (the posterior kernel's generation step, stored instead of multiplied):
// a workgroup covers 64 candidates × kKBlockRows training rows, wave w the candidates' 16-wide
// tile w.  Per 16-row tile: ⌈(d+2)/4⌉ MFMA k-steps against the fragment-packed rows (Xf) give r²
// (d ≤ 8; for d > 8 the cross term, r² then one fma), the Matern transform runs on the lane's 4
// values (kernel_of_r2_tab_x2), and each store instruction writes 4 rows × 16 consecutive
// candidates (128-byte segments), non-temporal (written once, never re-read here).  Against the
// previous VALU dot products (d FMAs plus d loads per element; tools/ablate/ablate_kblock2):
// 1.18 → 1.03 ms at n = 512, d = 6, N = 2^20 and 2.43 → 1.66 ms at n = 1024, d = 30, N = 2^19.
template <int DP, int KIND, bool kNT = true>   // kNT = false: plain stores (tools/ablate/ablate_kblock2.hip)
__global__ __launch_bounds__(256) void kernel_block_mfma_kernel(GPDev g, int d, const double* __restrict__ Xc,
                                                                int64_t N, double* __restrict__ K, ExpCoef ec) {
  constexpr bool kAug = DP <= 8;
  constexpr int KSD = kAug ? (DP + 5) / 4 : (DP + 3) / 4;
  constexpr int KSDP = ((DP + 5) / 4 + 1) / 2;   // = packed_X_pairs(DP)
  constexpr bool kTab256 = KIND == OMB_KERNEL_MATERN52;
  __shared__ double etab[kTab256 ? 256 : 64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if constexpr (kTab256)
    etab[tid] = kExp2Tab256[tid];   // 256 threads
  else if (tid < 64)
    etab[tid] = kExp2Tab64[tid];
  const int64_t col = (int64_t)blockIdx.x * 64 + 16 * wave + (lane & 15);
  const int64_t ci = col < N ? col : N - 1;
  double csq = 0.0;
#pragma unroll
  for (int j = 0; j < DP; ++j) {
    const double c = (j < d) ? Xc[ci * d + j] / g.ls[j] : 0.0;
    csq = fma(c, c, csq);
  }
  double bfr[KSD];
#pragma unroll
  for (int s = 0; s < KSD; ++s) {
    const int j = 4 * s + (lane >> 4);
    const double c = (j < d) ? Xc[ci * d + j] / g.ls[j] : 0.0;
    if constexpr (kAug)
      bfr[s] = (j < d) ? -2.0 * c : (j == d ? 1.0 : (j == d + 1 ? csq : 0.0));
    else
      bfr[s] = c;
  }
  const double pm[3] = {g.variance, kSqrt5 * g.variance, kFiveThirds * g.variance};
  __syncthreads();
  const int T0 = blockIdx.y * (kKBlockRows / 16);
  const int T1 = min((g.n + 15) / 16, T0 + kKBlockRows / 16);
  for (int T = T0; T < T1; ++T) {
    const d2* xa = reinterpret_cast<const d2*>(g.Xf + (int64_t)T * (KSDP * 128) + 2 * lane);
    d2 a[(KSD + 1) / 2];
#pragma unroll
    for (int p = 0; p < (KSD + 1) / 2; ++p) a[p] = xa[64 * p];
    d4 cr = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < KSD; ++s)
      cr = __builtin_amdgcn_mfma_f64_16x16x4f64((s & 1) ? a[s >> 1].y : a[s >> 1].x, bfr[s], cr, 0, 0, 0);
#pragma unroll
    for (int e = 0; e < 4; e += 2) {
      const int k0 = 16 * T + 4 * e + (lane >> 4), k1 = k0 + 4;
      const double r2a = kAug ? cr[e] : fma(-2.0, cr[e], g.xsq[k0] + csq);
      const double r2b = kAug ? cr[e + 1] : fma(-2.0, cr[e + 1], g.xsq[k1] + csq);
      double v0, v1;
      if constexpr (kTab256)
        matern_r2_tab256_x2(r2a, r2b, pm, ec, etab, v0, v1);
      else
        kernel_of_r2_tab_x2<KIND>(r2a, r2b, pm, ec, etab, v0, v1);
      if (col < N) {
        if constexpr (kNT) {
          if (k0 < g.n) __builtin_nontemporal_store(v0, K + (int64_t)k0 * N + col);
          if (k1 < g.n) __builtin_nontemporal_store(v1, K + (int64_t)k1 * N + col);
        } else {
          if (k0 < g.n) K[(int64_t)k0 * N + col] = v0;
          if (k1 < g.n) K[(int64_t)k1 * N + col] = v1;
        }
      }
    }
  }
}

// Exchange of two doubles between 16-lane groups: v_permlane16_swap on both dwords.  Afterwards
// x holds [x.g0, y.g0, x.g2, y.g2] and y holds [x.g1, y.g1, x.g3, y.g3] (g = 16-lane group).
__device__ __forceinline__ void permlane16_swap_f64(double& x, double& y) {
  const unsigned long long xi = __builtin_bit_cast(unsigned long long, x);
  const unsigned long long yi = __builtin_bit_cast(unsigned long long, y);
  const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)xi, (unsigned)yi, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(xi >> 32), (unsigned)(yi >> 32), false, false);
  x = __builtin_bit_cast(double, ((unsigned long long)hi[0] << 32) | lo[0]);
  y = __builtin_bit_cast(double, ((unsigned long long)hi[1] << 32) | lo[1]);
}

// K block, store-stream friendly.  kernel_block_mfma_kernel loaded each row tile's Xf fragment (and,
// for n_var > 8, ‖x/ℓ‖²) from global memory inside its loop; on gfx950 one counter (vmcnt) tracks
// loads AND stores, and the compiler's wait for such a load inside a loop with stores is vmcnt(0), so
// every iteration drained the wave's store queue.  Here the workgroup stages its rows' fragments in
// LDS once, the loop issues only stores, and the store queue stays full.  Store addresses are one
// per-lane base pointer plus wave-uniform row offsets (no 64-bit multiplies per store); interior tiles
// (16 rows < n, every candidate < N) store without per-lane guards.  512 threads: wave w owns the
// 16-candidate tile w of the workgroup's 128 candidates and sweeps kblock_rows(DP) training rows.
constexpr bool kKBlockSwap = false;   // 2 × 256-B store rows (see kSwap below); set from the ablation
constexpr int kblock_rows(int DP) {
  return (((DP + 5) / 4 + 1) / 2) <= 3 ? 256 : ((((DP + 5) / 4 + 1) / 2) <= 5 ? 128 : 64);
}

// kSwap: wave w computes the two adjacent candidate tiles 2(w&3), 2(w&3)+1 of the row tiles of parity
// w>>2, and one v_permlane16_swap per value (permlane16_swap_f64) turns the two accumulators (lane
// group g: row 4e+g of 16 candidates) into 2 rows × 32 consecutive candidates per register, so each
// store instruction writes 2 × 256 contiguous bytes instead of 4 × 128 (tools/microbench/mb_write:
// 5.9-6.0 vs 5.3-5.4 TB/s for the bare store streams).
// kTrans: the 8 waves' 16×16 tiles of a row tile go through LDS (tb, double buffered, one barrier per
// row tile) and wave w stores rows 2w, 2w+1 of the workgroup's 128 candidates, one 1-KB row segment
// per store instruction (b128 per lane), instead of 4 × 128 B.
constexpr int kTransPitch = 144;   // tb row pitch (doubles): the 4 row groups of a tile write land on disjoint banks
// RPI: row tiles per loop iteration (1 or 2, plain stores only).  With 2, the two tiles' cross-term MFMA
// chains and Matern transforms are independent and interleave (a wave otherwise waits out each tile's
// dependent 8-step chain at n_var > 8).  ABL (tools/ablate only): bit 1 drops the stores (the values are
// folded into one guarded store per lane), bit 2 drops the cross term and the transform.
template <int DP, int KIND, bool kNT = true, bool kSwap = false, bool kTrans = false, int RPI = 1, int ABL = 0>
__global__ __launch_bounds__(512) void kernel_block_pipe_kernel(GPDev g, int d, const double* __restrict__ Xc,
                                                                int64_t N, double* __restrict__ K, ExpCoef ec) {
  static_assert(RPI == 1 || (RPI == 2 && !kSwap && !kTrans), "two row tiles per iteration: plain stores only");
  constexpr bool kAug = DP <= 8;
  constexpr int KSD = kAug ? (DP + 5) / 4 : (DP + 3) / 4;
  constexpr int KSDP = ((DP + 5) / 4 + 1) / 2;   // = packed_X_pairs(DP)
  constexpr int NA = (KSD + 1) / 2;
  constexpr int TPW = kblock_rows(DP) / 16;      // row tiles per workgroup
  constexpr int NCT = kSwap ? 2 : 1;             // candidate tiles per wave
  constexpr bool kTab256 = KIND == OMB_KERNEL_MATERN52;
  __shared__ double etab[kTab256 ? 256 : 64];
  __shared__ double xfs[TPW * KSDP * 128];
  __shared__ double xsqs[kAug ? 1 : TPW * 16];
  __shared__ __attribute__((aligned(16))) double tb[kTrans ? 2 * 16 * kTransPitch : 1];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int T0 = blockIdx.y * TPW;
  const int T1 = min((g.n + 15) / 16, T0 + TPW);
  if (tid < (kTab256 ? 256 : 64)) etab[tid] = kTab256 ? kExp2Tab256[tid] : kExp2Tab64[tid];
  for (int i = tid; i < (T1 - T0) * KSDP * 128; i += 512) xfs[i] = g.Xf[(int64_t)T0 * KSDP * 128 + i];
  if constexpr (!kAug)
    for (int i = tid; i < (T1 - T0) * 16; i += 512) xsqs[i] = g.xsq[16 * T0 + i];
  // candidate tiles of this wave: 16·(wave·NCT + t) within the workgroup's 128 candidates (kSwap: wave&3)
  const int64_t cb = (int64_t)blockIdx.x * 128 + 16 * NCT * (kSwap ? (wave & 3) : wave);
  double csq[NCT], bfr[NCT][KSD];
#pragma unroll
  for (int t = 0; t < NCT; ++t) {
    const int64_t c = cb + 16 * t + (lane & 15);
    const int64_t ci = c < N ? c : N - 1;
    if constexpr (!kSwap) {
      // lane l needs only dims 4s + (l>>4) of its candidate (KSD divisions instead of d + KSD);
      // ‖x*/ℓ‖² from the four lane groups by two shuffles.  At n_var = 30 the staged kernel overtook
      // the round-1 kernel with this (1.70 → 1.44 ms, profiles/r02_v54_ablate_kblock_c5.txt); at
      // n_var = 6 it is 0.80 → 0.78 ms (profiles/r02_v55_ablate_kblock_c3*.txt)
      double s2 = 0.0, xs[KSD];
#pragma unroll
      for (int s = 0; s < KSD; ++s) {
        const int j = 4 * s + (lane >> 4);
        xs[s] = (j < d) ? Xc[ci * d + j] / g.ls[j] : 0.0;
        s2 = fma(xs[s], xs[s], s2);
      }
      s2 += __shfl_xor(s2, 16);
      s2 += __shfl_xor(s2, 32);
      csq[t] = s2;
#pragma unroll
      for (int s = 0; s < KSD; ++s) {
        const int j = 4 * s + (lane >> 4);
        bfr[t][s] = kAug ? ((j < d) ? -2.0 * xs[s] : (j == d ? 1.0 : (j == d + 1 ? s2 : 0.0))) : xs[s];
      }
      continue;
    }
    double s2 = 0.0;
#pragma unroll
    for (int j = 0; j < DP; ++j) {
      const double x = (j < d) ? Xc[ci * d + j] / g.ls[j] : 0.0;
      s2 = fma(x, x, s2);
    }
    csq[t] = s2;
#pragma unroll
    for (int s = 0; s < KSD; ++s) {
      const int j = 4 * s + (lane >> 4);
      const double x = (j < d) ? Xc[ci * d + j] / g.ls[j] : 0.0;
      if constexpr (kAug)
        bfr[t][s] = (j < d) ? -2.0 * x : (j == d ? 1.0 : (j == d + 1 ? s2 : 0.0));
      else
        bfr[t][s] = x;
    }
  }
  const double pm[3] = {g.variance, kSqrt5 * g.variance, kFiveThirds * g.variance};
  const bool cols_full = (int64_t)(blockIdx.x + 1) * 128 <= N;     // workgroup-uniform
  // kTrans row segments are 16-B aligned when K is and N is even
  const bool wide = cols_full && ((reinterpret_cast<uintptr_t>(K) & 15) == 0) && (N % 2 == 0);
  const int full_tiles = g.n / 16;                                  // tiles with all 16 rows < n
  // stored element e of a tile: row 16T + 4e + rsub, column col
  //   plain: rsub = lane>>4, col = cb + (lane&15);  swap: rsub = 2(lane>>5) (+1 for the second register),
  //   col = cb + (lane&31)
  const int rsub = kSwap ? 2 * (lane >> 5) : (lane >> 4);
  const int64_t col = cb + (kSwap ? (lane & 31) : (lane & 15));
  double* Kl = K + (int64_t)rsub * N + col;
  const int64_t N4 = 4 * N;
  auto st = [&](double* p, double v) {
    if constexpr (kNT)
      __builtin_nontemporal_store(v, p);
    else
      *p = v;
  };
  __syncthreads();
  const int Tstart = T0 + (kSwap ? (wave >> 2) : 0);
  if constexpr (RPI == 2) {
    double sink = 0.0;
    for (int T = Tstart; T < T1; T += 2) {
      const int Tb = min(T + 1, T1 - 1);            // a lone last tile is computed twice, stored once
      const d2* xa0 = reinterpret_cast<const d2*>(xfs + (T - T0) * (KSDP * 128) + 2 * lane);
      const d2* xa1 = reinterpret_cast<const d2*>(xfs + (Tb - T0) * (KSDP * 128) + 2 * lane);
      d2 a0[NA], a1[NA];
#pragma unroll
      for (int p = 0; p < NA; ++p) {
        a0[p] = xa0[64 * p];
        a1[p] = xa1[64 * p];
      }
      double v0[4], v1[4];
      if constexpr ((ABL & 2) != 0) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v0[e] = a0[0].x + e;
          v1[e] = a1[0].y + e;
        }
      } else {
        d4 c0 = d4{0.0, 0.0, 0.0, 0.0}, c1 = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int q = 0; q < KSD; ++q) {
          c0 = __builtin_amdgcn_mfma_f64_16x16x4f64((q & 1) ? a0[q >> 1].y : a0[q >> 1].x, bfr[0][q], c0, 0, 0, 0);
          c1 = __builtin_amdgcn_mfma_f64_16x16x4f64((q & 1) ? a1[q >> 1].y : a1[q >> 1].x, bfr[0][q], c1, 0, 0, 0);
        }
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          const int l0 = 16 * (T - T0) + 4 * e + (lane >> 4), m0 = 16 * (Tb - T0) + 4 * e + (lane >> 4);
          const double r0a = kAug ? c0[e] : fma(-2.0, c0[e], xsqs[kAug ? 0 : l0] + csq[0]);
          const double r0b = kAug ? c0[e + 1] : fma(-2.0, c0[e + 1], xsqs[kAug ? 0 : l0 + 4] + csq[0]);
          const double r1a = kAug ? c1[e] : fma(-2.0, c1[e], xsqs[kAug ? 0 : m0] + csq[0]);
          const double r1b = kAug ? c1[e + 1] : fma(-2.0, c1[e + 1], xsqs[kAug ? 0 : m0 + 4] + csq[0]);
          if constexpr (kTab256) {
            matern_r2_tab256_x2(r0a, r0b, pm, ec, etab, v0[e], v0[e + 1]);
            matern_r2_tab256_x2(r1a, r1b, pm, ec, etab, v1[e], v1[e + 1]);
          } else {
            kernel_of_r2_tab_x2<KIND>(r0a, r0b, pm, ec, etab, v0[e], v0[e + 1]);
            kernel_of_r2_tab_x2<KIND>(r1a, r1b, pm, ec, etab, v1[e], v1[e + 1]);
          }
        }
      }
      const bool second = Tb != T;
      if constexpr ((ABL & 1) != 0) {
#pragma unroll
        for (int e = 0; e < 4; ++e) sink += v0[e] + (second ? v1[e] : 0.0);
      } else {
        double* p0 = Kl + (int64_t)T * (4 * N4);
        double* p1 = p0 + 4 * N4;
        if (cols_full && Tb < full_tiles) {
#pragma unroll
          for (int e = 0; e < 4; ++e) st(p0 + e * N4, v0[e]);
          if (second) {
#pragma unroll
            for (int e = 0; e < 4; ++e) st(p1 + e * N4, v1[e]);
          }
        } else if (col < N) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (16 * T + 4 * e + rsub < g.n) st(p0 + e * N4, v0[e]);
            if (second && 16 * Tb + 4 * e + rsub < g.n) st(p1 + e * N4, v1[e]);
          }
        }
      }
    }
    if constexpr ((ABL & 1) != 0)
      if (sink == -1.2345e300 && col < N) K[col] = sink;       // never true: keeps the values live
    return;
  }
  double sink1 = 0.0;
  for (int T = Tstart; T < T1; T += (kSwap ? 2 : 1)) {
    const d2* xa = reinterpret_cast<const d2*>(xfs + (T - T0) * (KSDP * 128) + 2 * lane);
    d2 a[NA];
#pragma unroll
    for (int p = 0; p < NA; ++p) a[p] = xa[64 * p];
    double v[NCT][4];
#pragma unroll
    for (int t = 0; t < NCT; ++t) {
      if constexpr ((ABL & 2) != 0) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[t][e] = a[0].x + e;
        continue;
      }
      d4 cr = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s = 0; s < KSD; ++s)
        cr = __builtin_amdgcn_mfma_f64_16x16x4f64((s & 1) ? a[s >> 1].y : a[s >> 1].x, bfr[t][s], cr, 0, 0, 0);
#pragma unroll
      for (int e = 0; e < 4; e += 2) {
        const int l0 = 16 * (T - T0) + 4 * e + (lane >> 4), l1 = l0 + 4;
        const double r2a = kAug ? cr[e] : fma(-2.0, cr[e], xsqs[kAug ? 0 : l0] + csq[t]);
        const double r2b = kAug ? cr[e + 1] : fma(-2.0, cr[e + 1], xsqs[kAug ? 0 : l1] + csq[t]);
        if constexpr (kTab256)
          matern_r2_tab256_x2(r2a, r2b, pm, ec, etab, v[t][e], v[t][e + 1]);
        else
          kernel_of_r2_tab_x2<KIND>(r2a, r2b, pm, ec, etab, v[t][e], v[t][e + 1]);
      }
    }
    if constexpr ((ABL & 1) != 0) {
#pragma unroll
      for (int e = 0; e < 4; ++e) sink1 += v[0][e];
      continue;
    }
    double* p = Kl + (int64_t)T * (4 * N4);
    if constexpr (kSwap) {
#pragma unroll
      for (int e = 0; e < 4; ++e) permlane16_swap_f64(v[0][e], v[1][e]);
      if (cols_full && T < full_tiles) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          st(p + e * N4, v[0][e]);
          st(p + e * N4 + N, v[1][e]);
        }
      } else if (col < N) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int k = 16 * T + 4 * e + rsub;
          if (k < g.n) st(p + e * N4, v[0][e]);
          if (k + 1 < g.n) st(p + e * N4 + N, v[1][e]);
        }
      }
    } else {
      if (kTrans && wide && T < full_tiles) {
        double* B = tb + (T & 1) * (16 * kTransPitch);
#pragma unroll
        for (int e = 0; e < 4; ++e) B[(4 * e + (lane >> 4)) * kTransPitch + 16 * wave + (lane & 15)] = v[0][e];
        __syncthreads();
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int row = 2 * wave + h;
          const d2 val = *reinterpret_cast<const d2*>(B + row * kTransPitch + 2 * lane);
          d2* dst = reinterpret_cast<d2*>(K + (int64_t)(16 * T + row) * N + (int64_t)blockIdx.x * 128 + 2 * lane);
          if constexpr (kNT)
            __builtin_nontemporal_store(val, dst);
          else
            *dst = val;
        }
      } else if (cols_full && T < full_tiles) {
#pragma unroll
        for (int e = 0; e < 4; ++e) st(p + e * N4, v[0][e]);
      } else if (col < N) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (16 * T + 4 * e + rsub < g.n) st(p + e * N4, v[0][e]);
      }
    }
  }
  if constexpr ((ABL & 1) != 0)
    if (sink1 == -1.2345e300 && col < N) K[col] = sink1;        // never true: keeps the values live
}

// K block, persistent over candidate blocks: the workgroup stages its kblock_rows(DP) training rows' fragments
// once (as kernel_block_pipe_kernel does) and then sweeps CB blocks of 128 candidates, wave w owning the
// 16-candidate tile w of each.  The next block's coordinates are loaded while the current block's row tiles
// are computed and stored, so the staging and the candidate loads are paid once per CB blocks and their
// latency is hidden (the compiler's wait for the prefetch is a vmcnt that leaves the block's stores in
// flight).  RCP multiplies by 1/ℓ (one rounding more than GPy's division; ≤ 1 ulp in x/ℓ).  ROLL keeps the
// block loop rolled (unrolled, its registers cost occupancy).
// AW (n_var > 8 with d + 2 ≤ 4·⌈DP/4⌉, e.g. d = 30 in DP = 32): the packed rows already carry ‖x/ℓ‖² and 1 in
// dimensions d and d + 1 (pack_X_kernel), inside the cross term's k-steps, so B = [−2·x*/ℓ, 1, ‖x*/ℓ‖²] gives
// r² from the same 8 MFMA k-steps: the per-element fma, add and LDS read of ‖x/ℓ‖² go.
// XCD-aware workgroup order (round 4, nx > 0; the grid is then 1-D with ⌈nx/8⌉·8·ny workgroups): consecutive
// workgroups go to the 8 XCDs in turn, so workgroup b is mapped to candidate block x = 8·((b/8)/ny) + b mod 8 and
// row block y = (b/8) mod ny — the ny row blocks of one candidate slab run back to back on ONE XCD and re-read
// the slab from its L2 instead of from HBM (8 row blocks per slab at n = 1024, d = 30: 5.31 GB per launch
// against 4.42 GB of algorithmic bytes, profiles/r03_v19_pmc_c5).  nx = 0: the plain 2-D grid (tools/ablate).
template <int DP, int KIND, int CB, bool RCP = false, bool ROLL = false, bool AW = false>
__global__ __launch_bounds__(512) void kernel_block_persist_kernel(GPDev g, int d, const double* __restrict__ Xc,
                                                                   int64_t N, double* __restrict__ K, ExpCoef ec,
                                                                   int nx = 0, int ny = 0) {
  int bx = blockIdx.x, by = blockIdx.y;
  if (nx > 0) {
    const int slot = blockIdx.x >> 3;
    bx = 8 * (slot / ny) + (blockIdx.x & 7);
    by = slot % ny;
    if (bx >= nx) return;
  }
  constexpr bool kAug = DP <= 8 || AW;              // r² straight from the MFMA
  constexpr int KSD = DP <= 8 ? (DP + 5) / 4 : (DP + 3) / 4;
  constexpr int KSDP = ((DP + 5) / 4 + 1) / 2;   // = packed_X_pairs(DP)
  constexpr int NA = (KSD + 1) / 2;
  constexpr int TPW = kblock_rows(DP) / 16;
  constexpr bool kTab256 = KIND == OMB_KERNEL_MATERN52;
  __shared__ double etab[kTab256 ? 256 : 64];
  __shared__ double xfs[TPW * KSDP * 128];
  __shared__ double xsqs[kAug ? 1 : TPW * 16];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int T0 = by * TPW;
  const int T1 = min((g.n + 15) / 16, T0 + TPW);
  const int64_t base = (int64_t)bx * (128 * CB) + 16 * wave;
  double il[KSD];
#pragma unroll
  for (int s = 0; s < KSD; ++s) {
    const int j = 4 * s + (lane >> 4);
    il[s] = (j < d) ? (RCP ? 1.0 / g.ls[j] : g.ls[j]) : 1.0;
  }
  auto load_raw = [&](int64_t cb, double (&raw)[KSD]) {
    const int64_t c = cb + (lane & 15);
    const int64_t ci = c < N ? c : N - 1;
#pragma unroll
    for (int s = 0; s < KSD; ++s) {
      const int j = 4 * s + (lane >> 4);
      raw[s] = (j < d) ? Xc[ci * d + j] : 0.0;
    }
  };
  double raw[KSD];
  load_raw(base < N ? base : 0, raw);               // in flight during the staging
  if (tid < (kTab256 ? 256 : 64)) etab[tid] = kTab256 ? kExp2Tab256[tid] : kExp2Tab64[tid];
  for (int i = tid; i < (T1 - T0) * KSDP * 128; i += 512) xfs[i] = g.Xf[(int64_t)T0 * KSDP * 128 + i];
  if constexpr (!kAug)
    for (int i = tid; i < (T1 - T0) * 16; i += 512) xsqs[i] = g.xsq[16 * T0 + i];
  const double pm[3] = {g.variance, kSqrt5 * g.variance, kFiveThirds * g.variance};
  const int full_tiles = g.n / 16;
  const int rsub = lane >> 4;
  const int64_t N4 = 4 * N;
  __syncthreads();
#pragma unroll(ROLL ? 1 : CB)
  for (int jb = 0; jb < CB; ++jb) {
    const int64_t cb = base + (int64_t)jb * 128;
    if (cb >= N) break;                             // wave-uniform
    double xs[KSD], csq = 0.0;
#pragma unroll
    for (int s = 0; s < KSD; ++s) {
      xs[s] = RCP ? raw[s] * il[s] : raw[s] / il[s];
      csq = fma(xs[s], xs[s], csq);
    }
    csq += __shfl_xor(csq, 16);
    csq += __shfl_xor(csq, 32);
    double bfr[KSD];
#pragma unroll
    for (int s = 0; s < KSD; ++s) {
      const int j = 4 * s + (lane >> 4);
      bfr[s] = kAug ? ((j < d) ? -2.0 * xs[s] : (j == d ? 1.0 : (j == d + 1 ? csq : 0.0))) : xs[s];
    }
    if (jb + 1 < CB && cb + 128 < N) load_raw(cb + 128, raw);   // next block, in flight during this one
    const int64_t col = cb + (lane & 15);
    const bool cols_full = (int64_t)bx * (128 * CB) + (int64_t)(jb + 1) * 128 <= N;   // workgroup-uniform
    double* Kl = K + (int64_t)rsub * N + col;
    for (int T = T0; T < T1; ++T) {
      const d2* xa = reinterpret_cast<const d2*>(xfs + (T - T0) * (KSDP * 128) + 2 * lane);
      d2 a[NA];
#pragma unroll
      for (int p = 0; p < NA; ++p) a[p] = xa[64 * p];
      d4 cr = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int q = 0; q < KSD; ++q)
        cr = __builtin_amdgcn_mfma_f64_16x16x4f64((q & 1) ? a[q >> 1].y : a[q >> 1].x, bfr[q], cr, 0, 0, 0);
      double v[4];
#pragma unroll
      for (int e = 0; e < 4; e += 2) {
        const int l0 = 16 * (T - T0) + 4 * e + rsub;
        const double r2a = kAug ? cr[e] : fma(-2.0, cr[e], xsqs[kAug ? 0 : l0] + csq);
        const double r2b = kAug ? cr[e + 1] : fma(-2.0, cr[e + 1], xsqs[kAug ? 0 : l0 + 4] + csq);
        if constexpr (kTab256)
          matern_r2_tab256_x2(r2a, r2b, pm, ec, etab, v[e], v[e + 1]);
        else
          kernel_of_r2_tab_x2<KIND>(r2a, r2b, pm, ec, etab, v[e], v[e + 1]);
      }
      double* p = Kl + (int64_t)T * (4 * N4);
      if (cols_full && T < full_tiles) {
#pragma unroll
        for (int e = 0; e < 4; ++e) __builtin_nontemporal_store(v[e], p + e * N4);
      } else if (col < N) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (16 * T + 4 * e + rsub < g.n) __builtin_nontemporal_store(v[e], p + e * N4);
      }
    }
  }
}

// Per-workgroup phase timestamps of the posterior kernels for tools/ablate/ablate_posterior (empty here).
#ifndef OMB_POST_TRACE
#define OMB_POST_TRACE(id)
#endif

// ----------------------------------------------------------------------------- posterior
// ABL (ablation, tools/ablate only; the library instantiates ABL = 0): bit 1 replaces the Matern
// transform by the raw dot product, bit 2 skips the MFMA phase, bit 4 feeds a constant A
// operand instead of loading L⁻¹, bit 8 drops the per-chunk barrier (barrier mode only), bit 16
// uses libm exp/sqrt, bit 32 selects the 2-buffer / block-barrier pipeline instead of the
// counter-synchronised 3-buffer ring (tools/ablate: 12.03 → 11.23 ms at n = 512, N = 2^20); bit 128
// gives waves 4-7 static priority 1, bit 524288 applies exp's 2^m by an integer add to the high word (IEXP), bit 256 drops the σ_f² multiply, bit 512 starts the distance
// chain at ‖x‖² + ‖x*‖² with −2x* pre-scaled (one fma fewer per element), bit 65536 forces a spin
// bound of 0 on the counter-ring waits (the fault-word path).
// NW = waves per workgroup (8 or 16): waves w, w+4, w+8, w+12 share a SIMD.
// WPE: minimum waves per SIMD the register allocation must allow (launch bounds); default NW / 4 (one workgroup)
// The packed L⁻¹'s k-step pair P of row tile r (lane l: 16 B at Lp + 128 r(r+1) + 128 min(P, 2r+1) + 2l), as a buffer
// load whose wave-uniform part is the SGPR offset: the global-pointer form cost one 64-bit VALU address add per load
// on the FP64 pipe's issue port — 8 per k-step pair at RT = 8 — and was 2-3% slower (interleaved, bitwise the same:
// configs 3 / 4 / 5 10.12 / 0.621 / 10.35 → 9.92 / 0.601 / 10.02 ms, profiles/r05_t_ablate_posterior_bufA_c*.txt).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t lp_rsrc(const GPDev& g) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(g.Lp), (short)0, (int)(1024ll * g.R * (g.R + 1)),
                                           0x00020000);
}
__device__ __forceinline__ d2 load_lpair(__amdgpu_buffer_rsrc_t rsrc, int lane, int r, int P) {
  const int soff = 1024 * (r * (r + 1) + min(P, 2 * r + 1));
  return __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(rsrc, 16 * lane, soff, 0));
}

template <int RT, int CT, int DP, int KIND, int NW = 8, int ABL = 0, int WPE = NW / 4>
__global__ __launch_bounds__(64 * NW, WPE) void posterior_kernel(GPArgs args, const double* __restrict__ Xc,
                                                                     int64_t N, double* __restrict__ mu_out,
                                                                     double* __restrict__ var_out) {
  constexpr int NT = 64 * NW;                 // threads per workgroup
  constexpr int G = NW / 4;                   // waves sharing one SIMD
  constexpr int BN = 16 * CT;                 // candidates per workgroup
  constexpr int KS = kChunkRows / 4;          // MFMA k-steps per chunk (16)
  constexpr int CHUNK = kChunkRows * BN;      // doubles per LDS buffer
  constexpr int EPT = CHUNK / NT;             // generated K* elements per thread per chunk
  constexpr bool kCounters = (ABL & 32) == 0;   // counter-synchronised 3-buffer ring (default)
  constexpr int NBUF = kCounters ? 3 : 2;
  constexpr int kMaxChunks = OMB_MAX_TRAIN / kChunkRows;
  static_assert(NT % BN == 0 && CHUNK % NT == 0, "BN must divide the block");
  static_assert(2 * CHUNK >= NW * BN + NT, "epilogue scratch must fit in the K* buffers");
  // Candidate coordinates (x*/ℓ) live in registers for n_var ≤ 8; wider ones are staged in LDS
  // as [j][c] (lanes read consecutive doubles) so the 256-VGPR budget stays with the MFMA tiles.
  constexpr bool kCandLds = DP > 8 || RT >= 8;
  constexpr int kCtrDoubles = kCounters ? kMaxChunks : 0;
  // Matern: 256-entry exp table (matern_r2_tab256_x2).  ABL 16384 keeps the 64-entry table of the
  // RBF path (ablation: 10.21 → 10.12 ms at config 3, max rel. error 3.9e-14 → 1.6e-14), ABL 32768
  // drops the sqrt correction (a further −1.2%, but 5e-13 max rel. error: not used).
  constexpr bool kTab256 = !(ABL & 16384) && KIND == OMB_KERNEL_MATERN52;
  constexpr int kTabN = kTab256 ? 256 : 64;
  __shared__ double kbuf[NBUF * CHUNK + kCtrDoubles + (kCandLds ? DP * BN : 0) + kTabN];

  OMB_POST_TRACE(0);
  const int obj = blockIdx.y;
  const GPDev g = args.gp[obj];
  const int d = args.d;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t c0 = (int64_t)blockIdx.x * BN;

  // ---- this thread's generation candidate (fixed across chunks since BN | NT)
  const int cg = tid % BN;
  double b[kCandLds ? 1 : DP];
  double* cand = kbuf + NBUF * CHUNK + kCtrDoubles;
  double* etab = cand + (kCandLds ? DP * BN : 0);   // 2^(j/kTabN) for the table-driven exp
  for (int i = tid; i < kTabN; i += NT) etab[i] = kTab256 ? kExp2Tab256[i] : kExp2Tab64[i];
  __syncthreads();
  double csq = 0.0;
  if constexpr (kCandLds) {
    for (int e = tid; e < DP * BN; e += NT) {
      const int j = e / BN, c = e % BN;
      const int64_t cc = min(c0 + c, N - 1);
      cand[e] = (j < d) ? Xc[cc * d + j] / g.ls[j] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < DP; ++j) csq += cand[j * BN + cg] * cand[j * BN + cg];
  } else {
    const int64_t ci = min(c0 + cg, N - 1);
#pragma unroll
    for (int j = 0; j < DP; ++j) {
      b[j] = (j < d) ? Xc[ci * d + j] / g.ls[j] : 0.0;
      csq += b[j] * b[j];
    }
  }
  const int gen_ct = cg >> 4, gen_cc = cg & 15;
  // ---- MFMA generation: r² of a 16×16 K* tile is ⌈(d+2)/4⌉ MFMA k-steps,
  // A = training rows [x/ℓ, ‖x/ℓ‖², 1] (lane l: row l&15, dim l>>4; pre-packed Xf), B = this wave's
  // 16 candidates [−2·x*/ℓ, 1, ‖x*/ℓ‖²] (registers, loaded once).  The accumulator's register e
  // holds rows 4e + (l>>4) of the tile — exactly the B fragment of k-step 4t+e of the chunk — so
  // each lane applies the Matern transform to its 4 values and stores them to the ring as they are.
  // Rows past n need no guard: α and the L⁻¹ columns there are zero, and r² stays finite.
  constexpr bool kMfmaGen = !(ABL & 2048);   // ABL 2048: VALU dot products (ablation)
  // d ≤ 8: r² straight from the MFMA (−1% time at config 3).  Wider inputs keep the cross-term form:
  // the extra k-step bought nothing at d = 30 and its registers make the CT = 4 variants spill.
  constexpr bool kAug = DP <= 8 && !(ABL & 4096);   // ABL 4096: cross term only (ablation)
  constexpr int KSD = kAug ? (DP + 5) / 4 : (DP + 3) / 4;
  constexpr int KSDP = ((DP + 5) / 4 + 1) / 2;                 // = packed_X_pairs(DP)
  constexpr int TPC = 4 * CT;                                  // K* tiles per chunk
  constexpr int TPW = TPC >= NW ? TPC / NW : 1;                 // tiles per generating wave
  static_assert(!kMfmaGen || (NW % CT == 0 && (TPC % NW == 0 || NW % TPC == 0)), "tile deal");
  const int mg_ct = wave % CT;
  double bfr[kMfmaGen ? KSD : 1];
  double csq_m = 0.0;
  if constexpr (kMfmaGen) {
    const int64_t ci = min(c0 + 16 * mg_ct + (lane & 15), N - 1);
    auto coord = [&](int j) -> double {
      if constexpr (kCandLds) return cand[j * BN + 16 * mg_ct + (lane & 15)];
      return (j < d) ? Xc[ci * d + j] / g.ls[j] : 0.0;
    };
#pragma unroll
    for (int j = 0; j < DP; ++j) {
      const double c = coord(j);
      csq_m = fma(c, c, csq_m);
    }
#pragma unroll
    for (int s = 0; s < KSD; ++s) {
      const int j = 4 * s + (lane >> 4);
      if constexpr (kAug)
        bfr[s] = (j < d) ? -2.0 * coord(j) : (j == d ? 1.0 : (j == d + 1 ? csq_m : 0.0));
      else
        bfr[s] = (j < d) ? coord(j) : 0.0;
    }
  }
  if constexpr ((ABL & 128) != 0) {
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);
  }
  double bm2[(ABL & 512) && !kCandLds ? DP : 1];
  if constexpr ((ABL & 512) && !kCandLds) {
#pragma unroll
    for (int j = 0; j < DP; ++j) bm2[j] = -2.0 * b[j];
  }

  // ---- row-tile slots of this wave (SIMD balanced, see header): SIMD group s = wave & 3 owns
  // tile 4q + ((s + q) & 3) of every quad q; the G waves of the group take quads in snake order
  // (q mod 2G = 0,1,..,G-1,G-1,..,0), so wave h's j-th quad is 2G(j>>1) + (j odd ? 2G-1-h : h).
  const int simd = wave & 3, h = wave >> 2;
  const int Q = (g.R + 3) >> 2;  // chunks of 64 rows
  int slot_r[RT], slot_q[RT];
  const double* slot_A[RT];
#pragma unroll
  for (int j = 0; j < RT; ++j) {
    int q = 2 * G * (j >> 1) + ((j & 1) ? (2 * G - 1 - h) : h);
    int r = 4 * q + ((simd + q) & 3);
    bool ok = r < g.R;
    slot_q[j] = ok ? q : -1;
    slot_r[j] = ok ? r : 0;
    slot_A[j] = g.Lp + 128ll * slot_r[j] * (slot_r[j] + 1) + 2 * lane;
  }

  d4 acc[RT][CT];
#pragma unroll
  for (int j = 0; j < RT; ++j)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) acc[j][ct] = d4{0.0, 0.0, 0.0, 0.0};
  double mu_part = 0.0;
  const __amdgpu_buffer_rsrc_t rsrc_L = lp_rsrc(g);

  // one K* element: Matern (or RBF) of training row k and this thread's candidate
  auto element = [&](int k) -> double {
    const double* xr = g.Xs + (int64_t)k * DP;
    if constexpr ((ABL & 512) && !kCandLds) {
      double r2 = g.xsq[k] + csq;
#pragma unroll
      for (int j = 0; j < DP; ++j) r2 = fma(xr[j], bm2[j], r2);
      return (ABL & 16) ? kernel_of_r2<KIND, false>(r2, (ABL & 256) ? 1.0 : g.variance)
                        : kernel_of_r2_k<KIND>(r2, (ABL & 256) ? 1.0 : g.variance, args.ec);
    } else {
      double dot = 0.0;
#pragma unroll
      for (int j = 0; j < DP; ++j) dot = fma(xr[j], kCandLds ? cand[j * BN + cg] : b[j], dot);
      if constexpr (ABL & 1) return dot;
      return (ABL & 16) ? kernel_of_r2<KIND, false>(fma(-2.0, dot, g.xsq[k] + csq), (ABL & 256) ? 1.0 : g.variance)
                        : kernel_of_r2_k<KIND>(fma(-2.0, dot, g.xsq[k] + csq), (ABL & 256) ? 1.0 : g.variance,
                                               args.ec);
    }
  };
  // row of the chunk this lane generates in pass i; with BN = 64 a wave covers exactly one row, so
  // the row is wave-uniform and Xs / xsq / α come through scalar loads
  auto chunk_row = [&](int i) { return (BN == 64) ? wave + NW * i : (tid + NT * i) / BN; };
  static_assert(EPT % 2 == 0, "generation runs two rows per step");
  // the lockstep pair needs ~20 more VGPRs: variants already near the register limit keep one row per step
  constexpr bool kPairs = !kCandLds && !(ABL & (1 | 16 | 512));
  const double pm_s = (ABL & 256) ? 1.0 : g.variance;
  const double pm[3] = {pm_s, kSqrt5 * pm_s, kFiveThirds * pm_s};
  // n_var ≤ 8 (r² on MFMA): the generation's per-lane loads (training fragments, α) as buffer loads with the
  // wave-uniform part of the address in SGPRs, as load_lpair; rows ≥ n of α read as 0 (α's padding is 0).  Alternated
  // A/B (profiles/r05_zi_ablate_posterior_bufgen_c{3,5}.txt, r05_zj_…_c4.txt): config 3 9.94-9.98 → 9.87-9.89 ms; at d =
  // 30 (‖x/ℓ‖² loaded per element as well) it was 1.9% slower (10.01-10.08 → 10.21 ms) and stays off.  ABL 262144
  // flips the choice (tools/ablate).
  constexpr bool kBufGen = kAug != ((ABL & 262144) != 0);
  const __amdgpu_buffer_rsrc_t rsrc_X = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<double*>(g.Xf), (short)0, (int)(8ll * 4 * Q * KSDP * 128), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsrc_xsq =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(g.xsq), (short)0, 8 * g.n, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsrc_al =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(g.alpha), (short)0, 8 * g.n, 0x00020000);
  auto generate_mfma = [&](int kc, double* buf) {
    if constexpr (kMfmaGen) {
      if (NW > TPC && (wave / TPC) != kc % (NW / TPC)) return;   // other waves take this chunk
#pragma unroll
      for (int i = 0; i < TPW; ++i) {
        const int u = (NW > TPC) ? wave % TPC : wave + NW * i;
        const int t = u / CT;                                    // row tile of the chunk (0..3)
        const int rowbase = kc * kChunkRows + 16 * t;
        const d2* xa = reinterpret_cast<const d2*>(g.Xf + (int64_t)(4 * kc + t) * (KSDP * 128) + 2 * lane);
        d2 a[(KSD + 1) / 2];
#pragma unroll
        for (int p = 0; p < (KSD + 1) / 2; ++p) {
          if constexpr (kBufGen)
            a[p] = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(rsrc_X, 16 * lane,
                                                                                 8 * ((4 * kc + t) * (KSDP * 128) + 128 * p), 0));
          else
            a[p] = xa[64 * p];
        }
        d4 cr = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s = 0; s < KSD; ++s)
          cr = __builtin_amdgcn_mfma_f64_16x16x4f64((s & 1) ? a[s >> 1].y : a[s >> 1].x, bfr[s], cr, 0, 0, 0);
        auto row_val = [&](__amdgpu_buffer_rsrc_t rs, const double* __restrict__ v, int k, int kofs) -> double {
          if constexpr (kBufGen)
            return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, 8 * (lane >> 4), 8 * kofs, 0));
          else
            return v[k];
        };
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          const int k0 = rowbase + 4 * e + (lane >> 4), k1 = k0 + 4;
          double v0, v1;
          const double sf2 = (ABL & 256) ? 1.0 : g.variance;
          const double r2a = kAug ? cr[e] : fma(-2.0, cr[e], row_val(rsrc_xsq, g.xsq, k0, rowbase + 4 * e) + csq_m);
          const double r2b = kAug ? cr[e + 1] : fma(-2.0, cr[e + 1], row_val(rsrc_xsq, g.xsq, k1, rowbase + 4 * e + 4) + csq_m);
          if constexpr (ABL & 8192)   // ablation: the 17-instruction polynomial exp, two sqrt corrections
            kernel_of_r2_k_x2<KIND>(r2a, r2b, sf2, args.ec, v0, v1);
          else if constexpr (kTab256)
            matern_r2_tab256_x2<(ABL & 32768) != 0, (ABL & 524288) != 0>(r2a, r2b, pm, args.ec, etab, v0, v1);
          else
            kernel_of_r2_tab_x2<KIND>(r2a, r2b, pm, args.ec, etab, v0, v1);
          if constexpr (!kAug) {
            v0 = (k0 < g.n) ? v0 : 0.0;
            v1 = (k1 < g.n) ? v1 : 0.0;
          }
          mu_part = fma(row_val(rsrc_al, g.alpha, k0, rowbase + 4 * e), v0, mu_part);
          mu_part = fma(row_val(rsrc_al, g.alpha, k1, rowbase + 4 * e + 4), v1, mu_part);
          buf[((4 * t + e) * CT + mg_ct) * 64 + lane] = v0;
          buf[((4 * t + e + 1) * CT + mg_ct) * 64 + lane] = v1;
        }
      }
    }
  };
  auto generate = [&](int kc, double* buf) {
    if constexpr (kMfmaGen) {
      generate_mfma(kc, buf);
      return;
    }
    if (kPairs && (kc + 1) * kChunkRows <= g.n) {
      // whole chunk inside the training set: no per-row guard, and two independent rows per step
      // so the scheduler interleaves their ~50-deep fp64 dependency chains (one chain alone leaves
      // the VALU waiting on its own results about half the time)
#pragma unroll
      for (int i = 0; i < EPT; i += 2) {
        const int kl0 = chunk_row(i), kl1 = chunk_row(i + 1);
        const int k0 = kc * kChunkRows + kl0, k1 = kc * kChunkRows + kl1;
        double v0, v1;
        {
          const double* x0 = g.Xs + (int64_t)k0 * DP;
          const double* x1 = g.Xs + (int64_t)k1 * DP;
          double d0 = 0.0, d1 = 0.0;
#pragma unroll
          for (int j = 0; j < DP; ++j) {
            d0 = fma(x0[j], b[j], d0);
            d1 = fma(x1[j], b[j], d1);
          }
          kernel_of_r2_k_x2<KIND>(fma(-2.0, d0, g.xsq[k0] + csq), fma(-2.0, d1, g.xsq[k1] + csq),
                                  (ABL & 256) ? 1.0 : g.variance, args.ec, v0, v1);
        }
        mu_part = fma(g.alpha[k0], v0, mu_part);
        mu_part = fma(g.alpha[k1], v1, mu_part);
        buf[((kl0 >> 2) * CT + gen_ct) * 64 + (kl0 & 3) * 16 + gen_cc] = v0;
        buf[((kl1 >> 2) * CT + gen_ct) * 64 + (kl1 & 3) * 16 + gen_cc] = v1;
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int kl = chunk_row(i);
      const int k = kc * kChunkRows + kl;
      double val = 0.0;
      if (k < g.n) {
        val = element(k);
        mu_part = fma(g.alpha[k], val, mu_part);
      }
      buf[((kl >> 2) * CT + gen_ct) * 64 + (kl & 3) * 16 + gen_cc] = val;
    }
  };

  auto multiply = [&](int kc, const double* buf) {
    if constexpr (ABL & 2) return;
    // k-steps of each slot inside this chunk: 16 (below the diagonal quad), 4(r mod 4 + 1)
    // (diagonal quad), 0 (finished or empty slot).
    int nS[RT];
#pragma unroll
    for (int j = 0; j < RT; ++j)
      nS[j] = (slot_q[j] > kc) ? KS : (slot_q[j] == kc ? 4 * ((slot_r[j] & 3) + 1) : 0);
    const int P0 = kc * (KS / 2);
    // A (L⁻¹) k-step pairs are loaded PD pairs ahead of their MFMAs into a register ring (the sp
    // loop is fully unrolled, so ring indices are static).  With 2 waves per SIMD the ring hides
    // the L2 latency; with 4 the other waves do and the registers are worth more as occupancy.
    // PD 2 measured no faster (11.19 vs 11.16 ms); at 6 waves per SIMD (WPE, round 6) the other waves hide the latency
    constexpr int PD = (NW == 8 && WPE <= 2) ? ((ABL & 64) ? 2 : 1) : 0;
    d2 a_ring[PD + 1][RT];
    auto load_a = [&](int sp, d2* dst) {
#pragma unroll
      for (int j = 0; j < RT; ++j) {
        if constexpr (ABL & 4) {
          dst[j] = d2{1e-3 * lane + sp, 2e-3 * j};
        } else if constexpr (!(ABL & 131072)) {
          dst[j] = load_lpair(rsrc_L, lane, slot_r[j], P0 + sp);
        } else {   // ABL 131072: round 4's global load (a 64-bit VALU address add per load)
          dst[j] = *reinterpret_cast<const d2*>(slot_A[j] + 128 * min(P0 + sp, 2 * slot_r[j] + 1));
        }
      }
    };
#pragma unroll
    for (int p = 0; p < PD; ++p) load_a(p, a_ring[p]);
#pragma unroll
    for (int sp = 0; sp < KS / 2; ++sp) {
      if (sp + PD < KS / 2) load_a(sp + PD, a_ring[(sp + PD) % (PD + 1)]);
      const d2* a_cur = a_ring[sp % (PD + 1)];
      double b0[CT], b1[CT];
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        b0[ct] = buf[((2 * sp) * CT + ct) * 64 + lane];
        b1[ct] = buf[((2 * sp + 1) * CT + ct) * 64 + lane];
      }
#pragma unroll
      for (int j = 0; j < RT; ++j) {
        if (2 * sp < nS[j]) {
#pragma unroll
          for (int ct = 0; ct < CT; ++ct) {
            acc[j][ct] = __builtin_amdgcn_mfma_f64_16x16x4f64(a_cur[j].x, b0[ct], acc[j][ct], 0, 0, 0);
            acc[j][ct] = __builtin_amdgcn_mfma_f64_16x16x4f64(a_cur[j].y, b1[ct], acc[j][ct], 0, 0, 0);
          }
        }
      }
    }
  };

  if constexpr (kCounters) {
    // Three-buffer ring with per-chunk LDS counters instead of a block barrier per chunk:
    // ready[c] counts the waves whose share of K* chunk c is in LDS, done[c] the waves that have
    // finished multiplying chunk c.  A wave multiplies chunk c once ready[c] == NW and refills
    // ring slot (c+2)%3 once done[c-1] == NW, so fast waves run up to a chunk ahead of slow
    // ones.  Every wait refers to an earlier stage of every other wave (no cycle); the spins are
    // bounded anyway (args.spin_limit) so a broken invariant cannot hang the GPU, and reported.
    int* ready = reinterpret_cast<int*>(kbuf + NBUF * CHUNK);
    int* done = ready + kMaxChunks;
    if (tid < 2 * kMaxChunks) ready[tid] = 0;
    __syncthreads();
    auto signal = [&](int* ctr) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    // a wait that exhausts its bound marks the context's fault word (a system-scope vector store to
    // pinned host memory) so the next library call reports OMB_EHIP instead of returning bad moments
    const int spin_limit = (ABL & 65536) ? 0 : args.spin_limit;
    auto wait_all = [&](int* ctr) {
      if (lane == 0) {
        for (int spin = 0;; ++spin) {
          if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= NW) break;
          if (spin >= spin_limit) {
            if (args.fault) __hip_atomic_store(args.fault, kFaultSpin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    };
    OMB_POST_TRACE(1);
    generate(0, kbuf);
    signal(&ready[0]);
    if (Q > 1) {
      generate(1, kbuf + CHUNK);
      signal(&ready[1]);
    }
    for (int kc = 0; kc < Q; ++kc) {
      wait_all(&ready[kc]);
      multiply(kc, kbuf + (kc % 3) * CHUNK);
      signal(&done[kc]);
      if (kc + 2 < Q) {
        if (kc >= 1) wait_all(&done[kc - 1]);
        generate(kc + 2, kbuf + ((kc + 2) % 3) * CHUNK);
        signal(&ready[kc + 2]);
      }
    }
    OMB_POST_TRACE(2);
    __syncthreads();
    OMB_POST_TRACE(3);
  } else {
    generate(0, kbuf);
    __syncthreads();
    for (int kc = 0; kc < Q; ++kc) {
      if constexpr (NW == 8) {
        if (kc + 1 < Q) generate(kc + 1, kbuf + ((kc + 1) & 1) * CHUNK);
        multiply(kc, kbuf + (kc & 1) * CHUNK);
      } else {   // 4 waves per SIMD interleave across waves; keep each wave's live range short
        multiply(kc, kbuf + (kc & 1) * CHUNK);
        if (kc + 1 < Q) generate(kc + 1, kbuf + ((kc + 1) & 1) * CHUNK);
      }
      if constexpr (!(ABL & 8)) __syncthreads();
    }
  }

  // ---- σ²: Σ over rows of V² — registers, then lanes {l, l^16, l^32, l^48}, then waves.
  double part[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < RT; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) s = fma(acc[j][ct][i], acc[j][ct][i], s);
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    part[ct] = s;
  }
  double* red = kbuf;                 // NW waves × BN
  double* redmu = kbuf + NW * BN;     // NT partial μ
  if (lane < 16) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) red[wave * BN + ct * 16 + lane] = part[ct];
  }
  if constexpr (kMfmaGen) {
    // lanes l, l^16, l^32, l^48 hold the same candidate 16·(wave mod CT) + (l&15)
    double s = mu_part;
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    if (lane < 16) redmu[wave * 16 + lane] = s;
  } else {
    redmu[tid] = mu_part;
  }
  __syncthreads();
  if (tid < BN) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) s += red[w * BN + tid];
    double m = 0.0;
    if constexpr (kMfmaGen) {
      for (int w = tid >> 4; w < NW; w += CT) m += redmu[w * 16 + (tid & 15)];
    } else {
      for (int t = tid; t < NT; t += BN) m += redmu[t];
    }
    const int64_t c = c0 + tid;
    if (c < N) {
      mu_out[(int64_t)obj * N + c] = m;
      var_out[(int64_t)obj * N + c] = g.variance - s;
    }
  }
  OMB_POST_TRACE(4);
}

// ----------------------------------------------------------------------------- posterior, n ≤ 256
// Whole-tile variant for small training sets (BASELINE configs 2 and 4): the complete K* tile of the
// workgroup (16·RMAX rows × BN = 16·CT candidates, 64 KiB) is generated into LDS in one pass, one
// barrier, then V = L⁻¹K* runs with no further synchronisation.  With only 2-4 chunks of 64 rows the
// chunk pipeline of posterior_kernel spent a large share of each workgroup in its prologue and in
// per-chunk barriers, and its per-chunk MFMA split left SIMDs idle (at n = 128: 48 units on the
// busiest SIMD against 36 on average).  Here the multiply is balanced exactly: SIMD s owns row-tile
// pairs (q, RMAX−1−q), q ≡ s (mod 4), whose k-step counts 4(q+1) + 4(RMAX−q) are the same for every
// pair; the two waves of a SIMD split the candidate tiles.  At n_var ≤ 8 two 66-KiB workgroups share a
// CU; at n_var > 8 the staged candidates (DP·BN doubles) take a workgroup to 82–98 KiB and one per CU.
// The two workgroups do not overlap generation with multiply: FP64 VALU and FP64 MFMA share one pipe,
// and the per-workgroup timeline (tools/ablate/ablate_posterior trace, profiles/r02_v28_ablate_c2_tile_trace.txt,
// n = 128, 2^16 candidates, 2 objectives) shows a new workgroup's prologue (median 7.3 µs) waiting behind
// its neighbour's multiply (5.6 µs), then generation 2.7 µs: one workgroup leaves a CU every 8.7 µs
// against ≈ 5.8 µs of FP64-pipe work (144 MFMAs per SIMD for V, 16 for r², ≈ 640 transform VALU issues).
//   gen:  wave w takes candidate tile w mod CT and row tiles w/CT + (8/CT)·i (RMAX·CT/8 tiles).
//   K* in LDS in B-fragment order: element (row k, candidate c) at ((k/4)·CT + c/16)·64 + (k%4)·16 + c%16.
// ABL (tools/ablate only): bit 2 skips the multiply, bit 4 feeds a constant A operand, bit 8 scales the
// candidates by v_rcp_f64(ℓ) instead of dividing (timing only: not the GPy quotient).
template <int RMAX, int CT, int DP, int KIND, int ABL = 0>
__global__ __launch_bounds__(512, 2) void posterior_tile_kernel(GPArgs args, const double* __restrict__ Xc,
                                                                int64_t N, double* __restrict__ mu_out,
                                                                double* __restrict__ var_out) {
  constexpr int NW = 8, NT = 512;
  constexpr int BN = 16 * CT;
  constexpr int TILE = 4 * RMAX * CT * 64;          // doubles: 16·RMAX rows × BN candidates
  constexpr bool kAug = DP <= 8;
  constexpr int KSD = kAug ? (DP + 5) / 4 : (DP + 3) / 4;
  constexpr int KSDP = ((DP + 5) / 4 + 1) / 2;      // = packed_X_pairs(DP)
  constexpr bool kCandLds = DP > 8;
  constexpr bool kTab256 = KIND == OMB_KERNEL_MATERN52;
  constexpr int kTabN = kTab256 ? 256 : 64;
  constexpr int GT = RMAX * CT / NW;                 // generated tiles per wave
  constexpr int PPS = RMAX / 8;                      // row-tile pairs per SIMD
  constexpr int CPW = CT / 2;                        // candidate tiles per wave in the multiply
  static_assert(RMAX % 8 == 0 && CT % 2 == 0 && NW % CT == 0 && GT >= 1, "tile shape");
  static_assert(TILE >= 4 * BN + NW * 16, "reduction scratch must fit in the K* tile");
  __shared__ double kbuf[TILE + (kCandLds ? DP * BN : 0) + kTabN];

  OMB_POST_TRACE(0);
  const int obj = blockIdx.y;
  const GPDev g = args.gp[obj];
  const int d = args.d;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t c0 = (int64_t)blockIdx.x * BN;
  double* cand = kbuf + TILE;
  double* etab = cand + (kCandLds ? DP * BN : 0);
  for (int i = tid; i < kTabN; i += NT) etab[i] = kTab256 ? kExp2Tab256[i] : kExp2Tab64[i];
  if constexpr (kCandLds) {
    for (int e = tid; e < DP * BN; e += NT) {
      const int j = e / BN, c = e % BN;
      const int64_t cc = min(c0 + c, N - 1);
      cand[e] = (j < d) ? Xc[cc * d + j] / g.ls[j] : 0.0;
    }
  }

  // ---- generation operands: this wave's candidate tile as the B fragment [−2·x*/ℓ, 1, ‖x*/ℓ‖²]
  const int ct_g = wave % CT;
  const int64_t ci = min(c0 + 16 * ct_g + (lane & 15), N - 1);
  if constexpr (kCandLds) __syncthreads();
  auto coord = [&](int j) -> double {
    if constexpr (kCandLds) return cand[j * BN + 16 * ct_g + (lane & 15)];
    if constexpr (ABL & 8) return (j < d) ? Xc[ci * d + j] * __builtin_amdgcn_rcp(g.ls[j]) : 0.0;
    return (j < d) ? Xc[ci * d + j] / g.ls[j] : 0.0;
  };
  double csq = 0.0;
#pragma unroll
  for (int j = 0; j < DP; ++j) {
    const double c = coord(j);
    csq = fma(c, c, csq);
  }
  double bfr[KSD];
#pragma unroll
  for (int s = 0; s < KSD; ++s) {
    const int j = 4 * s + (lane >> 4);
    if constexpr (kAug)
      bfr[s] = (j < d) ? -2.0 * coord(j) : (j == d ? 1.0 : (j == d + 1 ? csq : 0.0));
    else
      bfr[s] = (j < d) ? coord(j) : 0.0;
  }
  const double pm[3] = {g.variance, kSqrt5 * g.variance, kFiveThirds * g.variance};
  if constexpr (!kCandLds) __syncthreads();          // etab
  OMB_POST_TRACE(1);

  double mu_part = 0.0;
#pragma unroll
  for (int i = 0; i < GT; ++i) {
    const int T = wave / CT + (NW / CT) * i;
    if (T < g.R) {
      const d2* xa = reinterpret_cast<const d2*>(g.Xf + (int64_t)T * (KSDP * 128) + 2 * lane);
      d2 a[(KSD + 1) / 2];
#pragma unroll
      for (int p = 0; p < (KSD + 1) / 2; ++p) a[p] = xa[64 * p];
      d4 cr = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s = 0; s < KSD; ++s)
        cr = __builtin_amdgcn_mfma_f64_16x16x4f64((s & 1) ? a[s >> 1].y : a[s >> 1].x, bfr[s], cr, 0, 0, 0);
#pragma unroll
      for (int e = 0; e < 4; e += 2) {
        const int k0 = 16 * T + 4 * e + (lane >> 4), k1 = k0 + 4;
        const double r2a = kAug ? cr[e] : fma(-2.0, cr[e], g.xsq[k0] + csq);
        const double r2b = kAug ? cr[e + 1] : fma(-2.0, cr[e + 1], g.xsq[k1] + csq);
        double v0, v1;
        if constexpr (kTab256)
          matern_r2_tab256_x2(r2a, r2b, pm, args.ec, etab, v0, v1);
        else
          kernel_of_r2_tab_x2<KIND>(r2a, r2b, pm, args.ec, etab, v0, v1);
        if constexpr (!kAug) {
          v0 = (k0 < g.n) ? v0 : 0.0;
          v1 = (k1 < g.n) ? v1 : 0.0;
        }
        mu_part = fma(g.alpha[k0], v0, mu_part);
        mu_part = fma(g.alpha[k1], v1, mu_part);
        kbuf[((4 * T + e) * CT + ct_g) * 64 + lane] = v0;
        kbuf[((4 * T + e + 1) * CT + ct_g) * 64 + lane] = v1;
      }
    }
  }
  OMB_POST_TRACE(2);
  __syncthreads();
  OMB_POST_TRACE(3);

  // ---- V = L⁻¹ K*: SIMD s owns the row-tile pairs (q, RMAX−1−q), q = s + 4p; wave h of the SIMD the
  // candidate tiles h·CPW .. h·CPW + CPW − 1.  A (L⁻¹) k-step pairs stream from the packed copy two
  // pairs ahead of their MFMAs.
  const int simd = wave & 3, h = wave >> 2;
  d4 acc[2 * PPS][CPW];
#pragma unroll
  for (int j = 0; j < 2 * PPS; ++j)
#pragma unroll
    for (int c = 0; c < CPW; ++c) acc[j][c] = d4{0.0, 0.0, 0.0, 0.0};
  if constexpr (!(ABL & 2)) {
#pragma unroll
    for (int j = 0; j < 2 * PPS; ++j) {
      const int q = simd + 4 * (j >> 1);
      const int r = (j & 1) ? RMAX - 1 - q : q;
      if (r >= g.R) continue;                              // wave-uniform
      const int nP = 2 * (r + 1);                          // k-step pairs of row tile r
      const d2* A = reinterpret_cast<const d2*>(g.Lp + 128ll * r * (r + 1)) + lane;
      auto ld = [&](int P) -> d2 {
        if constexpr (ABL & 4) return d2{1e-3 * lane + P, 2e-3 * j};
        return A[64 * min(P, nP - 1)];
      };
      d2 a0 = ld(0), a1 = ld(1), n0 = ld(2), n1 = ld(3);
      for (int P = 0; P < nP; P += 2) {
        const d2 f0 = ld(P + 4), f1 = ld(P + 5);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const d2 a = u ? a1 : a0;
          const int S = 2 * (P + u);
          double b0[CPW], b1[CPW];
#pragma unroll
          for (int c = 0; c < CPW; ++c) {
            b0[c] = kbuf[(S * CT + h * CPW + c) * 64 + lane];
            b1[c] = kbuf[((S + 1) * CT + h * CPW + c) * 64 + lane];
          }
#pragma unroll
          for (int c = 0; c < CPW; ++c) {
            acc[j][c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a.x, b0[c], acc[j][c], 0, 0, 0);
            acc[j][c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a.y, b1[c], acc[j][c], 0, 0, 0);
          }
        }
        a0 = n0; a1 = n1; n0 = f0; n1 = f1;
      }
    }
  }

  // ---- σ² = σ_f² − Σ rows V²: registers, lanes {l, l^16, l^32, l^48}, then the 4 SIMDs in a fixed
  // order; μ: the NW/CT generating waves of each candidate tile, in a fixed order.
  double part[CPW];
#pragma unroll
  for (int c = 0; c < CPW; ++c) {
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < 2 * PPS; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) s = fma(acc[j][c][i], acc[j][c][i], s);
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    part[c] = s;
  }
  double mp = mu_part;
  mp += __shfl_xor(mp, 16);
  mp += __shfl_xor(mp, 32);
  OMB_POST_TRACE(4);
  __syncthreads();                                  // every wave is done reading K*
  double* red = kbuf;                               // [4 SIMDs][BN]
  double* redmu = kbuf + 4 * BN;                    // [NW waves][16]
  if (lane < 16) {
#pragma unroll
    for (int c = 0; c < CPW; ++c) red[simd * BN + (h * CPW + c) * 16 + lane] = part[c];
    redmu[wave * 16 + lane] = mp;
  }
  __syncthreads();
  if (tid < BN) {
    const double s = ((red[tid] + red[BN + tid]) + red[2 * BN + tid]) + red[3 * BN + tid];
    double m = 0.0;
    for (int w = tid >> 4; w < NW; w += CT) m += redmu[w * 16 + (tid & 15)];
    const int64_t c = c0 + tid;
    if (c < N) {
      mu_out[(int64_t)obj * N + c] = m;
      var_out[(int64_t)obj * N + c] = g.variance - s;
    }
  }
  OMB_POST_TRACE(5);
}

// ----------------------------------------------------------------------------- posterior, n ≤ 128, n_var ≤ 8
// Persistent, barrier-free variant for BASELINE config 2 (n = 128, n_var = 6): L⁻¹ lives in LDS and
// K* never does.  The whole-tile kernel above spends a third of each workgroup's life outside the
// FP64 pipe (prologue behind the neighbour's multiply, one barrier, cross-wave reductions;
// profiles/r02_v28_ablate_c2_tile_trace.txt).  Here:
//   * each workgroup (one objective) stages the packed L⁻¹ (72 KiB at n = 128), α and the exp table
//     in LDS once, synchronises once, and its waves then loop independently over 16-candidate tiles
//     (wave-strided, every wave ends when the tiles run out — no further barrier);
//   * a wave generates the K* tile of training-row tile T (16 rows × its 16 candidates) with the
//     augmented r²-MFMA and the Matern transform; the accumulator's register e is the B fragment of
//     k-step 4T + e, so the four values feed the MFMAs of V = L⁻¹K* straight from registers:
//     acc[r] += L⁻¹[r, 4T..4T+3] · K*[4T..4T+3] for every row tile r ≥ T (A from LDS, 16-byte pair reads);
//   * the 8 accumulators stay in registers for the whole tile and σ² = σ_f² − Σ acc² is reduced over
//     the wave's 4 row groups by two shuffles; μ accumulates during generation the same way.
// Work per tile equals the tile kernel's (144 MFMAs for V, ⌈(d+2)/4⌉·8 for r², 32 transforms per lane);
// what goes is the idle pipe between phases.  Two 75-KiB workgroups (16 waves) share a CU; the grid is
// sized to stay resident (G·n_obj ≈ 2·CUs).  Requires n ≤ 128 (R ≤ 8) and n_var ≤ 8.
// RMAX (2, 4 or 8 row tiles) is a compile-time bound with no branch on the actual R: rows past n are
// zero in the staged L⁻¹ and α, and tiles T ≥ R reuse row tile R−1's fragments (finite values that
// meet only zeros), so the unrolled code has no wave-uniform control flow to merge around.
// Staging issues every load of the workgroup's share first (packed L⁻¹, Xf, α, the exp table: ≤ 8 per
// thread) and writes LDS after one wait, so the prologue costs one memory round trip, not one per loop
// trip and operand (the rolled loop waited vmcnt(0) after each of its 5 loads).  ℓ of the lane's B-fragment
// dimensions sits in registers from the start, so the per-tile coordinate division no longer reloads it
// (each reload's vmcnt(0) also drained the coordinate loads in flight).
// ABL (tools/ablate only): bit 1 stops after staging, bit 2 skips the multiply, bit 8 skips the
// Matern transform (K* = r²), bit 16 drops the sqrt's residual correction, bit 32 scales by 2^m with
// an integer exponent add instead of v_ldexp_f64, bit 64 loads the next tile's coordinates during the current
// tile (instead of at its start), bit 128 stages with the round-2 rolled loops and reloads ℓ per tile.
template <int RMAX, int DP, int KIND, int NW = 8, bool XL = false, int ABL = 0>
__global__ __launch_bounds__(64 * NW, NW == 8 ? 4 : NW / 4) void posterior_reg_kernel(
    GPArgs args, const double* __restrict__ Xc, int64_t N, double* __restrict__ mu_out, double* __restrict__ var_out) {
  constexpr int NT = 64 * NW;
  static_assert(DP <= 8, "augmented r² needs n_var ≤ 8");
  static_assert(RMAX >= 1 && RMAX <= 8, "n ≤ 128");
  constexpr int KSD = (DP + 5) / 4;                 // k-steps of [x/ℓ, ‖x/ℓ‖², 1]
  constexpr int KSDP = (KSD + 1) / 2;               // = packed_X_pairs(DP)
  constexpr bool kTab256 = KIND == OMB_KERNEL_MATERN52;
  constexpr int kTabN = kTab256 ? 256 : 64;
  constexpr int kL2 = 64 * RMAX * (RMAX + 1);       // d2 elements of the packed L⁻¹
  constexpr int kX2 = XL ? 64 * KSDP * RMAX : 1;    // d2 elements of the staged Xf (XL)
  __shared__ double lds_L[2 * kL2];
  __shared__ double lds_X[2 * kX2];
  __shared__ double lds_alpha[16 * RMAX];
  __shared__ double etab[kTabN];

  const int obj = blockIdx.y;
  const GPDev g = args.gp[obj];
  const int d = args.d;
  const int R = g.R;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t ntiles = (N + 15) / 16;
  const int64_t stride = (int64_t)gridDim.x * NW;
  const int64_t first = (int64_t)blockIdx.x * NW + wave;
  int64_t t = first;
  // the first tile's coordinates are in flight while the workgroup stages its operands
  auto load_raw = [&](int64_t tt, double (&raw)[KSD]) {
    const int64_t cc = min(16 * tt + (lane & 15), N - 1);
#pragma unroll
    for (int q = 0; q < KSD; ++q) {
      const int j = 4 * q + (lane >> 4);
      raw[q] = (j < d) ? Xc[cc * d + j] : 0.0;
    }
  };
  double raw[KSD];
  load_raw(t < ntiles ? t : 0, raw);
  double lsr[KSD];                                  // ℓ of this lane's B-fragment dimensions
#pragma unroll
  for (int q = 0; q < KSD; ++q) {
    const int j = 4 * q + (lane >> 4);
    lsr[q] = (j < d) ? g.ls[j] : 1.0;
  }
  if constexpr ((ABL & 128) != 0) {
    const int nL2 = 64 * R * (R + 1);
    const d2* src = reinterpret_cast<const d2*>(g.Lp);
    d2* dst = reinterpret_cast<d2*>(lds_L);
    for (int i = tid; i < kL2; i += NT) dst[i] = i < nL2 ? src[i] : d2{0.0, 0.0};
    if constexpr (XL) {
      const int nX2 = 64 * KSDP * R;
      const d2* xs2 = reinterpret_cast<const d2*>(g.Xf);
      d2* xd2 = reinterpret_cast<d2*>(lds_X);
      for (int i = tid; i < kX2; i += NT) xd2[i] = xs2[i < nX2 ? i : i % (64 * KSDP) + nX2 - 64 * KSDP];
    }
    if (tid < 16 * RMAX) lds_alpha[tid] = tid < 16 * R ? g.alpha[tid] : 0.0;
    for (int i = tid; i < kTabN; i += NT) etab[i] = kTab256 ? kExp2Tab256[i] : kExp2Tab64[i];
  } else {
    // every load first, one wait, then the LDS writes
    constexpr int kLper = (kL2 + NT - 1) / NT;
    constexpr int kXper = XL ? (kX2 + NT - 1) / NT : 0;
    constexpr int kTper = (kTabN + NT - 1) / NT;
    const int nL2 = 64 * R * (R + 1);
    const d2* src = reinterpret_cast<const d2*>(g.Lp);
    d2 lv[kLper];
#pragma unroll
    for (int k = 0; k < kLper; ++k) {
      const int i = tid + k * NT;
      lv[k] = (i < nL2) ? src[i] : d2{0.0, 0.0};   // i ≥ nL2 covers i ≥ kL2 (nL2 ≤ kL2)
    }
    d2 xv[kXper > 0 ? kXper : 1];
    if constexpr (XL) {
      const int nX2 = 64 * KSDP * R;                // row tiles past R repeat tile R−1 (see Tl below)
      const d2* xs2 = reinterpret_cast<const d2*>(g.Xf);
#pragma unroll
      for (int k = 0; k < kXper; ++k) {
        const int i = tid + k * NT;
        if (i < kX2) xv[k] = xs2[i < nX2 ? i : i % (64 * KSDP) + nX2 - 64 * KSDP];
      }
    }
    const double av = (tid < 16 * R) ? g.alpha[tid] : 0.0;
    double tv[kTper];
#pragma unroll
    for (int k = 0; k < kTper; ++k) {
      const int i = tid + k * NT;
      if (i < kTabN) tv[k] = kTab256 ? kExp2Tab256[i] : kExp2Tab64[i];
    }
    d2* dst = reinterpret_cast<d2*>(lds_L);
#pragma unroll
    for (int k = 0; k < kLper; ++k)
      if (tid + k * NT < kL2) dst[tid + k * NT] = lv[k];
    if constexpr (XL) {
      d2* xd2 = reinterpret_cast<d2*>(lds_X);
#pragma unroll
      for (int k = 0; k < kXper; ++k)
        if (tid + k * NT < kX2) xd2[tid + k * NT] = xv[k];
    }
    if (tid < 16 * RMAX) lds_alpha[tid] = av;
#pragma unroll
    for (int k = 0; k < kTper; ++k)
      if (tid + k * NT < kTabN) etab[tid + k * NT] = tv[k];
  }
  __syncthreads();
  if constexpr ((ABL & 1) != 0) return;

  const double pm[3] = {g.variance, kSqrt5 * g.variance, kFiveThirds * g.variance};
  const d2* xf = XL ? reinterpret_cast<const d2*>(lds_X) + lane : reinterpret_cast<const d2*>(g.Xf) + lane;
  for (; t < ntiles; t += stride) {
    const int64_t c = 16 * t + (lane & 15);
    if constexpr ((ABL & 64) == 0)
      if (t != first) load_raw(t, raw);
    // B fragment [−2·x*/ℓ, 1, ‖x*/ℓ‖²]: lane l needs dims 4s + (l>>4) only; ‖x*/ℓ‖² from the four
    // lane groups by two shuffles
    double xs[KSD], csq = 0.0;
#pragma unroll
    for (int q = 0; q < KSD; ++q) {
      const int j = 4 * q + (lane >> 4);
      if constexpr ((ABL & 128) != 0)
        xs[q] = (j < d) ? raw[q] / g.ls[j] : 0.0;
      else
        xs[q] = (j < d) ? raw[q] / lsr[q] : 0.0;
      csq = fma(xs[q], xs[q], csq);
    }
    if constexpr ((ABL & 64) != 0)      // the next tile's coordinates in flight during this tile
      if (t + stride < ntiles) load_raw(t + stride, raw);
    csq += __shfl_xor(csq, 16);
    csq += __shfl_xor(csq, 32);
    double bfr[KSD];
#pragma unroll
    for (int s = 0; s < KSD; ++s) {
      const int j = 4 * s + (lane >> 4);
      bfr[s] = (j < d) ? -2.0 * xs[s] : (j == d ? 1.0 : (j == d + 1 ? csq : 0.0));
    }

    d4 acc[RMAX];
    double mu_part = 0.0, s = 0.0;
#pragma unroll
    for (int T = 0; T < RMAX; ++T) {
      const int Tl = XL ? T : min(T, R - 1);        // T ≥ R: finite stand-in rows (zero L⁻¹ / α)
      d2 a[KSDP];
#pragma unroll
      for (int p = 0; p < KSDP; ++p) a[p] = xf[64 * (KSDP * Tl + p)];
      d4 cr = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int q = 0; q < KSD; ++q)
        cr = __builtin_amdgcn_mfma_f64_16x16x4f64((q & 1) ? a[q >> 1].y : a[q >> 1].x, bfr[q], cr, 0, 0, 0);
      double kv[4];
#pragma unroll
      for (int e = 0; e < 4; e += 2) {
        if constexpr ((ABL & 8) != 0) {
          kv[e] = cr[e];
          kv[e + 1] = cr[e + 1];
        } else if constexpr (kTab256) {
          matern_r2_tab256_x2<(ABL & 16) != 0, (ABL & 32) != 0>(cr[e], cr[e + 1], pm, args.ec, etab, kv[e], kv[e + 1]);
        } else {
          kernel_of_r2_tab_x2<KIND>(cr[e], cr[e + 1], pm, args.ec, etab, kv[e], kv[e + 1]);
        }
        mu_part = fma(lds_alpha[16 * T + 4 * e + (lane >> 4)], kv[e], mu_part);
        mu_part = fma(lds_alpha[16 * T + 4 * e + 4 + (lane >> 4)], kv[e + 1], mu_part);
      }
      if constexpr (!(ABL & 2)) {
#pragma unroll
        for (int r = T; r < RMAX; ++r) {
          const d2* A = reinterpret_cast<const d2*>(lds_L + 128 * r * (r + 1) + 256 * T) + lane;
          const d2 a0 = A[0], a1 = A[64];
          d4 v = (T == 0) ? d4{0.0, 0.0, 0.0, 0.0} : acc[r];
          v = __builtin_amdgcn_mfma_f64_16x16x4f64(a0.x, kv[0], v, 0, 0, 0);
          v = __builtin_amdgcn_mfma_f64_16x16x4f64(a0.y, kv[1], v, 0, 0, 0);
          v = __builtin_amdgcn_mfma_f64_16x16x4f64(a1.x, kv[2], v, 0, 0, 0);
          acc[r] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1.y, kv[3], v, 0, 0, 0);
        }
      } else {
        acc[T] = d4{kv[0], kv[1], kv[2], kv[3]};
      }
      // row tile T has all its k-steps (T' ≤ T): retire its accumulator, so at most RMAX − T are live
#pragma unroll
      for (int i = 0; i < 4; ++i) s = fma(acc[T][i], acc[T][i], s);
    }
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    mu_part += __shfl_xor(mu_part, 16);
    mu_part += __shfl_xor(mu_part, 32);
    if (lane < 16 && c < N) {
      mu_out[(int64_t)obj * N + c] = mu_part;
      var_out[(int64_t)obj * N + c] = g.variance - s;
    }
  }
}

// Resident grid of posterior_reg_kernel: two workgroups per CU over all objectives.
static int device_cu_count() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cached[dev] == 0) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    cached[dev] = cus;
  }
  return cached[dev];
}

static dim3 reg_grid(int64_t N, int n_obj, int NW = 8, int per_cu = 2) {
  const int64_t waves_needed = (N + 15) / 16;
  const int64_t wgs = (waves_needed + NW - 1) / NW;
  const int64_t resident = std::max<int64_t>(1, (per_cu * (int64_t)device_cu_count()) / std::max(1, n_obj));
  return dim3((unsigned)std::max<int64_t>(1, std::min(wgs, resident)), (unsigned)n_obj);
}

// ----------------------------------------------------------------------------- dispatch
template <int DP, int KIND>
static hipError_t launch_posterior_dp(hipStream_t stream, const GPArgs& args, int n_obj, int max_R,
                                      const double* Xc, int64_t N, double* mu, double* var) {
  const int Q = (max_R + 3) / 4;
  const int RTneed = (Q + 1) / 2;
  if (RTneed <= 1 && DP <= 8) {
    // n ≤ 128, n_var ≤ 8: persistent, L⁻¹ in LDS, K* in registers (posterior_reg_kernel)
    if constexpr (DP <= 8) {
      // 16 waves, one workgroup per CU, training rows staged in LDS: 0.062 ms at config 2 against
      // 0.066 for two 8-wave workgroups per CU (profiles/r02_v49_ablate_c2.txt)
      const dim3 grid = reg_grid(N, n_obj, 16, 1);
      const dim3 block(1024);
      if (max_R <= 2)
        hipLaunchKernelGGL((posterior_reg_kernel<2, DP, KIND, 16, true>), grid, block, 0, stream, args, Xc, N, mu, var);
      else if (max_R <= 4)
        hipLaunchKernelGGL((posterior_reg_kernel<4, DP, KIND, 16, true>), grid, block, 0, stream, args, Xc, N, mu, var);
      else
        hipLaunchKernelGGL((posterior_reg_kernel<8, DP, KIND, 16, true>), grid, block, 0, stream, args, Xc, N, mu, var);
    }
  } else if (RTneed <= 1) {
    // n ≤ 128, n_var > 8: the whole 128 × 64 K* tile in LDS, one barrier, balanced multiply (tools/ablate
    // at n = 128, 2 objectives, 2^16 candidates: 0.083 ms for the r01 chunk pipeline → 0.074 ms;
    // profiles/r02_v11_ablate_c2.txt)
    dim3 grid((unsigned)((N + 63) / 64), n_obj);
    hipLaunchKernelGGL((posterior_tile_kernel<8, 4, DP, KIND>), grid, dim3(kBlockThreads), 0, stream, args, Xc, N, mu, var);
  } else if (RTneed <= 2) {
    // 128 < n ≤ 256: 32-candidate blocks on the counter ring (48 KiB, several workgroups per CU);
    // tools/ablate at n = 256, 3 objectives, 2^17 candidates: 0.709 ms (CT 4, barrier) → 0.641 ms;
    // the whole-tile kernel (RMAX 16, CT 2) takes 0.688 ms there (profiles/r02_v2_ablate_c4.txt).
    // Round 6: n_var ≤ 8 (51 KiB of LDS) with the register budget of 6 waves per SIMD — three workgroups per CU
    // instead of two (80 VGPRs, a few spilled, no A-operand prefetch ring: the other waves hide its latency) — ≈ 4%
    // faster, alternated against the 2-wave build in one process (0.557-0.571 against 0.583-0.593 ms at config 4,
    // profiles/r06_s_ablate_posterior_c4_wpe6*.txt).  With staged candidates (n_var > 8) the LDS allows two.
    dim3 grid((unsigned)((N + 31) / 32), n_obj);
    if constexpr (DP <= 8)
      hipLaunchKernelGGL((posterior_kernel<2, 2, DP, KIND, 8, 0, 6>), grid, dim3(kBlockThreads), 0, stream, args, Xc, N, mu,
                         var);
    else
      hipLaunchKernelGGL((posterior_kernel<2, 2, DP, KIND, 8, 0>), grid, dim3(kBlockThreads), 0, stream, args, Xc, N, mu,
                         var);
  } else if (RTneed <= 4) {
    // 256 < n ≤ 512 (BASELINE config 3).  Round 6: n_var ≤ 8 as 32-candidate blocks (CT 2) in the register budget of
    // 4 waves per SIMD — two workgroups per CU (118 VGPRs, 51 KiB of LDS each) instead of one 64-candidate workgroup
    // (214 VGPRs, 100 KiB): one workgroup's prologue, chunk hand-offs and reduction overlap the other's multiply.
    // Alternated in one process at config 3 (n 512, 2^20 candidates, 2 objectives): 9.57 against 9.97 ms, μ within
    // 1.2e-14 relative (the per-wave μ partials meet in another order), σ² bitwise (profiles/r06_u_ablate_posterior_c3*.txt).
    // Wider inputs stage the candidates in LDS and spill at this budget: they keep the 64-candidate kernel.
    if constexpr (DP <= 8) {
      dim3 grid((unsigned)((N + 31) / 32), n_obj);
      hipLaunchKernelGGL((posterior_kernel<4, 2, DP, KIND, 8, 0, 4>), grid, dim3(kBlockThreads), 0, stream, args, Xc, N, mu,
                         var);
    } else {
      dim3 grid((unsigned)((N + 63) / 64), n_obj);
      hipLaunchKernelGGL((posterior_kernel<4, 4, DP, KIND>), grid, dim3(kBlockThreads), 0, stream, args, Xc, N, mu, var);
    }
  } else if (RTneed <= 8) {
    dim3 grid((unsigned)((N + 31) / 32), n_obj);
    hipLaunchKernelGGL((posterior_kernel<8, 2, DP, KIND>), grid, dim3(kBlockThreads), 0, stream, args, Xc, N, mu, var);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <int KIND>
static hipError_t launch_posterior_kind(hipStream_t stream, const GPArgs& args, int n_obj, int max_R,
                                        const double* Xc, int64_t N, double* mu, double* var) {
  switch (args.DP) {
    case 2: return launch_posterior_dp<2, KIND>(stream, args, n_obj, max_R, Xc, N, mu, var);
    case 4: return launch_posterior_dp<4, KIND>(stream, args, n_obj, max_R, Xc, N, mu, var);
    case 6: return launch_posterior_dp<6, KIND>(stream, args, n_obj, max_R, Xc, N, mu, var);
    case 8: return launch_posterior_dp<8, KIND>(stream, args, n_obj, max_R, Xc, N, mu, var);
    case 16: return launch_posterior_dp<16, KIND>(stream, args, n_obj, max_R, Xc, N, mu, var);
    case 32: return launch_posterior_dp<32, KIND>(stream, args, n_obj, max_R, Xc, N, mu, var);
    case 64: return launch_posterior_dp<64, KIND>(stream, args, n_obj, max_R, Xc, N, mu, var);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_posterior(hipStream_t stream, const GPArgs& args_in, int n_obj, int max_R, const double* Xc,
                            int64_t N, double* mu, double* var) {
  GPArgs args = args_in;
  args.ec = exp_coef();
  if (args.gp[0].kind == OMB_KERNEL_RBF) return launch_posterior_kind<OMB_KERNEL_RBF>(stream, args, n_obj, max_R, Xc, N, mu, var);
  return launch_posterior_kind<OMB_KERNEL_MATERN52>(stream, args, n_obj, max_R, Xc, N, mu, var);
}

template <int KIND>
static hipError_t launch_kblock_kind(hipStream_t stream, const GPArgs& args, int obj, const double* Xc, int64_t N,
                                     double* K) {
  const GPDev& g = args.gp[obj];
  // LDS-staged fragments (the store loop issues no loads, so the store queue never drains), persistent over
  // CB blocks of 128 candidates (kernel_block_persist_kernel; tools/ablate/ablate_kblock3,
  // profiles/r03_v7_ablate_kblock3_c*.txt):
  //   n_var ≤ 8: CB = 1 (n = 512, d = 6, N = 2^20: 0.867 ms for kernel_block_pipe_kernel → 0.828 ms; more
  //              blocks per workgroup cost occupancy there, 0.995 ms at CB = 4);
  //   n_var > 8: CB = 8 with 1/ℓ multiplies and the block loop not unrolled (n = 1024, d = 30, N = 2^19:
  //              1.463 → 1.230 ms, profiles/r03_v9_ablate_kblock3_c5.txt; the staging and the per-candidate
  //              divisions are paid once per 8 blocks; outputs within 1.2e-14 of the division form).
  //   small batches (TuRBO's K*, N ≤ 5000) keep CB = 1: the grid must still cover the CUs.
  auto grid = [&](int DP, int CB) {
    return dim3((unsigned)((N + 128 * CB - 1) / (128 * CB)), (unsigned)((g.n + kblock_rows(DP) - 1) / kblock_rows(DP)));
  };
  // the launch itself: 1-D, XCD-aware order when there are several row blocks (see the kernel)
  auto grid1 = [&](int DP, int CB) {
    const dim3 gr = grid(DP, CB);
    return gr.y > 1 ? dim3((unsigned)((gr.x + 7) / 8 * 8 * gr.y)) : gr;
  };
  auto nxy = [&](int DP, int CB, int& nx, int& ny) {
    const dim3 gr = grid(DP, CB);
    nx = gr.y > 1 ? (int)gr.x : 0;
    ny = (int)gr.y;
  };
  int nx = 0, ny = 0;
  auto pick_cb = [&](int DP) {
    for (int cb = 8; cb > 1; cb >>= 1) {
      const dim3 gr = grid(DP, cb);
      if ((int64_t)gr.x * gr.y >= 2048) return cb;
    }
    return 1;
  };
  if (args.DP > kMaxFusedDP)   // n_var > 64: GEMM-tiled cross term over LDS slabs (omb_wide.hip)
    return launch_kernel_block_wide(stream, g, args.d, args.DP, Xc, N, K, N);
  switch (args.DP) {
#define OMB_KBS(DPV) \
  case DPV:                                                                                                     \
    nxy(DPV, 1, nx, ny);                                                                                        \
    hipLaunchKernelGGL((kernel_block_persist_kernel<DPV, KIND, 1, false>), grid1(DPV, 1), dim3(512), 0, stream, g, args.d, Xc, N, K, exp_coef(), nx, ny); \
    break;
#define OMB_KBW_CB(DPV, CBV)                                                                                  \
  case CBV:                                                                                                     \
    nxy(DPV, CBV, nx, ny);                                                                                      \
    if (args.d + 2 <= 4 * ((DPV + 3) / 4))                                                                      \
      hipLaunchKernelGGL((kernel_block_persist_kernel<DPV, KIND, CBV, true, true, true>), grid1(DPV, CBV), dim3(512), 0, stream, g, args.d, Xc, N, K, exp_coef(), nx, ny); \
    else                                                                                                        \
      hipLaunchKernelGGL((kernel_block_persist_kernel<DPV, KIND, CBV, true, true>), grid1(DPV, CBV), dim3(512), 0, stream, g, args.d, Xc, N, K, exp_coef(), nx, ny); \
    break;
#define OMB_KBW(DPV) \
  case DPV:                                                                  \
    switch (pick_cb(DPV)) {                                                  \
      OMB_KBW_CB(DPV, 8) OMB_KBW_CB(DPV, 4) OMB_KBW_CB(DPV, 2) OMB_KBW_CB(DPV, 1) \
      default: return hipErrorInvalidValue;                                  \
    }                                                                        \
    break;
    OMB_KBS(2) OMB_KBS(4) OMB_KBS(6) OMB_KBS(8) OMB_KBW(16) OMB_KBW(32) OMB_KBW(64)
#undef OMB_KBS
#undef OMB_KBW
#undef OMB_KBW_CB
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_kernel_block(hipStream_t stream, const GPArgs& args, int obj, const double* Xc, int64_t N,
                               double* K) {
  if (args.gp[obj].kind == OMB_KERNEL_RBF) return launch_kblock_kind<OMB_KERNEL_RBF>(stream, args, obj, Xc, N, K);
  return launch_kblock_kind<OMB_KERNEL_MATERN52>(stream, args, obj, Xc, N, K);
}

}  // namespace omb
