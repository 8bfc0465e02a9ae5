// Dense fp64 linear algebra on gfx950 for TuRBO's Thompson sampling.
//
// TuRBO draws `batch_size` joint samples of the GP at up to 5,000 trust-region candidates
// (optimobo/algorithms/turbo.py:114, GPy GP.posterior_samples), i.e.
//   PosteriorExact._raw_predict(full_cov=True):  μ = K*ᵀα,  Σ = K(X*, X*) − (L⁻¹K*)ᵀ(L⁻¹K*)
//   numpy.random.multivariate_normal(μ, Σ, size)      (an O(N³) SVD on the host)
// and then takes the arg-min of every sample, greedily excluding earlier picks
// (TuRBO_1.select_candidates turbo.py:142-153, TuRBO_M._select_candidates turbo.py:365-383).
//
//   gemm_kernel        (omb_gemm.hip) V = L⁻¹K*, Σ −= VᵀV, the draws μ + L z and the triangular inverse.
//   cand_cov_kernel    lower triangle of K(X*, X*) (GPy _unscaled_dist: diagonal forced to 0).
//   chol_*_kernel      blocked right-looking Cholesky in 64-column steps (see "Cholesky, fused steps").
//   select_kernel      the greedy per-sample arg-min (np.argmin order) with an LDS exclusion bitmap.
// The factor is chol(Σ + jitter·I): numpy factors Σ by SVD instead; both draw from N(μ, Σ) up to
// the jitter, which the caller bounds (omb_posterior_samples).
#include <algorithm>
#include <mutex>
#include <type_traits>
#include <vector>

#include "omb_internal.h"
#include "omb_math.h"

namespace omb {

typedef double d4 __attribute__((ext_vector_type(4)));

// GEMM (gemm_kernel and its launchers): omb_gemm.hip


// ----------------------------------------------------------------------------- K(X*, X*)
// GPy Stationary._unscaled_dist(X) on X/ℓ: r² = −2·(aᵢ·aⱼ) + (‖aᵢ‖² + ‖aⱼ‖²), diagonal forced
// to 0, clipped at 0; then K_of_r.  Lower triangle only (j ≤ i).
//   cand_scale_kernel  a = X/ℓ (GPy divides; once per element, not per pair) into rows of KP = ⌈DP/4⌉·4
//                      doubles (zero padded) and ‖a‖² (a shuffle tree over the row's lanes);
//   cand_cov_kernel    one 64×64 lower tile per 256-thread workgroup (4 waves × 32×32, gemm_kernel's
//                      tiling), the cross term aᵢ·aⱼ on v_mfma_f64_16x16x4f64 over KP/4 k-steps from LDS,
//                      the kernel transform fused into the store.
// Round 2's kernel divided by ℓ inside every pair and read both rows per thread (203 µs for the
// lower triangle at N = 3000, d = 30: profiles/r02_v21_c6_kernel_stats.csv).
template <int DP>
__global__ __launch_bounds__(256) void cand_scale_kernel(const double* __restrict__ Xc, int d, int64_t N,
                                                         const double* __restrict__ ls, double* __restrict__ Xs,
                                                         double* __restrict__ xsq) {
  // one thread per (candidate, coordinate), KP (a power of two ≤ 64) lanes per candidate; ‖a‖² by a
  // shuffle tree over the candidate's lanes (round 2 ran one thread per candidate: 13.6 µs at N = 3000, d = 30)
  constexpr int KP = (DP + 3) / 4 * 4;
  static_assert((KP & (KP - 1)) == 0 && KP <= 64, "KP lanes of one wave per candidate");
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t i = t / KP;
  const int k = (int)(t % KP);
  double a = 0.0;
  if (i < N && k < d) a = Xc[i * d + k] / ls[k];
  if (i < N) Xs[i * KP + k] = a;
  double s = a * a;
#pragma unroll
  for (int o = KP / 2; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (i < N && k == 0) xsq[i] = s;
}

// TAB (Matern 5/2 only; omb_debug_set(OMB_DEBUG_COV_TABLE)): the posterior kernels' table-driven transform
// matern_r2_tab256_x2 in place of kernel_of_r2 (DESIGN §4b "Covariance on the table transform").
template <int DP, int KIND, bool TAB>
__global__ __launch_bounds__(256) void cand_cov_kernel(const double* __restrict__ Xs, const double* __restrict__ xsq,
                                                       int64_t N, double variance, double* __restrict__ S,
                                                       int64_t lds, double diag_add, ExpCoef ec) {
  constexpr int KP = (DP + 3) / 4 * 4;
  if (blockIdx.x > blockIdx.y) return;
  const int64_t m0 = (int64_t)blockIdx.y * 64, n0 = (int64_t)blockIdx.x * 64;
  __shared__ double As[KP][65], Bs[KP][65];   // As[k][m] = a_{m0+m}[k]
  __shared__ double etab[TAB ? 256 : 1];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  if constexpr (TAB) etab[tid] = kExp2Tab256[tid];                          // 256 threads
  for (int idx = tid; idx < 64 * KP; idx += 256) {
    const int m = idx / KP, k = idx % KP;
    As[k][m] = (m0 + m < N) ? Xs[(m0 + m) * KP + k] : 0.0;
    Bs[k][m] = (n0 + m < N) ? Xs[(n0 + m) * KP + k] : 0.0;
  }
  __syncthreads();
  d4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int ks = 0; ks < KP / 4; ++ks) {
    const int kk = 4 * ks + (lane >> 4);
    const double a0 = As[kk][32 * wm + (lane & 15)];
    const double a1 = As[kk][32 * wm + 16 + (lane & 15)];
    const double b0 = Bs[kk][32 * wn + (lane & 15)];
    const double b1 = Bs[kk][32 * wn + 16 + (lane & 15)];
    acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
  }
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    const int64_t col = n0 + 32 * wn + 16 * cb + (lane & 15);
    const double bsq = col < N ? xsq[col] : 0.0;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      double r2[4], kv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t row = m0 + 32 * wm + 16 * rb + (lane >> 4) + 4 * e;
        const double asq = row < N ? xsq[row] : 0.0;
        r2[e] = (row == col) ? 0.0 : fma(-2.0, acc[rb][cb][e], asq + bsq);
      }
      if constexpr (TAB && KIND == OMB_KERNEL_MATERN52) {
        const double pm[3] = {variance, kSqrt5 * variance, kFiveThirds * variance};
        matern_r2_tab256_x2(r2[0], r2[1], pm, ec, etab, kv[0], kv[1]);
        matern_r2_tab256_x2(r2[2], r2[3], pm, ec, etab, kv[2], kv[3]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) kv[e] = kernel_of_r2<KIND>(r2[e], variance);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t row = m0 + 32 * wm + 16 * rb + (lane >> 4) + 4 * e;
        if (row < N && col <= row) S[row * lds + col] = (row == col) ? kv[e] + diag_add : kv[e];
      }
    }
  }
}

__global__ __launch_bounds__(256) void mirror_lower_kernel(double* __restrict__ S, int64_t N, int64_t lds) {
  // S[i][j] = S[j][i] for j > i, 32×32 tiles through LDS (both sides coalesced)
  if (blockIdx.x < blockIdx.y) return;
  __shared__ double t[32][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 32 × 8
  const int64_t bi = (int64_t)blockIdx.y * 32, bj = (int64_t)blockIdx.x * 32;   // upper tile rows bi, cols bj
  for (int r = ty; r < 32; r += 8) {
    const int64_t src_row = bj + r, src_col = bi + tx;    // lower tile (rows bj.., cols bi..)
    if (src_row < N && src_col < N) t[r][tx] = S[src_row * lds + src_col];
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int64_t row = bi + r, col = bj + tx;
    if (row < N && col < N && col > row) S[row * lds + col] = t[tx][r];
  }
}

__global__ void add_diag_kernel(double* __restrict__ S, int64_t N, int64_t lds, double v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < N) S[i * lds + i] += v;
}

// ----------------------------------------------------------------------------- Cholesky
constexpr int kNB = 64;

// Phase timestamps of the diagonal-block factorisation for tools/ablate/ablate_chol (empty here).
#ifndef OMB_CHOL_TRACE
#define OMB_CHOL_TRACE(id, cond)
#endif
// per-column timestamps (wave w done with column j) for tools/ablate/ablate_chol (empty here)
#ifndef OMB_CHOL_COL
#define OMB_CHOL_COL(w, j, cond)
#endif

__device__ __forceinline__ double readlane_f64(double v, int l) {
  const long long b = __builtin_bit_cast(long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(b & 0xffffffffll), l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(b >> 32), l);
  return __builtin_bit_cast(double, (long long)(((unsigned long long)hi << 32) | lo));
}

// v[k] += s·w[k] for k = j+1 .. 63, w a same-address (broadcast) LDS row: the loads go out 16
// values (8 ds_read_b128) at a time ahead of their fmas, so the LDS latency is paid once per 16
// columns instead of once per load (j is a compile-time constant in the unrolled callers).
template <int J>
__device__ __forceinline__ void axpy_tail(double (&v)[kNB], double s, const double* w) {
#pragma unroll
  for (int kb = (J + 1) / 16 * 16; kb < kNB; kb += 16) {
    double2 wv[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) wv[q] = reinterpret_cast<const double2*>(w + kb)[q];
#pragma unroll
    for (int q = 0; q < 16; ++q)
      if (kb + q > J) v[kb + q] = fma(s, (q & 1) ? wv[q >> 1].y : wv[q >> 1].x, v[kb + q]);
  }
}

// Compile-time loop: f(std::integral_constant<int, I>) for I = B .. E-1.
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// ----------------------------------------------------------------------------- Cholesky, fused steps
// The blocked factorisation per 64-column step k (launch_cholesky; round 3 folds the panel into the update
// launch, see chol_update_kernel<FUSE>):
//   chol_panel_kernel   the panel below the diagonal block, L21 = A21 · W_kkᵀ with W_kk = L_kk⁻¹, on
//                       MFMA (16 rows per 2-wave workgroup; W_kk's B fragments read from the workspace);
//   chol_update_kernel  the trailing update A22 −= L21 L21ᵀ (lower triangle, 64×64 MFMA tiles) whose
//                       workgroup owning the next diagonal tile factors it right after its update
//                       (chol64_factor), inverts the factor and writes L_{k+1,k+1} and the fragments of
//                       W_{k+1,k+1} for the next panel (chol64_factor, chol64_inverse);
//   chol_diag_kernel    step 0's diagonal block (nothing precedes it).
// The serial chain of a step is the diagonal workgroup's factor + inverse.  Round 2's panel solved
// x · L_kkᵀ = b by substitution, a 64-step dependent chain per row with an LDS broadcast read at every
// step (29.5 µs per step at N = 3000, profiles/r02_v20_c6_top_kernels.txt), and the factor broadcast each
// column through LDS (29.9 µs for the update kernel's diagonal workgroup).  Solving with the explicit
// inverse of the 64×64 diagonal block is the usual GPU TRSM; its error grows with cond(L_kk), which
// the jitter of omb_posterior_samples bounds.

// LDS of the diagonal-block factorisation (diagonal workgroups of chol_update_kernel, chol_diag_kernel):
//   Lb    4 sub-blocks × 64 rows × kLbP doubles: Lb[(b·64 + r)·kLbP + q] = L[r][16b + q]; the 144-B row
//         pitch keeps 16 lanes reading 16 different rows conflict-free;
//   aux   cbuf (2 × 64: the current column, double buffered) | dinv (64: 1/L_jj);
//   prog  8 ints: columns of sub-block b published to Lb so far (0..3); W_bb in Lb (4..7).
constexpr int kLbP = 18;
constexpr int kLbDoubles = 4 * kNB * kLbP;
constexpr int kCholAux = 2 * kNB + kNB;

// The W fragments are stored and (by the fused step's waiting workgroups) read as agent-scope relaxed
// atomics: coherent across the XCDs' L2s without the L2 write-back / invalidate that an agent-scope
// release / acquire fence costs (those fences cost more than the launch they were meant to save).
__device__ __forceinline__ void wf_store(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), __builtin_bit_cast(unsigned long long, v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double wf_load(const double* p) {
  return __builtin_bit_cast(double, __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT));
}

// The off-diagonal blocks of W = L⁻¹ into Wf, the MFMA B fragments of chol_panel_kernel:
//   Wf[(jb·16 + s)·64 + l] = W[16jb + (l & 15)][m(s, l >> 4)],   m(s, g) = 16(s >> 2) + 4g + (s & 3)
// (k-step s of the panel's output column block jb; only s < 4(jb + 1) is read — the rest of that row
// block of W is zero — so the panel skips W's upper triangle in whole k-steps).
// Wave j forms its column block, W_ij = −W_ii Σ_{k=j}^{i−1} L_ik W_kj for i = j+1..3, on MFMA: a product's
// accumulator layout (lane l: rows 4e + (l >> 4), column l & 15) is the next product's B operand
// layout, so the W_kj (k > j) stay in registers and only L and the W_ii are read from LDS.
// Round 3: each wave runs this right after its own sub-block's tail, while the later waves still factor.
// The sums Σ L_ik W_kj need only L (complete for row block i once sub-blocks < i are factored) and the
// wave's own earlier blocks; only the final product waits for W_ii (wdone[i], set by wave i after its
// tail).  After the last sub-block only the three products with W_33 remain (the whole inverse used to
// follow a barrier after the factor: ≈ 4.8k cycles on the step's chain, profiles/r03_v37_chol_trace_paired_consumer.txt).
__device__ __forceinline__ void chol64_inverse(int w, int r, const double* Lb, int* wdone, double* __restrict__ Wf) {
  const int c = r & 15, g = r >> 4;
  d4 Wc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) Wc[i] = d4{0.0, 0.0, 0.0, 0.0};
  static_for<1, 4>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    if (i > w) {
      d4 T = d4{0.0, 0.0, 0.0, 0.0};
      static_for<0, i>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        if (k >= w) {
          static_for<0, 4>([&](auto sc) {
            constexpr int s = decltype(sc)::value;
            const double av = Lb[(k * 64 + 16 * i + c) * kLbP + 4 * s + g];   // L[16i + c][16k + 4s + g]
            // B operand W_kj[4s + g][c]: W_ww from LDS, the others from registers
            const double bv = (k == w) ? Lb[(k * 64 + 16 * k + 4 * s + g) * kLbP + c] : Wc[k][s];
            T = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, T, 0, 0, 0);
          });
        }
      });
      // W_ii in Lb (published by wave i after its tail)
      while (__hip_atomic_load(&wdone[i], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
        __builtin_amdgcn_s_sleep(1);
      d4 R = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s = 0; s < 4; ++s)
        R = __builtin_amdgcn_mfma_f64_16x16x4f64(Lb[(i * 64 + 16 * i + c) * kLbP + 4 * s + g], T[s], R, 0, 0, 0);
      Wc[i] = -R;
      // W[16i + 4e + g][16w + c]: jb = i, s = 4w + (c & 3), lane 4e + g + 16 (c >> 2)
#pragma unroll
      for (int e = 0; e < 4; ++e) wf_store(&Wf[(i * 16 + 4 * w + (c & 3)) * 64 + 4 * e + g + 16 * (c >> 2)], Wc[i][e]);
    }
  });
  OMB_CHOL_TRACE(16, w == 0 && r == 0);
}

// Factor a 64×64 SPD block with the 4 waves of a 256-thread workgroup: thread (wave w, lane r) holds
// a[q] = A[r][16w + q] (only 16w + q ≤ r is meaningful; rows past the block are identity rows).
// Wave b factors sub-block b (columns 16b..16b+15).  Before its turn it applies every earlier
// sub-block's columns to its own 16 columns as they are published (a progress counter per sub-block
// in LDS; L[r][j]·L[16w+q][j] from Lb), so when the previous wave finishes, the next one starts at once
// — round 2's bulk update after every 16 columns took ≈ 2 µs each (profiles/r02_v24_ablate_chol.txt).
// Column j of the own sub-block:
//   * the serial chain runs on wave-uniform values: d_{j+1} = A'_{j+1,j+1} − (a_{j+1,j}·inv_j)², where
//     A' and a_{j+1,j} were read (v_readlane) before inv_j is known — 9 dependent FP64 ops per column
//     (rsq, two Newton steps, one mul, one fma);
//   * the next two rows' entries of column j are applied at once (uniform scalars a_{j+k,j}·inv_j), the
//     rest one column later from an LDS broadcast of the column (software pipeline);
//   * the column goes to Lb for the later waves, then the progress counter moves (release order).
// Entries above the diagonal are not kept at zero (a[jj] is scaled on every row, no selects); they
// only ever feed entries above the diagonal of the same row, which nothing reads.
// When its sub-block is done, the wave stores its 16 columns of L into A (rows < nb), then inverts its
// 16×16 diagonal block by substitution (x[m] = (δ_mc − Σ_{p<m} L_ww[m][p] x[p]) / L_ww[m][m], lane l →
// column l & 15, rows of L_ww as LDS broadcasts), leaves W_ww in place of L_ww in Lb and writes W_ww's
// fragments to Wf (see chol64_inverse) — while the later waves are still factoring.
// bad_lds[0] = 1-based first non-positive pivot column or 0 (valid after the caller's barrier).
__device__ __forceinline__ void chol64_factor(double (&a)[16], int w, int r, int nb, double* Lb, double* aux,
                                              int* prog, int* bad_lds, double* __restrict__ A, int64_t lda,
                                              int64_t c0, double* __restrict__ Wf) {
  double* dinv = aux + 2 * kNB;
  // ---- earlier sub-blocks' columns, as they appear
#pragma unroll 1
  for (int b = 0; b < w; ++b) {
    // two published columns per step: row q's entries of columns jj, jj+1 are adjacent in Lb (one b128
    // read), so a step is 17 b128 reads and 32 fmas (in column order: bitwise the one-column loop); one
    // column per step took ≈ 530 cycles against the owner's ≈ 470 and fell ≈ 1,300 cycles behind per
    // sub-block (profiles/r03_v27_chol_column_trace.txt)
#pragma unroll 1   // rolled: unrolled, the column reads were merged and hoisted (512 VGPRs + spills)
    for (int jj = 0; jj < 16; jj += 2) {
      while (__hip_atomic_load(&prog[b], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <= jj + 1)
        __builtin_amdgcn_s_sleep(1);
      const double2 lr = *reinterpret_cast<const double2*>(Lb + (b * 64 + r) * kLbP + jj);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const double2 v = *reinterpret_cast<const double2*>(Lb + (b * 64 + 16 * w + q) * kLbP + jj);
        a[q] = fma(-lr.x, v.x, a[q]);
        a[q] = fma(-lr.y, v.y, a[q]);
      }
      OMB_CHOL_COL(w, 16 * b + jj + 1, r == 0);
    }
  }
  // ---- own sub-block
  static_for<0, 4>([&](auto bc) {
    constexpr int b = decltype(bc)::value;
    if (w != b) return;
    OMB_CHOL_TRACE(2 + 2 * b, r == 0);
    int bad = 0;
    double dj = readlane_f64(a[0], 16 * b);          // first pivot (every earlier column applied)
    double pl = 0.0;   // the previous column's entry of this row
    double pv[16];     // the previous column's entries L[16b+q][j−1] (q ≥ jj+2), from LDS
    // order within column j: chain (pre-read entries, inv, next pivot), scale + the next two rows,
    // publish (Lb, progress), then column j−1's deferred updates, then column j's broadcast loads —
    // the loads' LDS latency hides behind the next column's chain
    static_for<0, 16>([&](auto jc) {
      constexpr int jj = decltype(jc)::value;
      constexpr int j = 16 * b + jj;
      // entries for the chain and the next two rows (column j−1's deferred updates never touch them)
      double a1 = 0.0, a2 = 0.0, ap = 0.0;
      if constexpr (jj < 15) {
        a1 = readlane_f64(a[jj], j + 1);
        ap = readlane_f64(a[jj + 1], j + 1);
      }
      if constexpr (jj < 14) a2 = readlane_f64(a[jj], j + 2);
      if (!(dj > 0.0)) {
        if (bad == 0) bad = j + 1;
        dj = 1.0;                                      // continue without NaNs; flagged
      }
      const double y0 = __builtin_amdgcn_rsq(dj);
      const double hd = 0.5 * dj;
      const double y1 = fma(y0, fma(-hd * y0, y0, 0.5), y0);
      const double inv = fma(y1, fma(-hd * y1, y1, 0.5), y1);
      double s1 = 0.0, s2 = 0.0;
      if constexpr (jj < 15) {
        s1 = a1 * inv;                                 // L[j+1][j]
        dj = fma(-s1, s1, ap);                         // next pivot
      }
      if constexpr (jj < 14) s2 = a2 * inv;            // L[j+2][j]
      const double lrj = a[jj] * inv;                  // row j: dj·inv = √dj
      a[jj] = lrj;
      if constexpr (jj < 15) a[jj + 1] = fma(-lrj, s1, a[jj + 1]);
      if constexpr (jj < 14) a[jj + 2] = fma(-lrj, s2, a[jj + 2]);
      // publish the column, then release it to the later waves (before any new LDS load is queued)
      if (r == j) dinv[j] = inv;
      Lb[(b * 64 + r) * kLbP + jj] = lrj;
      if constexpr (b < 3) {
        if (r == 0) __hip_atomic_store(&prog[b], jj + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      // column j−1's remaining updates (q ≥ jj+2; loaded one column ago, their latency behind the chain)
      if constexpr (jj >= 1) {
#pragma unroll
        for (int q = jj + 2; q < 16; ++q) a[q] = fma(-pl, pv[q], a[q]);
      }
      if constexpr (jj < 13) {
        double* cb = aux + kNB * (jj & 1);
        cb[r] = lrj;
#pragma unroll
        for (int q = jj + 3; q < 16; ++q) pv[q] = cb[16 * b + q];
        pl = lrj;
      }
      OMB_CHOL_COL(w, j, r == 0);
      __builtin_amdgcn_sched_barrier(0);
    });
    OMB_CHOL_TRACE(3 + 2 * b, r == 0);
    if (r == 0 && bad) bad_lds[0] = bad;
    // ---- this sub-block's 16 columns of L into A: lane → (row 4i + (r >> 4), column r & 15)
    {
      const int q = r & 15;
      double lv[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) lv[i] = Lb[(b * 64 + 4 * i + (r >> 4)) * kLbP + q];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = 4 * i + (r >> 4);
        if (row < nb && 16 * b + q <= row) A[(c0 + row) * lda + c0 + 16 * b + q] = lv[i];
      }
    }
    // ---- W_bb = L_bb⁻¹, column c = r & 15 per lane
    const int c = r & 15, g = r >> 4;
    const double* Ld = Lb + (b * 64 + 16 * b) * kLbP;   // L_bb row m at Ld + m·kLbP
    double x[16];
    static_for<0, 16>([&](auto mc) {
      constexpr int m = decltype(mc)::value;
      // row m's offset passes through an empty asm that consumes x[m−2]: its reads issue one row
      // ahead of their use, not all 120 at once (which took the kernel to 256 VGPRs)
      int off = m * kLbP;
      if constexpr (m >= 2) asm volatile("" : "+v"(off) : "v"(x[m - 2]));
      double t0 = (m == c) ? 1.0 : 0.0, t1 = 0.0;
#pragma unroll
      for (int p = 0; p + 1 < m; p += 2) {
        const double2 l = *reinterpret_cast<const double2*>(Ld + off + p);
        t0 = fma(-l.x, x[p], t0);
        t1 = fma(-l.y, x[p + 1], t1);
      }
      if constexpr (m & 1) t0 = fma(-Ld[off + m - 1], x[m - 1], t0);
      x[m] = (t0 + t1) * dinv[16 * b + m];
    });
    // every lane's reads of L_bb precede the overwrite (LDS operations of a wave complete in order)
    if (r < 16) {
#pragma unroll
      for (int m = 0; m < 16; ++m) Lb[(b * 64 + 16 * b + m) * kLbP + c] = x[m];
    }
    // W_bb's fragments: rows jb = b, k-steps s = 4b + u: W[16b + c][16b + 4g + u]
#pragma unroll
    for (int u = 0; u < 4; ++u) wf_store(&Wf[(b * 16 + 4 * b + u) * 64 + r], Lb[(b * 64 + 16 * b + c) * kLbP + 4 * g + u]);
    // W_bb is in Lb: release it to the waves forming W's earlier column blocks (wdone = prog + 4)
    if (r == 0) __hip_atomic_store(&prog[4 + b], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    OMB_CHOL_TRACE(10 + b, r == 0);
  });
  chol64_inverse(w, r, Lb, prog + 4, Wf);
}

// ----------------------------------------------------------------------------- Cholesky, blocked diagonal block
// Round 4.  The 64×64 diagonal block is factored as 4 × 4 tiles of 16 (right-looking inside the block), with
// row ownership: wave w owns tile row w — the tiles (w, j), j ≤ w, of D in LDS (pitch kDP) — and runs
//   for b < w:  P_b  L_wb = D_wb · W_bbᵀ (W_bb = L_bb⁻¹), 4 MFMAs, formed transposed (L_wbᵀ = W_bb D_wbᵀ) so the
//                    accumulator is L_wb in the operand layout of the next products (lane (g, c): L_wb[c][4e + g]);
//              U_b  D_wj −= L_wb L_jbᵀ for b < j ≤ w, 4 MFMAs each (L_jb of wave j after its flag; for j = w both
//                   operands are the P_b accumulator);
//   F_w        the tile (w, w): its Cholesky factor and inverse W_ww in registers (chol16_factor);
// then, as chol64_inverse, W's column block w: W_iw = −W_ii Σ_{k=w}^{i−1} L_ik W_kw (i > w) on MFMA.
// The block's serial chain is F_0 → P_0 U_0 (wave 1) → F_1 → … → F_3 → the three products with W_33: four
// 16-column factors and three 8-MFMA hand-offs.  Round 3 ran one wave per 16-column strip of all 64 rows
// (≈ 470 cycles per column on the owner, ≈ 40k cycles for the block, profiles/r03_v38_chol_trace_pipelined_inverse.txt).
// The waves synchronise through LDS flags (wready: W_bb in Wl; lready: L_ib in D); no barrier inside.
// kCholDOuter (the diagonal workgroup of chol_update_kernel): D = A22_00 − L21_0 L21_0ᵀ, wave w forming its own tiles
// (16 MFMAs each, K = 64, the k index permuted so a lane reads 4 contiguous doubles per 16-column group), so wave
// 0 starts F_0 after one tile instead of after the whole 64×64 product.
// per-wave phase timestamps of chol64_blocked, and step-level timestamps of chol_update_kernel (workgroup 0,
// workgroup (1, 0)), for tools/ablate/ablate_chol (empty here)
#ifndef OMB_CHOL_BTRACE
#define OMB_CHOL_BTRACE(w, id, cond)
#endif
#ifndef OMB_CHOL_STRACE
#define OMB_CHOL_STRACE(step, id, cond)
#endif
constexpr int kDP = 66;                    // D row pitch in doubles
constexpr int kWlP = 16 * 18;              // one W_bb in Wl, column-major: Wl[b·kWlP + c·18 + m] = W_bb[m][c]
constexpr int kBlkFlags = 4 + 16 + 2;      // wready[4] | lready[4i + b] | bad | wait fault

// bounded (2^20 polls ≈ 30 ms): a wait that runs out marks fl[kBlkFlags − 1] (→ info = kCholSpinFault) and
// goes on, so a wrong flag protocol ends the kernel instead of hanging it
// epoch: the value a post writes (chol_persist_kernel posts step + 1, so its flags need no reset between steps)
__device__ __forceinline__ void lds_wait_flag(int* f, int* fault, int epoch = 1) {
  int polls = 0;
  while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < epoch) {
    if (++polls > (1 << 20)) {
      *fault = 1;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}
// lane 0 posts; the release orders the whole wave's earlier LDS stores before the flag
__device__ __forceinline__ void lds_post_flag(int* f, int lane, int epoch = 1) {
  if (lane == 0) __hip_atomic_store(f, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// orders one wave's LDS accesses across lanes for the compiler (LDS executes a wave's accesses in order)
__device__ __forceinline__ void wave_lds_order() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

// Cholesky of a 16×16 SPD tile held row-per-lane (lane → row r = lane & 15; the four 16-lane rows of the wave
// hold the same copy), with W = L⁻¹ by column-oriented forward substitution of L x = e_r sharing the broadcasts:
//   a[q] = D[r][q] (q ≤ r; entries above the diagonal start at 0 and are never broadcast) → L[r][q];
//   x = e_r → x[m] = W[m][r].
// Column j: inv_j = 1/√d_j (v_rsq + 2 Newton steps), L[r][j] = a[j]·inv_j; for k > j a[k] −= L[r][j]·L[k][j] and
// x[k] −= x[j]·L[k][j], L[k][j] being lane k's value (one v_mov_b64_dpp row_newbcast per k, shared by both; folding
// it into two inline-asm v_fmac_f64_dpp was slower: 3,784 against 3,188 cycles per factor,
// profiles/r04_f_mb_chol16.txt).
// The pivot chain runs ahead on wave-uniform values: d_{j+1} = a_{j+1}[j+1] − (a_{j+1}[j]·inv_j)² with both entries
// read (v_readlane) before inv_j is known — bitwise the value the update leaves in lane j+1 (the same fma).
// Returns 0 or the 1-based first column with a non-positive pivot (continued with 1.0: no NaNs; flagged).
__device__ __forceinline__ int chol16_factor(double (&a)[16], double (&x)[16]) {
  int bad = 0;
  double dj = readlane_f64(a[0], 0);
  static_for<0, 16>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    double a1 = 0.0, ap = 0.0;
    if constexpr (j < 15) {
      a1 = readlane_f64(a[j], j + 1);
      ap = readlane_f64(a[j + 1], j + 1);
    }
    if (!(dj > 0.0)) {
      if (bad == 0) bad = j + 1;
      dj = 1.0;
    }
    const double y0 = __builtin_amdgcn_rsq(dj);
#ifndef OMB_CHOL16_POLY2
    const double hd = 0.5 * dj;
    const double y1 = fma(y0, fma(-hd * y0, y0, 0.5), y0);
    const double inv = fma(y1, fma(-hd * y1, y1, 0.5), y1);
#else
    // tools (round 6, measured, not kept — DESIGN §11a): one second-order correction, y0 (1 − r/2 + 3r²/8) with
    // r = d·y0² − 1, 4 dependent operations instead of 6; as accurate (profiles/r06_p2_mb_rsq.txt), N = 3000 0.5% faster
    const double r = fma(dj * y0, y0, -1.0);
    const double inv = fma(y0 * r, fma(r, 0.375, -0.5), y0);
#endif
    if constexpr (j < 15) {
      const double s1 = a1 * inv;
      dj = fma(-s1, s1, ap);
    }
    const double l = a[j] * inv;
    a[j] = l;
    const double xj = x[j] * inv;
    x[j] = xj;
    const double nl = -l, nx = -xj;
    static_for<j + 1, 16>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      const double lk = __builtin_amdgcn_mov_dpp(l, 0x150 + k, 0xf, 0xf, true);   // v_mov_b64_dpp row_newbcast:k
      a[k] = fma(nl, lk, a[k]);
      x[k] = fma(nx, lk, x[k]);
    });
  });
  // the callers store a and x under a lane condition; without this the updates were sunk into that branch,
  // keeping every broadcast alive (256 VGPRs + 58 AGPRs)
#pragma unroll
  for (int q = 0; q < 16; ++q) asm volatile("" : "+v"(a[q]), "+v"(x[q]));
  return bad;
}

// 16 doubles of row `p` (k permuted: v[4q + u] = p[16q + u], p already offset by 4g), or zeros
__device__ __forceinline__ void load_row16(const double* __restrict__ p, bool ok, double (&v)[16]) {
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int u = 0; u < 4; ++u) v[4 * q + u] = ok ? p[16 * q + u] : 0.0;
}

// The diagonal block at rows / columns r0 .. r0+63 of A (nb ≤ 64 real rows; the rest identity), factored in place
// (lower triangle of rows < nb), with W = L⁻¹'s MFMA fragments to Wf (the layout of chol64_inverse).  kCholDOuter: A22_00
// minus the product of the panel rows A[r0 + ·][c0 .. c0+63].  Ds, Wl, fl: LDS (fl zeroed by the caller and a
// barrier passed).  The caller reads fl[20] (block-relative 1-based first bad column, 0 = none) after a barrier.
// MODE kCholDLoad (step 0 / chol_diag_blk_kernel): D = A_kk; kCholDOuter (chol_update_kernel): D = A22_00 − L21_0
// L21_0ᵀ from global; kCholDReady (chol_persist_kernel): each wave has already written its D tiles (w, j ≤ w) to Ds.
enum { kCholDLoad = 0, kCholDOuter = 1, kCholDReady = 2 };
// kCholDReady also leaves W's fragments in Wfl (LDS, the layout of Wf) for the walker's own panel tile.
template <int MODE>
__device__ __forceinline__ void chol64_blocked(double* __restrict__ A, int64_t lda, int64_t r0, int nb, int64_t c0,
                                               double* __restrict__ Wf, double* Ds, double* Wl, int* fl, int epoch = 1,
                                               double* Wfl = nullptr) {
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  OMB_CHOL_BTRACE(w, 0, lane == 0);
  // ---- D tiles (w, j), j ≤ w (accumulator layout: lane (g, c) → rows 4e + g, column c); tile j + 1's loads are
  // issued before tile j's product (one load latency per wave instead of one per tile)
  if constexpr (MODE != kCholDReady) {
    auto load_a22 = [&](int j, double (&av)[4]) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = 16 * w + 4 * e + g, col = 16 * j + c;
        av[e] = (row < nb && col <= row) ? A[(r0 + row) * lda + r0 + col] : (row == col ? 1.0 : 0.0);
      }
    };
    double xa[16], xb[16], av[4];
    if constexpr (MODE == kCholDOuter) {
      load_row16(A + (r0 + 16 * w + c) * lda + c0 + 4 * g, 16 * w + c < nb, xa);
      if (w > 0) {
        load_row16(A + (r0 + c) * lda + c0 + 4 * g, c < nb, xb);
      } else {
#pragma unroll
        for (int q = 0; q < 16; ++q) xb[q] = xa[q];
      }
    }
    load_a22(0, av);
    for (int j = 0; j <= w; ++j) {
      double nxb[16], nav[4];
      if (j < w) {
        if constexpr (MODE == kCholDOuter) {
          if (j + 1 < w) {
            load_row16(A + (r0 + 16 * (j + 1) + c) * lda + c0 + 4 * g, 16 * (j + 1) + c < nb, nxb);
          } else {
#pragma unroll
            for (int q = 0; q < 16; ++q) nxb[q] = xa[q];                  // tile (w, w): both operands the own rows
          }
        }
        load_a22(j + 1, nav);
      }
      d4 acc = d4{0.0, 0.0, 0.0, 0.0};
      if constexpr (MODE == kCholDOuter) {
#pragma unroll
        for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(xa[s], xb[s], acc, 0, 0, 0);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) Ds[(16 * w + 4 * e + g) * kDP + 16 * j + c] = av[e] - acc[e];
      if (j < w) {
#pragma unroll
        for (int e = 0; e < 4; ++e) av[e] = nav[e];
        if constexpr (MODE == kCholDOuter) {
#pragma unroll
          for (int q = 0; q < 16; ++q) xb[q] = nxb[q];
        }
      }
    }
  }
  OMB_CHOL_BTRACE(w, 1, lane == 0);
  // ---- P_b, U_b for b < w
  for (int b = 0; b < w; ++b) {
    double dop[4];                                                    // D_wb[c][4s + g], read before the wait
#pragma unroll
    for (int s = 0; s < 4; ++s) dop[s] = Ds[(16 * w + c) * kDP + 16 * b + 4 * s + g];
    lds_wait_flag(&fl[b], &fl[21], epoch);
    OMB_CHOL_BTRACE(w, 2 + 2 * b, lane == 0);
    const double* Wb = Wl + b * kWlP;
    d4 lt = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < 4; ++s)
      lt = __builtin_amdgcn_mfma_f64_16x16x4f64(Wb[(4 * s + g) * 18 + c], dop[s], lt, 0, 0, 0);   // W_bb[c][4s + g]
#pragma unroll
    for (int e = 0; e < 4; ++e) Ds[(16 * w + c) * kDP + 16 * b + 4 * e + g] = lt[e];     // L_wb[c][4e + g]
    lds_post_flag(&fl[4 + 4 * w + b], lane, epoch);
    // U_b: the own diagonal tile first (on the chain when b = w − 1), then the tiles (w, j), b < j < w
    for (int j = w; j > b; --j) {
      d4 u = d4{0.0, 0.0, 0.0, 0.0};
      if (j == w) {
#pragma unroll
        for (int s = 0; s < 4; ++s) u = __builtin_amdgcn_mfma_f64_16x16x4f64(lt[s], lt[s], u, 0, 0, 0);
      } else {
        lds_wait_flag(&fl[4 + 4 * j + b], &fl[21], epoch);
#pragma unroll
        for (int s = 0; s < 4; ++s)
          u = __builtin_amdgcn_mfma_f64_16x16x4f64(lt[s], Ds[(16 * j + c) * kDP + 16 * b + 4 * s + g], u, 0, 0, 0);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        double* p = Ds + (16 * w + 4 * e + g) * kDP + 16 * j + c;
        *p = *p - u[e];
      }
    }
    // the panel tile's L into A (after the flag: off the chain)
    if (16 * w + c < nb) {
#pragma unroll
      for (int e = 0; e < 4; ++e) A[(r0 + 16 * w + c) * lda + r0 + 16 * b + 4 * e + g] = lt[e];
    }
    OMB_CHOL_BTRACE(w, 3 + 2 * b, lane == 0);
  }
  // ---- F_w
  wave_lds_order();
  {
    // row c of the tile (entries above the diagonal are finite leftovers: never broadcast, never stored to A)
    double a[16], x[16];
    const double2* dr = reinterpret_cast<const double2*>(Ds + (16 * w + c) * kDP + 16 * w);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const double2 v = dr[q];
      a[2 * q] = v.x;
      a[2 * q + 1] = v.y;
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) x[q] = (q == c) ? 1.0 : 0.0;
    OMB_CHOL_BTRACE(w, 8, lane == 0);
    const int bad = chol16_factor(a, x);
    OMB_CHOL_BTRACE(w, 9, lane == 0);
    if (g == 0) {
      double2* drw = reinterpret_cast<double2*>(Ds + (16 * w + c) * kDP + 16 * w);
      double2* wc = reinterpret_cast<double2*>(Wl + w * kWlP + c * 18);                // W_ww[·][c]
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        drw[q] = double2{a[2 * q], a[2 * q + 1]};
        wc[q] = double2{x[2 * q], x[2 * q + 1]};
      }
      if (c == 0 && bad != 0 && fl[20] == 0) fl[20] = 16 * w + bad;
    }
    lds_post_flag(&fl[w], lane, epoch);
    OMB_CHOL_BTRACE(w, 10, lane == 0);
    if (g == 0 && 16 * w + c < nb) {
#pragma unroll
      for (int q = 0; q < 16; ++q)
        if (q <= c) A[(r0 + 16 * w + c) * lda + r0 + 16 * w + q] = a[q];
    }
  }
  // W_ww's fragments: block (w, w), k-step 4w + u: W[16w + c][16w + 4g + u]
  wave_lds_order();
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const double v = Wl[w * kWlP + (4 * g + u) * 18 + c];
    wf_store(&Wf[(w * 16 + 4 * w + u) * 64 + 16 * g + c], v);
    if constexpr (MODE == kCholDReady) Wfl[(w * 16 + 4 * w + u) * 64 + 16 * g + c] = v;   // the walker's LDS copy
  }
  // ---- W's column block w: W_iw = −W_ii Σ_{k=w}^{i−1} L_ik W_kw, i = w+1 .. 3 (Wc[k] = W_kw, accumulator layout,
  // is the B operand of the next product: lane (g, c) holds W_kw[4s + g][c] in register s)
  d4 Wc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) Wc[i] = d4{0.0, 0.0, 0.0, 0.0};
  static_for<1, 4>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    if (i > w) {
      d4 T = d4{0.0, 0.0, 0.0, 0.0};
      static_for<0, i>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        if (k >= w) {
          lds_wait_flag(&fl[4 + 4 * i + k], &fl[21], epoch);                                      // L_ik final
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const double av = Ds[(16 * i + c) * kDP + 16 * k + 4 * s + g];              // L_ik[c][4s + g]
            const double bv = (k == w) ? Wl[w * kWlP + c * 18 + 4 * s + g] : Wc[k][s];   // W_kw[4s + g][c]
            T = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, T, 0, 0, 0);
          }
        }
      });
      lds_wait_flag(&fl[i], &fl[21], epoch);                                                      // W_ii in Wl
      d4 R = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s = 0; s < 4; ++s)
        R = __builtin_amdgcn_mfma_f64_16x16x4f64(Wl[i * kWlP + (4 * s + g) * 18 + c], T[s], R, 0, 0, 0);   // W_ii[c][4s + g]
      Wc[i] = -R;
      // W[16i + 4e + g][16w + c]: row block i, k-step 4w + (c & 3), lane 4e + g + 16 (c >> 2)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        wf_store(&Wf[(i * 16 + 4 * w + (c & 3)) * 64 + 4 * e + g + 16 * (c >> 2)], Wc[i][e]);
        if constexpr (MODE == kCholDReady) Wfl[(i * 16 + 4 * w + (c & 3)) * 64 + 4 * e + g + 16 * (c >> 2)] = Wc[i][e];
      }
      OMB_CHOL_BTRACE(w, 10 + i, lane == 0);
    }
  });
}

// Step 0's diagonal block (chol_diag_kernel's blocked form); zeroes info and the fused steps' flags.
__global__ __launch_bounds__(256) void chol_diag_blk_kernel(double* __restrict__ A, int64_t N, int64_t lda,
                                                            double* __restrict__ ws, int* __restrict__ info,
                                                            int* __restrict__ flags, int nflags) {
  for (int i = threadIdx.x; i < nflags; i += blockDim.x) flags[i] = 0;
  if (threadIdx.x == 0) *info = 0;
  __shared__ __attribute__((aligned(16))) double Ds[kNB * kDP];
  __shared__ __attribute__((aligned(16))) double Wl[4 * kWlP];
  __shared__ int fl[kBlkFlags];
  if (threadIdx.x < kBlkFlags) fl[threadIdx.x] = 0;
  __syncthreads();
  chol64_blocked<kCholDLoad>(A, lda, 0, (int)(N < kNB ? N : kNB), 0, ws, Ds, Wl, fl);
  __syncthreads();
  if (threadIdx.x == 0 && (fl[20] || fl[21])) atomicCAS(info, 0, fl[21] ? kCholSpinFault : fl[20]);
}

__global__ __launch_bounds__(256) void chol_diag_kernel(double* __restrict__ A, int64_t N, int64_t lda,
                                                         double* __restrict__ ws, int* __restrict__ info,
                                                         int* __restrict__ flags, int nflags) {
  for (int i = threadIdx.x; i < nflags; i += blockDim.x) flags[i] = 0;
  if (threadIdx.x == 0) *info = 0;
  __shared__ __attribute__((aligned(16))) double Lb[kLbDoubles];
  __shared__ double aux[kCholAux];
  __shared__ int prog[8];   // column progress per sub-block | W_bb published
  __shared__ int bad_lds[1];
  const int nb = (int)(N < kNB ? N : kNB);
  const int r = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  OMB_CHOL_TRACE(0, threadIdx.x == 0);
  if (threadIdx.x == 0) bad_lds[0] = 0;
  if (threadIdx.x < 8) prog[threadIdx.x] = 0;
  double a[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int c = 16 * w + q;
    double v = (c == r) ? 1.0 : 0.0;
    if (r < nb && c <= r) v = A[(int64_t)r * lda + c];
    a[q] = v;
  }
  __syncthreads();
  OMB_CHOL_TRACE(1, threadIdx.x == 0);
  chol64_factor(a, w, r, nb, Lb, aux, prog, bad_lds, A, lda, 0, ws);   // with W = L⁻¹ (chol64_inverse)
  __syncthreads();
  OMB_CHOL_TRACE(15, threadIdx.x == 0);
  if (threadIdx.x == 0 && bad_lds[0]) atomicCAS(info, 0, bad_lds[0]);
}

// Panel of step `step`: rows c0+64 .. N−1, L21 = A21 · Wᵀ (W = L_kk⁻¹ from the fragments of chol64_factor /
// chol64_inverse).
// Workgroup = 16 rows, 2 waves: wave 0 the output column blocks 0 and 3, wave 1 blocks 1 and 2 (20
// MFMAs each).  The k index is permuted as m(s, g) = 16(s >> 2) + 4g + (s & 3) so a lane's A operands
// are 4 contiguous doubles per 16-column group; the barrier separates both waves' reads of the rows
// from the in-place writes.
// The persistent launch's sync words for t steps after k0 per-step launches (chol_persist_kernel's layout: wflag[t] |
// pflag[t·t] | cnt[t·t] | ticket | abort), word x.
__device__ __forceinline__ int chol_persist_init_word(int x, int t, int k0) {
  if (k0 > 0 && x >= t && x < t + t * t) {
    const int i = (x - t) / t, k = (x - t) % t;
    return (k == k0 && i > k0) ? 4 : 0;
  }
  if (k0 > 0 && x >= t + t * t && x < t + 2 * t * t) {
    const int i = (x - t - t * t) / t, j = (x - t - t * t) % t;
    return (j > k0 && j <= i) ? k0 : 0;
  }
  return 0;
}

// pinit (round 5, the hybrid schedule): step 0's panel launch also writes the later persistent launch's sync words
// (chol_persist_init_kernel's job; the per-step launches never touch them), one launch fewer on the chain.
template <bool VEC>
__global__ __launch_bounds__(128) void chol_panel_kernel(double* __restrict__ A, int64_t N, int64_t lda, int step,
                                                         const double* __restrict__ Wf, const int* __restrict__ info,
                                                         int* __restrict__ pinit = nullptr, int pt = 0, int pk0 = 0) {
  if (pinit) {
    const int pn = pt + 2 * pt * pt + 2;
    for (int x = blockIdx.x * blockDim.x + threadIdx.x; x < pn; x += gridDim.x * blockDim.x)
      pinit[x] = chol_persist_init_word(x, pt, pk0);
  }
  if (*info != 0) return;
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t c0 = (int64_t)step * kNB;
  const int64_t r0 = c0 + kNB + (int64_t)blockIdx.x * 16;
  const int64_t row = r0 + c;
  const int ngroups = wave == 0 ? 4 : 3;            // 16-column groups of A21 this wave reads
  double x[16];                                       // x[4sg + u] = A21[row][16sg + 4g + u]
  const double* rp = A + row * lda + c0 + 4 * g;
#pragma unroll
  for (int sg = 0; sg < 4; ++sg) {
    if (sg < ngroups && row < N) {
      if constexpr (VEC) {
        const double2 v0 = reinterpret_cast<const double2*>(rp + 16 * sg)[0];
        const double2 v1 = reinterpret_cast<const double2*>(rp + 16 * sg)[1];
        x[4 * sg] = v0.x;
        x[4 * sg + 1] = v0.y;
        x[4 * sg + 2] = v1.x;
        x[4 * sg + 3] = v1.y;
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) x[4 * sg + u] = rp[16 * sg + u];
      }
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) x[4 * sg + u] = 0.0;
    }
  }
  d4 acc[2];
  int jbs[2] = {wave == 0 ? 0 : 1, wave == 0 ? 3 : 2};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    acc[h] = d4{0.0, 0.0, 0.0, 0.0};
    const int jb = jbs[h];
    const double* wf = Wf + (int64_t)jb * 16 * 64 + lane;
#pragma unroll
    for (int s = 0; s < 16; ++s)
      if (s < 4 * (jb + 1)) acc[h] = __builtin_amdgcn_mfma_f64_16x16x4f64(x[s], wf[s * 64], acc[h], 0, 0, 0);
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t orow = r0 + 4 * e + g;
      if (orow < N) A[orow * lda + c0 + 16 * jbs[h] + c] = acc[h][e];
    }
}

// Trailing update of step `step` (A22 −= L21 L21ᵀ, lower 64×64 tiles, gemm_kernel's MFMA tiling with
// K = 64) fused with the factorisation and inversion of the next diagonal block by the workgroup that
// owns it.
// One workgroup per lower tile of A22 (t tiles a side, t(t+1)/2 workgroups): workgroup 0 is the diagonal
// tile (0, 0), workgroups 1 .. t−1 the tiles (m, 0) below it — the next step's panel rows — and the rest
// the tiles (m, n), 1 ≤ n ≤ m, in row order.
// FUSE (round 3): the workgroups of the tiles (m, 0) keep their updated tile in LDS, wait for the
// diagonal workgroup to publish W_{k+1} = L_{k+1,k+1}⁻¹ (flags[step], set after the fragments are in the
// workspace) and form the next step's panel rows L21 = A21 · Wᵀ themselves, so a step is one launch:
// the panel's own launch (≈ 5 µs plus a launch gap per step at N = 3000) leaves the chain.  Workgroup 0
// is dispatched first (in-order dispatch); the wait is bounded all the same (spin_limit polls, then
// info = kCholSpinFault and the workgroup finishes), so a waiting workgroup can never hang the grid.
// The fused step's hand-off of W_{k+1} (chol_update_kernel<FUSE>): the diagonal workgroup stores the fragments
// with agent-scope relaxed atomics (wf_store: sc1, coherent across the XCDs' L2s), waits for all of them (vmcnt 0)
// and sets the flag; a waiting workgroup polls the flag (relaxed), passes a barrier and reads the fragments with
// wf_load.  The compiler fences (signal fences) keep the fragment accesses on their side of the flag; the
// hardware order is the vmcnt wait (a store counts as done once it is acknowledged at the coherent level).
// acq_rel = 1 (tools/ablate/ablate_chol): the flag store a release and one acquire fence after the poll, at
// agent scope — the HIP memory model's own guarantee; its cost is measured in DESIGN §4b.
__device__ __forceinline__ void chol_publish_w(int* flag, int tid, int acq_rel) {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (tid == 0) {
    if (acq_rel)
      __hip_atomic_store(flag, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    else
      __hip_atomic_store(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
__device__ __forceinline__ void chol_wait_w(const int* flag, int tid, int spin_limit, int* info, int acq_rel) {
  if (tid == 0) {
    int polls = 0;
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
      if (++polls > spin_limit) {
        atomicCAS(info, 0, kCholSpinFault);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (acq_rel) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

__device__ __forceinline__ void chol_tile_of(int b, int t, int& mt, int& nt) {
  if (b < t) {
    mt = b;
    nt = 0;
    return;
  }
  const int q = b - t;                                       // tiles (m', n'), 0 ≤ n' ≤ m' ≤ t − 2
  int mp = (int)((sqrt(8.0 * q + 1.0) - 1.0) * 0.5);
  while ((mp + 1) * (mp + 2) / 2 <= q) ++mp;
  while (mp * (mp + 1) / 2 > q) --mp;
  mt = mp + 1;
  nt = q - mp * (mp + 1) / 2 + 1;
}

// BLK: the diagonal workgroup runs chol64_blocked (round 4, the default) instead of round 3's strip factor
template <bool FUSE, bool BLK>
__global__ __launch_bounds__(256, 3) void chol_update_kernel(double* __restrict__ A, int64_t N, int64_t lda, int step,
                                                          int t, double* __restrict__ ws, int* __restrict__ info,
                                                          int* __restrict__ flags, int spin_limit, int acq_rel,
                                                          int delay = 0) {
  OMB_CHOL_STRACE(step, blockIdx.x == 0 ? 0 : 3, threadIdx.x == 0 && blockIdx.x <= 1);
  // delay (tools/ablate knob): every workgroup but the diagonal one sleeps delay × 32·64 cycles (≈ 0.85 µs) first,
  // so the diagonal workgroup's loads meet an idle memory system
  for (int i = 0; i < delay && blockIdx.x != 0; ++i) __builtin_amdgcn_s_sleep(32);
  if (__hip_atomic_load(info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
  int mt, nt;
  chol_tile_of((int)blockIdx.x, t, mt, nt);
  const int64_t c0 = (int64_t)step * kNB;
  const int64_t r0 = c0 + kNB;                              // first row / column of A22
  const int64_t M = N - r0;
  const int64_t m0 = (int64_t)mt * kGT, n0 = (int64_t)nt * kGT;
  // one array: the GEMM's As and Bs, then (the diagonal workgroup) the 64 × 65 staging tile D, then
  // the factorisation's Lb
  static_assert(2 * 2 * kGK * kGP <= kLbDoubles && kNB * (kNB + 1) <= kLbDoubles, "LDS carve-up");
  __shared__ __attribute__((aligned(16))) double smem[kLbDoubles];
  __shared__ double aux[kCholAux];
  __shared__ int prog[8];   // column progress per sub-block | W_bb published
  auto& As = *reinterpret_cast<double (*)[2][kGK][kGP]>(smem);                      // As[buf][k][m] = L21(m0 + m, k0 + k)
  auto& Bs = *reinterpret_cast<double (*)[2][kGK][kGP]>(smem + 2 * kGK * kGP);      // Bs[buf][k][n] = L21(n0 + n, k0 + k)
  __shared__ int bad_lds[1];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const double* L21 = A + r0 * lda + c0;
  if constexpr (BLK) {
    // round 4: the next diagonal block factored by tiles of 16 (chol64_blocked), its product with the panel
    // formed by the waves that own the tiles
    if (mt == 0 && nt == 0) {
      __shared__ __attribute__((aligned(16))) double Wl[4 * kWlP];
      __shared__ int fl[kBlkFlags];
      if (tid < kBlkFlags) fl[tid] = 0;
      __syncthreads();
      chol64_blocked<kCholDOuter>(A, lda, r0, (int)(M < kNB ? M : kNB), c0, ws, smem, Wl, fl);
      __syncthreads();
      if (tid == 0 && (fl[20] || fl[21])) atomicCAS(info, 0, fl[21] ? kCholSpinFault : (int)(r0 + fl[20]));
      OMB_CHOL_STRACE(step, 1, tid == 0);
      if constexpr (FUSE) chol_publish_w(flags + step, tid, acq_rel);
      OMB_CHOL_STRACE(step, 2, tid == 0);
      return;
    }
  }
  // the next diagonal block (A22's first tile) belongs to workgroup (0, 0)
  if (!(mt == 0 && nt == 0)) {
    double ra[4], rb[4];
    auto fetch = [&](int k0) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int idx = tid + 256 * e;
        const int am = idx >> 4, ak = idx & 15;
        ra[e] = (m0 + am < M) ? L21[(m0 + am) * lda + k0 + ak] : 0.0;
        rb[e] = (n0 + am < M) ? L21[(n0 + am) * lda + k0 + ak] : 0.0;
      }
    };
    auto stash = [&](int buf) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int idx = tid + 256 * e;
        As[buf][idx & 15][idx >> 4] = ra[e];
        Bs[buf][idx & 15][idx >> 4] = rb[e];
      }
    };
    d4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};
    fetch(0);
    stash(0);
    __syncthreads();
    int buf = 0;
#pragma unroll
    for (int k0 = 0; k0 < kNB; k0 += kGK) {
      const bool more = k0 + kGK < kNB;
      if (more) fetch(k0 + kGK);
#pragma unroll
      for (int ks = 0; ks < kGK / 4; ++ks) {
        const int kk = 4 * ks + (lane >> 4);
        const double a0 = As[buf][kk][32 * wm + (lane & 15)];
        const double a1 = As[buf][kk][32 * wm + 16 + (lane & 15)];
        const double b0 = Bs[buf][kk][32 * wn + (lane & 15)];
        const double b1 = Bs[buf][kk][32 * wn + 16 + (lane & 15)];
        acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
      }
      if (more) stash(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
    // C/D map of v_mfma_f64_16x16x4f64: col = lane & 15, row = (lane >> 4) + 4·i
    if (!FUSE || nt != 0) {
#pragma unroll
      for (int rb2 = 0; rb2 < 2; ++rb2)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int lr = 32 * wm + 16 * rb2 + (lane >> 4) + 4 * i;
            const int lc = 32 * wn + 16 * cb + (lane & 15);
            const int64_t row = m0 + lr, col_g = n0 + lc;
            if (row < M && col_g < M && col_g <= row) {
              double* p = A + (r0 + row) * lda + r0 + col_g;
              *p = *p - acc[rb2][cb][i];
            }
          }
      return;
    }
    // FUSE, tile (m, 0): the updated tile (the next step's A21 rows) into LDS, D[lr·kPD + lc]; the
    // GEMM loop ended on a barrier, so As/Bs are free
    constexpr int kPD = kNB + 2;                              // 528-B rows: 16 lanes' b128 reads of 16 rows conflict-free
    static_assert(kNB * kPD <= kLbDoubles, "LDS carve-up");
    double* Dp = smem;
#pragma unroll
    for (int rb2 = 0; rb2 < 2; ++rb2)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int lr = 32 * wm + 16 * rb2 + (lane >> 4) + 4 * i;
          const int lc = 32 * wn + 16 * cb + (lane & 15);
          const int64_t row = m0 + lr;
          Dp[lr * kPD + lc] = (row < M) ? A[(r0 + row) * lda + r0 + lc] - acc[rb2][cb][i] : 0.0;
        }
    __syncthreads();
    // W_{k+1}'s fragments: wait for the diagonal workgroup's flag (bounded); relaxed polls and coherent
    // fragment loads (wf_load), no cache-wide invalidate
    OMB_CHOL_STRACE(step, 4, tid == 0 && mt == 1);
    chol_wait_w(flags + step, tid, spin_limit, info, acq_rel);
    OMB_CHOL_STRACE(step, 5, tid == 0 && mt == 1);
    // the next step's panel rows, as chol_panel_kernel: wave w → rows 16w + (lane & 15) of the tile,
    // all four output column blocks
    {
      const int c = lane & 15, g = lane >> 4;
      double x[16];                                           // x[4sg + u] = D[16w + c][16sg + 4g + u]
      const double* dr = Dp + (16 * wave + c) * kPD + 4 * g;
#pragma unroll
      for (int sg = 0; sg < 4; ++sg) {
        const double2 v0 = reinterpret_cast<const double2*>(dr + 16 * sg)[0];
        const double2 v1 = reinterpret_cast<const double2*>(dr + 16 * sg)[1];
        x[4 * sg] = v0.x;
        x[4 * sg + 1] = v0.y;
        x[4 * sg + 2] = v1.x;
        x[4 * sg + 3] = v1.y;
      }
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        const double* wf = ws + jb * 16 * 64 + lane;
        d4 pa = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s2 = 0; s2 < 16; ++s2)
          if (s2 < 4 * (jb + 1)) pa = __builtin_amdgcn_mfma_f64_16x16x4f64(x[s2], wf_load(wf + s2 * 64), pa, 0, 0, 0);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int64_t orow = m0 + 16 * wave + 4 * e + g;
          if (orow < M) A[(r0 + orow) * lda + r0 + 16 * jb + c] = pa[e];
        }
      }
    }
    OMB_CHOL_STRACE(step, 6, tid == 0 && mt == 1);
    return;
  }
  // Diagonal workgroup: the tile's 64 L21 rows and its A22 values are loaded at once (one load latency
  // instead of one per 16-column slab of the pipeline above), the product runs from one LDS copy
  // (A and B are the same rows), and D = A22 − L21 L21ᵀ is formed in place for the factorisation.
  double* D = smem;                                          // 64 × 65: first T[k·65 + m] = L21(m, k), then D
  {
    double lv[16], av[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int idx = tid + 256 * e, m = idx >> 6, k = idx & 63;
      lv[e] = (m < M) ? L21[m * lda + k] : 0.0;
      av[e] = (m < M && k <= m) ? A[(r0 + m) * lda + r0 + k] : 0.0;
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int idx = tid + 256 * e;
      D[(idx & 63) * 65 + (idx >> 6)] = lv[e];
    }
    __syncthreads();
    d4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};
    if (wm >= wn) {                                          // the upper-right quadrant is not needed
#pragma unroll
      for (int ks = 0; ks < kNB / 4; ++ks) {
        const int kk = 4 * ks + (lane >> 4);
        const double a0 = D[kk * 65 + 32 * wm + (lane & 15)];
        const double a1 = D[kk * 65 + 32 * wm + 16 + (lane & 15)];
        const double b0 = D[kk * 65 + 32 * wn + (lane & 15)];
        const double b1 = D[kk * 65 + 32 * wn + 16 + (lane & 15)];
        acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
      }
    }
    __syncthreads();                                         // T consumed
    if (wm >= wn) {
#pragma unroll
      for (int rb2 = 0; rb2 < 2; ++rb2)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            D[(32 * wm + 16 * rb2 + (lane >> 4) + 4 * i) * 65 + 32 * wn + 16 * cb + (lane & 15)] = acc[rb2][cb][i];
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int idx = tid + 256 * e, m = idx >> 6, k = idx & 63;
      if (k <= m) D[m * 65 + k] = av[e] - D[m * 65 + k];
    }
  }
  __syncthreads();
  const int nb = (int)(M < kNB ? M : kNB);
  const int r = lane, w = wave;
  double a[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int c = 16 * w + q;
    a[q] = (r < nb && c <= r) ? D[r * 65 + c] : (c == r ? 1.0 : 0.0);
  }
  if (tid == 0) bad_lds[0] = 0;
  if (tid < 8) prog[tid] = 0;
  __syncthreads();                                           // D consumed: smem becomes Lb
  chol64_factor(a, w, r, nb, smem, aux, prog, bad_lds, A, lda, r0, ws);   // with W = L⁻¹ (chol64_inverse)
  __syncthreads();
  if (tid == 0 && bad_lds[0]) atomicCAS(info, 0, (int)(r0 + bad_lds[0]));
  if constexpr (FUSE) chol_publish_w(flags + step, tid, acq_rel);
}

// ----------------------------------------------------------------------------- Cholesky, one persistent launch
// Round 4.  The per-step launches above pay a kernel boundary on the step's serial chain (≈ 5.7 µs of the ≈ 29-µs
// step at N = 3000: the end of the update launch to the next diagonal workgroup's start, profiles/r04_h_ablate_chol.txt)
// and the diagonal workgroup's first loads compete with the whole grid's.  Here the factorisation is ONE launch of one
// workgroup per CU:
//   * workgroup 0 walks the diagonal: at step k it forms D_kk = A_kk − L_{k,k−1} L_{k,k−1}ᵀ from the panel tile it
//     made itself one step earlier (kept in LDS), factors it (chol64_blocked<kCholDReady>: L_kk, W_k = L_kk⁻¹ fragments),
//     publishes W_k, then forms the next panel tile L_{k+1,k} = A_{k+1,k} W_kᵀ into LDS (and A) — the chain of a step
//     is the 64-column factor plus one 64×64×64 product, no launch and no hand-off to another workgroup;
//   * the other workgroups draw tasks from one ticket counter, in an order in which every task depends only on
//     tasks drawn before it (so the grid needs no co-residency and cannot deadlock):
//       step k:  P(i, k), i ≥ k + 2   L_ik = A_ik W_kᵀ                      (W_k flag, A_ik updated through step k−1)
//                U(i, j, k), k+1 ≤ j ≤ i, (i, j) ≠ (k+1, k+1), by columns j  A_ij −= L_ik L_jkᵀ  (the two panel flags,
//                                                                         A_ij updated through step k−1)
//     U(k+1, k+1, k) is the diagonal workgroup's own D product.
// Cross-workgroup data (panel tiles, A tiles between updates, W fragments) is written with sc1 (write-through) stores
// after which every storing wave waits vmcnt(0), the workgroup passes a barrier and one lane stores the flag or tile
// counter (relaxed, agent scope); readers poll relaxed, pass a barrier and read those bytes with sc1 loads only
// (MI355X_MICROARCH.md § inter-workgroup visibility, the sc1 valid form; one workgroup per CU as measured there).  Tile counters cnt(i, j) = number of updates applied: each update waits for
// cnt = k, so the updates of one tile, possibly on different XCDs, never overlap.  Every wait is bounded (spin_limit
// polls), after which an abort word stops all waits and info = kCholSpinFault.
// one workgroup per CU: the launch bounds (≈ 228 VGPRs + 32 AGPRs) and > 80 KB of static LDS (D, the panel tile,
// W_bb and the walker's W fragments).  Two per CU (225 VGPRs, 77 KB) was slower — N = 3000 1.64 against 1.11 ms: a
// worker sharing the diagonal workgroup's CU stretches its factor and panel (gpurun_out/r04_r).
constexpr int kPersistWgPerCu = 1;

// progress words for tools/ablate/chol_persist_check (host-mapped memory; empty here)
#ifndef OMB_PDBG
#define OMB_PDBG(word, value)
#endif
// timestamps (s_memrealtime) of the diagonal walk's phases and of every worker task (tools/ablate; empty here)
#ifndef OMB_PTIME
#define OMB_PTIME(slot)
#endif

// sc1 loads through a buffer descriptor over A (loads past num_records return 0: rows ≥ N read as zeros)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t chol_rsrc(const double* base, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(base), (short)0,
                                           (int)(bytes < 0x7fffffff ? bytes : 0x7fffffff), 0x00020000);
}
typedef int i4v __attribute__((ext_vector_type(4)));
typedef double d2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ d2v ld2_sc1(__amdgpu_buffer_rsrc_t r, int64_t elem) {
  return __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(elem * 8), 0, 16));
}
// v[4q + u] = A[row][c0 + 16q + u] (the k permutation of load_row16; elem = row·lda + c0, c0 ≡ 4g)
__device__ __forceinline__ void load_row16_sc1(__amdgpu_buffer_rsrc_t r, int64_t elem, double (&v)[16]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const d2v lo = ld2_sc1(r, elem + 16 * q), hi = ld2_sc1(r, elem + 16 * q + 2);
    v[4 * q] = lo.x;
    v[4 * q + 1] = lo.y;
    v[4 * q + 2] = hi.x;
    v[4 * q + 3] = hi.y;
  }
}
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct CholSync {
  int* wflag;   // [t]      W_k published
  int* pflag;   // [t·t]    panel tile (i, k) published: 4 (per-wave adds for the walker's tiles)
  int* cnt;     // [t·t]    updates applied to tile (i, j)
  int* ticket;  // task counter of the worker workgroups
  int* abort;   // set by the first wait that runs out
  const int* tab;   // the workers' tasks in order, (code, steps) pairs (chol_task_table), or null for the
                    // step-major arithmetic order
};

// Wave 0 waits (every lane of it, on wave-uniform values) until *p ≥ v: relaxed polls; false after an abort or
// spin_limit polls (then abort = the word's offset in the sync block + 1, for tools/ablate, and info =
// kCholSpinFault).  The waits, flags and the ticket are whole-wave operations on purpose: with them under
// `threadIdx.x == 0` the compiler merged the flag store, the loop back edge and the next ticket into one divergent
// region and let wave 0's other lanes run ahead into the next task's barrier with the old ticket (the launch hung
// at N = 130, gpurun_out/r04_o; the ISA showed the barrier inside a loop entered without the ticket).
// AR (chol_mode bit 4, tests): an agent-scope acquire fence after the poll — the HIP memory model's form of the
// hand-off, against which the default relaxed form is checked bitwise (tests/test_gpu_turbo.py stress test).
template <bool AR = false>
__device__ __forceinline__ bool chol_poll_ge(const int* p, int v, const CholSync& s, int spin_limit, int* info) {
  int polls = 0;
  while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < v) {
    const int ab = (polls & 63) == 0
                       ? __builtin_amdgcn_readfirstlane(__hip_atomic_load(s.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                       : 0;
    if (ab != 0 || ++polls > spin_limit) {
      atomicCAS(s.abort, 0, (int)(p - s.wflag) + 1);
      atomicCAS(info, 0, kCholSpinFault);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  if constexpr (AR) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return true;
}

// Wave 0 waits until the panel flags of rows i and j are ≥ 4 for every step of [k, k + B) (B ≤ 32): lane 2b + r
// polls row r's flag of step k + b, one round trip per poll for the whole set (a batch's flags are mostly set long
// before its task is drawn); the same bound, abort word and AR fence as chol_poll_ge.
template <bool AR = false>
__device__ __forceinline__ bool chol_poll_panels(const int* pflag, int t, int i, int j, int k, int B, const CholSync& s,
                                                 int spin_limit, int* info) {
  const int lane = threadIdx.x & 63;
  const bool mine = lane < 2 * B;
  const int* p = pflag + ((lane & 1) ? j : i) * t + k + (lane >> 1);
  int polls = 0;
  for (;;) {
    const int v = mine ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 4;
    if (__builtin_amdgcn_ballot_w64(v < 4) == 0) break;
    const int ab = (polls & 63) == 0
                       ? __builtin_amdgcn_readfirstlane(__hip_atomic_load(s.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                       : 0;
    if (ab != 0 || ++polls > spin_limit) {
      atomicCAS(s.abort, 0, (int)(pflag + i * t + k - s.wflag) + 1);
      atomicCAS(info, 0, kCholSpinFault);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  if constexpr (AR) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return true;
}

// every storing wave drains its sc1 stores, the workgroup meets, wave 0 raises the flag (all its lanes store the
// same value to the same word: one uniform store).  AR: the flag store is an agent-scope release.
template <bool AR = false>
__device__ __forceinline__ void chol_signal(int* flag, int value) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0) {
    if constexpr (AR)
      __hip_atomic_store(flag, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    else
      __hip_atomic_store(flag, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Panel tile L_ik = A_ik W_kᵀ (chol_panel_kernel's product, 4 waves × 16 rows): W from the fragments Wk (global,
// sc1; for the diagonal workgroup, Lp set, its LDS copy), the result to A (sc1) and, for the diagonal workgroup,
// into Lp (LDS, pitch kDP).
__device__ __forceinline__ void chol_persist_panel(__amdgpu_buffer_rsrc_t ra, double* __restrict__ A, int64_t N,
                                                   int64_t lda, int i, int k, const double* __restrict__ Wk, double* Lp) {
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t row = (int64_t)i * kNB + 16 * w + c;
  double x[16];
  load_row16_sc1(ra, row * lda + (int64_t)k * kNB + 4 * g, x);
  if (row >= N) {
#pragma unroll
    for (int s = 0; s < 16; ++s) x[s] = 0.0;
  }
#pragma unroll
  for (int jb = 0; jb < 4; ++jb) {
    const double* wf = Wk + jb * 16 * 64 + lane;
    d4 pa = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < 16; ++s)
      if (s < 4 * (jb + 1))
        pa = __builtin_amdgcn_mfma_f64_16x16x4f64(x[s], Lp ? wf[s * 64] : ld_sc1(wf + s * 64), pa, 0, 0, 0);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t orow = (int64_t)i * kNB + 16 * w + 4 * e + g;
      if (Lp)
        Lp[(16 * w + 4 * e + g) * kDP + 16 * jb + c] = pa[e];   // the walker: waves 2 and 3 store it (below)
      else if (orow < N)
        st_sc1(A + orow * lda + (int64_t)k * kNB + 16 * jb + c, pa[e]);
    }
  }
}

// U(i, j, k): A_ij −= L_ik L_jkᵀ, wave (wm, wn) the 32 × 32 quadrant (the upper-right one skipped on a diagonal tile,
// whose strict upper triangle is never written)
__device__ __forceinline__ void chol_persist_update(__amdgpu_buffer_rsrc_t ra, double* __restrict__ A, int64_t N,
                                                    int64_t lda, int i, int j, int k) {
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  if (i == j && wm < wn) return;
  const int64_t ri = (int64_t)i * kNB + 32 * wm, rj = (int64_t)j * kNB + 32 * wn, ck = (int64_t)k * kNB + 4 * g;
  double av[2][2][4];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t row = ri + 16 * rb + 4 * e + g, col = rj + 16 * cb + c;
        av[rb][cb][e] = (row < N && col < N) ? ld_sc1(A + row * lda + col) : 0.0;
      }
  double a0[16], a1[16], b0[16], b1[16];
  load_row16_sc1(ra, (ri + c) * lda + ck, a0);
  load_row16_sc1(ra, (ri + 16 + c) * lda + ck, a1);
  load_row16_sc1(ra, (rj + c) * lda + ck, b0);
  load_row16_sc1(ra, (rj + 16 + c) * lda + ck, b1);
  d4 acc[2][2];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) acc[rb][cb] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0[s], b0[s], acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0[s], b1[s], acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1[s], b0[s], acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1[s], b1[s], acc[1][1], 0, 0, 0);
  }
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t row = ri + 16 * rb + 4 * e + g, col = rj + 16 * cb + c;
        if (row < N && col < N && (i != j || col <= row)) st_sc1(A + row * lda + col, av[rb][cb][e] - acc[rb][cb][e]);
      }
}

// U(i, j, k .. k+B−1) (round 6): the updates of B consecutive steps to one tile in one task, A_ij loaded once,
// A_ij −= L_is L_jsᵀ for s = k, k+1, … in order and stored once — every step's product summed from zero and
// subtracted as U(i, j, s) does, so the tile is bitwise what B single tasks leave.  The next step's panel rows load
// while the current step's MFMAs run (two register sets, the loop unrolled by two).  A far tile (its deadline more
// than the near window ahead) takes its updates in batches: one A-tile round trip, one hand-off and one poll chain
// per B steps instead of per step, and B·64 MFMAs per wave behind one set of load latencies.
__device__ __forceinline__ void chol_persist_update_batch(__amdgpu_buffer_rsrc_t ra, double* __restrict__ A, int64_t N,
                                                          int64_t lda, int i, int j, int k, int B) {
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  if (i == j && wm < wn) return;
  const int64_t ri = (int64_t)i * kNB + 32 * wm, rj = (int64_t)j * kNB + 32 * wn;
  double av[2][2][4];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t row = ri + 16 * rb + 4 * e + g, col = rj + 16 * cb + c;
        av[rb][cb][e] = (row < N && col < N) ? ld_sc1(A + row * lda + col) : 0.0;
      }
  struct Rows {
    double a0[16], a1[16], b0[16], b1[16];
  };
  auto load = [&](int s, Rows& p) {
    const int64_t ck = (int64_t)s * kNB + 4 * g;
    load_row16_sc1(ra, (ri + c) * lda + ck, p.a0);
    load_row16_sc1(ra, (ri + 16 + c) * lda + ck, p.a1);
    load_row16_sc1(ra, (rj + c) * lda + ck, p.b0);
    load_row16_sc1(ra, (rj + 16 + c) * lda + ck, p.b1);
  };
  auto apply = [&](const Rows& p) {
    d4 acc[2][2];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) acc[rb][cb] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(p.a0[s], p.b0[s], acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(p.a0[s], p.b1[s], acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(p.a1[s], p.b0[s], acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(p.a1[s], p.b1[s], acc[1][1], 0, 0, 0);
    }
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int e = 0; e < 4; ++e) av[rb][cb][e] = av[rb][cb][e] - acc[rb][cb][e];
  };
  Rows p0, p1;
  load(k, p0);
  for (int s = 0; s < B; s += 2) {
    if (s + 1 < B) load(k + s + 1, p1);
    apply(p0);
    if (s + 1 < B) {
      if (s + 2 < B) load(k + s + 2, p0);
      apply(p1);
    }
  }
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t row = ri + 16 * rb + 4 * e + g, col = rj + 16 * cb + c;
        if (row < N && col < N && (i != j || col <= row)) st_sc1(A + row * lda + col, av[rb][cb][e]);
      }
}

// Waves [w0, w0 + nw) copy a 64 × 64 tile of A (rows r0.., columns c0..; rows from `rows` on read row rows − 1 and
// columns from `cols` on column cols − 1 or, 16-B aligned, cols — inside the row's padding, lda being even — values
// the caller masks) into LDS at pitch kDP with direct-to-LDS loads (round 6, the walker's next tiles).  The
// padded image is 64 rows of 528 B: with 16-B aligned rows (aligned: lda even, A 16-B aligned) 33 wave instructions of
// 1 KiB — lane l of instruction m fills 16-B chunk 64m + l, a row's 32 data chunks or its pad chunk (which reads the
// row's last two doubles again) — else 132 instructions of 4-B pieces.  sc1, as every cross-workgroup read of the
// persistent launch.  The callers wait vmcnt(0) and pass a barrier.
__device__ __forceinline__ void chol_dma_tile(const double* __restrict__ src, int64_t lda, int rows, int cols,
                                              double* lds_dst, bool aligned, int w0, int nw) {
  typedef __attribute__((address_space(3))) void lds_void;
  typedef __attribute__((address_space(1))) const void g_void;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) - w0;
  if (w < 0 || w >= nw) return;
  if (aligned) {
    for (int m = w; m < 33; m += nw) {
      const int chunk = 64 * m + lane, row = chunk / 33, cc = chunk - 33 * row;
      const int cq = cc < 32 ? cc : 31, cmax = (cols + 1) / 2 - 1;
      const double* gp = src + (int64_t)(row < rows ? row : rows - 1) * lda + 2 * (cq < cmax ? cq : cmax);
      __builtin_amdgcn_global_load_lds((g_void*)gp, (lds_void*)(lds_dst + 128 * m), 16, 0, 16);
    }
  } else {
    for (int m = w; m < 132; m += nw) {
      const int dw = 64 * m + lane, row = dw / 132, cd = dw - 132 * row;
      const int cq = cd < 128 ? cd : 127, cmax = 2 * cols - 1;
      const char* gp = reinterpret_cast<const char*>(src + (int64_t)(row < rows ? row : rows - 1) * lda) +
                       4 * (cq < cmax ? cq : cmax);
      __builtin_amdgcn_global_load_lds((g_void*)gp, (lds_void*)(lds_dst + 32 * m), 4, 0, 16);
    }
  }
}

// bulk tasks of step k (see above): P(i, k) for i = k+2 .. t−1, then the update tiles by columns
// k0 > 0 (chol_persist_kernel after k0 per-step launches): step k0's panel column is already in A, so step k0 has
// only its update tasks
__host__ __device__ __forceinline__ int chol_persist_np(int t, int k, int k0) {
  return (k0 > 0 && k == k0) ? 0 : (t - k - 2 > 0 ? t - k - 2 : 0);
}
__host__ __device__ __forceinline__ int chol_persist_step_tasks(int t, int k, int k0 = 0) {
  const int m = t - k - 1;
  const int nu = m > 1 ? m * (m + 1) / 2 - 1 : 0;
  return chol_persist_np(t, k, k0) + nu;
}

// The sync words of one persistent launch: all zero, except (k0 > 0) the state the per-step launches leave — step
// k0's panel tiles published (pflag(i, k0) = 4) and every trailing tile updated through step k0 − 1 (cnt = k0).
// One launch in place of a memset; k0 = 0 also zeroes info (the per-step path's first kernel does that otherwise).
__global__ __launch_bounds__(256) void chol_persist_init_kernel(int* __restrict__ ints, int t, int k0,
                                                                int* __restrict__ info) {
  const int n = t + 2 * t * t + 2;
  for (int x = threadIdx.x; x < n; x += 256) ints[x] = chol_persist_init_word(x, t, k0);
  if (threadIdx.x == 0 && k0 == 0) *info = 0;
}

template <bool AR>
__global__ __launch_bounds__(256, kPersistWgPerCu) void chol_persist_kernel(double* __restrict__ A, int64_t N, int64_t lda, int t,
                                                              int total, double* __restrict__ Wf, CholSync sync,
                                                              int* __restrict__ info, int spin_limit, int k0) {
  __shared__ __attribute__((aligned(16))) double Ds[kNB * kDP];
  __shared__ __attribute__((aligned(16))) double Lp[kNB * kDP];
  __shared__ __attribute__((aligned(16))) double Wl[4 * kWlP];
  __shared__ __attribute__((aligned(16))) double Wfl[kCholWsDoubles];   // the walker's W fragments
  __shared__ __attribute__((aligned(16))) double PD[kNB * kDP];       // the walker's next diagonal tile (round 6)
  __shared__ int fl[kBlkFlags];
  __shared__ int s_task[2];
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const __amdgpu_buffer_rsrc_t ra = chol_rsrc(A, ((N - 1) * lda + N) * 8);
  if (blockIdx.x == 0) {
    // ---------------- the diagonal walk
    double av[16];                                              // A_kk[16w + 4e + g][16j + c], index 4j + e
    auto load_av = [&](int k) {
      const int64_t r0 = (int64_t)k * kNB;
      const int nb = (int)(N - r0 < kNB ? N - r0 : kNB);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = 16 * w + 4 * e + g, col = 16 * j + c;
          av[4 * j + e] = (j <= w && row < nb && col <= row) ? ld_sc1(A + (r0 + row) * lda + r0 + col)
                                                             : (row == col ? 1.0 : 0.0);
        }
    };
    // k0 > 0: the per-step launches factored blocks 0 .. k0 and formed panel column k0; the walk starts at k0 + 1
    // from the panel tile (k0 + 1, k0) in A
    const int kstart = k0 > 0 ? k0 + 1 : 0;
    if (kstart > 0) {
      const int64_t rb = (int64_t)kstart * kNB, cb = (int64_t)k0 * kNB;
      for (int x = tid; x < kNB * kNB; x += 256) {
        const int r = x >> 6, cc = x & 63;
        Lp[r * kDP + cc] = rb + r < N ? ld_sc1(A + (rb + r) * lda + cb + cc) : 0.0;
      }
    }
    load_av(kstart);
    if (tid < kBlkFlags) fl[tid] = 0;
    // Round 6: the next panel tile and the next diagonal tile reach the walker through LDS (chol_dma_tile: all four
    // waves, direct-to-LDS) and the panel product reads them there — one load latency for both tiles instead of the
    // per-lane loads of load_av and chol_persist_panel (walk: panel phase 4.45 → 2.5 µs per step, the wait including
    // the copies 1.0 → 2.2 µs; N = 3000 0.911-0.922 → 0.895-0.900 ms, profiles/r06_aa_*)
    const bool aligned = (lda & 1) == 0 && (reinterpret_cast<uintptr_t>(A) & 15) == 0;
    __syncthreads();
    for (int k = kstart; k < t; ++k) {
      OMB_PDBG(0, 1000 * k + 1);
      OMB_PTIME(8 * k + 0);
      const int64_t r0 = (int64_t)k * kNB;
      const int nb = (int)(N - r0 < kNB ? N - r0 : kNB);
      // D tiles (w, j ≤ w) = A_kk − L_{k,k−1} L_{k,k−1}ᵀ (Lp: written before the previous step's last barrier).  No
      // barrier after them: the core's LDS flags carry the step (epoch k + 1), so wave 0 starts its first tile's
      // factor while the later waves still form theirs.
      {
        double xa[16];
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int u = 0; u < 4; ++u) xa[4 * q + u] = k > 0 ? Lp[(16 * w + c) * kDP + 16 * q + 4 * g + u] : 0.0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (j <= w) {
            d4 acc = d4{0.0, 0.0, 0.0, 0.0};
            if (k > 0) {
#pragma unroll
              for (int s = 0; s < 16; ++s) {
                const double xb = Lp[(16 * j + c) * kDP + 16 * (s >> 2) + 4 * g + (s & 3)];
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(xa[s], xb, acc, 0, 0, 0);
              }
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) Ds[(16 * w + 4 * e + g) * kDP + 16 * j + c] = av[4 * j + e] - acc[e];
          }
        }
      }
      if (k > kstart && w >= 2) {   // the previous step's panel tile (k, k − 1): this wave's rows drained, its share
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if constexpr (AR)
          __hip_atomic_fetch_add(sync.pflag + k * t + k - 1, lane == 0 ? 2 : 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        else
          __hip_atomic_fetch_add(sync.pflag + k * t + k - 1, lane == 0 ? 2 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      OMB_PDBG(0, 1000 * k + 2);
      OMB_PTIME(8 * k + 1);
      chol64_blocked<kCholDReady>(A, lda, r0, nb, 0, Wf + (int64_t)k * kCholWsDoubles, Ds, Wl, fl, k + 1, Wfl);
      OMB_PDBG(1 + w, 1000 * k + 3);
      const int64_t rb1 = (int64_t)(k + 1) * kNB;
      const int rows1 = (int)(N - rb1 < kNB ? N - rb1 : kNB);
      chol_signal<AR>(sync.wflag + k, 1);                           // W_k's fragments (wf_store: sc1) drained
      OMB_PDBG(0, 1000 * k + 4);
      if (w == 0 && (fl[20] || fl[21])) atomicCAS(info, 0, fl[21] ? kCholSpinFault : (int)(r0 + fl[20]));
      if (w == 0) fl[20] = 0;           // read above (wave 0, in order); the next step's writes follow a barrier
      OMB_PTIME(8 * k + 2);
      if (k + 1 < t) {
        // the next panel tile and the next diagonal tile: both updated through step k − 1 by the workers, copied into
        // Lp (free since the D tiles) and PD by all four waves
        if (w == 0) {
          const int i1 = (k + 1) * t;
          if (chol_poll_ge<AR>(sync.cnt + i1 + k, k, sync, spin_limit, info))
            chol_poll_ge<AR>(sync.cnt + i1 + k + 1, k, sync, spin_limit, info);
        }
        __syncthreads();
        OMB_PDBG(0, 1000 * k + 5);
        chol_dma_tile(A + rb1 * lda + (int64_t)k * kNB, lda, rows1, kNB, Lp, aligned, 0, 4);
        chol_dma_tile(A + rb1 * lda + rb1, lda, rows1, rows1, PD, aligned, 0, 4);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        OMB_PTIME(8 * k + 3);
        // A_{k+1,k+1}'s lower tiles into av (load_av's mask), and the panel tile L_{k+1,k} = A_{k+1,k} W_kᵀ formed in
        // place in Lp — each wave reads its 16 rows into registers, then writes the same rows (chol_persist_panel's
        // product, bitwise)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int row = 16 * w + 4 * e + g, col = 16 * j + c;
            av[4 * j + e] = (j <= w && row < rows1 && col <= row) ? PD[row * kDP + col] : (row == col ? 1.0 : 0.0);
          }
        {
          double x[16];
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int u = 0; u < 4; ++u)
              x[4 * q + u] = 16 * w + c < rows1 ? Lp[(16 * w + c) * kDP + 16 * q + 4 * g + u] : 0.0;
#pragma unroll
          for (int jb = 0; jb < 4; ++jb) {
            d4 pa = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int q = 0; q < 16; ++q)
              if (q < 4 * (jb + 1))
                pa = __builtin_amdgcn_mfma_f64_16x16x4f64(x[q], Wfl[jb * 16 * 64 + q * 64 + lane], pa, 0, 0, 0);
#pragma unroll
            for (int e = 0; e < 4; ++e) Lp[(16 * w + 4 * e + g) * kDP + 16 * jb + c] = pa[e];
          }
        }
        // Lp visible to every wave; waves 2 and 3 store the tile to A (32 rows each, sc1) and signal it in the next
        // step, after their D tiles, where they wait for W_00 anyway: the stores' drain (≈ 2.4 µs) stays off the
        // chain that waves 0 and 1 run (consumers wait for 4 = 2 + 2)
        __syncthreads();
        if (w >= 2) {
          const int64_t rbase = (int64_t)(k + 1) * kNB;
#pragma unroll 4
          for (int q = 0; q < 32; ++q) {
            const int lr = 32 * (w - 2) + q;
            if (rbase + lr < N) st_sc1(A + (rbase + lr) * lda + (int64_t)k * kNB + lane, Lp[lr * kDP + lane]);
          }
        }
        OMB_PDBG(0, 1000 * k + 6);
        OMB_PTIME(8 * k + 4);
      }
    }
    return;
  }
  // ---------------- workers
  for (;;) {
    if (w == 0) {                 // the whole wave adds 1 (lane 0) + 0 (the rest): lane 0's old value is the ticket
      const int old = __hip_atomic_fetch_add(sync.ticket, lane == 0 ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_task[0] = __builtin_amdgcn_readfirstlane(old);   // every lane: the same value, no divergent store
    }
    __syncthreads();
    // read as a wave-uniform value: loaded per lane, the compiler treats every branch on q as divergent and
    // restructures the loop around the barriers below (it sank the flag stores out of the task code, and the
    // launch hung at N = 130, gpurun_out/r04_o)
    int q = __builtin_amdgcn_readfirstlane(s_task[0]);
    OMB_PDBG(8 * blockIdx.x, q + 1);
    OMB_PTIME(8 * t + 4 * q);
    if (q >= total) {
      OMB_PDBG(8 * blockIdx.x + 1, 99);
      return;
    }
    // the task: from the table (round 5, lookahead order) or the step-major arithmetic order
    int k = k0, i = 0, j = 0, nb = 1;
    bool panel;
    if (sync.tab) {
      const int e = __builtin_amdgcn_readfirstlane(sync.tab[2 * q]);
      nb = __builtin_amdgcn_readfirstlane(sync.tab[2 * q + 1]);
      panel = (e >> 30) == 0;
      k = (e >> 20) & 1023;
      i = (e >> 10) & 1023;
      j = e & 1023;
    } else {
      for (; k < t; ++k) {
        const int nk = chol_persist_step_tasks(t, k, k0);
        if (q < nk) break;
        q -= nk;
      }
      const int np = chol_persist_np(t, k, k0);
      panel = q < np;
      if (panel) {
        i = k + 2 + q;
      } else {
        int u = q - np + 1;                                     // + 1: (k+1, k+1) is the diagonal workgroup's
        j = k + 1;
        while (u >= t - j) {
          u -= t - j;
          ++j;
        }
        i = j + u;
      }
    }
    if (panel) {
      if (w == 0 && chol_poll_ge<AR>(sync.wflag + k, 1, sync, spin_limit, info))
        chol_poll_ge<AR>(sync.cnt + i * t + k, k, sync, spin_limit, info);
      __syncthreads();
      OMB_PDBG(8 * blockIdx.x + 1, 1);
      OMB_PTIME(8 * t + 4 * s_task[0] + 1);
      chol_persist_panel(ra, A, N, lda, i, k, Wf + (int64_t)k * kCholWsDoubles, nullptr);
      OMB_PDBG(8 * blockIdx.x + 2 + w, 2);
      chol_signal<AR>(sync.pflag + i * t + k, 4);
      OMB_PDBG(8 * blockIdx.x + 1, 3);
      OMB_PTIME(8 * t + 4 * s_task[0] + 2);
    } else if (nb == 1) {
      if (w == 0 && chol_poll_ge<AR>(sync.pflag + i * t + k, 4, sync, spin_limit, info) &&
          chol_poll_ge<AR>(sync.pflag + j * t + k, 4, sync, spin_limit, info))
        chol_poll_ge<AR>(sync.cnt + i * t + j, k, sync, spin_limit, info);
      __syncthreads();
      OMB_PDBG(8 * blockIdx.x + 1, 11);
      OMB_PTIME(8 * t + 4 * s_task[0] + 1);
      chol_persist_update(ra, A, N, lda, i, j, k);
      OMB_PDBG(8 * blockIdx.x + 2 + w, 12);
      chol_signal<AR>(sync.cnt + i * t + j, k + 1);
      OMB_PDBG(8 * blockIdx.x + 1, 13);
      OMB_PTIME(8 * t + 4 * s_task[0] + 2);
    } else {
      // U(i, j, k .. k + nb − 1): the last step's panels first (the latest to appear), then all of them at once
      if (w == 0 && chol_poll_ge<AR>(sync.pflag + i * t + k + nb - 1, 4, sync, spin_limit, info) &&
          chol_poll_ge<AR>(sync.pflag + j * t + k + nb - 1, 4, sync, spin_limit, info) &&
          chol_poll_panels<AR>(sync.pflag, t, i, j, k, nb, sync, spin_limit, info))
        chol_poll_ge<AR>(sync.cnt + i * t + j, k, sync, spin_limit, info);
      __syncthreads();
      OMB_PDBG(8 * blockIdx.x + 1, 21);
      OMB_PTIME(8 * t + 4 * s_task[0] + 1);
      chol_persist_update_batch(ra, A, N, lda, i, j, k, nb);
      OMB_PDBG(8 * blockIdx.x + 2 + w, 22);
      chol_signal<AR>(sync.cnt + i * t + j, k + nb);
      OMB_PDBG(8 * blockIdx.x + 1, 13);
      OMB_PTIME(8 * t + 4 * s_task[0] + 2);
    }
  }
}

// ----------------------------------------------------------------------------- triangular inverse
// X = L⁻¹ for a lower-triangular L (n×n).  The 64×64 diagonal blocks are inverted in parallel (one
// wave per block; lane c solves L_ii x = e_c by column-oriented substitution, the column of L_ii
// read as an LDS broadcast), then block row i of X is −X_ii·(L[i, :i]·X[:i, :i]), two GEMMs per
// block row (trinv_rows).  The caller zeroes X first (its upper triangle stays zero).
__global__ __launch_bounds__(64) void trinv_diag_kernel(const double* __restrict__ L, int64_t n, int64_t lda,
                                                        double* __restrict__ X, int64_t ldx) {
  __shared__ __attribute__((aligned(16))) double LsT[kNB][kNB + 2];   // LsT[c][r] = L_ii[r][c]
  __shared__ double rinv[kNB];
  const int64_t c0 = (int64_t)blockIdx.x * kNB;
  const int nb = (int)((n - c0) < kNB ? (n - c0) : kNB);
  const int lane = threadIdx.x;
  for (int c = 0; c < kNB; ++c) {
    double v = (c == lane) ? 1.0 : 0.0;
    if (lane < nb && c <= lane) v = L[(c0 + lane) * lda + c0 + c];
    LsT[c][lane] = v;
  }
  __builtin_amdgcn_wave_barrier();
  rinv[lane] = 1.0 / LsT[lane][lane];
  __builtin_amdgcn_wave_barrier();
  double x[kNB];
#pragma unroll
  for (int r = 0; r < kNB; ++r) x[r] = (r == lane) ? 1.0 : 0.0;
  static_for<0, kNB>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    const double xj = x[j] * rinv[j];
    x[j] = xj;
    axpy_tail<j>(x, -xj, LsT[j]);
  });
  if (lane >= nb) return;
  double* dst = X + c0 * ldx + c0 + lane;   // column `lane` of the block
  if (nb == kNB) {
#pragma unroll
    for (int r = 0; r < kNB; ++r) dst[r * ldx] = x[r];
  } else {
    for (int r = 0; r < nb; ++r) {
      double v = 0.0;
#pragma unroll
      for (int q = 0; q < kNB; ++q) v = (q == r) ? x[q] : v;
      dst[r * ldx] = v;
    }
  }
}

// ----------------------------------------------------------------------------- GP marginal likelihood
// Gradient of GPy's log marginal likelihood for exact inference with a stationary ARD kernel,
//   dL/dθ = ½ Σ_ik W_ik ∂K_ik/∂θ,  W = ααᵀ − Ky⁻¹   (ExactGaussianInference: dL_dK = ½(ααᵀ − Wi)),
// θ = (log σ_f², log ℓ_1..d):  ∂K/∂log σ_f² = K (no noise),  ∂K/∂log ℓ_j = −(dK/dr / r)·(Δ_j/ℓ_j)².
// One 16×16 tile per workgroup over the lower triangle (off-diagonal pairs count twice); each
// workgroup writes its d+1 partial sums; gp_reduce_kernel adds them in a fixed order.
template <int DP, int KIND>
__global__ __launch_bounds__(256) void gp_grad_kernel(const double* __restrict__ X, int d, int64_t n,
                                                      const double* __restrict__ ls, double variance,
                                                      const double* __restrict__ alpha,
                                                      const double* __restrict__ Kinv, int64_t ldk,
                                                      double* __restrict__ partials) {
  __shared__ double red[4][DP + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t i = (int64_t)blockIdx.y * 16 + (tid >> 4);
  const int64_t k = (int64_t)blockIdx.x * 16 + (tid & 15);
  double acc[DP + 1];
#pragma unroll
  for (int q = 0; q <= DP; ++q) acc[q] = 0.0;
  if (blockIdx.x <= blockIdx.y && i < n && k <= i) {
    double a[DP], b[DP], aa = 0.0, bb = 0.0, dot = 0.0;
#pragma unroll
    for (int j = 0; j < DP; ++j) {
      a[j] = (j < d) ? X[i * d + j] / ls[j] : 0.0;
      b[j] = (j < d) ? X[k * d + j] / ls[j] : 0.0;
      aa += a[j] * a[j];
      bb += b[j] * b[j];
      dot = fma(a[j], b[j], dot);
    }
    double r2 = (i == k) ? 0.0 : fma(-2.0, dot, aa + bb);
    r2 = r2_range<KIND>(r2);
    const double r = sqrt_nonneg(r2);
    double Kik, dkr;   // K and (dK/dr)/r
    if constexpr (KIND == OMB_KERNEL_MATERN52) {
      const double e = exp_nonpos(-(kSqrt5 * r));
      Kik = (variance * ((1.0 + kSqrt5 * r) + kFiveThirds * (r * r))) * e;
      dkr = -kFiveThirds * variance * (1.0 + kSqrt5 * r) * e;
    } else {
      const double e = exp_nonpos(-0.5 * (r * r));
      Kik = variance * e;
      dkr = -variance * e;
    }
    const double f = (i == k) ? 0.5 : 1.0;
    const double W = f * (alpha[i] * alpha[k] - Kinv[i * ldk + k]);
    acc[0] = W * Kik;
#pragma unroll
    for (int j = 0; j < DP; ++j) {
      const double dj = a[j] - b[j];
      acc[1 + j] = W * (-dkr) * (dj * dj);
    }
  }
#pragma unroll
  for (int q = 0; q <= DP; ++q) {
    double v = acc[q];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off);
    if (lane == 0) red[wave][q] = v;
  }
  __syncthreads();
  const int64_t blk = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
  if (tid <= DP) partials[blk * (DP + 1) + tid] = ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
}

// out[q] = Σ_blocks partials (q ≤ DP, fixed order); out[DP+1] = Σ log L_ii; out[DP+2] = yᵀα.
__global__ __launch_bounds__(256) void gp_reduce_kernel(const double* __restrict__ partials, int64_t nblk, int P,
                                                        const double* __restrict__ L, int64_t n, int64_t lda,
                                                        const double* __restrict__ y,
                                                        const double* __restrict__ alpha, double* __restrict__ out) {
  __shared__ double red[256];
  const int tid = threadIdx.x;
  for (int q = 0; q < P + 2; ++q) {
    double v = 0.0;
    if (q < P) {
      for (int64_t b = tid; b < nblk; b += 256) v += partials[b * P + q];
    } else if (q == P) {
      for (int64_t t = tid; t < n; t += 256) v += log(L[t * lda + t]);
    } else {
      for (int64_t t = tid; t < n; t += 256) v = fma(y[t], alpha[t], v);
    }
    red[tid] = v;
    __syncthreads();
    for (int s2 = 128; s2 > 0; s2 >>= 1) {
      if (tid < s2) red[tid] += red[tid + s2];
      __syncthreads();
    }
    if (tid == 0) out[q] = red[0];
    __syncthreads();
  }
}

// ----------------------------------------------------------------------------- GP fit, n ≤ 128: one workgroup
// The whole log-marginal-likelihood + gradient evaluation in one launch for the training-set sizes of a
// BO loop (n_init .. n_init + budget; the README run has n = 20 … 119), where the blocked path above is
// ~15 dependent launches and two host synchronisations.  Ky (full, symmetric, padded to 16·NB with an
// identity block) lives in LDS:
//   * Ky⁻¹ by the block sweep operator, 16 pivots per step: for the pivot block B (tile p) and the rest R,
//         A_BB ← −A_BB⁻¹,  A_BR ← A_BB⁻¹ A_BR,  A_RB ← A_BRᵀ,  A_RR ← A_RR − A_RB A_BB⁻¹ A_BR,
//     and after all NB steps A = −Ky⁻¹ (Goodnight's sweep, blocked).  With A_BB = L_B L_Bᵀ the update is
//     taken in its Cholesky form, A_RR −= W_Rᵀ W_R with W = L_B⁻¹ A_BR (the error of W grows with
//     cond(L_B) = cond(A_BB)^½; the form A_RB (A_BB⁻¹ A_BR) lost digits against scikit-learn on the
//     ill-conditioned K of a BO loop).  Step p:
//       (A) wave 0 factors the 16×16 diagonal tile in registers, one column per lane, the pivot column's
//           entries as wave-uniform v_readlane values; the pivots L_kk² are those of right-looking
//           Cholesky/LDLᵀ (log|Ky| = Σ log d_k, the positive-definiteness test !(d_k > 0) and GPy jitchol's
//           jitter retries as before); then L_B⁻¹ (lane c solves L x = e_c);
//       (B) wave J forms W_J = L_B⁻¹ A_BJ and V_J = L_B⁻ᵀ W_J = A_BB⁻¹ A_BJ on FP64 MFMA (wave p:
//           V_p = L_B⁻ᵀ L_B⁻¹ = A_BB⁻¹) and stores W_J over A_BJ;
//       (C) the lower trailing tiles A_IJ −= W_Iᵀ W_J (I ≥ J) on FP64 MFMA (4 k-steps), dealt over all
//           waves, mirrored into A_JI;
//       (D) wave J writes the panel tiles A_BJ = V_J, A_JB = V_Jᵀ; wave p the diagonal tile −A_BB⁻¹.
//     Three barriers per 16 pivots (the 2-pivot scalar sweep this replaced needed n/2 barriers and n³/2
//     scalar LDS updates: 0.18 ms at n = 96 against 0.24 ms for the multi-launch path at n = 128).  Every
//     update keeps A exactly symmetric (products formed symmetrically, tiles mirrored).
//   * α = Ky⁻¹y, then ½ Σ_ik W_ik ∂K_ik/∂θ with W = ααᵀ − Ky⁻¹ over the full matrix (the same sums as
//     gp_grad_kernel), all reductions in a fixed order (deterministic).
// out[0..DP] gradient, out[DP+1] = Σ log L_ii, out[DP+2] = yᵀα, out[DP+3] = jitter, out[DP+4] = info
// (0, or the 1-based column of the failed pivot after the last retry).
constexpr int kSmallFitN = 128;
constexpr int kSmallFitLD = 136;    // row pitch (doubles) of the LDS copy of Ky
constexpr int kSmallFitThreads = 512;
constexpr int kSmallFitMax = 128;
constexpr int kSmallFitXs = 1024;   // LDS doubles for X/ℓ: n·DP ≤ 1024 (d ≤ 8 at n = 128)

// the one-workgroup fit takes n_var ≤ 8 (gp_lml_small_fits), so its lengthscale argument is 8 doubles
// (an OMB_MAX_DIM-wide one would be a 2-KiB kernel argument and a 2-KiB local array in the batch kernel)
constexpr int kSmallFitMaxDP = 8;
struct FitLs {
  double v[kSmallFitMaxDP];
};

// K and (dK/dr)/r of scaled rows a (LDS, wave-uniform row) and b (registers): gp_grad_kernel's arithmetic
template <int DP, int KIND>
__device__ __forceinline__ void fit_pair(const double* __restrict__ a, const double (&b)[DP], bool diag,
                                         double variance, double& K, double& dkr) {
  double aa = 0.0, bb = 0.0, dot = 0.0;
#pragma unroll
  for (int j = 0; j < DP; ++j) {
    aa += a[j] * a[j];
    bb += b[j] * b[j];
    dot = fma(a[j], b[j], dot);
  }
  double r2 = diag ? 0.0 : fma(-2.0, dot, aa + bb);
  r2 = r2_range<KIND>(r2);
  const double r = sqrt_nonneg(r2);
  if constexpr (KIND == OMB_KERNEL_MATERN52) {
    const double e = exp_nonpos(-(kSqrt5 * r));
    K = (variance * ((1.0 + kSqrt5 * r) + kFiveThirds * (r * r))) * e;
    dkr = -kFiveThirds * variance * (1.0 + kSqrt5 * r) * e;
  } else {
    const double e = exp_nonpos(-0.5 * (r * r));
    K = variance * e;
    dkr = -variance * e;
  }
}

// Lane k of each 16-lane row, to every lane of that row (DPP row_newbcast, gfx90a+), for a double; k must
// be a compile-time constant after unrolling (the switch folds away).
__device__ __forceinline__ double row_bcast_f64(double v, int k) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  int rl = lo, rh = hi;
  switch (k) {
#define OMB_RB(K)                                                       \
  case K:                                                               \
    rl = __builtin_amdgcn_update_dpp(0, lo, 0x150 + K, 0xf, 0xf, false); \
    rh = __builtin_amdgcn_update_dpp(0, hi, 0x150 + K, 0xf, 0xf, false); \
    break;
    OMB_RB(0) OMB_RB(1) OMB_RB(2) OMB_RB(3) OMB_RB(4) OMB_RB(5) OMB_RB(6) OMB_RB(7)
    OMB_RB(8) OMB_RB(9) OMB_RB(10) OMB_RB(11) OMB_RB(12) OMB_RB(13) OMB_RB(14) OMB_RB(15)
#undef OMB_RB
    default: break;
  }
  return __hiloint2double(rh, rl);
}

// Phase timestamps of the block sweep for tools/ablate/ablate_gpfit (empty here): OMB_FIT_TRACE(p, id).
#ifndef OMB_FIT_TRACE
#define OMB_FIT_TRACE(p, id)
#endif

// Thread map of the K build / gradient: wave w owns rows i ≡ w (mod NW), lane l owns columns l and l + 64.
// ABL (tools/ablate/ablate_gpfit only): bit 1 skips the block sweep, bit 2 the gradient sums, bit 4 the
// kernel evaluations of the K build.
template <int DP, int KIND, int ABL = 0>
__device__ __forceinline__ void gp_lml_small_body(const double* __restrict__ X, int d, int n, const FitLs& ls,
                                                  double variance, double base, const double* __restrict__ y,
                                                  double* __restrict__ out) {
  constexpr int NW = kSmallFitThreads / 64, LD = kSmallFitLD, RPW = kSmallFitN / NW;
  __shared__ double A[kSmallFitN * LD];
  __shared__ double xs[kSmallFitXs];
  __shared__ double Ls[16 * 17];                   // L_B⁻¹ (inverse Cholesky factor of the pivot block)
  __shared__ double Lf[16 * 17];                   // L_B
  __shared__ double piv[kSmallFitN], alpha[kSmallFitN];
  __shared__ double red[NW][DP + 3];
  __shared__ int flag;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int NB = (n + 15) >> 4, np = 16 * NB;     // padded size: Ky ⊕ I
  const int c16 = lane & 15, g4 = lane >> 4;      // MFMA fragment coordinates
  for (int e = tid; e < n * DP; e += kSmallFitThreads) {
    const int i = e / DP, j = e - i * DP;
    xs[e] = (j < d) ? X[i * d + j] / ls.v[j] : 0.0;
  }
  __syncthreads();
  const int j0 = lane, j1 = lane + 64;
  const bool h0 = j0 < n, h1 = j1 < n;
  // this lane's two columns' scaled coordinates (LDS; loaded where used so they are not live across the sweep)
  auto load_cols = [&](double (&b0)[DP], double (&b1)[DP]) {
#pragma unroll
    for (int q = 0; q < DP; ++q) {
      b0[q] = h0 ? xs[j0 * DP + q] : 0.0;
      b1[q] = h1 ? xs[j1 * DP + q] : 0.0;
    }
  };
  const double mean_diag = variance + base;
  int bad = 0;
  double jit = 0.0;
  for (int t = -1; t < 5; ++t) {
    jit = (t < 0) ? 0.0 : mean_diag * 1e-6 * pow(10.0, (double)t);
    double b0[DP], b1[DP];
    load_cols(b0, b1);
    for (int m = 0; m < RPW; ++m) {
      const int i = wave + NW * m;
      if (i >= np) break;
      if (i >= n) {                                 // padding rows: the identity block
        if (j0 < np) A[i * LD + j0] = (i == j0) ? 1.0 : 0.0;
        if (j1 < np) A[i * LD + j1] = (i == j1) ? 1.0 : 0.0;
        continue;
      }
      double K, dkr;
      if constexpr ((ABL & 4) != 0) {
        if (j0 < np) A[i * LD + j0] = (i == j0) ? 2.0 : 0.0;
        if (j1 < np) A[i * LD + j1] = (i == j1) ? 2.0 : 0.0;
        continue;
      }
      if (h0) {
        fit_pair<DP, KIND>(xs + i * DP, b0, i == j0, variance, K, dkr);
        A[i * LD + j0] = (i == j0) ? K + (base + jit) : K;
      } else if (j0 < np) {
        A[i * LD + j0] = 0.0;
      }
      if (h1) {
        fit_pair<DP, KIND>(xs + i * DP, b1, i == j1, variance, K, dkr);
        A[i * LD + j1] = (i == j1) ? K + (base + jit) : K;
      } else if (j1 < np) {
        A[i * LD + j1] = 0.0;
      }
    }
    __syncthreads();
    bad = 0;
    // fragment layout of a 16×16 tile in one wave: element (r, c) in lane ((r & 3) << 4) + c, register r >> 2
    // (the FP64 MFMA accumulator layout: register e holds rows 4e + (lane >> 4))
    for (int p = 0; p < ((ABL & 1) ? 0 : NB); ++p) {
      const int p16 = 16 * p;
      // (A) wave 0: Cholesky of the diagonal tile (the current Schur complement) in the fragment layout:
      //     the pivot by v_readlane, the pivot column's entries of a lane's 4 rows by DPP row_newbcast (lane k
      //     of each 16-lane row), the pivot row's entry of its column by one shuffle issued ahead of the
      //     pivot (off the dependent chain); then L_B⁻¹ with lane c solving L x = e_c (L from LDS).
      if (wave == 0) {
        double D[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) D[e] = A[(p16 + 4 * e + g4) * LD + p16 + c16];
        double ild[16];
        int fail = 0;
        // look-ahead: the next pivot and the next pivot row's entry of this lane's column are formed from
        // values read before the current update (x = D[k+1][k], the row k+1 shuffled ahead), with the same
        // expressions as the element update, so the dependent chain per pivot is sqrt, rcp and one fma
        double dk = readlane_f64(D[0], 0);                                       // D[0][0]
        double rowk = __shfl(D[0], c16);                                         // D[0][c]
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          double x = 0.0, dn = 0.0, rown = 0.0;
          if (k < 15) {
            const int k1 = k + 1;
            x = readlane_f64(D[k1 >> 2], ((k1 & 3) << 4) + k);                  // D[k+1][k]
            dn = readlane_f64(D[k1 >> 2], ((k1 & 3) << 4) + k1);                // D[k+1][k+1]
            rown = __shfl(D[k1 >> 2], ((k1 & 3) << 4) + c16);                   // D[k+1][c], before this update
          }
          ild[k] = 0.0;
          if (fail) continue;
          if (!(dk > 0.0)) {                        // uniform
            fail = p16 + k + 1;
            continue;
          }
          const double lkk = sqrt_nonneg(dk);
          double il = __builtin_amdgcn_rcp(lkk);
          il = fma(il, fma(-lkk, il, 1.0), il);
          il = fma(il, fma(-lkk, il, 1.0), il);
          ild[k] = il;
          const double il2 = il * il;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int r = 4 * e + g4;
            const double colk = row_bcast_f64(D[e], k);                          // D[r][k]
            double v = D[e];
            if (r > k && c16 > k) v = fma(-(colk * rowk), il2, v);               // symmetric in (r, c)
            if (c16 == k) v = (r > k) ? colk * il : (r == k ? lkk : 0.0);
            if (r == k && c16 > k) v = 0.0;
            D[e] = v;
          }
          if (lane == 0) piv[p16 + k] = dk;
          if (k < 15) {
            const double dnext = fma(-(x * x), il2, dn);                          // = the updated D[k+1][k+1]
            rowk = fma(-(x * rowk), il2, rown);                                   // = the updated D[k+1][c] (c > k+1)
            dk = dnext;
          }
        }
        if (lane == 0) flag = fail;
        OMB_FIT_TRACE(p, 1);
#pragma unroll
        for (int e = 0; e < 4; ++e) Lf[(4 * e + g4) * 17 + c16] = D[e];
        const int c = lane & 15;
        if (!fail) {
          // x = L_B⁻¹ e_c: x[m] = acc[m] / L[m][m], acc[r] −= L[r][m] x[m] (r > m); L[r][m] as an LDS
          // broadcast (one wave: its LDS accesses complete in order)
          double x[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) x[r] = (r == c) ? 1.0 : 0.0;
#pragma unroll
          for (int m = 0; m < 16; ++m) {
            x[m] *= ild[m];
#pragma unroll
            for (int r = m + 1; r < 16; ++r) x[r] = fma(-Lf[r * 17 + m], x[m], x[r]);
          }
          if (lane < 16) {
#pragma unroll
            for (int r = 0; r < 16; ++r) Ls[r * 17 + c] = x[r];                  // L_B⁻¹[r][c]
          }
        }
      }
      OMB_FIT_TRACE(p, 2);
      __syncthreads();
      OMB_FIT_TRACE(p, 3);
      bad = flag;
      if (bad) break;
      // (B) wave J ≠ p: W_J = L_B⁻¹ A_BJ and V_J = L_B⁻ᵀ W_J = A_BB⁻¹ A_BJ on FP64 MFMA (W_J's accumulator is
      //     the B fragment of the second product and of the trailing update); W_J replaces A_BJ in LDS.
      //     Wave p: V_p = L_B⁻ᵀ L_B⁻¹ = A_BB⁻¹.
      const int J = wave;
      const bool active = J < NB;
      double W[4], V[4];
      if (active) {
        d4 w = d4{0.0, 0.0, 0.0, 0.0};
        if (J != p) {
#pragma unroll
          for (int s = 0; s < 4; ++s)
            w = __builtin_amdgcn_mfma_f64_16x16x4f64(Ls[c16 * 17 + 4 * s + g4], A[(p16 + 4 * s + g4) * LD + 16 * J + c16],
                                                    w, 0, 0, 0);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) w[e] = Ls[(4 * e + g4) * 17 + c16];
        }
        d4 v = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s = 0; s < 4; ++s)
          v = __builtin_amdgcn_mfma_f64_16x16x4f64(Ls[(4 * s + g4) * 17 + c16], w[s], v, 0, 0, 0);   // (L⁻ᵀ)[c16][4s+g4]
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          W[e] = w[e];
          V[e] = v[e];
        }
        if (J != p) {
#pragma unroll
          for (int e = 0; e < 4; ++e) A[(p16 + 4 * e + g4) * LD + 16 * J + c16] = W[e];
        }
      }
      OMB_FIT_TRACE(p, 4);
      __syncthreads();
      OMB_FIT_TRACE(p, 5);
      // (C) the lower trailing tiles (I ≥ J, both ≠ p) dealt over all waves: A_IJ −= W_Iᵀ W_J on FP64 MFMA,
      //     both operands from the W tiles in LDS, mirrored into A_JI
      {
        const int nt = (NB - 1) * NB / 2;           // lower tiles of the (NB−1)-block trailing matrix
        for (int t2 = wave; t2 < nt; t2 += NW) {
          // t2 → (i, j) over 0 ≤ j ≤ i < NB − 1, then skip the pivot block
          int i = (int)((sqrt(8.0 * t2 + 1.0) - 1.0) * 0.5);
          while (i * (i + 1) / 2 > t2) --i;
          while ((i + 1) * (i + 2) / 2 <= t2) ++i;
          const int j = t2 - i * (i + 1) / 2;
          const int I = i + (i >= p), Jt = j + (j >= p);
          d4 T;
#pragma unroll
          for (int e = 0; e < 4; ++e) T[e] = A[(16 * I + 4 * e + g4) * LD + 16 * Jt + c16];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const double a = -A[(p16 + 4 * q + g4) * LD + 16 * I + c16];    // −W_I[4q + g4][c16]
            const double b = A[(p16 + 4 * q + g4) * LD + 16 * Jt + c16];    // W_J[4q + g4][c16]
            T = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, T, 0, 0, 0);
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int r = 4 * e + g4;
            if (I != Jt || r >= c16) {              // diagonal tile: the lower half, mirrored
              A[(16 * I + r) * LD + 16 * Jt + c16] = T[e];
              A[(16 * Jt + c16) * LD + 16 * I + r] = T[e];
            }
          }
        }
      }
      OMB_FIT_TRACE(p, 6);
      __syncthreads();
      OMB_FIT_TRACE(p, 7);
      // (D) the panel A_BJ = V_J, A_JB = V_Jᵀ, and the diagonal tile −A_BB⁻¹ (lower half, mirrored)
      if (active) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * e + g4;
          if (J != p) {
            A[(p16 + r) * LD + 16 * J + c16] = V[e];
            A[(16 * J + c16) * LD + p16 + r] = V[e];
          } else if (r >= c16) {
            A[(p16 + r) * LD + p16 + c16] = -V[e];
            A[(p16 + c16) * LD + p16 + r] = -V[e];
          }
        }
      }
    }
    __syncthreads();
    if (!bad) break;
  }
  if (bad) {
    if (tid == 0) {
      for (int q = 0; q < DP + 3; ++q) out[q] = 0.0;
      out[DP + 3] = jit;
      out[DP + 4] = (double)bad;
    }
    return;
  }
  // α = Ky⁻¹ y = −A y: one wave per row, lanes over columns, fixed-order wave reduction
  const double y0 = h0 ? y[j0] : 0.0, y1 = h1 ? y[j1] : 0.0;
  for (int m = 0; m < RPW; ++m) {
    const int i = wave + NW * m;
    if (i >= n) break;
    double s = h0 ? A[i * LD + j0] * y0 : 0.0;
    if (h1) s = fma(A[i * LD + j1], y1, s);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    if (lane == 0) alpha[i] = -s;
  }
  __syncthreads();
  double acc[DP + 3];
#pragma unroll
  for (int q = 0; q < DP + 3; ++q) acc[q] = 0.0;
  const double al0 = h0 ? alpha[j0] : 0.0, al1 = h1 ? alpha[j1] : 0.0;
  double b0[DP], b1[DP];
  load_cols(b0, b1);
  for (int m = 0; m < ((ABL & 2) ? 0 : RPW); ++m) {
    const int i = wave + NW * m;
    if (i >= n) break;
    const double* a = xs + i * DP;
    const double ai = alpha[i];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h == 0 ? !h0 : !h1) continue;
      const int k = h == 0 ? j0 : j1;
      double K, dkr;
      fit_pair<DP, KIND>(a, h == 0 ? b0 : b1, i == k, variance, K, dkr);
      const double W = 0.5 * (ai * (h == 0 ? al0 : al1) + A[i * LD + k]);   // ½ (ααᵀ − Ky⁻¹)
      acc[0] = fma(W, K, acc[0]);
      const double wd = W * (-dkr);
#pragma unroll
      for (int q = 0; q < DP; ++q) {
        const double dq = a[q] - (h == 0 ? b0[q] : b1[q]);
        acc[1 + q] = fma(wd, dq * dq, acc[1 + q]);
      }
    }
  }
  if (tid < n) {
    acc[DP + 1] = 0.5 * log(piv[tid]);
    acc[DP + 2] = y[tid] * alpha[tid];
  }
#pragma unroll
  for (int q = 0; q < DP + 3; ++q) {
    double v = acc[q];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (lane == 0) red[wave][q] = v;
  }
  __syncthreads();
  if (tid < DP + 3) {
    double v = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[w][tid];
    out[tid] = v;
  }
  if (tid == 0) {
    out[DP + 3] = jit;
    out[DP + 4] = 0.0;
  }
}

template <int DP, int KIND>
__global__ __launch_bounds__(kSmallFitThreads) void gp_lml_small_kernel(const double* __restrict__ X, int d, int n,
                                                                        FitLs ls, double variance, double base,
                                                                        const double* __restrict__ y,
                                                                        double* __restrict__ out) {
  gp_lml_small_body<DP, KIND>(X, d, n, ls, variance, base, y, out);
}

// Several GPs on the same inputs (the drivers' per-objective fits), one workgroup each, one launch:
// workgroup b evaluates problem b with exactly the single-problem arithmetic.
struct FitBatch {
  const double* y[kFitBatchMax];
  double* out[kFitBatchMax];
  double ls[kFitBatchMax][8];
  double variance[kFitBatchMax];
};

template <int DP, int KIND, int ABL = 0>
__global__ __launch_bounds__(kSmallFitThreads) void gp_lml_small_batch_kernel(const double* __restrict__ X, int d,
                                                                              int n, FitBatch b, double base) {
  const int p = blockIdx.x;
  FitLs ls;
#pragma unroll
  for (int j = 0; j < kSmallFitMaxDP; ++j) ls.v[j] = b.ls[p][j];
  gp_lml_small_body<DP, KIND, ABL>(X, d, n, ls, b.variance[p], base, b.y[p], b.out[p]);
}

// DP ≤ 8: the two candidate columns' scaled coordinates stay in registers (DP = 16 spills at 1024 threads).
// n ≤ 128: Ky and its block sweep fit one CU's LDS (the scalar 2-pivot sweep this replaced took 0.18 ms at
// n = 96 and lost to the multi-launch path above n = 96).
bool gp_lml_small_fits(int n, int DP) { return n >= 1 && n <= kSmallFitMax && DP <= 8 && n * DP <= kSmallFitXs; }

hipError_t launch_gp_lml_small(hipStream_t stream, int kind, int DP, const double* X, int d, int n,
                               const double* ls_host, double variance, double base, const double* y, double* out) {
  if (!gp_lml_small_fits(n, DP) || d < 1 || d > DP || DP > kSmallFitMaxDP) return hipErrorInvalidValue;
  FitLs ls{};
  for (int j = 0; j < kSmallFitMaxDP; ++j) ls.v[j] = (j < d) ? ls_host[j] : 1.0;
#define OMB_GS(DPV)                                                                                              \
  case DPV:                                                                                                      \
    if (kind == OMB_KERNEL_RBF)                                                                                  \
      hipLaunchKernelGGL((gp_lml_small_kernel<DPV, OMB_KERNEL_RBF>), dim3(1), dim3(kSmallFitThreads), 0, stream, \
                         X, d, n, ls, variance, base, y, out);                                                   \
    else                                                                                                         \
      hipLaunchKernelGGL((gp_lml_small_kernel<DPV, OMB_KERNEL_MATERN52>), dim3(1), dim3(kSmallFitThreads), 0,    \
                         stream, X, d, n, ls, variance, base, y, out);                                           \
    break;
  switch (DP) {
    OMB_GS(2) OMB_GS(4) OMB_GS(6) OMB_GS(8)
    default: return hipErrorInvalidValue;
  }
#undef OMB_GS
  return hipGetLastError();
}

hipError_t launch_gp_lml_small_batch(hipStream_t stream, int kind, int DP, const double* X, int d, int n, int k,
                                     const double* const* y, const double* ls_host, const double* variance,
                                     double base, double* const* out) {
  if (!gp_lml_small_fits(n, DP) || d < 1 || d > DP || DP > 8 || k < 1 || k > kFitBatchMax)
    return hipErrorInvalidValue;
  FitBatch b{};
  for (int p = 0; p < k; ++p) {
    b.y[p] = y[p];
    b.out[p] = out[p];
    b.variance[p] = variance[p];
    for (int j = 0; j < 8; ++j) b.ls[p][j] = (j < d) ? ls_host[p * d + j] : 1.0;
  }
#define OMB_GSB(DPV)                                                                                        \
  case DPV:                                                                                                 \
    if (kind == OMB_KERNEL_RBF)                                                                             \
      hipLaunchKernelGGL((gp_lml_small_batch_kernel<DPV, OMB_KERNEL_RBF>), dim3(k), dim3(kSmallFitThreads), 0, \
                         stream, X, d, n, b, base);                                                          \
    else                                                                                                    \
      hipLaunchKernelGGL((gp_lml_small_batch_kernel<DPV, OMB_KERNEL_MATERN52>), dim3(k),                    \
                         dim3(kSmallFitThreads), 0, stream, X, d, n, b, base);                              \
    break;
  switch (DP) {
    OMB_GSB(2) OMB_GSB(4) OMB_GSB(6) OMB_GSB(8)
    default: return hipErrorInvalidValue;
  }
#undef OMB_GSB
  return hipGetLastError();
}

// ----------------------------------------------------------------------------- selection
// np.argmin order: the first NaN wins, else the smallest value, lowest index among ties.
__device__ __forceinline__ bool sel_better(double v, int64_t i, double bv, int64_t bi) {
  if (i < 0) return false;
  if (bi < 0) return true;
  const bool vn = v != v, bn = bv != bv;
  if (vn || bn) return vn && (!bn || i < bi);
  return v < bv || (v == bv && i < bi);
}

__global__ __launch_bounds__(1024) void select_kernel(const double* __restrict__ Y, int B, int64_t N,
                                                      int64_t* __restrict__ idx_out) {
  __shared__ unsigned excl[kSelectMaxN / 32];
  __shared__ double sv[16];
  __shared__ int64_t si[16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  for (int64_t w = tid; w < (N + 31) / 32; w += blockDim.x) excl[w] = 0u;
  __syncthreads();
  for (int b = 0; b < B; ++b) {
    const double* y = Y + (int64_t)b * N;
    double bv = 0.0;
    int64_t bi = -1;
    for (int64_t i = tid; i < N; i += blockDim.x) {
      // a picked candidate reads as +inf for every later sample (turbo.py:151, :381)
      const double v = ((excl[i >> 5] >> (i & 31)) & 1u) ? __builtin_inf() : y[i];
      if (sel_better(v, i, bv, bi)) {
        bv = v;
        bi = i;
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const double ov = __shfl_down(bv, off);
      const int64_t oi = (int64_t)__shfl_down((long long)bi, off);
      if (sel_better(ov, oi, bv, bi)) {
        bv = ov;
        bi = oi;
      }
    }
    if (lane == 0) {
      sv[wave] = bv;
      si[wave] = bi;
    }
    __syncthreads();
    if (tid == 0) {
      for (int w = 1; w < nw; ++w)
        if (sel_better(sv[w], si[w], bv, bi)) {
          bv = sv[w];
          bi = si[w];
        }
      idx_out[b] = bi;
      if (bi >= 0) excl[bi >> 5] |= 1u << (bi & 31);
    }
    __syncthreads();
  }
}

// Sorted path (N ≤ kSelectSortN): sample b's pick is the first entry of its row in np.argmin order
// that no earlier sample took, and at most b entries are taken, so the first min(B, N) entries of
// every row in that order decide all picks.
//   select_sort_kernel    one workgroup per sample: the row as (key, index) pairs in LDS, bitonic sort,
//                         the head written out (index, bit 62 set when the value is +inf);
//   select_greedy_kernel  one wave walks the samples in order over the heads with an LDS bitmap of
//                         taken candidates (a ballot per 64 entries).
// key: NaN → 0 (np.argmin returns the first NaN), else the order-preserving map of the IEEE bits
// (−0 folded onto +0, which compare equal); ties resolve by index.  A taken candidate reads as +inf
// (turbo.py:151, :381): when the first free entry is +inf, the pick is the lowest index among it and
// the taken ones.
constexpr int kSelThreads = 1024;
constexpr unsigned long long kSelKeyInf = 0xFFF0000000000000ull;
constexpr long long kSelInfFlag = 1ll << 62;

__device__ __forceinline__ unsigned long long sel_key(double v) {
  if (v != v) return 0ull;
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v + 0.0);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

__global__ __launch_bounds__(kSelThreads) void select_sort_kernel(const double* __restrict__ Y, int64_t N, int N2,
                                                                  int K, long long* __restrict__ heads) {
  __shared__ unsigned long long key[kSelectSortN];
  __shared__ unsigned short ix[kSelectSortN];
  const int b = blockIdx.x, tid = threadIdx.x;
  const double* y = Y + (int64_t)b * N;
  for (int i = tid; i < N2; i += kSelThreads) {
    key[i] = i < N ? sel_key(y[i]) : ~0ull;
    ix[i] = (unsigned short)i;
  }
  __syncthreads();
  for (int k = 2; k <= N2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int t = tid; t < (N2 >> 1); t += kSelThreads) {
        // t-th compare-exchange of this stage: i has bit j clear, partner i + j
        const int i = ((t & ~(j - 1)) << 1) | (t & (j - 1));
        const int p = i + j;
        const unsigned long long ki = key[i], kp = key[p];
        const unsigned short xi = ix[i], xp = ix[p];
        const bool gt = ki > kp || (ki == kp && xi > xp);
        if (((i & k) == 0) == gt) {
          key[i] = kp;
          key[p] = ki;
          ix[i] = xp;
          ix[p] = xi;
        }
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < K; i += kSelThreads)
    heads[(int64_t)b * K + i] = (long long)ix[i] | (key[i] == kSelKeyInf ? kSelInfFlag : 0ll);
}

// The same heads for K ≤ 64 without the full sort (round 3): a radix select finds the K-th smallest key T
// (8 passes of 8 bits over an LDS histogram), the entries below T and the lowest-index ties at T are gathered
// (K of them), and one wave bitonic-sorts those K (key, index) pairs in registers.  The bitonic sort of the
// whole row spent 78 barrier-separated LDS stages on 4,096 slots to keep 64 (config 6: 50 µs per step,
// profiles/r03_v23_c6_kernel_per_step.txt).  Rows are read with E = ⌈N/1024⌉ consecutive entries per thread,
// so a block scan over threads numbers the ties in index order.
constexpr int kSelTopK = 64;
__global__ __launch_bounds__(kSelThreads) void select_topk_kernel(const double* __restrict__ Y, int64_t N, int K,
                                                                  long long* __restrict__ heads) {
  constexpr int kE = kSelectSortN / kSelThreads;
  __shared__ unsigned hist[256];
  __shared__ unsigned long long s_prefix;
  __shared__ unsigned s_rank, s_less;
  __shared__ int s_done;
  __shared__ unsigned wsum[kSelThreads / 64];
  __shared__ unsigned s_slot;
  __shared__ unsigned long long sk[kSelTopK];
  __shared__ unsigned short si[kSelTopK];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const double* y = Y + (int64_t)b * N;
  const int E = (int)((N + kSelThreads - 1) / kSelThreads);
  unsigned long long key[kE];
#pragma unroll
  for (int e = 0; e < kE; ++e) {
    const int64_t i = (int64_t)tid * E + e;
    key[e] = (e < E && i < N) ? sel_key(y[i]) : ~0ull;
  }
  if (tid == 0) {
    s_prefix = 0ull;
    s_rank = (unsigned)K;            // 1-based rank of T among the keys matching the prefix
    s_less = 0u;
    s_done = -1;
  }
  // ---- radix select of T = the K-th smallest key, most significant byte first.  Round 5: a pass whose chosen bin
  // is needed whole (its count equals the rank still to take) ends the search — the K smallest keys are then the
  // keys whose bits from `shift` up are ≤ the prefix's, with no tie at the boundary (equal keys share every bin), so
  // the heads are the same; random draws get there in 2-3 of the 8 passes.
  for (int shift = 56; shift >= 0; shift -= 8) {
    for (int i = tid; i < 256; i += kSelThreads) hist[i] = 0u;
    __syncthreads();
    const unsigned long long prefix = s_prefix;
    const unsigned long long hmask = shift == 56 ? 0ull : (~0ull << (shift + 8));
#pragma unroll
    for (int e = 0; e < kE; ++e)
      if (e < E && (int64_t)tid * E + e < N && (key[e] & hmask) == prefix)
        atomicAdd(&hist[(key[e] >> shift) & 255u], 1u);
    __syncthreads();
    if (wave == 0) {
      // inclusive scan of the 256 bins, 4 per lane; the first bin whose running count reaches the rank
      unsigned c[4], run = 0u;
#pragma unroll
      for (int q = 0; q < 4; ++q) c[q] = hist[4 * lane + q];
      const unsigned tot = c[0] + c[1] + c[2] + c[3];
      unsigned incl = tot;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
      }
      run = incl - tot;                                     // count before this lane's first bin
      const unsigned rank = s_rank;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (run < rank && run + c[q] >= rank) {             // exactly one (lane, q) satisfies this
          s_prefix = prefix | ((unsigned long long)(4 * lane + q) << shift);
          s_rank = rank - run;
          s_less += run;
          if (run + c[q] == rank) s_done = shift;
        }
        run += c[q];
      }
    }
    __syncthreads();
    if (s_done >= 0) break;
  }
  const unsigned long long T = s_prefix;
  if (s_done > 0) {
    // the whole bin: every key whose bits from s_done up are ≤ T's (K of them, slot order arbitrary)
    const int sd = s_done;
    if (tid == 0) s_slot = 0u;
    __syncthreads();
#pragma unroll
    for (int e = 0; e < kE; ++e) {
      const int64_t i = (int64_t)tid * E + e;
      if (e < E && i < N && (key[e] >> sd) <= (T >> sd)) {
        const unsigned slot = atomicAdd(&s_slot, 1u);
        sk[slot] = key[e];
        si[slot] = (unsigned short)i;
      }
    }
    __syncthreads();
  } else {
  const unsigned need_ties = (unsigned)K - s_less;         // ties at T to take, lowest indices first
  // ---- number the ties at T in index order (block scan of per-thread counts)
  unsigned nt = 0u;
#pragma unroll
  for (int e = 0; e < kE; ++e) nt += (e < E && key[e] == T) ? 1u : 0u;
  unsigned incl = nt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned v = __shfl_up(incl, o);
    if (lane >= o) incl += v;
  }
  if (lane == 63) wsum[wave] = incl;
  if (tid == 0) s_slot = 0u;
  __syncthreads();
  unsigned before = incl - nt;
  for (int w = 0; w < wave; ++w) before += wsum[w];
  // ---- gather the K selected entries (slot order arbitrary)
#pragma unroll
  for (int e = 0; e < kE; ++e) {
    const int64_t i = (int64_t)tid * E + e;
    if (e >= E || i >= N) continue;
    bool take = key[e] < T;
    if (key[e] == T) {
      take = before < need_ties;
      ++before;
    }
    if (take) {
      const unsigned slot = atomicAdd(&s_slot, 1u);
      sk[slot] = key[e];
      si[slot] = (unsigned short)i;
    }
  }
  __syncthreads();
  }
  // ---- one wave sorts the K pairs by (key, index); slots past K hold +max sentinels
  if (wave == 0) {
    unsigned long long kk = lane < K ? sk[lane] : ~0ull;
    unsigned ii = lane < K ? si[lane] : 0xFFFFu;
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
      for (int j = k >> 1; j > 0; j >>= 1) {
        const unsigned long long ko = __shfl_xor(kk, j);
        const unsigned io = __shfl_xor(ii, j);
        const bool mine_gt = kk > ko || (kk == ko && ii > io);
        const bool lower = (lane & j) == 0, up = (lane & k) == 0;
        if ((lower == up) == mine_gt) {                     // keep the smaller at the lower slot when ascending
          kk = ko;
          ii = io;
        }
      }
    }
    if (lane < K) heads[(int64_t)b * K + lane] = (long long)ii | (kk == kSelKeyInf ? kSelInfFlag : 0ll);
  }
}

constexpr int kSelHeadLds = 4096;   // staged head entries (64 per sample, samples 0..63)
__global__ __launch_bounds__(256) void select_greedy_kernel(const long long* __restrict__ heads, int B, int64_t N,
                                                            int K, int64_t* __restrict__ idx_out) {
  __shared__ unsigned taken[kSelectSortN / 32];
  __shared__ long long hl[kSelHeadLds];
  const int tid = threadIdx.x, lane = tid & 63;
  const int H = K < 64 ? K : 64;                      // staged entries per sample
  const int Bs = B < kSelHeadLds / 64 ? B : kSelHeadLds / 64;
  for (int w = tid; w < kSelectSortN / 32; w += 256) taken[w] = 0u;
  for (int i = tid; i < Bs * H; i += 256) hl[i] = heads[(int64_t)(i / H) * K + i % H];
  __syncthreads();
  if (tid >= 64) return;
  long long min_taken = N;
  for (int b = 0; b < B; ++b) {
    long long pick = -1;
    for (int c0 = 0; c0 < K && pick < 0; c0 += 64) {
      long long e = -1;
      if (c0 + lane < K) e = (c0 == 0 && b < Bs) ? hl[b * H + lane] : heads[(int64_t)b * K + c0 + lane];
      const long long i = e >= 0 ? (e & (kSelInfFlag - 1)) : 0;
      const bool free_ = e >= 0 && !((taken[i >> 5] >> (i & 31)) & 1u);
      const unsigned long long m = __ballot(free_);
      if (m) {
        const int f = __builtin_ctzll(m);
        const long long ef = __shfl(e, f);
        const long long fi = ef & (kSelInfFlag - 1);
        pick = (ef & kSelInfFlag) ? (fi < min_taken ? fi : min_taken) : fi;
      }
    }
    if (pick < 0) pick = min_taken;   // every candidate taken: all read +inf, the lowest index wins
    if (lane == 0) {
      idx_out[b] = pick;
      taken[pick >> 5] |= 1u << (pick & 31);
    }
    min_taken = pick < min_taken ? pick : min_taken;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// The same picks for B ≤ 64 in rounds (round 5), one lane per sample.  Sample b's pick depends only on the picks of
// the samples below it, so the sequential picks are the unique fixed point of
//     pick_b ← the first head entry of b that no sample below b holds (the +inf rule as above, min_taken = the lowest
//              pick below b; every entry held: min_taken),
// and each round applies it to every sample at once against the previous round's picks (owner[i] = the lowest sample
// whose pick is i).  A prefix stays final: with all samples below F final, sample F's new pick is final, and so is
// every sample up to the first one ≥ F whose pick changed in the round (c): F → c + 1; a round that changes no pick
// ends it (F = B).  Samples rarely share their minima, so that takes two or three rounds (≈ 1 µs, against ≈ 22 µs for
// 64 sequential steps).  After kGreedyRounds rounds (long conflict chains: a collapsed posterior whose samples order
// the candidates alike) the samples from F on are picked by the sequential walk, against the final picks below F.
constexpr int kGreedyHeadRegs = 4;      // head entries per sample kept in registers (later ones read from `heads`)
constexpr int kGreedyRounds = 8;
__global__ __launch_bounds__(64) void select_greedy_par_kernel(const long long* __restrict__ heads, int B, int64_t N,
                                                               int K, int64_t* __restrict__ idx_out) {
  __shared__ int owner[kSelectSortN];
  __shared__ long long hl[kSelHeadLds];
  const int lane = threadIdx.x;
  const bool act = lane < B;
  for (int i = lane; i < N; i += 64) owner[i] = 0x7fffffff;
  long long h[kGreedyHeadRegs];
#pragma unroll
  for (int j = 0; j < kGreedyHeadRegs; ++j) h[j] = (act && j < K) ? heads[(int64_t)lane * K + j] : -1;
  auto lds_order = [] {
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  lds_order();
  long long pick = -1;
  int F = 0;
  for (int round = 0; round < kGreedyRounds && F < B; ++round) {
    // the lowest pick below each sample (N: none), an exclusive prefix min over the lanes
    long long m = (act && pick >= 0) ? pick : N;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const long long t = __shfl_up(m, o);
      if (lane >= o) m = t < m ? t : m;
    }
    long long below = __shfl_up(m, 1);
    if (lane == 0) below = N;
    long long np = pick;
    if (act && lane >= F) {
      np = -1;
      for (int j = 0; j < K; ++j) {
        const long long e = j == 0 ? h[0] : j == 1 ? h[1] : j == 2 ? h[2] : j == 3 ? h[3] : heads[(int64_t)lane * K + j];
        if (e < 0) break;
        const long long i = e & (kSelInfFlag - 1);
        if (owner[i] < lane) continue;                      // held by a lower sample
        np = (e & kSelInfFlag) ? (i < below ? i : below) : i;
        break;
      }
      if (np < 0) np = below;
    }
    const unsigned long long changed = __ballot(act && np != pick) & (~0ull << F);
    const int c = changed ? __builtin_ctzll(changed) : B;
    const int Fn = c >= B ? B : c + 1;
    // owner ← the new picks: every old pick reset, then every new one min-ed in
    if (act && pick >= 0) owner[pick] = 0x7fffffff;
    lds_order();
    if (act) atomicMin(&owner[np], lane);
    lds_order();
    pick = np;
    F = Fn;
  }
  if (F < B) {
    // the sequential walk from F (select_greedy_kernel's loop) against the final picks below F
    if (act && lane >= F) owner[pick] = 0x7fffffff;
    lds_order();
    if (act && lane < F) atomicMin(&owner[pick], lane);
    const int H = K < 64 ? K : 64;
    for (int i = lane; i < (B - F) * H; i += 64) hl[i] = heads[(int64_t)(F + i / H) * K + i % H];
    long long m = (act && lane < F) ? pick : N;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const long long t = __shfl_xor(m, o);
      m = t < m ? t : m;
    }
    long long min_taken = m;
    lds_order();
    for (int b = F; b < B; ++b) {
      long long p = -1;
      for (int c0 = 0; c0 < K && p < 0; c0 += 64) {
        long long e = -1;
        if (c0 + lane < K) e = c0 == 0 ? hl[(b - F) * H + lane] : heads[(int64_t)b * K + c0 + lane];
        const long long i = e >= 0 ? (e & (kSelInfFlag - 1)) : 0;
        const bool free_ = e >= 0 && owner[i] == 0x7fffffff;
        const unsigned long long msk = __ballot(free_);
        if (msk) {
          const int f = __builtin_ctzll(msk);
          const long long ef = __shfl(e, f);
          const long long fi = ef & (kSelInfFlag - 1);
          p = (ef & kSelInfFlag) ? (fi < min_taken ? fi : min_taken) : fi;
        }
      }
      if (p < 0) p = min_taken;
      if (lane == 0) owner[p] = b;
      if (lane == b) pick = p;
      min_taken = p < min_taken ? p : min_taken;
      lds_order();
    }
  }
  if (act) idx_out[lane] = pick;
}

// ----------------------------------------------------------------------------- launchers
int64_t cand_cov_ws_doubles(int64_t N, int DP) { return N * ((DP + 3) / 4 * 4) + N; }

hipError_t launch_cand_cov(hipStream_t stream, const GPDev& g, int d, int DP, const double* Xc, int64_t N, double* S,
                           int64_t lds, double* ws, double diag_add, bool table) {
  if (N <= 0) return hipSuccess;
  if (DP > kMaxFusedDP) return launch_cand_cov_wide(stream, g, d, DP, Xc, N, S, lds, ws, diag_add);
  const ExpCoef ec = exp_coef();
  const int KP = (DP + 3) / 4 * 4;
  double* Xs = ws;
  double* xsq = ws + N * KP;
  const unsigned sb = (unsigned)((N * KP + 255) / 256);
  const unsigned nt = (unsigned)((N + 63) / 64);
  dim3 grid(nt, nt);
#define OMB_COV(DPV)                                                                                          \
  case DPV:                                                                                                   \
    hipLaunchKernelGGL((cand_scale_kernel<DPV>), dim3(sb), dim3(256), 0, stream, Xc, d, N, g.ls, Xs, xsq);    \
    if (g.kind == OMB_KERNEL_RBF)                                                                             \
      hipLaunchKernelGGL((cand_cov_kernel<DPV, OMB_KERNEL_RBF, false>), grid, dim3(256), 0, stream, Xs, xsq, N, \
                         g.variance, S, lds, diag_add, ec);                                                   \
    else if (table)                                                                                           \
      hipLaunchKernelGGL((cand_cov_kernel<DPV, OMB_KERNEL_MATERN52, true>), grid, dim3(256), 0, stream, Xs, xsq,  \
                         N, g.variance, S, lds, diag_add, ec);                                                \
    else                                                                                                      \
      hipLaunchKernelGGL((cand_cov_kernel<DPV, OMB_KERNEL_MATERN52, false>), grid, dim3(256), 0, stream, Xs, xsq, \
                         N, g.variance, S, lds, diag_add, ec);                                                \
    break;
  switch (DP) {
    OMB_COV(2) OMB_COV(4) OMB_COV(6) OMB_COV(8) OMB_COV(16) OMB_COV(32) OMB_COV(64)
    default: return hipErrorInvalidValue;
  }
#undef OMB_COV
  return hipGetLastError();
}

int launch_cand_scale(hipStream_t stream, const GPDev& g, int d, int DP, const double* Xc, int64_t N, double* ws,
                      hipError_t* err) {
  *err = hipSuccess;
  if (N <= 0 || DP > kMaxFusedDP) return 0;
  const int KP = (DP + 3) / 4 * 4;
  const unsigned sb = (unsigned)((N * KP + 255) / 256);
  switch (DP) {
#define OMB_CS(DPV)                                                                                               \
  case DPV:                                                                                                       \
    hipLaunchKernelGGL((cand_scale_kernel<DPV>), dim3(sb), dim3(256), 0, stream, Xc, d, N, g.ls, ws, ws + N * KP); \
    break;
    OMB_CS(2) OMB_CS(4) OMB_CS(6) OMB_CS(8) OMB_CS(16) OMB_CS(32) OMB_CS(64)
#undef OMB_CS
    default:
      return 0;
  }
  *err = hipGetLastError();
  return KP;
}

hipError_t launch_mirror_lower(hipStream_t stream, double* S, int64_t N, int64_t lds) {
  const unsigned nt = (unsigned)((N + 31) / 32);
  hipLaunchKernelGGL(mirror_lower_kernel, dim3(nt, nt), dim3(256), 0, stream, S, N, lds);
  return hipGetLastError();
}

hipError_t launch_add_diag(hipStream_t stream, double* S, int64_t N, int64_t lds, double v) {
  if (v == 0.0 || N <= 0) return hipSuccess;
  hipLaunchKernelGGL(add_diag_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, stream, S, N, lds, v);
  return hipGetLastError();
}

int64_t chol_ws_doubles(int64_t N) {
  const int64_t steps = (N + kNB - 1) / kNB;
  const int64_t launches = (int64_t)kCholWsDoubles + (steps + 1) / 2 + 2;     // W fragments | one int flag per step
  // chol_persist_kernel: W fragments of every step | wflag[t] | pflag[t·t] | cnt[t·t] | ticket | abort
  const int64_t persist = steps * kCholWsDoubles + (steps + 2 * steps * steps + 2 + 1) / 2 + 2;
  return launches > persist ? launches : persist;
}

// The persistent launch's sync words inside ws (chol_persist_kernel's layout; all zero before a k0 = 0 launch, which
// chol_persist_init_kernel or, in the Thompson chain, the covariance SYRK writes)
int chol_persist_sync_words(double* ws, int64_t N, int** ints) {
  const int t = (int)((N + kNB - 1) / kNB);
  *ints = reinterpret_cast<int*>(ws + (int64_t)t * kCholWsDoubles);
  return t + 2 * t * t + 2;
}

struct CholPersistInit {
  int* ints = nullptr;   // the persistent launch's sync words (nullptr: none to write)
  int t = 0, k0 = 0;
};
static hipError_t chol_panel(hipStream_t stream, double* A, int64_t N, int64_t lda, int k, const double* ws,
                             const int* info, bool vec, CholPersistInit pi = {}) {
  const int64_t rest = N - (int64_t)(k + 1) * kNB;          // rows below the diagonal block
  const unsigned pblocks = (unsigned)((rest + 15) / 16);
  if (vec)
    hipLaunchKernelGGL((chol_panel_kernel<true>), dim3(pblocks), dim3(128), 0, stream, A, N, lda, k, ws, info, pi.ints,
                       pi.t, pi.k0);
  else
    hipLaunchKernelGGL((chol_panel_kernel<false>), dim3(pblocks), dim3(128), 0, stream, A, N, lda, k, ws, info, pi.ints,
                       pi.t, pi.k0);
  return hipGetLastError();
}

// Dynamic LDS added to every chol_update_kernel workgroup: it caps the workgroups per CU.  A knob of
// tools/ablate/ablate_chol only (built with OMB_TOOLS_KNOBS); the library launches with none.
#ifdef OMB_TOOLS_KNOBS
static size_t g_chol_update_lds = 0;
void set_chol_update_lds(size_t bytes) { g_chol_update_lds = bytes; }
static int g_chol_update_delay = 0;
void set_chol_update_delay(int n) { g_chol_update_delay = n; }
#else
constexpr size_t g_chol_update_lds = 0;
constexpr int g_chol_update_delay = 0;
#endif

// Round 4: the diagonal blocks by tiles of 16 (chol64_blocked), one launch per step with the next panel inside.
static hipError_t launch_cholesky_blocked(hipStream_t stream, double* A, int64_t N, int64_t lda, int* info, double* ws,
                                          int spin_limit, int acq_rel, int steps_limit, CholPersistInit pi) {
  int steps = (int)((N + kNB - 1) / kNB);
  // steps_limit k0 ≥ 1: only the launches that factor blocks 0 .. k0 and form panel columns 0 .. k0
  if (steps_limit > 0 && steps_limit + 1 < steps) steps = steps_limit + 1;
  const bool vec = (lda % 2 == 0) && ((reinterpret_cast<uintptr_t>(A) & 15) == 0);
  int* flags = reinterpret_cast<int*>(ws + kCholWsDoubles);
  hipLaunchKernelGGL(chol_diag_blk_kernel, dim3(1), dim3(256), 0, stream, A, N, lda, ws, info, flags, steps);
  hipError_t e = hipGetLastError();
  for (int k = 0; k + 1 < steps && e == hipSuccess; ++k) {
    const int64_t rest = N - (int64_t)(k + 1) * kNB;
    const int t = (int)((rest + kGT - 1) / kGT);
    if (k == 0) {
      e = chol_panel(stream, A, N, lda, k, ws, info, vec, pi);
      if (e != hipSuccess) break;
    }
    hipLaunchKernelGGL((chol_update_kernel<true, true>), dim3((unsigned)(t * (t + 1) / 2)), dim3(256), g_chol_update_lds,
                       stream, A, N, lda, k, t, ws, info, flags, spin_limit, acq_rel, g_chol_update_delay);
    e = hipGetLastError();
  }
  return e;
}

// Per-step launches before the persistent one (k0, launch_cholesky_persist); tools/ablate sets it, the library
// picks it from the number of 64-column steps t.
#ifdef OMB_TOOLS_KNOBS
static int g_chol_hybrid_k0 = -1;
void set_chol_hybrid_k0(int k0) { g_chol_hybrid_k0 = k0; }
#else
constexpr int g_chol_hybrid_k0 = -1;
#endif
// Rounds 4-5: the persistent launch's trailing updates kept up with the walk only once ≤ ≈ 32 block columns remained,
// so the first t − 32 steps ran as per-step launches (three workgroups per CU, LDS-staged).  Round 6: with the far
// tiles' updates batched (chol_task_table) the persistent launch alone is the fastest schedule at every size measured
// (GPU time, tools/ablate/chol_hybrid_sweep): N = 3000 0.910 ms (round 5's hybrid 0.98, per-step 1.10), 5000 2.358
// (2.48, 2.56), 6500 4.55-4.69 for every k0 (per-step 4.68), 8000 7.38 (k0 = 16 … 93: 7.75-7.89, per-step 7.90;
// profiles/r06_d_chol_sweep.txt, r06_e_chol_sweep.txt, r06_f_chol_sweep_large_n.txt).  The per-step prefix stays
// available to the tools (k0 > 0).
static int chol_hybrid_k0(int t) {
  (void)t;
  return g_chol_hybrid_k0 >= 0 ? g_chol_hybrid_k0 : 0;
}

// Round 4: one persistent launch (chol_persist_kernel), kPersistWgPerCu workgroups per CU.
static int device_cus() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cus[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cus[dev] = n;
  }
  return cus[dev];
}

static bool chol_persist_fits(int64_t N, int64_t lda) {
  return ((N + kNB) * lda + kNB) * 8 < 0x7fffffff;   // 32-bit buffer offsets (rows past N included)
}

static hipError_t launch_cholesky_blocked(hipStream_t stream, double* A, int64_t N, int64_t lda, int* info, double* ws,
                                          int spin_limit, int acq_rel, int steps_limit = -1, CholPersistInit pi = {});

// Round 5: the persistent launch's task order.  Step-major tickets put step k's critical tasks (its panel tiles, the
// next column's updates) behind every far-column update of step k − 1, and the diagonal walk waited for them.  Here
// the host sorts the tasks by
//     P(i, k): (k + 1, k, 0, ·, i)        U(i, j, k): (min(j, k + L), k, 1, j, i)
// — step k's update of column j no later than "step" k + L, the near columns by their deadline j (the step whose
// panel needs them).  Every task's inputs (U(i, j, k − 1), P(i, k), P(j, k); P(i, k)'s U(i, k, k − 1)) sort before
// it, and everything the walk waits for at step k (tiles (k + 1, k), (k + 1, k + 1) through step k − 1) sorts before
// every task that needs W_k, so the order stays topological and the grid needs no co-residency.  The table (per task
// the code — panel flag, k, i, j in 10-bit fields — and its number of steps) is built once per (device, t, k0, L,
// batch, window) and kept.
#ifdef OMB_TOOLS_KNOBS
static int g_chol_lookahead = -1;
void set_chol_lookahead(int L) { g_chol_lookahead = L; }
#else
constexpr int g_chol_lookahead = -1;
#endif
// Round 6 (with the batched far updates below): L = 2 — N = 3000 0.910 against 0.920 ms at L = 3, N = 5000 2.358 against
// 2.403 ms (tools/ablate/chol_hybrid_sweep, profiles/r06_e_chol_sweep.txt)
constexpr int kCholLookahead = 2;

// Round 6: far tiles take their updates in batches (chol_persist_update_batch).  Tile (i, j)'s worker steps are
// [k0, e) — e = j below the diagonal, i − 1 on it (the walker applies step i − 1 to its own D); the last `window`
// steps before e (the ones the walk is about to need) stay single tasks, the earlier ones go in batches of up to
// `batch` steps aligned to multiples of `batch`.  A batch [ka, kb) sorts as its last step's update would,
// (min(j, kb − 1 + L), kb − 1, 1, j, i): its inputs — the panels of its steps, the tile's previous batch — still sort
// before it, and a tile the walk waits for at step k (its last worker step k − 1, inside the window) is a single
// task sorting before every task that needs W_k, so the order stays topological.  The entries are pairs (code,
// steps); batch 1 is round 5's table.
#ifdef OMB_TOOLS_KNOBS
static int g_chol_batch = -1, g_chol_window = -1;
void set_chol_batch(int batch, int window) {
  g_chol_batch = batch;
  g_chol_window = window;
}
#else
constexpr int g_chol_batch = -1, g_chol_window = -1;
#endif
// batch 16, window 4: N = 3000 0.910 ms (1 / 0: 1.045; 8 / 4: 0.932; 32 / 4: 1.011; 16 / 2: 0.979), N = 5000 2.358 ms
// (profiles/r06_d_chol_sweep.txt, r06_e_chol_sweep.txt)
constexpr int kCholBatch = 16;
constexpr int kCholWindow = 4;

struct CholTaskTab {
  int dev, t, k0, L, batch, window, total;
  int* d;
};

static const int* chol_task_table(int t, int k0, int L, int batch, int window, int* total_out) {
  static std::mutex mu;
  static std::vector<CholTaskTab> tabs;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || t > 1024 || batch < 1 || batch > 32) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  for (const CholTaskTab& e : tabs)
    if (e.dev == dev && e.t == t && e.k0 == k0 && e.L == L && e.batch == batch && e.window == window) {
      *total_out = e.total;
      return e.d;
    }
  struct Key {
    int a, b, c, d, e, code, steps;
  };
  std::vector<Key> keys;
  for (int k = k0; k < t; ++k)
    if (!(k0 > 0 && k == k0))
      for (int i = k + 2; i < t; ++i) keys.push_back({k + 1, k, 0, 0, i, (k << 20) | (i << 10), 1});
  auto add_update = [&](int i, int j, int ka, int kb) {   // steps [ka, kb) of tile (i, j)
    const int kl = kb - 1;
    keys.push_back({std::min(j, kl + L), kl, 1, j, i, (1 << 30) | (ka << 20) | (i << 10) | j, kb - ka});
  };
  for (int j = k0 + 1; j < t; ++j)
    for (int i = j; i < t; ++i) {
      const int e = (i == j) ? i - 1 : j;                     // worker steps [k0, e)
      const int near = std::max(k0, e - window);
      for (int ka = k0; ka < near;) {                         // batches, aligned to multiples of `batch`
        const int kb = std::min(near, (ka / batch + 1) * batch);
        add_update(i, j, ka, kb);
        ka = kb;
      }
      for (int k = near; k < e; ++k) add_update(i, j, k, k + 1);
    }
  std::sort(keys.begin(), keys.end(), [](const Key& x, const Key& y) {
    if (x.a != y.a) return x.a < y.a;
    if (x.b != y.b) return x.b < y.b;
    if (x.c != y.c) return x.c < y.c;
    if (x.d != y.d) return x.d < y.d;
    return x.e < y.e;
  });
  const int total = (int)keys.size();
  std::vector<int> codes(2 * (size_t)total);
  for (int q = 0; q < total; ++q) {
    codes[2 * q] = keys[q].code;
    codes[2 * q + 1] = keys[q].steps;
  }
  int* d = nullptr;
  if (hipMalloc(&d, sizeof(int) * (size_t)std::max(2 * total, 1)) != hipSuccess) return nullptr;
  if (hipMemcpy(d, codes.data(), sizeof(int) * 2 * (size_t)total, hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(d);
    return nullptr;
  }
  tabs.push_back({dev, t, k0, L, batch, window, total, d});
  *total_out = total;
  return d;
}

// k0 > 0: steps 0 .. k0 − 1 as per-step launches (their bulk trailing updates run at three workgroups per CU), the
// rest in one persistent launch (the diagonal walk without kernel boundaries once the trailing matrix is small).
static hipError_t launch_cholesky_persist(hipStream_t stream, double* A, int64_t N, int64_t lda, int* info, double* ws,
                                          int spin_limit, int k0 = 0, int acq_rel = 0, int single_steps = 0,
                                          bool sync_zeroed = false) {
  const int t = (int)((N + kNB - 1) / kNB);
  if (k0 > t - 2) k0 = 0;
  hipError_t e = hipSuccess;
  double* Wf = ws;
  int* ints = reinterpret_cast<int*>(ws + (int64_t)t * kCholWsDoubles);
  if (k0 > 0) e = launch_cholesky_blocked(stream, A, N, lda, info, ws, spin_limit, acq_rel, k0, CholPersistInit{ints, t, k0});
  if (e != hipSuccess) return e;
  int total = 0;
  for (int k = k0; k < t; ++k) total += chol_persist_step_tasks(t, k, k0);
  const int L = g_chol_lookahead >= 0 ? g_chol_lookahead : kCholLookahead;
  const int batch = single_steps ? 1 : (g_chol_batch >= 1 ? g_chol_batch : kCholBatch);
  const int window = g_chol_window >= 0 ? g_chol_window : kCholWindow;
  // L = 0 (tools): the step-major arithmetic order of round 4 (single-step tasks)
  int tab_total = 0;
  const int* tab = L > 0 ? chol_task_table(t, k0, L, batch, window, &tab_total) : nullptr;
  if (tab) total = tab_total;
  CholSync sync{ints, ints + t, ints + t + t * t, ints + t + 2 * t * t, ints + t + 2 * t * t + 1, tab};
  if (k0 == 0 && !sync_zeroed) {   // with k0 > 0 step 0's panel launch wrote the sync words
    hipLaunchKernelGGL(chol_persist_init_kernel, dim3(1), dim3(256), 0, stream, ints, t, k0, info);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  const int slots = kPersistWgPerCu * device_cus() - 1;
  const int grid = 1 + (total < slots ? total : slots);
  if (acq_rel)
    hipLaunchKernelGGL(chol_persist_kernel<true>, dim3((unsigned)grid), dim3(256), 0, stream, A, N, lda, t, total, Wf,
                       sync, info, spin_limit, k0);
  else
    hipLaunchKernelGGL(chol_persist_kernel<false>, dim3((unsigned)grid), dim3(256), 0, stream, A, N, lda, t, total, Wf,
                       sync, info, spin_limit, k0);
  return hipGetLastError();
}

hipError_t launch_cholesky_mode(hipStream_t stream, double* A, int64_t N, int64_t lda, int* info, double* ws, int mode,
                                int spin_limit, int acq_rel, int single_steps, bool sync_zeroed) {
  if (N <= 0) return hipSuccess;
  if (mode == kCholAuto) mode = kCholPersistent;
  if (mode == kCholPersistOnly) {
    if (chol_persist_fits(N, lda))
      return launch_cholesky_persist(stream, A, N, lda, info, ws, spin_limit, 0, acq_rel, single_steps, sync_zeroed);
    mode = kCholBlocked;
  }
  if (mode == kCholPersistent) {
    if (chol_persist_fits(N, lda))
      return launch_cholesky_persist(stream, A, N, lda, info, ws, spin_limit, chol_hybrid_k0((int)((N + kNB - 1) / kNB)),
                                     acq_rel, single_steps, sync_zeroed);
    mode = kCholBlocked;
  }
  if (acq_rel && mode == kCholBlocked) mode = kCholBlockedAcqRel;
  const int steps = (int)((N + kNB - 1) / kNB);
  const bool vec = (lda % 2 == 0) && ((reinterpret_cast<uintptr_t>(A) & 15) == 0);
  const bool fuse = mode == kCholFused;
  const bool blk = mode == kCholBlocked || mode == kCholBlockedAcqRel;
  if (blk) return launch_cholesky_blocked(stream, A, N, lda, info, ws, spin_limit, mode == kCholBlockedAcqRel ? 1 : 0);
  int* flags = reinterpret_cast<int*>(ws + kCholWsDoubles);
  hipLaunchKernelGGL(chol_diag_kernel, dim3(1), dim3(256), 0, stream, A, N, lda, ws, info, flags, fuse ? steps : 0);
  hipError_t e = hipGetLastError();
  for (int k = 0; k + 1 < steps && e == hipSuccess; ++k) {
    const int64_t rest = N - (int64_t)(k + 1) * kNB;
    const int t = (int)((rest + kGT - 1) / kGT);
    // fused: step k's panel came from step k−1's update launch (step 0's from its own launch)
    if (!fuse || k == 0) {
      e = chol_panel(stream, A, N, lda, k, ws, info, vec);
      if (e != hipSuccess) break;
    }
    const unsigned wgs = (unsigned)(t * (t + 1) / 2);
    if (fuse)
      hipLaunchKernelGGL((chol_update_kernel<true, false>), dim3(wgs), dim3(256), g_chol_update_lds, stream, A, N, lda, k,
                         t, ws, info, flags, spin_limit, 0, 0);
    else
      hipLaunchKernelGGL((chol_update_kernel<false, false>), dim3(wgs), dim3(256), g_chol_update_lds, stream, A, N, lda,
                         k, t, ws, info, flags, spin_limit, 0, 0);
    e = hipGetLastError();
  }
  return e;
}

hipError_t launch_cholesky(hipStream_t stream, double* A, int64_t N, int64_t lda, int* info, double* ws, int spin_limit) {
  return launch_cholesky_mode(stream, A, N, lda, info, ws, kCholAuto, spin_limit);
}

hipError_t launch_trinv(hipStream_t stream, const double* L, int64_t n, int64_t lda, double* X, int64_t ldx,
                        double* T) {
  const int64_t nbk = (n + kNB - 1) / kNB;
  hipLaunchKernelGGL(trinv_diag_kernel, dim3((unsigned)nbk), dim3(64), 0, stream, L, n, lda, X, ldx);
  hipError_t e = hipGetLastError();
  for (int64_t i = 1; i < nbk && e == hipSuccess; ++i) {
    const int64_t r0 = i * kNB, rows = (n - r0) < kNB ? (n - r0) : kNB;
    // T (rows, r0) = L[r0:, :r0] · X[:r0, :r0];  X[r0:, :r0] = −X_ii · T
    e = launch_gemm_nn(stream, rows, r0, r0, 1.0, L + r0 * lda, lda, X, ldx, 0.0, T, r0);
    if (e == hipSuccess)
      e = launch_gemm_nn(stream, rows, r0, rows, -1.0, X + r0 * ldx + r0, ldx, T, r0, 0.0, X + r0 * ldx, ldx);
  }
  return e;
}

int64_t gp_grad_blocks(int64_t n) {
  const int64_t t = (n + 15) / 16;
  return t * t;
}

hipError_t launch_gp_grad(hipStream_t stream, int kind, int DP, const double* X, int d, int64_t n, const double* ls,
                          double variance, const double* alpha, const double* Kinv, int64_t ldk, double* partials,
                          const double* L, int64_t lda, const double* y, double* out) {
  const unsigned t = (unsigned)((n + 15) / 16);
  dim3 grid(t, t);
  if (DP > kMaxFusedDP) {   // n_var > 64 (omb_wide.hip): the same partial sums, one thread per dimension
    hipError_t e = launch_gp_grad_partials_wide(stream, kind, DP, X, d, n, ls, variance, alpha, Kinv, ldk, partials);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(gp_reduce_kernel, dim3(1), dim3(256), 0, stream, partials, (int64_t)t * t, DP + 1, L, n, lda, y,
                       alpha, out);
    return hipGetLastError();
  }
#define OMB_GG(DPV)                                                                                              \
  case DPV:                                                                                                      \
    if (kind == OMB_KERNEL_RBF)                                                                                  \
      hipLaunchKernelGGL((gp_grad_kernel<DPV, OMB_KERNEL_RBF>), grid, dim3(256), 0, stream, X, d, n, ls, variance, \
                         alpha, Kinv, ldk, partials);                                                            \
    else                                                                                                         \
      hipLaunchKernelGGL((gp_grad_kernel<DPV, OMB_KERNEL_MATERN52>), grid, dim3(256), 0, stream, X, d, n, ls,      \
                         variance, alpha, Kinv, ldk, partials);                                                  \
    break;
  switch (DP) {
    OMB_GG(2) OMB_GG(4) OMB_GG(6) OMB_GG(8) OMB_GG(16) OMB_GG(32) OMB_GG(64)
    default: return hipErrorInvalidValue;
  }
#undef OMB_GG
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(gp_reduce_kernel, dim3(1), dim3(256), 0, stream, partials, (int64_t)t * t, DP + 1, L, n, lda, y,
                     alpha, out);
  return hipGetLastError();
}

// μ_c = Σ_k α_k K*_kc, σ²_c = σ_f² − Σ_k V_kc² for the columns of one candidate chunk (the dense
// posterior path, n_train > OMB_MAX_TRAIN, and the Thompson-sampling mean).  Workgroup = 64 candidates
// × 16 row slices (coalesced 512-B row segments); the slices' partial sums are added in slice order.
// One thread per candidate over all rows ran 12 workgroups at N = 3000 (142 µs,
// profiles/r02_v23_c6_kernel_stats.csv).
// μ = αᵀK*, σ² = σ_f² − ΣV² per candidate column: 16 row slices of ⌈n/16⌉ rows, each summed in row order by one thread,
// the slices' partials met in slice order.  16 columns per workgroup (lane = slice-in-wave × 16 + column: 128-B row
// segments), so N = 3000 candidates spread over 188 workgroups (round 5; 64 columns per 1,024-thread workgroup ran on
// 47 CUs) and each thread keeps 8 rows' loads in flight (one row per load latency: 12.9 µs per config-6 step, and
// 12.75 µs with the wider grid alone) — the same sums in the same order, bitwise.
constexpr int kColSlices = 16;
constexpr int kColTile = 16;
// sc (round 5, omb_posterior_samples): the launch also writes cand_scale_kernel's rows for its kColTile candidates —
// Xs[i·KP + k] = X*[i][k] / ℓ_k and ‖Xs_i‖² by the same xor tree over the KP lanes of one wave — one launch fewer.
struct ColScale {
  const double* Xc = nullptr;   // nullptr: no scaling job
  const double* ls = nullptr;
  int d = 0, KP = 0;
  double* Xs = nullptr;
  double* xsq = nullptr;
};
__global__ __launch_bounds__(kColSlices * kColTile) void post_colreduce_kernel(const double* __restrict__ Kst,
                                                                                const double* __restrict__ V, int64_t n,
                                                                                int64_t Nc, const double* __restrict__ alpha,
                                                                                double variance, double* __restrict__ mu,
                                                                                double* __restrict__ var, ColScale sc) {
  if (sc.Xc) {
    const int KP = sc.KP;
    for (int p = threadIdx.x; p < kColTile * KP; p += kColSlices * kColTile) {   // KP | 64: a candidate's lanes in one wave
      const int64_t i = (int64_t)blockIdx.x * kColTile + p / KP;
      const int k = p % KP;
      double a = 0.0;
      if (i < Nc && k < sc.d) a = sc.Xc[i * sc.d + k] / sc.ls[k];
      if (i < Nc) sc.Xs[i * KP + k] = a;
      double q = a * a;
      for (int o = KP / 2; o > 0; o >>= 1) q += __shfl_xor(q, o);
      if (i < Nc && k == 0) sc.xsq[i] = q;
    }
  }
  __shared__ double pm[kColSlices][kColTile], ps[kColSlices][kColTile];
  const int col = threadIdx.x % kColTile, sl = threadIdx.x / kColTile;
  const int64_t c = (int64_t)blockIdx.x * kColTile + col;
  const int64_t rs = (n + kColSlices - 1) / kColSlices;
  const int64_t k0 = sl * rs, k1 = (k0 + rs) < n ? (k0 + rs) : n;
  double m = 0.0, s = 0.0;
  if (c < Nc) {
    // 8 rows' loads in flight before their fmas (the sums keep row order): one memory latency per 8 rows, not per row
    constexpr int U = 8;
    int64_t k = k0;
    for (; k + U <= k1; k += U) {
      double kv[U], vv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        kv[u] = Kst[(k + u) * Nc + c];
        vv[u] = V[(k + u) * Nc + c];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        m = fma(alpha[k + u], kv[u], m);
        s = fma(vv[u], vv[u], s);
      }
    }
    for (; k < k1; ++k) {
      m = fma(alpha[k], Kst[k * Nc + c], m);
      const double v = V[k * Nc + c];
      s = fma(v, v, s);
    }
  }
  pm[sl][col] = m;
  ps[sl][col] = s;
  __syncthreads();
  if (sl == 0 && c < Nc) {
#pragma unroll
    for (int j = 1; j < kColSlices; ++j) {
      m += pm[j][col];
      s += ps[j][col];
    }
    mu[c] = m;
    var[c] = variance - s;
  }
}

hipError_t launch_post_colreduce(hipStream_t stream, const double* Kst, const double* V, int64_t n, int64_t Nc,
                                 const double* alpha, double variance, double* mu, double* var, const GPDev* scale_g,
                                 int d, int DP, const double* Xc, double* ws) {
  if (Nc <= 0) return hipSuccess;
  ColScale sc;
  if (scale_g && DP <= kMaxFusedDP) {
    sc.KP = (DP + 3) / 4 * 4;
    sc.Xc = Xc;
    sc.ls = scale_g->ls;
    sc.d = d;
    sc.Xs = ws;
    sc.xsq = ws + Nc * sc.KP;
  }
  hipLaunchKernelGGL(post_colreduce_kernel, dim3((unsigned)((Nc + kColTile - 1) / kColTile)), dim3(kColSlices * kColTile),
                     0, stream, Kst, V, n, Nc, alpha, variance, mu, var, sc);
  return hipGetLastError();
}

static bool select_sorted(int B, int64_t N) { return N <= kSelectSortN && B >= 1; }

int64_t select_ws_bytes(int B, int64_t N) {
  if (!select_sorted(B, N)) return 0;
  const int64_t K = B < N ? B : N;
  return (int64_t)B * K * (int64_t)sizeof(long long);
}

hipError_t launch_select(hipStream_t stream, const double* Y, int B, int64_t N, int64_t* idx, void* ws, bool seq) {
  if (B <= 0) return hipSuccess;
  if (select_sorted(B, N)) {
    int N2 = 2;
    while (N2 < N) N2 <<= 1;
    const int K = (int)(B < N ? B : N);
    long long* heads = static_cast<long long*>(ws);
    if (K <= kSelTopK)
      hipLaunchKernelGGL(select_topk_kernel, dim3((unsigned)B), dim3(kSelThreads), 0, stream, Y, N, K, heads);
    else
      hipLaunchKernelGGL(select_sort_kernel, dim3((unsigned)B), dim3(kSelThreads), 0, stream, Y, N, N2, K, heads);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (B <= 64 && !seq)
      hipLaunchKernelGGL(select_greedy_par_kernel, dim3(1), dim3(64), 0, stream, heads, B, N, K, idx);
    else
      hipLaunchKernelGGL(select_greedy_kernel, dim3(1), dim3(256), 0, stream, heads, B, N, K, idx);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(select_kernel, dim3(1), dim3(1024), 0, stream, Y, B, N, idx);
  return hipGetLastError();
}

}  // namespace omb
