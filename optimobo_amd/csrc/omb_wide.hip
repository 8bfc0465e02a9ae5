// Wide inputs on gfx950: n_var from 65 to OMB_MAX_DIM (DP = 128 / 256).
//
// The reference puts no bound on n_var: every surrogate is GPy.kern.Matern52(n_vars, ARD=True)
// (optimobo/algorithms/optimisers.py:226, turbo.py:217), and TuRBO — the reference's method for
// high-dimensional problems — scores min(100·n_vars, 5000) trust-region candidates (turbo.py:36).
// The fused posterior kernel and the register-fragment K-block / covariance / gradient kernels hold
// one candidate's coordinates in registers (as MFMA B fragments, ⌈DP/4⌉ of them per lane), which is
// only affordable up to kMaxFusedDP = 64.  Above it the same quantities are formed here:
//
//   wide_cross_kernel     C = k(A, B) for 64×64 tiles of row pairs: the cross term a·b on
//                         v_mfma_f64_16x16x4f64 with the k loop over slabs of kWideSlab = 16
//                         dimensions staged through LDS (the next slab's loads in flight during the
//                         current slab's MFMAs), then r² = −2·a·b + (‖a‖² + ‖b‖²) (GPy
//                         Stationary._unscaled_dist) and the kernel transform fused into the store.
//                         RAWB: B is the caller's raw X*, divided by ℓ as it is staged (GPy divides),
//                         and ‖b‖² accumulates during the staging.  SYM: lower triangle of a symmetric
//                         matrix (K(X*, X*), K(X, X)), diagonal r² forced to 0 and the jitter added.
//   wide_scale_kernel     a = X/ℓ into rows of KP = ⌈d/16⌉·16 doubles and ‖a‖² (one wave per row).
//   gp_grad_wide_kernel   gp_grad_kernel's partial sums for one 16×16 tile of pairs: the tile's 32
//                         rows staged in LDS, one thread per pair for r², K and (dK/dr)/r, then one
//                         thread per dimension for Σ_pairs W·(−dK/dr/r)·(Δ_j)² in a fixed order.
//
// The posterior at n_var > 64 is the dense path of posterior_any (omb_api.hip): this K block, then
// V = L⁻¹K* (gemm) and the column reduction.  Bound: the cross-term MFMAs (2·d flop per pair against
// ≈ 30 for the transform) — these paths carry correctness for the reference's whole input range; the
// BASELINE configurations (n_var 6 and 30) stay on the fused kernels.
#include "omb_internal.h"
#include "omb_math.h"

namespace omb {

typedef double d4 __attribute__((ext_vector_type(4)));

namespace {

inline int wide_kp(int d) { return (d + kWideSlab - 1) / kWideSlab * kWideSlab; }

template <int KIND, bool SYM, bool RAWB>
__global__ __launch_bounds__(256) void wide_cross_kernel(const double* __restrict__ A, int64_t lda,
                                                         const double* __restrict__ asq, int64_t M,
                                                         const double* __restrict__ B, int64_t ldb,
                                                         const double* __restrict__ bsq, int64_t Nc,
                                                         const double* __restrict__ ls, int d, int KP,
                                                         double variance, double* __restrict__ C, int64_t ldc,
                                                         double diag_add) {
  if (SYM && blockIdx.x > blockIdx.y) return;
  const int64_t m0 = (int64_t)blockIdx.y * 64, n0 = (int64_t)blockIdx.x * 64;
  __shared__ double As[kWideSlab][65], Bs[kWideSlab][65];   // As[k][m] = a_{m0+m}[k0 + k]
  __shared__ double bn[64];                                 // RAWB: ‖b‖² of the tile's 64 columns
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  // staging: thread t loads dims sq .. sq+3 of the slab for row sr (rows past M / Nc are clamped: they only
  // feed entries that are never stored)
  const int sr = tid >> 2, sq = 4 * (tid & 3);
  const int64_t ar = (m0 + sr < M) ? m0 + sr : M - 1;
  const int64_t br = (n0 + sr < Nc) ? n0 + sr : Nc - 1;
  const double* Ap = A + ar * lda + sq;
  const double* Bp = B + br * ldb + sq;
  double ra[4], rb[4], bs2 = 0.0;
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) ra[i] = Ap[k0 + i];           // A rows are zero padded to KP
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (RAWB) {
        const int k = k0 + sq + i;
        rb[i] = (k < d) ? Bp[k0 + i] / ls[k] : 0.0;
      } else {
        rb[i] = Bp[k0 + i];
      }
    }
  };
  d4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};
  load(0);
  for (int k0 = 0; k0 < KP; k0 += kWideSlab) {
    __syncthreads();                                         // the previous slab's MFMAs are done with As / Bs
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      As[sq + i][sr] = ra[i];
      Bs[sq + i][sr] = rb[i];
      if constexpr (RAWB) bs2 = fma(rb[i], rb[i], bs2);
    }
    __syncthreads();
    if (k0 + kWideSlab < KP) load(k0 + kWideSlab);           // in flight during this slab's MFMAs
#pragma unroll
    for (int ks = 0; ks < kWideSlab / 4; ++ks) {
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
  }
  if constexpr (RAWB) {
    // the 4 staging threads of a column are adjacent lanes: a fixed xor tree
    bs2 += __shfl_xor(bs2, 1);
    bs2 += __shfl_xor(bs2, 2);
    if ((tid & 3) == 0) bn[sr] = bs2;
    __syncthreads();
  }
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    const int cl = 32 * wn + 16 * cb + (lane & 15);
    const int64_t col = n0 + cl;
    const double b2 = RAWB ? bn[cl] : (col < Nc ? bsq[col] : 0.0);
#pragma unroll
    for (int rbk = 0; rbk < 2; ++rbk) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t row = m0 + 32 * wm + 16 * rbk + (lane >> 4) + 4 * e;
        const double a2 = row < M ? asq[row] : 0.0;
        const double r2 = (SYM && row == col) ? 0.0 : fma(-2.0, acc[rbk][cb][e], a2 + b2);
        const double kv = kernel_of_r2<KIND>(r2, variance);
        if constexpr (SYM) {
          if (row < M && col <= row) C[row * ldc + col] = (row == col) ? kv + diag_add : kv;
        } else {
          if (row < M && col < Nc) __builtin_nontemporal_store(kv, C + row * ldc + col);
        }
      }
    }
  }
}

__global__ __launch_bounds__(256) void wide_scale_kernel(const double* __restrict__ Xc, int d, int64_t N,
                                                         const double* __restrict__ ls, int KP,
                                                         double* __restrict__ Xs, double* __restrict__ xsq) {
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);   // one wave per row
  const int lane = threadIdx.x & 63;
  if (i >= N) return;                                                // wave-uniform
  double s = 0.0;
  for (int k = lane; k < KP; k += 64) {
    const double a = (k < d) ? Xc[i * d + k] / ls[k] : 0.0;
    Xs[i * KP + k] = a;
    s = fma(a, a, s);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if (lane == 0) xsq[i] = s;
}

template <int KIND>
__global__ __launch_bounds__(256) void gp_grad_wide_kernel(const double* __restrict__ X, int d, int64_t n,
                                                           const double* __restrict__ ls, double variance,
                                                           const double* __restrict__ alpha,
                                                           const double* __restrict__ Kinv, int64_t ldk, int P,
                                                           double* __restrict__ partials) {
  __shared__ double Ai[16][OMB_MAX_DIM + 1], Bk[16][OMB_MAX_DIM + 1];
  __shared__ double cg[256], c0[256];
  const int tid = threadIdx.x;
  const int64_t i0 = (int64_t)blockIdx.y * 16, k0 = (int64_t)blockIdx.x * 16;
  const int64_t blk = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
  const bool live = blockIdx.x <= blockIdx.y;                       // lower triangle of tiles
  if (live) {
    for (int e = tid; e < 16 * d; e += 256) {
      const int r = e / d, j = e - r * d;
      Ai[r][j] = (i0 + r < n) ? X[(i0 + r) * d + j] / ls[j] : 0.0;   // GPy divides by ℓ
      Bk[r][j] = (k0 + r < n) ? X[(k0 + r) * d + j] / ls[j] : 0.0;
    }
  }
  __syncthreads();
  const int pi = tid >> 4, pk = tid & 15;
  const int64_t i = i0 + pi, k = k0 + pk;
  double gw = 0.0, kw = 0.0;
  if (live && i < n && k <= i) {
    double aa = 0.0, bb = 0.0, dot = 0.0;
    for (int j = 0; j < d; ++j) {
      const double a = Ai[pi][j], b = Bk[pk][j];
      aa += a * a;
      bb += b * b;
      dot = fma(a, b, dot);
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
    const double f = (i == k) ? 0.5 : 1.0;                          // off-diagonal pairs count twice
    const double W = f * (alpha[i] * alpha[k] - Kinv[i * ldk + k]);
    kw = W * Kik;
    gw = W * (-dkr);
  }
  cg[tid] = gw;
  c0[tid] = kw;
  __syncthreads();
  // q = 0: ∂/∂log σ_f²; q = 1 + j: ∂/∂log ℓ_j = Σ_pairs W·(−dK/dr / r)·(Δ_j)², pairs in index order
  for (int q = tid; q < P; q += 256) {
    double s = 0.0;
    if (q == 0) {
      for (int p = 0; p < 256; ++p) s += c0[p];
    } else if (live && q - 1 < d) {
      const int j = q - 1;
      for (int p = 0; p < 256; ++p) {
        const double dj = Ai[p >> 4][j] - Bk[p & 15][j];
        s = fma(cg[p], dj * dj, s);
      }
    }
    partials[blk * P + q] = s;
  }
}

}  // namespace

hipError_t launch_kernel_block_wide(hipStream_t stream, const GPDev& g, int d, int DP, const double* Xc, int64_t N,
                                    double* K, int64_t ldk) {
  if (N <= 0) return hipSuccess;
  const int KP = wide_kp(d);
  if (d < 1 || KP > DP) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((N + 63) / 64), (unsigned)((g.n + 63) / 64));
  if (g.kind == OMB_KERNEL_RBF)
    hipLaunchKernelGGL((wide_cross_kernel<OMB_KERNEL_RBF, false, true>), grid, dim3(256), 0, stream, g.Xs,
                       (int64_t)DP, g.xsq, (int64_t)g.n, Xc, (int64_t)d, nullptr, N, g.ls, d, KP, g.variance, K, ldk,
                       0.0);
  else
    hipLaunchKernelGGL((wide_cross_kernel<OMB_KERNEL_MATERN52, false, true>), grid, dim3(256), 0, stream, g.Xs,
                       (int64_t)DP, g.xsq, (int64_t)g.n, Xc, (int64_t)d, nullptr, N, g.ls, d, KP, g.variance, K, ldk,
                       0.0);
  return hipGetLastError();
}

hipError_t launch_cand_cov_wide(hipStream_t stream, const GPDev& g, int d, int DP, const double* Xc, int64_t N,
                                double* S, int64_t lds, double* ws, double diag_add) {
  if (N <= 0) return hipSuccess;
  const int KP = wide_kp(d);
  if (d < 1 || KP > DP) return hipErrorInvalidValue;
  // ws: cand_cov_ws_doubles(N, DP) = N·DP + N ≥ N·KP + N
  double* Xs = ws;
  double* xsq = ws + N * KP;
  hipLaunchKernelGGL(wide_scale_kernel, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, stream, Xc, d, N, g.ls, KP, Xs,
                     xsq);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const unsigned nt = (unsigned)((N + 63) / 64);
  if (g.kind == OMB_KERNEL_RBF)
    hipLaunchKernelGGL((wide_cross_kernel<OMB_KERNEL_RBF, true, false>), dim3(nt, nt), dim3(256), 0, stream, Xs,
                       (int64_t)KP, xsq, N, Xs, (int64_t)KP, xsq, N, g.ls, d, KP, g.variance, S, lds, diag_add);
  else
    hipLaunchKernelGGL((wide_cross_kernel<OMB_KERNEL_MATERN52, true, false>), dim3(nt, nt), dim3(256), 0, stream, Xs,
                       (int64_t)KP, xsq, N, Xs, (int64_t)KP, xsq, N, g.ls, d, KP, g.variance, S, lds, diag_add);
  return hipGetLastError();
}

hipError_t launch_gp_grad_partials_wide(hipStream_t stream, int kind, int DP, const double* X, int d, int64_t n,
                                        const double* ls, double variance, const double* alpha, const double* Kinv,
                                        int64_t ldk, double* partials) {
  if (d < 1 || d > DP || DP > OMB_MAX_DIM) return hipErrorInvalidValue;
  const unsigned t = (unsigned)((n + 15) / 16);
  const dim3 grid(t, t);
  if (kind == OMB_KERNEL_RBF)
    hipLaunchKernelGGL((gp_grad_wide_kernel<OMB_KERNEL_RBF>), grid, dim3(256), 0, stream, X, d, n, ls, variance, alpha,
                       Kinv, ldk, DP + 1, partials);
  else
    hipLaunchKernelGGL((gp_grad_wide_kernel<OMB_KERNEL_MATERN52>), grid, dim3(256), 0, stream, X, d, n, ls, variance,
                       alpha, Kinv, ldk, DP + 1, partials);
  return hipGetLastError();
}

}  // namespace omb
