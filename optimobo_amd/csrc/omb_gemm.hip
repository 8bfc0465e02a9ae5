// Dense fp64 GEMM on gfx950 for the Thompson-sampling chain (omb_api.hip posterior_samples, §4b of
// DESIGN.md) and the GP fit:
//   V = L⁻¹K* (dense posterior, full covariance), Σ −= VᵀV (lower triangle), Y = μ + Z·Lᵀ (joint draws),
//   the blocked triangular inverse (launch_trinv) and the GP fit's α.
//
//   gemm_kernel        C = β·C + α·op(A)·op(B) (+ column bias) on v_mfma_f64_16x16x4f64: one 64×64 C
//                      tile per 256-thread workgroup (4 waves × 32×32), k-slabs of 16 double-buffered
//                      in LDS behind a register prefetch.  Variants: store the lower triangle only
//                      (SYRK-shaped Σ update), "op(B)(k, j) = 0 for k > j" (a lower-triangular factor
//                      read transposed: the samples μ + L z) and "op(A)(m, k) = 0 for k > m" (L⁻¹).
//
// Built on its own with -mllvm -amdgpu-mfma-vgpr-form (Makefile): in the default AGPR form the compiler
// carries the accumulators across the slab loop in VGPRs and copies all 32 registers to AGPRs and back
// every slab (64 VALU instructions per 16 MFMAs; FP64 MFMA does not overlap VALU on gfx950).  The
// Cholesky kernels in omb_linalg.hip keep the default form: their diagonal-block chain runs slower in
// the VGPR form (N = 3000 factorisation 1.37 → 1.40 ms, profiles/r03_z2_chol_{agpr,vgpr}.txt).
#include <algorithm>
#include <mutex>
#include <vector>

#include "omb_internal.h"

namespace omb {

typedef double d4 __attribute__((ext_vector_type(4)));

// ATRI (round 3): op(A) is lower-triangular (op(A)(m, k) = 0 for k > m, e.g. the dense L⁻¹ of V = L⁻¹K*):
// slabs past the tile's last row are skipped and the entries above the diagonal read as zero, so the
// upper triangle is never read (as the packed posterior path never reads it) and half the work goes.
// KSS (round 5, the posterior covariance): C = K(X*, X*) − op(A)·op(B) on the lower triangle, the kernel block of
// the tile formed in the epilogue from the scaled candidates (CovEpi: X*/ℓ rows of kp doubles and ‖·‖², as
// cand_scale_kernel writes them) — cand_cov_kernel's arithmetic in its order (the cross term on MFMA over k-steps of
// 4 ascending, r² = −2·a·b + (‖a‖² + ‖b‖²) with the diagonal forced to 0, kernel_of_r2, + diag_add on the
// diagonal), so C is what cand_cov_kernel then gemm_kernel(β = 1, α = −1) store — to the ulp of the Matern
// polynomial, whose FMA contraction the compiler picks per kernel (measured ≤ 6e-17 absolute at σ_f² ≈ 0.5, the
// diagonal bitwise; gpurun_out/r05_j) — without the 8N² bytes of K(X*, X*) written and read back and its launch.
struct CovEpi {
  const double* xs;
  const double* xsq;
  int kp;
  int kind;
  double variance;
  double diag_add;
  int* zero_ints;   // n_zero words every workgroup's share of which it sets to 0 (the next Cholesky's sync words)
  int n_zero;
  int* zero_info;   // set to 0 by workgroup 0 (that Cholesky's status)
};

// The launch's side job (zero_ints / zero_info), run by every workgroup before any early return
__device__ __forceinline__ void cov_zero_side(const CovEpi& ce) {
  const int64_t b = (int64_t)blockIdx.y * gridDim.x + blockIdx.x, nb = (int64_t)gridDim.x * gridDim.y;
  for (int64_t x = b * blockDim.x + threadIdx.x; x < ce.n_zero; x += nb * blockDim.x) ce.zero_ints[x] = 0;
  if (ce.zero_info && b == 0 && threadIdx.x == 0) *ce.zero_info = 0;
}

// KSS epilogue (gemm_kernel, syrk_glds_kernel): C = K(X*, X*) + α·acc on the tile's lower triangle, the kernel block's
// cross term over kp dimensions in slabs of 16 staged through the LDS scratch As / Bs ([16][pitch] doubles each).
__device__ __forceinline__ void cov_epilogue(int64_t m0, int64_t n0, int64_t M, int64_t Nc, const d4 (&acc)[2][2],
                                             double alpha, const CovEpi& ce, double* __restrict__ C, int64_t ldc,
                                             double* As, double* Bs, int pitch) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  d4 cr[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) cr[i][j] = d4{0.0, 0.0, 0.0, 0.0};
  for (int k0 = 0; k0 < ce.kp; k0 += kGK) {
    __syncthreads();                                       // the product's last slab is read by every wave
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int idx = tid + 256 * e, r = idx >> 4, k = idx & 15;
      const int64_t ra = m0 + r < M ? m0 + r : M - 1, rb = n0 + r < Nc ? n0 + r : Nc - 1;
      As[k * pitch + r] = k0 + k < ce.kp ? ce.xs[ra * ce.kp + k0 + k] : 0.0;
      Bs[k * pitch + r] = k0 + k < ce.kp ? ce.xs[rb * ce.kp + k0 + k] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < kGK / 4; ++ks) {
      const int kk = 4 * ks + (lane >> 4);
      const double a0 = As[kk * pitch + 32 * wm + (lane & 15)];
      const double a1 = As[kk * pitch + 32 * wm + 16 + (lane & 15)];
      const double b0 = Bs[kk * pitch + 32 * wn + (lane & 15)];
      const double b1 = Bs[kk * pitch + 32 * wn + 16 + (lane & 15)];
      cr[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, cr[0][0], 0, 0, 0);
      cr[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, cr[0][1], 0, 0, 0);
      cr[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, cr[1][0], 0, 0, 0);
      cr[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, cr[1][1], 0, 0, 0);
    }
  }
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    const int64_t col = n0 + 32 * wn + 16 * cb + (lane & 15);
    const double bsq = col < Nc ? ce.xsq[col] : 0.0;
#pragma unroll
    for (int rb2 = 0; rb2 < 2; ++rb2)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t row = m0 + 32 * wm + 16 * rb2 + (lane >> 4) + 4 * i;
        if (row < M && col < Nc && col <= row) {
          const double r2 = (row == col) ? 0.0 : fma(-2.0, cr[rb2][cb][i], ce.xsq[row] + bsq);
          double kv = ce.kind == OMB_KERNEL_RBF ? kernel_of_r2<OMB_KERNEL_RBF>(r2, ce.variance)
                                                : kernel_of_r2<OMB_KERNEL_MATERN52>(r2, ce.variance);
          if (row == col) kv = kv + ce.diag_add;
          C[row * ldc + col] = fma(1.0, kv, alpha * acc[rb2][cb][i]);
        }
      }
  }
}

template <bool TA, bool TB, bool BTRI, bool LOWER, bool ATRI = false, bool KSS = false>
__global__ __launch_bounds__(256) void gemm_kernel(int64_t M, int64_t Nc, int64_t K, double alpha,
                                                   const double* __restrict__ A, int64_t lda,
                                                   const double* __restrict__ B, int64_t ldb, double beta,
                                                   double* __restrict__ C, int64_t ldc,
                                                   const double* __restrict__ col_bias, int64_t kchunk,
                                                   int64_t zstride, CovEpi ce,
                                                   const int* __restrict__ tmap = nullptr) {
  if constexpr (KSS) cov_zero_side(ce);
  // ATRI: the last row tiles carry the most slabs, so they are dispatched first
  int64_t m0 = (int64_t)(ATRI ? gridDim.y - 1 - blockIdx.y : blockIdx.y) * kGT, n0 = (int64_t)blockIdx.x * kGT;
  if (tmap) {   // 1-D grid, workgroup b → tile tmap[b] = (row tile << 16 | column tile), −1: none (syrk_tile_map)
    const int code = tmap[blockIdx.x];
    if (code < 0) return;
    m0 = (int64_t)(code >> 16) * kGT;
    n0 = (int64_t)(code & 0xffff) * kGT;
  }
  if (LOWER && n0 > m0) return;   // tile strictly above the diagonal
  __shared__ double As[2][kGK][kGP];   // As[k][m] = op(A)(m0 + m, k0 + k)
  __shared__ double Bs[2][kGK][kGP];   // Bs[k][n] = op(B)(k0 + k, n0 + n)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  // with BTRI, slabs past the tile's last column are all zero in op(B)
  int64_t kend = BTRI ? (K < n0 + kGT ? K : n0 + kGT) : K;
  if (ATRI && kend > m0 + kGT) kend = m0 + kGT;
  // split K (gridDim.z > 1): slice z covers [z·kchunk, (z+1)·kchunk) into its own partial C + z·zstride
  const int64_t kbeg = (int64_t)blockIdx.z * kchunk;
  if (gridDim.z > 1) {
    kend = kend < kbeg + kchunk ? kend : kbeg + kchunk;
    if (BTRI && kend <= kbeg) return;   // a slice past the tile's last column: zero, never read (splitk_reduce_kernel)
    C += (int64_t)blockIdx.z * zstride;
  }

  // 1024 elements of each operand per slab, 4 per thread; consecutive threads walk the
  // contiguous dimension of the stored matrix (coalesced), LDS stores land conflict-free.
  // Rows of op(A) past M and columns of op(B) past Nc only feed C entries that are never stored,
  // so their addresses are clamped into the matrix rather than masked; each element keeps a
  // running pointer (one 64-bit add per slab), and only the last slab, when it reaches past K,
  // checks k.
  const double* pa[4];
  const double* pb[4];
  int ak_[4], bk_[4];
  int64_t gm_[4], gn_[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int idx = tid + 256 * e;
    const int am = TA ? (idx & 63) : (idx >> 4), ak = TA ? (idx >> 6) : (idx & 15);
    const int bn = TB ? (idx >> 4) : (idx & 63), bk = TB ? (idx & 15) : (idx >> 6);
    gm_[e] = m0 + am;
    gn_[e] = n0 + bn;
    ak_[e] = ak;
    bk_[e] = bk;
    const int64_t cm = gm_[e] < M ? gm_[e] : M - 1, cn = gn_[e] < Nc ? gn_[e] : Nc - 1;
    pa[e] = TA ? A + (kbeg + ak) * lda + cm : A + cm * lda + kbeg + ak;
    pb[e] = TB ? B + cn * ldb + kbeg + bk : B + (kbeg + bk) * ldb + cn;
  }
  const int64_t sa = TA ? kGK * lda : kGK, sb = TB ? kGK : kGK * ldb;   // one slab along k
  double ra[4], rb[4];
  auto fetch = [&](int64_t k0, bool edge) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t gka = k0 + ak_[e], gkb = k0 + bk_[e];
      double va, vb;
      if (edge) {
        va = gka < kend ? *pa[e] : 0.0;
        vb = gkb < kend ? *pb[e] : 0.0;
      } else {
        va = *pa[e];
        vb = *pb[e];
      }
      ra[e] = (ATRI && gka > gm_[e]) ? 0.0 : va;
      rb[e] = (BTRI && gkb > gn_[e]) ? 0.0 : vb;
      pa[e] += sa;
      pb[e] += sb;
    }
  };
  auto stash = [&](int buf) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int idx = tid + 256 * e;
      As[buf][TA ? (idx >> 6) : (idx & 15)][TA ? (idx & 63) : (idx >> 4)] = ra[e];
      Bs[buf][TB ? (idx & 15) : (idx >> 6)][TB ? (idx >> 4) : (idx & 63)] = rb[e];
    }
  };

  d4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};
  auto multiply = [&](int buf) {
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
  };

  if (kend > kbeg) {
    fetch(kbeg, kbeg + kGK > kend);
    stash(0);
    __syncthreads();
    // every slab followed by a full one: its loads are in flight while this one multiplies
    int buf = 0;
    int64_t k0 = kbeg;
    for (; k0 + 2 * kGK <= kend; k0 += kGK) {
      fetch(k0 + kGK, false);
      multiply(buf);
      // the other buffer was last read in the previous slab, which every wave has finished
      stash(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
    if (k0 + kGK < kend) {   // a last, partial slab (kend = K, K not a multiple of 16)
      fetch(k0 + kGK, true);
      multiply(buf);
      stash(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
    multiply(buf);
  }

  if constexpr (KSS) {
    cov_epilogue(m0, n0, M, Nc, acc, alpha, ce, C, ldc, &As[0][0][0], &Bs[0][0][0], kGP);
    return;
  }

  // C/D map of v_mfma_f64_16x16x4f64: col = lane & 15, row = (lane >> 4) + 4·i
#pragma unroll
  for (int rb2 = 0; rb2 < 2; ++rb2)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t row = m0 + 32 * wm + 16 * rb2 + (lane >> 4) + 4 * i;
        const int64_t col = n0 + 32 * wn + 16 * cb + (lane & 15);
        if (row < M && col < Nc && (!LOWER || col <= row)) {
          double v = alpha * acc[rb2][cb][i];
          if (beta != 0.0) v = fma(beta, C[row * ldc + col], v);
          if (col_bias) v += col_bias[col];
          C[row * ldc + col] = v;
        }
      }
}

// Round 6: the covariance SYRK (Σ = K(X*, X*) − VᵀV, lower triangle, V (K, N) row-major) with a three-stage operand
// pipeline filled by direct-to-LDS loads (gemm_kernel's waves waited on their slab loads 66% of
// their cycles, and a second register slab spilled).  Stage s holds slab k's A and B tiles — 16 rows of
// V × 64 columns each, XOR-swizzled in pairs of columns so the four 16-lane row groups of an MFMA operand read hit
// both halves of the bank row — written by global_load_lds_dwordx4: one wave-instruction is 1 KiB, two rows, lane l
// the 16 B at row 2p + (l >> 5), column pair (l & 31) ^ 8·(row & 1) of the source (linear LDS, swizzle on the source
// and on the read).  Slab k + 2 is issued after the barrier that retires slab k, so two slabs stay in flight while
// one multiplies; the wait is a counted vmcnt and the barrier a raw s_barrier (a __syncthreads would drain the DMA).
// Every LDS byte lives in the one __shared__ array (a second __shared__ object can make hipcc wait vmcnt(0) before
// each ds_read).  Requires K a multiple of 16 and N even with V 16-B aligned (launch_cov_syrk checks); the products
// are summed in gemm_kernel's k order, so C is bitwise gemm_kernel<…, KSS>'s.
__device__ __forceinline__ int syrk_swz(int row, int col) { return ((((col >> 1) ^ ((row & 1) << 3)) << 1) | (col & 1)); }

// s_waitcnt vmcnt(n) for a wave-uniform n ≤ 15 (the immediate is an encoding field)
__device__ __forceinline__ void wait_vmcnt_le(int n) {
  switch (n) {
#define OMB_VMC(X) \
  case X: asm volatile("s_waitcnt vmcnt(" #X ")" ::: "memory"); break;
    OMB_VMC(1) OMB_VMC(2) OMB_VMC(3) OMB_VMC(4) OMB_VMC(5) OMB_VMC(6) OMB_VMC(7) OMB_VMC(8) OMB_VMC(9) OMB_VMC(10)
    OMB_VMC(11) OMB_VMC(12) OMB_VMC(13) OMB_VMC(14) OMB_VMC(15)
#undef OMB_VMC
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// STAGES slabs of SR rows in flight, MINB workgroups per CU for the register allocation (the library: 3 × 16, 1;
// tools/ablate/ablate_syrk times the others)
template <int STAGES, int SR, int MINB = 1>
__global__ __launch_bounds__(256, MINB) void syrk_glds_kernel(int64_t N, int64_t K, double alpha, const double* __restrict__ V,
                                                        int64_t ldv, double* __restrict__ C, int64_t ldc, CovEpi ce,
                                                        const int* __restrict__ tmap) {
  static_assert(SR % 8 == 0 && STAGES >= 2, "slabs of whole 8-row groups (one 2-row piece per wave)");
  cov_zero_side(ce);
  int64_t m0 = (int64_t)blockIdx.y * kGT, n0 = (int64_t)blockIdx.x * kGT;
  if (tmap) {
    const int code = tmap[blockIdx.x];
    if (code < 0) return;
    m0 = (int64_t)(code >> 16) * kGT;
    n0 = (int64_t)(code & 0xffff) * kGT;
  }
  if (n0 > m0) return;
  constexpr int kSlab = SR * kGT;                           // doubles of one operand's slab
  constexpr int PPW = SR / 8;                               // 1-KiB pieces (2 rows) per wave per operand and slab
  __shared__ __attribute__((aligned(16))) double sm[STAGES * 2 * kSlab];
  typedef __attribute__((address_space(3))) void lds_void;
  typedef __attribute__((address_space(1))) const void g_void;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  // piece p = PPW·wave + j covers rows 2p, 2p + 1; this lane's source column pair (lane & 31) ^ 8·(row & 1), clamped
  // into the matrix (columns past N feed C entries that are never stored)
  const int q = lane & 31;
  int64_t colA[2], colB[2];
#pragma unroll
  for (int par = 0; par < 2; ++par) {                       // row parity of the lane's rows: (lane >> 5) of an even base
    const int gq = q ^ (par << 3);
    colA[par] = m0 + 2 * gq < N - 1 ? m0 + 2 * gq : N - 2;
    colB[par] = n0 + 2 * gq < N - 1 ? n0 + 2 * gq : N - 2;
  }
  const int par = lane >> 5;
  const int ns = (int)(K / SR);
  auto issue = [&](int stage, int slab) {
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const int r0 = 2 * (PPW * wave + j);                  // even: the lane's row is r0 + par
      const double* src = V + ((int64_t)slab * SR + r0 + par) * ldv;
      double* dA = sm + (stage * 2 + 0) * kSlab + r0 * kGT;   // wave-uniform
      double* dB = sm + (stage * 2 + 1) * kSlab + r0 * kGT;
      __builtin_amdgcn_global_load_lds((g_void*)(src + colA[par]), (lds_void*)dA, 16, 0, 0);
      __builtin_amdgcn_global_load_lds((g_void*)(src + colB[par]), (lds_void*)dB, 16, 0, 0);
    }
  };
  d4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int st = 0; st < STAGES - 1; ++st)
    if (st < ns) issue(st, st);
  for (int sl = 0; sl < ns; ++sl) {
    // slab sl's DMAs of this wave retired (the later ones already issued may stay in flight), then every wave's
    const int later = ns - 1 - sl < STAGES - 2 ? ns - 1 - sl : STAGES - 2;
    wait_vmcnt_le(2 * PPW * later);
    __builtin_amdgcn_s_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    // the stage slab sl + STAGES − 1 refills was last read by slab sl − 1, which every wave has finished
    if (sl + STAGES - 1 < ns) issue((sl + STAGES - 1) % STAGES, sl + STAGES - 1);
    const double* As = sm + ((sl % STAGES) * 2 + 0) * kSlab;
    const double* Bs = sm + ((sl % STAGES) * 2 + 1) * kSlab;
#pragma unroll
    for (int ks = 0; ks < SR / 4; ++ks) {
      const int kk = 4 * ks + (lane >> 4);
      const double a0 = As[kk * kGT + syrk_swz(kk, 32 * wm + (lane & 15))];
      const double a1 = As[kk * kGT + syrk_swz(kk, 32 * wm + 16 + (lane & 15))];
      const double b0 = Bs[kk * kGT + syrk_swz(kk, 32 * wn + (lane & 15))];
      const double b1 = Bs[kk * kGT + syrk_swz(kk, 32 * wn + 16 + (lane & 15))];
      acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
    }
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
  }
  // the epilogue's cross-term scratch: stage 0's A / B tiles (16 of their rows, after the epilogue's first barrier)
  cov_epilogue(m0, n0, N, N, acc, alpha, ce, C, ldc, sm, sm + kSlab, kGT);
}
constexpr int kSyrkStages = 3, kSyrkRows = 16;

template <bool TA, bool TB, bool BTRI, bool LOWER, bool ATRI = false>
static hipError_t gemm(hipStream_t stream, int64_t M, int64_t Nc, int64_t K, double alpha, const double* A,
                       int64_t lda, const double* B, int64_t ldb, double beta, double* C, int64_t ldc,
                       const double* col_bias) {
  if (M <= 0 || Nc <= 0) return hipSuccess;
  dim3 grid((unsigned)((Nc + kGT - 1) / kGT), (unsigned)((M + kGT - 1) / kGT));
  hipLaunchKernelGGL((gemm_kernel<TA, TB, BTRI, LOWER, ATRI>), grid, dim3(256), 0, stream, M, Nc, K, alpha, A, lda, B,
                     ldb, beta, C, ldc, col_bias, (int64_t)0, (int64_t)0, CovEpi{});
  return hipGetLastError();
}

// C (M, Nc) = bias + Σ_z P[z] in slice order (deterministic), P[z] (M, Nc) dense at P + z·zstride.  With kchunk > 0
// (op(B) lower-triangular, BTRI), column c sums only the slices that start below its tile's last row, the others
// being zero and left unwritten by gemm_kernel.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const double* __restrict__ P, int S, int64_t zstride,
                                                            int64_t M, int64_t Nc, const double* __restrict__ bias,
                                                            double* __restrict__ C, int64_t ldc, int64_t kchunk) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * Nc) return;
  const int64_t r = i / Nc, c = i - r * Nc;
  int Sc = S;
  if (kchunk > 0) {                               // the product's K is Nc here (Y = Z·Lᵀ, L square)
    int64_t kend = (c / kGT + 1) * kGT;
    kend = kend < Nc ? kend : Nc;
    const int64_t a = (kend + kchunk - 1) / kchunk;
    Sc = a < S ? (int)a : S;
  }
  double v = 0.0;
  int z = 0;
  for (; z + 8 <= Sc; z += 8) {   // 8 slices' loads in flight, added in slice order
    double p[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) p[u] = P[(z + u) * zstride + i];
#pragma unroll
    for (int u = 0; u < 8; ++u) v += p[u];
  }
  for (; z < Sc; ++z) v += P[z * zstride + i];
  C[r * ldc + c] = v + (bias ? bias[c] : 0.0);
}


// ----------------------------------------------------------------------------- launchers
// Tile tables for 1-D launches in an XCD-aware order (round 5): workgroups reach the 8 XCDs in turn (b mod 8), so
// workgroup 8j + x runs the j-th tile of XCD x's list (−1 past its end); codes are (row tile << 16 | column tile).
// Built on the host once per (device, kind, shape) and kept (the first 64 shapes).
//   kMapSyrk (T × T lower tiles of Σ = K** − VᵀV): tile (m, n) streams V's column panels m and n (K × 64 doubles,
//     256 KB at K = 512); with the 2-D grid every XCD ran tiles from the whole triangle, cycling its 4-MB L2 through
//     all ⌈N/64⌉ panels (12 MB at N = 3000): L2 hit rate 0.54 (PMC, profiles/r05_zt_pmc_c6_gemm.txt).  The panels form
//     4 contiguous groups and the 10 group pairs (g_m ≥ g_n) go to the XCDs largest first onto the least-loaded one,
//     so an XCD's tiles touch two groups (≈ 6 MB, the least for ≈ 141 tiles): hit rate 0.84.
// (The same grouping by column tiles for V = L⁻¹K* raised its L2 hit rate from 0.45 to 0.74 and left it at 38 µs,
// profiles/r05_zv_ltri_xcd_map_ab.txt: that launch is bound by its heaviest row tiles, not by their loads.)
enum { kMapSyrk = 0 };
static const int* xcd_tile_map(int kind, int T1, int T2, int* grid) {
  struct Map {
    int dev, kind, T1, T2, grid;
    int* d;
  };
  static std::mutex mu;
  static std::vector<Map> maps;
  int dev = 0;
  if (T1 > 0xffff || T2 > 0xffff || hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  for (const Map& e : maps)
    if (e.dev == dev && e.kind == kind && e.T1 == T1 && e.T2 == T2) {
      *grid = e.grid;
      return e.d;
    }
  if (maps.size() >= 64) return nullptr;   // shapes past the first 64 launch on the 2-D grid (bounded host cache)
  constexpr int X = 8;
  std::vector<std::vector<int>> lists(X);
  if (kind == kMapSyrk) {
    constexpr int G = 4;
    const int T = T1;
    auto gstart = [&](int g) { return (int)((int64_t)T * g / G); };
    std::vector<std::pair<int, int>> pairs;
    for (int a = 0; a < G; ++a)
      for (int b = 0; b <= a; ++b) pairs.push_back({a, b});
    auto ntiles = [&](std::pair<int, int> p) {
      const int ra = gstart(p.first + 1) - gstart(p.first), rb = gstart(p.second + 1) - gstart(p.second);
      return p.first == p.second ? ra * (ra + 1) / 2 : ra * rb;
    };
    std::stable_sort(pairs.begin(), pairs.end(), [&](auto x, auto y) { return ntiles(x) > ntiles(y); });
    for (const auto& p : pairs) {
      int x = 0;
      for (int q = 1; q < X; ++q)
        if (lists[q].size() < lists[x].size()) x = q;
      for (int m = gstart(p.first); m < gstart(p.first + 1); ++m)
        for (int n = gstart(p.second); n < gstart(p.second + 1) && (p.first != p.second || n <= m); ++n)
          lists[x].push_back((m << 16) | n);
    }
  }
  size_t len = 0;
  for (const auto& l : lists) len = std::max(len, l.size());
  std::vector<int> codes(X * len, -1);
  for (int x = 0; x < X; ++x)
    for (size_t j = 0; j < lists[x].size(); ++j) codes[X * j + x] = lists[x][j];
  int* d = nullptr;
  if (hipMalloc(&d, sizeof(int) * codes.size()) != hipSuccess) return nullptr;
  if (hipMemcpy(d, codes.data(), sizeof(int) * codes.size(), hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(d);
    return nullptr;
  }
  maps.push_back({dev, kind, T1, T2, (int)codes.size(), d});
  *grid = (int)codes.size();
  return d;
}

hipError_t launch_gemm_ltri_nn(hipStream_t s, int64_t M, int64_t Nc, double alpha, const double* L, int64_t ldl,
                               const double* B, int64_t ldb, double beta, double* C, int64_t ldc) {
  return gemm<false, false, false, false, true>(s, M, Nc, M, alpha, L, ldl, B, ldb, beta, C, ldc, nullptr);
}

hipError_t launch_gemm_nn(hipStream_t s, int64_t M, int64_t Nc, int64_t K, double alpha, const double* A, int64_t lda,
                          const double* B, int64_t ldb, double beta, double* C, int64_t ldc) {
  return gemm<false, false, false, false>(s, M, Nc, K, alpha, A, lda, B, ldb, beta, C, ldc, nullptr);
}

hipError_t launch_gemm_tn_lower(hipStream_t s, int64_t N, int64_t K, double alpha, const double* A, int64_t lda,
                                double beta, double* C, int64_t ldc) {
  return gemm<true, false, false, true>(s, N, N, K, alpha, A, lda, A, lda, beta, C, ldc, nullptr);
}

// K slices of the sample product: enough (tile, slice) workgroups to fill the chip (≥ 2048), slices of
// ≥ 96 columns.  At B = 64 draws of N = 3000 candidates the unsplit product has 47 workgroups
// (208 µs, profiles/r02_v21_c6_kernel_stats.csv); 16 slices of 192 columns 33.9 + 5.7 µs (product + reduction),
// 32 slices of 96 with the zero slices neither written nor read 22.3 + 10.9 µs (profiles/r04_ar_*).
static int samples_split(int64_t N, int B) {
  const int64_t tiles = ((B + kGT - 1) / kGT) * ((N + kGT - 1) / kGT);
  int64_t S = (2048 + tiles - 1) / tiles;
  const int64_t smax = (N + 95) / 96;
  if (S > smax) S = smax;
  if (S > 32) S = 32;
  return S < 1 ? 1 : (int)S;
}

int64_t chol_samples_ws_doubles(int64_t N, int B) {
  const int S = samples_split(N, B);
  return S > 1 ? (int64_t)S * B * N : 0;
}

hipError_t launch_chol_samples(hipStream_t stream, const double* L, int64_t N, int64_t ldl, const double* mu,
                               const double* Zt, int B, double* Y, double* ws) {
  // Y (B, N) = Zt · Lᵀ + μ  with  op(B)(k, j) = L[j][k] for k ≤ j (the factor's upper part is ignored)
  const int S = samples_split(N, B);
  if (S == 1) return gemm<false, true, true, false>(stream, B, N, N, 1.0, Zt, N, L, ldl, 0.0, Y, N, mu);
  const int64_t kchunk = ((N + S - 1) / S + kGK - 1) / kGK * kGK;
  const int64_t zstride = (int64_t)B * N;
  dim3 grid((unsigned)((N + kGT - 1) / kGT), (unsigned)((B + kGT - 1) / kGT), (unsigned)S);
  hipLaunchKernelGGL((gemm_kernel<false, true, true, false>), grid, dim3(256), 0, stream, (int64_t)B, N, N, 1.0, Zt,
                     N, L, ldl, 0.0, ws, N, (const double*)nullptr, kchunk, zstride, CovEpi{});
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int64_t tot = (int64_t)B * N;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, ws, S, zstride,
                     (int64_t)B, N, mu, Y, N, kchunk);
  return hipGetLastError();
}

#ifdef OMB_TOOLS_KNOBS
static bool g_syrk_xcd_map = true;
void set_syrk_xcd_map(bool on) { g_syrk_xcd_map = on; }
#elif defined(OMB_SYRK_NOMAP)
constexpr bool g_syrk_xcd_map = false;
#else
constexpr bool g_syrk_xcd_map = true;
#endif

hipError_t launch_cov_syrk(hipStream_t s, int64_t N, int64_t K, const double* V, int64_t ldv, double* S, int64_t lds,
                           const double* xs, const double* xsq, int kp, int kind, double variance, double diag_add,
                           bool glds, int* zero_ints, int n_zero, int* zero_info) {
  if (N <= 0) return hipSuccess;
  const int T = (int)((N + kGT - 1) / kGT);
  int g1 = 0;
  const int* tmap = g_syrk_xcd_map ? xcd_tile_map(kMapSyrk, T, T, &g1) : nullptr;
  const dim3 grid = tmap ? dim3((unsigned)g1) : dim3((unsigned)T, (unsigned)T);
  // the direct-to-LDS pipeline needs whole 16-row slabs and 16-B column pairs inside each row
  if (glds && K % kSyrkRows == 0 && N % 2 == 0 && N >= 2 && ldv % 2 == 0 &&
      (reinterpret_cast<uintptr_t>(V) & 15) == 0) {
    hipLaunchKernelGGL((syrk_glds_kernel<kSyrkStages, kSyrkRows>), grid, dim3(256), 0, s, N, K, -1.0, V, ldv, S, lds,
                       CovEpi{xs, xsq, kp, kind, variance, diag_add, zero_ints, n_zero, zero_info}, tmap);
    return hipGetLastError();
  }
  hipLaunchKernelGGL((gemm_kernel<true, false, false, true, false, true>), grid, dim3(256), 0, s, N, N, K, -1.0, V, ldv,
                     V, ldv, 0.0, S, lds, (const double*)nullptr, (int64_t)0, (int64_t)0,
                     CovEpi{xs, xsq, kp, kind, variance, diag_add, zero_ints, n_zero, zero_info}, tmap);
  return hipGetLastError();
}

hipError_t launch_gemm_tn(hipStream_t s, int64_t M, int64_t Nc, int64_t K, double alpha, const double* A, int64_t lda,
                          const double* B, int64_t ldb, double beta, double* C, int64_t ldc) {
  return gemm<true, false, false, false>(s, M, Nc, K, alpha, A, lda, B, ldb, beta, C, ldc, nullptr);
}

}  // namespace omb
