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

// ----------------------------------------------------------------------------- posterior
// ABL (ablation, tools/ablate only; the library instantiates ABL = 0): bit 1 replaces the Matern
// transform by the raw dot product, bit 2 skips the MFMA phase, bit 4 feeds a constant A
// operand instead of loading L⁻¹, bit 8 drops the per-chunk barrier (barrier mode only), bit 16
// uses libm exp/sqrt, bit 32 selects the 2-buffer / block-barrier pipeline instead of the
// counter-synchronised 3-buffer ring (tools/ablate: 12.03 → 11.23 ms at n = 512, N = 2^20); bit 128
// gives waves 4-7 static priority 1, bit 256 drops the σ_f² multiply, bit 512 starts the distance
// chain at ‖x‖² + ‖x*‖² with −2x* pre-scaled (one fma fewer per element), bit 65536 forces a spin
// bound of 0 on the counter-ring waits (the fault-word path).
// NW = waves per workgroup (8 or 16): waves w, w+4, w+8, w+12 share a SIMD.
template <int RT, int CT, int DP, int KIND, int NW = 8, int ABL = 0>
__global__ __launch_bounds__(64 * NW, NW / 4) void posterior_kernel(GPArgs args, const double* __restrict__ Xc,
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
        for (int p = 0; p < (KSD + 1) / 2; ++p) a[p] = xa[64 * p];
        d4 cr = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s = 0; s < KSD; ++s)
          cr = __builtin_amdgcn_mfma_f64_16x16x4f64((s & 1) ? a[s >> 1].y : a[s >> 1].x, bfr[s], cr, 0, 0, 0);
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          const int k0 = rowbase + 4 * e + (lane >> 4), k1 = k0 + 4;
          double v0, v1;
          const double sf2 = (ABL & 256) ? 1.0 : g.variance;
          const double r2a = kAug ? cr[e] : fma(-2.0, cr[e], g.xsq[k0] + csq_m);
          const double r2b = kAug ? cr[e + 1] : fma(-2.0, cr[e + 1], g.xsq[k1] + csq_m);
          if constexpr (ABL & 8192)   // ablation: the 17-instruction polynomial exp, two sqrt corrections
            kernel_of_r2_k_x2<KIND>(r2a, r2b, sf2, args.ec, v0, v1);
          else if constexpr (kTab256)
            matern_r2_tab256_x2<(ABL & 32768) != 0>(r2a, r2b, pm, args.ec, etab, v0, v1);
          else
            kernel_of_r2_tab_x2<KIND>(r2a, r2b, pm, args.ec, etab, v0, v1);
          if constexpr (!kAug) {
            v0 = (k0 < g.n) ? v0 : 0.0;
            v1 = (k1 < g.n) ? v1 : 0.0;
          }
          mu_part = fma(g.alpha[k0], v0, mu_part);
          mu_part = fma(g.alpha[k1], v1, mu_part);
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
    constexpr int PD = (NW == 8) ? ((ABL & 64) ? 2 : 1) : 0;   // PD 2 measured no faster (11.19 vs 11.16 ms)
    d2 a_ring[PD + 1][RT];
    auto load_a = [&](int sp, d2* dst) {
#pragma unroll
      for (int j = 0; j < RT; ++j) {
        if constexpr (ABL & 4)
          dst[j] = d2{1e-3 * lane + sp, 2e-3 * j};
        else
          dst[j] = *reinterpret_cast<const d2*>(slot_A[j] + 128 * min(P0 + sp, 2 * slot_r[j] + 1));
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
    __syncthreads();
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
}

// ----------------------------------------------------------------------------- dispatch
template <int DP, int KIND>
static hipError_t launch_posterior_dp(hipStream_t stream, const GPArgs& args, int n_obj, int max_R,
                                      const double* Xc, int64_t N, double* mu, double* var) {
  const int Q = (max_R + 3) / 4;
  const int RTneed = (Q + 1) / 2;
  if (RTneed <= 1) {
    dim3 grid((unsigned)((N + 63) / 64), n_obj);
    // n ≤ 256: two 64-KiB workgroups per CU beat the 96-KiB counter ring
    hipLaunchKernelGGL((posterior_kernel<1, 4, DP, KIND, 8, 32>), grid, dim3(kBlockThreads), 0, stream, args, Xc, N, mu, var);
  } else if (RTneed <= 2) {
    // 128 < n ≤ 256: 32-candidate blocks on the counter ring (48 KiB, several workgroups per CU);
    // tools/ablate at n = 256, 3 objectives, 2^17 candidates: 0.709 ms (CT 4, barrier) → 0.600 ms
    dim3 grid((unsigned)((N + 31) / 32), n_obj);
    hipLaunchKernelGGL((posterior_kernel<2, 2, DP, KIND, 8, 0>), grid, dim3(kBlockThreads), 0, stream, args, Xc, N, mu, var);
  } else if (RTneed <= 4) {
    dim3 grid((unsigned)((N + 63) / 64), n_obj);
    hipLaunchKernelGGL((posterior_kernel<4, 4, DP, KIND>), grid, dim3(kBlockThreads), 0, stream, args, Xc, N, mu, var);
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
  dim3 grid((unsigned)((N + 63) / 64), (unsigned)((g.n + kKBlockRows - 1) / kKBlockRows));
  switch (args.DP) {
#define OMB_KB(DPV) \
  case DPV: hipLaunchKernelGGL((kernel_block_mfma_kernel<DPV, KIND>), grid, dim3(256), 0, stream, g, args.d, Xc, N, K, exp_coef()); break;
    OMB_KB(2) OMB_KB(4) OMB_KB(6) OMB_KB(8) OMB_KB(16) OMB_KB(32) OMB_KB(64)
#undef OMB_KB
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
