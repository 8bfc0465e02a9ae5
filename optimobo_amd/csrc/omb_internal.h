// Internal declarations shared by the HIP translation units of liboptimobo_hip.so.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/optimobo_hip.h"
#include "omb_host.h"
#include "omb_math.h"

namespace omb {

// Rows of the training set handled per streamed K* chunk (4 row tiles of 16).
constexpr int kChunkRows = 64;
constexpr int kBlockThreads = 512;
// Training rows per workgroup of the standalone K-block kernel.
constexpr int kKBlockRows = 256;

// Device-side state of one fitted GP (objective), built by omb_set_gp.
struct GPDev {
  const double* Xs;     // (n_pad, DP) training inputs / ℓ, zero padded
  const double* xsq;    // (n_pad) Σ_j Xs[k][j]²
  const double* alpha;  // (n_pad) woodbury vector, zero padded
  const double* Lp;     // packed lower-triangular L^-1 in MFMA fragment order (see pack kernel)
  const double* ls;     // (DP) lengthscales, padded with 1
  double variance;      // σ_f²
  int n;                // n_train
  int R;                // row tiles = ceil(n / 16)
  int kind;             // OMB_KERNEL_*
  int pad_;
  const double* Xf;     // Xs in A-fragment order for the MFMA cross term (see pack_X_kernel)
};

struct GPArgs {
  GPDev gp[OMB_MAX_OBJ];
  int d;    // true n_var (≤ DP)
  int DP;   // padded dim used by the packed Xs
  ExpCoef ec;      // exp_nonpos coefficients as kernel arguments (set by launch_posterior)
  int* fault;      // context fault word (pinned host memory): bit 0 = an LDS-counter wait ran out
  int spin_limit;  // polls per LDS-counter wait before the fault word is marked
};

constexpr int kFaultSpin = 1;          // fault word bit: posterior counter-ring wait exhausted
constexpr int kDefaultSpinLimit = 1 << 22;

// ---------------------------------------------------------------------------------------
// Launchers (host functions; each launches on `stream` and returns hipGetLastError()).
hipError_t launch_pack_gp(hipStream_t stream, int n, int d, int DP, const double* X, const double* ls_dev,
                          const double* alpha, const double* Linv, double* Xs, double* xsq, double* alpha_p,
                          double* Lp, int R, int n_pad);
// Xf = Xs in the A-fragment order of the posterior kernel's MFMA cross term (after launch_pack_gp)
hipError_t launch_pack_x(hipStream_t stream, int d, int DP, int n_pad, const double* Xs, const double* xsq,
                         double* Xf);

hipError_t launch_kernel_block(hipStream_t stream, const GPArgs& args, int obj, const double* Xc, int64_t N,
                               double* K);

hipError_t launch_posterior(hipStream_t stream, const GPArgs& args, int n_obj, int max_R, const double* Xc,
                            int64_t N, double* mu, double* var);

// EHVI-2D and the arg-max in one launch (omb_acquisition.hip): each workgroup's (value, index) pair goes to
// `partials` (2 doubles per workgroup, ehvi2d_argmax_blocks(N) ≤ kArgmaxMaxBlocks); the last workgroup to finish (an
// agent-scope ticket, 0 between launches) reduces them and writes result = {value, index + offset} — or, with
// ticket == nullptr, a second launch (argmax_pass2) does.
struct ArgmaxOut {
  double* partials;
  unsigned* ticket;
  double* result;
  int64_t offset;
};
int64_t ehvi2d_argmax_blocks(int64_t N);
hipError_t launch_ehvi2d_argmax(hipStream_t stream, const double* mu, const double* var, int64_t ld, int64_t N,
                                const double* pf, int P, double r0, double r1, double s00, double s01, int mode,
                                const ArgmaxOut& am);

hipError_t launch_ehvi2d(hipStream_t stream, const double* mu, const double* var, int64_t ld, int64_t N,
                         const double* pf, int P, double r0, double r1, double s00, double s01, int mode,
                         double* out);

hipError_t launch_ehvi_mc(hipStream_t stream, int k, const double* mu, const double* var, int64_t ld, int64_t N,
                          const double* cache, int M, const double* r, double hv_pf, double* out, int32_t* raised);

hipError_t launch_ehvi_boxes(hipStream_t stream, int k, const double* mu, const double* var, int64_t ld, int64_t N,
                             const double* coords, int C, const uint16_t* boxes, int B, double* out);

hipError_t launch_hvpoi(hipStream_t stream, const double* mu, const double* var, int64_t ld, int64_t N,
                        const double* cells, int C, double* out);


hipError_t launch_expdec(hipStream_t stream, const ScalParams& sp, const double* mu, const double* var,
                         int64_t ld, int64_t N, const double* cache, int M, double* out);

hipError_t launch_ei(hipStream_t stream, int kind, int k, const double* mu, const double* var, int64_t ld, int64_t N,
                     double best, double var_eps, double pof_eps, double* out);

// Deterministic arg-max; `partials` must hold kArgmaxMaxBlocks (val, idx) pairs followed by one zeroed ticket word
// (one_pass: both passes in one launch, the last workgroup to arrive reducing; it leaves the word zeroed again).
constexpr int kArgmaxMaxBlocks = 1024;
hipError_t launch_argmax(hipStream_t stream, const double* vals, int64_t N, int64_t offset, double* partials,
                         double* result, bool one_pass = false);
// argmax_pass2 alone: nb (value, index) pairs → result {value, index + offset}
hipError_t launch_argmax_reduce(hipStream_t stream, const double* partials, int nb, int64_t offset, double* result);

// Scrambled Sobol' generation (omb_sobol.hip).  The packed state holds the direction
// numbers, shift and box of one engine; sobol_pack_state (omb_host.cpp) fills a host buffer of
// sobol_state_bytes(d, bits) that is then copied to the device.
hipError_t launch_sobol(hipStream_t stream, const void* state_dev, int d, int bits, int64_t start, int64_t N,
                        double* X);

// Dense fp64 linear algebra for Thompson sampling (omb_linalg.hip).  Row-major throughout.
constexpr int64_t kSelectMaxN = 1 << 18;    // candidates per selection (LDS exclusion bitmap)
constexpr int64_t kMaxCovN = 32768;         // candidates of one full posterior covariance
// GEMM tile geometry (omb_gemm.hip; the Cholesky trailing update and K(X*, X*) reuse it)
constexpr int kGT = 64;         // C tile edge
constexpr int kGK = 16;         // k slab
constexpr int kGP = kGT + 2;    // LDS row pitch in doubles (rows 528 B apart: conflict-free stores)
// C (M, Nc) = β·C + α·L·B with L (M, M) lower-triangular: its upper triangle is never read, and slabs past
// each row tile are skipped (half the work of launch_gemm_nn)
hipError_t launch_gemm_ltri_nn(hipStream_t s, int64_t M, int64_t Nc, double alpha, const double* L, int64_t ldl,
                               const double* B, int64_t ldb, double beta, double* C, int64_t ldc);
// C (M, Nc) = β C + α A B, A (M, K), B (K, Nc).
hipError_t launch_gemm_nn(hipStream_t s, int64_t M, int64_t Nc, int64_t K, double alpha, const double* A, int64_t lda,
                          const double* B, int64_t ldb, double beta, double* C, int64_t ldc);
// lower triangle of C (N, N) = β C + α AᵀA, A (K, N).
hipError_t launch_gemm_tn_lower(hipStream_t s, int64_t N, int64_t K, double alpha, const double* A, int64_t lda,
                                double beta, double* C, int64_t ldc);
// lower triangle of K(X*, X*) of one GP's kernel (ℓ, σ_f² from g) at Xc (N, d), diag_add added to the
// diagonal as it is stored (the jitter, without an add_diag launch); ws: cand_cov_ws_doubles device doubles
// (X*/ℓ and its squared norms).
int64_t cand_cov_ws_doubles(int64_t N, int DP);
hipError_t launch_cand_cov(hipStream_t stream, const GPDev& g, int d, int DP, const double* Xc, int64_t N, double* S,
                           int64_t lds, double* ws, double diag_add = 0.0, bool table = false);
// X*/ℓ rows (kp = ⌈DP/4⌉·4 doubles, written to ws) and their squared norms (ws + N·kp), as launch_cand_cov stages
// them; returns kp (0 for DP > kMaxFusedDP: the wide path has its own staging)
int launch_cand_scale(hipStream_t stream, const GPDev& g, int d, int DP, const double* Xc, int64_t N, double* ws,
                      hipError_t* err);
// lower triangle of S = K(X*, X*) + diag_add·I − VᵀV, V (K, N): the covariance SYRK with K(X*, X*) formed in its
// epilogue from launch_cand_scale's rows (omb_gemm.hip gemm_kernel<…, KSS>; glds: syrk_glds_kernel, the three-stage
// direct-to-LDS operand pipeline, where K % 16 = 0 and N, ldv even — bitwise the same C)
// zero_ints (n_zero ints) and zero_info: words the launch's workgroups set to 0 on the side (the next persistent
// Cholesky's sync words and status), so that factorisation needs no init launch
hipError_t launch_cov_syrk(hipStream_t s, int64_t N, int64_t K, const double* V, int64_t ldv, double* S, int64_t lds,
                           const double* xs, const double* xsq, int kp, int kind, double variance, double diag_add,
                           bool glds = true, int* zero_ints = nullptr, int n_zero = 0, int* zero_info = nullptr);
hipError_t launch_mirror_lower(hipStream_t stream, double* S, int64_t N, int64_t lds);
hipError_t launch_add_diag(hipStream_t stream, double* S, int64_t N, int64_t lds, double v);
// in-place lower Cholesky; info (device int, zeroed by the first kernel) = first bad column (1-based);
// ws: chol_ws_doubles(N) device doubles of workspace (the inverse of the current diagonal block, as MFMA
// fragments for the panel product, then one int flag per step).  info = kCholSpinFault: a workgroup's
// wait for the diagonal block ran out after spin_limit polls (the factor is invalid; reported as OMB_EHIP).
constexpr int kCholWsDoubles = 64 * 64;
constexpr int kCholSpinFault = -2147483647;
// kCholBlocked (round 4): the diagonal blocks by tiles of 16 (chol64_blocked); kCholBlockedAcqRel: the same with
// the fused step's flag as an agent-scope release / acquire (tools/ablate/ablate_chol)
// kCholPersistent (round 4): the whole factorisation in one launch (chol_persist_kernel; kCholBlocked when A is too
// large for its 32-bit buffer offsets)
// kCholPersistent: the last min(t, 32) of the t 64-column steps in one persistent launch, the steps before it as
// per-step launches (their trailing updates are faster while the trailing matrix is large; omb_linalg.hip
// chol_hybrid_k0).  kCholAuto (launch_cholesky) = kCholPersistent where A fits its 32-bit buffer offsets, else
// kCholBlocked.
// kCholPersistOnly: the whole factorisation in one persistent launch (k0 = 0; kCholBlocked when A is too large).
enum { kCholTwoLaunch = 0, kCholFused = 1, kCholBlocked = 2, kCholBlockedAcqRel = 3, kCholPersistent = 4, kCholAuto = 5,
       kCholPersistOnly = 6 };
int64_t chol_ws_doubles(int64_t N);
hipError_t launch_cholesky(hipStream_t stream, double* A, int64_t N, int64_t lda, int* info, double* ws,
                           int spin_limit = kDefaultSpinLimit);
// acq_rel = 1: every cross-workgroup hand-off of the schedule as an agent-scope release / acquire pair (the HIP memory
// model's form; the default relaxed / sc1 form is measured valid on gfx950 and checked bitwise against this one).
// single_steps = 1: the persistent launch's workers take every trailing update as its own task (round 5's table; the
// default batches far tiles' updates, bitwise the same factor — checked against this one)
// sync_zeroed: the persistent launch's sync words (chol_persist_sync_words) and info are already zero (written by the
// covariance SYRK of the Thompson chain), so the k0 = 0 persistent launch goes without its init kernel
hipError_t launch_cholesky_mode(hipStream_t stream, double* A, int64_t N, int64_t lda, int* info, double* ws, int mode,
                                int spin_limit = kDefaultSpinLimit, int acq_rel = 0, int single_steps = 0,
                                bool sync_zeroed = false);
int chol_persist_sync_words(double* ws, int64_t N, int** ints);
// Y (B, N) = μ + Zt Lᵀ (L lower, N×N): row b of Y is the sample μ + L z_b.
// ws: chol_samples_ws_doubles(N, B) device doubles (split-K partial products; 0 when unsplit).
int64_t chol_samples_ws_doubles(int64_t N, int B);
hipError_t launch_chol_samples(hipStream_t stream, const double* L, int64_t N, int64_t ldl, const double* mu,
                               const double* Zt, int B, double* Y, double* ws);
// greedy per-sample arg-min (TuRBO select_candidates); ws: select_ws_bytes(B, N) bytes of device memory
// (the sorted heads of every sample when N ≤ kSelectSortN; 0 otherwise).
constexpr int64_t kSelectSortN = 8192;
int64_t select_ws_bytes(int B, int64_t N);
hipError_t launch_select(hipStream_t stream, const double* Y, int B, int64_t N, int64_t* idx, void* ws, bool seq = false);
// C (M, Nc) = β C + α AᵀB, A (K, M), B (K, Nc).
hipError_t launch_gemm_tn(hipStream_t s, int64_t M, int64_t Nc, int64_t K, double alpha, const double* A, int64_t lda,
                          const double* B, int64_t ldb, double beta, double* C, int64_t ldc);
// X (n, n) = L⁻¹ for lower-triangular L; X zeroed by the caller; T: workspace of 64·n doubles.
hipError_t launch_trinv(hipStream_t stream, const double* L, int64_t n, int64_t lda, double* X, int64_t ldx,
                        double* T);
// GP log-marginal-likelihood pieces: out[0..DP] = ½ Σ W ∂K/∂θ (θ = log σ_f², log ℓ_j; entries past
// d are 0), out[DP+1] = Σ log L_ii, out[DP+2] = yᵀα.  partials: gp_grad_blocks(n)·(DP+1) doubles.
int64_t gp_grad_blocks(int64_t n);
// n ≤ 128 and n_var ≤ 8 (gp_lml_small_fits): the whole evaluation in one workgroup (sweep-operator
// inverse in LDS, jitter retries in-kernel); out (DP+5 doubles): the launch_gp_grad layout +
// out[DP+3] = jitter, out[DP+4] = info.
bool gp_lml_small_fits(int n, int DP);
hipError_t launch_gp_lml_small(hipStream_t stream, int kind, int DP, const double* X, int d, int n,
                               const double* ls_host, double variance, double base, const double* y, double* out);
// k ≤ kFitBatchMax problems on the same X (y[p], ls_host[p·d..], variance[p] → out[p]), one workgroup each
constexpr int kFitBatchMax = 4;
hipError_t launch_gp_lml_small_batch(hipStream_t stream, int kind, int DP, const double* X, int d, int n, int k,
                                     const double* const* y, const double* ls_host, const double* variance,
                                     double base, double* const* out);
// dense posterior path: μ, σ² of a candidate chunk from K* (n, Nc) and V = L⁻¹K* (n, Nc).
hipError_t launch_post_colreduce(hipStream_t stream, const double* Kst, const double* V, int64_t n, int64_t Nc,
                                 const double* alpha, double variance, double* mu, double* var,
                                 const GPDev* scale_g = nullptr, int d = 0, int DP = 0, const double* Xc = nullptr,
                                 double* ws = nullptr);   // scale_g: also launch_cand_scale's rows into ws
hipError_t launch_gp_grad(hipStream_t stream, int kind, int DP, const double* X, int d, int64_t n, const double* ls,
                          double variance, const double* alpha, const double* Kinv, int64_t ldk, double* partials,
                          const double* L, int64_t lda, const double* y, double* out);

// ParEGO / KEEP evolutionary acquisition search (omb_ea.hip): one workgroup runs the whole search from a
// host-replayed tape of the reference's random draws.  ldt_ws: n0·n0 doubles (L0⁻¹ transposed).
constexpr int kEAMaxPop = 32;
constexpr int kEAMaxTrain = 2048;
constexpr int kEALdsN = 128;      // L0⁻¹ kept in LDS (packed lower) up to this n_train
struct EASearch {
  GPDev g0, g1;          // g0: the EI model; g1: KEEP's Pareto-membership model (mode 1)
  const double* Ld0;     // dense row-major L0⁻¹ (n0, n0)
  int mode, d, DP, P, iters;
  double best, var_eps;
  const double* pop;
  const int* sel;
  const int8_t* cross;
  const double* beta;
  const int8_t* mut;
  const double* lower;
  const double* upper;
  double* out;
};
hipError_t launch_ea_search(hipStream_t stream, const EASearch& s, double* ldt_ws);

// ---------------------------------------------------------------------------------------
// Wide inputs (omb_wide.hip): n_var 65 .. OMB_MAX_DIM, DP = 128 or 256.  The fused posterior kernel and the
// register-fragment K-block / covariance / gradient kernels hold a candidate's coordinates in registers, which
// is only affordable up to kMaxFusedDP; above it the cross terms run as GEMM tiles with the k loop over slabs of
// kWideSlab dimensions staged in LDS, and the posterior takes the dense path (K block → V = L⁻¹K* → column
// reduction, posterior_any).  Every entry point keeps its meaning and its parity bar.
constexpr int kMaxFusedDP = 64;
constexpr int kWideSlab = 16;
// K (M, N) row-major, pitch ldk: K[i][c] = k(X_i, X*_c) for the training rows of g (pre-scaled g.Xs, g.xsq, pitch
// DP) against the raw candidates Xc (N, d), divided by ℓ as they are staged.
hipError_t launch_kernel_block_wide(hipStream_t stream, const GPDev& g, int d, int DP, const double* Xc, int64_t N,
                                    double* K, int64_t ldk);
// launch_cand_cov for DP > kMaxFusedDP (same arguments and workspace, cand_cov_ws_doubles(N, DP))
hipError_t launch_cand_cov_wide(hipStream_t stream, const GPDev& g, int d, int DP, const double* Xc, int64_t N,
                                double* S, int64_t lds, double* ws, double diag_add);
// gp_grad_kernel's partial sums for DP > kMaxFusedDP (the same layout: gp_grad_blocks(n) blocks × (DP + 1))
hipError_t launch_gp_grad_partials_wide(hipStream_t stream, int kind, int DP, const double* X, int d, int64_t n,
                                        const double* ls, double variance, const double* alpha, const double* Kinv,
                                        int64_t ldk, double* partials);

// Packed-L^-1 size in doubles for R row tiles: Σ_{r<R} 4(r+1)·64 = 128·R·(R+1).
inline int64_t packed_L_size(int R) { return 128ll * R * (R + 1); }
// k-step pairs of the training-row A fragments [x/ℓ, ‖x/ℓ‖², 1]: ⌈⌈(DP+2)/4⌉/2⌉
inline int packed_X_pairs(int DP) { return ((DP + 5) / 4 + 1) / 2; }
inline int64_t packed_X_size(int n_pad, int DP) { return (int64_t)(n_pad / 16) * packed_X_pairs(DP) * 128; }

}  // namespace omb
