/*
 * optimobo_hip.h — C-ABI of liboptimobo_hip.so, the MI355X (gfx950) hot path of
 * OptiMOBO's acquisition maximisation.
 *
 * The reference (aje220/OptiMOBO v0.2.1) is pure Python: its "boundary" is duck typing, not
 * an FFI.  Each entry point below replaces one arithmetic site of the reference (cited
 * file:line, relative to the reference root) and is bound from Python with ctypes
 * (optimobo_amd/_lib.py; INTEGRATION.md shows the binding a maintainer would add).
 *
 * Conventions
 *   - Every array argument named *_dev is a DEVICE pointer owned by the caller (e.g. a torch
 *     tensor's data_ptr()); fp64, C-contiguous.  Small fixed-size vectors (reference point,
 *     weights, bounds, scalarisation parameters) are HOST pointers read during the call.
 *   - Calls are asynchronous on the context's stream (omb_set_stream), except omb_argmax,
 *     omb_synchronize and omb_timing_read, which synchronise.  Device memory is allocated by
 *     omb_create, omb_set_gp, the omb_plan_* calls (geometry) and the fused-chain calls
 *     (workspace, grown on demand); a grow synchronises the stream first.
 *   - Return 0 (OMB_OK) on success or a negative OMB_E* code; omb_last_error() describes the
 *     last failure.  No C++ exception crosses the ABI.
 *   - One context per device; a context is not thread-safe; different contexts are
 *     independent.
 *   - Posterior moments are laid out objective-major: mu_dev[o * ld + i], var_dev likewise.
 */
#ifndef OPTIMOBO_HIP_H
#define OPTIMOBO_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OMB_ABI_VERSION 1
#define OMB_MAX_OBJ 8      /* objectives held by one context */
#define OMB_MAX_DIM 256    /* n_var.  Up to 64 the fused / register-fragment kernels; 65..256 the wide path
                              (DP 128 / 256: GEMM-tiled cross terms over 16-dim slabs, the dense posterior) */
#define OMB_MAX_TRAIN 1024 /* n_train handled by the fused posterior kernel */
#define OMB_MAX_TRAIN_DENSE 16384 /* n_train of the GEMM-based posterior path used above OMB_MAX_TRAIN */

enum {
  OMB_OK = 0,
  OMB_EINVAL = -1,   /* bad argument */
  OMB_EHIP = -2,     /* HIP runtime error */
  OMB_ENOMEM = -3,   /* device allocation failed */
  OMB_ESTATE = -4,   /* objective not set (omb_set_gp) */
  OMB_EUNSUP = -5,   /* size outside what the kernels support */
  OMB_ENOTPD = -6    /* matrix not positive definite (Cholesky), even with the allowed jitter */
};

enum { OMB_KERNEL_MATERN52 = 0, OMB_KERNEL_RBF = 1 };
enum { OMB_EHVI_REFERENCE = 0, OMB_EHVI_TEXTBOOK = 1, OMB_EHVI_SIGMA = 2 };
enum { OMB_EI_PLAIN = 0, OMB_EI_PARETO = 1, OMB_EI_CONSTRAINED = 2 };

/* Scalarisation ids (optimobo/scalarisations.py:37-397) and their params[] layout. */
enum {
  OMB_SCAL_WS = 0,    /* WeightedSum                       params: -            */
  OMB_SCAL_TCH = 1,   /* Tchebicheff                       params: -            */
  OMB_SCAL_ATCH = 2,  /* AugmentedTchebicheff              params: alpha        */
  OMB_SCAL_MTCH = 3,  /* ModifiedTchebicheff               params: alpha        */
  OMB_SCAL_EWC = 4,   /* ExponentialWeightedCriterion      params: p            */
  OMB_SCAL_WN = 5,    /* WeightedNorm                      params: p            */
  OMB_SCAL_WPO = 6,   /* WeightedPower                     params: p            */
  OMB_SCAL_WPR = 7,   /* WeightedProduct                   params: -            */
  OMB_SCAL_PBI = 8,   /* PBI                               params: theta        */
  OMB_SCAL_IPBI = 9,  /* IPBI                              params: theta        */
  OMB_SCAL_QPBI = 10, /* QPBI                              params: theta, alpha, H */
  OMB_SCAL_APD = 11   /* APD                               params: FE, FE_max, gamma */
};

typedef struct omb_ctx omb_ctx;

int omb_abi_version(void);

/* Create a context on HIP device `device` (own non-blocking stream). */
int omb_create(int device, omb_ctx** out);
int omb_destroy(omb_ctx* ctx);
/* Run subsequent calls on `hip_stream` (a hipStream_t, e.g. torch's current stream;
 * NULL is the HIP null stream).  omb_use_own_stream restores the context's own stream. */
int omb_set_stream(omb_ctx* ctx, void* hip_stream);
int omb_use_own_stream(omb_ctx* ctx);
int omb_synchronize(omb_ctx* ctx);
const char* omb_last_error(const omb_ctx* ctx);

/* Device fault word.  The fused posterior kernel's waves hand K* chunks to each other through
 * LDS counters; every wait is bounded (by default 2^22 polls).  A wait that runs out — which
 * only a broken invariant can cause — marks the context's fault word (pinned host memory) and
 * lets the kernel finish.  The next call on the context that enters the library (and
 * omb_synchronize after its sync) then returns OMB_EHIP once, describing the fault: the moments
 * and acquisition values computed since the previous report are invalid.
 * The same bound limits the fused Cholesky steps' wait for the diagonal block (omb_cholesky,
 * omb_posterior_samples, the GP fit above n = 128): running out returns OMB_EHIP from that call.
 * omb_debug_set(ctx, OMB_DEBUG_SPIN_LIMIT, polls) changes the bound (tests force the path with 0).
 * omb_debug_set(ctx, OMB_DEBUG_COV_TABLE, 1) builds K(X, X) / K(X*, X*) (GP-fit state, posterior covariance) with
 * the posterior kernels' table-driven Matern transform instead of the polynomial exp (a parity check of that
 * transform near r = 0; default 0).
 * omb_debug_set(ctx, OMB_DEBUG_FUSED_CHAIN, m) picks how omb_eval_argmax[_sobol] with an EHVI-2D plan runs the
 * acquisition and the arg-max: 0 the EHVI launch, then the arg-max's passes; 1 one launch (the last workgroup at
 * an agent-scope ticket reduces: the ticket's same-address atomics serialise, 23 vs 13.5 µs at config 2);
 * 2 the EHVI launch reducing to one pair per workgroup, then the arg-max's second pass.  Bit-identical pair.
 * omb_debug_set(ctx, OMB_DEBUG_ARGMAX_PASSES, 1) runs the arg-max as one launch (the last workgroup to finish
 * reduces the per-workgroup pairs) instead of two (default 2: config 2 measured 719.6 vs 719.5 M candidates/s,
 * gpurun_out/r04_l; bit-identical pair).
 * omb_debug_set(ctx, OMB_DEBUG_CHOL_MODE, m) picks the Cholesky schedule of omb_cholesky / omb_posterior_samples /
 * omb_gp_fit_state: 0 auto (default: where A fits the persistent launch's 32-bit buffer offsets, the whole
 * factorisation in one persistent launch — round 5 ran per-step launches for all but the last 32 steps first; else 1),
 * 1 one launch per step, 2 the persistent launch whatever the size; m + 4 runs schedule m with every cross-workgroup hand-off
 * an agent-scope release / acquire pair (the HIP memory model's guarantee; the default form — sc1 payloads, a vmcnt
 * wait and relaxed flags — is measured valid on gfx950), bitwise the same factor as schedule m; m + 8 has the persistent
 * launch's workers apply every trailing update as its own task instead of batching the far tiles' updates (round 5's
 * schedule), again bitwise the same factor.
 * omb_debug_set(ctx, OMB_DEBUG_TIMING_STRIDE, s) records omb_timing's events on every s-th chain only (default 1;
 * omb_timing_read then averages over the recorded chains), so that a timed loop carries fewer event records. *
 * Value 7 (round 5's OMB_DEBUG_POSTERIOR_PERSIST, a persistent-ring posterior kernel measured 2-5% slower at every
 * configuration) is retired: the library has one posterior kernel per shape, and omb_debug_set(ctx, 7, ·) fails.
 * omb_debug_set(ctx, OMB_DEBUG_COV_FUSED, 0) builds the posterior covariance as K(X*, X*) then the VᵀV update (two
 * launches) instead of one SYRK with K(X*, X*) in its epilogue (default 1; the same matrix to the ulp).
 * omb_debug_set(ctx, OMB_DEBUG_SELECT_SEQ, 1) makes omb_thompson_select walk the samples in order for B ≤ 64 too
 * (default 0: the picks in parallel rounds to their fixed point; the same picks).
 * omb_debug_set(ctx, OMB_DEBUG_SYRK_GLDS, 0) builds the posterior covariance's SYRK with the register-staged two-slab
 * pipeline instead of the three-stage direct-to-LDS one (default 1 where n_train % 16 = 0 and N is even; the same
 * matrix bit for bit). */
enum {
  OMB_DEBUG_SPIN_LIMIT = 1,
  OMB_DEBUG_COV_TABLE = 2,
  OMB_DEBUG_FUSED_CHAIN = 3,
  OMB_DEBUG_ARGMAX_PASSES = 4,
  OMB_DEBUG_CHOL_MODE = 5,
  OMB_DEBUG_TIMING_STRIDE = 6,
  OMB_DEBUG_COV_FUSED = 8,
  OMB_DEBUG_SELECT_SEQ = 9,
  OMB_DEBUG_SYRK_GLDS = 10
};
int omb_debug_set(omb_ctx* ctx, int what, int64_t value);

/* Fitted-GP state of objective `obj` — replaces the fitted GPy model
 * (GPRegression + Matern52(ARD) with noise fixed to 0, optimisers.py:223-231).
 *   X_dev     (n, d)  training inputs, unscaled
 *   lengthscale_host (d) ARD lengthscales ℓ;  variance = σ_f²
 *   alpha_dev (n)     woodbury vector (K + 1e-8 I)^-1 y
 *   Linv_dev  (n, n)  row-major inverse of the lower Cholesky factor of K + 1e-8 I
 * The context packs this into its own layout (Lp: MFMA-fragment order) on its stream. */
int omb_set_gp(omb_ctx* ctx, int obj, int kernel, int n, int d, const double* X_dev,
               const double* lengthscale_host, double variance, const double* alpha_dev,
               const double* Linv_dev);

/* K(X_train, X*) block of objective `obj` (GPy Stationary._scaled_dist + Matern52.K_of_r,
 * the first half of model.predict at util_functions.py:156): K_dev (n, N) row-major. */
int omb_kernel_block(omb_ctx* ctx, int obj, const double* Xc_dev, int64_t N, double* K_dev);

/* Posterior μ, σ² of objectives 0..n_obj-1 at N candidates Xc_dev (N, d)
 * (GPy PosteriorExact._raw_predict via model.predict, util_functions.py:155-158):
 * mu_dev/var_dev (n_obj, N).  Fused K-block generation + FP64-MFMA L^-1 K* + reductions for
 * n_train ≤ OMB_MAX_TRAIN; above it (≤ OMB_MAX_TRAIN_DENSE) candidate chunks go through the K block,
 * an FP64-MFMA GEMM V = L^-1 K* and a column reduction. */
int omb_posterior(omb_ctx* ctx, int n_obj, const double* Xc_dev, int64_t N, double* mu_dev,
                  double* var_dev);

/* EHVI for 2 objectives (util_functions.py:136-167 + EHVI_2D_aux :81-128).
 *   pf_sorted_dev (P, 2): Pareto front sorted by f2 ascending (util_functions.py:98)
 *   r_host (2): reference (max) point;  s00, s01: np.cov(cache) entries (per-solve constants)
 *   mode OMB_EHVI_REFERENCE: σA = σ²0·s00, σB = σ²0·s01, last stripe omitted (bug-compatible)
 *   mode OMB_EHVI_TEXTBOOK : σA = sqrt(σ²0), σB = sqrt(σ²1), all P+1 stripes (exact EHVI)
 *   mode OMB_EHVI_SIGMA    : var_dev holds (σA, σB) directly — EHVI_2D_aux(PF, r, μ, σ) itself */
int omb_ehvi2d(omb_ctx* ctx, const double* mu_dev, const double* var_dev, int64_t ld, int64_t N,
               const double* pf_sorted_dev, int P, const double* r_host, double s00, double s01,
               int mode, double* out_dev);

/* EHVI_3D reference Monte-Carlo form (util_functions.py:170-214):
 *   out = mean_s max(0, Π_j(r_j − s_j) − hv_pf),  s = cache·sqrt(σ²0) + μ (util_functions.py:217-237)
 * raised_dev (N, int32, may be NULL) is set to 1 where pygmo's hypervolume would raise
 * (a sample outside the reference box); out is NaN there. */
int omb_ehvi3d_mc(omb_ctx* ctx, const double* mu_dev, const double* var_dev, int64_t ld, int64_t N,
                  const double* cache_dev, int M, const double* r_host, double hv_pf, double* out_dev,
                  int32_t* raised_dev);
/* The same Monte-Carlo EHVI for any 2 ≤ k ≤ OMB_MAX_OBJ objectives (omb_ehvi3d_mc is k = 3): the
 * reference calls EHVI_3D for every n_obj != 2 (optimisers.py:245-248), and EHVI_3D's per-sample volume
 * is pygmo's k-D hypervolume([s]).compute(r) = Π_{j<k}(r_j − s_j) (util_functions.py:205-206; the 3-term
 * product of :204 is overwritten).  cache_dev (M, k) row-major, r_host (k), hv_pf = HV(PF, r) in k-D;
 * k·M ≤ 8192 (the cache is staged in LDS). */
int omb_ehvi_mc(omb_ctx* ctx, int k, const double* mu_dev, const double* var_dev, int64_t ld, int64_t N,
                const double* cache_dev, int M, const double* r_host, double hv_pf, double* out_dev,
                int32_t* raised_dev);

/* Exact ("textbook") EHVI for k = 2 or 3 objectives — the exact value the Monte-Carlo
 * EHVI_3D (util_functions.py:170-214) estimates — from a disjoint box decomposition of the
 * non-dominated region (optimobo_amd.pareto.box_decomposition):
 *   coords_dev (k, C) f64: per objective a sorted grid [-inf, front values..., r_j] (padded)
 *   boxes_dev  (B, 2k) uint16: [lo_0, hi_0, lo_1, hi_1, ...] grid indices of each box
 *   EHVI = Σ_b Π_j E[(hi_j − max(Y_j, lo_j))⁺],  Y_j ~ N(μ_j, σ²_j) independent.
 * One wavefront per candidate; 9·k·C ≤ 8192 (grid and per-wave Φ/φ tables in LDS). */
int omb_ehvi_boxes(omb_ctx* ctx, int k, const double* mu_dev, const double* var_dev, int64_t ld, int64_t N,
                   const double* coords_dev, int C, const uint16_t* boxes_dev, int B, double* out_dev);

/* Hypervolume-based PoI of EMO (emo.py:176-228): cells_dev (C, 2, 2) [upper, lower]. */
int omb_hvpoi(omb_ctx* ctx, const double* mu_dev, const double* var_dev, int64_t ld, int64_t N,
              const double* cells_dev, int C, double* out_dev);

/* expected_decomposition (util_functions.py:285-327) for k objectives:
 *   cache_dev (M, k); weights/ideal/max host (k); params_host per OMB_SCAL_* (may be NULL). */
int omb_expdec(omb_ctx* ctx, int k, const double* mu_dev, const double* var_dev, int64_t ld, int64_t N,
               const double* cache_dev, int M, int scal_id, const double* params_host,
               const double* weights_host, const double* ideal_host, const double* max_host,
               double agg_min, double* out_dev);

/* Expected improvement (optimisers.py:325-344 with var_eps = 0; parego.py:126-145 and
 * keep.py:118-137 with var_eps = 1e-6). */
int omb_ei(omb_ctx* ctx, const double* mu_dev, const double* var_dev, int64_t N, double best,
           double var_eps, double* out_dev);
/* EI and its products with further models, over k posterior rows (row o at mu_dev + o·ld):
 *   OMB_EI_PLAIN       k = 1   EI(μ0, σ²0 + var_eps)                              (= omb_ei)
 *   OMB_EI_PARETO      k = 2   μ1 · EI(μ0, σ²0 + var_eps), var_eps = 1e-6 in the reference:
 *                              KEEP.pareto_expected_improvement (keep.py:118-151), row 1 = the
 *                              Pareto-membership model
 *   OMB_EI_CONSTRAINED k ≥ 2   EI(μ0, σ²0 + var_eps) · Π_{c=1}^{k-1} Φ(−μc / sqrt(σ²c + pof_eps)),
 *                              var_eps = 0, pof_eps = 1e-5 in the reference:
 *                              ParEGO_C2.consraint_ei (cparego.py:450-496), rows 1.. = constraints */
int omb_ei_ext(omb_ctx* ctx, int kind, int k, const double* mu_dev, const double* var_dev, int64_t ld, int64_t N,
               double best, double var_eps, double pof_eps, double* out_dev);

/* Arg-max over vals_dev (N): lowest index among maxima, NaN and -inf never win
 * (replaces scipy differential_evolution(lambda x: -acq(x)), optimisers.py:87,118).
 * result_dev (2 doubles, device): {best value, best index + offset (as double)};
 * index -1 when nothing qualifies.  Asynchronous. */
int omb_argmax_dev(omb_ctx* ctx, const double* vals_dev, int64_t N, int64_t offset, double* result_dev);
/* Same, synchronising and returning to host. */
int omb_argmax(omb_ctx* ctx, const double* vals_dev, int64_t N, int64_t offset, double* best_val,
               int64_t* best_idx);

/* ---------------------------------------------------------------------------------------
 * Fused chain.  One BO iteration of the reference calls
 *   differential_evolution(lambda x: -acq(x, models, ...), bounds)      (optimisers.py:87,118)
 * where acq is fixed for the iteration.  Here the acquisition and its per-iteration geometry
 * are uploaded once as a *plan* (HOST pointers, copied into context-owned device memory; the
 * call synchronises the stream first), then each candidate batch is one call that runs
 * posterior (objectives 0..k-1) → acquisition → arg-max on the stream, with the moments in a
 * context-owned workspace (grown on demand).  Setting a plan replaces the previous one; a
 * failed plan call leaves no plan (OMB_ESTATE from the eval calls).
 * ------------------------------------------------------------------------------------- */
/* util_functions.EHVI / EHVI_2D_aux (k = 2): as omb_ehvi2d, pf_sorted_host (P, 2). */
int omb_plan_ehvi2d(omb_ctx* ctx, const double* pf_sorted_host, int P, const double* r_host, double s00,
                    double s01, int mode);
/* util_functions.EHVI_3D reference Monte-Carlo form (k = 3): as omb_ehvi3d_mc, cache_host (M, 3). */
int omb_plan_ehvi3d_mc(omb_ctx* ctx, const double* cache_host, int M, const double* r_host, double hv_pf);
/* EHVI_3D's Monte-Carlo form for k objectives (2 ≤ k ≤ OMB_MAX_OBJ): as omb_ehvi_mc, cache_host (M, k). */
int omb_plan_ehvi_mc(omb_ctx* ctx, int k, const double* cache_host, int M, const double* r_host, double hv_pf);
/* Exact EHVI (k = 2, 3): as omb_ehvi_boxes, coords_host (k, C), boxes_host (B, 2k). */
int omb_plan_ehvi_boxes(omb_ctx* ctx, int k, const double* coords_host, int C, const uint16_t* boxes_host, int B);
/* EMO hypervolume-based PoI (k = 2): as omb_hvpoi, cells_host (C, 2, 2). */
int omb_plan_hvpoi(omb_ctx* ctx, const double* cells_host, int C);
/* expected_decomposition (k objectives): as omb_expdec, cache_host (M, k). */
int omb_plan_expdec(omb_ctx* ctx, int k, const double* cache_host, int M, int scal_id, const double* params_host,
                    const double* weights_host, const double* ideal_host, const double* max_host, double agg_min);
/* Expected improvement of objective 0 (k = 1): as omb_ei. */
int omb_plan_ei(omb_ctx* ctx, double best, double var_eps);
/* EI family over objectives 0..k-1: as omb_ei_ext. */
int omb_plan_ei_ext(omb_ctx* ctx, int kind, int k, double best, double var_eps, double pof_eps);

/* Scrambled Sobol' candidates generated on the device (replaces the host-side sampling that
 * feeds the maximiser; same sequence as scipy.stats.qmc.Sobol, which the reference uses for
 * its MC cache at optimisers.py:121-141).  sv_host (d, bits) and shift_host (d) are the
 * engine's scrambled direction numbers and digital shift (scipy: Sobol._sv, Sobol._shift);
 * point i of the engine, mapped to the box, is
 *   x_ij = lo_j + u_ij (hi_j − lo_j),  u_ij = (shift_j ⊕ ⨁_{b ∈ gray(i)} sv_jb) · 2^-bits,
 * bit-identical to numpy's `lo + U * (hi - lo)` on scipy's U.  bits ≤ 32, d ≤ OMB_MAX_DIM. */
int omb_set_sobol(omb_ctx* ctx, int d, int bits, const uint32_t* sv_host, const uint32_t* shift_host,
                  const double* lo_host, const double* hi_host);
/* Points start .. start+N-1 → X_dev (N, d). */
int omb_sobol(omb_ctx* ctx, int64_t start, int64_t N, double* X_dev);

/* Acquisition values of the plan at candidates Xc_dev (N, d) → vals_dev (N). */
int omb_eval(omb_ctx* ctx, const double* Xc_dev, int64_t N, double* vals_dev);
/* posterior → plan → arg-max: result_dev = {best value, best index + offset} (see omb_argmax_dev). */
int omb_eval_argmax(omb_ctx* ctx, const double* Xc_dev, int64_t N, int64_t offset, double* result_dev);
/* Same over the Sobol' points start .. start+N-1 generated into the workspace; the index in
 * result_dev is the Sobol index (offset = start). */
int omb_eval_argmax_sobol(omb_ctx* ctx, int64_t start, int64_t N, double* result_dev);

/* Device timing of the fused chain (HIP events on the context's stream), up to 4096 chains.
 * omb_timing(ctx, level): 0 off; 1 the posterior stage only (2 events per chain); 2 every
 * stage (5 events; each record costs a few µs of GPU time).  omb_timing_read synchronises
 * and returns the summed milliseconds of {Sobol generation, posterior, acquisition, arg-max}
 * (0 for stages not recorded) over the chains recorded since the last read, and their count.
 * Changing the level discards unread records. */
int omb_timing(omb_ctx* ctx, int enable);
int omb_timing_read(omb_ctx* ctx, double* stage_ms /* [4] */, int64_t* chains);

/* ---------------------------------------------------------------------------------------
 * Thompson sampling — TuRBO's candidate scoring (turbo.py:75-117 create_candidates,
 * turbo.py:142-153 / 365-383 candidate selection).  The reference draws `batch_size` joint
 * samples with GPy's GP.posterior_samples(X_cand, size) (turbo.py:114): a full posterior
 * covariance (PosteriorExact._raw_predict, full_cov=True) and numpy's multivariate_normal
 * (SVD).  Here: Σ on FP64 MFMA, a blocked Cholesky of Σ + jitter·I, samples μ + L z.
 * ------------------------------------------------------------------------------------- */
/* μ (N) and the full symmetric posterior covariance cov_dev (N, N) of objective `obj` at Xc_dev
 * (N, d):  Σ = K(X*, X*) − (L⁻¹K*)ᵀ(L⁻¹K*)  (GPy _raw_predict(full_cov=True) + σ_n² = 0).
 * N ≤ 32768.  Asynchronous. */
int omb_posterior_cov(omb_ctx* ctx, int obj, const double* Xc_dev, int64_t N, double* mu_dev, double* cov_dev);
/* In-place lower Cholesky factor of A + jitter·I (A_dev (N, N) row-major with leading dimension
 * lda; the lower triangle is read and overwritten, the upper triangle is left untouched —
 * LAPACK dpotrf('L') on the row-major lower triangle).  Synchronises; *info = 0 on success,
 * else the 1-based column of the first non-positive pivot (dpotrf's info). */
int omb_cholesky(omb_ctx* ctx, double* A_dev, int64_t N, int64_t lda, double jitter, int* info);
/* B joint posterior samples of objective `obj` at Xc_dev (N, d) (GPy posterior_samples_f):
 *   Y_dev (B, N) row b = μ + L z_b,  L = chol(Σ + j I),  Zt_dev (B, N) standard normals z_b.
 * Try t = 0 .. max_tries-1 uses j = jitter_rel · σ_f² · 10^t until the factorisation succeeds
 * (OMB_ENOTPD otherwise); *jitter_used (may be NULL) receives the j used.  Synchronises.  When the call fails after
 * the draws were queued (OMB_ENOTPD, or OMB_EHIP from a factor wait that ran out), Y_dev is filled with NaN. */
int omb_posterior_samples(omb_ctx* ctx, int obj, const double* Xc_dev, int64_t N, const double* Zt_dev, int B,
                          double jitter_rel, int max_tries, double* Y_dev, double* jitter_used);
/* Greedy selection of TuRBO_1.select_candidates (turbo.py:142-153) / TuRBO_M._select_candidates
 * (turbo.py:365-383): for b = 0 .. B-1, idx_dev[b] = np.argmin over row b of Y_dev (B, N)
 * (first NaN, else the lowest index among minima), every earlier pick reading as +inf
 * (the reference sets y_cand[pick, :] = inf).  N ≤ 2^18.  Y is not modified.  Asynchronous. */
int omb_thompson_select(omb_ctx* ctx, const double* Y_dev, int B, int64_t N, int64_t* idx_dev);

/* ---------------------------------------------------------------------------------------
 * ParEGO / KEEP evolutionary acquisition search (parego.py:223-271, keep.py:240-292): the
 * reference's steady-state GA over a temporary population (20: mutants of archive members + Latin
 * hypercube points), 1,000 generations of binary tournaments without replacement (parego.py:78-111),
 * simulated binary crossover (:58-75) and ×1.05 / ×0.95 mutation (:37-56), the child replacing the
 * first parent unless the parent is strictly fitter; the proposal is the best individual seen at the
 * start of any generation (initially `lower` with fitness 0).  Fitness of objective 0's model:
 *   OMB_EA_EI         EI(μ0, σ = sqrt(σ²0 + var_eps))                  ParEGO (var_eps 1e-6)
 *   OMB_EA_PARETO_EI  μ1 · EI(μ0, ...) with objective 1 the Pareto-membership model   KEEP
 * The random draws come as a tape replayed on the host in the reference's call order (see
 * optimobo_amd/ea.py): sel_dev (iters, 4) int32 — tournament 1's random.sample over range(1, P),
 * tournament 2's over range(1, P − 1) (indices into the population without the first winner; the
 * caller guarantees these ranges); cross_dev (iters) int8 crossover flags; beta_dev (iters, d) the
 * crossover β per gene; mut_dev (iters, d) int8 mutation codes (0 none, 1 ×1.05, 2 ×0.95).
 * pop_dev (P, d), lower_dev / upper_dev (d), out_dev (d + 1) = best x, best fitness.  3 ≤ P ≤ 32,
 * n_train ≤ 2048.  One workgroup runs the search.  Asynchronous. */
enum { OMB_EA_EI = 0, OMB_EA_PARETO_EI = 1 };
int omb_ea_search(omb_ctx* ctx, int mode, double best, double var_eps, const double* pop_dev, int P, int iters,
                  const int32_t* sel_dev, const int8_t* cross_dev, const double* beta_dev, const int8_t* mut_dev,
                  const double* lower_dev, const double* upper_dev, double* out_dev);

/* ---------------------------------------------------------------------------------------
 * GP fit on the device — GPy GPRegression(X, y, Matern52(d, ARD=True)) with the noise variance
 * fixed (optimisers.py:223-231 and every other driver's fit): exact inference with GPy's jitchol
 * (Ky = K + (σ_n² + 1e-8) I; on failure + mean(diag Ky)·1e-6·10^t, t < 5), the log marginal
 * likelihood and its gradient for the hyperparameter search.  X_dev (n, d), y_dev (n) device.
 * ------------------------------------------------------------------------------------- */
/* *lml = log p(y | X, θ) = −½ yᵀα − Σ log L_ii − ½ n log 2π;  grad_host (d + 1) = ∂ lml / ∂(log σ_f²,
 * log ℓ_1 .. log ℓ_d);  *jitter_used (may be NULL) = jitchol's extra jitter.  n ≤ 16384.
 * Synchronises.  OMB_ENOTPD when even the jittered matrix is not positive definite. */
int omb_gp_lml_grad(omb_ctx* ctx, int kernel, int n, int d, const double* X_dev, const double* y_dev,
                    const double* lengthscale_host, double variance, double noise, double* lml, double* grad_host,
                    double* jitter_used);
/* k ≤ 4 GPs on the same inputs at once (the drivers fit one GP per objective on the same X;
 * optimisers.py:186): problem p has targets y_dev[p] (device pointer, n), lengthscales
 * lengthscale_host[p·d .. p·d + d − 1] and variance_host[p]; its results go to lml[p], grad_host[p·(d+1) ..],
 * jitter_used[p] (may be NULL) and status[p] (OMB_OK or OMB_ENOTPD, per problem: one non-positive-definite
 * problem does not fail the others).  Each problem's results are exactly omb_gp_lml_grad's: for n ≤ 96
 * and n_var ≤ 8 they run as one launch (one workgroup each) and one synchronisation, otherwise one after
 * another through omb_gp_lml_grad.  Replaces GPy
 * model.optimize's per-objective evaluations (optimisers.py:231).  Returns OMB_OK unless an argument or the
 * device call fails. */
int omb_gp_lml_grad_batch(omb_ctx* ctx, int kernel, int k, int n, int d, const double* X_dev,
                          const double* const* y_dev, const double* lengthscale_host, const double* variance_host,
                          double noise, double* lml, double* grad_host, double* jitter_used, int* status);
/* Fit the exact-inference state of objective `obj` on the device (Cholesky, L⁻¹, α) and install
 * it as omb_set_gp would — the device replacement for the host O(n³) factorisation. */
int omb_gp_fit_state(omb_ctx* ctx, int obj, int kernel, int n, int d, const double* X_dev, const double* y_dev,
                     const double* lengthscale_host, double variance, double noise, double* jitter_used);

#ifdef __cplusplus
}
#endif

#endif /* OPTIMOBO_HIP_H */
