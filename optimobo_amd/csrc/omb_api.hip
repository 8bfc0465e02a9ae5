// C-ABI of liboptimobo_hip.so (declared in include/optimobo_hip.h): context, GP state,
// argument validation and dispatch to the kernels.  No exception crosses this boundary.
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <new>
#include <string>
#include <vector>

#include "omb_internal.h"

using namespace omb;

struct ObjState {
  bool set = false;
  int n = 0, d = 0, DP = 0, R = 0, n_pad = 0, kind = 0;
  double variance = 0.0;
  double* buf = nullptr;  // one allocation: Xs | xsq | alpha | ls | Lp | Ld
  size_t cap = 0;         // bytes
  const double* Ld = nullptr;  // dense row-major L⁻¹ (n, n): the full-covariance path's GEMM operand
  GPDev dev{};
};

// Acquisition of the fused chain (omb_plan_*), with its geometry resident in ctx->geo.
enum PlanKind { PLAN_NONE = 0, PLAN_EHVI2D, PLAN_EHVI_MC, PLAN_EHVI_BOXES, PLAN_HVPOI, PLAN_EXPDEC, PLAN_EI };

struct Plan {
  int kind = PLAN_NONE;
  int k = 0;                    // objectives the acquisition reads (posterior of 0..k-1)
  int P = 0, M = 0, C = 0, B = 0, mode = 0;
  double r[OMB_MAX_OBJ] = {};
  double s00 = 0, s01 = 0, hv = 0, best = 0, var_eps = 0, pof_eps = 0;
  int ei_kind = OMB_EI_PLAIN;
  ScalParams sp{};
  const double* geo = nullptr;  // pf / cache / coords / cells on the device
  const uint16_t* boxes = nullptr;
};

struct omb_ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  std::string err;
  ObjState obj[OMB_MAX_OBJ];
  double* partials = nullptr;  // argmax pass-1 output
  double* result_dev = nullptr;
  double* result_host = nullptr;  // pinned
  int* info_host = nullptr;       // pinned: the Cholesky status read back by run_cholesky / chol_wait
  // fused chain
  Plan plan;
  void* geo = nullptr;    // device: plan geometry
  size_t geo_cap = 0;
  void* stage = nullptr;  // pinned host staging of uploads
  size_t stage_cap = 0;
  void* work = nullptr;   // device: mu | var | vals | raised | X of the fused chain
  size_t work_cap = 0;
  void* sob = nullptr;    // device: packed Sobol state (fixed capacity)
  int sob_d = 0, sob_bits = 0;
  // timing of the fused chain: 5 events per chain (level 2) or 2 around the posterior (level 1)
  int timing = 0;
  int timing_stride = 1;     // OMB_DEBUG_TIMING_STRIDE: events on every stride-th chain only
  int64_t timing_calls = 0;  // chains since omb_timing
  std::vector<hipEvent_t> ev;
  size_t ev_used = 0;
  // Thompson sampling: K* | V | μ | σ² | Σ workspace, and Cholesky info + step counters
  void* tws = nullptr;
  size_t tws_cap = 0;
  void* ichol = nullptr;
  size_t ichol_cap = 0;
  // Thompson selection: per-sample sorted heads (select_sort_kernel)
  void* sws = nullptr;
  size_t sws_cap = 0;
  // evolutionary search: L0⁻¹ transposed
  void* ews = nullptr;
  size_t ews_cap = 0;
  // GP fit: Ky | L⁻¹ | Ky⁻¹ | scratch workspace
  void* fws = nullptr;
  size_t fws_cap = 0;
  // dense posterior path (n_train > OMB_MAX_TRAIN): K* | V chunk workspace
  void* dws = nullptr;
  size_t dws_cap = 0;
  // device fault word (pinned, mapped host memory): kernels mark it, enter() reports it
  int* fault_host = nullptr;
  int* fault_dev = nullptr;
  // GP-fit results (omb_gp_lml_grad): pinned, host-mapped; the one-workgroup kernel stores into it
  // directly (no D2H copy on the per-evaluation path), the blocked path copies into it
  double* fit_host = nullptr;
  double* fit_dev = nullptr;
  int spin_limit = kDefaultSpinLimit;
  bool cov_table = false;   // OMB_DEBUG_COV_TABLE
  bool cov_fused = true;    // OMB_DEBUG_COV_FUSED: K(X*, X*) in the covariance SYRK's epilogue
  bool syrk_glds = true;    // OMB_DEBUG_SYRK_GLDS: the covariance SYRK's direct-to-LDS operand pipeline
  int fused_chain = 0;  // OMB_DEBUG_FUSED_CHAIN: 0 EHVI-2D then the arg-max's passes, 1 one ticketed launch, 2 EHVI
                        // with the per-workgroup pairs, then the arg-max's second pass
  bool argmax_one_pass = false;  // OMB_DEBUG_ARGMAX_PASSES: 1 (one launch) or 2 (default: measured level)
  int chol_mode = kCholAuto;     // OMB_DEBUG_CHOL_MODE (value & 3)
  int chol_acq_rel = 0;          // OMB_DEBUG_CHOL_MODE (value & 4): release / acquire hand-offs
  int chol_single = 0;           // OMB_DEBUG_CHOL_MODE (value & 8): every trailing update its own task
  bool select_seq = false;       // OMB_DEBUG_SELECT_SEQ: the sequential greedy walk for B ≤ 64 too
};

namespace {

int fail(omb_ctx* ctx, int code, const char* fmt, ...) {
  if (ctx) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    ctx->err = buf;
  }
  return code;
}

int hip_fail(omb_ctx* ctx, hipError_t e, const char* where) {
  return fail(ctx, OMB_EHIP, "%s: %s", where, hipGetErrorString(e));
}

#define OMB_HIP(ctx, call)                                   \
  do {                                                       \
    hipError_t e_ = (call);                                  \
    if (e_ != hipSuccess) return hip_fail(ctx, e_, #call);   \
  } while (0)

// Reports (once) a fault a kernel marked since the last report.
int check_fault(omb_ctx* ctx) {
  const int f = __atomic_exchange_n(ctx->fault_host, 0, __ATOMIC_ACQ_REL);
  if (f & kFaultSpin)
    return fail(ctx, OMB_EHIP, "posterior kernel: an LDS counter-ring wait exceeded %d polls; the posterior "
                "moments (and acquisition values) computed since the previous call are invalid", ctx->spin_limit);
  return OMB_OK;
}

int enter(omb_ctx* ctx) {
  if (!ctx) return OMB_EINVAL;
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
  return check_fault(ctx);
}

// GPArgs of the posterior launches: zeroed, with the context's fault word and spin bound.
void init_args(omb_ctx* ctx, GPArgs* args) {
  memset(args, 0, sizeof(*args));
  args->fault = ctx->fault_dev;
  args->spin_limit = ctx->spin_limit;
}

// GP state of objectives 0..n_obj-1, all set, sharing d.
int gather_gp(omb_ctx* ctx, int n_obj, GPArgs* args, int* max_R) {
  if (n_obj < 1 || n_obj > OMB_MAX_OBJ) return fail(ctx, OMB_EINVAL, "n_obj=%d outside [1, %d]", n_obj, OMB_MAX_OBJ);
  init_args(ctx, args);
  *max_R = 0;
  for (int o = 0; o < n_obj; ++o) {
    const ObjState& s = ctx->obj[o];
    if (!s.set) return fail(ctx, OMB_ESTATE, "objective %d has no GP state (call omb_set_gp)", o);
    if (s.d != ctx->obj[0].d) return fail(ctx, OMB_EINVAL, "objectives disagree on n_var (%d vs %d)", s.d, ctx->obj[0].d);
    if (s.kind != ctx->obj[0].kind) return fail(ctx, OMB_EINVAL, "objectives disagree on kernel kind");
    args->gp[o] = s.dev;
    if (s.R > *max_R) *max_R = s.R;
  }
  args->d = ctx->obj[0].d;
  args->DP = ctx->obj[0].DP;
  return OMB_OK;
}

// The context's error sink for the host-only checks (omb_host.cpp).
std::string* E(omb_ctx* ctx) { return ctx ? &ctx->err : nullptr; }

// ---- ctx-owned buffers
int grow_dev(omb_ctx* ctx, void** buf, size_t* cap, size_t bytes, const char* what) {
  if (bytes <= *cap) return OMB_OK;
  OMB_HIP(ctx, hipStreamSynchronize(ctx->stream));  // queued kernels may still read the old buffer
  if (*buf) (void)hipFree(*buf);
  *buf = nullptr;
  *cap = 0;
  if (hipMalloc(buf, bytes) != hipSuccess) return fail(ctx, OMB_ENOMEM, "hipMalloc(%zu) for %s", bytes, what);
  *cap = bytes;
  return OMB_OK;
}

// Pinned staging for a host→device upload of `bytes`; the previous upload is complete on return.
int stage_begin(omb_ctx* ctx, size_t bytes, void** host) {
  OMB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (bytes > ctx->stage_cap) {
    if (ctx->stage) (void)hipHostFree(ctx->stage);
    ctx->stage = nullptr;
    ctx->stage_cap = 0;
    if (hipHostMalloc(&ctx->stage, bytes, hipHostMallocDefault) != hipSuccess)
      return fail(ctx, OMB_ENOMEM, "hipHostMalloc(%zu) for staging", bytes);
    ctx->stage_cap = bytes;
  }
  *host = ctx->stage;
  return OMB_OK;
}

// Uploads the staged bytes as the plan geometry.
int stage_to_geo(omb_ctx* ctx, size_t bytes) {
  int rc = grow_dev(ctx, &ctx->geo, &ctx->geo_cap, bytes, "plan geometry");
  if (rc) return rc;
  OMB_HIP(ctx, hipMemcpyAsync(ctx->geo, ctx->stage, bytes, hipMemcpyHostToDevice, ctx->stream));
  return OMB_OK;
}

int plan_begin(omb_ctx* ctx, size_t bytes, void** host) {
  int rc = enter(ctx);
  if (rc) return rc;
  ctx->plan = Plan();  // an invalid request leaves no plan behind
  return bytes ? stage_begin(ctx, bytes, host) : OMB_OK;
}

// Posterior of objectives 0..n_obj-1 (their state in args.gp, dense L⁻¹ in Ld[o]): the fused kernel
// when every n_train fits it, else per objective and candidate chunk K block → V = L⁻¹K* (GEMM) →
// column reduction.
hipError_t posterior_any(omb_ctx* ctx, const GPArgs& args, const double* const* Ld, int n_obj, int max_R,
                         const double* Xc, int64_t N, double* mu, double* var) {
  // the fused kernel keeps the candidates' B fragments in registers: n_var ≤ 64 (kMaxFusedDP)
  if (16 * max_R <= OMB_MAX_TRAIN && args.DP <= kMaxFusedDP)
    return launch_posterior(ctx->stream, args, n_obj, max_R, Xc, N, mu, var);
  for (int o = 0; o < n_obj; ++o) {
    const int64_t n = args.gp[o].n;
    int64_t Nc = (int64_t)(((size_t)256 << 20) / (16 * (size_t)n));   // K* and V chunks of 128 MiB each
    Nc = Nc < 256 ? 256 : (Nc / 256) * 256;
    if (Nc > N) Nc = N;
    if (grow_dev(ctx, &ctx->dws, &ctx->dws_cap, sizeof(double) * 2 * (size_t)n * Nc, "dense posterior workspace"))
      return hipErrorOutOfMemory;
    double* Kst = static_cast<double*>(ctx->dws);
    double* V = Kst + (size_t)n * Nc;
    for (int64_t c0 = 0; c0 < N; c0 += Nc) {
      const int64_t nc = (N - c0) < Nc ? (N - c0) : Nc;
      hipError_t e = launch_kernel_block(ctx->stream, args, o, Xc + c0 * args.d, nc, Kst);
      if (e == hipSuccess) e = launch_gemm_ltri_nn(ctx->stream, n, nc, 1.0, Ld[o], n, Kst, nc, 0.0, V, nc);
      if (e == hipSuccess)
        e = launch_post_colreduce(ctx->stream, Kst, V, n, nc, args.gp[o].alpha, args.gp[o].variance,
                                  mu + (int64_t)o * N + c0, var + (int64_t)o * N + c0);
      if (e != hipSuccess) return e;
    }
  }
  return hipSuccess;
}

void gather_Ld(omb_ctx* ctx, int n_obj, const double** Ld) {
  for (int o = 0; o < n_obj; ++o) Ld[o] = ctx->obj[o].Ld;
}

// The fused chain: [Sobol →] posterior(0..k-1) → planned acquisition → [arg-max].
int run_chain(omb_ctx* ctx, const double* Xc, bool sobol, int64_t start, int64_t N, int64_t offset, double* vals_out,
              double* result_dev) {
  int rc = enter(ctx);
  if (rc) return rc;
  const Plan& pl = ctx->plan;
  if (pl.kind == PLAN_NONE) return fail(ctx, OMB_ESTATE, "no acquisition plan (call an omb_plan_* function)");
  if (N < 0) return fail(ctx, OMB_EINVAL, "N=%lld < 0", (long long)N);
  GPArgs args;
  int max_R = 0;
  if ((rc = gather_gp(ctx, pl.k, &args, &max_R))) return rc;
  if (sobol) {
    if (ctx->sob_d == 0) return fail(ctx, OMB_ESTATE, "no Sobol state (call omb_set_sobol)");
    if (ctx->sob_d != args.d) return fail(ctx, OMB_EINVAL, "Sobol dimension %d != n_var %d", ctx->sob_d, args.d);
    if (start < 0 || start + N > (int64_t)(1ull << ctx->sob_bits))
      return fail(ctx, OMB_EINVAL, "Sobol indices [%lld, %lld) outside [0, 2^%d)", (long long)start,
                  (long long)(start + N), ctx->sob_bits);
  } else if (N > 0 && !Xc) {
    return fail(ctx, OMB_EINVAL, "null candidate pointer");
  }
  if ((N + 31) / 32 > 0x7fffffffLL) return fail(ctx, OMB_EUNSUP, "N=%lld too large", (long long)N);
  const int k = pl.k;
  const size_t nd = (size_t)N;
  // EHVI-2D with the arg-max's first pass in its launch (launch_ehvi2d_argmax) when only the pair is wanted; its
  // per-workgroup pairs (≤ kArgmaxMaxBlocks) go to ctx->partials
  const bool acq_argmax = result_dev && !vals_out && N > 0 && ctx->fused_chain && pl.kind == PLAN_EHVI2D;
  const size_t doubles = 2 * (size_t)k * nd + nd + (nd + 1) / 2 + (sobol ? nd * args.d : 0);
  if ((rc = grow_dev(ctx, &ctx->work, &ctx->work_cap, (doubles ? doubles : 1) * sizeof(double), "chain workspace")))
    return rc;
  double* mu = static_cast<double*>(ctx->work);
  double* var = mu + (size_t)k * nd;
  double* vals = vals_out ? vals_out : var + (size_t)k * nd;
  int32_t* raised = reinterpret_cast<int32_t*>(var + (size_t)k * nd + nd);
  double* Xs = var + (size_t)k * nd + nd + (nd + 1) / 2;

  hipEvent_t* ev = nullptr;
  if (ctx->timing && ctx->timing_calls++ % ctx->timing_stride == 0) {
    if (ctx->ev_used + 5 > ctx->ev.size() && ctx->ev.size() < 5 * 4096) {
      for (int i = 0; i < 5 * 64; ++i) {
        hipEvent_t e;
        OMB_HIP(ctx, hipEventCreate(&e));
        ctx->ev.push_back(e);
      }
    }
    if (ctx->ev_used + 5 <= ctx->ev.size()) {
      ev = ctx->ev.data() + ctx->ev_used;
      ctx->ev_used += 5;
    }
  }
  // Each event record costs a few µs of GPU time, so level 1 records only around the posterior.
  const int level = ctx->timing;
  auto mark = [&](int i) -> hipError_t {
    if (!ev) return hipSuccess;
    if (level == 1 && i != 1 && i != 2) return hipSuccess;
    return hipEventRecord(ev[i], ctx->stream);
  };
  hipError_t e = mark(0);
  if (e == hipSuccess && sobol && N > 0) e = launch_sobol(ctx->stream, ctx->sob, ctx->sob_d, ctx->sob_bits, start, N, Xs);
  if (sobol) Xc = Xs;
  if (e == hipSuccess) e = mark(1);
  const double* Ld[OMB_MAX_OBJ];
  gather_Ld(ctx, k, Ld);
  if (e == hipSuccess && N > 0) e = posterior_any(ctx, args, Ld, k, max_R, Xc, N, mu, var);
  if (e == hipSuccess) e = mark(2);
  if (e == hipSuccess && N > 0) {
    switch (pl.kind) {
      case PLAN_EHVI2D:
        if (acq_argmax) {
          unsigned* ticket = ctx->fused_chain == 1 ? reinterpret_cast<unsigned*>(ctx->partials + 2 * kArgmaxMaxBlocks)
                                                   : nullptr;
          const ArgmaxOut am{ctx->partials, ticket, result_dev, offset};
          e = launch_ehvi2d_argmax(ctx->stream, mu, var, N, N, pl.geo, pl.P, pl.r[0], pl.r[1], pl.s00, pl.s01, pl.mode,
                                   am);
        } else {
          e = launch_ehvi2d(ctx->stream, mu, var, N, N, pl.geo, pl.P, pl.r[0], pl.r[1], pl.s00, pl.s01, pl.mode, vals);
        }
        break;
      case PLAN_EHVI_MC:
        e = launch_ehvi_mc(ctx->stream, k, mu, var, N, N, pl.geo, pl.M, pl.r, pl.hv, vals, raised);
        break;
      case PLAN_EHVI_BOXES:
        e = launch_ehvi_boxes(ctx->stream, k, mu, var, N, N, pl.geo, pl.C, pl.boxes, pl.B, vals);
        break;
      case PLAN_HVPOI:
        e = launch_hvpoi(ctx->stream, mu, var, N, N, pl.geo, pl.C, vals);
        break;
      case PLAN_EXPDEC:
        e = launch_expdec(ctx->stream, pl.sp, mu, var, N, N, pl.geo, pl.M, vals);
        break;
      case PLAN_EI:
        e = launch_ei(ctx->stream, pl.ei_kind, k, mu, var, N, N, pl.best, pl.var_eps, pl.pof_eps, vals);
        break;
      default:
        return fail(ctx, OMB_ESTATE, "corrupt plan");
    }
  }
  if (e == hipSuccess) e = mark(3);
  if (e == hipSuccess && result_dev && !acq_argmax)
    e = launch_argmax(ctx->stream, vals, N, offset, ctx->partials, result_dev, ctx->argmax_one_pass);
  if (e == hipSuccess) e = mark(4);
  if (e != hipSuccess) return hip_fail(ctx, e, "fused chain");
  return OMB_OK;
}

}  // namespace

extern "C" {

int omb_abi_version(void) { return OMB_ABI_VERSION; }

int omb_create(int device, omb_ctx** out) {
  if (!out) return OMB_EINVAL;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) return OMB_EINVAL;
  omb_ctx* ctx = new (std::nothrow) omb_ctx();
  if (!ctx) return OMB_ENOMEM;
  ctx->device = device;
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&ctx->partials, sizeof(double) * (2 * kArgmaxMaxBlocks + 2)) != hipSuccess ||
      hipMemset(ctx->partials, 0, sizeof(double) * (2 * kArgmaxMaxBlocks + 2)) != hipSuccess ||
      hipMalloc(&ctx->result_dev, sizeof(double) * 2) != hipSuccess ||
      hipHostMalloc(&ctx->result_host, sizeof(double) * 2, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc(&ctx->info_host, sizeof(int) * 4, hipHostMallocDefault) != hipSuccess ||
      hipMalloc(&ctx->sob, sobol_state_bytes(OMB_MAX_DIM, 32)) != hipSuccess ||
      hipHostMalloc(&ctx->fault_host, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->fault_dev), ctx->fault_host, 0) != hipSuccess ||
      hipHostMalloc(&ctx->fit_host, sizeof(double) * (OMB_MAX_DIM + 8), hipHostMallocMapped | hipHostMallocCoherent) !=
          hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->fit_dev), ctx->fit_host, 0) != hipSuccess) {
    omb_destroy(ctx);
    return OMB_ENOMEM;
  }
  *ctx->fault_host = 0;
  ctx->stream = ctx->own_stream;
  *out = ctx;
  return OMB_OK;
}

int omb_destroy(omb_ctx* ctx) {
  if (!ctx) return OMB_OK;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  for (auto& s : ctx->obj)
    if (s.buf) (void)hipFree(s.buf);
  if (ctx->partials) (void)hipFree(ctx->partials);
  if (ctx->result_dev) (void)hipFree(ctx->result_dev);
  if (ctx->result_host) (void)hipHostFree(ctx->result_host);
  if (ctx->info_host) (void)hipHostFree(ctx->info_host);
  if (ctx->geo) (void)hipFree(ctx->geo);
  if (ctx->stage) (void)hipHostFree(ctx->stage);
  if (ctx->work) (void)hipFree(ctx->work);
  if (ctx->sob) (void)hipFree(ctx->sob);
  if (ctx->tws) (void)hipFree(ctx->tws);
  if (ctx->ichol) (void)hipFree(ctx->ichol);
  if (ctx->sws) (void)hipFree(ctx->sws);
  if (ctx->ews) (void)hipFree(ctx->ews);
  if (ctx->fws) (void)hipFree(ctx->fws);
  if (ctx->dws) (void)hipFree(ctx->dws);
  if (ctx->fault_host) (void)hipHostFree(ctx->fault_host);
  if (ctx->fit_host) (void)hipHostFree(ctx->fit_host);
  for (hipEvent_t e : ctx->ev) (void)hipEventDestroy(e);
  if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
  delete ctx;
  return OMB_OK;
}

int omb_set_stream(omb_ctx* ctx, void* hip_stream) {
  if (!ctx) return OMB_EINVAL;
  ctx->stream = reinterpret_cast<hipStream_t>(hip_stream);
  return OMB_OK;
}

int omb_use_own_stream(omb_ctx* ctx) {
  if (!ctx) return OMB_EINVAL;
  ctx->stream = ctx->own_stream;
  return OMB_OK;
}

int omb_synchronize(omb_ctx* ctx) {
  int rc = enter(ctx);
  if (rc) return rc;
  OMB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return check_fault(ctx);
}

int omb_debug_set(omb_ctx* ctx, int what, int64_t value) {
  if (!ctx) return OMB_EINVAL;
  if (what == OMB_DEBUG_SPIN_LIMIT) {
    if (value < 0 || value > 0x7fffffff) return fail(ctx, OMB_EINVAL, "spin limit %lld outside [0, 2^31)", (long long)value);
    ctx->spin_limit = (int)value;
    return OMB_OK;
  }
  if (what == OMB_DEBUG_FUSED_CHAIN) {
    if (value < 0 || value > 2) return fail(ctx, OMB_EINVAL, "fused chain %lld (0, 1 or 2)", (long long)value);
    ctx->fused_chain = (int)value;
    return OMB_OK;
  }
  if (what == OMB_DEBUG_ARGMAX_PASSES) {
    if (value != 1 && value != 2) return fail(ctx, OMB_EINVAL, "arg-max passes %lld (1 or 2)", (long long)value);
    ctx->argmax_one_pass = value == 1;
    return OMB_OK;
  }
  if (what == OMB_DEBUG_COV_TABLE) {
    ctx->cov_table = value != 0;
    return OMB_OK;
  }
  if (what == OMB_DEBUG_TIMING_STRIDE) {
    if (value < 1 || value > 0x7fffffff) return fail(ctx, OMB_EINVAL, "timing stride %lld < 1", (long long)value);
    ctx->timing_stride = (int)value;
    return OMB_OK;
  }
  if (what == OMB_DEBUG_COV_FUSED) {
    ctx->cov_fused = value != 0;
    return OMB_OK;
  }
  if (what == OMB_DEBUG_SYRK_GLDS) {
    ctx->syrk_glds = value != 0;
    return OMB_OK;
  }
  if (what == OMB_DEBUG_SELECT_SEQ) {
    ctx->select_seq = value != 0;
    return OMB_OK;
  }
  if (what == OMB_DEBUG_CHOL_MODE) {
    if ((value & 3) == 3 || value < 0 || value > 14)
      return fail(ctx, OMB_EINVAL, "Cholesky mode %lld (0 auto, 1 per-step launches, 2 one persistent launch; + 4: "
                  "release / acquire hand-offs; + 8: the persistent launch's trailing updates one task per step)",
                  (long long)value);
    const int modes[3] = {kCholAuto, kCholBlocked, kCholPersistOnly};
    ctx->chol_mode = modes[value & 3];
    ctx->chol_acq_rel = (value & 4) ? 1 : 0;
    ctx->chol_single = (value & 8) ? 1 : 0;
    return OMB_OK;
  }
  return fail(ctx, OMB_EINVAL, "unknown debug setting %d", what);
}

const char* omb_last_error(const omb_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int omb_set_gp(omb_ctx* ctx, int obj, int kernel, int n, int d, const double* X_dev, const double* lengthscale_host,
               double variance, const double* alpha_dev, const double* Linv_dev) {
  int rc = enter(ctx);
  if (rc) return rc;
  if ((rc = check_gp_args(E(ctx), obj, kernel, n, d, X_dev, lengthscale_host, variance, alpha_dev, Linv_dev)))
    return rc;

  ObjState& s = ctx->obj[obj];
  // The previous state may still be read by queued kernels.
  OMB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  const int DP = pad_dim(d);
  const int R = (n + 15) / 16;
  const int Q = (R + 3) / 4;
  const int n_pad = kChunkRows * Q;
  const int R_pack = (n <= OMB_MAX_TRAIN) ? R : 0;   // the packed L⁻¹ feeds only the fused kernel
  const size_t doubles = (size_t)n_pad * DP + 2 * (size_t)n_pad + DP + (size_t)packed_L_size(R_pack) + (size_t)n * n +
                         (size_t)packed_X_size(n_pad, DP);
  const size_t bytes = doubles * sizeof(double);
  if (bytes > s.cap) {
    if (s.buf) (void)hipFree(s.buf);
    s.buf = nullptr;
    s.cap = 0;
    if (hipMalloc(&s.buf, bytes) != hipSuccess) {
      s.set = false;
      return fail(ctx, OMB_ENOMEM, "hipMalloc(%zu) for objective %d", bytes, obj);
    }
    s.cap = bytes;
  }
  double* Xs = s.buf;
  double* xsq = Xs + (size_t)n_pad * DP;
  double* alpha_p = xsq + n_pad;
  double* ls_p = alpha_p + n_pad;
  double* Lp = ls_p + DP;
  double* Ld = Lp + packed_L_size(R_pack);
  double* Xf = Ld + (size_t)n * n;
  hipError_t e = launch_pack_gp(ctx->stream, n, d, DP, X_dev, lengthscale_host, alpha_dev, Linv_dev, Xs, xsq,
                                alpha_p, Lp, R_pack, n_pad);
  if (e == hipSuccess) e = launch_pack_x(ctx->stream, d, DP, n_pad, Xs, xsq, Xf);
  if (e == hipSuccess)
    e = hipMemcpyAsync(Ld, Linv_dev, sizeof(double) * (size_t)n * n, hipMemcpyDeviceToDevice, ctx->stream);
  if (e != hipSuccess) {
    s.set = false;
    return hip_fail(ctx, e, "pack_gp");
  }
  s.set = true;
  s.n = n;
  s.d = d;
  s.DP = DP;
  s.R = R;
  s.n_pad = n_pad;
  s.kind = kernel;
  s.variance = variance;
  s.Ld = Ld;
  s.dev = GPDev{Xs, xsq, alpha_p, Lp, ls_p, variance, n, R, kernel, 0, Xf};
  return OMB_OK;
}

int omb_kernel_block(omb_ctx* ctx, int obj, const double* Xc_dev, int64_t N, double* K_dev) {
  int rc = enter(ctx);
  if (rc) return rc;
  if (obj < 0 || obj >= OMB_MAX_OBJ || !ctx->obj[obj].set) return fail(ctx, OMB_ESTATE, "objective %d not set", obj);
  if (N < 0 || (N > 0 && (!Xc_dev || !K_dev))) return fail(ctx, OMB_EINVAL, "bad candidate/output arguments");
  if (N == 0) return OMB_OK;
  GPArgs args;
  init_args(ctx, &args);
  args.gp[obj] = ctx->obj[obj].dev;
  args.d = ctx->obj[obj].d;
  args.DP = ctx->obj[obj].DP;
  hipError_t e = launch_kernel_block(ctx->stream, args, obj, Xc_dev, N, K_dev);
  if (e != hipSuccess) return hip_fail(ctx, e, "kernel_block");
  return OMB_OK;
}

int omb_posterior(omb_ctx* ctx, int n_obj, const double* Xc_dev, int64_t N, double* mu_dev, double* var_dev) {
  int rc = enter(ctx);
  if (rc) return rc;
  if (N < 0 || (N > 0 && (!Xc_dev || !mu_dev || !var_dev)))
    return fail(ctx, OMB_EINVAL, "bad candidate/output arguments");
  GPArgs args;
  int max_R = 0;
  rc = gather_gp(ctx, n_obj, &args, &max_R);
  if (rc) return rc;
  if (N == 0) return OMB_OK;
  if ((N + 31) / 32 > 0x7fffffffLL) return fail(ctx, OMB_EUNSUP, "N=%lld too large", (long long)N);
  const double* Ld[OMB_MAX_OBJ];
  gather_Ld(ctx, n_obj, Ld);
  hipError_t e = posterior_any(ctx, args, Ld, n_obj, max_R, Xc_dev, N, mu_dev, var_dev);
  if (e != hipSuccess) return hip_fail(ctx, e, "posterior");
  return OMB_OK;
}

int omb_ehvi2d(omb_ctx* ctx, const double* mu_dev, const double* var_dev, int64_t ld, int64_t N,
               const double* pf_sorted_dev, int P, const double* r_host, double s00, double s01, int mode,
               double* out_dev) {
  int rc = enter(ctx);
  if (rc) return rc;
  if ((rc = check_moments(E(ctx), mu_dev, var_dev, ld, N, 2, out_dev))) return rc;
  if (!pf_sorted_dev) return fail(ctx, OMB_EINVAL, "null Pareto front");
  if ((rc = check_ehvi2d(E(ctx), P, r_host, mode))) return rc;
  if (N == 0) return OMB_OK;
  hipError_t e = launch_ehvi2d(ctx->stream, mu_dev, var_dev, ld, N, pf_sorted_dev, P, r_host[0], r_host[1], s00, s01,
                               mode, out_dev);
  if (e != hipSuccess) return hip_fail(ctx, e, "ehvi2d");
  return OMB_OK;
}

int omb_ehvi_mc(omb_ctx* ctx, int k, const double* mu_dev, const double* var_dev, int64_t ld, int64_t N,
                const double* cache_dev, int M, const double* r_host, double hv_pf, double* out_dev,
                int32_t* raised_dev) {
  int rc = enter(ctx);
  if (rc) return rc;
  if ((rc = check_ehvi_mc(E(ctx), k, M, r_host))) return rc;
  if ((rc = check_moments(E(ctx), mu_dev, var_dev, ld, N, k, out_dev))) return rc;
  if (!cache_dev) return fail(ctx, OMB_EINVAL, "null cache");
  if (N == 0) return OMB_OK;
  hipError_t e = launch_ehvi_mc(ctx->stream, k, mu_dev, var_dev, ld, N, cache_dev, M, r_host, hv_pf, out_dev,
                                raised_dev);
  if (e != hipSuccess) return hip_fail(ctx, e, "ehvi_mc");
  return OMB_OK;
}

int omb_ehvi3d_mc(omb_ctx* ctx, const double* mu_dev, const double* var_dev, int64_t ld, int64_t N,
                  const double* cache_dev, int M, const double* r_host, double hv_pf, double* out_dev,
                  int32_t* raised_dev) {
  return omb_ehvi_mc(ctx, 3, mu_dev, var_dev, ld, N, cache_dev, M, r_host, hv_pf, out_dev, raised_dev);
}

int omb_ehvi_boxes(omb_ctx* ctx, int k, const double* mu_dev, const double* var_dev, int64_t ld, int64_t N,
                   const double* coords_dev, int C, const uint16_t* boxes_dev, int B, double* out_dev) {
  int rc = enter(ctx);
  if (rc) return rc;
  if ((rc = check_boxes(E(ctx), k, C, B))) return rc;
  if ((rc = check_moments(E(ctx), mu_dev, var_dev, ld, N, k, out_dev))) return rc;
  if (!coords_dev || !boxes_dev) return fail(ctx, OMB_EINVAL, "null grid/box list");
  if (N == 0) return OMB_OK;
  hipError_t e = launch_ehvi_boxes(ctx->stream, k, mu_dev, var_dev, ld, N, coords_dev, C, boxes_dev, B, out_dev);
  if (e != hipSuccess) return hip_fail(ctx, e, "ehvi_boxes");
  return OMB_OK;
}

int omb_hvpoi(omb_ctx* ctx, const double* mu_dev, const double* var_dev, int64_t ld, int64_t N,
              const double* cells_dev, int C, double* out_dev) {
  int rc = enter(ctx);
  if (rc) return rc;
  if ((rc = check_moments(E(ctx), mu_dev, var_dev, ld, N, 2, out_dev))) return rc;
  if (!cells_dev) return fail(ctx, OMB_EINVAL, "null cells");
  if ((rc = check_hvpoi(E(ctx), C))) return rc;
  if (N == 0) return OMB_OK;
  hipError_t e = launch_hvpoi(ctx->stream, mu_dev, var_dev, ld, N, cells_dev, C, out_dev);
  if (e != hipSuccess) return hip_fail(ctx, e, "hvpoi");
  return OMB_OK;
}

int omb_expdec(omb_ctx* ctx, int k, const double* mu_dev, const double* var_dev, int64_t ld, int64_t N,
               const double* cache_dev, int M, int scal_id, const double* params_host, const double* weights_host,
               const double* ideal_host, const double* max_host, double agg_min, double* out_dev) {
  int rc = enter(ctx);
  if (rc) return rc;
  ScalParams sp;
  if ((rc = build_scal(E(ctx), k, M, scal_id, params_host, weights_host, ideal_host, max_host, agg_min, &sp))) return rc;
  if ((rc = check_moments(E(ctx), mu_dev, var_dev, ld, N, k, out_dev))) return rc;
  if (!cache_dev) return fail(ctx, OMB_EINVAL, "null cache");
  if (N == 0) return OMB_OK;
  hipError_t e = launch_expdec(ctx->stream, sp, mu_dev, var_dev, ld, N, cache_dev, M, out_dev);
  if (e != hipSuccess) return hip_fail(ctx, e, "expdec");
  return OMB_OK;
}

int omb_ei(omb_ctx* ctx, const double* mu_dev, const double* var_dev, int64_t N, double best, double var_eps,
           double* out_dev) {
  return omb_ei_ext(ctx, OMB_EI_PLAIN, 1, mu_dev, var_dev, N, N, best, var_eps, 0.0, out_dev);
}

int omb_ei_ext(omb_ctx* ctx, int kind, int k, const double* mu_dev, const double* var_dev, int64_t ld, int64_t N,
               double best, double var_eps, double pof_eps, double* out_dev) {
  int rc = enter(ctx);
  if (rc) return rc;
  if ((rc = check_ei(E(ctx), kind, k, var_eps, pof_eps))) return rc;
  if ((rc = check_moments(E(ctx), mu_dev, var_dev, ld, N, k, out_dev))) return rc;
  if (N == 0) return OMB_OK;
  hipError_t e = launch_ei(ctx->stream, kind, k, mu_dev, var_dev, ld, N, best, var_eps, pof_eps, out_dev);
  if (e != hipSuccess) return hip_fail(ctx, e, "ei");
  return OMB_OK;
}

int omb_argmax_dev(omb_ctx* ctx, const double* vals_dev, int64_t N, int64_t offset, double* result_dev) {
  int rc = enter(ctx);
  if (rc) return rc;
  if (!result_dev || N < 0 || (N > 0 && !vals_dev)) return fail(ctx, OMB_EINVAL, "bad arg-max arguments");
  hipError_t e = launch_argmax(ctx->stream, vals_dev, N, offset, ctx->partials, result_dev, ctx->argmax_one_pass);
  if (e != hipSuccess) return hip_fail(ctx, e, "argmax");
  return OMB_OK;
}

int omb_argmax(omb_ctx* ctx, const double* vals_dev, int64_t N, int64_t offset, double* best_val, int64_t* best_idx) {
  int rc = omb_argmax_dev(ctx, vals_dev, N, offset, ctx ? ctx->result_dev : nullptr);
  if (rc) return rc;
  OMB_HIP(ctx, hipMemcpyAsync(ctx->result_host, ctx->result_dev, 2 * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  OMB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (best_val) *best_val = ctx->result_host[0];
  if (best_idx) *best_idx = (int64_t)ctx->result_host[1];
  return OMB_OK;
}

// ---------------------------------------------------------------------------------------
// Fused chain: per-iteration plans, device Sobol' generation, one-call batch evaluation.

int omb_plan_ehvi2d(omb_ctx* ctx, const double* pf_sorted_host, int P, const double* r_host, double s00, double s01,
                    int mode) {
  void* h = nullptr;
  int rc = enter(ctx);
  if (rc) return rc;
  ctx->plan = Plan();
  if ((rc = check_ehvi2d(E(ctx), P, r_host, mode))) return rc;
  if (!pf_sorted_host) return fail(ctx, OMB_EINVAL, "null Pareto front");
  const size_t bytes = sizeof(double) * 2 * (size_t)P;
  if ((rc = plan_begin(ctx, bytes, &h))) return rc;
  memcpy(h, pf_sorted_host, bytes);
  if ((rc = stage_to_geo(ctx, bytes))) return rc;
  Plan pl;
  pl.kind = PLAN_EHVI2D;
  pl.k = 2;
  pl.P = P;
  pl.mode = mode;
  pl.r[0] = r_host[0];
  pl.r[1] = r_host[1];
  pl.s00 = s00;
  pl.s01 = s01;
  pl.geo = static_cast<const double*>(ctx->geo);
  ctx->plan = pl;
  return OMB_OK;
}

int omb_plan_ehvi_mc(omb_ctx* ctx, int k, const double* cache_host, int M, const double* r_host, double hv_pf) {
  void* h = nullptr;
  int rc = enter(ctx);
  if (rc) return rc;
  ctx->plan = Plan();
  if ((rc = check_ehvi_mc(E(ctx), k, M, r_host))) return rc;
  if (!cache_host) return fail(ctx, OMB_EINVAL, "null cache");
  const size_t bytes = sizeof(double) * (size_t)k * M;
  if ((rc = plan_begin(ctx, bytes, &h))) return rc;
  memcpy(h, cache_host, bytes);
  if ((rc = stage_to_geo(ctx, bytes))) return rc;
  Plan pl;
  pl.kind = PLAN_EHVI_MC;
  pl.k = k;
  pl.M = M;
  for (int j = 0; j < k; ++j) pl.r[j] = r_host[j];
  pl.hv = hv_pf;
  pl.geo = static_cast<const double*>(ctx->geo);
  ctx->plan = pl;
  return OMB_OK;
}

int omb_plan_ehvi3d_mc(omb_ctx* ctx, const double* cache_host, int M, const double* r_host, double hv_pf) {
  return omb_plan_ehvi_mc(ctx, 3, cache_host, M, r_host, hv_pf);
}

int omb_plan_ehvi_boxes(omb_ctx* ctx, int k, const double* coords_host, int C, const uint16_t* boxes_host, int B) {
  void* h = nullptr;
  int rc = enter(ctx);
  if (rc) return rc;
  ctx->plan = Plan();
  if ((rc = check_boxes(E(ctx), k, C, B))) return rc;
  if (!coords_host || !boxes_host) return fail(ctx, OMB_EINVAL, "null grid/box list");
  const size_t cbytes = sizeof(double) * (size_t)k * C;
  const size_t bbytes = sizeof(uint16_t) * 2 * (size_t)k * B;
  if ((rc = plan_begin(ctx, cbytes + bbytes, &h))) return rc;
  memcpy(h, coords_host, cbytes);
  memcpy(static_cast<char*>(h) + cbytes, boxes_host, bbytes);
  if ((rc = stage_to_geo(ctx, cbytes + bbytes))) return rc;
  Plan pl;
  pl.kind = PLAN_EHVI_BOXES;
  pl.k = k;
  pl.C = C;
  pl.B = B;
  pl.geo = static_cast<const double*>(ctx->geo);
  pl.boxes = reinterpret_cast<const uint16_t*>(static_cast<const char*>(ctx->geo) + cbytes);
  ctx->plan = pl;
  return OMB_OK;
}

int omb_plan_hvpoi(omb_ctx* ctx, const double* cells_host, int C) {
  void* h = nullptr;
  int rc = enter(ctx);
  if (rc) return rc;
  ctx->plan = Plan();
  if ((rc = check_hvpoi(E(ctx), C))) return rc;
  if (!cells_host) return fail(ctx, OMB_EINVAL, "null cells");
  const size_t bytes = sizeof(double) * 4 * (size_t)C;
  if ((rc = plan_begin(ctx, bytes, &h))) return rc;
  memcpy(h, cells_host, bytes);
  if ((rc = stage_to_geo(ctx, bytes))) return rc;
  Plan pl;
  pl.kind = PLAN_HVPOI;
  pl.k = 2;
  pl.C = C;
  pl.geo = static_cast<const double*>(ctx->geo);
  ctx->plan = pl;
  return OMB_OK;
}

int omb_plan_expdec(omb_ctx* ctx, int k, const double* cache_host, int M, int scal_id, const double* params_host,
                    const double* weights_host, const double* ideal_host, const double* max_host, double agg_min) {
  void* h = nullptr;
  int rc = enter(ctx);
  if (rc) return rc;
  ctx->plan = Plan();
  ScalParams sp;
  if ((rc = build_scal(E(ctx), k, M, scal_id, params_host, weights_host, ideal_host, max_host, agg_min, &sp))) return rc;
  if (!cache_host) return fail(ctx, OMB_EINVAL, "null cache");
  const size_t bytes = sizeof(double) * (size_t)k * M;
  if ((rc = plan_begin(ctx, bytes, &h))) return rc;
  memcpy(h, cache_host, bytes);
  if ((rc = stage_to_geo(ctx, bytes))) return rc;
  Plan pl;
  pl.kind = PLAN_EXPDEC;
  pl.k = k;
  pl.M = M;
  pl.sp = sp;
  pl.geo = static_cast<const double*>(ctx->geo);
  ctx->plan = pl;
  return OMB_OK;
}

int omb_plan_ei(omb_ctx* ctx, double best, double var_eps) {
  return omb_plan_ei_ext(ctx, OMB_EI_PLAIN, 1, best, var_eps, 0.0);
}

int omb_plan_ei_ext(omb_ctx* ctx, int kind, int k, double best, double var_eps, double pof_eps) {
  int rc = enter(ctx);
  if (rc) return rc;
  ctx->plan = Plan();
  if ((rc = check_ei(E(ctx), kind, k, var_eps, pof_eps))) return rc;
  Plan pl;
  pl.kind = PLAN_EI;
  pl.ei_kind = kind;
  pl.k = k;
  pl.best = best;
  pl.var_eps = var_eps;
  pl.pof_eps = pof_eps;
  ctx->plan = pl;
  return OMB_OK;
}

int omb_set_sobol(omb_ctx* ctx, int d, int bits, const uint32_t* sv_host, const uint32_t* shift_host,
                  const double* lo_host, const double* hi_host) {
  int rc = enter(ctx);
  if (rc) return rc;
  ctx->sob_d = 0;
  if ((rc = check_sobol_args(E(ctx), d, bits, sv_host, shift_host, lo_host, hi_host))) return rc;
  const size_t bytes = sobol_state_bytes(d, bits);
  void* h = nullptr;
  if ((rc = stage_begin(ctx, bytes, &h))) return rc;
  sobol_pack_state(d, bits, sv_host, shift_host, lo_host, hi_host, h);
  OMB_HIP(ctx, hipMemcpyAsync(ctx->sob, h, bytes, hipMemcpyHostToDevice, ctx->stream));
  ctx->sob_d = d;
  ctx->sob_bits = bits;
  return OMB_OK;
}

int omb_sobol(omb_ctx* ctx, int64_t start, int64_t N, double* X_dev) {
  int rc = enter(ctx);
  if (rc) return rc;
  if (ctx->sob_d == 0) return fail(ctx, OMB_ESTATE, "no Sobol state (call omb_set_sobol)");
  if (N < 0 || (N > 0 && !X_dev)) return fail(ctx, OMB_EINVAL, "bad output arguments");
  if (start < 0 || start + N > (int64_t)(1ull << ctx->sob_bits))
    return fail(ctx, OMB_EINVAL, "Sobol indices [%lld, %lld) outside [0, 2^%d)", (long long)start, (long long)(start + N),
                ctx->sob_bits);
  hipError_t e = launch_sobol(ctx->stream, ctx->sob, ctx->sob_d, ctx->sob_bits, start, N, X_dev);
  if (e != hipSuccess) return hip_fail(ctx, e, "sobol");
  return OMB_OK;
}

int omb_eval(omb_ctx* ctx, const double* Xc_dev, int64_t N, double* vals_dev) {
  if (ctx && N > 0 && !vals_dev) return fail(ctx, OMB_EINVAL, "null output");
  return run_chain(ctx, Xc_dev, false, 0, N, 0, vals_dev, nullptr);
}

int omb_eval_argmax(omb_ctx* ctx, const double* Xc_dev, int64_t N, int64_t offset, double* result_dev) {
  if (ctx && !result_dev) return fail(ctx, OMB_EINVAL, "null result");
  return run_chain(ctx, Xc_dev, false, 0, N, offset, nullptr, result_dev);
}

int omb_eval_argmax_sobol(omb_ctx* ctx, int64_t start, int64_t N, double* result_dev) {
  if (ctx && !result_dev) return fail(ctx, OMB_EINVAL, "null result");
  return run_chain(ctx, nullptr, true, start, N, start, nullptr, result_dev);
}

int omb_timing(omb_ctx* ctx, int enable) {
  int rc = enter(ctx);
  if (rc) return rc;
  OMB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (enable < 0 || enable > 2) return fail(ctx, OMB_EINVAL, "timing level %d outside [0, 2]", enable);
  ctx->timing = enable;
  ctx->timing_calls = 0;
  ctx->ev_used = 0;
  // create the events of the first 256 chains now, not inside the timed chains
  while (enable && ctx->ev.size() < 5 * 256) {
    hipEvent_t e;
    OMB_HIP(ctx, hipEventCreate(&e));
    ctx->ev.push_back(e);
  }
  return OMB_OK;
}

int omb_timing_read(omb_ctx* ctx, double* stage_ms, int64_t* chains) {
  int rc = enter(ctx);
  if (rc) return rc;
  if (!stage_ms) return fail(ctx, OMB_EINVAL, "null output");
  OMB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  for (int s = 0; s < 4; ++s) stage_ms[s] = 0.0;
  const size_t n = ctx->ev_used / 5;
  for (size_t c = 0; c < n; ++c) {
    for (int s = 0; s < 4; ++s) {
      if (ctx->timing == 1 && s != 1) continue;
      float ms = 0.0f;
      OMB_HIP(ctx, hipEventElapsedTime(&ms, ctx->ev[5 * c + s], ctx->ev[5 * c + s + 1]));
      stage_ms[s] += ms;
    }
  }
  if (chains) *chains = (int64_t)n;
  ctx->ev_used = 0;
  return OMB_OK;
}

// ---------------------------------------------------------------------------------------
// Thompson sampling (TuRBO, turbo.py:75-153): full posterior covariance, Cholesky, joint
// samples and the greedy per-sample arg-min (omb_linalg.hip).

static int check_obj(omb_ctx* ctx, int obj) {
  if (obj < 0 || obj >= OMB_MAX_OBJ || !ctx->obj[obj].set) return fail(ctx, OMB_ESTATE, "objective %d not set", obj);
  return OMB_OK;
}

static int check_cov_n(omb_ctx* ctx, int64_t N) {
  if (N < 0) return fail(ctx, OMB_EINVAL, "N=%lld < 0", (long long)N);
  if (N > kMaxCovN) return fail(ctx, OMB_EUNSUP, "N=%lld candidates exceed the full-covariance limit %lld",
                                (long long)N, (long long)kMaxCovN);
  return OMB_OK;
}

// K* (n, N) by the K block, V = L⁻¹K* (n, N) by GEMM, μ = K*ᵀα and σ² = σ_f² − Σ V² by the column
// reduction over those two (the fused posterior kernel would recompute K* and V; at TuRBO's ≤ 5,000
// candidates it also runs on a few dozen workgroups: 90 µs of a 3 ms step, profiles/r02_v21_c6_kernel_stats.csv).
// scale_ws (omb_posterior_samples): the column reduction also writes launch_cand_scale's rows into it, for the first
// cov_build (prescaled); the fused SYRK path only.
static bool cov_fused_path(const omb_ctx* ctx, const ObjState& s) {
  return !ctx->cov_table && ctx->cov_fused && s.DP <= kMaxFusedDP;
}
static hipError_t cov_prepare(omb_ctx* ctx, const ObjState& s, const double* Xc, int64_t N, double* Kst, double* V,
                              double* mu, double* var, double* scale_ws = nullptr) {
  GPArgs args;
  init_args(ctx, &args);
  args.gp[0] = s.dev;
  args.d = s.d;
  args.DP = s.DP;
  hipError_t e = launch_kernel_block(ctx->stream, args, 0, Xc, N, Kst);
  if (e == hipSuccess) e = launch_gemm_ltri_nn(ctx->stream, s.n, N, 1.0, s.Ld, s.n, Kst, N, 0.0, V, N);
  if (e == hipSuccess)
    e = launch_post_colreduce(ctx->stream, Kst, V, s.n, N, s.dev.alpha, s.dev.variance, mu, var,
                              scale_ws ? &s.dev : nullptr, s.d, s.DP, Xc, scale_ws);
  return e;
}

// lower triangle of Σ = K(X*, X*) − VᵀV (GPy PosteriorExact._raw_predict, full_cov=True); cws:
// cand_cov_ws_doubles(N, DP) doubles.
// zero_ints / n_zero / zero_info: the next Cholesky's sync words and status, zeroed by the fused SYRK's workgroups on
// the side (*zeroed = true when it did: that factorisation then skips its init launch)
static hipError_t cov_build(omb_ctx* ctx, const ObjState& s, const double* Xc, int64_t N, const double* V, double* S,
                            int64_t lds, double* cws, double jitter = 0.0, bool prescaled = false,
                            int* zero_ints = nullptr, int n_zero = 0, int* zero_info = nullptr, bool* zeroed = nullptr) {
  if (zeroed) *zeroed = false;
  if (cov_fused_path(ctx, s)) {
    // K(X*, X*) formed in the SYRK's epilogue (launch_cov_syrk): the two-launch result below to the ulp
    hipError_t e = hipSuccess;
    const int kp = prescaled ? (s.DP + 3) / 4 * 4 : launch_cand_scale(ctx->stream, s.dev, s.d, s.DP, Xc, N, cws, &e);
    if (e == hipSuccess && kp > 0) {
      if (zeroed) *zeroed = zero_ints != nullptr;
      return launch_cov_syrk(ctx->stream, N, s.n, V, N, S, lds, cws, cws + N * kp, kp, s.kind, s.variance, jitter,
                             ctx->syrk_glds, zero_ints, n_zero, zero_info);
    }
    if (e != hipSuccess) return e;
  }
  hipError_t e = launch_cand_cov(ctx->stream, s.dev, s.d, s.DP, Xc, N, S, lds, cws, jitter, ctx->cov_table);
  if (e == hipSuccess) e = launch_gemm_tn_lower(ctx->stream, N, s.n, -1.0, V, N, 1.0, S, lds);
  return e;
}

// In-place lower Cholesky of A + jitter·I; synchronises and returns LAPACK's info in *info.
// The factorisation in two halves, so that a caller can queue work that reads the factor before it waits for the
// status: chol_enqueue queues A += jitter·I, the factor and the status's copy into pinned memory; chol_wait
// synchronises and reads it.
// The factorisation workspace: [info int | pad to 16 B | factor workspace (chol_ws_doubles)]
static int chol_workspace(omb_ctx* ctx, int64_t N, int** dinfo, double** ws) {
  int rc = grow_dev(ctx, &ctx->ichol, &ctx->ichol_cap, 16 + sizeof(double) * chol_ws_doubles(N), "Cholesky workspace");
  if (rc) return rc;
  *dinfo = static_cast<int*>(ctx->ichol);
  *ws = reinterpret_cast<double*>(static_cast<char*>(ctx->ichol) + 16);
  return OMB_OK;
}

// sync_zeroed: the persistent launch's sync words and info were zeroed by the covariance SYRK (cov_build)
static int chol_enqueue(omb_ctx* ctx, double* A, int64_t N, int64_t lda, double jitter, bool sync_zeroed = false) {
  int* dinfo = nullptr;
  double* ws = nullptr;
  int rc = chol_workspace(ctx, N, &dinfo, &ws);
  if (rc) return rc;
  OMB_HIP(ctx, launch_add_diag(ctx->stream, A, N, lda, jitter));
  OMB_HIP(ctx, launch_cholesky_mode(ctx->stream, A, N, lda, dinfo, ws, ctx->chol_mode, ctx->spin_limit,
                                    ctx->chol_acq_rel, ctx->chol_single, sync_zeroed));
  OMB_HIP(ctx, hipMemcpyAsync(ctx->info_host, dinfo, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  return OMB_OK;
}

static int chol_wait(omb_ctx* ctx, int* info) {
  OMB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  const int h = *ctx->info_host;
  if (h == kCholSpinFault)
    return fail(ctx, OMB_EHIP, "Cholesky: a workgroup's wait for the diagonal block exceeded %d polls; the factor is "
                               "invalid", ctx->spin_limit);
  *info = h;
  return OMB_OK;
}

static int run_cholesky(omb_ctx* ctx, double* A, int64_t N, int64_t lda, double jitter, int* info) {
  int rc = chol_enqueue(ctx, A, N, lda, jitter);
  return rc ? rc : chol_wait(ctx, info);
}

int omb_posterior_cov(omb_ctx* ctx, int obj, const double* Xc_dev, int64_t N, double* mu_dev, double* cov_dev) {
  int rc = enter(ctx);
  if (rc) return rc;
  if ((rc = check_obj(ctx, obj)) || (rc = check_cov_n(ctx, N))) return rc;
  if (N > 0 && (!Xc_dev || !mu_dev || !cov_dev)) return fail(ctx, OMB_EINVAL, "null device pointer");
  if (N == 0) return OMB_OK;
  const ObjState& s = ctx->obj[obj];
  const size_t nN = (size_t)s.n * N;
  const size_t cw = (size_t)cand_cov_ws_doubles(N, s.DP);
  if ((rc = grow_dev(ctx, &ctx->tws, &ctx->tws_cap, sizeof(double) * (2 * nN + N + cw), "covariance workspace")))
    return rc;
  double* Kst = static_cast<double*>(ctx->tws);
  double* V = Kst + nN;
  double* var = V + nN;
  double* cws = var + N;
  hipError_t e = cov_prepare(ctx, s, Xc_dev, N, Kst, V, mu_dev, var, nullptr);
  if (e == hipSuccess) e = cov_build(ctx, s, Xc_dev, N, V, cov_dev, N, cws);
  if (e == hipSuccess) e = launch_mirror_lower(ctx->stream, cov_dev, N, N);
  if (e != hipSuccess) return hip_fail(ctx, e, "posterior_cov");
  return OMB_OK;
}

int omb_cholesky(omb_ctx* ctx, double* A_dev, int64_t N, int64_t lda, double jitter, int* info) {
  int rc = enter(ctx);
  if (rc) return rc;
  if (!info || N < 0 || lda < N || (N > 0 && !A_dev)) return fail(ctx, OMB_EINVAL, "bad Cholesky arguments");
  if (!(jitter >= 0.0)) return fail(ctx, OMB_EINVAL, "jitter=%g must be >= 0", jitter);
  *info = 0;
  if (N == 0) return OMB_OK;
  return run_cholesky(ctx, A_dev, N, lda, jitter, info);
}

// The draws are queued before the factor's status is read (omb_posterior_samples), so a failed call would leave
// draws from an invalid factor in Y: they are overwritten with NaN (all-ones bit patterns) instead.
static void poison_draws(omb_ctx* ctx, double* Y, size_t count) {
  (void)hipMemsetAsync(Y, 0xff, count * sizeof(double), ctx->stream);
  (void)hipStreamSynchronize(ctx->stream);
}

int omb_posterior_samples(omb_ctx* ctx, int obj, const double* Xc_dev, int64_t N, const double* Zt_dev, int B,
                          double jitter_rel, int max_tries, double* Y_dev, double* jitter_used) {
  int rc = enter(ctx);
  if (rc) return rc;
  if ((rc = check_obj(ctx, obj)) || (rc = check_cov_n(ctx, N))) return rc;
  if (N < 1 || B < 1) return fail(ctx, OMB_EINVAL, "need N >= 1 candidates and B >= 1 samples (N=%lld, B=%d)",
                                  (long long)N, B);
  if (!Xc_dev || !Zt_dev || !Y_dev) return fail(ctx, OMB_EINVAL, "null device pointer");
  if (!(jitter_rel >= 0.0) || max_tries < 1 || max_tries > 32)
    return fail(ctx, OMB_EINVAL, "jitter_rel=%g must be >= 0 and max_tries=%d in [1, 32]", jitter_rel, max_tries);
  const ObjState& s = ctx->obj[obj];
  const size_t nN = (size_t)s.n * N;
  const size_t cw = (size_t)cand_cov_ws_doubles(N, s.DP);
  const size_t sw = (size_t)chol_samples_ws_doubles(N, B);
  const size_t doubles = 2 * nN + 2 * (size_t)N + (size_t)N * N + (cw > sw ? cw : sw);
  if ((rc = grow_dev(ctx, &ctx->tws, &ctx->tws_cap, sizeof(double) * doubles, "sampling workspace"))) return rc;
  double* Kst = static_cast<double*>(ctx->tws);
  double* V = Kst + nN;
  double* mu = V + nN;
  double* var = mu + N;
  double* S = var + N;
  double* cws = S + (size_t)N * N;
  // the first try's scaled candidates come from the column reduction's launch; later tries rescale (the draws'
  // split-K partials share cws)
  const bool prescale = cov_fused_path(ctx, s);
  hipError_t e = cov_prepare(ctx, s, Xc_dev, N, Kst, V, mu, var, prescale ? cws : nullptr);
  if (e != hipSuccess) return hip_fail(ctx, e, "posterior_samples (posterior)");
  // the factorisation's workspace placed before the covariance build, whose SYRK zeroes its sync words and status
  int* dinfo = nullptr;
  double* cws_chol = nullptr;
  if ((rc = chol_workspace(ctx, N, &dinfo, &cws_chol))) return rc;
  int* sync_ints = nullptr;
  const int n_sync = chol_persist_sync_words(cws_chol, N, &sync_ints);
  double jit = jitter_rel * s.variance;
  int info = -1, t = 0;
  for (; t < max_tries; ++t, jit *= 10.0) {
    bool zeroed = false;
    if ((e = cov_build(ctx, s, Xc_dev, N, V, S, N, cws, jit, prescale && t == 0, sync_ints, n_sync, dinfo, &zeroed)) !=
        hipSuccess)   // Σ + jit·I
      return hip_fail(ctx, e, "posterior_samples (cov)");
    if ((rc = chol_enqueue(ctx, S, N, N, 0.0, zeroed))) return rc;
    // the draws are queued before the status is read (no idle GPU between the factor and them); a failed factor's
    // draws are overwritten by the next try's
    if ((e = launch_chol_samples(ctx->stream, S, N, N, mu, Zt_dev, B, Y_dev, cws)) != hipSuccess)
      return hip_fail(ctx, e, "posterior_samples (samples)");
    if ((rc = chol_wait(ctx, &info))) {
      poison_draws(ctx, Y_dev, (size_t)B * N);
      return rc;
    }
    if (info == 0) break;
  }
  if (info != 0) {
    poison_draws(ctx, Y_dev, (size_t)B * N);
    return fail(ctx, OMB_ENOTPD, "posterior covariance + %g I is not positive definite (column %d) after %d tries",
                jit / 10.0, info, max_tries);
  }
  if (jitter_used) *jitter_used = jit;
  return OMB_OK;
}

int omb_thompson_select(omb_ctx* ctx, const double* Y_dev, int B, int64_t N, int64_t* idx_dev) {
  int rc = enter(ctx);
  if (rc) return rc;
  if (B < 0 || N < 1) return fail(ctx, OMB_EINVAL, "need B >= 0 samples over N >= 1 candidates");
  if (N > kSelectMaxN) return fail(ctx, OMB_EUNSUP, "N=%lld candidates exceed %lld", (long long)N,
                                   (long long)kSelectMaxN);
  if (B > 0 && (!Y_dev || !idx_dev)) return fail(ctx, OMB_EINVAL, "null device pointer");
  if (B == 0) return OMB_OK;
  const size_t sw = (size_t)select_ws_bytes(B, N);
  if (sw && (rc = grow_dev(ctx, &ctx->sws, &ctx->sws_cap, sw, "selection workspace"))) return rc;
  hipError_t e = launch_select(ctx->stream, Y_dev, B, N, idx_dev, ctx->sws, ctx->select_seq);
  if (e != hipSuccess) return hip_fail(ctx, e, "thompson_select");
  return OMB_OK;
}

// ---------------------------------------------------------------------------------------
// GP fit on the device: GPy ExactGaussianInference + jitchol, log marginal
// likelihood and its gradient for the L-BFGS hyperparameter search (optimisers.py:226-231).

struct GPFactor {
  double* Ky;      // (n, n): Ky, then its Cholesky factor (lower)
  double* Linv;    // (n, n): L⁻¹ (upper triangle zero)
  double* Kinv;    // (n, n): Ky⁻¹ (lower triangle)
  double* T;       // (64, n) scratch of the triangular inverse
  double* alpha;   // (n)
  double* v;       // (n)
  double* ls;      // (DP)
  double* part;    // gp_grad_blocks(n)·(DP+1)
  double* out;     // DP + 3
  double* cws;     // cand_cov_ws_doubles(n, DP): X/ℓ and its squared norms for K(X, X)
  double jitter;   // jitter added by jitchol (0 when the first factorisation succeeded)
};

// Ky = K + (noise + 1e-8) I, L = jitchol(Ky) (GPy.util.linalg.jitchol: on failure add
// mean(diag)·1e-6·10^t, t = 0..4), L⁻¹, α = Ky⁻¹ y.  Synchronises (the factorisation status).
static int gp_factor(omb_ctx* ctx, int kernel, int n, int d, const double* X, const double* y, const double* ls_host,
                     double variance, double noise, GPFactor* f) {
  const int DP = pad_dim(d);
  const size_t nn = (size_t)n * n;
  const size_t doubles = 3 * nn + 64 * (size_t)n + 2 * (size_t)n + DP +
                         (size_t)gp_grad_blocks(n) * (DP + 1) + DP + 3 + (size_t)cand_cov_ws_doubles(n, DP);
  int rc = grow_dev(ctx, &ctx->fws, &ctx->fws_cap, sizeof(double) * doubles, "GP fit workspace");
  if (rc) return rc;
  double* p = static_cast<double*>(ctx->fws);
  f->Ky = p; p += nn;
  f->Linv = p; p += nn;
  f->Kinv = p; p += nn;
  f->T = p; p += 64 * (size_t)n;
  f->alpha = p; p += n;
  f->v = p; p += n;
  f->ls = p; p += DP;
  f->part = p; p += (size_t)gp_grad_blocks(n) * (DP + 1);
  f->out = p; p += DP + 3;
  f->cws = p;
  void* h = nullptr;
  if ((rc = stage_begin(ctx, sizeof(double) * DP, &h))) return rc;
  for (int j = 0; j < DP; ++j) static_cast<double*>(h)[j] = (j < d) ? ls_host[j] : 1.0;
  OMB_HIP(ctx, hipMemcpyAsync(f->ls, h, sizeof(double) * DP, hipMemcpyHostToDevice, ctx->stream));
  GPDev g{};
  g.ls = f->ls;
  g.variance = variance;
  g.kind = kernel;
  const double base = noise + 1e-8;
  const double mean_diag = variance + base;
  int info = -1;
  f->jitter = 0.0;
  for (int t = -1; t < 5; ++t) {
    const double jit = (t < 0) ? 0.0 : mean_diag * 1e-6 * pow(10.0, (double)t);
    OMB_HIP(ctx, launch_cand_cov(ctx->stream, g, d, DP, X, n, f->Ky, n, f->cws, base + jit, ctx->cov_table));   // Ky = K + (base+jit)·I
    if ((rc = run_cholesky(ctx, f->Ky, n, n, 0.0, &info))) return rc;
    if (info == 0) {
      f->jitter = jit;
      break;
    }
  }
  if (info != 0) return fail(ctx, OMB_ENOTPD, "K + jitter is not positive definite, even with jitter (column %d)", info);
  OMB_HIP(ctx, hipMemsetAsync(f->Linv, 0, sizeof(double) * nn, ctx->stream));
  OMB_HIP(ctx, launch_trinv(ctx->stream, f->Ky, n, n, f->Linv, n, f->T));
  // α = L⁻ᵀ (L⁻¹ y)
  OMB_HIP(ctx, launch_gemm_nn(ctx->stream, n, 1, n, 1.0, f->Linv, n, y, 1, 0.0, f->v, 1));
  OMB_HIP(ctx, launch_gemm_tn(ctx->stream, n, 1, n, 1.0, f->Linv, n, f->v, 1, 0.0, f->alpha, 1));
  return OMB_OK;
}

int omb_gp_lml_grad(omb_ctx* ctx, int kernel, int n, int d, const double* X_dev, const double* y_dev,
                    const double* lengthscale_host, double variance, double noise, double* lml, double* grad,
                    double* jitter_used) {
  int rc = enter(ctx);
  if (rc) return rc;
  if (kernel != OMB_KERNEL_MATERN52 && kernel != OMB_KERNEL_RBF) return fail(ctx, OMB_EINVAL, "unknown kernel %d", kernel);
  if (n < 1 || n > 16384) return fail(ctx, OMB_EUNSUP, "n_train=%d outside [1, 16384]", n);
  if (d < 1 || d > OMB_MAX_DIM) return fail(ctx, OMB_EUNSUP, "n_var=%d outside [1, %d]", d, OMB_MAX_DIM);
  if (!X_dev || !y_dev || !lengthscale_host || !lml || !grad) return fail(ctx, OMB_EINVAL, "null pointer");
  for (int j = 0; j < d; ++j)
    if (!(lengthscale_host[j] > 0.0)) return fail(ctx, OMB_EINVAL, "lengthscale[%d]=%g must be > 0", j, lengthscale_host[j]);
  if (!(variance > 0.0) || !(noise >= 0.0)) return fail(ctx, OMB_EINVAL, "variance must be > 0 and noise >= 0");
  const int DP = pad_dim(d);
  if (gp_lml_small_fits(n, DP)) {
    // one workgroup, one launch, one synchronisation (launch_gp_lml_small); the kernel stores its
    // DP + 5 results straight into the pinned, host-mapped fit_host (no D2H copy per evaluation)
    OMB_HIP(ctx, launch_gp_lml_small(ctx->stream, kernel, DP, X_dev, d, n, lengthscale_host, variance, noise + 1e-8,
                                     y_dev, ctx->fit_dev));
    OMB_HIP(ctx, hipStreamSynchronize(ctx->stream));
    const volatile double* h = ctx->fit_host;
    if (h[DP + 4] != 0.0)
      return fail(ctx, OMB_ENOTPD, "K + jitter is not positive definite, even with jitter (column %d)", (int)h[DP + 4]);
    *lml = -0.5 * h[DP + 2] - h[DP + 1] - 0.5 * n * log(2.0 * M_PI);
    for (int q = 0; q <= d; ++q) grad[q] = h[q];
    if (jitter_used) *jitter_used = h[DP + 3];
    return OMB_OK;
  }
  GPFactor f;
  if ((rc = gp_factor(ctx, kernel, n, d, X_dev, y_dev, lengthscale_host, variance, noise, &f))) return rc;
  // Ky⁻¹ = L⁻ᵀ L⁻¹ (lower triangle), then the gradient sums, log det and yᵀα
  OMB_HIP(ctx, launch_gemm_tn_lower(ctx->stream, n, n, 1.0, f.Linv, n, 0.0, f.Kinv, n));
  OMB_HIP(ctx, launch_gp_grad(ctx->stream, kernel, DP, X_dev, d, n, f.ls, variance, f.alpha, f.Kinv, n, f.part,
                              f.Ky, n, y_dev, f.out));
  OMB_HIP(ctx, hipMemcpyAsync(ctx->fit_host, f.out, sizeof(double) * (DP + 3), hipMemcpyDeviceToHost, ctx->stream));
  OMB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  const volatile double* h = ctx->fit_host;
  // GPy: log p(y) = −½ yᵀα − Σ log L_ii − ½ n log 2π
  *lml = -0.5 * h[DP + 2] - h[DP + 1] - 0.5 * n * log(2.0 * M_PI);
  for (int q = 0; q <= d; ++q) grad[q] = h[q];
  if (jitter_used) *jitter_used = f.jitter;
  return OMB_OK;
}

int omb_gp_lml_grad_batch(omb_ctx* ctx, int kernel, int k, int n, int d, const double* X_dev,
                          const double* const* y_dev, const double* lengthscale_host, const double* variance_host,
                          double noise, double* lml, double* grad_host, double* jitter_used, int* status) {
  int rc = enter(ctx);
  if (rc) return rc;
  if (k < 1 || k > kFitBatchMax) return fail(ctx, OMB_EUNSUP, "k=%d outside [1, %d]", k, kFitBatchMax);
  if (kernel != OMB_KERNEL_MATERN52 && kernel != OMB_KERNEL_RBF) return fail(ctx, OMB_EINVAL, "unknown kernel %d", kernel);
  if (n < 1 || n > 16384) return fail(ctx, OMB_EUNSUP, "n_train=%d outside [1, 16384]", n);
  if (d < 1 || d > OMB_MAX_DIM) return fail(ctx, OMB_EUNSUP, "n_var=%d outside [1, %d]", d, OMB_MAX_DIM);
  if (!X_dev || !y_dev || !lengthscale_host || !variance_host || !lml || !grad_host || !status)
    return fail(ctx, OMB_EINVAL, "null pointer");
  for (int p = 0; p < k; ++p) {
    if (!y_dev[p]) return fail(ctx, OMB_EINVAL, "null y_dev[%d]", p);
    for (int j = 0; j < d; ++j)
      if (!(lengthscale_host[p * d + j] > 0.0))
        return fail(ctx, OMB_EINVAL, "lengthscale[%d][%d]=%g must be > 0", p, j, lengthscale_host[p * d + j]);
    if (!(variance_host[p] > 0.0)) return fail(ctx, OMB_EINVAL, "variance[%d] must be > 0", p);
  }
  if (!(noise >= 0.0)) return fail(ctx, OMB_EINVAL, "noise must be >= 0");
  const int DP = pad_dim(d);
  // n ≤ 96, n_var ≤ 8: one launch.  (Batching up to the one-workgroup kernel's n ≤ 128 was 17% faster on
  // config 1, but between n = 97 and 128 a single evaluation takes the blocked path, and on ill-conditioned
  // K the two agree only to ~1e-7 in log p(y) — enough for the concurrent and sequential fits to reach
  // different optima; every problem here gives exactly what omb_gp_lml_grad gives.)
  if (!gp_lml_small_fits(n, DP)) {
    // blocked path: the problems one after another, each exactly omb_gp_lml_grad
    for (int p = 0; p < k; ++p) {
      rc = omb_gp_lml_grad(ctx, kernel, n, d, X_dev, y_dev[p], lengthscale_host + p * d, variance_host[p], noise,
                           lml + p, grad_host + p * (d + 1), jitter_used ? jitter_used + p : nullptr);
      if (rc != OMB_OK && rc != OMB_ENOTPD) return rc;
      status[p] = rc;
    }
    return OMB_OK;
  }
  // fit_host holds OMB_MAX_DIM + 8 doubles: problem p's DP + 5 results at p·(DP + 5) (k·13 ≤ 52 ≤ 72)
  double* outs[kFitBatchMax];
  for (int p = 0; p < k; ++p) outs[p] = ctx->fit_dev + p * (DP + 5);
  OMB_HIP(ctx, launch_gp_lml_small_batch(ctx->stream, kernel, DP, X_dev, d, n, k, y_dev, lengthscale_host,
                                         variance_host, noise + 1e-8, outs));
  OMB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  for (int p = 0; p < k; ++p) {
    const volatile double* h = ctx->fit_host + p * (DP + 5);
    status[p] = h[DP + 4] != 0.0 ? OMB_ENOTPD : OMB_OK;
    lml[p] = -0.5 * h[DP + 2] - h[DP + 1] - 0.5 * n * log(2.0 * M_PI);
    for (int q = 0; q <= d; ++q) grad_host[p * (d + 1) + q] = h[q];
    if (jitter_used) jitter_used[p] = h[DP + 3];
  }
  return OMB_OK;
}

int omb_gp_fit_state(omb_ctx* ctx, int obj, int kernel, int n, int d, const double* X_dev, const double* y_dev,
                     const double* lengthscale_host, double variance, double noise, double* jitter_used) {
  int rc = enter(ctx);
  if (rc) return rc;
  if (obj < 0 || obj >= OMB_MAX_OBJ) return fail(ctx, OMB_EINVAL, "obj=%d outside [0, %d)", obj, OMB_MAX_OBJ);
  if (kernel != OMB_KERNEL_MATERN52 && kernel != OMB_KERNEL_RBF) return fail(ctx, OMB_EINVAL, "unknown kernel %d", kernel);
  if (n < 1 || n > OMB_MAX_TRAIN_DENSE)
    return fail(ctx, OMB_EUNSUP, "n_train=%d outside [1, %d]", n, OMB_MAX_TRAIN_DENSE);
  if (d < 1 || d > OMB_MAX_DIM) return fail(ctx, OMB_EUNSUP, "n_var=%d outside [1, %d]", d, OMB_MAX_DIM);
  if (!X_dev || !y_dev || !lengthscale_host) return fail(ctx, OMB_EINVAL, "null pointer");
  for (int j = 0; j < d; ++j)
    if (!(lengthscale_host[j] > 0.0)) return fail(ctx, OMB_EINVAL, "lengthscale[%d]=%g must be > 0", j, lengthscale_host[j]);
  if (!(variance > 0.0) || !(noise >= 0.0)) return fail(ctx, OMB_EINVAL, "variance must be > 0 and noise >= 0");
  GPFactor f;
  if ((rc = gp_factor(ctx, kernel, n, d, X_dev, y_dev, lengthscale_host, variance, noise, &f))) return rc;
  if (jitter_used) *jitter_used = f.jitter;
  return omb_set_gp(ctx, obj, kernel, n, d, X_dev, lengthscale_host, variance, f.alpha, f.Linv);
}

// ---------------------------------------------------------------------------------------
// ParEGO / KEEP evolutionary acquisition search: parego.py:223-271, keep.py:240-292.
int omb_ea_search(omb_ctx* ctx, int mode, double best, double var_eps, const double* pop_dev, int P, int iters,
                  const int32_t* sel_dev, const int8_t* cross_dev, const double* beta_dev, const int8_t* mut_dev,
                  const double* lower_dev, const double* upper_dev, double* out_dev) {
  int rc = enter(ctx);
  if (rc) return rc;
  if (mode != OMB_EA_EI && mode != OMB_EA_PARETO_EI) return fail(ctx, OMB_EINVAL, "unknown search mode %d", mode);
  if ((rc = check_obj(ctx, 0))) return rc;
  if (mode == OMB_EA_PARETO_EI && (rc = check_obj(ctx, 1))) return rc;
  const ObjState& s0 = ctx->obj[0];
  if (mode == OMB_EA_PARETO_EI && ctx->obj[1].d != s0.d)
    return fail(ctx, OMB_EINVAL, "objectives 0 and 1 disagree on n_var (%d vs %d)", s0.d, ctx->obj[1].d);
  if (P < 3 || P > kEAMaxPop) return fail(ctx, OMB_EINVAL, "population size %d outside [3, %d]", P, kEAMaxPop);
  if (iters < 0) return fail(ctx, OMB_EINVAL, "iters=%d must be >= 0", iters);
  if (s0.n > kEAMaxTrain || (mode == OMB_EA_PARETO_EI && ctx->obj[1].n > kEAMaxTrain))
    return fail(ctx, OMB_EUNSUP, "n_train above %d", kEAMaxTrain);
  if (!(var_eps >= 0.0)) return fail(ctx, OMB_EINVAL, "var_eps=%g must be >= 0", var_eps);
  if (!pop_dev || !lower_dev || !upper_dev || !out_dev || (iters > 0 && (!sel_dev || !cross_dev || !beta_dev || !mut_dev)))
    return fail(ctx, OMB_EINVAL, "null device pointer");
  if ((rc = grow_dev(ctx, &ctx->ews, &ctx->ews_cap, sizeof(double) * (size_t)s0.n * s0.n, "search workspace")))
    return rc;
  EASearch es{};
  es.g0 = s0.dev;
  es.g1 = (mode == OMB_EA_PARETO_EI) ? ctx->obj[1].dev : s0.dev;
  es.Ld0 = s0.Ld;
  es.mode = mode;
  es.d = s0.d;
  es.DP = s0.DP;
  es.P = P;
  es.iters = iters;
  es.best = best;
  es.var_eps = var_eps;
  es.pop = pop_dev;
  es.sel = sel_dev;
  es.cross = cross_dev;
  es.beta = beta_dev;
  es.mut = mut_dev;
  es.lower = lower_dev;
  es.upper = upper_dev;
  es.out = out_dev;
  hipError_t e = launch_ea_search(ctx->stream, es, static_cast<double*>(ctx->ews));
  if (e != hipSuccess) return hip_fail(ctx, e, "ea_search");
  return OMB_OK;
}

}  // extern "C"
