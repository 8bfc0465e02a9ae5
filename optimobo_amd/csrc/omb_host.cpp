// Host-only validation and packing of the C-ABI's arguments (see omb_host.h).  Every size product is formed in
// 64 bits: the entry points take int / int64_t counts straight from the caller, so a hostile M or C must fail the
// check, not overflow it (UBSan in `make asan` holds this file to that).
#include "omb_host.h"

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

namespace omb {

int errf(std::string* err, int code, const char* fmt, ...) {
  if (err) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    *err = buf;
  }
  return code;
}

int pad_dim(int d) {
  const int opts[] = {2, 4, 6, 8, 16, 32, 64, 128, 256};   // > 64: the wide path (omb_wide.hip)
  for (int o : opts)
    if (d <= o) return o;
  return -1;
}

int check_moments(std::string* err, const void* mu, const void* var, int64_t ld, int64_t N, int k, const void* out) {
  if (N < 0) return errf(err, OMB_EINVAL, "N=%lld < 0", (long long)N);
  if (N > 0 && (!mu || !var || !out)) return errf(err, OMB_EINVAL, "null device pointer");
  if (k > 1 && ld < N) return errf(err, OMB_EINVAL, "ld=%lld < N=%lld", (long long)ld, (long long)N);
  return OMB_OK;
}

int check_ehvi2d(std::string* err, int P, const double* r, int mode) {
  // stripes y1[0..P], y2[1..P] are staged in ≤ 64 KiB of LDS
  if (P < 1 || P > kMaxStripes) return errf(err, OMB_EUNSUP, "Pareto front size P=%d outside [1, %d]", P, kMaxStripes);
  if (!r) return errf(err, OMB_EINVAL, "null reference point");
  if (mode != OMB_EHVI_REFERENCE && mode != OMB_EHVI_TEXTBOOK && mode != OMB_EHVI_SIGMA)
    return errf(err, OMB_EINVAL, "unknown EHVI mode %d", mode);
  return OMB_OK;
}

int check_ehvi_mc(std::string* err, int k, int M, const double* r) {
  if (k < 2 || k > OMB_MAX_OBJ)
    return errf(err, OMB_EINVAL, "Monte-Carlo EHVI needs 2 <= k <= %d objectives (k=%d)", OMB_MAX_OBJ, k);
  // the (M, k) cache is staged in <= 64 KiB of dynamic LDS
  if (M < 1 || (int64_t)k * M > kMaxLdsDoubles)
    return errf(err, OMB_EUNSUP, "cache size M=%d outside [1, %d] for k=%d", M, kMaxLdsDoubles / k, k);
  if (!r) return errf(err, OMB_EINVAL, "null reference point");
  return OMB_OK;
}

int check_boxes(std::string* err, int k, int C, int B) {
  if (k != 2 && k != 3) return errf(err, OMB_EUNSUP, "exact EHVI needs k = 2 or 3 objectives (k=%d)", k);
  // grid + 4 per-wave Φ/φ tables must fit the 64 KiB of dynamic LDS
  if (C < 2 || (int64_t)k * C * 9 > kMaxLdsDoubles)
    return errf(err, OMB_EUNSUP, "grid size C=%d outside [2, %d] for k=%d", C, kMaxLdsDoubles / (9 * k), k);
  if (B < 1) return errf(err, OMB_EINVAL, "empty box list");
  return OMB_OK;
}

int check_ei(std::string* err, int kind, int k, double var_eps, double pof_eps) {
  const bool ok = (kind == OMB_EI_PLAIN && k == 1) || (kind == OMB_EI_PARETO && k == 2) ||
                  (kind == OMB_EI_CONSTRAINED && k >= 2 && k <= OMB_MAX_OBJ);
  if (!ok) return errf(err, OMB_EINVAL, "EI kind %d does not take k=%d posterior rows", kind, k);
  if (!(var_eps >= 0.0) || !(pof_eps >= 0.0)) return errf(err, OMB_EINVAL, "var_eps/pof_eps must be >= 0");
  return OMB_OK;
}

int check_hvpoi(std::string* err, int C) {
  if (C < 1 || 4 * (int64_t)C > kMaxLdsDoubles)
    return errf(err, OMB_EUNSUP, "cell count C=%d outside [1, %d]", C, kMaxLdsDoubles / 4);
  return OMB_OK;
}

int build_scal(std::string* err, int k, int M, int scal_id, const double* params_host, const double* weights_host,
               const double* ideal_host, const double* max_host, double agg_min, ScalParams* out) {
  if (k < 1 || k > OMB_MAX_OBJ) return errf(err, OMB_EINVAL, "k=%d outside [1, %d]", k, OMB_MAX_OBJ);
  if (M < 1 || (int64_t)k * M > kMaxLdsDoubles)
    return errf(err, OMB_EUNSUP, "cache size M=%d x k=%d exceeds %d doubles of LDS", M, k, kMaxLdsDoubles);
  if (scal_id < OMB_SCAL_WS || scal_id > OMB_SCAL_APD) return errf(err, OMB_EINVAL, "unknown scalarisation %d", scal_id);
  if (!weights_host || !ideal_host || !max_host) return errf(err, OMB_EINVAL, "null weights/ideal/max");
  ScalParams& sp = *out;
  memset(&sp, 0, sizeof(sp));
  sp.id = scal_id;
  sp.k = k;
  sp.agg_min = agg_min;
  double wq = 0.0, rsum = 0.0;
  for (int i = 0; i < k; ++i) {
    sp.w[i] = weights_host[i];
    sp.ideal[i] = ideal_host[i];
    sp.range[i] = max_host[i] - ideal_host[i];
    wq += sp.w[i] * sp.w[i];
    rsum += sp.range[i];
  }
  sp.wnorm = sqrt(wq);
  const int np = (scal_id == OMB_SCAL_QPBI || scal_id == OMB_SCAL_APD) ? 3
                 : (scal_id == OMB_SCAL_WS || scal_id == OMB_SCAL_TCH || scal_id == OMB_SCAL_WPR) ? 0 : 1;
  if (np > 0 && !params_host) return errf(err, OMB_EINVAL, "scalarisation %d needs %d parameter(s)", scal_id, np);
  for (int i = 0; i < np; ++i) sp.p[i] = params_host[i];
  if (scal_id == OMB_SCAL_APD && sp.wnorm == 0.0) {
    // scalarisations.py:392-393 substitutes 1e-5 weights (the reference then fails for k > 1).
    for (int i = 0; i < k; ++i) sp.w[i] = 1e-5;
    sp.wnorm = sqrt(k * 1e-10);
  }
  if (scal_id == OMB_SCAL_QPBI) {
    // scalarisations.py:347: alpha * (1/H * 1/k * Σ(max − ideal))
    sp.d_star = sp.p[1] * ((1.0 / sp.p[2]) * (1.0 / (double)k) * rsum);
  }
  return OMB_OK;
}

int check_gp_args(std::string* err, int obj, int kernel, int n, int d, const void* X_dev, const double* lengthscale_host,
                  double variance, const void* alpha_dev, const void* Linv_dev) {
  if (obj < 0 || obj >= OMB_MAX_OBJ) return errf(err, OMB_EINVAL, "obj=%d outside [0, %d)", obj, OMB_MAX_OBJ);
  if (kernel != OMB_KERNEL_MATERN52 && kernel != OMB_KERNEL_RBF) return errf(err, OMB_EINVAL, "unknown kernel %d", kernel);
  if (n < 1 || n > OMB_MAX_TRAIN_DENSE)
    return errf(err, OMB_EUNSUP, "n_train=%d outside [1, %d]", n, OMB_MAX_TRAIN_DENSE);
  if (d < 1 || d > OMB_MAX_DIM) return errf(err, OMB_EUNSUP, "n_var=%d outside [1, %d]", d, OMB_MAX_DIM);
  if (!X_dev || !lengthscale_host || !alpha_dev || !Linv_dev) return errf(err, OMB_EINVAL, "null pointer");
  for (int j = 0; j < d; ++j)
    if (!(lengthscale_host[j] > 0.0))
      return errf(err, OMB_EINVAL, "lengthscale[%d]=%g must be > 0", j, lengthscale_host[j]);
  if (!(variance >= 0.0)) return errf(err, OMB_EINVAL, "variance=%g must be >= 0", variance);
  return OMB_OK;
}

int check_sobol_args(std::string* err, int d, int bits, const void* sv_host, const void* shift_host,
                     const double* lo_host, const double* hi_host) {
  if (d < 1 || d > OMB_MAX_DIM) return errf(err, OMB_EUNSUP, "Sobol dimension %d outside [1, %d]", d, OMB_MAX_DIM);
  if (bits < 1 || bits > 32) return errf(err, OMB_EUNSUP, "Sobol bits=%d outside [1, 32]", bits);
  if (!sv_host || !shift_host || !lo_host || !hi_host) return errf(err, OMB_EINVAL, "null Sobol state");
  for (int j = 0; j < d; ++j)
    if (!(hi_host[j] >= lo_host[j]))
      return errf(err, OMB_EINVAL, "box [%g, %g] of dimension %d is empty", lo_host[j], hi_host[j], j);
  return OMB_OK;
}

size_t sobol_state_bytes(int d, int bits) {
  const int words = d * bits + d;
  return (size_t)((words + 1) & ~1) * 4 + (size_t)2 * d * sizeof(double);
}

void sobol_pack_state(int d, int bits, const uint32_t* sv, const uint32_t* shift, const double* lo, const double* hi,
                      void* dst) {
  uint32_t* w = static_cast<uint32_t*>(dst);
  const int words = d * bits + d;
  for (int t = 0; t < d * bits; ++t) w[t] = sv[t];
  for (int t = 0; t < d; ++t) w[d * bits + t] = shift[t];
  if (words & 1) w[words] = 0;
  double* f = reinterpret_cast<double*>(w + ((words + 1) & ~1));
  for (int t = 0; t < d; ++t) {
    f[t] = lo[t];
    f[d + t] = hi[t] - lo[t];   // numpy's (hi - lo), rounded once
  }
}

}  // namespace omb
