// Device fp64 math shared by the kernels: the reference's scalar formulas, restated for gfx950.
#pragma once

#include <hip/hip_runtime.h>

namespace omb {

constexpr double kSqrt5 = 2.23606797749979;            // np.sqrt(5.)
constexpr double kFiveThirds = 5.0 / 3.0;               // 5./3
constexpr double kSqrt2Pi = 2.5066282746310002;         // np.sqrt(2*np.pi)   (scipy _norm_pdf_C)
constexpr double kSqrt1_2 = 0.70710678118654752440;     // NPY_SQRT1_2

// scipy.special.ndtr (cephes ndtr.c) — scipy.stats.norm.cdf.
__device__ __forceinline__ double ndtr(double a) {
  double x = a * kSqrt1_2;
  double z = fabs(x);
  if (z < kSqrt1_2) return 0.5 + 0.5 * erf(x);
  double y = 0.5 * erfc(z);
  return (x > 0.0) ? 1.0 - y : y;
}

// scipy.stats.norm.pdf: exp(-x**2/2.0) / sqrt(2π).
__device__ __forceinline__ double npdf(double t) { return exp(-(t * t) / 2.0) / kSqrt2Pi; }

// util_functions.py:130-133  ψ(a,b,m,s) = s·φ((b−m)/s) + (a−m)·Φ((b−m)/s), given t=(b−m)/s.
__device__ __forceinline__ double psi_t(double a, double m, double s, double t, double pdf_t, double cdf_t) {
  (void)t;
  return s * pdf_t + (a - m) * cdf_t;
}

// exp(x) for x ≤ 0 — the only range the kernels need (−√5 r, −r²/2).  Cody–Waite reduction
// x = k·ln2 + f, |f| ≤ ln2/2, degree-11 near-minimax polynomial (fitted with mpmath.chebyfit;
// max relative error 2.2e-16 in double), result 2^k·p(f).  Without the overflow / NaN branches
// of the libm exp it is 17 instead of 22 fp64 instructions; x < −745 underflows to 0 in ldexp.
__device__ __forceinline__ double exp_nonpos(double x) {
  const double k = rint(x * 1.4426950408889634);          // log2(e)
  double f = fma(-k, 6.93147180369123816490e-01, x);       // ln2_hi (k·ln2_hi exact)
  f = fma(-k, 1.90821492927058770002e-10, f);              // ln2_lo
  double p = 2.5110037605963777e-08;
  p = fma(p, f, 2.763263963904103e-07);
  p = fma(p, f, 2.755724091857897e-06);
  p = fma(p, f, 2.4801485482328494e-05);
  p = fma(p, f, 0.00019841269890047113);
  p = fma(p, f, 0.0013888888952314775);
  p = fma(p, f, 0.008333333333319601);
  p = fma(p, f, 0.0416666666664881);
  p = fma(p, f, 0.1666666666666668);
  p = fma(p, f, 0.5000000000000019);
  p = fma(p, f, 1.0);
  p = fma(p, f, 1.0);
  return ldexp(p, (int)k);
}

// sqrt(a) for a ≥ 0: v_rsq_f64 seed, one Goldschmidt step and two residual corrections (the
// libm sequence without its denormal rescaling and special-value branches: 10 instead of 17
// instructions).  a below 1e-300 — far under any squared distance that matters — returns 0.
__device__ __forceinline__ double sqrt_nonneg(double a) {
  const double y = __builtin_amdgcn_rsq(a);
  double g = a * y, h = 0.5 * y;
  const double r = fma(-g, h, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  double d = fma(-g, g, a);
  g = fma(d, h, g);
  d = fma(-g, g, a);
  g = fma(d, h, g);
  return a > 1e-300 ? g : 0.0;
}

// GPy Matern52.K_of_r: variance*(1+sqrt(5)*r+5/3*r**2)*exp(-sqrt(5)*r)  (r ≥ 0)
// GPy RBF.K_of_r     : variance*exp(-r**2/2)
// FAST selects exp_nonpos / sqrt_nonneg (default) or the libm functions (ablation reference).
template <int KIND, bool FAST = true>
__device__ __forceinline__ double kernel_of_r2(double r2, double variance) {
  r2 = r2 > 0.0 ? r2 : 0.0;                 // np.clip(r2, 0, inf)
  const double r = FAST ? sqrt_nonneg(r2) : sqrt(r2);
  if constexpr (KIND == OMB_KERNEL_MATERN52) {
    const double poly = (1.0 + kSqrt5 * r) + kFiveThirds * (r * r);
    return (variance * poly) * (FAST ? exp_nonpos(-(kSqrt5 * r)) : exp(-(kSqrt5 * r)));
  } else {
    return variance * (FAST ? exp_nonpos(-0.5 * (r * r)) : exp(-0.5 * (r * r)));
  }
}

}  // namespace omb
