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

// GPy Matern52.K_of_r: variance*(1+sqrt(5)*r+5/3*r**2)*exp(-sqrt(5)*r)  (r ≥ 0)
// GPy RBF.K_of_r     : variance*exp(-r**2/2)
template <int KIND>
__device__ __forceinline__ double kernel_of_r2(double r2, double variance) {
  r2 = r2 > 0.0 ? r2 : 0.0;                 // np.clip(r2, 0, inf)
  if constexpr (KIND == OMB_KERNEL_MATERN52) {
    double r = sqrt(r2);
    double poly = (1.0 + kSqrt5 * r) + kFiveThirds * (r * r);
    return (variance * poly) * exp(-(kSqrt5 * r));
  } else {
    double r = sqrt(r2);
    return variance * exp(-0.5 * (r * r));
  }
}

}  // namespace omb
