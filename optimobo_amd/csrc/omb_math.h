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

// exp_nonpos's polynomial (degree 11, highest first; the last two coefficients are 1.0) as a value
// the kernels take as an ARGUMENT: kernel arguments live in SGPRs, and v_fma_f64 accepts an SGPR
// operand, whereas a literal coefficient makes the compiler emit the v_fmac form with the addend
// materialised by two v_mov_b32 per Horner step (20 extra VALU issues per element in the posterior
// and K-block generation loops).
struct ExpCoef {
  double c[10];
};
__host__ __device__ constexpr ExpCoef exp_coef() {
  return ExpCoef{{2.5110037605963777e-08, 2.763263963904103e-07, 2.755724091857897e-06, 2.4801485482328494e-05,
                  0.00019841269890047113, 0.0013888888952314775, 0.008333333333319601, 0.0416666666664881,
                  0.1666666666666668, 0.5000000000000019}};
}

// a·b + c with c a wave-uniform value: the VOP3 v_fma_f64 takes c straight from an SGPR pair (the
// compiler otherwise picks the two-address v_fmac and first copies c into VGPRs, 2 v_mov_b32 each).
__device__ __forceinline__ double fma_vvs(double a, double b, double c) {
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
  return r;
}

// exp_nonpos with its coefficients from `ec` (bit-identical results).
__device__ __forceinline__ double exp_nonpos_k(double x, const ExpCoef& ec) {
  const double k = rint(x * 1.4426950408889634);
  double f = fma(-k, 6.93147180369123816490e-01, x);
  f = fma(-k, 1.90821492927058770002e-10, f);
  double p = ec.c[0];
#pragma unroll
  for (int i = 1; i < 10; ++i) p = fma_vvs(p, f, ec.c[i]);
  p = fma(p, f, 1.0);
  p = fma(p, f, 1.0);
  return ldexp(p, (int)k);
}

// kernel_of_r2 (FAST form) with exp_nonpos_k.
template <int KIND>
__device__ __forceinline__ double kernel_of_r2_k(double r2, double variance, const ExpCoef& ec) {
  r2 = r2 > 0.0 ? r2 : 0.0;
  const double r = sqrt_nonneg(r2);
  if constexpr (KIND == OMB_KERNEL_MATERN52) {
    const double poly = (1.0 + kSqrt5 * r) + kFiveThirds * (r * r);
    return (variance * poly) * exp_nonpos_k(-(kSqrt5 * r), ec);
  } else {
    return variance * exp_nonpos_k(-0.5 * (r * r), ec);
  }
}

// Two independent kernel_of_r2_k evaluations written in lockstep (bit-identical to two calls): the
// ~50-deep fp64 dependency chain of one evaluation leaves the VALU waiting on its own results, and
// the compiler does not interleave two calls on its own at the posterior kernel's register pressure.
template <int KIND>
__device__ __forceinline__ void kernel_of_r2_k_x2(double r2a, double r2b, double variance, const ExpCoef& ec,
                                                  double& outa, double& outb) {
  r2a = r2a > 0.0 ? r2a : 0.0;
  r2b = r2b > 0.0 ? r2b : 0.0;
  // sqrt_nonneg ×2
  const double ya = __builtin_amdgcn_rsq(r2a), yb = __builtin_amdgcn_rsq(r2b);
  double ga = r2a * ya, gb = r2b * yb, ha = 0.5 * ya, hb = 0.5 * yb;
  const double qa = fma(-ga, ha, 0.5), qb = fma(-gb, hb, 0.5);
  ga = fma(ga, qa, ga);
  gb = fma(gb, qb, gb);
  ha = fma(ha, qa, ha);
  hb = fma(hb, qb, hb);
  double da = fma(-ga, ga, r2a), db = fma(-gb, gb, r2b);
  ga = fma(da, ha, ga);
  gb = fma(db, hb, gb);
  da = fma(-ga, ga, r2a);
  db = fma(-gb, gb, r2b);
  ga = fma(da, ha, ga);
  gb = fma(db, hb, gb);
  const double ra = r2a > 1e-300 ? ga : 0.0, rb = r2b > 1e-300 ? gb : 0.0;
  double xa, xb, pa_, pb_;
  if constexpr (KIND == OMB_KERNEL_MATERN52) {
    pa_ = (1.0 + kSqrt5 * ra) + kFiveThirds * (ra * ra);
    pb_ = (1.0 + kSqrt5 * rb) + kFiveThirds * (rb * rb);
    xa = -(kSqrt5 * ra);
    xb = -(kSqrt5 * rb);
  } else {
    pa_ = 1.0;
    pb_ = 1.0;
    xa = -0.5 * (ra * ra);
    xb = -0.5 * (rb * rb);
  }
  // exp_nonpos_k ×2
  const double ka = rint(xa * 1.4426950408889634), kb = rint(xb * 1.4426950408889634);
  double fa = fma(-ka, 6.93147180369123816490e-01, xa), fb = fma(-kb, 6.93147180369123816490e-01, xb);
  fa = fma(-ka, 1.90821492927058770002e-10, fa);
  fb = fma(-kb, 1.90821492927058770002e-10, fb);
  double pa = ec.c[0], pb = ec.c[0];
#pragma unroll
  for (int i = 1; i < 10; ++i) {
    pa = fma_vvs(pa, fa, ec.c[i]);
    pb = fma_vvs(pb, fb, ec.c[i]);
  }
  pa = fma(pa, fa, 1.0);
  pb = fma(pb, fb, 1.0);
  pa = fma(pa, fa, 1.0);
  pb = fma(pb, fb, 1.0);
  const double ea = ldexp(pa, (int)ka), eb = ldexp(pb, (int)kb);
  if constexpr (KIND == OMB_KERNEL_MATERN52) {
    outa = (variance * pa_) * ea;
    outb = (variance * pb_) * eb;
  } else {
    outa = variance * ea;
    outb = variance * eb;
  }
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
