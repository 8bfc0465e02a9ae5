// Device fp64 math shared by the kernels: the reference's scalar formulas, restated for gfx950.
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/optimobo_hip.h"

namespace omb {

constexpr double kSqrt5 = 2.23606797749979;            // np.sqrt(5.)
constexpr double kFiveThirds = 5.0 / 3.0;               // 5./3
constexpr double kSqrt2Pi = 2.5066282746310002;         // np.sqrt(2*np.pi)   (scipy _norm_pdf_C)
constexpr double kSqrt1_2 = 0.70710678118654752440;     // NPY_SQRT1_2

// scipy.special.ndtr (cephes ndtr.c) — scipy.stats.norm.cdf.
// The acquisition arithmetic below runs unfused (fp contract off): the same function inlined into two kernels
// must give bitwise the same value (the one-launch chains against the separate launches), and the contraction
// choices of -ffp-contract=fast depend on the surrounding code (a 1-ulp EHVI difference, gpurun_out/r04_d).
__device__ __forceinline__ double ndtr(double a) {
#pragma clang fp contract(off)
  double x = a * kSqrt1_2;
  double z = fabs(x);
  if (z < kSqrt1_2) return 0.5 + 0.5 * erf(x);
  double y = 0.5 * erfc(z);
  return (x > 0.0) ? 1.0 - y : y;
}

// scipy.stats.norm.pdf: exp(-x**2/2.0) / sqrt(2π).
__device__ __forceinline__ double npdf(double t) {
#pragma clang fp contract(off)
  return exp(-(t * t) / 2.0) / kSqrt2Pi;
}

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
// The same struct carries the constants of the table-driven exp (exp_tab below) in t[].
struct ExpCoef {
  double c[10];
  double t[8];   // −√5·64/ln2, ln2_hi/64, ln2_lo/64, 1/120, 1/24, 1/6, 1/2, r²_min
  double u[8];   // kernel_of_r2_tab256_x2: −√5·256/ln2, c_hi, c_lo (c = ln2/(256√5)), a4, a3, a2, a1 (a_i = (−√5)^i/i!)
};
__host__ __device__ constexpr ExpCoef exp_coef() {
  return ExpCoef{{2.5110037605963777e-08, 2.763263963904103e-07, 2.755724091857897e-06, 2.4801485482328494e-05,
                  0.00019841269890047113, 0.0013888888952314775, 0.008333333333319601, 0.0416666666664881,
                  0.1666666666666668, 0.5000000000000019},
                 {-2.23606797749979 * 92.33248261689366, 6.93147180369123816490e-01 / 64, 1.90821492927058770002e-10 / 64, 1.0 / 120,
                  1.0 / 24, 1.0 / 6, 0.5, 1e-300},
                 {-825.8468306507675, 0.00121087829230028, 5.726751604518302e-20, 1.0416666666666667,
                  -1.8633899812498247, 2.5, -2.23606797749979, 0.0}};
}

// 2^(j/64), j = 0..63, correctly rounded (computed with 50-digit decimal arithmetic).
__device__ constexpr double kExp2Tab64[64] = {
    0x1.0000000000000p+0, 0x1.02c9a3e778061p+0, 0x1.059b0d3158574p+0, 0x1.0874518759bc8p+0,
    0x1.0b5586cf9890fp+0, 0x1.0e3ec32d3d1a2p+0, 0x1.11301d0125b51p+0, 0x1.1429aaea92de0p+0,
    0x1.172b83c7d517bp+0, 0x1.1a35beb6fcb75p+0, 0x1.1d4873168b9aap+0, 0x1.2063b88628cd6p+0,
    0x1.2387a6e756238p+0, 0x1.26b4565e27cddp+0, 0x1.29e9df51fdee1p+0, 0x1.2d285a6e4030bp+0,
    0x1.306fe0a31b715p+0, 0x1.33c08b26416ffp+0, 0x1.371a7373aa9cbp+0, 0x1.3a7db34e59ff7p+0,
    0x1.3dea64c123422p+0, 0x1.4160a21f72e2ap+0, 0x1.44e086061892dp+0, 0x1.486a2b5c13cd0p+0,
    0x1.4bfdad5362a27p+0, 0x1.4f9b2769d2ca7p+0, 0x1.5342b569d4f82p+0, 0x1.56f4736b527dap+0,
    0x1.5ab07dd485429p+0, 0x1.5e76f15ad2148p+0, 0x1.6247eb03a5585p+0, 0x1.6623882552225p+0,
    0x1.6a09e667f3bcdp+0, 0x1.6dfb23c651a2fp+0, 0x1.71f75e8ec5f74p+0, 0x1.75feb564267c9p+0,
    0x1.7a11473eb0187p+0, 0x1.7e2f336cf4e62p+0, 0x1.82589994cce13p+0, 0x1.868d99b4492edp+0,
    0x1.8ace5422aa0dbp+0, 0x1.8f1ae99157736p+0, 0x1.93737b0cdc5e5p+0, 0x1.97d829fde4e50p+0,
    0x1.9c49182a3f090p+0, 0x1.a0c667b5de565p+0, 0x1.a5503b23e255dp+0, 0x1.a9e6b5579fdbfp+0,
    0x1.ae89f995ad3adp+0, 0x1.b33a2b84f15fbp+0, 0x1.b7f76f2fb5e47p+0, 0x1.bcc1e904bc1d2p+0,
    0x1.c199bdd85529cp+0, 0x1.c67f12e57d14bp+0, 0x1.cb720dcef9069p+0, 0x1.d072d4a07897cp+0,
    0x1.d5818dcfba487p+0, 0x1.da9e603db3285p+0, 0x1.dfc97337b9b5fp+0, 0x1.e502ee78b3ff6p+0,
    0x1.ea4afa2a490dap+0, 0x1.efa1bee615a27p+0, 0x1.f50765b6e4540p+0, 0x1.fa7c1819e90d8p+0};

// 2^(j/256), j = 0..255, correctly rounded (tools/gen_exp2_table.py: 60-digit decimal arithmetic).
__device__ constexpr double kExp2Tab256[256] = {
    0x1.0000000000000p+0, 0x1.00b1afa5abcbfp+0, 0x1.0163da9fb3335p+0, 0x1.02168143b0281p+0,
    0x1.02c9a3e778061p+0, 0x1.037d42e11bbccp+0, 0x1.04315e86e7f85p+0, 0x1.04e5f72f654b1p+0,
    0x1.059b0d3158574p+0, 0x1.0650a0e3c1f89p+0, 0x1.0706b29ddf6dep+0, 0x1.07bd42b72a836p+0,
    0x1.0874518759bc8p+0, 0x1.092bdf66607e0p+0, 0x1.09e3ecac6f383p+0, 0x1.0a9c79b1f3919p+0,
    0x1.0b5586cf9890fp+0, 0x1.0c0f145e46c85p+0, 0x1.0cc922b7247f7p+0, 0x1.0d83b23395decp+0,
    0x1.0e3ec32d3d1a2p+0, 0x1.0efa55fdfa9c5p+0, 0x1.0fb66affed31bp+0, 0x1.1073028d7233ep+0,
    0x1.11301d0125b51p+0, 0x1.11edbab5e2ab6p+0, 0x1.12abdc06c31ccp+0, 0x1.136a814f204abp+0,
    0x1.1429aaea92de0p+0, 0x1.14e95934f312ep+0, 0x1.15a98c8a58e51p+0, 0x1.166a45471c3c2p+0,
    0x1.172b83c7d517bp+0, 0x1.17ed48695bbc0p+0, 0x1.18af9388c8deap+0, 0x1.1972658375d2fp+0,
    0x1.1a35beb6fcb75p+0, 0x1.1af99f8138a1cp+0, 0x1.1bbe084045cd4p+0, 0x1.1c82f95281c6bp+0,
    0x1.1d4873168b9aap+0, 0x1.1e0e75eb44027p+0, 0x1.1ed5022fcd91dp+0, 0x1.1f9c18438ce4dp+0,
    0x1.2063b88628cd6p+0, 0x1.212be3578a819p+0, 0x1.21f49917ddc96p+0, 0x1.22bdda27912d1p+0,
    0x1.2387a6e756238p+0, 0x1.2451ffb82140ap+0, 0x1.251ce4fb2a63fp+0, 0x1.25e85711ece75p+0,
    0x1.26b4565e27cddp+0, 0x1.2780e341ddf29p+0, 0x1.284dfe1f56381p+0, 0x1.291ba7591bb70p+0,
    0x1.29e9df51fdee1p+0, 0x1.2ab8a66d10f13p+0, 0x1.2b87fd0dad990p+0, 0x1.2c57e39771b2fp+0,
    0x1.2d285a6e4030bp+0, 0x1.2df961f641589p+0, 0x1.2ecafa93e2f56p+0, 0x1.2f9d24abd886bp+0,
    0x1.306fe0a31b715p+0, 0x1.31432edeeb2fdp+0, 0x1.32170fc4cd831p+0, 0x1.32eb83ba8ea32p+0,
    0x1.33c08b26416ffp+0, 0x1.3496266e3fa2dp+0, 0x1.356c55f929ff1p+0, 0x1.36431a2de883bp+0,
    0x1.371a7373aa9cbp+0, 0x1.37f26231e754ap+0, 0x1.38cae6d05d866p+0, 0x1.39a401b7140efp+0,
    0x1.3a7db34e59ff7p+0, 0x1.3b57fbfec6cf4p+0, 0x1.3c32dc313a8e5p+0, 0x1.3d0e544ede173p+0,
    0x1.3dea64c123422p+0, 0x1.3ec70df1c5175p+0, 0x1.3fa4504ac801cp+0, 0x1.40822c367a024p+0,
    0x1.4160a21f72e2ap+0, 0x1.423fb2709468ap+0, 0x1.431f5d950a897p+0, 0x1.43ffa3f84b9d4p+0,
    0x1.44e086061892dp+0, 0x1.45c2042a7d232p+0, 0x1.46a41ed1d0057p+0, 0x1.4786d668b3237p+0,
    0x1.486a2b5c13cd0p+0, 0x1.494e1e192aed2p+0, 0x1.4a32af0d7d3dep+0, 0x1.4b17dea6db7d7p+0,
    0x1.4bfdad5362a27p+0, 0x1.4ce41b817c114p+0, 0x1.4dcb299fddd0dp+0, 0x1.4eb2d81d8abffp+0,
    0x1.4f9b2769d2ca7p+0, 0x1.508417f4531eep+0, 0x1.516daa2cf6642p+0, 0x1.5257de83f4eefp+0,
    0x1.5342b569d4f82p+0, 0x1.542e2f4f6ad27p+0, 0x1.551a4ca5d920fp+0, 0x1.56070dde910d2p+0,
    0x1.56f4736b527dap+0, 0x1.57e27dbe2c4cfp+0, 0x1.58d12d497c7fdp+0, 0x1.59c0827ff07ccp+0,
    0x1.5ab07dd485429p+0, 0x1.5ba11fba87a03p+0, 0x1.5c9268a5946b7p+0, 0x1.5d84590998b93p+0,
    0x1.5e76f15ad2148p+0, 0x1.5f6a320dceb71p+0, 0x1.605e1b976dc09p+0, 0x1.6152ae6cdf6f4p+0,
    0x1.6247eb03a5585p+0, 0x1.633dd1d1929fdp+0, 0x1.6434634ccc320p+0, 0x1.652b9febc8fb7p+0,
    0x1.6623882552225p+0, 0x1.671c1c70833f6p+0, 0x1.68155d44ca973p+0, 0x1.690f4b19e9538p+0,
    0x1.6a09e667f3bcdp+0, 0x1.6b052fa75173ep+0, 0x1.6c012750bdabfp+0, 0x1.6cfdcddd47645p+0,
    0x1.6dfb23c651a2fp+0, 0x1.6ef9298593ae5p+0, 0x1.6ff7df9519484p+0, 0x1.70f7466f42e87p+0,
    0x1.71f75e8ec5f74p+0, 0x1.72f8286ead08ap+0, 0x1.73f9a48a58174p+0, 0x1.74fbd35d7cbfdp+0,
    0x1.75feb564267c9p+0, 0x1.77024b1ab6e09p+0, 0x1.780694fde5d3fp+0, 0x1.790b938ac1cf6p+0,
    0x1.7a11473eb0187p+0, 0x1.7b17b0976cfdbp+0, 0x1.7c1ed0130c132p+0, 0x1.7d26a62ff86f0p+0,
    0x1.7e2f336cf4e62p+0, 0x1.7f3878491c491p+0, 0x1.80427543e1a12p+0, 0x1.814d2add106d9p+0,
    0x1.82589994cce13p+0, 0x1.8364c1eb941f7p+0, 0x1.8471a4623c7adp+0, 0x1.857f4179f5b21p+0,
    0x1.868d99b4492edp+0, 0x1.879cad931a436p+0, 0x1.88ac7d98a6699p+0, 0x1.89bd0a478580fp+0,
    0x1.8ace5422aa0dbp+0, 0x1.8be05bad61778p+0, 0x1.8cf3216b5448cp+0, 0x1.8e06a5e0866d9p+0,
    0x1.8f1ae99157736p+0, 0x1.902fed0282c8ap+0, 0x1.9145b0b91ffc6p+0, 0x1.925c353aa2fe2p+0,
    0x1.93737b0cdc5e5p+0, 0x1.948b82b5f98e5p+0, 0x1.95a44cbc8520fp+0, 0x1.96bdd9a7670b3p+0,
    0x1.97d829fde4e50p+0, 0x1.98f33e47a22a2p+0, 0x1.9a0f170ca07bap+0, 0x1.9b2bb4d53fe0dp+0,
    0x1.9c49182a3f090p+0, 0x1.9d674194bb8d5p+0, 0x1.9e86319e32323p+0, 0x1.9fa5e8d07f29ep+0,
    0x1.a0c667b5de565p+0, 0x1.a1e7aed8eb8bbp+0, 0x1.a309bec4a2d33p+0, 0x1.a42c980460ad8p+0,
    0x1.a5503b23e255dp+0, 0x1.a674a8af46052p+0, 0x1.a799e1330b358p+0, 0x1.a8bfe53c12e59p+0,
    0x1.a9e6b5579fdbfp+0, 0x1.ab0e521356ebap+0, 0x1.ac36bbfd3f37ap+0, 0x1.ad5ff3a3c2774p+0,
    0x1.ae89f995ad3adp+0, 0x1.afb4ce622f2ffp+0, 0x1.b0e07298db666p+0, 0x1.b20ce6c9a8952p+0,
    0x1.b33a2b84f15fbp+0, 0x1.b468415b749b1p+0, 0x1.b59728de5593ap+0, 0x1.b6c6e29f1c52ap+0,
    0x1.b7f76f2fb5e47p+0, 0x1.b928cf22749e4p+0, 0x1.ba5b030a1064ap+0, 0x1.bb8e0b79a6f1fp+0,
    0x1.bcc1e904bc1d2p+0, 0x1.bdf69c3f3a207p+0, 0x1.bf2c25bd71e09p+0, 0x1.c06286141b33dp+0,
    0x1.c199bdd85529cp+0, 0x1.c2d1cd9fa652cp+0, 0x1.c40ab5fffd07ap+0, 0x1.c544778fafb22p+0,
    0x1.c67f12e57d14bp+0, 0x1.c7ba88988c933p+0, 0x1.c8f6d9406e7b5p+0, 0x1.ca3405751c4dbp+0,
    0x1.cb720dcef9069p+0, 0x1.ccb0f2e6d1675p+0, 0x1.cdf0b555dc3fap+0, 0x1.cf3155b5bab74p+0,
    0x1.d072d4a07897cp+0, 0x1.d1b532b08c968p+0, 0x1.d2f87080d89f2p+0, 0x1.d43c8eacaa1d6p+0,
    0x1.d5818dcfba487p+0, 0x1.d6c76e862e6d3p+0, 0x1.d80e316c98398p+0, 0x1.d955d71ff6075p+0,
    0x1.da9e603db3285p+0, 0x1.dbe7cd63a8315p+0, 0x1.dd321f301b460p+0, 0x1.de7d5641c0658p+0,
    0x1.dfc97337b9b5fp+0, 0x1.e11676b197d17p+0, 0x1.e264614f5a129p+0, 0x1.e3b333b16ee12p+0,
    0x1.e502ee78b3ff6p+0, 0x1.e653924676d76p+0, 0x1.e7a51fbc74c83p+0, 0x1.e8f7977cdb740p+0,
    0x1.ea4afa2a490dap+0, 0x1.eb9f4867cca6ep+0, 0x1.ecf482d8e67f1p+0, 0x1.ee4aaa2188510p+0,
    0x1.efa1bee615a27p+0, 0x1.f0f9c1cb6412ap+0, 0x1.f252b376bba97p+0, 0x1.f3ac948dd7274p+0,
    0x1.f50765b6e4540p+0, 0x1.f6632798844f8p+0, 0x1.f7bfdad9cbe14p+0, 0x1.f91d802243c89p+0,
    0x1.fa7c1819e90d8p+0, 0x1.fbdba3692d514p+0, 0x1.fd3c22b8f71f1p+0, 0x1.fe9d96b2a23d9p+0,
};

// a·b + c with c a wave-uniform value: the VOP3 v_fma_f64 takes c straight from an SGPR pair (the
// compiler otherwise picks the two-address v_fmac and first copies c into VGPRs, 2 v_mov_b32 each).
__device__ __forceinline__ double fma_vvs(double a, double b, double c) {
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
  return r;
}

constexpr double kMaternR2Max = 160000.0;   // r = 400: exp(−√5·400) = exp(−894.4) → 0
constexpr double kRbfR2Max = 2048.0;        // exp(−1024) → 0
// max(r², 0) with the same upper clamp, for the exp_nonpos paths (exp_nonpos itself saturates k
// to INT_MIN and stays 0 up to r ~ 1e18, but its polynomial overflows past that).
template <int KIND>
__device__ __forceinline__ double r2_range(double r2) {
  r2 = r2 > 0.0 ? r2 : 0.0;
  return fmin(r2, KIND == OMB_KERNEL_MATERN52 ? kMaternR2Max : kRbfR2Max);
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
  r2 = r2_range<KIND>(r2);
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
  r2a = r2_range<KIND>(r2a);
  r2b = r2_range<KIND>(r2b);
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

// Two kernel values from r² (lockstep pair), with the table-driven exp and a one-correction sqrt —
// the posterior kernel's generation step, where every fp64 VALU instruction is taken from the
// MFMA's time (FP64 VALU and MFMA share the pipe):
//   * exp(x), x ≤ 0: x = (64m + j)·ln2/64 + f with |f| ≤ ln2/128 (Cody–Waite, fdlibm's ln2 split);
//     exp(x) = 2^m · T[j] · (1 + p(f)), p the degree-5 Taylor polynomial (remainder < 3.5e-17).
//     ≤ 1 ulp against np.exp over [−740, 0]; 12 instead of 17 fp64 instructions.  `tab` = the
//     64-entry kExp2Tab64 staged in LDS.
//   * sqrt: v_rsq_f64 seed, one Goldschmidt step, one residual correction (≤ 1 ulp; the second
//     correction of sqrt_nonneg only settles round-to-nearest ties).  r² is clamped to ≥ 1e-300 in
//     place of the zero test: r = 1e-150 gives exactly σ_f², as r = 0 does.
//   * Matern polynomial from r² itself: 1 + √5 r + 5/3 r² (GPy squares r; ≤ 1 ulp apart).
// r² clamp: |r²| + r²_min (r²_min = 1e-300, an SGPR kernel argument) is one v_add_f64 with an abs
// source modifier.  It equals max(r², r²_min) except for r² < 0 (rounding of the augmented dot
// product, |r²| ~ 1e-16 where GPy clips to 0: the kernel value differs by < 1e-16 relative) and for
// 0 < r² < 1e-284 (r < 1e-142: the value is σ_f² either way).  Round 1 used an inline-asm v_max_f64
// here; the compiler's hazard recognizer does not see inside inline asm, and as the first reader of
// an FP64 MFMA result it could issue before the required wait states (found in r02 when a variant
// with more registers scheduled it straight after the r²-MFMA and returned wrong moments).
//
// Upper clamp (round 4): the table reductions round k = −√5·r·256/ln2 (or −r²/2·64/ln2) with the 1.5·2^52
// shift, which is exact only for |k| < 2^51 — r > 2.7e12 (Matern) or r² > 2.4e13 (RBF).  A degenerate
// lengthscale fit (ℓ = 2.3e-16 in a DTLZ2 run) puts r far past that and the low word of the
// shifted sum is then garbage: K entries of ±inf/NaN instead of 0.  Clamping r² at the exp underflow
// point (Matern √5·r > 894, RBF r²/2 > 1024: exp underflows to exactly 0 in double beyond either)
// returns the reference's value, 0, for every larger r².  One v_min_f64 per element.
__device__ __forceinline__ double r2_clamp(double r2, double r2min) {
  return fmin(fabs(r2) + r2min, kMaternR2Max);
}


// Round-to-nearest-even of y with |y| < 2^51, as a double and as an int, from one add: the
// 1.5·2^52 shift leaves the integer in the low word (replaces v_rndne + v_cvt_i32).
struct RoundedK {
  double k;
  int ki;
};
__device__ __forceinline__ RoundedK round_shift(double y_plus_shift) {
  return RoundedK{y_plus_shift - 6755399441055744.0, __double2loint(y_plus_shift)};
}

// pm = (σ_f², √5·σ_f², 5/3·σ_f²): the Matern polynomial with the variance folded in.
template <int KIND>
__device__ __forceinline__ void kernel_of_r2_tab_x2(double r2a, double r2b, const double (&pm)[3], const ExpCoef& ec,
                                                    const double* tab, double& outa, double& outb) {
  double xa, xb, ka_, kb_, pa_ = pm[0], pb_ = pm[0];
  if constexpr (KIND == OMB_KERNEL_MATERN52) {
    r2a = r2_clamp(r2a, ec.t[7]);
    r2b = r2_clamp(r2b, ec.t[7]);
    const double ya = __builtin_amdgcn_rsq(r2a), yb = __builtin_amdgcn_rsq(r2b);
    double ga = r2a * ya, gb = r2b * yb, ha = 0.5 * ya, hb = 0.5 * yb;
    const double qa = fma(-ga, ha, 0.5), qb = fma(-gb, hb, 0.5);
    ga = fma(ga, qa, ga);
    gb = fma(gb, qb, gb);
    ha = fma(ha, qa, ha);
    hb = fma(hb, qb, hb);
    ga = fma(fma(-ga, ga, r2a), ha, ga);
    gb = fma(fma(-gb, gb, r2b), hb, gb);
    pa_ = fma(pm[2], r2a, fma(pm[1], ga, pm[0]));
    pb_ = fma(pm[2], r2b, fma(pm[1], gb, pm[0]));
    xa = -(kSqrt5 * ga);
    xb = -(kSqrt5 * gb);
    ka_ = fma(ga, ec.t[0], 6755399441055744.0);     // −√5·r·64/ln2 + 1.5·2^52
    kb_ = fma(gb, ec.t[0], 6755399441055744.0);
  } else {
    xa = -0.5 * fmin(fabs(r2a), kRbfR2Max);       // GPy clips r² < 0 (rounding, ~1e-16) to 0
    xb = -0.5 * fmin(fabs(r2b), kRbfR2Max);
    ka_ = fma(xa, -ec.t[0] / kSqrt5, 6755399441055744.0);
    kb_ = fma(xb, -ec.t[0] / kSqrt5, 6755399441055744.0);
  }
  const RoundedK rka = round_shift(ka_), rkb = round_shift(kb_);
  const double ka = rka.k, kb = rkb.k;
  double fa = fma(-ka, ec.t[1], xa), fb = fma(-kb, ec.t[1], xb);
  fa = fma(-ka, ec.t[2], fa);
  fb = fma(-kb, ec.t[2], fb);
  double qa = fma(fa, ec.t[3], ec.t[4]), qb = fma(fb, ec.t[3], ec.t[4]);
  qa = fma_vvs(qa, fa, ec.t[5]);
  qb = fma_vvs(qb, fb, ec.t[5]);
  qa = fma_vvs(qa, fa, ec.t[6]);
  qb = fma_vvs(qb, fb, ec.t[6]);
  qa = fma(qa, fa, 1.0);
  qb = fma(qb, fb, 1.0);
  const int ia = rka.ki, ib = rkb.ki;
  const double Ta = tab[ia & 63], Tb = tab[ib & 63];
  const double ea = ldexp(fma(Ta, qa * fa, Ta), ia >> 6), eb = ldexp(fma(Tb, qb * fb, Tb), ib >> 6);
  outa = pa_ * ea;
  outb = pb_ * eb;
}

// Matern 5/2 with the 256-entry table (tab = kExp2Tab256 staged in LDS), two elements in lockstep.
// The reduction runs in r-space, so −√5 r is never formed:
//     k = rne(−√5 r · 256/ln2),  f' = r + k·c  (c = ln2/(256√5), two-constant fma Cody–Waite),
//     exp(−√5 r) = 2^(k>>8) · T[k & 255] · (1 + f'·(a1 + a2 f' + a3 f'² + a4 f'³)),  a_i = (−√5)^i/i!
// |f'| ≤ c/2, so |−√5 f'| ≤ ln2/512 and the degree-4 remainder is < 4e-17.  18 fp64 instructions
// per element + rsq instead of 21 (no −√5 r product, one polynomial degree fewer).  SHORT drops the
// residual correction of the sqrt (r from one Goldschmidt step on the v_rsq_f64 seed).
template <bool SHORT = false, bool IEXP = false>
__device__ __forceinline__ void matern_r2_tab256_x2(double r2a, double r2b, const double (&pm)[3], const ExpCoef& ec,
                                                    const double* tab, double& outa, double& outb) {
  r2a = r2_clamp(r2a, ec.t[7]);
  r2b = r2_clamp(r2b, ec.t[7]);
  const double ya = __builtin_amdgcn_rsq(r2a), yb = __builtin_amdgcn_rsq(r2b);
  double ga = r2a * ya, gb = r2b * yb, ha = 0.5 * ya, hb = 0.5 * yb;
  const double qa = fma(-ga, ha, 0.5), qb = fma(-gb, hb, 0.5);
  ga = fma(ga, qa, ga);
  gb = fma(gb, qb, gb);
  if constexpr (!SHORT) {
    ha = fma(ha, qa, ha);
    hb = fma(hb, qb, hb);
    ga = fma(fma(-ga, ga, r2a), ha, ga);
    gb = fma(fma(-gb, gb, r2b), hb, gb);
  }
  const double pa_ = fma(pm[2], r2a, fma(pm[1], ga, pm[0]));
  const double pb_ = fma(pm[2], r2b, fma(pm[1], gb, pm[0]));
  const RoundedK rka = round_shift(fma(ga, ec.u[0], 6755399441055744.0));
  const RoundedK rkb = round_shift(fma(gb, ec.u[0], 6755399441055744.0));
  double fa = fma(rka.k, ec.u[1], ga), fb = fma(rkb.k, ec.u[1], gb);
  fa = fma(rka.k, ec.u[2], fa);
  fb = fma(rkb.k, ec.u[2], fb);
  double sa = fma(fa, ec.u[3], ec.u[4]), sb = fma(fb, ec.u[3], ec.u[4]);
  sa = fma_vvs(sa, fa, ec.u[5]);
  sb = fma_vvs(sb, fb, ec.u[5]);
  sa = fma_vvs(sa, fa, ec.u[6]);
  sb = fma_vvs(sb, fb, ec.u[6]);
  const int ia = rka.ki, ib = rkb.ki;
  const double Ta = tab[ia & 255], Tb = tab[ib & 255];
  if constexpr (IEXP) {
    // 2^(k>>8) applied as an integer add to the high word (integer VALU instead of v_ldexp_f64); the
    // scale is clamped at 2^-1021 so the result stays normal (K* < 1e-300·σ_f² there instead of 0)
    const double xa = fma(Ta, sa * fa, Ta), xb = fma(Tb, sb * fb, Tb);
    const int ma = max(ia >> 8, -1021), mb = max(ib >> 8, -1021);
    const double ea = __hiloint2double(__double2hiint(xa) + (ma << 20), __double2loint(xa));
    const double eb = __hiloint2double(__double2hiint(xb) + (mb << 20), __double2loint(xb));
    outa = pa_ * ea;
    outb = pb_ * eb;
  } else {
    const double ea = ldexp(fma(Ta, sa * fa, Ta), ia >> 8), eb = ldexp(fma(Tb, sb * fb, Tb), ib >> 8);
    outa = pa_ * ea;
    outb = pb_ * eb;
  }
}

// φ for EHVI-2D's stripes: exp_nonpos (≤ 1 ulp, 17 instead of 22 fp64 instructions) times 1/√(2π) instead of the
// division (≈ 10 instructions), so within 2 ulp of npdf; −t²/2 below −746 (t = ±inf from a zero σ) is clamped
// there, where exp is 0 either way, and NaN stays NaN.
constexpr double kInvSqrt2Pi = 0.3989422804014327;      // 1/√(2π) rounded
// Φ for EHVI-2D's stripes: 0.5·erfc(−a/√2) on every range (cephes' ndtr switches to 0.5 + 0.5·erf inside
// |a| < 1, and lanes on both sides of the switch run both paths); within a few ulp of ndtr.
__device__ __forceinline__ double ndtr_fast(double a) {
#pragma clang fp contract(off)
  return 0.5 * erfc(-(a * kSqrt1_2));
}
__device__ __forceinline__ double npdf_fast(double t) {
#pragma clang fp contract(off)
  double x = -(t * t) * 0.5;
  x = x < -746.0 ? -746.0 : x;
  return exp_nonpos(x) * kInvSqrt2Pi;
}

// EHVI-2D of one candidate over L lanes (L = 1, 2, 4): util_functions.py:81-128 (EHVI_2D_aux) with the stripe
// array S = [(r0,−∞), PF↑f2, (−∞,r1)] of :93-109; y1[0] = r0, y1[i] / y2[i−1] = stripe i's f1 / f2 (i = 1..P).
// The stripes 1..P form four contiguous quarters; lane g (0..L−1; the candidate's lanes are l, l + 64/L, … of one
// wave) sums quarter g (L = 4), quarters 2g and 2g + 1 (L = 2) or all four (L = 1); within a quarter φ/Φ of t_i = (y1[i]−μ0)/σA are reused by stripe i+1 (the
// reference evaluates ψ(y1[i−1], y1[i−1]) from the same t), so a stripe costs 2 Φ + 2 φ instead of 7 calls, and a
// quarter one Φ + φ more for its first t.  The quarters' partial sums meet in one fixed order for every L: every lane
// of the candidate returns the same value, identical in every kernel that calls this (ehvi2d_kernel and the one-launch
// chains) and at every batch size, which is what makes their arg-max bitwise the same.  One lane per candidate sums
// the four quarters serially (4× the latency, but no lane idles on a short last quarter): the kernels take L = 1 for
// batches large enough to fill every SIMD with waves (ehvi2d_lanes).
template <int L>
__device__ __forceinline__ double ehvi2d_point(double m0, double m1, double v0, double v1, const double* y1,
                                               const double* y2, int P, double r1, double s00, double s01, int mode,
                                               int g) {
#pragma clang fp contract(off)
  double sA, sB;
  bool nan = false;
  if (mode == OMB_EHVI_REFERENCE) {
    // change() scales the cached samples by sqrt(σ²0) (util_functions.py:233-235): a negative variance makes
    // every sample NaN, and np.cov of them NaN.
    nan = !(v0 >= 0.0);
    sA = v0 * s00;   // c00 = σ²0·Cov(cache)00   (util_functions.py:163-167, 114-115)
    sB = v0 * s01;   // c01 = σ²0·Cov(cache)01   (a covariance used as a std: quirk 2)
  } else if (mode == OMB_EHVI_TEXTBOOK) {
    sA = sqrt(v0);
    sB = sqrt(v1);
  } else {   // OMB_EHVI_SIGMA: EHVI_2D_aux called with σ directly
    sA = v0;
    sB = v1;
  }
  // The stripes are always summed as four fixed quarters (chunk = ⌈P/4⌉), each from 0 with its own first t, and
  // the quarters meet as ((q0 + q1) + (q2 + q3)) whatever L is: L only decides which lane sums which quarters (L = 4:
  // one each, met by two xor-shuffles; L = 2: two each, then one shuffle; L = 1: all four).  So a candidate's value
  // does not depend on the batch size its lane count came from (polish compared a 4-lane single-point
  // score against 1- or 2-lane batch values).
  const int chunk = (P + 3) / 4;
  double iA = 0.0, iB = 0.0;
  if (!nan) {
    // (b − m)/s as (b − m)·(1/s): one division per candidate instead of two per stripe (≤ 1 ulp in t; x/0 and
    // x·(1/0) agree, ±inf or NaN)
    iA = 1.0 / sA;
    iB = 1.0 / sB;
  }
  auto quarter = [&](int q, double& s1, double& s2) {
    const int i0 = 1 + q * chunk, i1 = min(P, (q + 1) * chunk);
    s1 = 0.0;
    s2 = 0.0;
    if (nan || i0 > i1) return;
    const double tp = (y1[i0 - 1] - m0) * iA;
    double cdf_p = ndtr_fast(tp), pdf_p = npdf_fast(tp);
    for (int i = i0; i <= i1; ++i) {
      const double y1p = y1[i - 1], y1i = y1[i], y2i = y2[i - 1];
      const double t = (y1i - m0) * iA;
      const double cdf_t = ndtr_fast(t), pdf_t = npdf_fast(t);
      const double u = (y2i - m1) * iB;
      const double p2 = sB * npdf_fast(u) + (y2i - m1) * ndtr_fast(u);     // ψ(y2i, y2i, μ1, σB)
      s1 = s1 + (y1p - y1i) * cdf_t * p2;
      const double psi_pp = sA * pdf_p + (y1p - m0) * cdf_p;          // ψ(y1[i−1], y1[i−1], μ0, σA)
      const double psi_pi = sA * pdf_t + (y1p - m0) * cdf_t;          // ψ(y1[i−1], y1[i],   μ0, σA)
      s2 = s2 + (psi_pp - psi_pi) * p2;
      cdf_p = cdf_t;
      pdf_p = pdf_t;
    }
  };
  double sum1, sum2;
  if constexpr (L == 4) {
    quarter(g, sum1, sum2);
    sum1 += __shfl_xor(sum1, 16);
    sum1 += __shfl_xor(sum1, 32);
    sum2 += __shfl_xor(sum2, 16);
    sum2 += __shfl_xor(sum2, 32);
  } else if constexpr (L == 2) {
    double a1, a2, b1, b2;
    quarter(2 * g, a1, a2);
    quarter(2 * g + 1, b1, b2);
    sum1 = a1 + b1;
    sum2 = a2 + b2;
    sum1 += __shfl_xor(sum1, 32);
    sum2 += __shfl_xor(sum2, 32);
  } else {
    double q1[4], q2[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) quarter(q, q1[q], q2[q]);
    sum1 = (q1[0] + q1[1]) + (q1[2] + q1[3]);
    sum2 = (q2[0] + q2[1]) + (q2[2] + q2[3]);
  }
  if (nan) return __builtin_nan("");
  double res = sum1 + sum2;
  if (mode == OMB_EHVI_TEXTBOOK) {
    // the stripe i = P+1 that range(1, n+1) leaves out (quirk 3): ψ(y1P,y1P,μ0,σA)·ψ(r1,r1,μ1,σB)
    const double tP = (y1[P] - m0) / sA;
    const double psiA = sA * npdf_fast(tP) + (y1[P] - m0) * ndtr_fast(tP);
    const double u = (r1 - m1) / sB;
    res += psiA * (sB * npdf_fast(u) + (r1 - m1) * ndtr_fast(u));
  }
  return res;
}

// Agent-scope relaxed f64 store / load (coherent across the XCDs' L2s): the fused chains' per-workgroup pairs.
__device__ __forceinline__ void wf_store_f64(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), __builtin_bit_cast(unsigned long long, v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double wf_load_f64(const double* p) {
  return __builtin_bit_cast(double, __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT));
}

// Arg-max pair of the one-launch chains: higher value wins, the lower index on ties; index < 0 = none (NaN and −∞
// never enter).  The same rule as omb_argmax.hip's `better`.
__device__ __forceinline__ bool argmax_better(double av, long long ai, double bv, long long bi) {
  if (ai < 0) return false;
  if (bi < 0) return true;
  return (av > bv) || (av == bv && ai < bi);
}

// (v, i) of the whole workgroup into thread 0 (shuffles per wave, then wave 0's pairs from LDS in wave order);
// red_v / red_i: one slot per wave.  Ends with a barrier passed by every thread.
__device__ __forceinline__ void argmax_wave_block(double& v, long long& i, double* red_v, long long* red_i) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double ov = __shfl_xor(v, off);
    const long long oi = __shfl_xor(i, off);
    if (argmax_better(ov, oi, v, i)) {
      v = ov;
      i = oi;
    }
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red_v[wave] = v;
    red_i[wave] = i;
  }
  __syncthreads();
  if (threadIdx.x == 0)
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w)
      if (argmax_better(red_v[w], red_i[w], v, i)) {
        v = red_v[w];
        i = red_i[w];
      }
}

// GPy Matern52.K_of_r: variance*(1+sqrt(5)*r+5/3*r**2)*exp(-sqrt(5)*r)  (r ≥ 0)
// GPy RBF.K_of_r     : variance*exp(-r**2/2)
// FAST selects exp_nonpos / sqrt_nonneg (default) or the libm functions (ablation reference).
template <int KIND, bool FAST = true>
__device__ __forceinline__ double kernel_of_r2(double r2, double variance) {
  r2 = r2_range<KIND>(r2);                  // np.clip(r2, 0, inf); above the clamp K = 0 either way
  const double r = FAST ? sqrt_nonneg(r2) : sqrt(r2);
  if constexpr (KIND == OMB_KERNEL_MATERN52) {
    const double poly = (1.0 + kSqrt5 * r) + kFiveThirds * (r * r);
    return (variance * poly) * (FAST ? exp_nonpos(-(kSqrt5 * r)) : exp(-(kSqrt5 * r)));
  } else {
    return variance * (FAST ? exp_nonpos(-0.5 * (r * r)) : exp(-0.5 * (r * r)));
  }
}

}  // namespace omb
