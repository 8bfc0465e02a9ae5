// ParEGO / KEEP evolutionary acquisition search on the device.
//
// The reference maximises its acquisition with a steady-state GA (ParEGO.solve parego.py:223-271,
// KEEP.solve keep.py:240-292): 20 individuals, 1,000 generations, each generation = best-of-population
// tracking, two binary tournaments without replacement (parego.py:78-111), simulated binary crossover
// (p = 0.2, η = 2, one child; :58-75) and per-gene ×1.05 / ×0.95 mutation (p = 1/d; :37-56); the child
// replaces the first parent unless the parent is strictly fitter.  Fitness: EI with σ = sqrt(σ² + 1e-6)
// (parego.py:126-145) or μ_pareto · EI (keep.py:142-151).  ~26,000 single-point GP predictions per
// search in the reference.
//
// No random draw of the search depends on a fitness value, so the host replays the draws into a tape
// (optimobo_amd/ea.py: tournament samples, crossover flag and β, mutation codes) and one 256-thread
// workgroup runs all generations: the population and its fitness stay in LDS (the reference recomputes
// the same fitness every generation), and each generation evaluates one child — its K* row on all
// threads, L⁻¹k* with a thread per row (L⁻¹ packed in LDS for n ≤ 128, else a transposed global copy
// read column-wise), μ and ‖L⁻¹k*‖² by fixed-order reductions (wave shuffles, then the 4 waves).
// Child arithmetic uses unfused IEEE ops in numpy's order, so with
// the same tape the device search makes the reference's choices.
#include "omb_internal.h"
#include "omb_math.h"

namespace omb {

constexpr int kEAThreads = 256;

struct EAArgs {
  GPDev g0, g1;          // the scalarised (EI) model, and KEEP's Pareto-membership model (mode 1)
  const double* LdT;     // (n0, n0): L0⁻¹ transposed, LdT[j·n + i] = L⁻¹[i][j] (j ≤ i)
  int mode;              // 0: EI (ParEGO), 1: μ1 · EI (KEEP)
  int d, P, iters;
  double best, var_eps;
  const double* pop;     // (P, d) initial population
  const int* sel;        // (iters, 4)
  const int8_t* cross;   // (iters)
  const double* beta;    // (iters, d)
  const int8_t* mut;     // (iters, d)
  const double* lower;   // (d)
  const double* upper;   // (d)
  double* out;           // (d + 1): best x, best fitness
};

// μ and (with L) σ² of one point x (LDS, d values) under model g; every thread returns the result.
// L⁻¹k* with a thread per row: Lds (n ≤ kEALdsN) is the packed lower L⁻¹ by columns in LDS — element
// (i, j) at j·n − j(j−1)/2 + (i − j), consecutive rows at consecutive addresses; otherwise LdT (global,
// transposed) is read over each row's columns, two accumulators.
template <int DP>
__device__ double ea_moments(const GPDev& g, const double* __restrict__ LdT, const double* Lds, int d,
                             const double* x, double* ab, double* kst, double* red, double* var_out) {
  const int tid = threadIdx.x;
  if (tid < DP) ab[tid] = (tid < d) ? x[tid] / g.ls[tid] : 0.0;     // GPy divides by ℓ
  __syncthreads();
  double asq = 0.0;
  for (int j = 0; j < d; ++j) asq += ab[j] * ab[j];
  double mp = 0.0;
  for (int i = tid; i < g.n; i += kEAThreads) {
    const double* xr = g.Xs + (int64_t)i * DP;
    double dot = 0.0;
    if constexpr (DP <= kMaxFusedDP) {
#pragma unroll
      for (int j = 0; j < DP; ++j) dot = fma(xr[j], ab[j], dot);
    } else {   // wide inputs: unrolled, the row's loads would take every register (392 spilled at DP = 256)
#pragma unroll 8
      for (int j = 0; j < DP; ++j) dot = fma(xr[j], ab[j], dot);
    }
    const double r2 = fma(-2.0, dot, g.xsq[i] + asq);              // −2a·b + (‖a‖² + ‖b‖²)
    const double k = (g.kind == OMB_KERNEL_RBF) ? kernel_of_r2<OMB_KERNEL_RBF>(r2, g.variance)
                                                : kernel_of_r2<OMB_KERNEL_MATERN52>(r2, g.variance);
    kst[i] = k;
    mp = fma(g.alpha[i], k, mp);
  }
  __syncthreads();
  double vp = 0.0;
  const int n = g.n;
  if (Lds) {
    for (int i = tid; i < n; i += kEAThreads) {
      double v0 = 0.0, v1 = 0.0;
      int addr = i;                                                  // column 0, row i
      int j = 0;
      for (; j + 1 <= i; j += 2) {
        v0 = fma(Lds[addr], kst[j], v0);
        addr += n - j - 1;
        v1 = fma(Lds[addr], kst[j + 1], v1);
        addr += n - j - 2;
      }
      if (j <= i) v0 = fma(Lds[addr], kst[j], v0);
      const double v = v0 + v1;
      vp = fma(v, v, vp);
    }
  } else if (LdT) {
    for (int i = tid; i < n; i += kEAThreads) {
      double v0 = 0.0, v1 = 0.0;
      int j = 0;
      for (; j + 1 <= i; j += 2) {
        v0 = fma(LdT[(int64_t)j * n + i], kst[j], v0);
        v1 = fma(LdT[(int64_t)(j + 1) * n + i], kst[j + 1], v1);
      }
      if (j <= i) v0 = fma(LdT[(int64_t)j * n + i], kst[j], v0);
      const double v = v0 + v1;
      vp = fma(v, v, vp);
    }
  }
  // fixed-order reduction: within each wave by xor shuffles, then the 4 waves in order
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    mp += __shfl_xor(mp, off);
    vp += __shfl_xor(vp, off);
  }
  if ((tid & 63) == 0) {
    red[tid >> 6] = mp;
    red[4 + (tid >> 6)] = vp;
  }
  __syncthreads();
  if (tid == 0) {
    red[2 * kEAThreads] = (red[0] + red[1]) + (red[2] + red[3]);
    red[2 * kEAThreads + 1] = g.variance - ((red[4] + red[5]) + (red[6] + red[7]));
  }
  __syncthreads();
  const double mu = red[2 * kEAThreads];
  if (var_out) *var_out = red[2 * kEAThreads + 1];
  __syncthreads();                                                  // red, ab, kst free again
  return mu;
}

template <int DP>
__device__ double ea_fitness(const EAArgs& A, const double* Lds, const double* x, double* ab, double* kst,
                             double* red) {
  double var0;
  const double mu0 = ea_moments<DP>(A.g0, A.LdT, Lds, A.d, x, ab, kst, red, &var0);
  const double sigma = sqrt(var0 + A.var_eps);
  const double gamma = (A.best - mu0) / (sigma + 1e-10);
  double v = sigma * (gamma * ndtr(gamma) + npdf(gamma));
  if (A.mode == 1) v = ea_moments<DP>(A.g1, nullptr, nullptr, A.d, x, ab, kst, red, nullptr) * v;
  return v;
}

template <int DP>
__global__ __launch_bounds__(kEAThreads) void ea_search_kernel(EAArgs A) {
  __shared__ double pop[kEAMaxPop * DP];
  __shared__ double F[kEAMaxPop];
  __shared__ double child[DP];
  __shared__ double ab[DP];
  __shared__ double kst[kEAMaxTrain];
  __shared__ double red[2 * kEAThreads + 2];
  __shared__ int ctl[4];                                            // w1, w2, best row (−1: none yet)
  __shared__ double lds_l[kEALdsN * (kEALdsN + 1) / 2];             // packed L0⁻¹ (n0 ≤ kEALdsN)
  const int tid = threadIdx.x, d = A.d, P = A.P;
  const int n0 = A.g0.n;
  const double* Lds = nullptr;
  if (n0 <= kEALdsN) {
    for (int j = 0, off = 0; j < n0; off += n0 - j, ++j)
      for (int i = j + tid; i < n0; i += kEAThreads) lds_l[off + i - j] = A.LdT[(int64_t)j * n0 + i];
    Lds = lds_l;
  }
  for (int i = tid; i < P * DP; i += kEAThreads) {
    const int p = i / DP, j = i % DP;
    pop[i] = (j < d) ? A.pop[p * d + j] : 0.0;
  }
  if (tid == 0) ctl[2] = -1;                                        // best_solution_found = self.lower
  __syncthreads();
  for (int p = 0; p < P; ++p) {
    const double f = ea_fitness<DP>(A, Lds, pop + p * DP, ab, kst, red);
    if (tid == 0) F[p] = f;
  }
  double best_f = 0.0;                                              // best_EI = 0 (thread 0's copy)
  __syncthreads();
  for (int it = 0; it < A.iters; ++it) {
    if (tid == 0) {
      // best of the population before this generation: np.max (NaN if any fitness is NaN, and then
      // no update) and np.argmax (the first maximum).  The reference keeps a view of that row
      // (parego.py:248-251, keep.py:268-271), so only its index is recorded here: a later replacement
      // of the row changes the proposal, as it does in the reference.
      int bi = 0;
      bool nan = F[0] != F[0];
      for (int p = 1; p < P; ++p) {
        nan |= F[p] != F[p];
        if (F[p] > F[bi]) bi = p;
      }
      if (!nan && F[bi] > best_f) {
        best_f = F[bi];
        ctl[2] = bi;
      }
      const int* s = A.sel + 4 * it;
      const int w1 = F[s[0]] > F[s[1]] ? s[0] : s[1];              // tournament 1 (whole population)
      const int a = s[2] < w1 ? s[2] : s[2] + 1, b = s[3] < w1 ? s[3] : s[3] + 1;   // without w1
      ctl[0] = w1;
      ctl[1] = F[a] > F[b] ? a : b;
    }
    __syncthreads();
    const int w1 = ctl[0], w2 = ctl[1];
    if (tid < d) {
#pragma clang fp contract(off)   // numpy rounds every product and sum: no fma contraction here
      const double p1 = pop[w1 * DP + tid], p2 = pop[w2 * DP + tid];
      const double lo = A.lower[tid], hi = A.upper[tid];
      double c = p1;
      if (A.cross[it]) {
        // 0.5 * ((1 + β) * p1 + (1 − β) * p2), numpy's order, no contraction
        const double bt = A.beta[(int64_t)it * d + tid];
        c = 0.5 * ((1.0 + bt) * p1 + (1.0 - bt) * p2);
        c = fmin(fmax(c, lo), hi);
      }
      const int8_t m = A.mut[(int64_t)it * d + tid];
      if (m == 1) c = c * 1.05;
      if (m == 2) c = c * 0.95;
      child[tid] = fmin(fmax(c, lo), hi);
    } else if (tid < DP) {
      child[tid] = 0.0;
    }
    __syncthreads();
    const double fc = ea_fitness<DP>(A, Lds, child, ab, kst, red);
    if (!(F[w1] > fc)) {                                            // the parent stays only if strictly fitter
      if (tid < DP) pop[w1 * DP + tid] = child[tid];
      if (tid == 0) F[w1] = fc;
    }
    __syncthreads();
  }
  const int br = ctl[2];
  if (tid < d) A.out[tid] = (br >= 0) ? pop[br * DP + tid] : A.lower[tid];
  if (tid == 0) A.out[d] = best_f;
}

// LdT[j·n + i] = Ld[i·n + j] for j ≤ i, 0 above the diagonal (32×32 tiles through LDS).
__global__ __launch_bounds__(256) void lower_transpose_kernel(const double* __restrict__ Ld, int64_t n,
                                                              double* __restrict__ LdT) {
  __shared__ double t[32][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int64_t r0 = (int64_t)blockIdx.y * 32, c0 = (int64_t)blockIdx.x * 32;   // source tile rows r0.., cols c0..
  for (int r = ty; r < 32; r += 8)
    if (r0 + r < n && c0 + tx < n) t[r][tx] = (c0 + tx <= r0 + r) ? Ld[(r0 + r) * n + c0 + tx] : 0.0;
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int64_t j = c0 + r, i = r0 + tx;                          // destination row j (= source column)
    if (j < n && i < n) LdT[j * n + i] = t[tx][r];
  }
}

hipError_t launch_ea_search(hipStream_t stream, const EASearch& s, double* ldt_ws) {
  const int64_t n = s.g0.n;
  const unsigned nt = (unsigned)((n + 31) / 32);
  hipLaunchKernelGGL(lower_transpose_kernel, dim3(nt, nt), dim3(256), 0, stream, s.Ld0, n, ldt_ws);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  EAArgs A{s.g0, s.g1, ldt_ws, s.mode, s.d, s.P, s.iters, s.best, s.var_eps, s.pop, s.sel, s.cross, s.beta, s.mut,
           s.lower, s.upper, s.out};
#define OMB_EA(DPV)                                                                                  \
  case DPV:                                                                                          \
    hipLaunchKernelGGL((ea_search_kernel<DPV>), dim3(1), dim3(kEAThreads), 0, stream, A);            \
    break;
  switch (s.DP) {
    OMB_EA(2) OMB_EA(4) OMB_EA(6) OMB_EA(8) OMB_EA(16) OMB_EA(32) OMB_EA(64) OMB_EA(128) OMB_EA(256)
    default: return hipErrorInvalidValue;
  }
#undef OMB_EA
  return hipGetLastError();
}

}  // namespace omb
