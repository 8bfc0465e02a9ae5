// Acquisition kernels on gfx950: EHVI-2D, EHVI-3D (reference Monte-Carlo form), HV-PoI,
// expected decomposition over the twelve scalarisations, and EI.
//
// Each kernel evaluates one candidate per thread from the posterior moments produced by
// omb_posterior; the per-iteration constant geometry (Pareto stripes, cells, the cached
// normal samples) is staged once per workgroup in LDS and read as a broadcast.  All fp64.
#include <math.h>

#include "omb_internal.h"
#include "omb_math.h"

namespace omb {

constexpr int kAcqThreads = 256;

static unsigned acq_grid(int64_t N) {
  int64_t b = (N + kAcqThreads - 1) / kAcqThreads;
  if (b > 65536) b = 65536;
  return (unsigned)(b < 1 ? 1 : b);
}

// ------------------------------------------------------------------------------ EHVI 2-D
// L lanes per candidate (ehvi2d_point<L>, omb_math.h — shared with the one-launch chain, so both give bitwise the
// same values and the same arg-max): wave w of a workgroup takes 64/L candidates, lane group g = lane / (64/L) an
// L-th of their stripes.  L by batch size (ehvi2d_lanes): more lanes per candidate only while the batch leaves SIMDs
// short of waves (config 3's 2^20: one lane, EHVI 197 → 135 µs; config 2's 2^16: two lanes, 15.6 → 14.0 µs).
int ehvi2d_lanes(int64_t N) { return N >= (1 << 19) ? 1 : (N >= (1 << 16) ? 2 : 4); }

template <int L>
__global__ __launch_bounds__(kAcqThreads) void ehvi2d_kernel(const double* __restrict__ mu,
                                                             const double* __restrict__ var, int64_t ld, int64_t N,
                                                             const double* __restrict__ pf, int P, double r0,
                                                             double r1, double s00, double s01, int mode,
                                                             double* __restrict__ out) {
  extern __shared__ double sm[];
  double* y1 = sm;          // y1[0..P]
  double* y2 = sm + P + 1;  // y2[1..P] stored at y2[i-1]
  for (int i = threadIdx.x; i < P; i += blockDim.x) {
    y1[i + 1] = pf[2 * i];
    y2[i] = pf[2 * i + 1];
  }
  if (threadIdx.x == 0) y1[0] = r0;
  __syncthreads();
  constexpr int CPW = 64 / L;                            // candidates per wave
  const int lane = threadIdx.x & 63, g = lane / CPW;
  const int64_t per_block = kAcqThreads / L;
  for (int64_t base = (int64_t)blockIdx.x * per_block; base < N; base += (int64_t)gridDim.x * per_block) {
    const int64_t c = base + CPW * (threadIdx.x >> 6) + (lane % CPW);
    const int64_t cc = c < N ? c : N - 1;                // every lane of the wave takes part in the shuffles
    const double v = ehvi2d_point<L>(mu[cc], mu[ld + cc], var[cc], mode == OMB_EHVI_REFERENCE ? 0.0 : var[ld + cc],
                                     y1, y2, P, r1, s00, s01, mode, g);
    if (g == 0 && c < N) out[c] = v;
  }
}

hipError_t launch_ehvi2d(hipStream_t stream, const double* mu, const double* var, int64_t ld, int64_t N,
                         const double* pf, int P, double r0, double r1, double s00, double s01, int mode,
                         double* out) {
  size_t shm = sizeof(double) * (2 * P + 1);
  const int L = ehvi2d_lanes(N);
  if (L == 4)
    hipLaunchKernelGGL(ehvi2d_kernel<4>, dim3(acq_grid(4 * N)), dim3(kAcqThreads), shm, stream, mu, var, ld, N, pf, P,
                       r0, r1, s00, s01, mode, out);
  else if (L == 2)
    hipLaunchKernelGGL(ehvi2d_kernel<2>, dim3(acq_grid(2 * N)), dim3(kAcqThreads), shm, stream, mu, var, ld, N, pf, P,
                       r0, r1, s00, s01, mode, out);
  else
    hipLaunchKernelGGL(ehvi2d_kernel<1>, dim3(acq_grid(N)), dim3(kAcqThreads), shm, stream, mu, var, ld, N, pf, P, r0,
                       r1, s00, s01, mode, out);
  return hipGetLastError();
}

// EHVI-2D with the arg-max (omb_eval_argmax[_sobol] with an EHVI-2D plan): the values of ehvi2d_kernel, bit for bit,
// are reduced in the same launch — per wave by shuffles, per workgroup in LDS, per grid by the last workgroup to
// take the ticket — by the rule of argmax_pass1/2 (higher value, lower index; NaN and −∞ never win).  Two launches
// (the arg-max's) and the values' round trip through HBM leave the chain.  With am.ticket == nullptr the launch
// stops at the per-workgroup pairs (argmax_pass1's output) and argmax_pass2 reduces them: the ticket's
// same-address agent-scope atomics serialise (≈ 10 ns each, 1024 of them at config 2: 23.3 µs for the one launch
// against 13.5 µs for the EHVI alone, rocprofv3, gpurun_out/r04_ac).  The grid is at most kArgmaxMaxBlocks
// workgroups (grid-stride), so the pairs fit the context's arg-max buffer.
template <int L>
__global__ __launch_bounds__(kAcqThreads) void ehvi2d_argmax_kernel(const double* __restrict__ mu,
                                                                    const double* __restrict__ var, int64_t ld,
                                                                    int64_t N, const double* __restrict__ pf, int P,
                                                                    double r0, double r1, double s00, double s01,
                                                                    int mode, ArgmaxOut am) {
  extern __shared__ double sm[];
  double* y1 = sm;
  double* y2 = sm + P + 1;
  __shared__ double red_v[kAcqThreads / 64];
  __shared__ long long red_i[kAcqThreads / 64];
  __shared__ int is_last;
  for (int i = threadIdx.x; i < P; i += blockDim.x) {
    y1[i + 1] = pf[2 * i];
    y2[i] = pf[2 * i + 1];
  }
  if (threadIdx.x == 0) y1[0] = r0;
  __syncthreads();
  constexpr int CPW = 64 / L;
  const int lane = threadIdx.x & 63, g = lane / CPW, wave = threadIdx.x >> 6;
  const int64_t per_block = kAcqThreads / L;
  double bv = -__builtin_inf();
  long long bi = -1;
  for (int64_t base = (int64_t)blockIdx.x * per_block; base < N; base += (int64_t)gridDim.x * per_block) {
    const int64_t c = base + CPW * wave + (lane % CPW);
    const int64_t cc = c < N ? c : N - 1;
    const double v = ehvi2d_point<L>(mu[cc], mu[ld + cc], var[cc], mode == OMB_EHVI_REFERENCE ? 0.0 : var[ld + cc],
                                     y1, y2, P, r1, s00, s01, mode, g);
    if (g == 0 && c < N && v == v && v > -__builtin_inf() && argmax_better(v, c, bv, bi)) {
      bv = v;
      bi = c;
    }
  }
  argmax_wave_block(bv, bi, red_v, red_i);          // thread 0: the workgroup's pair
  if (!am.ticket) {                                  // kernel argument: uniform
    if (threadIdx.x == 0) {
      am.partials[2 * blockIdx.x] = bv;
      am.partials[2 * blockIdx.x + 1] = __builtin_bit_cast(double, bi);
    }
    return;
  }
  if (threadIdx.x == 0) {
    // the pair as agent-scope (sc1) stores, complete (vmcnt 0) before the ticket: the ordering the Cholesky's W
    // hand-off uses (chol_publish_w).  An acquire-release ticket made every workgroup write back its XCD's L2
    // (config 2: 31 µs for the one launch against 20 + 9 µs for the separate EHVI and arg-max launches).
    wf_store_f64(&am.partials[2 * blockIdx.x], bv);
    wf_store_f64(&am.partials[2 * blockIdx.x + 1], __builtin_bit_cast(double, bi));
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned prev = __hip_atomic_fetch_add(am.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    is_last = prev == gridDim.x - 1;
  }
  __syncthreads();
  if (!__builtin_amdgcn_readfirstlane(is_last)) return;   // uniform: the reduction below has barriers
  double v = -__builtin_inf();
  long long i = -1;
  for (int b = threadIdx.x; b < (int)gridDim.x; b += blockDim.x) {
    const double pv = wf_load_f64(&am.partials[2 * b]);
    const long long pi = __builtin_bit_cast(long long, wf_load_f64(&am.partials[2 * b + 1]));
    if (argmax_better(pv, pi, v, i)) {
      v = pv;
      i = pi;
    }
  }
  __syncthreads();                                   // red_v / red_i reused
  argmax_wave_block(v, i, red_v, red_i);
  if (threadIdx.x == 0) {
    am.result[0] = i < 0 ? -__builtin_inf() : v;
    am.result[1] = i < 0 ? -1.0 : (double)(i + am.offset);
    __hip_atomic_store(am.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

int64_t ehvi2d_argmax_blocks(int64_t N) {
  const int64_t b = acq_grid(ehvi2d_lanes(N) * N);
  return b < kArgmaxMaxBlocks ? b : kArgmaxMaxBlocks;
}

hipError_t launch_ehvi2d_argmax(hipStream_t stream, const double* mu, const double* var, int64_t ld, int64_t N,
                                const double* pf, int P, double r0, double r1, double s00, double s01, int mode,
                                const ArgmaxOut& am) {
  size_t shm = sizeof(double) * (2 * P + 1);
  const int64_t nb = ehvi2d_argmax_blocks(N);
  const int L = ehvi2d_lanes(N);
  if (L == 4)
    hipLaunchKernelGGL(ehvi2d_argmax_kernel<4>, dim3((unsigned)nb), dim3(kAcqThreads), shm, stream, mu, var, ld, N, pf,
                       P, r0, r1, s00, s01, mode, am);
  else if (L == 2)
    hipLaunchKernelGGL(ehvi2d_argmax_kernel<2>, dim3((unsigned)nb), dim3(kAcqThreads), shm, stream, mu, var, ld, N, pf,
                       P, r0, r1, s00, s01, mode, am);
  else
    hipLaunchKernelGGL(ehvi2d_argmax_kernel<1>, dim3((unsigned)nb), dim3(kAcqThreads), shm, stream, mu, var, ld, N, pf,
                       P, r0, r1, s00, s01, mode, am);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || am.ticket) return e;
  return launch_argmax_reduce(stream, am.partials, (int)nb, am.offset, am.result);
}

// ------------------------------------------------------------------------------ EHVI, Monte-Carlo (k objectives)
// util_functions.py:170-214 (EHVI_3D, which the reference calls for every n_obj != 2, optimisers.py:245-248):
// samples s = cache·sqrt(σ²0) + μ (change, :217-237), then mean_s max(0, HV({s}) − HV(PF)) with HV({s}) =
// pygmo's hypervolume([s]).compute(r) = Π_{j<K}(r_j − s_j), multiplied left to right (:205-206; the 3-term
// product of :204 is dead code).  pygmo raises ValueError when a sample is not inside the reference box (some
// s_j > r_j, or s == r): flagged per candidate, value NaN.  One thread per candidate, the (M, K) cache in LDS
// read as a broadcast; μ_j and r_j in registers (K is a template parameter, so nothing spills to scratch).
struct RefPoint {
  double r[OMB_MAX_OBJ];
};

template <int K>
__global__ __launch_bounds__(kAcqThreads) void ehvi_mc_kernel(const double* __restrict__ mu,
                                                              const double* __restrict__ var, int64_t ld, int64_t N,
                                                              const double* __restrict__ cache, int M, RefPoint rp,
                                                              double hv_pf, double* __restrict__ out,
                                                              int32_t* __restrict__ raised) {
  extern __shared__ double sm[];
  for (int i = threadIdx.x; i < K * M; i += blockDim.x) sm[i] = cache[i];
  __syncthreads();
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < N; c += (int64_t)gridDim.x * blockDim.x) {
    double m[K];
#pragma unroll
    for (int j = 0; j < K; ++j) m[j] = mu[j * ld + c];
    const double sd = sqrt(var[c]);   // σ²0 for every objective (quirk 1)
    double answer = 0.0;
    bool bad = !(sd == sd);
    for (int s = 0; s < M; ++s) {
      double x[K];
#pragma unroll
      for (int j = 0; j < K; ++j) x[j] = sm[K * s + j] * sd + m[j];
      bool out_of_box = false, at_r = true;
      double vol = rp.r[0] - x[0];
#pragma unroll
      for (int j = 0; j < K; ++j) {
        out_of_box |= x[j] > rp.r[j];
        at_r = at_r && (x[j] == rp.r[j]);
        if (j > 0) vol *= rp.r[j] - x[j];
      }
      bad |= out_of_box || at_r;
      const double h = vol - hv_pf;
      if (h > 0.0) answer += h;
    }
    out[c] = bad ? __builtin_nan("") : answer / M;
    if (raised) raised[c] = bad ? 1 : 0;
  }
}

hipError_t launch_ehvi_mc(hipStream_t stream, int k, const double* mu, const double* var, int64_t ld, int64_t N,
                          const double* cache, int M, const double* r, double hv_pf, double* out, int32_t* raised) {
  const size_t shm = sizeof(double) * (size_t)k * M;
  RefPoint rp{};
  for (int j = 0; j < k; ++j) rp.r[j] = r[j];
  const dim3 g(acq_grid(N)), b(kAcqThreads);
  switch (k) {
#define OMB_MC(KV) \
  case KV: hipLaunchKernelGGL(ehvi_mc_kernel<KV>, g, b, shm, stream, mu, var, ld, N, cache, M, rp, hv_pf, out, raised); break;
    OMB_MC(2) OMB_MC(3) OMB_MC(4) OMB_MC(5) OMB_MC(6) OMB_MC(7) OMB_MC(8)
#undef OMB_MC
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ------------------------------------------------------------------------------ exact EHVI over boxes
// "textbook" EHVI for k = 2, 3 objectives from a disjoint box decomposition of the non-dominated
// region (optimobo_amd.pareto.box_decomposition; replaces the Monte-Carlo EHVI_3D of
// util_functions.py:170-214 by its exact value):
//   EHVI = Σ_b Π_j G(lo_bj, hi_bj),  G(l, u) = (u−l)Φ(α) + (u−μ)(Φ(β)−Φ(α)) + σ(φ(β)−φ(α)),
//   α = (l−μ)/σ, β = (u−μ)/σ, σ_j = sqrt(σ²_j) per objective.
// One wavefront per candidate: its lanes tabulate Φ and φ at every grid coordinate (k·C values,
// a per-wave LDS table), then stride over the box list (staged once per workgroup in LDS when it
// fits) and reduce the box sum across the wave.  −∞ grid values arrive as −1e300 so
// (u − l)·Φ(α) is an exact 0 with no inf·0.
constexpr int kBoxWaves = 4;

template <int K, bool BOXES_LDS>
__global__ __launch_bounds__(64 * kBoxWaves) void ehvi_boxes_kernel(const double* __restrict__ mu,
                                                                    const double* __restrict__ var, int64_t ld,
                                                                    int64_t N, const double* __restrict__ coords,
                                                                    int C, const uint16_t* __restrict__ boxes, int B,
                                                                    double* __restrict__ out) {
  extern __shared__ double sm[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  double* grid = sm;                                    // K·C coordinates (−∞ → −1e300)
  double* tabP = grid + K * C + wave * 2 * K * C;      // this wave's Φ table
  double* tabp = tabP + K * C;                          // this wave's φ table
  uint16_t* lbox = reinterpret_cast<uint16_t*>(sm + K * C + kBoxWaves * 2 * K * C);
  for (int i = threadIdx.x; i < K * C; i += blockDim.x) grid[i] = fmax(coords[i], -1e300);
  if constexpr (BOXES_LDS) {
    for (int i = threadIdx.x; i < 2 * K * B; i += blockDim.x) lbox[i] = boxes[i];
  }
  __syncthreads();
  const uint16_t* bx = BOXES_LDS ? lbox : boxes;
  for (int64_t c = (int64_t)blockIdx.x * kBoxWaves + wave; c < N; c += (int64_t)gridDim.x * kBoxWaves) {
    double m[K], s[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      m[j] = mu[j * ld + c];
      s[j] = sqrt(var[j * ld + c]);
    }
    for (int i = lane; i < K * C; i += 64) {
      const int j = i / C;
      double mj = m[0], sj = s[0];
#pragma unroll
      for (int q = 1; q < K; ++q)
        if (j == q) {
          mj = m[q];
          sj = s[q];
        }
      const double t = (grid[i] - mj) / sj;
      tabP[i] = ndtr(t);
      tabp[i] = npdf(t);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    double acc = 0.0;
    for (int b = lane; b < B; b += 64) {
      double prod = 1.0;
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const int il = j * C + bx[2 * K * b + 2 * j], ih = j * C + bx[2 * K * b + 2 * j + 1];
        const double l = grid[il], u = grid[ih];
        const double Pl = tabP[il], Pu = tabP[ih];
        prod *= (u - l) * Pl + (u - m[j]) * (Pu - Pl) + s[j] * (tabp[ih] - tabp[il]);
      }
      acc += prod;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if (lane == 0) out[c] = acc;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");   // table reads done before the next candidate
  }
}

hipError_t launch_ehvi_boxes(hipStream_t stream, int k, const double* mu, const double* var, int64_t ld, int64_t N,
                             const double* coords, int C, const uint16_t* boxes, int B, double* out) {
  const size_t table = sizeof(double) * (size_t)k * C * (1 + 2 * kBoxWaves);
  const size_t box_bytes = sizeof(uint16_t) * 2 * (size_t)k * B;
  const bool in_lds = table + box_bytes <= 64 * 1024;
  const size_t shm = table + (in_lds ? box_bytes : 0);
  int64_t nb = (N + kBoxWaves - 1) / kBoxWaves;
  const unsigned grid = (unsigned)(nb > 16384 ? 16384 : (nb < 1 ? 1 : nb));
  dim3 g(grid), b(64 * kBoxWaves);
  if (k == 2) {
    if (in_lds) hipLaunchKernelGGL((ehvi_boxes_kernel<2, true>), g, b, shm, stream, mu, var, ld, N, coords, C, boxes, B, out);
    else hipLaunchKernelGGL((ehvi_boxes_kernel<2, false>), g, b, shm, stream, mu, var, ld, N, coords, C, boxes, B, out);
  } else {
    if (in_lds) hipLaunchKernelGGL((ehvi_boxes_kernel<3, true>), g, b, shm, stream, mu, var, ld, N, coords, C, boxes, B, out);
    else hipLaunchKernelGGL((ehvi_boxes_kernel<3, false>), g, b, shm, stream, mu, var, ld, N, coords, C, boxes, B, out);
  }
  return hipGetLastError();
}

// ------------------------------------------------------------------------------ HV-PoI
// emo.py:192-228 with vol5 (:176-189):  s = sqrt(σ² + 1e-5);
//   PoI = Σ_c Π_k [Φ((u_k−μ_k)/s_k) − Φ((l_k−μ_k)/s_k)],  I = Σ_c [u > μ]·Π_k(u_k − max(l_k, μ_k)).
__global__ __launch_bounds__(kAcqThreads) void hvpoi_kernel(const double* __restrict__ mu,
                                                            const double* __restrict__ var, int64_t ld, int64_t N,
                                                            const double* __restrict__ cells, int C,
                                                            double* __restrict__ out) {
  extern __shared__ double sm[];   // C × [up0, up1, lo0, lo1]
  for (int i = threadIdx.x; i < 4 * C; i += blockDim.x) sm[i] = cells[i];
  __syncthreads();
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < N; c += (int64_t)gridDim.x * blockDim.x) {
    const double m0 = mu[c], m1 = mu[ld + c];
    const double s0 = sqrt(var[c] + 1e-5), s1 = sqrt(var[ld + c] + 1e-5);
    double poi = 0.0, imp = 0.0;
    for (int j = 0; j < C; ++j) {
      const double u0 = sm[4 * j], u1 = sm[4 * j + 1], l0 = sm[4 * j + 2], l1 = sm[4 * j + 3];
      const double p0 = ndtr((u0 - m0) / s0) - ndtr((l0 - m0) / s0);
      const double p1 = ndtr((u1 - m1) / s1) - ndtr((l1 - m1) / s1);
      poi = poi + p0 * p1;
      if (u0 > m0 && u1 > m1) imp = imp + (u0 - fmax(l0, m0)) * (u1 - fmax(l1, m1));
    }
    out[c] = poi * imp;
  }
}

hipError_t launch_hvpoi(hipStream_t stream, const double* mu, const double* var, int64_t ld, int64_t N,
                        const double* cells, int C, double* out) {
  size_t shm = sizeof(double) * 4 * C;
  hipLaunchKernelGGL(hvpoi_kernel, dim3(acq_grid(N)), dim3(kAcqThreads), shm, stream, mu, var, ld, N, cells, C, out);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------ scalarisations
// optimobo/scalarisations.py:37-397 on one objective vector s (k entries), normalised by
// (s − ideal)/(max − ideal).  NaN propagates like numpy's max/sum.
__device__ __forceinline__ double nanmax(double a, double b) { return (a != a || b != b) ? __builtin_nan("") : (a > b ? a : b); }

template <int K>
__device__ double scalarise(const ScalParams& sp, const double* s) {
  double o[K];
#pragma unroll
  for (int i = 0; i < K; ++i) o[i] = (s[i] - sp.ideal[i]) / sp.range[i];
  switch (sp.id) {
    case OMB_SCAL_WS: {
      double a = 0.0;
#pragma unroll
      for (int i = 0; i < K; ++i) a += o[i] * sp.w[i];
      return a;
    }
    case OMB_SCAL_TCH: {
      double m = sp.w[0] * o[0];
#pragma unroll
      for (int i = 1; i < K; ++i) m = nanmax(m, sp.w[i] * o[i]);
      return m;
    }
    case OMB_SCAL_ATCH: {
      double m = fabs(o[0]) * sp.w[0], a = fabs(o[0]);
#pragma unroll
      for (int i = 1; i < K; ++i) {
        m = nanmax(m, fabs(o[i]) * sp.w[i]);
        a += fabs(o[i]);
      }
      return m + sp.p[0] * a;
    }
    case OMB_SCAL_MTCH: {
      double a = 0.0;
#pragma unroll
      for (int i = 0; i < K; ++i) a += fabs(o[i]);
      const double right = sp.p[0] * a;
      double m = (fabs(o[0]) + right) * sp.w[0];
#pragma unroll
      for (int i = 1; i < K; ++i) m = nanmax(m, (fabs(o[i]) + right) * sp.w[i]);
      return m;
    }
    case OMB_SCAL_EWC: {
      double a = 0.0;
#pragma unroll
      for (int i = 0; i < K; ++i) a += exp(sp.p[0] * sp.w[i] - 1.0) * exp(sp.p[0] * o[i]);
      return a;
    }
    case OMB_SCAL_WN: {
      double a = 0.0;
#pragma unroll
      for (int i = 0; i < K; ++i) a += pow(fabs(o[i]), sp.p[0]) * sp.w[i];
      return pow(a, 1.0 / sp.p[0]);
    }
    case OMB_SCAL_WPO: {
      double a = 0.0;
#pragma unroll
      for (int i = 0; i < K; ++i) a += pow(o[i], sp.p[0]) * sp.w[i];
      return a;
    }
    case OMB_SCAL_WPR: {
      double a = 1.0;
#pragma unroll
      for (int i = 0; i < K; ++i) a *= pow(o[i] + 100000.0, sp.w[i]);
      return a;
    }
    case OMB_SCAL_PBI:
    case OMB_SCAL_IPBI:
    case OMB_SCAL_QPBI: {
      double W[K];
      double d1 = 0.0;
#pragma unroll
      for (int i = 0; i < K; ++i) {
        W[i] = sp.w[i] / sp.wnorm;
        d1 += o[i] * W[i];
      }
      double q = 0.0;
#pragma unroll
      for (int i = 0; i < K; ++i) {
        const double e = o[i] - d1 * W[i];
        q += e * e;
      }
      const double d2 = sqrt(q);
      if (sp.id == OMB_SCAL_PBI) return d1 + sp.p[0] * d2;
      if (sp.id == OMB_SCAL_IPBI) return sp.p[0] * d2 - d1;
      return d1 + sp.p[0] * d2 * (d2 / sp.d_star);
    }
    case OMB_SCAL_APD: {
      double q = 0.0;
      bool zero = true;
#pragma unroll
      for (int i = 0; i < K; ++i) {
        q += o[i] * o[i];
        zero = zero && (o[i] == 0.0);
      }
      const double nrm = sqrt(q);                // norm_trans_f, before the zero fix-up (:384)
      double t[K];
      double tq = 0.0;
#pragma unroll
      for (int i = 0; i < K; ++i) {
        t[i] = zero ? 1e-5 : o[i];
        tq += t[i] * t[i];
      }
      const double tn = sqrt(tq);
      double dot = 0.0;
#pragma unroll
      for (int i = 0; i < K; ++i) dot += (t[i] / tn) * (sp.w[i] / sp.wnorm);
      dot = fmin(fmax(dot, -1.0), 1.0);
      const double theta = acos(dot);
      return (1.0 + (K * (sp.p[0] / sp.p[1])) * (theta / sp.p[2])) * nrm;
    }
    default:
      return __builtin_nan("");
  }
}

// util_functions.py:285-327: mean_j max(0, min − g(change(μ, σ²0)_j)).
template <int K>
__global__ __launch_bounds__(kAcqThreads) void expdec_kernel(ScalParams sp, const double* __restrict__ mu,
                                                             const double* __restrict__ var, int64_t ld, int64_t N,
                                                             const double* __restrict__ cache, int M,
                                                             double* __restrict__ out) {
  extern __shared__ double sm[];
  for (int i = threadIdx.x; i < K * M; i += blockDim.x) sm[i] = cache[i];
  __syncthreads();
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < N; c += (int64_t)gridDim.x * blockDim.x) {
    double m[K];
#pragma unroll
    for (int i = 0; i < K; ++i) m[i] = mu[i * ld + c];
    const double sd = sqrt(var[c]);             // σ²0 for every objective (quirk 1)
    double acc = 0.0;
    for (int j = 0; j < M; ++j) {
      double s[K];
#pragma unroll
      for (int i = 0; i < K; ++i) s[i] = sm[j * K + i] * sd + m[i];
      const double x = sp.agg_min - scalarise<K>(sp, s);
      acc += (x < 0.0) ? 0.0 : x;                // np.maximum(0, x): NaN propagates
    }
    out[c] = acc / M;
  }
}

hipError_t launch_expdec(hipStream_t stream, const ScalParams& sp, const double* mu, const double* var,
                         int64_t ld, int64_t N, const double* cache, int M, double* out) {
  size_t shm = sizeof(double) * sp.k * M;
  dim3 g(acq_grid(N)), b(kAcqThreads);
  switch (sp.k) {
#define OMB_ED(KV) \
  case KV: hipLaunchKernelGGL(expdec_kernel<KV>, g, b, shm, stream, sp, mu, var, ld, N, cache, M, out); break;
    OMB_ED(1) OMB_ED(2) OMB_ED(3) OMB_ED(4) OMB_ED(5) OMB_ED(6) OMB_ED(7) OMB_ED(8)
#undef OMB_ED
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ------------------------------------------------------------------------------ EI
// optimisers.py:325-344 / parego.py:126-145: σ = sqrt(σ² + eps); γ = (best − μ)/(σ + 1e-10);
// EI = σ(γΦ(γ) + φ(γ)).
// EI and its products with a second model (one thread per candidate).
//   MODE 0  EI(μ0, σ²0 + var_eps)                           optimisers.py:325-344, parego.py:126-145
//   MODE 1  μ1 · EI(μ0, σ²0 + var_eps)                      KEEP pareto_expected_improvement, keep.py:142-151
//   MODE 2  EI(μ0, σ²0 + var_eps) · Π_{c=1}^{k-1} Φ(−μc / sqrt(σ²c + pof_eps))
//                                                           ParEGO_C2.consraint_ei, cparego.py:471-496
template <int MODE>
__global__ __launch_bounds__(kAcqThreads) void ei_kernel(const double* __restrict__ mu, const double* __restrict__ var,
                                                         int64_t ld, int64_t N, int k, double best, double var_eps,
                                                         double pof_eps, double* __restrict__ out) {
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < N; c += (int64_t)gridDim.x * blockDim.x) {
    const double sigma = sqrt(var[c] + var_eps);
    const double gamma = (best - mu[c]) / (sigma + 1e-10);
    double v = sigma * (gamma * ndtr(gamma) + npdf(gamma));
    if (MODE == 1) v = mu[ld + c] * v;
    if (MODE == 2) {
      double pof = 1.0;
      for (int j = 1; j < k; ++j) pof *= ndtr((0.0 - mu[j * ld + c]) / sqrt(var[j * ld + c] + pof_eps));
      v = v * pof;
    }
    out[c] = v;
  }
}

hipError_t launch_ei(hipStream_t stream, int kind, int k, const double* mu, const double* var, int64_t ld, int64_t N,
                     double best, double var_eps, double pof_eps, double* out) {
  const dim3 grid(acq_grid(N)), block(kAcqThreads);
  if (kind == OMB_EI_PARETO)
    hipLaunchKernelGGL(ei_kernel<1>, grid, block, 0, stream, mu, var, ld, N, k, best, var_eps, pof_eps, out);
  else if (kind == OMB_EI_CONSTRAINED)
    hipLaunchKernelGGL(ei_kernel<2>, grid, block, 0, stream, mu, var, ld, N, k, best, var_eps, pof_eps, out);
  else
    hipLaunchKernelGGL(ei_kernel<0>, grid, block, 0, stream, mu, var, ld, N, k, best, var_eps, pof_eps, out);
  return hipGetLastError();
}

}  // namespace omb
