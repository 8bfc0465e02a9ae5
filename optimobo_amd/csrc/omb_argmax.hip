// Deterministic arg-max over the acquisition values (replaces scipy's differential_evolution
// maximiser, optimisers.py:87,118): lowest index among maxima; NaN and −inf never win.
// Pass 1: ≤ kArgmaxMaxBlocks workgroups, grid-stride scan + wave/LDS reduction → partials.
// Pass 2: one workgroup reduces the partials in index order → result {value, index+offset}.
// Round 4: both passes in one launch (argmax_onepass): the workgroup that arrives last at a ticket reduces the
// partials, so the chain saves a dependent launch.
#include "omb_internal.h"
#include "omb_math.h"

namespace omb {

struct VI {
  double v;
  int64_t i;
};

__device__ __forceinline__ bool better(const VI& a, const VI& b) {  // is a strictly preferred to b?
  if (a.i < 0) return false;
  if (b.i < 0) return true;
  return (a.v > b.v) || (a.v == b.v && a.i < b.i);
}

__device__ VI block_reduce(VI x) {
  __shared__ double sv[16];
  __shared__ int64_t si[16];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    VI y{__shfl_down(x.v, off), (int64_t)__shfl_down((long long)x.i, off)};
    if (better(y, x)) x = y;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    sv[wave] = x.v;
    si[wave] = x.i;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nw = blockDim.x >> 6;
    for (int w = 1; w < nw; ++w) {
      VI y{sv[w], si[w]};
      if (better(y, x)) x = y;
    }
  }
  return x;
}

__global__ __launch_bounds__(256) void argmax_pass1(const double* __restrict__ vals, int64_t N,
                                                    double* __restrict__ partials) {
  VI best{-__builtin_inf(), -1};
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < N; c += (int64_t)gridDim.x * blockDim.x) {
    const double v = vals[c];
    if (v == v && v > -__builtin_inf()) {
      VI y{v, c};
      if (better(y, best)) best = y;
    }
  }
  best = block_reduce(best);
  if (threadIdx.x == 0) {
    partials[2 * blockIdx.x] = best.v;
    partials[2 * blockIdx.x + 1] = __builtin_bit_cast(double, (long long)best.i);
  }
}

__global__ __launch_bounds__(256) void argmax_pass2(const double* __restrict__ partials, int nb, int64_t offset,
                                                    double* __restrict__ result) {
  VI best{-__builtin_inf(), -1};
  for (int b = threadIdx.x; b < nb; b += blockDim.x) {
    VI y{partials[2 * b], (int64_t)__builtin_bit_cast(long long, partials[2 * b + 1])};
    if (better(y, best)) best = y;
  }
  best = block_reduce(best);
  if (threadIdx.x == 0) {
    result[0] = best.i < 0 ? -__builtin_inf() : best.v;
    result[1] = best.i < 0 ? -1.0 : (double)(best.i + offset);
  }
}

// Pass 1 and pass 2 in one launch.  Each workgroup stores its pair with agent-scope (sc1) stores, waits for them
// (vmcnt 0) and takes a ticket (relaxed agent-scope add); the one that draws gridDim − 1 reads every pair with sc1
// loads and reduces them in workgroup order, as pass 2 does, then resets the ticket for the next launch
// (MI355X_MICROARCH.md § inter-workgroup visibility: the sc1 form with one unsharded counter).  The result is
// bitwise pass 2's: the same pairs reduced by the same block_reduce.
__global__ __launch_bounds__(256) void argmax_onepass(const double* __restrict__ vals, int64_t N,
                                                      double* __restrict__ partials, unsigned* __restrict__ ticket,
                                                      int64_t offset, double* __restrict__ result) {
  __shared__ int is_last;
  VI best{-__builtin_inf(), -1};
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < N; c += (int64_t)gridDim.x * blockDim.x) {
    const double v = vals[c];
    if (v == v && v > -__builtin_inf()) {
      VI y{v, c};
      if (better(y, best)) best = y;
    }
  }
  best = block_reduce(best);
  if (threadIdx.x == 0) {
    wf_store_f64(&partials[2 * blockIdx.x], best.v);
    wf_store_f64(&partials[2 * blockIdx.x + 1], __builtin_bit_cast(double, (long long)best.i));
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    is_last = prev == gridDim.x - 1;
  }
  __syncthreads();
  if (!__builtin_amdgcn_readfirstlane(is_last)) return;   // uniform: the reduction below has barriers
  VI x{-__builtin_inf(), -1};
  for (int b = threadIdx.x; b < (int)gridDim.x; b += blockDim.x) {
    VI y{wf_load_f64(&partials[2 * b]), (int64_t)__builtin_bit_cast(long long, wf_load_f64(&partials[2 * b + 1]))};
    if (better(y, x)) x = y;
  }
  x = block_reduce(x);
  if (threadIdx.x == 0) {
    result[0] = x.i < 0 ? -__builtin_inf() : x.v;
    result[1] = x.i < 0 ? -1.0 : (double)(x.i + offset);
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

hipError_t launch_argmax_reduce(hipStream_t stream, const double* partials, int nb, int64_t offset, double* result) {
  hipLaunchKernelGGL(argmax_pass2, dim3(1), dim3(256), 0, stream, partials, nb, offset, result);
  return hipGetLastError();
}

hipError_t launch_argmax(hipStream_t stream, const double* vals, int64_t N, int64_t offset, double* partials,
                         double* result, bool one_pass) {
  int64_t nb = (N + 255) / 256;
  if (nb > kArgmaxMaxBlocks) nb = kArgmaxMaxBlocks;
  if (nb < 1) nb = 1;
  if (one_pass) {
    unsigned* ticket = reinterpret_cast<unsigned*>(partials + 2 * kArgmaxMaxBlocks);
    hipLaunchKernelGGL(argmax_onepass, dim3((unsigned)nb), dim3(256), 0, stream, vals, N, partials, ticket, offset,
                       result);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(argmax_pass1, dim3((unsigned)nb), dim3(256), 0, stream, vals, N, partials);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(argmax_pass2, dim3(1), dim3(256), 0, stream, partials, (int)nb, offset, result);
  return hipGetLastError();
}

}  // namespace omb
