// Scrambled Sobol' candidate generation on the device: the candidate
// batch the maximiser scores is written straight into HBM instead of being generated on the
// host and copied over PCIe.
//
// The sequence is scipy.stats.qmc.Sobol's (the reference draws its MC cache with it,
// optimisers.py:121-141): with the (scrambled) direction numbers sv[j][b] and digital shift
// shift[j] of a Sobol engine, point i is
//     u_ij = (shift[j] ⊕ ⨁_{b : bit b of gray(i) set} sv[j][b]) · 2^-bits,  gray(i) = i ⊕ (i >> 1),
// the closed form of the engine's gray-code recurrence, so any index range [start, start + N)
// is generated without a sequential scan.  x_ij = lo_j + u_ij · (hi_j − lo_j), rounded as
// numpy rounds `lo + U * (hi - lo)` (no fused multiply-add), so the device points are
// bit-identical to the host expression on scipy's output.
//
// Bound: HBM writes (8·d bytes per point); the XOR walk is ~popcount(gray(i)) integer ops.
#include "omb_internal.h"

namespace omb {

namespace {

constexpr int kSobolThreads = 256;
constexpr int kSobolMaxBlocks = 16384;

// Device layout of SobolDev (see omb_set_sobol): sv (d·bits uint32) | shift (d uint32) |
// lo (d f64) | width (d f64); `words` = d·bits + d rounded up to an even count.
// MAXD: the LDS copy's capacity in dimensions (64 for the usual n_var, so the workgroup's LDS stays at 10 KiB;
// OMB_MAX_DIM above that)
template <int MAXD>
__global__ __launch_bounds__(kSobolThreads) void sobol_kernel(const uint32_t* __restrict__ state, int d, int bits,
                                                             int64_t start, int64_t total, double scale,
                                                             double* __restrict__ X) {
#pragma clang fp contract(off)
  __shared__ uint32_t sv[MAXD * 32];
  __shared__ uint32_t shift[MAXD];
  __shared__ double lo[MAXD], width[MAXD];
  const int words = d * bits + d;
  const double* fstate = reinterpret_cast<const double*>(state + ((words + 1) & ~1));
  for (int t = threadIdx.x; t < d * bits; t += blockDim.x) sv[t] = state[t];
  for (int t = threadIdx.x; t < d; t += blockDim.x) {
    shift[t] = state[d * bits + t];
    lo[t] = fstate[t];
    width[t] = fstate[d + t];
  }
  __syncthreads();
  // one output element per thread and iteration: e = i·d + j, so stores are fully coalesced
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / d;
    const int j = (int)(e - i * d);
    const uint64_t p = (uint64_t)(start + i);
    uint64_t g = p ^ (p >> 1);
    uint32_t q = shift[j];
    const uint32_t* v = sv + j * bits;
    while (g) {
      q ^= v[__builtin_ctzll(g)];
      g &= g - 1;
    }
    const double u = (double)q * scale;
    X[e] = lo[j] + u * width[j];
  }
}

}  // namespace

hipError_t launch_sobol(hipStream_t stream, const void* state_dev, int d, int bits, int64_t start, int64_t N,
                        double* X) {
  const int64_t total = N * d;
  if (total <= 0) return hipSuccess;
  int64_t nb = (total + kSobolThreads - 1) / kSobolThreads;
  if (nb > kSobolMaxBlocks) nb = kSobolMaxBlocks;
  const double scale = 1.0 / (double)(1ull << bits);
  if (d <= 64)
    hipLaunchKernelGGL(sobol_kernel<64>, dim3((unsigned)nb), dim3(kSobolThreads), 0, stream,
                       static_cast<const uint32_t*>(state_dev), d, bits, start, total, scale, X);
  else
    hipLaunchKernelGGL(sobol_kernel<OMB_MAX_DIM>, dim3((unsigned)nb), dim3(kSobolThreads), 0, stream,
                       static_cast<const uint32_t*>(state_dev), d, bits, start, total, scale, X);
  return hipGetLastError();
}

}  // namespace omb
