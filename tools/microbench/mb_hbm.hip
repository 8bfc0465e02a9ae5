// HBM ceilings on MI355X for the K-block roofline: a write-only stream (the K block's pattern:
// 16-byte stores, consecutive lanes contiguous, plain and non-temporal), a read-only stream and
// a copy.  Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench/mb_hbm tools/microbench/mb_hbm.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double d2 __attribute__((ext_vector_type(2)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)

template <bool NT>
__global__ __launch_bounds__(256) void write_kernel(d2* __restrict__ dst, int64_t n2, int rows_per_block, int64_t pitch2) {
  // like kernel_block_kernel: a thread owns one 16-B column slot and walks `rows_per_block` rows
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= pitch2) return;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_block;
  for (int r = 0; r < rows_per_block; ++r) {
    const int64_t i = (r0 + r) * pitch2 + c;
    if (i >= n2) return;
    const d2 v = d2{(double)r, (double)c};
    if constexpr (NT)
      __builtin_nontemporal_store(v, dst + i);
    else
      dst[i] = v;
  }
}

__global__ __launch_bounds__(256) void read_kernel(const d2* __restrict__ src, int64_t n2, double* out) {
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (int64_t)gridDim.x * blockDim.x) {
    const d2 v = src[i];
    s += v.x + v.y;
  }
  if (s == 1234.5) out[0] = s;   // keep the loads
}

__global__ __launch_bounds__(256) void copy_kernel(const d2* __restrict__ src, d2* __restrict__ dst, int64_t n2) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

template <typename F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  const int64_t rows = 512, cols = 1 << 20;     // the K block of config 3: (512, 2^20) fp64 = 4 GiB
  const int64_t n = rows * cols, n2 = n / 2, pitch2 = cols / 2;
  d2 *A, *B;
  double* out;
  CK(hipMalloc(&A, n * 8));
  CK(hipMalloc(&B, n * 8));
  CK(hipMalloc(&out, 8));
  const double bytes = n * 8.0;
  dim3 wgrid((unsigned)(pitch2 / 256), (unsigned)(rows / 256));
  float t;
  t = timeit([&] { hipLaunchKernelGGL(write_kernel<false>, wgrid, dim3(256), 0, 0, A, n2, 256, pitch2); }, 5);
  printf("write plain, K-block pattern    %7.3f ms  %7.0f GB/s\n", t, bytes / (t * 1e-3) / 1e9);
  t = timeit([&] { hipLaunchKernelGGL(write_kernel<true>, wgrid, dim3(256), 0, 0, A, n2, 256, pitch2); }, 5);
  printf("write nontemporal, K-block pat. %7.3f ms  %7.0f GB/s\n", t, bytes / (t * 1e-3) / 1e9);
  dim3 wgrid2((unsigned)(pitch2 / 256), (unsigned)(rows / 16));
  t = timeit([&] { hipLaunchKernelGGL(write_kernel<true>, wgrid2, dim3(256), 0, 0, A, n2, 16, pitch2); }, 5);
  printf("write nontemporal, 16 rows/WG   %7.3f ms  %7.0f GB/s\n", t, bytes / (t * 1e-3) / 1e9);
  t = timeit([&] { hipLaunchKernelGGL(read_kernel, dim3(8192), dim3(256), 0, 0, A, n2, out); }, 5);
  printf("read                            %7.3f ms  %7.0f GB/s\n", t, bytes / (t * 1e-3) / 1e9);
  t = timeit([&] { hipLaunchKernelGGL(copy_kernel, dim3(8192), dim3(256), 0, 0, A, B, n2); }, 5);
  printf("copy (read + write)             %7.3f ms  %7.0f GB/s\n", t, 2 * bytes / (t * 1e-3) / 1e9);
  return 0;
}
