// Write-stream ceilings on MI355X for the K-block roofline: what a 4 GiB (512 × 2^20 fp64) row-major
// block can be written at, per store shape.  Each variant writes the whole block once per launch.
//   linear16   grid-stride, 16 B per lane, consecutive lanes contiguous (1 KiB per wave-instruction)
//   rows4x128  the current K-block shape: 8 B per lane, 4 rows × 16 lanes (4 × 128-B segments)
//   rows2x256  8 B per lane, 2 rows × 32 lanes (2 × 256-B segments)
//   row512     8 B per lane, 1 row × 64 lanes (512 B)
//   row1k16    16 B per lane, 1 row × 64 lanes (1 KiB)
//   rows2x512  16 B per lane, 2 rows × 32 lanes (2 × 512 B)
// each plain and non-temporal; a workgroup (256 threads) covers 64 or 128 columns × 256 rows like the
// K-block kernel.  hipMemsetD32 of the block is timed too.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench/mb_write tools/microbench/mb_write.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double d2 __attribute__((ext_vector_type(2)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)

template <bool NT, typename T>
__device__ __forceinline__ void st(T* p, T v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <bool NT>
__global__ __launch_bounds__(256) void linear16(d2* __restrict__ dst, int64_t n2) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (int64_t)gridDim.x * blockDim.x)
    st<NT>(dst + i, d2{(double)i, 1.0});
}

// SHAPE: 0 rows4x128, 1 rows2x256, 2 row512 (8 B/lane); 3 row1k16, 4 rows2x512 (16 B/lane).
// A workgroup covers COLS columns × 256 rows; wave w owns columns [w·COLS/4, (w+1)·COLS/4) for SHAPE 0
// and every wave sweeps all COLS columns of its own quarter of the rows otherwise.
template <int SHAPE, bool NT>
__global__ __launch_bounds__(256) void rows(double* __restrict__ K, int64_t N, int n) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r0 = blockIdx.y * 256;
  if constexpr (SHAPE == 0) {
    // 64 columns per WG, wave w: columns 16w..16w+15; lanes: row 4e + (lane>>4), column lane&15
    const int64_t col = (int64_t)blockIdx.x * 64 + 16 * wave + (lane & 15);
    for (int T = 0; T < 16; ++T)
      for (int e = 0; e < 4; ++e) {
        const int k = r0 + 16 * T + 4 * e + (lane >> 4);
        st<NT>(K + (int64_t)k * N + col, (double)k);
      }
  } else if constexpr (SHAPE == 1) {
    // 64 columns per WG: 2 rows × 32 columns per instruction; wave w: rows r0 + 64w ..
    for (int rr = 0; rr < 64; rr += 2)
      for (int h = 0; h < 2; ++h) {
        const int k = r0 + 64 * wave + rr + (lane >> 5);
        const int64_t col = (int64_t)blockIdx.x * 64 + 32 * h + (lane & 31);
        st<NT>(K + (int64_t)k * N + col, (double)k);
      }
  } else if constexpr (SHAPE == 2) {
    for (int rr = 0; rr < 64; ++rr) {
      const int k = r0 + 64 * wave + rr;
      const int64_t col = (int64_t)blockIdx.x * 64 + lane;
      st<NT>(K + (int64_t)k * N + col, (double)k);
    }
  } else if constexpr (SHAPE == 3) {
    // 128 columns per WG, one row per instruction (64 lanes × 16 B)
    for (int rr = 0; rr < 64; ++rr) {
      const int k = r0 + 64 * wave + rr;
      const int64_t col = (int64_t)blockIdx.x * 128 + 2 * lane;
      st<NT>(reinterpret_cast<d2*>(K + (int64_t)k * N + col), d2{(double)k, 1.0});
    }
  } else {
    // 64 columns per WG, 2 rows × 32 lanes × 16 B per instruction
    for (int rr = 0; rr < 64; rr += 2) {
      const int k = r0 + 64 * wave + rr + (lane >> 5);
      const int64_t col = (int64_t)blockIdx.x * 64 + 2 * (lane & 31);
      st<NT>(reinterpret_cast<d2*>(K + (int64_t)k * N + col), d2{(double)k, 1.0});
    }
  }
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
  const int n = 512;
  const int64_t N = 1 << 20;
  const int64_t tot = (int64_t)n * N;
  double* K;
  CK(hipMalloc(&K, tot * 8));
  const double bytes = tot * 8.0;
  auto report = [&](const char* name, float t) { printf("%-22s %7.3f ms  %7.0f GB/s\n", name, t, bytes / (t * 1e-3) / 1e9); };
  for (int rep = 0; rep < 2; ++rep) {
    report("memsetD32", timeit([&] { CK(hipMemsetD32((hipDeviceptr_t)K, 0, tot * 2)); }, 5));
    report("linear16 plain", timeit([&] { hipLaunchKernelGGL(linear16<false>, dim3(16384), dim3(256), 0, 0, (d2*)K, tot / 2); }, 5));
    report("linear16 nt", timeit([&] { hipLaunchKernelGGL(linear16<true>, dim3(16384), dim3(256), 0, 0, (d2*)K, tot / 2); }, 5));
    dim3 g64((unsigned)(N / 64), n / 256), g128((unsigned)(N / 128), n / 256);
#define V(S, NTV, G, NAME) report(NAME, timeit([&] { hipLaunchKernelGGL((rows<S, NTV>), G, dim3(256), 0, 0, K, N, n); }, 5));
    V(0, false, g64, "rows4x128 plain") V(0, true, g64, "rows4x128 nt")
    V(1, false, g64, "rows2x256 plain") V(1, true, g64, "rows2x256 nt")
    V(2, false, g64, "row512 plain") V(2, true, g64, "row512 nt")
    V(3, false, g128, "row1k16 plain") V(3, true, g128, "row1k16 nt")
    V(4, false, g64, "rows2x512 plain") V(4, true, g64, "rows2x512 nt")
#undef V
  }
  return 0;
}
