// Accuracy of the Cholesky pivot's inverse square root (chol16_factor): v_rsq_f64 + two Newton steps (the library)
// against v_rsq_f64 + one second-order correction (OMB_CHOL16_POLY2, tools), over 2^22 pivots log-uniform in [1e-300, 1e300]
// and 2^22 in [0.5, 2], in ulps of the correctly rounded 1/sqrt(d) (host long double).  Tools only.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/microbench/mb_rsq tools/microbench/mb_rsq.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)

__global__ void rsq_kernel(const double* __restrict__ d, double* __restrict__ out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double dj = d[i];
  const double y0 = __builtin_amdgcn_rsq(dj);
  const double hd = 0.5 * dj;
  const double y1 = fma(y0, fma(-hd * y0, y0, 0.5), y0);
  out[4 * i + 0] = fma(y1, fma(-hd * y1, y1, 0.5), y1);
  const double r = fma(dj * y0, y0, -1.0);
  out[4 * i + 1] = fma(y0 * r, fma(r, 0.375, -0.5), y0);
  out[4 * i + 2] = y0;
  out[4 * i + 3] = r;
}

static double ulps(double got, long double ref) {
  const double rr = (double)ref;
  const double u = std::nextafter(rr, INFINITY) - rr;
  return (double)std::fabs(((long double)got - ref) / (long double)u);
}

int main() {
  const int n = 1 << 22;
  std::mt19937_64 rng(7);
  for (int range = 0; range < 2; ++range) {
    std::vector<double> h(n);
    std::uniform_real_distribution<double> U(range ? std::log(0.5) : std::log(1e-300), range ? std::log(2.0) : std::log(1e300));
    for (auto& x : h) x = std::exp(U(rng));
    double *d, *o;
    CK(hipMalloc(&d, n * 8));
    CK(hipMalloc(&o, 4 * (size_t)n * 8));
    CK(hipMemcpy(d, h.data(), n * 8, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(rsq_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, d, o, n);
    CK(hipDeviceSynchronize());
    std::vector<double> out(4 * (size_t)n);
    CK(hipMemcpy(out.data(), o, out.size() * 8, hipMemcpyDeviceToHost));
    double m[2] = {0, 0}, mean[2] = {0, 0}, seed = 0;
    long long exact[2] = {0, 0};
    for (int i = 0; i < n; ++i) {
      const long double ref = 1.0L / std::sqrt((long double)h[i]);
      for (int v = 0; v < 2; ++v) {
        const double e = ulps(out[4 * i + v], ref);
        m[v] = std::max(m[v], e);
        mean[v] += e / n;
        if (out[4 * i + v] == (double)ref) ++exact[v];
      }
      seed = std::max(seed, (double)std::fabs(((long double)out[4 * i + 2] - ref) / ref));
    }
    printf("%s: v_rsq_f64 seed max rel err %.3e (2^%.1f)\n", range ? "[0.5, 2]" : "[1e-300, 1e300]", seed, std::log2(seed));
    printf("  two Newton steps (library):   max %.3f ulp, mean %.4f, correctly rounded %.4f\n", m[0], mean[0], (double)exact[0] / n);
    printf("  second-order correction:      max %.3f ulp, mean %.4f, correctly rounded %.4f\n", m[1], mean[1], (double)exact[1] / n);
    CK(hipFree(d));
    CK(hipFree(o));
  }
  return 0;
}
