// Host-only argument validation and upload packing of liboptimobo_hip.so's C-ABI (no HIP runtime, no device code).
//
// omb_api.hip calls these before it touches the device, so every entry point's argument checks, the
// expected-decomposition parameter block and the Sobol' state packing are plain C++ that builds with a host
// compiler alone: `make -C optimobo_amd/csrc asan` compiles this file under ASan + UBSan into the fuzz driver
// tests/asan/omb_host_fuzz.cpp (and into an ASan build of the library that tests/test_lib_cpu.py loads).
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <string>

#include "../../include/optimobo_hip.h"

namespace omb {

// Acquisition kernels stage their per-iteration geometry in ≤ 64 KiB of dynamic LDS.
constexpr int kMaxLdsDoubles = 8192;
constexpr int kMaxStripes = (kMaxLdsDoubles - 1) / 2;

// Parameters of one expected_decomposition scalarisation (omb_acquisition.hip's expdec_kernel).
struct ScalParams {
  int id;
  int k;
  double w[OMB_MAX_OBJ];
  double ideal[OMB_MAX_OBJ];
  double range[OMB_MAX_OBJ];   // max − ideal
  double p[4];
  double wnorm;                // ‖w‖ (PBI family)
  double d_star;               // QPBI
  double agg_min;
};

// Formats the message into *err (when err is non-null) and returns code.
int errf(std::string* err, int code, const char* fmt, ...) __attribute__((format(printf, 3, 4)));

// n_var padded to the posterior kernels' DP ∈ {2, 4, 6, 8, 16, 32, 64, 128, 256}; −1 above OMB_MAX_DIM.
int pad_dim(int d);

int check_moments(std::string* err, const void* mu, const void* var, int64_t ld, int64_t N, int k, const void* out);
int check_ehvi2d(std::string* err, int P, const double* r, int mode);
int check_ehvi_mc(std::string* err, int k, int M, const double* r);
int check_boxes(std::string* err, int k, int C, int B);
int check_ei(std::string* err, int kind, int k, double var_eps, double pof_eps);
int check_hvpoi(std::string* err, int C);
// Validates an expected_decomposition request and fills its ScalParams.
int build_scal(std::string* err, int k, int M, int scal_id, const double* params_host, const double* weights_host,
               const double* ideal_host, const double* max_host, double agg_min, ScalParams* out);
// omb_set_gp's host-side checks (before any device work).
int check_gp_args(std::string* err, int obj, int kernel, int n, int d, const void* X_dev, const double* lengthscale_host,
                  double variance, const void* alpha_dev, const void* Linv_dev);
// omb_set_sobol's host-side checks.
int check_sobol_args(std::string* err, int d, int bits, const void* sv_host, const void* shift_host,
                     const double* lo_host, const double* hi_host);

// The packed Sobol' state (sobol_kernel's layout): sv (d·bits uint32) | shift (d uint32) | [pad] | lo (d f64) |
// width (d f64).
size_t sobol_state_bytes(int d, int bits);
void sobol_pack_state(int d, int bits, const uint32_t* sv, const uint32_t* shift, const double* lo, const double* hi,
                      void* dst);

}  // namespace omb
