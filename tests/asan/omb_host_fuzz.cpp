// Fuzz driver of the C-ABI's host-only argument checks and packing (optimobo_amd/csrc/omb_host.cpp), built by
// `make -C optimobo_amd/csrc asan` under ASan + UBSan and run by tests/test_asan_host.py (CPU only).
//
// Every call draws its arguments from the edges of each range (INT_MIN, −1, 0, 1, the limit, limit + 1, INT_MAX,
// huge products) and random values, with every array allocated to EXACTLY the length the function may read — so an
// over-read is an ASan report, an overflowed size product a UBSan report — and compares the return code with the
// specification written out independently below (include/optimobo_hip.h's contract).  Exit 0 = every call as
// specified and no sanitizer report; the sanitizers abort on the first report (-fno-sanitize-recover=all).
#include <limits.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <memory>
#include <string>
#include <vector>

#include "../../optimobo_amd/csrc/omb_host.h"

using namespace omb;

namespace {

uint64_t g_state = 0x9E3779B97F4A7C15ull;
uint64_t next_u64() {
  g_state ^= g_state << 13;
  g_state ^= g_state >> 7;
  g_state ^= g_state << 17;
  return g_state;
}
int pick(const std::vector<int>& edges, int lo, int hi) {
  if (next_u64() % 3 == 0) return lo + (int)(next_u64() % (uint64_t)(hi - lo + 1));
  return edges[next_u64() % edges.size()];
}
double pick_d() {
  const double edges[] = {0.0, -0.0, 1.0, -1.0, 1e-300, -1e-300, 1e300, INFINITY, -INFINITY, NAN, 0.5, 3.0};
  if (next_u64() % 2) return edges[next_u64() % 12];
  return ((double)(next_u64() % 2000001) - 1000000.0) / 1000.0;
}

// A heap array of exactly n doubles (n ≥ 1 so the pointer is valid), filled with `fill`.
std::unique_ptr<double[]> darr(int64_t n, double fill) {
  std::unique_ptr<double[]> p(new double[n < 1 ? 1 : n]);
  for (int64_t i = 0; i < (n < 1 ? 1 : n); ++i) p[i] = fill;
  return p;
}

long g_calls = 0, g_fail = 0;
void expect(int got, int want, const char* what, const std::string& err) {
  ++g_calls;
  if (got != want) {
    if (g_fail++ < 20) fprintf(stderr, "MISMATCH %s: got %d want %d (%s)\n", what, got, want, err.c_str());
  }
  if (got != OMB_OK && err.empty()) {
    if (g_fail++ < 20) fprintf(stderr, "MISSING MESSAGE %s: code %d\n", what, got);
  }
}

const std::vector<int> kIntEdges = {INT_MIN, -1000000, -1, 0, 1, 2, 3, 4, 7, 8, 9, 16, 64, 255, 256, 257, 1024, 2048,
                                    2049, 4095, 4096, 4097, 8191, 8192, 8193, 16384, 16385, 1 << 20, 1 << 30, INT_MAX};

void fuzz_moments() {
  for (int it = 0; it < 20000; ++it) {
    std::string err;
    const int64_t N = (int64_t)pick(kIntEdges, -5, 5) * (next_u64() % 2 ? 1 : 4096);
    const int64_t ld = (int64_t)pick(kIntEdges, -5, 5) * (next_u64() % 2 ? 1 : 4096);
    const int k = pick(kIntEdges, 0, 9);
    double x = 0.0;
    const void* mu = next_u64() % 5 ? &x : nullptr;
    const void* var = next_u64() % 5 ? &x : nullptr;
    const void* out = next_u64() % 5 ? &x : nullptr;
    int want = OMB_OK;
    if (N < 0) want = OMB_EINVAL;
    else if (N > 0 && (!mu || !var || !out)) want = OMB_EINVAL;
    else if (k > 1 && ld < N) want = OMB_EINVAL;
    expect(check_moments(&err, mu, var, ld, N, k, out), want, "check_moments", err);
  }
}

void fuzz_acq_checks() {
  for (int it = 0; it < 40000; ++it) {
    std::string err;
    double r[OMB_MAX_OBJ] = {1, 1, 1, 1, 1, 1, 1, 1};
    const double* rp = next_u64() % 6 ? r : nullptr;
    {
      const int P = pick(kIntEdges, -2, 4100), mode = pick({-1, 0, 1, 2, 3, INT_MAX}, -1, 3);
      int want = OMB_OK;
      if (P < 1 || P > kMaxStripes) want = OMB_EUNSUP;
      else if (!rp) want = OMB_EINVAL;
      else if (mode < 0 || mode > 2) want = OMB_EINVAL;
      err.clear();
      expect(check_ehvi2d(&err, P, rp, mode), want, "check_ehvi2d", err);
    }
    {
      const int k = pick({INT_MIN, -1, 0, 1, 2, 3, 4, 5, 8, 9, INT_MAX}, 0, 9), M = pick(kIntEdges, -2, 8200);
      int want = OMB_OK;
      if (k < 2 || k > OMB_MAX_OBJ) want = OMB_EINVAL;
      else if (M < 1 || (long long)k * M > 8192) want = OMB_EUNSUP;
      else if (!rp) want = OMB_EINVAL;
      err.clear();
      expect(check_ehvi_mc(&err, k, M, rp), want, "check_ehvi_mc", err);
    }
    {
      const int k = pick({INT_MIN, 0, 1, 2, 3, 4, INT_MAX}, 0, 4), C = pick(kIntEdges, -2, 500);
      const int B = pick(kIntEdges, -2, 5);
      int want = OMB_OK;
      if (k != 2 && k != 3) want = OMB_EUNSUP;
      else if (C < 2 || (long long)k * C * 9 > 8192) want = OMB_EUNSUP;
      else if (B < 1) want = OMB_EINVAL;
      err.clear();
      expect(check_boxes(&err, k, C, B), want, "check_boxes", err);
    }
    {
      const int kind = pick({-1, 0, 1, 2, 3, INT_MAX}, 0, 2), k = pick({INT_MIN, 0, 1, 2, 3, 8, 9, INT_MAX}, 0, 9);
      const double ve = pick_d(), pe = pick_d();
      const bool ok_k = (kind == OMB_EI_PLAIN && k == 1) || (kind == OMB_EI_PARETO && k == 2) ||
                        (kind == OMB_EI_CONSTRAINED && k >= 2 && k <= 8);
      int want = OMB_OK;
      if (!ok_k) want = OMB_EINVAL;
      else if (!(ve >= 0.0) || !(pe >= 0.0)) want = OMB_EINVAL;
      err.clear();
      expect(check_ei(&err, kind, k, ve, pe), want, "check_ei", err);
    }
    {
      const int C = pick(kIntEdges, -2, 2100);
      const int want = (C < 1 || 4LL * C > 8192) ? OMB_EUNSUP : OMB_OK;
      err.clear();
      expect(check_hvpoi(&err, C), want, "check_hvpoi", err);
    }
  }
}

void fuzz_build_scal() {
  for (int it = 0; it < 40000; ++it) {
    std::string err;
    const int k = pick({INT_MIN, -1, 0, 1, 2, 3, 4, 5, 8, 9, INT_MAX}, 1, 8);
    const int M = pick(kIntEdges, 1, 2048);
    const int id = pick({INT_MIN, -1, 0, 1, 5, 11, 12, 13, INT_MAX}, 0, 11);
    const int np = (id == OMB_SCAL_QPBI || id == OMB_SCAL_APD) ? 3
                   : (id == OMB_SCAL_WS || id == OMB_SCAL_TCH || id == OMB_SCAL_WPR) ? 0 : 1;
    const int kk = (k >= 1 && k <= 8) ? k : 1;
    const bool zero_w = next_u64() % 5 == 0;
    auto w = darr(kk, zero_w ? 0.0 : 0.25), ideal = darr(kk, pick_d()), mx = darr(kk, pick_d());
    auto params = darr(np, pick_d());
    const double* pp = (np > 0 && next_u64() % 6) ? params.get() : nullptr;
    const double* wp = next_u64() % 8 ? w.get() : nullptr;
    ScalParams sp;
    int want = OMB_OK;
    if (k < 1 || k > 8) want = OMB_EINVAL;
    else if (M < 1 || (long long)k * M > 8192) want = OMB_EUNSUP;
    else if (id < 0 || id > 11) want = OMB_EINVAL;
    else if (!wp) want = OMB_EINVAL;
    else if (np > 0 && !pp) want = OMB_EINVAL;
    const int got = build_scal(&err, k, M, id, pp, wp, ideal.get(), mx.get(), pick_d(), &sp);
    expect(got, want, "build_scal", err);
    if (got == OMB_OK) {
      ++g_calls;
      bool ok = sp.k == k && sp.id == id;
      for (int i = 0; i < k; ++i) ok = ok && sp.w[i] == (id == OMB_SCAL_APD && zero_w ? 1e-5 : w[i]);
      for (int i = k; i < OMB_MAX_OBJ; ++i) ok = ok && sp.w[i] == 0.0 && sp.range[i] == 0.0;
      for (int i = np; i < 4; ++i) ok = ok && sp.p[i] == 0.0;
      if (!ok && g_fail++ < 20) fprintf(stderr, "build_scal: block mismatch (k=%d id=%d)\n", k, id);
    }
  }
}

void fuzz_gp_and_sobol() {
  for (int it = 0; it < 20000; ++it) {
    std::string err;
    const int obj = pick({INT_MIN, -1, 0, 7, 8, INT_MAX}, 0, 7), kern = pick({-1, 0, 1, 2}, 0, 1);
    const int n = pick(kIntEdges, 1, 2000), d = pick(kIntEdges, 1, 300);
    const bool d_ok = d >= 1 && d <= OMB_MAX_DIM;
    const double lsv = next_u64() % 4 ? 0.7 : pick_d();
    auto ls = darr(d_ok ? d : 1, 0.5);
    const int bad_j = d_ok ? (int)(next_u64() % d) : 0;
    ls[bad_j] = lsv;
    double x = 0;
    const void* X = next_u64() % 7 ? &x : nullptr;
    const double var = next_u64() % 4 ? 1.0 : pick_d();
    int want = OMB_OK;
    if (obj < 0 || obj >= 8) want = OMB_EINVAL;
    else if (kern != 0 && kern != 1) want = OMB_EINVAL;
    else if (n < 1 || n > OMB_MAX_TRAIN_DENSE) want = OMB_EUNSUP;
    else if (!d_ok) want = OMB_EUNSUP;
    else if (!X) want = OMB_EINVAL;
    else if (!(lsv > 0.0)) want = OMB_EINVAL;
    else if (!(var >= 0.0)) want = OMB_EINVAL;
    expect(check_gp_args(&err, obj, kern, n, d, X, ls.get(), var, &x, &x), want, "check_gp_args", err);
    if (d_ok) expect(pad_dim(d) >= d && pad_dim(d) <= 256 ? OMB_OK : -99, OMB_OK, "pad_dim", "pad_dim out of range");

    // omb_set_sobol: the checks, then the packing into exactly sobol_state_bytes(d, bits) and its layout read back
    const int sd = pick({INT_MIN, 0, 1, 2, 6, 64, 255, 256, 257, INT_MAX}, 1, 256);
    const int bits = pick({INT_MIN, 0, 1, 30, 31, 32, 33, INT_MAX}, 1, 32);
    const bool sd_ok = sd >= 1 && sd <= OMB_MAX_DIM, bits_ok = bits >= 1 && bits <= 32;
    const int dd = sd_ok ? sd : 1;
    auto lo = darr(dd, 0.0), hi = darr(dd, 1.0);
    const bool empty_box = next_u64() % 6 == 0;
    if (empty_box) hi[dd - 1] = -1.0;
    std::vector<uint32_t> sv((size_t)dd * (bits_ok ? bits : 1)), shift(dd);
    for (auto& v : sv) v = (uint32_t)next_u64();
    for (auto& v : shift) v = (uint32_t)next_u64();
    int swant = OMB_OK;
    if (!sd_ok || !bits_ok) swant = OMB_EUNSUP;
    else if (empty_box) swant = OMB_EINVAL;
    err.clear();
    const int sgot = check_sobol_args(&err, sd, bits, sv.data(), shift.data(), lo.get(), hi.get());
    expect(sgot, swant, "check_sobol_args", err);
    if (sgot == OMB_OK && next_u64() % 8 == 0) {
      const size_t bytes = sobol_state_bytes(sd, bits);
      std::unique_ptr<unsigned char[]> buf(new unsigned char[bytes]);
      sobol_pack_state(sd, bits, sv.data(), shift.data(), lo.get(), hi.get(), buf.get());
      const uint32_t* w = reinterpret_cast<const uint32_t*>(buf.get());
      const int words = sd * bits + sd;
      const double* f = reinterpret_cast<const double*>(w + ((words + 1) & ~1));
      bool ok = memcmp(w, sv.data(), sizeof(uint32_t) * sd * bits) == 0 &&
                memcmp(w + sd * bits, shift.data(), sizeof(uint32_t) * sd) == 0;
      for (int t = 0; t < sd; ++t) ok = ok && f[t] == lo[t] && f[sd + t] == hi[t] - lo[t];
      ++g_calls;
      if (!ok && g_fail++ < 20) fprintf(stderr, "sobol_pack_state: layout mismatch (d=%d bits=%d)\n", sd, bits);
    }
  }
}

void long_messages() {
  std::string err;
  std::string big(2000, 'x');
  expect(errf(&err, OMB_EINVAL, "%s", big.c_str()), OMB_EINVAL, "errf", err);
  ++g_calls;
  if (err.size() != 511 && g_fail++ < 20) fprintf(stderr, "errf: message not truncated to the buffer\n");
  expect(errf(nullptr, OMB_EUNSUP, "no sink %d", 1), OMB_EUNSUP, "errf(null)", "sinkless");
}

}  // namespace

int main() {
  fuzz_moments();
  fuzz_acq_checks();
  fuzz_build_scal();
  fuzz_gp_and_sobol();
  long_messages();
  printf("omb_host_fuzz: %ld calls, %ld mismatches\n", g_calls, g_fail);
  return g_fail == 0 ? 0 : 1;
}
