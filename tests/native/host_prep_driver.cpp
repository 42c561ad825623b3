// ThreadSanitizer driver for csrc/host_prep.cpp: the persistent worker pool
// (generation counter, spin-then-condvar sleep, pending_ countdown) and the host conversions
// that run on it inside every bench step.  The HIP half of the pipeline (dmlp_host_ops_h2d in
// prep.hip) is reproduced with its copies stubbed by memcpy into "device" buffers, chunk by
// chunk exactly as it issues them.  Checks, besides TSan's own reports:
//   * chunked tile rendering == one-shot rendering, byte for byte (no lost or torn part);
//   * every job gives identical bytes when repeated back to back (the spin path) and after the
//     workers went to sleep (the condvar path);
//   * the queries' operands match a serial scalar recomputation of the documented rounding.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "dmlp.h"

static int fails = 0;
#define EXPECT(c)                                                         \
  do {                                                                    \
    if (!(c)) {                                                           \
      std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c);    \
      ++fails;                                                            \
    }                                                                     \
  } while (0)

// fp32 -> fp16 bits, round to nearest even, by arithmetic (independent of host_prep.cpp's
// bit manipulation and of F16C): the fp16 grid spacing at |f| is 2^(e - 10) for normal values
// (2^-24 below 2^-14), rounding is done on the exact double quotient with nearbyint (ties to even).
static uint16_t f16_rn_ref(float f) {
  const double a = std::fabs((double)f);
  const uint16_t sign = std::signbit(f) ? 0x8000 : 0;
  if (a == 0.0) return sign;
  int e;
  std::frexp(a, &e);  // a = m 2^e, m in [0.5, 1)
  const int ex = std::max(e - 1, -14);            // unbiased exponent of the fp16 binade
  const double step = std::ldexp(1.0, ex - 10);   // spacing of the fp16 grid there
  double m = std::nearbyint(a / step);            // exact quotient, rounded half to even
  int bex = ex;
  if (m >= 2048.0) { m /= 2.0; ++bex; }           // rounded up into the next binade
  if (m < 1024.0) return (uint16_t)(sign | (uint16_t)m);  // subnormal (bex == -14)
  return (uint16_t)(sign | (uint16_t)((bex + 15) << 10) | (uint16_t)(m - 1024.0));
}

struct Ops {
  std::vector<uint16_t> xhi, qhi;
  std::vector<float> xin, qn;
  unsigned xnm = 0;
};

// dmlp_host_ops_h2d's sequence with memcpy as the copy engine
static int host_ops_stub(const std::vector<double>& X, int64_t N, const std::vector<double>& Qx,
                         int64_t Q, int A, const std::vector<double>& mu, int KT, int chunks,
                         Ops& dev) {
  const int64_t n_tiles = (N + 63) / 64, W = (int64_t)KT * 32;
  std::vector<uint16_t> xhi_h(n_tiles * 64 * W), qhi_h(Q * W);
  std::vector<float> xin_h(n_tiles * 64), qn_h(Q);
  dev.xhi.assign(xhi_h.size(), 0xdead);
  dev.xin.assign(xin_h.size(), -1.0f);
  dev.qhi.assign(qhi_h.size(), 0xdead);
  dev.qn.assign(qn_h.size(), -1.0f);
  int rc = 0;
  float m = 0.0f;
  for (int c = 0; c < chunks; ++c) {
    const int64_t t0 = n_tiles * c / chunks, t1 = n_tiles * (c + 1) / chunks;
    if (t1 <= t0) continue;
    float mc = 0.0f;
    if (dmlp_cpu_prep_data_tiles(X.data(), N, A, mu.data(), KT, t0, t1, xhi_h.data(),
                                 xin_h.data(), &mc))
      rc |= 1;
    m = mc > m ? mc : m;
    std::memcpy(dev.xhi.data() + t0 * 64 * W, xhi_h.data() + t0 * 64 * W, (t1 - t0) * 64 * W * 2);
    std::memcpy(dev.xin.data() + t0 * 64, xin_h.data() + t0 * 64, (t1 - t0) * 64 * 4);
  }
  std::memcpy(&dev.xnm, &m, 4);
  for (int c = 0; c < chunks; ++c) {
    const int64_t q0 = Q * c / chunks, q1 = Q * (c + 1) / chunks;
    if (q1 <= q0) continue;
    if (dmlp_cpu_prep_queries(Qx.data() + q0 * A, q1 - q0, A, mu.data(), KT, qhi_h.data() + q0 * W,
                              qn_h.data() + q0))
      rc |= 2;
    std::memcpy(dev.qhi.data() + q0 * W, qhi_h.data() + q0 * W, (q1 - q0) * W * 2);
    std::memcpy(dev.qn.data() + q0, qn_h.data() + q0, (q1 - q0) * 4);
  }
  return rc;
}

static bool same(const Ops& a, const Ops& b) {
  return a.xhi == b.xhi && a.xin == b.xin && a.qhi == b.qhi && a.qn == b.qn && a.xnm == b.xnm;
}

int main() {
  std::mt19937_64 rng(5);
  std::uniform_real_distribution<double> U(0.0, 1000.0);
  const int shapes[][3] = {{1, 1, 1}, {63, 7, 5}, {64, 64, 32}, {1000, 333, 17}, {5000, 1200, 64},
                           {4097, 65, 32}};
  for (const auto& sh : shapes) {
    const int64_t N = sh[0], Q = sh[1];
    const int A = sh[2], KT = (A + 31) / 32;
    std::vector<double> X(N * A), Qx(Q * A), mu(A);
    for (auto& v : X) v = std::round(U(rng) * 1e6) / 1e6;
    for (auto& v : Qx) v = std::round(U(rng) * 1e6) / 1e6;
    dmlp_cpu_center(X.data(), N, A, mu.data());
    Ops one, many, again, slept;
    EXPECT(host_ops_stub(X, N, Qx, Q, A, mu, KT, 1, one) == 0);
    EXPECT(host_ops_stub(X, N, Qx, Q, A, mu, KT, 5, many) == 0);
    EXPECT(host_ops_stub(X, N, Qx, Q, A, mu, KT, 1, again) == 0);  // back to back: spin path
    std::this_thread::sleep_for(std::chrono::milliseconds(30));      // workers fall asleep
    EXPECT(host_ops_stub(X, N, Qx, Q, A, mu, KT, 3, slept) == 0);
    EXPECT(same(one, many));
    EXPECT(same(one, again));
    EXPECT(same(one, slept));
    // queries: serial recomputation of the documented rounding (c = q - mu in fp64,
    // hi = fp16_rn(fp32(c)), |c|^2 accumulated in fp64 and rounded to fp32 once)
    for (int64_t q = 0; q < Q; ++q) {
      for (int a = 0; a < KT * 32; ++a) {
        const uint16_t want = a < A ? f16_rn_ref((float)(Qx[q * A + a] - mu[a])) : 0;
        if (one.qhi[q * KT * 32 + a] != want) { EXPECT(one.qhi[q * KT * 32 + a] == want); break; }
      }
      EXPECT(std::isfinite(one.qn[q]) && one.qn[q] >= 0.0f);
    }
    // center: the mean of the first min(N, 4096) rows
    std::vector<double> m2(A, 0.0);
    const int64_t nc = N < 4096 ? N : 4096;
    for (int64_t i = 0; i < nc; ++i)
      for (int a = 0; a < A; ++a) m2[a] += X[i * A + a];
    for (int a = 0; a < A; ++a) EXPECT(std::fabs(m2[a] / nc - mu[a]) <= 1e-9 * (1.0 + std::fabs(mu[a])));
  }
  // out-of-range data is reported, not converted silently
  {
    std::vector<double> X(64 * 4, 1.0), Qx(4 * 4, 1.0), mu(4, 0.0);
    X[5] = 1e16;
    Ops o;
    EXPECT((host_ops_stub(X, 64, Qx, 4, 4, mu, 1, 2, o) & 1) == 1);
  }
  std::printf("host prep driver: %s (%d pool threads)\n", fails ? "FAILED" : "OK",
              dmlp_host_threads());
  return fails ? 1 : 0;
}
