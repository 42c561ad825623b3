// Host-code sanitizer driver: exercises every CPU entry point of libdmlp (parser, brute force,
// KD-tree, merge, vote/checksum, formatters) on adversarial inputs — ties, k > N, k = 0, empty
// shards — so an ASan/UBSan build of csrc/cpu.cpp can catch memory and UB errors
// (SURVEY.md §5 "race detection / sanitizers": host code only; GPU sanitizers are unavailable).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "dmlp.h"

static int fails = 0;
#define EXPECT(c)                                                  \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                                     \
    }                                                              \
  } while (0)

int main() {
  // ---- parser: a small input with duplicate points and k > N
  std::string txt = "6 4 3\n";
  const double pts[6][3] = {{0, 0, 0}, {1, 1, 1}, {1, 1, 1}, {2, 2, 2}, {-1, 0.5, 3}, {1, 1, 1}};
  const int lab[6] = {0, 1, 2, 1, 0, 2};
  char line[256];
  for (int i = 0; i < 6; ++i) {
    std::snprintf(line, sizeof line, "%d %.6f %.6f %.6f\n", lab[i], pts[i][0], pts[i][1], pts[i][2]);
    txt += line;
  }
  const int qk[4] = {3, 9, 0, 6};
  const double qp[4] = {1, 0, 5, 1.5};
  for (int i = 0; i < 4; ++i) {
    std::snprintf(line, sizeof line, "Q %d %.6f %.6f %.6f\n", qk[i], qp[i], qp[i], qp[i]);
    txt += line;
  }
  int64_t N, Q, body;
  int A;
  EXPECT(dmlp_parse_header(txt.data(), txt.size(), &N, &Q, &A, &body) == 0);
  EXPECT(N == 6 && Q == 4 && A == 3);
  std::vector<int> labels(N), k(Q);
  std::vector<double> X(N * A), Qx(Q * A);
  EXPECT(dmlp_parse_body(txt.data(), txt.size(), body, N, Q, A, labels.data(), X.data(), k.data(),
                         Qx.data(), 3) == 0);
  EXPECT(k[1] == 9 && labels[5] == 2);
  // ---- the pool-formatted input writer reproduces the text byte for byte
  {
    const char* wp = "/tmp/dmlp_host_driver_input.txt";
    EXPECT(dmlp_cpu_write_input(wp, labels.data(), X.data(), N, k.data(), Qx.data(), Q, A) == 0);
    std::FILE* f = std::fopen(wp, "rb");
    std::string back;
    if (f) {
      char buf[4096];
      size_t n;
      while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) back.append(buf, n);
      std::fclose(f);
    }
    std::remove(wp);
    EXPECT(back == txt);
  }
  const std::string bad = "2 1 2\n0 1 2\n1 x 2\nQ 1 0 0\n";
  int64_t bN, bQ, bb;
  int bA;
  EXPECT(dmlp_parse_header(bad.data(), bad.size(), &bN, &bQ, &bA, &bb) == 0);
  std::vector<int> bl(2), bk(1);
  std::vector<double> bX(4), bQx(2);
  EXPECT(dmlp_parse_body(bad.data(), bad.size(), bb, bN, bQ, bA, bl.data(), bX.data(), bk.data(),
                         bQx.data(), 2) < 0);

  // ---- brute force vs KD-tree, kstride = kmax = 9 (k > N pads with (+inf, -1))
  const int ks = 9;
  std::vector<double> d1(Q * ks, INFINITY), d2(Q * ks, INFINITY);
  std::vector<int> i1(Q * ks, -1), i2(Q * ks, -1);
  EXPECT(dmlp_cpu_knn(X.data(), N, A, Qx.data(), Q, k.data(), ks, d1.data(), i1.data(), 4) == 0);
  EXPECT(dmlp_kdtree_knn(X.data(), N, A, Qx.data(), Q, k.data(), ks, d2.data(), i2.data()) == 0);
  EXPECT(std::memcmp(i1.data(), i2.data(), i1.size() * 4) == 0);
  // query 0 = (1,1,1): ties at distance 0 -> ids 5, 2, 1 (id descending)
  EXPECT(i1[0] == 5 && i1[1] == 2 && i1[2] == 1);

  // ---- merge two shards (second shard ids offset by 3)
  std::vector<double> sd(2 * Q * ks, INFINITY), md(Q * ks);
  std::vector<int> si(2 * Q * ks, -1), mi(Q * ks);
  EXPECT(dmlp_cpu_knn(X.data(), 3, A, Qx.data(), Q, k.data(), ks, sd.data(), si.data(), 2) == 0);
  EXPECT(dmlp_cpu_knn(X.data() + 3 * A, 3, A, Qx.data(), Q, k.data(), ks, sd.data() + Q * ks,
                      si.data() + Q * ks, 2) == 0);
  for (int64_t j = Q * ks; j < 2 * Q * ks; ++j)
    if (si[j] >= 0) si[j] += 3;
  EXPECT(dmlp_cpu_merge(sd.data(), si.data(), 2, Q * ks, ks, k.data(), Q, md.data(), mi.data(), ks) == 0);
  for (int64_t q = 0; q < Q; ++q)
    for (int j = 0; j < std::min<int>(k[q], (int)N); ++j) EXPECT(mi[q * ks + j] == i1[q * ks + j]);

  // ---- vote + checksum + formatters
  std::vector<int> pl(Q);
  std::vector<uint64_t> cs(Q);
  EXPECT(dmlp_cpu_finalize(d1.data(), i1.data(), ks, k.data(), Q, labels.data(), pl.data(), cs.data()) == 0);
  EXPECT(pl[2] == -1);  // k = 0: empty vote
  std::vector<char> rep(48 * Q + 64);
  const int64_t n = dmlp_cpu_format_report(cs.data(), Q, 0, rep.data());
  EXPECT(n > 0 && std::strncmp(rep.data(), "Query 0 checksum: ", 18) == 0);
  std::vector<char> dbg(4096);
  EXPECT(dmlp_cpu_format_debug(d1.data(), i1.data(), ks, k.data(), pl.data(), Q, dbg.data(),
                               (int64_t)dbg.size()) > 0);

  // ---- larger random case: brute force == KD-tree, many threads
  const int64_t N2 = 3000, Q2 = 200;
  const int A2 = 5, ks2 = 40;
  std::vector<double> X2(N2 * A2), Q2x(Q2 * A2);
  std::vector<int> k2(Q2);
  unsigned s = 12345;
  auto rnd = [&]() { s = s * 1103515245u + 12345u; return (double)((s >> 8) % 1000) / 10.0; };
  for (auto& v : X2) v = rnd();
  for (auto& v : Q2x) v = rnd();
  for (auto& v : k2) v = 1 + (int)(rnd() * 10) % ks2;
  std::vector<double> e1(Q2 * ks2), e2(Q2 * ks2);
  std::vector<int> j1(Q2 * ks2), j2(Q2 * ks2);
  EXPECT(dmlp_cpu_knn(X2.data(), N2, A2, Q2x.data(), Q2, k2.data(), ks2, e1.data(), j1.data(), 8) == 0);
  EXPECT(dmlp_kdtree_knn(X2.data(), N2, A2, Q2x.data(), Q2, k2.data(), ks2, e2.data(), j2.data()) == 0);
  for (int64_t q = 0; q < Q2; ++q)
    for (int j = 0; j < k2[q]; ++j) EXPECT(j1[q * ks2 + j] == j2[q * ks2 + j]);

  std::printf("host driver: %s (%d failures)\n", fails ? "FAIL" : "OK", fails);
  return fails ? 1 : 0;
}
