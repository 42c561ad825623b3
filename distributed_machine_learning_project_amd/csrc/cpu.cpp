#include <cstdint>
// cpu.cpp — host implementations: exact brute-force k-NN, serial KD-tree (bench.debug analog),
// top-k merge, vote/checksum, report formatting and the multi-threaded input parser.
//
// These serve (a) the CPU world (no GPU), (b) the `serial` strategy
// (bench.debug B0: KD-tree @0xb890 build, @0xb040 search) and (c) the byte-exact oracle used by
// the tests.  Compiled with -ffp-contract=off and without -march flags, so x86-64 emits
// separate mulsd/addsd exactly as the reference's SSE2 code does (engine.cpp:12-18).
#include "dmlp.h"

#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <thread>
#include <unordered_map>
#include <string>
#include <vector>

namespace {

inline double exact_dist(const double* q, const double* x, int A) {
  double s = 0.0;
  for (int a = 0; a < A; ++a) {
    const double d = q[a] - x[a];
    s = s + d * d;
  }
  return s;
}

struct Key {
  double d;
  int id;
};
inline bool key_less(const Key& a, const Key& b) {
  return a.d < b.d || (a.d == b.d && a.id > b.id);
}

template <typename F>
void parallel_for(int64_t n, int nthreads, F&& f) {
  if (nthreads <= 1 || n < 2) {
    for (int64_t i = 0; i < n; ++i) f(i);
    return;
  }
  std::atomic<int64_t> next{0};
  const int64_t chunk = std::max<int64_t>(1, n / (nthreads * 8));
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t)
    th.emplace_back([&] {
      for (;;) {
        const int64_t b = next.fetch_add(chunk);
        if (b >= n) break;
        const int64_t e = std::min(n, b + chunk);
        for (int64_t i = b; i < e; ++i) f(i);
      }
    });
  for (auto& t : th) t.join();
}

int default_threads(int n) {
  if (n > 0) return n;
  const unsigned h = std::thread::hardware_concurrency();
  return h ? (int)std::min(h, 64u) : 1;
}

int vote(const int* ids, int k, const int* labels) {
  if (k <= 0) return -1;
  std::unordered_map<int, int> cnt;
  for (int i = 0; i < k; ++i)
    if (ids[i] >= 0) cnt[labels[ids[i]]]++;
  int best = -1, bc = 0;
  for (auto& kv : cnt)
    if (kv.second > bc || (kv.second == bc && kv.first > best)) {
      bc = kv.second;
      best = kv.first;
    }
  return best;
}

uint64_t fnv(int label, const int* ids, int k) {
  uint64_t h = 1469598103934665603ULL;
  h ^= (uint64_t)(int64_t)label;
  h *= 1099511628211ULL;
  for (int i = 0; i < k; ++i) {
    h ^= (uint64_t)(int64_t)(ids[i] + 1);
    h *= 1099511628211ULL;
  }
  return h;
}

// ---------------------------------------------------------------- KD-tree (bench.debug B0)
struct KdNode {
  int pt;     // point index
  int left;   // node index or -1
  int right;
  int axis;
};

struct KdTree {
  const double* X;
  int A;
  std::vector<KdNode> nodes;
  std::vector<int> idx;
  int root = -1;

  int build(int lo, int hi, int depth) {  // [lo, hi)
    if (lo >= hi) return -1;
    const int axis = depth % A;
    const int mid = lo + (hi - lo) / 2;
    std::nth_element(idx.begin() + lo, idx.begin() + mid, idx.begin() + hi, [&](int a, int b) {
      const double va = X[(int64_t)a * A + axis], vb = X[(int64_t)b * A + axis];
      return va < vb || (va == vb && a < b);
    });
    const int me = (int)nodes.size();
    nodes.push_back({idx[mid], -1, -1, axis});
    const int l = build(lo, mid, depth + 1);
    const int r = build(mid + 1, hi, depth + 1);
    nodes[me].left = l;
    nodes[me].right = r;
    return me;
  }

  // bounded max-heap of the k best keys (heap top = worst under key_less)
  void search(int n, const double* q, int k, std::vector<Key>& heap) const {
    if (n < 0) return;
    const KdNode& nd = nodes[n];
    const double* p = X + (int64_t)nd.pt * A;
    const Key cand{exact_dist(q, p, A), nd.pt};
    auto worse = [](const Key& a, const Key& b) { return key_less(a, b); };  // max-heap by key
    if ((int)heap.size() < k) {
      heap.push_back(cand);
      std::push_heap(heap.begin(), heap.end(), worse);
    } else if (k > 0 && key_less(cand, heap.front())) {
      std::pop_heap(heap.begin(), heap.end(), worse);
      heap.back() = cand;
      std::push_heap(heap.begin(), heap.end(), worse);
    }
    const double diff = q[nd.axis] - p[nd.axis];
    const int nearer = diff < 0 ? nd.left : nd.right;
    const int farther = diff < 0 ? nd.right : nd.left;
    search(nearer, q, k, heap);
    // any point across the split has (q_axis - x_axis)^2 >= diff^2 (monotone rounding), and the
    // full sequential sum is >= that term, so <= keeps exact ties reachable.
    const double lb = diff * diff;
    if ((int)heap.size() < k || (k > 0 && lb <= heap.front().d)) search(farther, q, k, heap);
  }
};

// ---------------------------------------------------------------- parsing helpers
inline const char* skip_ws(const char* p, const char* e) {
  while (p < e && (*p == ' ' || *p == '\t' || *p == '\r')) ++p;
  return p;
}

// strtod needs a NUL-terminated buffer: copy each token (<64 chars) into a small local buffer.
inline bool parse_double(const char*& p, const char* e, double& out) {
  p = skip_ws(p, e);
  char tmp[80];
  int n = 0;
  while (p < e && n < 79 && *p != ' ' && *p != '\t' && *p != '\n' && *p != '\r') tmp[n++] = *p++;
  if (n == 0) return false;
  tmp[n] = 0;
  char* end = nullptr;
  out = std::strtod(tmp, &end);
  return end == tmp + n;
}

inline bool parse_int(const char*& p, const char* e, int64_t& out) {
  p = skip_ws(p, e);
  bool neg = false;
  if (p < e && (*p == '-' || *p == '+')) { neg = *p == '-'; ++p; }
  if (p >= e || *p < '0' || *p > '9') return false;
  int64_t v = 0;
  while (p < e && *p >= '0' && *p <= '9') v = v * 10 + (*p++ - '0');
  out = neg ? -v : v;
  return true;
}

char* put_u64(char* o, uint64_t v) {
  char tmp[24];
  int n = 0;
  do { tmp[n++] = (char)('0' + v % 10); v /= 10; } while (v);
  while (n) *o++ = tmp[--n];
  return o;
}
char* put_i64(char* o, int64_t v) {
  if (v < 0) { *o++ = '-'; return put_u64(o, (uint64_t)(-(v + 1)) + 1); }
  return put_u64(o, (uint64_t)v);
}

}  // namespace

extern "C" int dmlp_cpu_knn(const double* X, int64_t N, int A, const double* Qx, int64_t Q,
                            const int* qk, int kstride, double* out_d, int* out_i, int nthreads) {
  nthreads = default_threads(nthreads);
  parallel_for(Q, nthreads, [&](int64_t q) {
    const int k = qk[q];
    std::vector<Key> keys((size_t)N);
    const double* qv = Qx + q * A;
    for (int64_t n = 0; n < N; ++n) keys[n] = Key{exact_dist(qv, X + n * A, A), (int)n};
    const int kk = (int)std::min<int64_t>(k, N);
    if (kk > 0) {
      std::partial_sort(keys.begin(), keys.begin() + kk, keys.end(), key_less);
    }
    for (int i = 0; i < k; ++i) {
      out_d[q * kstride + i] = i < kk ? keys[i].d : INFINITY;
      out_i[q * kstride + i] = i < kk ? keys[i].id : -1;
    }
  });
  return 0;
}

extern "C" int dmlp_cpu_finalize(const double* d, const int* ids, int kstride, const int* qk,
                                 int64_t Q, const int* labels, int* out_label, uint64_t* out_cs) {
  (void)d;
  for (int64_t q = 0; q < Q; ++q) {
    const int* iq = ids + q * kstride;
    const int lbl = vote(iq, qk[q], labels);
    out_label[q] = lbl;
    out_cs[q] = fnv(lbl, iq, qk[q]);
  }
  return 0;
}

extern "C" int dmlp_cpu_merge(const double* in_d, const int* in_i, int L, int64_t list_stride,
                              int kin, const int* qk, int64_t Q, double* out_d, int* out_i,
                              int kout) {
  std::vector<int> head(L);
  for (int64_t q = 0; q < Q; ++q) {
    const int k = qk[q];
    const int lim = std::min(k, kin);
    std::fill(head.begin(), head.end(), 0);
    for (int o = 0; o < k; ++o) {
      int best = -1;
      Key bk{INFINITY, -1};
      for (int l = 0; l < L; ++l) {
        if (head[l] >= lim) continue;
        const int64_t off = l * list_stride + q * kin + head[l];
        if (in_i[off] < 0) continue;
        const Key c{in_d[off], in_i[off]};
        if (best < 0 || key_less(c, bk)) { best = l; bk = c; }
      }
      if (best >= 0) head[best]++;
      out_d[q * kout + o] = bk.d;
      out_i[q * kout + o] = bk.id;
    }
  }
  return 0;
}

extern "C" int dmlp_kdtree_knn(const double* X, int64_t N, int A, const double* Qx, int64_t Q,
                               const int* qk, int kstride, double* out_d, int* out_i) {
  KdTree t;
  t.X = X;
  t.A = A;
  t.idx.resize((size_t)N);
  std::iota(t.idx.begin(), t.idx.end(), 0);
  t.nodes.reserve((size_t)N);
  t.root = t.build(0, (int)N, 0);
  std::vector<Key> heap;
  for (int64_t q = 0; q < Q; ++q) {
    const int k = qk[q];
    heap.clear();
    heap.reserve(k > 0 ? k : 1);
    t.search(t.root, Qx + q * A, k, heap);
    std::sort(heap.begin(), heap.end(), key_less);
    for (int i = 0; i < k; ++i) {
      out_d[q * kstride + i] = i < (int)heap.size() ? heap[i].d : INFINITY;
      out_i[q * kstride + i] = i < (int)heap.size() ? heap[i].id : -1;
    }
  }
  return 0;
}

extern "C" int64_t dmlp_cpu_format_report(const uint64_t* cs, int64_t Q, int64_t qid_base,
                                          char* out) {
  char* o = out;
  for (int64_t q = 0; q < Q; ++q) {
    std::memcpy(o, "Query ", 6); o += 6;
    o = put_i64(o, qid_base + q);
    std::memcpy(o, " checksum: ", 11); o += 11;
    o = put_u64(o, cs[q]);
    *o++ = '\n';
  }
  return o - out;
}

// DEBUG-build report (common.cpp:72-78): distances printed like `std::cout << double`
// (default precision 6, %g style).
extern "C" int64_t dmlp_cpu_format_debug(const double* d, const int* ids, int kstride,
                                         const int* qk, const int* labels_pred, int64_t Q,
                                         char* out, int64_t cap) {
  int64_t o = 0;
  char line[128];
  for (int64_t q = 0; q < Q; ++q) {
    int n = std::snprintf(line, sizeof line, "Label for Query %lld : %d\nTop-%d neighbors:\n",
                          (long long)q, labels_pred[q], qk[q]);
    if (o + n >= cap) return -1;
    std::memcpy(out + o, line, n); o += n;
    for (int i = 0; i < qk[q]; ++i) {
      n = std::snprintf(line, sizeof line, "%d : %g\n", ids[q * kstride + i], d[q * kstride + i]);
      if (o + n >= cap) return -1;
      std::memcpy(out + o, line, n); o += n;
    }
  }
  return o;
}

extern "C" int dmlp_parse_header(const char* buf, int64_t len, int64_t* N, int64_t* Q, int* A,
                                 int64_t* body_off) {
  const char* p = buf;
  const char* e = buf + len;
  const char* nl = (const char*)std::memchr(p, '\n', (size_t)len);
  const char* le = nl ? nl : e;
  int64_t n, q, a;
  if (!parse_int(p, le, n) || !parse_int(p, le, q) || !parse_int(p, le, a)) return -1;
  *N = n; *Q = q; *A = (int)a;
  *body_off = nl ? (nl - buf) + 1 : len;
  return 0;
}

extern "C" int64_t dmlp_parse_body(const char* buf, int64_t len, int64_t body_off, int64_t N,
                                   int64_t Q, int A, int* labels, double* X, int* qk, double* Qx,
                                   int nthreads) {
  // line starts
  const int64_t L = N + Q;
  std::vector<int64_t> starts((size_t)L + 1);
  int64_t pos = body_off;
  for (int64_t i = 0; i < L; ++i) {
    if (pos >= len) return -(i + 1);
    starts[i] = pos;
    const char* nl = (const char*)std::memchr(buf + pos, '\n', (size_t)(len - pos));
    pos = nl ? (nl - buf) + 1 : len;
  }
  starts[L] = pos;
  std::atomic<int64_t> bad{0};
  nthreads = default_threads(nthreads);
  parallel_for(L, nthreads, [&](int64_t i) {
    const char* p = buf + starts[i];
    const char* e = buf + starts[i + 1];
    if (e > p && e[-1] == '\n') --e;
    bool ok = true;
    int64_t iv = 0;
    if (i < N) {
      ok = parse_int(p, e, iv);
      labels[i] = (int)iv;
      for (int a = 0; ok && a < A; ++a) ok = parse_double(p, e, X[i * A + a]);
    } else {
      const int64_t qi = i - N;
      p = skip_ws(p, e);
      if (p >= e || *p != 'Q') ok = false;
      else ++p;
      ok = ok && parse_int(p, e, iv);
      qk[qi] = (int)iv;
      for (int a = 0; ok && a < A; ++a) ok = parse_double(p, e, Qx[qi * A + a]);
    }
    if (!ok) {
      int64_t cur = bad.load();
      while ((cur == 0 || i + 1 < cur) && !bad.compare_exchange_weak(cur, i + 1)) {}
    }
  });
  const int64_t b = bad.load();
  return b ? -b : 0;
}

// [min, max] of an int32 array in one pass (the label range and k bounds every KNN call scans:
// engine.cpp:27-35 broadcasts the sizes, the vote needs the label range).  n == 0: lo > hi.
__attribute__((target("avx2"))) static void i32_range_avx2(const int* a, int64_t n, int* lo,
                                                           int* hi);
extern "C" void dmlp_cpu_i32_range(const int* a, int64_t n, int* lo, int* hi) {
  static const bool avx2 = __builtin_cpu_supports("avx2");
  if (avx2) return i32_range_avx2(a, n, lo, hi);
  int mn = INT32_MAX, mx = INT32_MIN;
  int64_t i = 0;
  int m4[8], x4[8];
  for (int j = 0; j < 8; ++j) { m4[j] = INT32_MAX; x4[j] = INT32_MIN; }
  for (; i + 8 <= n; i += 8)  // 8 independent lanes: vectorised by the compiler
    for (int j = 0; j < 8; ++j) {
      m4[j] = a[i + j] < m4[j] ? a[i + j] : m4[j];
      x4[j] = a[i + j] > x4[j] ? a[i + j] : x4[j];
    }
  for (int j = 0; j < 8; ++j) { mn = m4[j] < mn ? m4[j] : mn; mx = x4[j] > mx ? x4[j] : mx; }
  for (; i < n; ++i) { mn = a[i] < mn ? a[i] : mn; mx = a[i] > mx ? a[i] : mx; }
  *lo = mn;
  *hi = mx;
}

__attribute__((target("avx2"))) static void i32_range_avx2(const int* a, int64_t n, int* lo,
                                                           int* hi) {
  // four independent min/max chains of 8 lanes (32 ints per iteration): load-bound
  __m256i mn0 = _mm256_set1_epi32(INT32_MAX), mn1 = mn0, mn2 = mn0, mn3 = mn0;
  __m256i mx0 = _mm256_set1_epi32(INT32_MIN), mx1 = mx0, mx2 = mx0, mx3 = mx0;
  int64_t i = 0;
  for (; i + 32 <= n; i += 32) {
    const __m256i v0 = _mm256_loadu_si256((const __m256i*)(a + i));
    const __m256i v1 = _mm256_loadu_si256((const __m256i*)(a + i + 8));
    const __m256i v2 = _mm256_loadu_si256((const __m256i*)(a + i + 16));
    const __m256i v3 = _mm256_loadu_si256((const __m256i*)(a + i + 24));
    mn0 = _mm256_min_epi32(mn0, v0); mx0 = _mm256_max_epi32(mx0, v0);
    mn1 = _mm256_min_epi32(mn1, v1); mx1 = _mm256_max_epi32(mx1, v1);
    mn2 = _mm256_min_epi32(mn2, v2); mx2 = _mm256_max_epi32(mx2, v2);
    mn3 = _mm256_min_epi32(mn3, v3); mx3 = _mm256_max_epi32(mx3, v3);
  }
  mn0 = _mm256_min_epi32(_mm256_min_epi32(mn0, mn1), _mm256_min_epi32(mn2, mn3));
  mx0 = _mm256_max_epi32(_mm256_max_epi32(mx0, mx1), _mm256_max_epi32(mx2, mx3));
  alignas(32) int m8[8], x8[8];
  _mm256_store_si256((__m256i*)m8, mn0);
  _mm256_store_si256((__m256i*)x8, mx0);
  int mn = INT32_MAX, mx = INT32_MIN;
  for (int j = 0; j < 8; ++j) { mn = m8[j] < mn ? m8[j] : mn; mx = x8[j] > mx ? x8[j] : mx; }
  for (; i < n; ++i) { mn = a[i] < mn ? a[i] : mn; mx = a[i] > mx ? a[i] : mx; }
  *lo = mn;
  *hi = mx;
}

extern "C" const char* dmlp_version(void) { return "dmlp 0.1.0 (gfx950)"; }

// Sequentially consistent fetch-and-add on a 64-bit word that several processes map (the
// node-shared segment's work counter, utils/shm.py): the dynamic farm's chunk claim.
extern "C" int64_t dmlp_atomic_fetch_add_i64(int64_t* p, int64_t v) {
  return __atomic_fetch_add(p, v, __ATOMIC_SEQ_CST);
}
extern "C" void dmlp_atomic_store_i64(int64_t* p, int64_t v) { __atomic_store_n(p, v, __ATOMIC_SEQ_CST); }

// The input file of the reference's format (generate_input.py:6-23: "<N> <Q> <A>", then
// "<label> <a_0> ... <a_{A-1}>" per point and "Q <k> <a_0> ..." per query, attributes "%.6f") for
// arrays in memory — bench.py's reference-contract runs write hundreds of MB of it, formatted on
// the render pool in row ranges and written in order.  0, or -1 when the file cannot be written.
extern "C" int dmlp_cpu_write_input(const char* path, const int* labels, const double* X,
                                    int64_t N, const int* k, const double* Qx, int64_t Q, int A) {
  FILE* f = std::fopen(path, "wb");
  if (!f) return -1;
  std::fprintf(f, "%lld %lld %d\n", (long long)N, (long long)Q, A);
  const int64_t rows = N + Q, block = 1 << 14;
  int rc = 0;
  std::vector<std::string> part;
  for (int64_t b0 = 0; b0 < rows && rc == 0; b0 += block * 64) {
    const int64_t b1 = std::min(rows, b0 + block * 64);
    const int64_t nb = (b1 - b0 + block - 1) / block;
    part.assign(nb, std::string());
    struct Job {
      std::vector<std::string>* part;
      int64_t b0, b1, block, N;
      int A;
      const int *labels, *k;
      const double *X, *Qx;
    } j{&part, b0, b1, block, N, A, labels, k, X, Qx};
    dmlp_host_pool_run([](void* c, int t, int nt) {
      Job& J = *(Job*)c;
      char buf[64];
      for (int64_t p = t; p < (int64_t)J.part->size(); p += nt) {
        std::string& s = (*J.part)[p];
        s.reserve((size_t)J.block * (J.A * 12 + 16));
        const int64_t r0 = J.b0 + p * J.block, r1 = std::min(J.b1, r0 + J.block);
        for (int64_t r = r0; r < r1; ++r) {
          const bool q = r >= J.N;
          const double* row = q ? J.Qx + (r - J.N) * J.A : J.X + r * J.A;
          int n = q ? std::snprintf(buf, sizeof buf, "Q %d", J.k[r - J.N])
                    : std::snprintf(buf, sizeof buf, "%d", J.labels[r]);
          s.append(buf, (size_t)n);
          for (int a = 0; a < J.A; ++a) {
            n = std::snprintf(buf, sizeof buf, " %.6f", row[a]);
            if (n >= (int)sizeof buf) {  // (a huge value: its own buffer)
              std::vector<char> big((size_t)n + 1);
              std::snprintf(big.data(), big.size(), " %.6f", row[a]);
              s.append(big.data(), (size_t)n);
            } else {
              s.append(buf, (size_t)n);
            }
          }
          s.push_back('\n');
        }
      }
    }, &j);
    for (const std::string& s : part)
      if (std::fwrite(s.data(), 1, s.size(), f) != s.size()) rc = -1;
  }
  if (std::fclose(f) != 0) rc = -1;
  return rc;
}
