// host_prep.cpp — query preparation on the host, run while the dataset is still crossing PCIe.
//
// The single-term screen reads only bf16(q - mu) and |q - mu|^2 of each query; the fp64 query
// rows are needed later, by the exact re-rank.  Rendering the screen operands here (8.4 MB for
// the bench shape instead of the 33.5 MB of fp64 rows) lets the screen start once the dataset and
// these operands have landed, with the fp64 queries copied behind the screen.  mu is the mean of
// the first min(N, 4096) rows, exactly the rows k_center (prep.hip) uses.
//
// The host render is the fp16 single-term image (hl = 1 for dmlp_screen_x1 / dmlp_refine_groups):
// c = q - mu in fp64; hi = fp16_rn(fp32_rn(c)) — 11 significant bits where bf16 has 8, so the
// single-term error bound is 4x tighter and fewer groups reach the re-rank; |c| >= 65504 (the
// fp16 range) or NaN flags the input as outside the screen's range (the caller then takes the
// device path, whose bf16 hi/lo image covers any finite data below 1e15).
#include "dmlp.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include <immintrin.h>
#include <sched.h>

namespace {

constexpr double kMaxAbs = 65504.0;  // the largest finite fp16
constexpr int kMaxPool = 16;  // pool size cap; also sizes the per-part scratch of the data prep

// pause iterations a worker spins after a job before it sleeps (DMLP_POOL_SPIN; default 100000,
// ~2 ms, so one rank's workers are still awake when its next call's render starts instead of
// paying a futex wake each step — the pool size leaves CPU quota for that, see pool_threads;
// 40000 with several ranks per node, whose pools share the cores)
int spin_budget() {
  static const int v = [] {
    const char* e = std::getenv("DMLP_POOL_SPIN");
    if (e) return std::max(0, std::atoi(e));
    // several ranks on the node (their pools share the cores): the shorter round-1 spin
    for (const char* v : {"LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_SIZE", "MPI_LOCALNRANKS"})
      if (const char* l = std::getenv(v)) return std::atoi(l) > 1 ? 40000 : 100000;
    return 100000;
  }();
  return v;
}

// Persistent workers: a per-call std::thread spawn (tens of microseconds each) would cost more
// than the conversion itself.  After a job a worker spins (spin_budget) on the generation
// counter before it sleeps on the condition variable, so back-to-back jobs (the chunked host-ops
// pipeline dispatches one per PCIe slice, and the next call's follow within a step) start in
// about a microsecond instead of a futex wake.
class Pool {
 public:
  // The worker count is fixed before any worker starts: workers read it (size(),
  // oversubscribed()) while the constructor is still spawning — reading th_.size() there raced
  // with the vector's growth (found by the TSan driver, tests/native/host_prep_driver.cpp).
  explicit Pool(int n) : n_(n > 0 ? n : 0) {
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) cpus_ = std::max(1, (int)CPU_COUNT(&set));
    th_.reserve(n_);
    for (int t = 0; t < n_; ++t) th_.emplace_back([this, t] { loop(t); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
      gen_.fetch_add(1);
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() const { return n_ + 1; }
  // f(part, parts) on every worker and the caller; returns when all parts are done
  void run(const std::function<void(int, int)>& f) {
    const int parts = size();
    job_ = &f;
    pending_.store(parts - 1, std::memory_order_relaxed);
    gen_.fetch_add(1);  // seq_cst: a worker either sees it or is counted in sleepers_
    if (sleepers_.load() > 0) {
      { std::lock_guard<std::mutex> g(m_); }
      cv_.notify_all();
    }
    f(parts - 1, parts);
    for (int spin = 0; pending_.load(std::memory_order_acquire) != 0; ++spin) {
      if (spin < 4096) _mm_pause();
      else std::this_thread::yield();  // a preempted worker: give it the CPU
    }
  }

 private:
  bool oversubscribed() const { return n_ + 1 > cpus_; }
  void loop(int t) {
    uint64_t seen = 0;  // gen_ starts at 0: a job dispatched before this thread ran is not missed
    for (;;) {
      uint64_t g = gen_.load(std::memory_order_acquire);
      // spin only while the pool fits the CPUs it may use: oversubscribed workers would burn
      // the time slices of the threads they wait for
      const int spins = oversubscribed() ? 0 : spin_budget();
      for (int spin = 0; g == seen && spin < spins; ++spin) {
        _mm_pause();
        g = gen_.load(std::memory_order_acquire);
      }
      if (g == seen) {
        std::unique_lock<std::mutex> lk(m_);
        sleepers_.fetch_add(1);
        cv_.wait(lk, [&] { return gen_.load() != seen; });
        sleepers_.fetch_sub(1);
        g = gen_.load();
      }
      seen = g;
      if (stop_) return;
      (*job_)(t, size());
      pending_.fetch_sub(1, std::memory_order_release);
    }
  }
  const int n_;
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_;
  std::atomic<uint64_t> gen_{0};
  std::atomic<int> sleepers_{0};
  std::atomic<bool> stop_{false};
  const std::function<void(int, int)>* job_ = nullptr;
  std::atomic<int> pending_{0};
  int cpus_ = 1 << 30;
};

// CPUs this process may run on (the affinity mask, not the machine: a GPU box grants each job a
// share of a 256-thread host), divided among the ranks of the node that share that mask
// (DMLP_NODE_RANKS / LOCAL_WORLD_SIZE, set by the NUMA binding / torchrun / the MPI launchers), at most 16 — the conversions are bound
// by memory, not cores.  DMLP_HOST_THREADS overrides (clamped to [1, 16]).
// CPUs' worth of time the cgroup grants (cgroup v2 cpu.max "quota period"; 0 = unlimited or
// unknown).  A container can see a 256-CPU affinity mask with a 16-CPU quota: sizing the pool by
// the mask alone would let spinning workers run the quota out and get the whole process throttled.
int cgroup_cpus() {
  FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r");
  if (!f) return 0;
  char quota[32] = {0};
  long period = 0;
  const int got = std::fscanf(f, "%31s %ld", quota, &period);
  std::fclose(f);
  if (got != 2 || period <= 0 || std::strcmp(quota, "max") == 0) return 0;
  const long q = std::atol(quota);
  return q > 0 ? (int)std::max(1L, q / period) : 0;
}

int pool_threads() {
  if (const char* e = std::getenv("DMLP_HOST_THREADS"))
    return std::max(1, std::min(std::atoi(e), kMaxPool));
  cpu_set_t set;
  int n = 0;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) n = CPU_COUNT(&set);
  if (n <= 0) n = (int)std::thread::hardware_concurrency();
  int local = 1;
  for (const char* v : {"LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_SIZE", "MPI_LOCALNRANKS"})
    if (const char* e = std::getenv(v)) { local = std::max(1, std::atoi(e)); break; }
  // ranks pinned to disjoint CPU sets see only their own share; a shared mask is split among the
  // ranks that share it: those bound to this NUMA node (DMLP_NODE_RANKS, set by the NUMA binding:
  // parallel/comm.py, engine_runtime.h), else every local rank
  int sharing = local;
  if (const char* e = std::getenv("DMLP_NODE_RANKS")) sharing = std::max(1, std::atoi(e));
  if (sharing > 1 && n >= 2 * sharing) n /= sharing;
  // the cgroup quota is shared by the node's ranks too; leave 2 CPUs of each rank's share to
  // its main thread and the HIP runtime, so spinning workers never run the quota out
  if (const int c = cgroup_cpus()) {
    const int share = std::max(1, c / local);
    n = std::min(n, share > 4 ? share - 2 : share);
  }
  return std::max(1, std::min(n, kMaxPool));
}

Pool& pool() {
  static Pool p(pool_threads() - 1);
  return p;
}

// fp32 -> fp16, round to nearest even, subnormals included (|f| < 65504 by the range check;
// the same bits as F16C's vcvtps2ph with _MM_FROUND_TO_NEAREST_INT).
inline uint16_t f16_rn(float f) {
  uint32_t x;
  std::memcpy(&x, &f, 4);
  const uint32_t sign = (x >> 16) & 0x8000u, ax = x & 0x7fffffffu;
  if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);  // >= 65520: inf (flagged anyway)
  if (ax < 0x38800000u) {                                    // < 2^-14: fp16 subnormal or zero
    float af;
    std::memcpy(&af, &ax, 4);
    // af * 2^24 is exact; nearbyint rounds half to even in the default rounding mode
    return (uint16_t)(sign | (uint32_t)std::nearbyint(af * 16777216.0f));
  }
  uint32_t r = ax - 0x38000000u;        // rebias the exponent 127 -> 15
  r += 0xfffu + ((r >> 13) & 1u);       // round the 13 dropped mantissa bits to nearest even
  return (uint16_t)(sign | (r >> 13));  // a carry into the exponent is the correct rounding
}

}  // namespace

extern "C" int dmlp_host_threads(void) { return pool().size(); }

// (min, max) of an int32 array on the render pool (the native step's label / k scans: ~15 us
// single-threaded at the bench shape, on the step's critical path); (0, -1) when empty.
extern "C" void dmlp_host_i32_range(const int* a, int64_t n, int* lo, int* hi) {
  if (n <= 0) {
    *lo = 0;
    *hi = -1;
    return;
  }
  int mn[64], mx[64];
  const int parts = n < (1 << 16) ? 1 : std::min(pool().size(), 64);
  std::function<void(int, int)> job = [&](int part, int np) {
    if (part >= parts) return;
    const int64_t b = n * part / std::min(np, parts), e = n * (part + 1) / std::min(np, parts);
    int l = INT32_MAX, h = INT32_MIN;
    for (int64_t i = b; i < e; ++i) {
      l = std::min(l, a[i]);
      h = std::max(h, a[i]);
    }
    mn[part] = l;
    mx[part] = h;
  };
  for (int i = 0; i < parts; ++i) { mn[i] = INT32_MAX; mx[i] = INT32_MIN; }
  if (parts == 1) job(0, 1);
  else pool().run(job);
  int l = INT32_MAX, h = INT32_MIN;
  for (int i = 0; i < parts; ++i) { l = std::min(l, mn[i]); h = std::max(h, mx[i]); }
  *lo = l;
  *hi = h;
}

// fn(ctx, part, parts) on every worker of the render pool and the caller (parts = the pool's
// size); returns when all parts are done.  For host passes of other modules (the drop-in's
// index of the harness's vectors) that should not pay a thread start each.
extern "C" void dmlp_host_pool_run(void (*fn)(void*, int, int), void* ctx) {
  std::function<void(int, int)> job = [&](int part, int parts) { fn(ctx, part, parts); };
  pool().run(job);
}

namespace {

// Row sources: a row-major block, or a table of row pointers (the engine.h drop-in reads the
// harness's per-point attribute vectors in place — no packing pass over the AoS input).
struct FlatRows {
  const double* X;
  int A;
  const double* operator()(int64_t i) const { return X + i * A; }
};
struct TableRows {
  const double* const* R;
  const double* operator()(int64_t i) const { return R[i]; }
};

template <class Src>
void center(Src src, int64_t N, int A, double* mu) {
  const int64_t n = std::min<int64_t>(N, 4096);
  // column sums in a local block: accumulating in place would reload / store mu[a] on every
  // row (the compiler cannot rule out mu aliasing X)
  for (int a0 = 0; a0 < A; a0 += 64) {
    const int w = std::min(64, A - a0);
    double acc[64] = {0.0};
    for (int64_t i = 0; i < n; ++i) {
      const double* r = src(i) + a0;
      for (int a = 0; a < w; ++a) acc[a] += r[a];
    }
    for (int a = 0; a < w; ++a) mu[a0 + a] = n ? acc[a] / (double)n : 0.0;
  }
}

}  // namespace

extern "C" void dmlp_cpu_center(const double* X, int64_t N, int A, double* mu) {
  center(FlatRows{X, A}, N, A, mu);
}
extern "C" void dmlp_cpu_center_rows(const double* const* rows, int64_t N, int A, double* mu) {
  center(TableRows{rows}, N, A, mu);
}

namespace {

// Portable row: the reference for the AVX2 path's bits (four fixed partial sums for |c|^2).
template <class Src>
int prep_range_scalar(Src src, int64_t q0, int64_t q1, int A, const double* mu, int W,
                      uint16_t* qhi, float* qn) {
  int ok = 1;
  for (int64_t q = q0; q < q1; ++q) {
    const double* r = src(q);
    uint16_t* h = qhi + q * W;
    double s4[4] = {0.0, 0.0, 0.0, 0.0};
    for (int a = 0; a < A; ++a) {
      double c = r[a] - mu[a];
      if (!(std::fabs(c) < kMaxAbs)) { ok = 0; c = 0.0; }
      s4[a & 3] += c * c;
      h[a] = f16_rn((float)c);
    }
    for (int a = A; a < W; ++a) h[a] = 0;
    qn[q] = (float)((s4[0] + s4[2]) + (s4[1] + s4[3]));
  }
  return ok;
}

// A multiple of 8: 4 doubles per vector, partial sums s4[a & 3] exactly as the scalar row.
template <class Src>
__attribute__((target("avx2,f16c"))) int prep_range_avx2(Src src, int64_t q0, int64_t q1,
                                                          int A, const double* mu, int W,
                                                          uint16_t* qhi, float* qn) {
  const __m256d lim = _mm256_set1_pd(kMaxAbs);
  const __m256d sgn = _mm256_set1_pd(-0.0);
  __m256d okv = _mm256_castsi256_pd(_mm256_set1_epi64x(-1));
  for (int64_t q = q0; q < q1; ++q) {
    const double* r = src(q);
    uint16_t* h = qhi + q * W;
    __m256d acc = _mm256_setzero_pd();
    for (int a = 0; a < A; a += 8) {
      __m256d c0 = _mm256_sub_pd(_mm256_loadu_pd(r + a), _mm256_loadu_pd(mu + a));
      __m256d c1 = _mm256_sub_pd(_mm256_loadu_pd(r + a + 4), _mm256_loadu_pd(mu + a + 4));
      const __m256d m0 = _mm256_cmp_pd(_mm256_andnot_pd(sgn, c0), lim, _CMP_LT_OQ);
      const __m256d m1 = _mm256_cmp_pd(_mm256_andnot_pd(sgn, c1), lim, _CMP_LT_OQ);
      okv = _mm256_and_pd(okv, _mm256_and_pd(m0, m1));
      c0 = _mm256_and_pd(c0, m0);
      c1 = _mm256_and_pd(c1, m1);
      acc = _mm256_add_pd(acc, _mm256_mul_pd(c0, c0));
      acc = _mm256_add_pd(acc, _mm256_mul_pd(c1, c1));
      const __m256 f = _mm256_set_m128(_mm256_cvtpd_ps(c1), _mm256_cvtpd_ps(c0));
      _mm_storeu_si128((__m128i*)(h + a),
                       _mm256_cvtps_ph(f, _MM_FROUND_TO_NEAREST_INT | _MM_FROUND_NO_EXC));
    }
    for (int a = A; a < W; ++a) h[a] = 0;
    alignas(32) double s4[4];
    _mm256_store_pd(s4, acc);
    qn[q] = (float)((s4[0] + s4[2]) + (s4[1] + s4[3]));
  }
  return _mm256_movemask_pd(okv) == 0xf;
}

template <class Src>
int prep_range_any(Src src, int64_t q0, int64_t q1, int A, const double* mu, int W,
                   uint16_t* qhi, float* qn) {
  static const bool avx2 = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("f16c");
  if (avx2 && A % 8 == 0) return prep_range_avx2(src, q0, q1, A, mu, W, qhi, qn);
  return prep_range_scalar(src, q0, q1, A, mu, W, qhi, qn);
}

template <class Src>
int prep_queries(Src src, int64_t Q, int A, const double* mu, int KT, uint16_t* qhi, float* qn) {
  if (KT < 1 || KT > 8 || A > KT * 32) return 1;
  const int W = KT * 32;
  std::atomic<int> ok{1};
  std::function<void(int, int)> job = [&](int part, int parts) {
    const int64_t q0 = Q * part / parts, q1 = Q * (part + 1) / parts;
    if (!prep_range_any(src, q0, q1, A, mu, W, qhi, qn)) ok.store(0, std::memory_order_relaxed);
  };
  if (Q * (int64_t)A < (int64_t)1 << 14) job(0, 1);
  else pool().run(job);
  return ok.load() ? 0 : 1;
}

}  // namespace

// qhi: [Q][KT*32] fp16 bits (zero padded), qn: [Q] fp32 |q - mu|^2.  Returns 1 if some
// |q - mu| is outside the screen's range (outputs then not usable), else 0.
extern "C" int dmlp_cpu_prep_queries(const double* Qx, int64_t Q, int A, const double* mu, int KT,
                                     uint16_t* qhi, float* qn) {
  return prep_queries(FlatRows{Qx, A}, Q, A, mu, KT, qhi, qn);
}
// The same from a table of row pointers (qhi / qn indexed like the table).
extern "C" int dmlp_cpu_prep_queries_rows(const double* const* rows, int64_t Q, int A,
                                          const double* mu, int KT, uint16_t* qhi, float* qn) {
  return prep_queries(TableRows{rows}, Q, A, mu, KT, qhi, qn);
}

namespace {

// One point's contribution to the fp16 hi-only tile image: 8 attributes (one 16-byte fragment chunk)
// per (kt, kg), |c|^2 in fp64.  The chunk of point p = t*64 + rt*16 + r, attributes kt*32 + kg*8
// .. +7, sits at uint4 index ((t*4 + rt)*KT + kt)*64 + kg*16 + r (prep.hip's layout, lo dropped).
template <class Src>
int prep_data_range(Src X, int64_t N, int64_t p0, int64_t p1, int A, const double* mu,
                    int KT, uint16_t* xhi, float* xinit, float* nmax) {
  static const bool avx2 = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("f16c");
  const int W = KT * 32;
  int ok = 1;
  float mx = 0.0f;
  alignas(32) uint16_t h[256];  // W <= 256 (KT <= 8; dmlp_cpu_prep_data_tiles checks)
  alignas(32) float qn1[1];
  for (int64_t p = p0; p < p1; ++p) {
    float ssf;
    if (p < N) {
      const FlatRows row{X(p), A};
      if (avx2 && A % 8 == 0) {
        if (!prep_range_avx2(row, 0, 1, A, mu, W, h, qn1)) ok = 0;
      } else {
        if (!prep_range_scalar(row, 0, 1, A, mu, W, h, qn1)) ok = 0;
      }
      ssf = qn1[0];
      xinit[p] = -0.5f * ssf;
      const float up = ssf * (1.0f + 1.0e-6f) + 1.0e-30f;
      mx = std::max(mx, up);
    } else {
      std::memset(h, 0, sizeof(uint16_t) * W);
      xinit[p] = -INFINITY;
    }
    const int64_t t = p >> 6;
    const int pl = (int)(p & 63), rt = pl >> 4, r = pl & 15;
    for (int kt = 0; kt < KT; ++kt)
      for (int kg = 0; kg < 4; ++kg)
        std::memcpy(xhi + ((((t * 4 + rt) * KT + kt) * 64 + kg * 16 + r) * 8), h + kt * 32 + kg * 8, 16);
  }
  *nmax = mx;
  return ok;
}

}  // namespace

namespace {

// Lossless 6-decimal ingest: x == fl(m / 1e6) for an int32 m (text inputs written with "%.6f",
// like generate_input.py's, parse to exactly these doubles).  Bitwise check, so -0.0 and any
// value with more digits fail and the caller ships fp64 instead.
int rows_i32_scalar(const double* src, int64_t a, int64_t b, int32_t* dst) {
  int ok = 1;
  for (int64_t i = a; i < b; ++i) {
    const double m = std::nearbyint(src[i] * 1.0e6);
    if (!(std::fabs(m) <= 2147483647.0)) { ok = 0; dst[i] = 0; continue; }
    dst[i] = (int32_t)m;
    const double back = (double)dst[i] / 1.0e6;  // from the int, as the device does (-0.0 fails)
    if (std::memcmp(&back, src + i, 8) != 0) ok = 0;
  }
  return ok;
}

__attribute__((target("avx2"))) int rows_i32_avx2(const double* src, int64_t a, int64_t b,
                                                  int32_t* dst) {
  const __m256d sc = _mm256_set1_pd(1.0e6);
  const __m256d lim = _mm256_set1_pd(2147483647.0);
  const __m256d sgn = _mm256_set1_pd(-0.0);
  __m256i okv = _mm256_set1_epi64x(-1);
  int64_t i = a;
  for (; i + 4 <= b; i += 4) {
    const __m256d x = _mm256_loadu_pd(src + i);
    const __m256d m = _mm256_round_pd(_mm256_mul_pd(x, sc), _MM_FROUND_TO_NEAREST_INT | _MM_FROUND_NO_EXC);
    const __m256d inr = _mm256_cmp_pd(_mm256_andnot_pd(sgn, m), lim, _CMP_LE_OQ);
    const __m256d mm = _mm256_and_pd(m, inr);  // out of range (or NaN): 0, flagged below
    const __m128i mi = _mm256_cvtpd_epi32(mm);
    const __m256d back = _mm256_div_pd(_mm256_cvtepi32_pd(mi), sc);
    const __m256i same = _mm256_cmpeq_epi64(_mm256_castpd_si256(back), _mm256_castpd_si256(x));
    okv = _mm256_and_si256(okv, _mm256_and_si256(same, _mm256_castpd_si256(inr)));
    _mm_storeu_si128((__m128i*)(dst + i), mi);
  }
  int ok = _mm256_movemask_pd(_mm256_castsi256_pd(okv)) == 0xf;
  return rows_i32_scalar(src, i, b, dst) && ok;
}

}  // namespace

// The same over rows [0, nrows) of a pointer table (A values each, dst row-major).
extern "C" int dmlp_cpu_rows_i32_rows(const double* const* rows, int64_t nrows, int A,
                                      int32_t* dst) {
  static const bool avx2 = __builtin_cpu_supports("avx2");
  std::atomic<int> ok{1};
  std::function<void(int, int)> job = [&](int part, int parts) {
    const int64_t a = nrows * part / parts, b = nrows * (part + 1) / parts;
    int good = 1;
    for (int64_t r = a; r < b; ++r)
      good &= avx2 ? rows_i32_avx2(rows[r], 0, A, dst + r * A)
                   : rows_i32_scalar(rows[r], 0, A, dst + r * A);
    if (!good) ok.store(0, std::memory_order_relaxed);
  };
  if (nrows * (int64_t)A < (int64_t)1 << 14) job(0, 1);
  else pool().run(job);
  return ok.load() ? 0 : 1;
}

// Pack the rows of a pointer table row-major into dst (fp64, the pool's threads).
extern "C" void dmlp_cpu_gather_rows(const double* const* rows, int64_t nrows, int A,
                                     double* dst) {
  std::function<void(int, int)> job = [&](int part, int parts) {
    const int64_t a = nrows * part / parts, b = nrows * (part + 1) / parts;
    for (int64_t r = a; r < b; ++r) std::memcpy(dst + r * A, rows[r], sizeof(double) * A);
  };
  if (nrows * (int64_t)A < (int64_t)1 << 14) job(0, 1);
  else pool().run(job);
}

// src[0 .. n) -> dst as int32 m with src[i] == fl(m / 1e6) bit for bit; returns 0 when every value
// passed (dst then reconstructs src exactly: prep.hip dmlp_rows_from_i32), 1 otherwise.
extern "C" int dmlp_cpu_rows_i32(const double* src, int64_t n, int32_t* dst) {
  static const bool avx2 = __builtin_cpu_supports("avx2");
  std::atomic<int> ok{1};
  std::function<void(int, int)> job = [&](int part, int parts) {
    const int64_t a = n * part / parts, b = n * (part + 1) / parts;
    const int r = avx2 ? rows_i32_avx2(src, a, b, dst) : rows_i32_scalar(src, a, b, dst);
    if (!r) ok.store(0, std::memory_order_relaxed);
  };
  if (n < (int64_t)1 << 14) job(0, 1);
  else pool().run(job);
  return ok.load() ? 0 : 1;
}

// Dataset screen operands on the host for tiles [t0, t1) of the image: xhi = prep.hip's tile
// image with the lo halves dropped ([n_tiles][4][KT][64] x 16 B, what the single-term screen and
// the group refine read), xinit[n_tiles*64] = -|x - mu|^2 / 2 (fp32; -inf for padding rows),
// *nmax = the rounded-up max |x - mu|^2 over these tiles (fp32).  The buffers are the whole
// image's (tile offsets are applied here).  Returns 1 if some |x - mu| is outside the screen's
// range.
namespace {
template <class Src>
int prep_data_tiles(Src X, int64_t N, int A, const double* mu, int KT, int64_t t0, int64_t t1,
                    uint16_t* xhi, float* xinit, float* nmax) {
  if (KT < 1 || KT > 8 || A > KT * 32) return 1;
  std::atomic<int> ok{1};
  float mx[kMaxPool] = {0.0f};  // one slot per pool part (pool().size() <= kMaxPool)
  std::function<void(int, int)> job = [&](int part, int parts) {
    const int64_t nt = t1 - t0;
    const int64_t p0 = (t0 + nt * part / parts) * 64, p1 = (t0 + nt * (part + 1) / parts) * 64;
    if (!prep_data_range(X, N, p0, p1, A, mu, KT, xhi, xinit, &mx[part])) ok.store(0);
  };
  if ((t1 - t0) * 64 * (int64_t)A < (int64_t)1 << 14) job(0, 1);
  else pool().run(job);
  float m = 0.0f;
  for (float v : mx) m = std::max(m, v);
  *nmax = m;
  return ok.load() ? 0 : 1;
}
}  // namespace

extern "C" int dmlp_cpu_prep_data_tiles(const double* X, int64_t N, int A, const double* mu,
                                        int KT, int64_t t0, int64_t t1, uint16_t* xhi,
                                        float* xinit, float* nmax) {
  return prep_data_tiles(FlatRows{X, A}, N, A, mu, KT, t0, t1, xhi, xinit, nmax);
}
extern "C" int dmlp_cpu_prep_data_tiles_rows(const double* const* rows, int64_t N, int A,
                                             const double* mu, int KT, int64_t t0, int64_t t1,
                                             uint16_t* xhi, float* xinit, float* nmax) {
  return prep_data_tiles(TableRows{rows}, N, A, mu, KT, t0, t1, xhi, xinit, nmax);
}

// The whole image; *xnmax_bits = the max as fp32 bits.
extern "C" int dmlp_cpu_prep_data(const double* X, int64_t N, int A, const double* mu, int KT,
                                  uint16_t* xhi, float* xinit, unsigned* xnmax_bits) {
  float m = 0.0f;
  const int bad = dmlp_cpu_prep_data_tiles(X, N, A, mu, KT, 0, (N + 63) / 64, xhi, xinit, &m);
  std::memcpy(xnmax_bits, &m, 4);
  return bad;
}
