// pipeline.hip — the ONE native single-GPU k-NN pipeline of the framework.  Every front end
// runs it: the Python engine (ops/knn.py: every strategy's local k-NN, and each rank's whole call
// of the node-shared farm at any world size), the standalone knn_engine and the engine.h drop-in
// linked with the reference's own common.cpp (engine_core.h).  Reference semantics: the
// distance loop engine.cpp:12-18 / bench_4 @0xcb80, the bounded-heap top-k bench_1
// @0xcfc7-0xd10c (here a screen + exact re-rank), the vote engine.cpp:319-332 and the report
// common.cpp:57-79.
//
// Two entry points over one dispatcher (class Local):
//
//   dmlp_knn_local  rows already on the device (the sharded strategies' shards, the ring's
//                   travelling shards, the out-of-core chunks): per-query classes
//                     1 <= k <= 64         single-term MFMA screen (screen_x1.hip) + group refine
//                     64 < k <= 256        3-term LDS screen (screen.hip) + refine
//                     k > 256, A > 256     exact fp64 paths (exact.hip / fallback.hip)
//                   on a device-rendered bf16 image (prep.hip); a query whose screen candidates
//                   overflow escalates alone (3-term screen, then exact).
//
//   dmlp_step       rows in host memory (flat arrays, or the drop-in's tables of row pointers
//                   into the harness's own vectors), the call the reference times: the host
//                   renders the single-term screen's fp16 operands (host_prep.cpp) and copies them
//                   on a side stream; the screen starts on them while the fp64 rows (lossless
//                   int32 when every value is a 6-decimal number) cross PCIe behind it; k in
//                   (64, 256] takes the two-pass single-term screen on the same operands; then
//                   exact re-rank + vote + FNV checksum, the report text rendered on the GPU and
//                   copied into the caller's page-locked buffer (or kept on the device for a
//                   multi-rank egress, dmlp_step_emit).  One host sync in the common case; an
//                   overflowed query escalates natively (no call is ever re-run elsewhere).
//
// Early start (dmlp_step, every k in [1, 64], one screen slice): the query operands cross first
// and the screen starts on them while the dataset image follows in slices, each with a ready word
// the screen waits on (screen_x1.hip k_screen_x1 rdy): the wait is bounded by elapsed time, its
// waits / eps growths / timeouts are counted on the device and returned in dmlp_step_args, and
// the first timeout turns the early start off for the rest of the process.
//
// Memory: grow-only buffers carved from bump arenas reserved once (dmlp_arena_reserve, untimed:
// the reference harness times ONE call per process, so no hipMalloc may land inside it).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "dmlp.h"
#include "dmlp_device.h"

namespace {

// ---------------------------------------------------------------- errors
struct Fail {
  int code;
};
#define CK(x)                                                   \
  do {                                                          \
    const hipError_t e_ = (x);                                  \
    if (e_ != hipSuccess) throw Fail{-(int)e_};                 \
  } while (0)
#define CKL(x)                                                  \
  do {                                                          \
    const int r_ = (x);                                         \
    if (r_ != 0) throw Fail{r_ < 0 ? r_ : -1000 - r_};          \
  } while (0)
template <class T>
T* need(T* p) {
  if (!p) throw Fail{-(int)hipErrorOutOfMemory};
  return p;
}

// ---------------------------------------------------------------- arenas
struct Arena {
  char* base = nullptr;
  size_t size = 0, used = 0;
  int dev = -1;  // the device the (device) arena was reserved on
  std::mutex mu;
  void* take(size_t bytes) {
    std::lock_guard<std::mutex> g(mu);
    const size_t b = (bytes + 255) & ~size_t(255);
    if (!base || used + b > size) return nullptr;
    void* p = base + used;
    used += b;
    return p;
  }
  bool owns(const void* p) const {
    return base && (const char*)p >= base && (const char*)p < base + size;
  }
};
Arena g_dev, g_host;

void* dev_alloc(size_t bytes) {
  // the arena lives on one device: a buffer for another device (a process driving two GPUs)
  // comes from hipMalloc on the current one
  int d = -1;
  void* p = nullptr;
  if (g_dev.base && hipGetDevice(&d) == hipSuccess && d == g_dev.dev) p = g_dev.take(bytes);
  if (!p && hipMalloc(&p, std::max<size_t>(bytes, 1)) != hipSuccess) p = nullptr;
  return p;
}
void dev_free(void* p) {
  if (p && !g_dev.owns(p)) (void)hipFree(p);
}
void* host_alloc(size_t bytes) {
  void* p = g_host.take(bytes);
  if (!p && hipHostMalloc(&p, std::max<size_t>(bytes, 1), hipHostMallocDefault) != hipSuccess)
    p = nullptr;
  return p;
}
void host_free(void* p) {
  if (p && !g_host.owns(p)) (void)hipHostFree(p);
}

template <typename T>
struct DBuf {  // grow-only device buffer (throws when it cannot grow)
  T* p = nullptr;
  size_t n = 0;
  T* get(size_t m) {
    m = std::max<size_t>(m, 1);
    if (m > n) {
      dev_free(p);
      p = need((T*)dev_alloc(m * sizeof(T)));
      n = m;
    }
    return p;
  }
};
template <typename T>
struct HBuf {  // grow-only page-locked host buffer
  T* p = nullptr;
  size_t n = 0;
  T* get(size_t m) {
    m = std::max<size_t>(m, 1);
    if (m > n) {
      host_free(p);
      p = need((T*)host_alloc(m * sizeof(T)));
      n = m;
    }
    return p;
  }
};

// ---------------------------------------------------------------- switches
bool env_off(const char* name) {
  const char* e = std::getenv(name);
  return e && e[0] == '0';
}
int env_int(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e && *e ? std::atoi(e) : dflt;
}
// early start of dmlp_step (DMLP_FAST_EARLY=0: off, =1: on; dmlp_step_early); off for the rest
// of the process after a wait timed out.  Default: on, unless several ranks share this GPU
// (DMLP_DEVICE_RANKS > 1, set by both front ends): one rank's screen spinning on its slices
// then holds the CUs the other ranks' copies need — P = 3 on one MI355X measured 20.8 ms/step
// with it against 7.3 ms without (profiles/r7h_host_budget.md).
int g_early = -1;
bool early_on() {
  if (g_early < 0) {
    const char* e = std::getenv("DMLP_FAST_EARLY");
    g_early = e && *e ? (std::string(e) != "0") : env_int("DMLP_DEVICE_RANKS", 1) <= 1;
  }
  return g_early != 0;
}
constexpr int kEarlySlices = 8;  // dataset image slices behind the query operands (profiles/r6f)
// The pair refine reads its members from a point-major copy of the fp16 image (one 64-byte run
// per member: k_refine_pair 211 -> 177 us, profiles/r7n_refine_ab.txt r8i); DMLP_PAIR_ROWMAJOR=0
// keeps the tile image
bool rowmajor_on() {
  static const bool on = !(getenv("DMLP_PAIR_ROWMAJOR") && getenv("DMLP_PAIR_ROWMAJOR")[0] == '0');
  return on;
}
// query render slices under the early start (profiles/r6i: 4 is best)
int early_qchunks() {
  static const int q = std::min(16, std::max(1, env_int("DMLP_FAST_QCHUNKS", 4)));
  return q;
}
// Device render (DMLP_DEVICE_RENDER=1): the screen's fp16 operands rendered on the GPU (prep.hip
// k_render) from the rows that cross PCIe for the exact re-rank anyway (lossless int32): the host
// only packs int32 rows.  Off by default: the operands then wait for the int32 rows, and it
// measured slower than the host render (host_prep.cpp) at every size (profiles/r9r).
bool dr_on();  // (Tuning::device_render below)
// The render kernels (k_render: one-wave workgroups, 40 VGPRs, no LDS) would have to run beside
// an early-start screen that fills the GPU and spins on their ready words.  Measured
// (profiles/r9e-r9g): with 256-thread workgroups they never started beside it (every wave timed
// out); with one-wave workgroups beside the KT 1 / k <= 16 screen they ran in one session and
// never started in the next (same code and shape), and never beside the k > 16 variant.  The
// dispatcher does not reliably hand them slots, so an early-start step keeps the host render
// (host_prep.cpp: its copies do get through) and the device render serves the steps without
// an early start.
bool dr_early_ok(int, int) { return false; }
// The early start's copies (small ones run as blit kernels) need a wave slot beside the spinning
// screen: the screen variant must leave registers free (of 512 per SIMD lane; hipcc
// -Rpass-analysis=kernel-resource-usage): KT 1 k <= 16 2 x 208 (96 free), KT 1 k > 16 320,
// KT 2 k > 16 350, KT 4 322 / 415 — but KT 2 k <= 16 takes 2 x 241 (16 free after the allocation
// granule: every wave timed out, profiles/r9h) and KT 8 up to all 512.
bool early_room(int KT, int kmax) { return KT == 1 || (KT == 2 && kmax > 16) || KT == 4; }
// test knob: the host sleeps this long before each dataset image slice of an early-start call,
// so the screen provably waits mid-scan (tests/test_engine_gpu.py)
int g_early_delay_us = -1;
int early_delay_us() {
  if (g_early_delay_us < 0) g_early_delay_us = std::max(0, env_int("DMLP_FAST_EARLY_DELAY_US", 0));
  return g_early_delay_us;
}
// host render + H2D of the screen operands in pipelined slices (profiles/r2t: 2)
int host_slices() {
  static const int s = std::max(1, env_int("DMLP_HOST_OPS_CHUNKS", 2));
  return s;
}
// fp64 rows as lossless int32 when every value is a 6-decimal number (DMLP_ROWS_I32=0: fp64)
bool rows_i32_on() {
  static const bool on = !env_off("DMLP_ROWS_I32");
  return on;
}
// 3-term streaming screen for the escalation of k <= 32 (KNN_SCREEN=lds: the LDS screen)
bool stream_screen_on() {
  static const bool on = !(std::getenv("KNN_SCREEN") && std::string(std::getenv("KNN_SCREEN")) == "lds");
  return on;
}

// Tuning / A-B switches (dmlp_pipeline_set): CUs the slice choice fills (tests shrink it to force
// wide slices), the first screen of the k <= 32 class on the device image (0 single-term, 1 3-term
// streaming, 2 3-term LDS), the two-pass single-term screen for k in (32, 256] on the host
// operands (0: the 3-term LDS screen on the device image), the host-rendered operands (0: the
// device image path for every step, 1: when the render pool has >= 2 threads, 2: always).
struct Tuning {
  int num_cus = 256;
  int screen = 0;
  int x1k = 1;
  int host_ops = 1;
  // device render: -1 (default) by the cost model below, 0 never, 1 always (DMLP_DEVICE_RENDER)
  int device_render = -1;
};
Tuning make_tuning() {
  Tuning t;
  // environment defaults (A/B runs of the binaries): KNN_SCREEN=stream|lds, KNN_X1K=0
  if (const char* e = std::getenv("KNN_SCREEN"))
    t.screen = std::string(e) == "stream" ? 1 : std::string(e) == "lds" ? 2 : 0;
  if (env_off("KNN_X1K") || env_off("DMLP_X1K")) t.x1k = 0;
  // DMLP_HOST_OPS=0: the device path; =1: the host operands whatever the pool size; unset: the
  // host operands when the render pool has at least 2 threads (Step::run: with 1 the device path
  // measured faster, 4.86 vs 5.64 ms/step; at 2 threads the host operands still win, 3.58 vs
  // 3.74: profiles/r7h_host_budget.md)
  if (const char* e = std::getenv("DMLP_DEVICE_RENDER"); e && *e) t.device_render = e[0] != '0';
  if (env_off("DMLP_HOST_OPS")) t.host_ops = 0;
  else if (const char* e = std::getenv("DMLP_HOST_OPS"); e && *e) t.host_ops = 2;  // forced on
  return t;
}
Tuning g_tune = make_tuning();
bool dr_on() { return g_tune.device_render > 0; }
// The device render's share of the work by the cost model: the host render ships 6 bytes per
// value (the fp16 image + the int32 rows) after a host pass that writes both, the device render 4
// (the int32 rows; the GPU renders the image from them) — at large N the step is bound by that
// host pass and PCIe (profiles/r10a_large_n_render_ab.jsonl: N = 1e6, A = 128: 21.1 / 22.4 vs
// 28.8 / 38.2 ms).  Below the early start's reach (one screen slice, nt <= 4096) the host render
// keeps the early start (the render kernels get no wave slots beside its spinning screen).
constexpr int64_t kDrMinValues = int64_t(1) << 23;
bool dr_auto(int64_t N, int A) { return g_tune.device_render < 0 && N * A >= kDrMinValues; }
// Every small host <-> device copy of the step goes through the SDMA engines (dmlp::dma_copy: a
// copy below ~32 KiB would otherwise be a blit kernel, a memset a fill kernel) — its words are
// cleared by a DMA copy from this page-locked block of zeros.
constexpr int kZeroBytes = 4096;
const void* zero_block() {
  static void* z = [] {
    void* p = nullptr;
    if (hipHostMalloc(&p, kZeroBytes, hipHostMallocDefault) != hipSuccess) return (void*)nullptr;
    std::memset(p, 0, kZeroBytes);
    return p;
  }();
  return z;
}
hipError_t dma_zero(void* dst, size_t bytes, hipStream_t s) {
  const void* z = zero_block();
  if (!z || bytes > (size_t)kZeroBytes) return hipMemsetAsync(dst, 0, bytes, s);
  return dmlp::dma_copy(dst, z, bytes, s);
}
// memcpy on the render pool (large host staging copies: labels, k)
void pool_memcpy(void* dst, const void* src, int64_t bytes) {
  if (bytes < (int64_t(1) << 18)) {
    std::memcpy(dst, src, (size_t)std::max<int64_t>(bytes, 0));
    return;
  }
  struct Cp { char* d; const char* s; int64_t n; } cp{(char*)dst, (const char*)src, bytes};
  dmlp_host_pool_run([](void* c, int t, int nt) {
    const Cp& p = *(const Cp*)c;
    const int64_t lo = p.n * t / nt & ~int64_t(63), hi = t + 1 == nt ? p.n : p.n * (t + 1) / nt & ~int64_t(63);
    if (hi > lo) std::memcpy(p.d + lo, p.s + lo, (size_t)(hi - lo));
  }, &cp);
}
// an early-start slice's ready word: its max norm's fp32 bits, never 0 (0 = not landed): a
// norm of 0 is published as the smallest denormal (a valid upper bound)
unsigned ready_bits(float nm) {
  unsigned b = 0;
  std::memcpy(&b, &nm, 4);
  return b ? b : 1u;
}
// what the last call did (dmlp_pipeline_stats)
struct Stats {
  int64_t n_exact = 0, n_escalated = 0, path = 0, early = 0;
  int64_t n_exact_f64 = 0, n_exact_f64_redo = 0;  // exact-path queries on the fp64 MFMA screen
  int64_t device_render = 0;  // the screen operands were rendered on the device
};
Stats g_stats;

// ---------------------------------------------------------------- slices of the screens
int slices_stream(int nq, int qw, int64_t n_tiles, int waves_per_cu, int64_t s_lo = 1) {
  const int nqb = (nq + qw - 1) / qw;
  const int slots = waves_per_cu * g_tune.num_cus;
  const int s_min = (int)std::max<int64_t>(std::max<int64_t>(1, s_lo),
                                           (n_tiles * 64 + (1ll << 29) - 1) >> 29);
  if (nqb >= slots) return s_min;
  int best = s_min;
  double best_eff = 0.0;
  for (int S = s_min; S < s_min + 64 && S <= std::max<int64_t>(s_min, n_tiles / 4); ++S) {
    const double w = (double)nqb * S;
    const double eff = w / (std::ceil(w / slots) * slots);
    if (eff >= 0.9) return S;
    if (eff > best_eff + 1e-9) {
      best = S;
      best_eff = eff;
    }
  }
  return best;
}
int slices_lds(int nq, int waves, int64_t n_tiles) {
  const int nqb = (nq + waves * 16 - 1) / (waves * 16);
  int S = 1;
  while ((int64_t)nqb * S < 2 * g_tune.num_cus && S * 2 <= std::max<int64_t>(1, n_tiles) && S < 256) S *= 2;
  return S;
}
// data slices of the single-term x1 pass over nq queries of class bound kcls.  Every (query,
// slice) keeps its slice's own top-k groups (all k may sit in one slice) in <= 120 entries, so a
// slice must hold many more groups than k: for k > 32 at least 32 k points per slice (a slice of
// a few hundred groups would keep most of them within 2 eps of its k-th key and overflow)
int x1_slices(int nq, int KT, int kcls, int64_t nt) {
  const int64_t smin = dmlp_screen_x1_min_slices(nt);
  int S = slices_stream(nq, dmlp_screen_x1_cols(KT, kcls), nt,
                        dmlp_screen_x1_waves_per_cu_kt(KT, kcls), smin);
  if (kcls > 32) S = (int)std::max<int64_t>(smin, std::min<int64_t>(S, nt * 64 / (32 * kcls)));
  return std::max(S, 1);
}

// sum of the decimal digit counts of v over [a, b)
int64_t digits_sum(int64_t a, int64_t b) {
  int64_t s = 0, lo = 0, hi = 10;
  for (int d = 1; d <= 19 && lo < b; ++d, lo = hi, hi = hi > INT64_MAX / 10 ? INT64_MAX : hi * 10) {
    const int64_t x = std::max(a, lo), y = std::min(b, hi);
    if (y > x) s += (y - x) * d;
  }
  return s;
}

// ---------------------------------------------------------------- per-device workspace
enum { M_ENTER, M_OPS, M_DATA, M_ROWS, M_SCREEN, M_REFINE, M_FORMAT, M_D2H, M_N };
const char* const kMarkNames[M_N] = {"enter", "operands_landed", "data_landed", "rows_landed",
                                     "screen_done", "knn_done", "format_done",
                                     "report_d2h_done"};

struct Ctx {
  int dev = -1;
  hipStream_t side = nullptr;  // host->device copies of dmlp_step
  hipEvent_t ev_ops = nullptr, ev_rows = nullptr;
  bool marks_on = false, marks_valid = false;
  hipEvent_t marks[M_N] = {};
  unsigned marks_rec = 0;  // marks recorded in the last call (a path may skip some)
  // Local: device image, query fragments, candidates, class lists, exact workspace
  DBuf<double> mu;
  DBuf<char> xfrag;
  DBuf<float> xinit;
  DBuf<unsigned> words;  // [0] xnmax bits, [1] bad
  DBuf<short> qhi, qlo;
  DBuf<float> qn, cand_h, k1_h, k1_seed;
  DBuf<int> qidx_a, qidx_b, qidx_c, qidx_e, qidx_e2, qidx_f, qidx_r, kdev, kfull, cand_ids,
      cand_cnt, status, ovf, ident, k1_ids, k1_cnt, kp_d, qidx_f2, f64_stat, f64_ovf;
  DBuf<char> fb_ws, f64_ws;
  // page-locked staging of the per-call host lists (one per list: no copy waits for a reuse)
  HBuf<int> kk_h, kp_h, kfull_h, ident_h, small_h, la_h, lb_h, lc_h, le_h, le2_h, lf_h, lr_h,
      lf2_h, f64_h, f64_st_h;
  int64_t ident_len = 0;
  // dmlp_step: host-rendered operands (staging + device), rows, labels, outputs, report
  HBuf<uint16_t> sx_hi, sq_hi;
  HBuf<float> sx_in, sq_n;
  HBuf<unsigned> sx_nm;
  HBuf<double> s_mu, s_f64;
  HBuf<int> s_i32, s_lab;
  HBuf<int64_t> s_len, small64_h;
  DBuf<int64_t> small64_d;
  hipEvent_t ev_done = nullptr;
  hipEvent_t ev_chunk[kEarlySlices] = {};  // the large-N pipeline's chunk events
  DBuf<short> dx_hi, dq_hi;
  DBuf<short> dx_row;  // the fp16 image point-major (dmlp_x1_rowmajor) for the pair refine
  DBuf<double> d_mu;   // device render: the centre
  DBuf<unsigned> dr_words;  // device render: [0, 8) slice done counters, [8, 72) query-block
                            // done counters, [72] out-of-range flag
  DBuf<float> dx_in, dq_n;
  DBuf<unsigned> dwords;  // the step's words (kW_*): cleared by one DMA copy per call
  DBuf<int> d_i32, d_lab, d_lb;
  DBuf<double> d_X, d_Q, d_od;
  DBuf<int> d_oi;
  DBuf<uint64_t> d_cs;
  DBuf<int64_t> d_off;
  DBuf<char> d_text;
  int64_t text_len = 0;  // the last dmlp_step's report bytes on the device (dmlp_step_emit)
};

// dmlp_step's device words (Ctx::dwords): [kW_XNMAX] the image's max norm, [kW_BAD] out of range,
// [kW_RDY, + kEarlySlices) the early start's ready words (norm bits), [kW_EST, + 4) early-start
// counters, [kW_OVF] the overflow counter.  All zeroed per call (one DMA copy).
constexpr int kW_XNMAX = 0, kW_BAD = 1, kW_RDY = 2, kW_EST = kW_RDY + kEarlySlices,
              kW_OVF = kW_EST + 4, kW_N = kW_OVF + 1;

Ctx& ctx() {
  static Ctx c[16];
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= 16) d = 0;
  Ctx& w = c[d];
  if (!w.side) {
    w.dev = d;
    CK(hipStreamCreateWithFlags(&w.side, hipStreamNonBlocking));
    CK(hipEventCreateWithFlags(&w.ev_ops, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&w.ev_rows, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&w.ev_done, hipEventDisableTiming));
    for (hipEvent_t& e : w.ev_chunk) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  return w;
}

// The step's small results in one word block: [0] report length, [1] overflowed queries,
// [2..4] early-start waits / eps growths / timeouts.
__global__ void k_pack_small(const int64_t* __restrict__ len, const int* __restrict__ ovf,
                             const unsigned* __restrict__ estats, const unsigned* __restrict__ rbad,
                             int64_t* __restrict__ out) {
  if (threadIdx.x == 0) {
    out[0] = len ? *len : 0;
    out[1] = *ovf;
    out[2] = estats ? estats[0] : 0;
    out[3] = estats ? estats[1] : 0;
    out[4] = estats ? estats[2] : 0;
    out[5] = estats ? estats[3] : 0;
    out[6] = rbad ? *rbad : 0;
  }
}

// Keep one wave per CU busy for `us` microseconds of the constant-rate wall clock (tick_khz
// ticks per ms): the clocks of an idle GPU ramp up before a timed call (dmlp_step_prewarm).
__global__ void k_busy(long long ticks) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
}

// Wait for the step's last event by polling it (the host thread spins for the ~2 ms a step takes
// instead of sleeping in the runtime's blocking wait, whose wake-up sat on every step's tail).
void spin_wait(hipEvent_t e) {
  for (;;) {
    const hipError_t r = hipEventQuery(e);
    if (r == hipSuccess) return;
    if (r != hipErrorNotReady) {
      (void)hipGetLastError();
      CK(hipEventSynchronize(e));  // (reports the error)
      return;
    }
    __builtin_ia32_pause();
  }
}

int* identity(Ctx& w, int64_t n, hipStream_t st) {  // device 0, 1, ..., n-1 (grow-only)
  const int64_t m = std::max<int64_t>(n, 1 << 16);
  int* p = w.ident.get(m);
  if (w.ident_len < n) {
    int* h = w.ident_h.get(m);
    for (int64_t i = 0; i < m; ++i) h[i] = (int)i;
    CK(dmlp::dma_copy(p, h, m * sizeof(int), st));
    w.ident_len = m;
  }
  return p;
}

// The host-rendered single-term operands (host_prep.cpp, fp16, hl = 1) on the device or in flight
// on the stream; rdy != nullptr: the all-queries x1 pass starts while the dataset image is still
// crossing PCIe (screen_x1.hip dmlp_screen_x1_early).
struct HostOps {
  const void* xhi = nullptr;
  const float* xin = nullptr;
  unsigned* words = nullptr;  // [0] xnmax bits, [1] bad (0)
  const void* qhi = nullptr;
  const float* qn = nullptr;
  const unsigned* rdy = nullptr;  // ready words, one per slice (the slice's norm bits)
  int rdy_tiles = 1, rdy_n = 0;
  unsigned* estats = nullptr;
  // the large-N pipeline (Step::run): the dataset lands in chunk_n chunks of the S-slice screen,
  // chunk c = slices [chunk_s[c], chunk_s[c + 1]) complete once chunk_ev[c] fired — each chunk's
  // screen is launched behind its own event while later chunks still cross PCIe
  int chunk_n = 0, chunk_S = 0;
  const int* chunk_s = nullptr;
  const hipEvent_t* chunk_ev = nullptr;
  std::function<void(int)> issue_chunk;  // queues chunk c's rows + render on the side stream
  const void* xrow = nullptr;  // xhi point-major (set once its copy kernel is queued), or none
};

// ---------------------------------------------------------------- the dispatcher
// One local call: launch() queues every pass on `st` without a host sync; the caller reads the
// overflow counter (*ovf, device) with its own sync and hands it to finish(), which escalates the
// overflowed queries (and synchronizes) only when there are some.
struct Local {
  Ctx& w;  // (a Local lives on its caller's stack for one call)
  // inputs
  const double* X = nullptr;  // device [N][A] (complete once `rows` fires)
  int64_t N = 0;
  int A = 0, KT = 1;
  const double* Qx = nullptr;  // device [Q][A]
  int64_t Q = 0;
  const int* k_host = nullptr;
  int kstride = 1;
  double* out_d = nullptr;
  int* out_i = nullptr;
  const int* labels = nullptr;  // device, nullable (no vote / checksum)
  int lo = 0, hi = 1;
  int* lab = nullptr;
  uint64_t* cs = nullptr;
  bool exact = false;
  hipStream_t st = nullptr;
  const HostOps* hx = nullptr;
  hipEvent_t rows = nullptr;
  std::function<void()> issue_rows;
  // (dmlp_step) k already clamped to N and on the device (kd_pre), every k in [1, 64] and <= N
  // (all_a_pre), the overflow counter zeroed on the device (ovf_pre): no host pass over the
  // queries and no copy or memset on `st` between the operands' event and the screen
  const int* kk_pre = nullptr;
  int* kd_pre = nullptr;
  int* ovf_pre = nullptr;
  bool all_a_pre = false;
  int kmax_pre = 0;
  // state
  int* kk = nullptr;
  int* kd = nullptr;
  int* stat = nullptr;
  int* ovf = nullptr;
  std::vector<int> a, b, c, f, rest;
  bool all_a = false, lds_ok = false, x1_ok = false, rows_issued = false, rows_waited = false;
  bool dev_ready = false, qprep = false, filled = false, bc_single = false;
  int first_a = 0;
  int64_t n_exact = 0, n_escalated = 0;

  explicit Local(Ctx& c_) : w(c_) {}

  void launch_rows() {
    if (!rows_issued) {
      rows_issued = true;
      if (issue_rows) issue_rows();
    }
  }
  void wait_rows() {
    launch_rows();
    if (!rows_waited) {
      if (rows) CK(hipStreamWaitEvent(st, rows, 0));
      rows_waited = true;
    }
  }
  // the device bf16 hi/lo image (prep.hip) and the device query fragments: the 3-term screens'
  // operands, and every screen's when the host did not render any
  void need_dev() {
    if (!dev_ready) {
      wait_rows();
      const int64_t nt = (N + 63) / 64;
      CK(hipMemsetAsync(w.words.get(2), 0, 2 * sizeof(unsigned), st));
      CKL(dmlp_center(X, N, A, w.mu.get(A), st));
      CKL(dmlp_prep_data(X, N, A, w.mu.p, KT, w.xfrag.get(nt * 64 * KT * 32 * 2 * sizeof(short)),
                         w.xinit.get(nt * 64), w.words.p, w.words.p + 1, st));
      dev_ready = true;
    }
    if (!qprep) {
      CKL(dmlp_prep_queries(Qx, Q, A, w.mu.p, KT, w.qhi.get(Q * KT * 32), w.qlo.get(Q * KT * 32),
                            w.qn.get(Q), w.words.p + 1, st));
      qprep = true;
    }
  }
  void fill() {
    if (filled) return;
    // padding (+inf, -1) for k > N, like bench_2's {1e18, -1} sentinel (@0xc608)
    CK(hipMemsetAsync(out_i, 0xff, (size_t)Q * kstride * sizeof(int), st));
    CKL(dmlp_fill_f64(out_d, (int64_t)Q * kstride, INFINITY, st));
    CK(hipMemsetAsync(stat, 0, Q * sizeof(int), st));
    filled = true;
  }

  // impl: 0 x1 single-term (k <= 32), 1 3-term streaming (k <= 32), 2 3-term LDS (k <= 256),
  // 4 two-pass single-term x1 on the host operands (k <= 256)
  void pass(const std::vector<int>* idx, int impl, DBuf<int>& qbuf, HBuf<int>& hbuf) {
    const int nq = idx ? (int)idx->size() : (int)Q;
    if (nq == 0) return;
    int* qi;
    if (idx) {
      qi = qbuf.get(nq);
      int* h = hbuf.get((size_t)nq);
      std::memcpy(h, idx->data(), nq * sizeof(int));
      CK(dmlp::dma_copy(qi, h, nq * sizeof(int), st));
    } else {
      qi = identity(w, Q, st);
    }
    int kcls = 1;
    if (idx) for (int q : *idx) kcls = std::max(kcls, kk[q]);
    else if (kmax_pre > 0) kcls = kmax_pre;
    else for (int64_t q = 0; q < Q; ++q) kcls = std::max(kcls, kk[q]);
    const int64_t nt = (N + 63) / 64;
    const bool fin = labels != nullptr;
    if (impl == 0) {
      const int cap = dmlp_screen_x1_cap(kcls);
      // (the large-N pipeline cut its chunks for its own slice count)
      const int S = hx && hx->chunk_n > 0 && !idx ? hx->chunk_S : x1_slices(nq, KT, kcls, nt);
      int* ci = w.cand_ids.get((size_t)nq * S * cap);
      int* cc = w.cand_cnt.get((size_t)nq * S);
      float* ch = w.cand_h.get((size_t)nq * S * 2);
      const void* xf = hx ? hx->xhi : (const void*)w.xfrag.p;
      const float* xi = hx ? hx->xin : w.xinit.p;
      unsigned* wd = hx ? hx->words : w.words.p;
      const void* qh = hx ? hx->qhi : (const void*)w.qhi.p;
      const float* qnn = hx ? hx->qn : w.qn.p;
      const int hl = hx ? 1 : 2;
      if (hx && hx->rdy) {
        // the caller sized the early start for this all-queries pass with one slice
        if (S != 1 || idx) throw Fail{-7};
        CKL(dmlp_screen_x1_early(KT, A, xf, xi, nt, N, qh, qnn, qi, kd, nq, kcls, wd + 1, hx->rdy,
                                 hx->rdy_tiles, hx->rdy_n, ci, cc, ch, hx->estats, st));
      } else if (hx && hx->chunk_n > 0 && !idx) {
        // the large-N pipeline: each chunk's slices as soon as its rows are rendered
        for (int c = 0; c < hx->chunk_n; ++c) {
          hx->issue_chunk(c);  // (the host packs chunk c + 1 while chunk c's screen runs)
          CK(hipStreamWaitEvent(st, hx->chunk_ev[c], 0));
          CKL(dmlp_screen_x1_part(KT, hl, A, xf, xi, nt, N, qh, qnn, qi, kd, nq, kcls, wd, wd + 1,
                                  S, hx->chunk_s[c], hx->chunk_s[c + 1] - hx->chunk_s[c], ci, cc,
                                  ch, st));
        }
      } else {
        CKL(dmlp_screen_x1(KT, hl, A, xf, xi, nt, N, qh, qnn, qi, kd, nq, kcls, wd, wd + 1, S, ci,
                           cc, ch, st));
      }
      wait_rows();  // (issues the row copies first) the re-rank reads the fp64 rows
      CKL(dmlp_refine_groups_rm(cap, ci, cc, ch, S, X, A, Qx, xf, hx ? hx->xrow : nullptr, xi,
                                qh, KT, hl, N, idx ? qi : nullptr, kd, nq, out_d, out_i, kstride,
                                fin ? labels : nullptr, lo, hi, lab, cs, stat, ovf, kcls, st));
      return;
    }
    if (impl == 4) {
      // pass 1: S1 slices at k' = ceil(k / S1) -> per-query seeds; pass 2: COLLECT at the seed
      // into kCcap group ids per (query, slice); the large-k group refine (ops: screen_x1.hip)
      constexpr int kCcap = 1024, kS1 = 16;
      const int S2 = x1_slices(nq, KT, 16, nt);
      const int S1 = std::max(kS1, S2);
      int* kp = w.kp_h.get(Q);
      for (int64_t q = 0; q < Q; ++q) kp[q] = (std::max(kk[q], 1) + S1 - 1) / S1;
      int kmax1 = 1;
      for (int q : *idx) kmax1 = std::max(kmax1, kp[q]);
      int* kpd = w.kp_d.get(Q);
      CK(dmlp::dma_copy(kpd, kp, Q * sizeof(int), st));
      const int cap1 = dmlp_screen_x1_cap(kmax1);
      int* i1 = w.k1_ids.get((size_t)nq * S1 * cap1);
      int* c1 = w.k1_cnt.get((size_t)nq * S1);
      float* h1 = w.k1_h.get((size_t)nq * S1 * 2);
      float* hs = w.k1_seed.get(nq);
      int* i2 = w.cand_ids.get((size_t)nq * S2 * kCcap);
      int* c2 = w.cand_cnt.get((size_t)nq * S2);
      float* h2 = w.cand_h.get((size_t)nq * S2 * 2);
      CKL(dmlp_screen_x1(KT, 1, A, hx->xhi, hx->xin, nt, N, hx->qhi, hx->qn, qi, kpd, nq, kmax1,
                         hx->words, hx->words + 1, S1, i1, c1, h1, st));
      CKL(dmlp_x1_seed(h1, c1, S1, nq, hs, st));
      CKL(dmlp_screen_x1_collect(KT, A, hx->xhi, hx->xin, nt, N, hx->qhi, hx->qn, qi, kd, nq,
                                 hx->words, hx->words + 1, hs, kCcap, S2, i2, c2, h2, st));
      wait_rows();
      CKL(dmlp_refine_groups2(kCcap, i2, c2, h2, S2, X, A, Qx, hx->xhi, hx->xin, hx->qhi, KT, 1, N,
                              qi, kd, nq, out_d, out_i, kstride, fin ? labels : nullptr, lo, hi,
                              lab, cs, stat, ovf, 1, st));
      return;
    }
    need_dev();
    const float er = 2.0f * (float)(3.0 * std::ldexp(1.0, -16) + (3 * A + 8) * std::ldexp(1.0, -24));
    if (impl == 1) {
      const int cap = dmlp_screen_stream_cap(kcls);
      const int S = slices_stream(nq, dmlp_screen_stream_qw(KT), nt,
                                  dmlp_screen_stream_waves_per_cu(kcls));
      int* ci = w.cand_ids.get((size_t)nq * S * cap);
      int* cc = w.cand_cnt.get((size_t)nq * S);
      CKL(dmlp_screen_stream(KT, w.xfrag.p, w.xinit.p, nt, w.qhi.p, w.qlo.p, w.qn.p, qi, kd, nq,
                             kcls, w.words.p, w.words.p + 1, er, S, ci, cc, st));
      CKL(dmlp_refine(cap, ci, cc, S, X, A, Qx, qi, kd, nq, out_d, out_i, kstride,
                      fin ? labels : nullptr, lo, hi, lab, cs, stat, ovf, st));
      return;
    }
    const int cap = kcls <= 32 ? 128 : kcls <= 128 ? 256 : 512;
    const int S = slices_lds(nq, dmlp_screen_waves_hl(KT, cap, 2), nt);
    int* ci = w.cand_ids.get((size_t)nq * S * cap);
    int* cc = w.cand_cnt.get((size_t)nq * S);
    CKL(dmlp_screen(KT, cap, w.xfrag.p, w.xinit.p, nt, w.qhi.p, w.qlo.p, w.qn.p, qi, kd, nq,
                    w.words.p, w.words.p + 1, er, S, ci, cc, st));
    CKL(dmlp_refine(cap, ci, cc, S, X, A, Qx, qi, kd, nq, out_d, out_i, kstride,
                    fin ? labels : nullptr, lo, hi, lab, cs, stat, ovf, st));
  }

  // exact fp64 top-k of the queries in f (k <= 64/256: the fused streaming kernel; k <= 2048:
  // radix select over exact rows; larger k: rows + segmented sort)
  void exact_pass(std::vector<int>& fq) {
    if (fq.empty()) return;
    wait_rows();
    std::sort(fq.begin(), fq.end());
    std::vector<int> fused, small, big;
    // DMLP_EXACT_FUSED: 0 never the fused kernel, 2 for every k it supports, else the policy
    const char* fe = std::getenv("DMLP_EXACT_FUSED");
    const int kf = fe && fe[0] == '0' ? 0
                   : fe && fe[0] == '2' ? dmlp_exact_topk_kmax() : dmlp_exact_topk_kmax_for(N);
    const int ksel = dmlp_fallback_select_kmax();
    int kfmax = 0;
    for (int q : fq) {
      if (kk[q] <= kf) {
        fused.push_back(q);
        kfmax = std::max(kfmax, kk[q]);
      } else {
        (kk[q] <= ksel ? small : big).push_back(q);
      }
    }
    int* qi = w.qidx_f.get(fq.size());
    int* h = w.lf_h.get(fq.size());
    size_t base = 0;
    for (const auto* v : {&fused, &small, &big}) {
      std::memcpy(h + base, v->data(), v->size() * sizeof(int));
      base += v->size();
    }
    CK(dmlp::dma_copy(qi, h, fq.size() * sizeof(int), st));
    base = 0;
    if (!fused.empty()) {
      // A <= 32, 1 <= k <= 64: the fp64 MFMA screen + exact group re-rank (screen_f64.hip); its
      // overflows (pathological ties) go to the fused VALU kernel.  DMLP_EXACT_F64=0: never.
      int kfmin = kfmax;
      for (int q : fused) kfmin = std::min(kfmin, kk[q]);
      const bool f64 = !env_off("DMLP_EXACT_F64") && A <= dmlp_exact_f64_amax() && kfmin >= 1 &&
                       kfmax <= dmlp_exact_f64_kmax();
      std::vector<int> redo;
      if (f64) {
        const int64_t wb = dmlp_exact_f64_bytes(N, A, (int)fused.size(), kfmax);
        char* fws = w.f64_ws.get(wb);
        int* fst = w.f64_stat.get(Q);
        int* fov = w.f64_ovf.get(1);
        int* oh = w.f64_h.get(1);
        CK(dma_zero(fov, sizeof(int), st));
        CKL(dmlp_exact_f64(X, N, A, Qx, qi, kd, (int)fused.size(), kfmax, out_d, out_i, kstride,
                           fst, fov, fws, wb, st));
        CK(dmlp::dma_copy(oh, fov, sizeof(int), st));
        CK(hipStreamSynchronize(st));
        if (*oh > 0) {
          int* sh = w.f64_st_h.get(Q);
          CK(dmlp::dma_copy(sh, fst, Q * sizeof(int), st));
          CK(hipStreamSynchronize(st));
          for (int q : fused)
            if (sh[q]) redo.push_back(q);
        }
        g_stats.n_exact_f64 += (int64_t)fused.size();
        g_stats.n_exact_f64_redo += (int64_t)redo.size();
      }
      if (!f64 || !redo.empty()) {
        const int* ql = qi;
        int n = (int)fused.size(), km = kfmax;
        if (f64) {
          int* q2 = w.qidx_f2.get(redo.size());
          int* h2 = w.lf2_h.get(redo.size());
          std::memcpy(h2, redo.data(), redo.size() * sizeof(int));
          CK(dmlp::dma_copy(q2, h2, redo.size() * sizeof(int), st));
          ql = q2;
          n = (int)redo.size();
          km = 0;
          for (int q : redo) km = std::max(km, kk[q]);
        }
        CKL(dmlp_exact_topk(X, N, A, Qx, ql, kd, n, km, out_d, out_i, kstride, st));
      }
      base += fused.size();
    }
    for (int pz = 0; pz < 2; ++pz) {
      const std::vector<int>& v = pz == 0 ? small : big;
      if (v.empty()) continue;
      const int rws = (int)std::max<int64_t>(
          1, std::min<int64_t>((int64_t)v.size(), (1ll << 27) / std::max<int64_t>(1, N)));
      const int64_t wsb = pz == 0 ? dmlp_fallback_select_bytes(rws, N) : dmlp_fallback_bytes(rws, N);
      char* ws = w.fb_ws.get(wsb);
      for (size_t c0 = 0; c0 < v.size(); c0 += rws) {
        const int nb = (int)std::min<size_t>(rws, v.size() - c0);
        if (pz == 0)
          CKL(dmlp_fallback_select(X, N, A, Qx, qi + base + c0, kd, nb, ws, wsb, out_d, out_i,
                                   kstride, st));
        else
          CKL(dmlp_fallback_topk(X, N, A, Qx, qi + base + c0, kd, nb, ws, wsb, out_d, out_i,
                                 kstride, st));
      }
      base += v.size();
    }
  }

  // vote + checksum of the rows no refine finalized correctly: exact-path queries, k < 1, and
  // k > N (their checksum covers the (+inf, -1) padding, so the unclamped k)
  void finalize_rest(std::vector<int> r) {
    if (!labels || r.empty()) return;
    wait_rows();
    std::sort(r.begin(), r.end());
    r.erase(std::unique(r.begin(), r.end()), r.end());
    int* kf = w.kfull.get(Q);
    int* kh = w.kfull_h.get(Q);
    std::memcpy(kh, k_host, Q * sizeof(int));
    CK(dmlp::dma_copy(kf, kh, Q * sizeof(int), st));
    int* qi = w.qidx_r.get(r.size());
    int* h = w.lr_h.get(r.size());
    std::memcpy(h, r.data(), r.size() * sizeof(int));
    CK(dmlp::dma_copy(qi, h, r.size() * sizeof(int), st));
    CKL(dmlp_finalize(out_d, out_i, kstride, kf, qi, (int)r.size(), labels, lo, hi, lab, cs, st));
  }

  void launch() {
    g_stats.n_exact_f64 = g_stats.n_exact_f64_redo = 0;
    if (Q == 0) return;
    KT = dmlp_screen_kt(A);
    lds_ok = KT <= 8 && !exact;
    x1_ok = dmlp_screen_x1_qw(KT) > 0 && !exact;
    const bool screen = (lds_ok || x1_ok) && N > 0;
    all_a = screen && x1_ok;
    const int ka = dmlp_screen_x1_kmax();  // the single-term one-pass class: k <= 64
    if (kd_pre) {
      // (the step's bounds: every k in [1, 64] and <= N, so kk == k; on the device already)
      kk = const_cast<int*>(kk_pre);
      all_a = all_a && all_a_pre;
    } else {
      kk = w.kk_h.get(Q);
      for (int64_t q = 0; q < Q; ++q) {
        kk[q] = (int)std::min<int64_t>(k_host[q], N);
        all_a = all_a && k_host[q] >= 1 && k_host[q] <= ka && k_host[q] <= N;
      }
    }
    // the first screen of class a: the single-term one (k <= 64), or on the device image the
    // 3-term streaming screen (k <= 32; the A/B switch "screen") or LDS screen
    first_a = hx || g_tune.screen == 0 ? 0
              : g_tune.screen == 1 && dmlp_screen_stream_qw(KT) > 0 ? 1 : 2;
    const int ka_eff = first_a == 0 ? ka : first_a == 1 ? dmlp_screen_stream_kmax() : 32;
    if (ka_eff < ka) {
      for (int64_t q = 0; q < Q && all_a; ++q) all_a = k_host[q] <= ka_eff;
    }
    for (int64_t q = 0; q < Q && !all_a; ++q) {
      if (kk[q] < 1) {
        rest.push_back((int)q);
        continue;
      }
      if (screen && kk[q] <= ka_eff && x1_ok) a.push_back((int)q);
      else if (screen && lds_ok && kk[q] <= 128) b.push_back((int)q);
      else if (screen && lds_ok && kk[q] <= 256) c.push_back((int)q);
      else f.push_back((int)q);
      if (k_host[q] > N) rest.push_back((int)q);
    }
    if (kd_pre) {
      kd = kd_pre;
    } else {
      kd = w.kdev.get(Q);
      CK(dmlp::dma_copy(kd, kk, Q * sizeof(int), st));
    }
    stat = w.status.get(Q);
    if (ovf_pre) {
      ovf = ovf_pre;
    } else {
      ovf = w.ovf.get(1);
      CK(dma_zero(ovf, sizeof(int), st));
    }
    if (hx && hx->rdy && !all_a) throw Fail{-8};  // early start sized for one all-queries pass
    // every refine writes its queries' padding and status itself; the fill is only needed for
    // rows no refine covers (exact path, k < 1)
    if (!all_a || !hx) fill();
    if (all_a || !a.empty() || !b.empty() || !c.empty()) {
      if (!hx) need_dev();  // the device operands of every screen
      if (all_a || !a.empty()) pass(all_a ? nullptr : &a, first_a, w.qidx_a, w.la_h);
      if (!b.empty() || !c.empty()) {
        bc_single = hx && x1_ok && g_tune.x1k;
        if (bc_single) {  // both k > 32 classes in one two-pass single-term screen
          std::vector<int> bc(b);
          bc.insert(bc.end(), c.begin(), c.end());
          pass(&bc, 4, w.qidx_b, w.lb_h);
        } else {
          pass(&b, 2, w.qidx_b, w.lb_h);
          pass(&c, 2, w.qidx_c, w.lc_h);
        }
      }
    }
    launch_rows();
    exact_pass(f);
    n_exact += (int64_t)f.size();
    std::vector<int> r = rest;
    r.insert(r.end(), f.begin(), f.end());
    finalize_rest(r);
  }

  // novf: the overflow counter the caller read after its sync.  Escalates the overflowed queries
  // (single-term -> 3-term screen -> exact) and returns the number of queries redone.
  int finish(int novf) {
    if (novf <= 0) return 0;
    std::vector<int> sh(Q);
    CK(hipMemcpyAsync(sh.data(), stat, Q * sizeof(int), hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    std::vector<int> esc, esc_bc, fq;
    const bool stream_ok = dmlp_screen_stream_qw(KT) > 0 && stream_screen_on();
    const int ka = dmlp_screen_x1_kmax(), ks = dmlp_screen_stream_kmax();
    for (int64_t q = 0; q < Q; ++q) {
      if (!sh[q]) continue;
      // a single-term screen's overflow escalates to a 3-term screen (the streaming one for
      // k <= 32, the LDS one above); a 3-term screen's goes exact
      const bool single = (kk[q] <= ka && first_a == 0) || (kk[q] > ka && kk[q] <= 256 && bc_single);
      if (single && kk[q] <= ks && stream_ok) esc.push_back((int)q);
      else if (single && lds_ok) esc_bc.push_back((int)q);
      else fq.push_back((int)q);
    }
    // a 3-term screen's own overflow goes to the exact path (escalated twice: no third screen)
    const int redone = (int)(esc.size() + esc_bc.size() + fq.size());
    if (!esc.empty() || !esc_bc.empty()) {
      CK(dma_zero(ovf, sizeof(int), st));
      for (int q : esc) CK(hipMemsetAsync(stat + q, 0, sizeof(int), st));
      for (int q : esc_bc) CK(hipMemsetAsync(stat + q, 0, sizeof(int), st));
      const HostOps* keep = hx;
      hx = nullptr;  // the 3-term screens run on the device image
      if (!esc.empty()) pass(&esc, 1, w.qidx_e, w.le_h);
      if (!esc_bc.empty()) pass(&esc_bc, 2, w.qidx_e2, w.le2_h);
      hx = keep;
      int n2 = 0;
      int* h = w.small_h.get(4);
      CK(dmlp::dma_copy(h, ovf, sizeof(int), st));
      CK(hipStreamSynchronize(st));
      n2 = h[0];
      if (n2) {
        CK(hipMemcpyAsync(sh.data(), stat, Q * sizeof(int), hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
        for (int q : esc) if (sh[q]) fq.push_back(q);
        for (int q : esc_bc) if (sh[q]) fq.push_back(q);
      }
    }
    exact_pass(fq);
    n_exact += (int64_t)fq.size();
    n_escalated += (int64_t)(esc.size() + esc_bc.size());
    std::vector<int> r = rest;
    r.insert(r.end(), fq.begin(), fq.end());
    finalize_rest(r);
    return redone;
  }
};

// ---------------------------------------------------------------- dmlp_step
struct Step {
  Ctx& w;
  dmlp_step_args* a;
  hipStream_t st;
  explicit Step(Ctx& c_, dmlp_step_args* a_) : w(c_), a(a_), st((hipStream_t)a_->stream) {}

  hipError_t mark(int i, hipStream_t s) {
    if (!w.marks_on) return hipSuccess;
    w.marks_rec |= 1u << i;
    return hipEventRecord(w.marks[i], s);
  }

  // labels + fp64 rows (X, then Qx) on the side stream: lossless int32 when every value is a
  // 6-decimal number (half the PCIe bytes; the device divides back), else fp64
  void issue_rows_now(double* Xd, double* Qd, int* lab_d) {
    const int64_t N = a->N, Q = a->Q, A = a->A;
    if (a->labels && N) {
      int* lh = w.s_lab.get(N);
      pool_memcpy(lh, a->labels, N * sizeof(int));
      CK(dmlp::dma_copy(lab_d, lh, N * sizeof(int), w.side));
    }
    const int64_t nx = N * A, nqa = Q * A, at = (nx + 3) & ~int64_t(3);  // (16-B aligned)
    auto rows = [&](const double* src, const double* const* tab, int64_t nr, double* dst,
                    int64_t off) {
      const int64_t n = nr * A;
      if (n == 0) return;
      if (rows_i32_on()) {
        int* h32 = w.s_i32.get(at + nqa) + off;
        if ((tab ? dmlp_cpu_rows_i32_rows(tab, nr, (int)A, h32) : dmlp_cpu_rows_i32(src, n, h32)) ==
            0) {
          int* d32 = w.d_i32.get(at + nqa) + off;
          CK(dmlp::dma_copy(d32, h32, n * 4, w.side));
          CKL(dmlp_rows_from_i32(d32, n, dst, w.side));
          return;
        }
      }
      if (tab) {  // not 6-decimal: pack the fp64 rows from the table first
        double* h = w.s_f64.get(at + nqa) + off;
        dmlp_cpu_gather_rows(tab, nr, (int)A, h);
        src = h;
      }
      CK(hipMemcpyAsync(dst, src, n * 8, hipMemcpyHostToDevice, w.side));
    };
    if (a->X32d) {
      // the dataset's rows are on the device already (the xGMI replica): fp64 from them
      if (nx) CKL(dmlp_rows_from_i32(a->X32d, nx, Xd, w.side));
      rows(a->Qx, a->Qr, Q, Qd, at);
    } else if (const dmlp_plane* pl = a->plane) {
      // the dataset's rows through the node render plane: this rank renders its row slices into
      // the segment, its own query rows privately, then copies every slice from the segment
      plane_slices(2, [&](int i, int bits, float) {
        int64_t t0 = 0, t1 = 0;
        dmlp_plane_slice(N, (int)A, i, &t0, &t1);
        const int64_t r0 = std::min<int64_t>(N, t0 * 64), r1 = std::min<int64_t>(N, t1 * 64);
        const int64_t n = (r1 - r0) * A;
        if (n <= 0) return;
        void *r32 = nullptr, *r64 = nullptr;
        CKL(dmlp_plane_regions(pl, N, (int)A, nullptr, nullptr, &r32, &r64));
        if (bits & 2) {  // not 6-decimal: fp64 from the segment, or from the node-shared X
          const double* src = r64 ? (const double*)r64 + r0 * A : a->X ? a->X + r0 * A : nullptr;
          if (!src) throw Fail{-10};
          CK(hipMemcpyAsync(Xd + r0 * A, src, n * 8, hipMemcpyHostToDevice, w.side));
        } else {
          int* d32 = w.d_i32.get(at + nqa) + r0 * A;
          CK(dmlp::dma_copy(d32, (const int*)r32 + r0 * A, n * 4, w.side));
          CKL(dmlp_rows_from_i32(d32, n, Xd + r0 * A, w.side));
        }
      }, [&]() { rows(a->Qx, a->Qr, Q, Qd, at); });
    } else {
      rows(a->X, a->Xr, N, Xd, 0);
      rows(a->Qx, a->Qr, Q, Qd, at);
    }
    CK(hipEventRecord(w.ev_rows, w.side));
    CK(mark(M_ROWS, w.side));
  }

  // The node render plane's slices of kind `what` (1 image, 2 rows): this rank renders its own
  // (i % renderers == rank) and publishes each, then `between` (this rank's private work that
  // needs no other rank), then consumes every slice in order — each as soon as its flag of this
  // call is set (consume(i, bits, nmax): the copies out of the segment).  A wait bounded by the
  // plane's wait_s that expires throws (the call fails; the other ranks' waits expire too).
  template <class F, class G>
  void plane_slices(int what, F&& consume, G&& between) {
    const dmlp_plane* pl = a->plane;
    int64_t t0 = 0, t1 = 0;
    const int ns = dmlp_plane_slice(a->N, a->A, 0, &t0, &t1);
    if (ns <= 0) throw Fail{-9};
    int next = 0;
    auto drain = [&](bool block) {
      while (next < ns) {
        if (!block && !dmlp_plane_ready(pl, what, next)) return;
        int bits = 0;
        float nm = 0.0f;
        if (dmlp_plane_wait(pl, what, next, &bits, &nm) != 0) {
          std::fprintf(stderr, "[dmlp] plane rank %d: no slice %d (kind %d) of call %lld from rank %d\n",
                       pl->rank, next, what, (long long)pl->gen, next % std::max(1, pl->renderers));
          throw Fail{-9};
        }
        consume(next, bits, nm);
        ++next;
      }
    };
    if (pl->rank < pl->renderers)
      for (int i = pl->rank; i < ns; i += std::max(1, pl->renderers)) {
        if (dmlp_plane_render(pl, a->X, a->Xr, a->N, a->A, w.s_mu.p, what, i) < 0) throw Fail{-9};
        drain(false);
      }
    between();
    drain(true);
  }

  int run() {
    const int64_t N = a->N, Q = a->Q;
    const int A = a->A;
    const auto t_enter = std::chrono::steady_clock::now();
    a->host_ms = 0.0f;
    a->report_len = 0;
    a->path = 0;
    a->early = 0;
    a->n_escalated = 0;
    a->early_waits = a->early_grows = a->early_timeouts = 0;
    w.marks_valid = false;
    w.marks_rec = 0;
    w.text_len = 0;  // dmlp_step_emit copies only what THIS call rendered
    if (Q < 0 || N < 0 || A < 1 || Q > (1 << 30)) return -1;
    const dmlp_plane* pl = a->plane;
    if (pl && (!pl->base || pl->rank < 0 || pl->renderers < 1 || pl->gen <= 0 ||
               dmlp_plane_bytes(N, A, pl->with_f64) < 0 ||
               pl->bytes < dmlp_plane_bytes(N, A, pl->with_f64)))
      return -1;
    // (a plane rank that renders no slice needs no dataset rows: the engine.h drop-in's ranks > 0)
    const bool need_x = N > 0 && (!pl || pl->rank < pl->renderers);
    if ((a->X == nullptr && a->Xr == nullptr && need_x) || (a->Qx == nullptr && a->Qr == nullptr && Q > 0) ||
        (Q > 0 && !a->k))
      return -1;
    const bool want_report = a->report_mode != 0 && a->labels;
    if (a->report_mode == 1 && a->report_cap < dmlp_format_bound((int)Q)) return -2;
    CK(mark(M_ENTER, w.side));
    // the caller's stream may hold work on the buffers of the previous call: the side stream's
    // copies into them start after it
    CK(hipEventRecord(w.ev_ops, st));
    CK(hipStreamWaitEvent(w.side, w.ev_ops, 0));
    int kmin = a->kmin, kmax = a->kmax;
    if (Q > 0 && kmax < kmin) {  // k bounds not given: one pass on the render pool
      dmlp_host_i32_range(a->k, Q, &kmin, &kmax);
      a->kmin = kmin;
      a->kmax = kmax;
    }
    if (a->labels && a->label_hi <= a->label_lo) {  // label range not given: the same
      int lmin = 0, lmax = -1;
      if (N > 0) dmlp_host_i32_range(a->labels, N, &lmin, &lmax);
      a->label_lo = N > 0 ? lmin : 0;
      a->label_hi = N > 0 ? lmax + 1 : 1;
    }
    const int kst = a->kstride > 0 ? a->kstride : std::max(1, Q ? kmax : 1);
    if (Q > 0 && kmax > kst) return -3;
    const int KT = dmlp_screen_kt(A);
    const int64_t nt = (N + 63) / 64, W = (int64_t)KT * 32;
    // outputs (the caller's device tensors, or workspace)
    double* od = a->out_d ? a->out_d : w.d_od.get((size_t)std::max<int64_t>(Q, 1) * kst);
    int* oi = a->out_i ? a->out_i : w.d_oi.get((size_t)std::max<int64_t>(Q, 1) * kst);
    int* olab = a->out_lab ? a->out_lab : w.d_lb.get(Q);
    uint64_t* ocs = a->out_cs ? a->out_cs : w.d_cs.get(Q);
    double* Xd = w.d_X.get((size_t)std::max<int64_t>(N, 1) * A);
    double* Qd = w.d_Q.get((size_t)std::max<int64_t>(Q, 1) * A);
    int* lab_d = a->labels ? w.d_lab.get(N) : nullptr;
    // (with a plane every rank must take the same front: not a function of its own pool size)
    const bool x1_front = !a->exact && N > 0 && KT <= 8 && dmlp_screen_x1_qw(KT) > 0 &&
                          g_tune.screen == 0 &&
                          (g_tune.host_ops >= 2 ||
                           (g_tune.host_ops == 1 &&
                            (pl || dr_on() || dr_auto(N, A) || dmlp_host_threads() >= 2)));
    // device render (opt-in, DMLP_DEVICE_RENDER=1): the GPU renders the screen operands from the
    // landed rows.  With a plane every rank must render the same slice kinds, so a plane step
    // always renders on the host (a device-render rank never renders its image slices)
    bool dr = x1_front && !pl && (dr_on() || dr_auto(N, A));
    if (Q == 0) {
      a->report_len = 0;
      w.text_len = 0;
      // no queries here, but this rank's share of the node render plane is still owed
      if (pl && pl->rank < pl->renderers && N > 0) {
        double* mu = w.s_mu.get(A);
        if (x1_front) {
          if (pl->rank == 0) {
            if (a->Xr) dmlp_cpu_center_rows(a->Xr, std::min<int64_t>(N, 4096), A, mu);
            else dmlp_cpu_center(a->X, std::min<int64_t>(N, 4096), A, mu);
            CKL(dmlp_plane_put_mu(pl, A, mu));
          } else if (dmlp_plane_get_mu(pl, A, mu) != 0) {
            throw Fail{-9};
          }
        }
        render_plane_share(mu, x1_front ? 1 : 2, a->X32d ? 1 : 2);
      }
      return 0;
    }
    const bool all_a = kmin >= 1 && kmax <= dmlp_screen_x1_kmax() && kmax <= N;
    // early_room: the early screen's waves spin while the image copies land, and on this runtime
    // small host->device copies are blit KERNELS that need a free wave slot beside them.
    const bool early = x1_front && all_a && early_on() && early_room(KT, kmax) && nt >= 2 &&
                       nt <= 4096 && x1_slices((int)Q, KT, kmax, nt) == 1;
    // an early-start shape whose screen leaves the render kernels no room: the host render
    if (early && !dr_early_ok(KT, kmax)) dr = false;
    const int NS = early ? (int)std::min<int64_t>(kEarlySlices, nt) : 0;
    const int rt = early ? (int)((nt + NS - 1) / NS) : 1;  // image tiles per early slice
    unsigned* words = w.dwords.get(kW_N);
    unsigned* rdy = words + kW_RDY;
    unsigned* estats = words + kW_EST;
    HostOps hx;
    bool use_hx = false, early_bad = false;
    // ---- the step's words (norm, bad, ready words, counters, overflow) zeroed by one DMA copy, and
    // on the all-class-a path k on the device — both on the side stream ahead of the operands,
    // so nothing sits on `st` between the operands' event and the screen
    CK(dma_zero(words, kW_N * sizeof(unsigned), w.side));
    int* kd_pre = nullptr;
    if (x1_front && all_a) {
      int* kh = w.kk_h.get(Q);
      pool_memcpy(kh, a->k, Q * sizeof(int));
      kd_pre = w.kdev.get(Q);
      CK(dmlp::dma_copy(kd_pre, kh, Q * sizeof(int), w.side));
    }
    // ---- device render: the rows (lossless int32, fp64 where a block is not 6-decimal) cross
    // PCIe on the side stream, the query block first, then the dataset, each block followed by its
    // render kernel (prep.hip k_render: the fp64 rows for the re-rank, the fp16 image / query
    // fragments, the norms).  The large-N pipeline (every k in class a): the dataset in up to 8
    // chunks of the screen's S slices, each chunk's event recorded behind its render, so the
    // screen of chunk c runs while chunk c + 1 crosses PCIe (Local::pass); the labels last (only
    // the vote reads them).  Otherwise one chunk, and every screen waits for all of it.
    // Each chunk's screen launch must fill the GPU by itself, so the pipeline splits the scan into
    // kPipeChunks x the slices one launch needs (x1_slices) — more (query, slice) lists for the
    // refine, each chunk's screen at full occupancy (one slice per chunk ran at 1/8 of the chip:
    // profiles/r10d_large_n_pipeline.txt)
    constexpr int kPipeChunks = 4;
    int S_all = 0, n_chunks = 1;
    if (dr && x1_front && all_a) {
      const int S1 = x1_slices((int)Q, KT, kmax, nt);
      int64_t S_cap = std::min<int64_t>(256, nt / 16);  // (refine: <= 256 slices; >= 16 tiles each)
      if (kmax > 32) S_cap = std::min<int64_t>(S_cap, nt * 64 / (32 * kmax));
      S_all = (int)std::max<int64_t>(S1, std::min<int64_t>((int64_t)S1 * kPipeChunks, S_cap));
      n_chunks = std::min(kEarlySlices, std::max(1, S_all / S1));
    }
    int chunk_s[kEarlySlices + 1] = {0};
    for (int c = 0; c <= n_chunks; ++c)
      chunk_s[c] = (int)((int64_t)std::max(1, S_all) * c / n_chunks);
    const int64_t dr_at = (N * A + 3) & ~int64_t(3);  // (16-B aligned)
    int* h32 = nullptr;
    int* d32 = nullptr;
    // rows [r0, r1) of X (or Qx) -> int32 staging at h32 + off + r0 A, else fp64; returns the
    // render's source (device int32 base or the device fp64 rows)
    auto ship = [&](const double* src, const double* const* tab, int64_t r0, int64_t r1,
                      int64_t off, double* dst64, const int** s32, const double** s64) {
        const int64_t n = (r1 - r0) * A;
        *s32 = nullptr;
        *s64 = nullptr;
        if (n <= 0) return;
        if (rows_i32_on() &&
            (tab ? dmlp_cpu_rows_i32_rows(tab + r0, r1 - r0, A, h32 + off + r0 * A)
                 : dmlp_cpu_rows_i32(src + r0 * A, n, h32 + off + r0 * A)) == 0) {
          CK(dmlp::dma_copy(d32 + off + r0 * A, h32 + off + r0 * A, n * 4, w.side));
          *s32 = d32 + off;
          return;
        }
        const double* from = src ? src + r0 * A : nullptr;
        if (tab) {
          double* h = w.s_f64.get(dr_at + Q * A) + off + r0 * A;
          dmlp_cpu_gather_rows(tab + r0, r1 - r0, A, h);
          from = h;
        }
        CK(hipMemcpyAsync(dst64 + r0 * A, from, n * 8, hipMemcpyHostToDevice, w.side));
        *s64 = dst64;
    };
    // what: 0 the queries, 1 + c dataset chunk c, -1 the labels and the rows' event (the tail)
    std::function<void(int)> dr_part = [&](int what) {
        const int64_t nqa = Q * A, at = dr_at;
        unsigned* drw = w.dr_words.p;
        unsigned* rbad = drw + 72;
        const double* mud = w.d_mu.p;
        short* xhi_d = (short*)const_cast<void*>(hx.xhi);
        float* xin_d = const_cast<float*>(hx.xin);
        h32 = w.s_i32.get(dr_at + nqa);
        d32 = w.d_i32.get(dr_at + nqa);
        if (what == 0) {
          const int* s32;
          const double* s64;
          ship(a->Qx, a->Qr, 0, Q, at, Qd, &s32, &s64);
          CKL(dmlp_render_rows(KT, A, s32, s64, 0, Q, Q, mud, Qd, 1, w.dq_hi.p, w.dq_n.p, nullptr,
                               nullptr, rbad, drw + 8, nullptr, w.side));
          CK(mark(M_OPS, w.side));
          if (S_all > 0) CK(hipEventRecord(w.ev_ops, w.side));  // (the pipeline's screens: + chunk)
          return;
        }
        if (what > 0) {  // slices [chunk_s[c], chunk_s[c + 1]) of S_all, tiles of tps each
          const int c = what - 1;
          const int64_t tps = S_all > 0 ? (nt + S_all - 1) / S_all : nt;
          const int64_t t0 = std::min<int64_t>(nt, chunk_s[c] * tps);
          const int64_t t1 = std::min<int64_t>(nt, chunk_s[c + 1] * tps);
          if (t1 > t0) {
            const int* s32 = a->X32d;  // (the xGMI replica: rendered straight from the device)
            const double* s64 = nullptr;
            if (!s32) ship(a->X, a->Xr, std::min(N, t0 * 64), std::min(N, t1 * 64), 0, Xd, &s32, &s64);
            CKL(dmlp_render_rows(KT, A, s32, s64 ? s64 : s32 ? nullptr : Xd, t0 * 64,
                                 (t1 - t0) * 64, N, mud, Xd, 0, xhi_d, xin_d,
                                 const_cast<void*>(hx.xrow), words + kW_XNMAX, rbad, drw + c,
                                 nullptr, w.side));
          }
          CK(hipEventRecord(w.ev_chunk[c], w.side));
          return;
        }
        CK(mark(M_DATA, w.side));
        if (a->labels && N) {
          int* lh = w.s_lab.get(N);
          pool_memcpy(lh, a->labels, N * sizeof(int));
          CK(dmlp::dma_copy(lab_d, lh, N * sizeof(int), w.side));
        }
        CK(hipEventRecord(w.ev_rows, w.side));
        CK(mark(M_ROWS, w.side));
    };
    // ---- front: the host renders the single-term screen's fp16 operands
    if (x1_front) {
      uint16_t* xhi_h = w.sx_hi.get(nt * 64 * W);
      float* xin_h = w.sx_in.get(nt * 64);
      unsigned* xnm_h = w.sx_nm.get(2 + kEarlySlices);
      uint16_t* qhi_h = w.sq_hi.get(Q * W);
      float* qn_h = w.sq_n.get(Q);
      double* mu = w.s_mu.get(A);
      short* xhi = w.dx_hi.get(nt * 64 * W);
      float* xin = w.dx_in.get(nt * 64);
      short* qhi = w.dq_hi.get(Q * W);
      float* qn = w.dq_n.get(Q);
      if (pl && pl->rank != 0) {
        if (dmlp_plane_get_mu(pl, A, mu) != 0) throw Fail{-9};  // rank 0's centre, same bits
      } else {
        if (a->Xr) dmlp_cpu_center_rows(a->Xr, std::min<int64_t>(N, 4096), A, mu);
        else dmlp_cpu_center(a->X, std::min<int64_t>(N, 4096), A, mu);
        if (pl) CKL(dmlp_plane_put_mu(pl, A, mu));
      }
      auto h2d_tiles = [&](int64_t t0, int64_t t1, const double* qx, const double* const* qr,
                           int64_t nq, unsigned* xnm_hw, void* xhi_d, void* xin_d, void* xnm_d,
                           void* qhi_d, void* qn_d, int chunks) {
        return a->Xr || a->Qr
                   ? dmlp_host_ops_h2d_tiles_rows(a->Xr, N, t0, t1, qr, nq, A, mu, KT, xhi_h, xin_h,
                                                  xnm_hw, qhi_h, qn_h, xhi_d, xin_d, xnm_d, qhi_d,
                                                  qn_d, chunks, w.side)
                   : dmlp_host_ops_h2d_tiles(a->X, N, t0, t1, qx, nq, A, mu, KT, xhi_h, xin_h,
                                             xnm_hw, qhi_h, qn_h, xhi_d, xin_d, xnm_d, qhi_d, qn_d,
                                             chunks, w.side);
      };
      int rc;
      if (dr) {
        // the centre on the device; the render counters cleared; the rows and the render precede
        // each chunk's screen (device render never starts early)
        double* mud = w.d_mu.get(A);
        CK(dmlp::dma_copy(mud, mu, A * sizeof(double), w.side));
        CK(dma_zero(w.dr_words.get(80), 80 * sizeof(unsigned), w.side));
        // (the pair refine's point-major image: one screen slice only)
        if (KT <= 2 && rowmajor_on() && S_all <= 1) hx.xrow = w.dx_row.get(nt * 64 * W);
        hx.xhi = xhi;
        hx.xin = xin;
        dr_part(0);
        if (S_all > 0) {  // the pipeline: each chunk issued by the screen pass, then its screen
          hx.chunk_n = n_chunks;
          hx.chunk_S = S_all;
          hx.chunk_s = chunk_s;
          hx.chunk_ev = w.ev_chunk;
          hx.issue_chunk = [&](int c) { dr_part(1 + c); };
        } else {  // every chunk and the tail now: the screens wait for all of it
          for (int c = 0; c < n_chunks; ++c) dr_part(1 + c);
          dr_part(-1);
        }
        rc = 0;
      } else if (early) {
        // query operands first (the whole front of the step); the image follows the screen's launch
        rc = h2d_tiles(nt, nt, a->Qx, a->Qr, Q, xnm_h + 1, xhi, xin, nullptr, qhi, qn,
                       early_qchunks());
      } else if (pl) {
        // this rank's query operands, then the dataset image from the node render plane; the
        // image's max norm (+inf when a slice is outside the fp16 range) into words[XNMAX]
        rc = h2d_tiles(nt, nt, a->Qx, a->Qr, Q, xnm_h + 1, xhi, xin, nullptr, qhi, qn,
                       host_slices());
        float mx = 0.0f;
        if (plane_image(xhi, xin, nullptr, &mx)) rc |= 1;
        std::memcpy(xnm_h, &mx, 4);
        CK(dmlp::dma_copy(words + kW_XNMAX, xnm_h, 4, w.side));
        CK(mark(M_DATA, w.side));
      } else {
        rc = h2d_tiles(0, nt, a->Qx, a->Qr, Q, xnm_h, xhi, xin, words + kW_XNMAX, qhi, qn,
                       host_slices());
        CK(mark(M_DATA, w.side));
      }
      if (rc & 4) throw Fail{-(int)hipErrorUnknown};
      if (rc != 0 && pl && early) {
        // this rank falls back to the device image path (its queries are outside the fp16
        // range), but its share of the plane's image slices is still owed to the other ranks
        // (its row slices follow in issue_rows_now as usual)
        render_plane_share(mu, 1, 1);
      }
      if (rc == 0) {
        if (!dr) CK(mark(M_OPS, w.side));
        if (!dr || S_all == 0) CK(hipEventRecord(w.ev_ops, w.side));
        CK(hipStreamWaitEvent(st, w.ev_ops, 0));
        hx.xhi = xhi;
        hx.xin = xin;
        hx.words = words;
        hx.qhi = qhi;
        hx.qn = qn;
        if (early) {
          hx.rdy = rdy;
          hx.rdy_tiles = rt;
          hx.rdy_n = NS;
          hx.estats = estats;
        }
        use_hx = true;
        a->early = early ? 1 : 0;
      }
      // (rc != 0: data or queries outside the fp16 screen's range -> the device image path)
    }
    char* text = want_report ? w.d_text.get((size_t)dmlp_format_bound((int)Q)) : nullptr;
    // ---- dispatch: screens on `st`, the rows behind the first of them on the side stream
    auto run_local = [&](bool with_hx, bool rows_pending) {
      std::unique_ptr<Local> Lp(new Local(w));
      Local& L = *Lp;
      L.X = Xd; L.N = N; L.A = A; L.Qx = Qd; L.Q = Q; L.k_host = a->k; L.kstride = kst;
      L.out_d = od; L.out_i = oi; L.labels = lab_d; L.lo = a->label_lo; L.hi = a->label_hi;
      L.lab = olab; L.cs = ocs; L.exact = a->exact != 0; L.st = st;
      L.hx = with_hx ? &hx : nullptr;
      L.rows = w.ev_rows;
      if (with_hx && kd_pre) {
        // (the words' zero copy and k's copy precede the operands' event on the side stream)
        L.kd_pre = kd_pre;
        L.kk_pre = w.kk_h.p;
        L.all_a_pre = true;
        L.kmax_pre = kmax;
        L.ovf_pre = (int*)(words + kW_OVF);
      }
      if (rows_pending) {
        L.issue_rows = [&]() {
          // (host operands: called right after the first screen launch, so this mark completes
          // when it does; the device path calls it before its image is built: no mark)
          if (with_hx) CK(mark(M_SCREEN, st));
          if (dr) {  // device render: the rows and their render are queued; the pipeline's tail
            if (S_all > 0) dr_part(-1);
            return;
          }
          if (with_hx && hx.rdy) {
            // the dataset image behind the queries, slice by slice, each followed by its ready
            // word (the slice's norm bits: the running screen waits on it); every word is
            // written even when a slice is outside the fp16 range, so the screen always drains
            const int dly = early_delay_us();
            if (pl) {
              if (plane_image(hx.xhi, hx.xin, rdy, nullptr)) early_bad = true;
            } else {
              for (int i = 0; i < NS; ++i) {
                if (dly) std::this_thread::sleep_for(std::chrono::microseconds(dly));
                const int64_t t0 = (int64_t)i * rt, t1 = std::min<int64_t>(nt, t0 + rt);
                const int r2 = h2d_tiles_data(t0, t1, i);
                if (r2 & 4) throw Fail{-(int)hipErrorUnknown};
                if (r2) early_bad = true;
              }
            }
            CK(mark(M_DATA, w.side));
          }
          if (with_hx && KT <= 2 && rowmajor_on()) {
            // the pair refine's point-major image, behind the whole image on the side stream
            // (the re-rank waits for the rows' event recorded after it)
            short* xr = w.dx_row.get(nt * 64 * W);
            CKL(dmlp_x1_rowmajor(hx.xhi, nt, KT, xr, w.side));
            hx.xrow = xr;
          }
          issue_rows_now(Xd, Qd, lab_d);
        };
      }
      L.launch();
      return Lp;
    };
    hx_ = &hx;
    std::unique_ptr<Local> Lp = run_local(use_hx, true);
    if (early_bad) {
      // a dataset slice outside the fp16 range behind a running early screen: drain, then the
      // device image path over the rows that are already on their way
      CK(hipStreamSynchronize(w.side));
      CK(hipStreamSynchronize(st));
      a->early = 0;
      use_hx = false;
      Lp = run_local(false, false);
    }
    // ---- the report behind the re-rank, then the one host sync.  The small results (report
    // length, overflow count, early-start counters) are packed on the device and cross in ONE
    // DMA copy: each separate small D2H cost a copy command's latency on the step's tail.
    int64_t* small = w.small64_h.get(8);
    int64_t* small_d = w.small64_d.get(8);
    unsigned* dr_bad = dr ? w.dr_words.p + 72 : nullptr;  // device render: a value out of range
    auto render = [&]() {
      const int64_t* len_src = nullptr;
      if (want_report) {
        int64_t* off = w.d_off.get((size_t)dmlp_format_scratch((int)Q));
        CKL(dmlp_format_report(ocs, (int)Q, (int)a->qid_base, off, text, st));
        CK(mark(M_FORMAT, st));
        len_src = off + Q;
      }
      hipLaunchKernelGGL(k_pack_small, dim3(1), dim3(64), 0, st, len_src, Lp->ovf,
                         a->early ? estats : nullptr, dr_bad, small_d);
      CK(hipGetLastError());
      CK(dmlp::dma_copy(small, small_d, 8 * sizeof(int64_t), st));
      if (want_report && a->report_mode == 1)
        CK(dmlp::dma_copy(a->report_dst, w.d_text.p, (size_t)dmlp_format_bound((int)Q), st));
    };
    a->host_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t_enter)
                     .count();
    CK(mark(M_REFINE, st));
    render();
    CK(mark(M_D2H, st));
    CK(hipEventRecord(w.ev_done, st));
    spin_wait(w.ev_done);
    CK(hipStreamSynchronize(w.side));
    w.marks_valid = w.marks_on;
    if (dr_bad && small[6]) {
      // device render: some fp64 value lies outside the fp16 screen's range, so the screen ran on
      // an unusable image — the whole call again on the device image path over the fp64 rows,
      // which are complete on the device
      a->early = 0;
      use_hx = false;
      dr_bad = nullptr;
      w.marks_valid = false;
      Lp = run_local(false, false);
      render();
      CK(hipEventRecord(w.ev_done, st));
      spin_wait(w.ev_done);
    }
    if (a->early) {
      a->early_waits = (int)small[2];
      a->early_grows = (int)small[3];
      a->early_timeouts = (int)small[4];
      if (small[4] && g_early != 0) {
        std::fprintf(stderr, "[dmlp] early start: %d screen wave(s) timed out waiting for the "
                     "dataset image (overflowed queries were escalated); early start is off for "
                     "the rest of this process\n", (int)small[4]);
        g_early = 0;
      }
    }
    const int novf = (int)small[1];
    if (novf) {
      a->n_escalated = Lp->finish(novf);
      w.marks_valid = false;
      render();
      CK(hipStreamSynchronize(st));
    }
    if (want_report) {
      a->report_len = small[0];
      w.text_len = a->report_len;
    }
    if (!use_hx) a->path = 2;
    g_stats.n_exact = Lp->n_exact;
    g_stats.n_escalated = Lp->n_escalated;
    g_stats.path = a->path;
    g_stats.early = a->early;
    g_stats.device_render = dr && use_hx ? 1 : 0;
    return 0;
  }

  // This rank's share of the node render plane's slices of kinds [what_lo, what_hi] (1 image,
  // 2 rows; i % renderers == rank), rendered and published without consuming any.
  void render_plane_share(const double* mu, int what_lo, int what_hi) {
    const dmlp_plane* pl = a->plane;
    if (!pl || pl->rank >= pl->renderers || a->N <= 0) return;
    int64_t t0 = 0, t1 = 0;
    const int ns = dmlp_plane_slice(a->N, a->A, 0, &t0, &t1);
    for (int what = what_lo; what <= what_hi; ++what)
      for (int i = pl->rank; i < ns; i += pl->renderers)
        if (dmlp_plane_render(pl, a->X, a->Xr, a->N, a->A, mu, what, i) < 0) throw Fail{-9};
  }

  // The dataset image from the node render plane: every slice (rendered by this rank or another)
  // copied from the segment into the device image xhi / xin on the side stream.  Early start
  // (rdy != null): each slice's ready word (its norm bits) behind its copies.  Else the max over
  // the slices -> *mx.  Returns 1 when some slice is outside the fp16 range.
  int plane_image(const void* xhi, const float* xin, unsigned* rdy, float* mx) {
    const dmlp_plane* pl = a->plane;
    const int64_t N = a->N;
    const int A = a->A;
    const int64_t W = (int64_t)dmlp_screen_kt(A) * 32;
    void *img = nullptr, *xi = nullptr;
    CKL(dmlp_plane_regions(pl, N, A, &img, &xi, nullptr, nullptr));
    unsigned* nh = w.sx_nm.get(2 + kEarlySlices);  // [2 + i] slice i's ready word
    const int dly = rdy ? early_delay_us() : 0;
    int bad = 0;
    float m = 0.0f;
    plane_slices(1, [&](int i, int bits, float nm) {
      if (dly) std::this_thread::sleep_for(std::chrono::microseconds(dly));
      int64_t t0 = 0, t1 = 0;
      dmlp_plane_slice(N, A, i, &t0, &t1);
      if (t1 > t0) {
        CK(dmlp::dma_copy((short*)const_cast<void*>(xhi) + t0 * 64 * W,
                          (const uint16_t*)img + t0 * 64 * W, (t1 - t0) * 64 * W * 2, w.side));
        CK(dmlp::dma_copy(const_cast<float*>(xin) + t0 * 64, (const float*)xi + t0 * 64,
                          (t1 - t0) * 64 * 4, w.side));
      }
      bad |= bits & 1;
      m = std::max(m, nm);
      if (rdy) {
        nh[2 + i] = ready_bits(nm);
        CK(dmlp::dma_copy(rdy + i, nh + 2 + i, 4, w.side));
      }
    }, [] {});
    if (mx) *mx = bad ? INFINITY : m;
    return bad;
  }

  // early start: dataset image tiles [t0, t1) = slice i rendered on the host and copied, then its
  // ready word (the slice's max norm bits; +inf when outside the fp16 range)
  int h2d_tiles_data(int64_t t0, int64_t t1, int i) {
    const int64_t W = (int64_t)dmlp_screen_kt(a->A) * 32;
    double* mu = w.s_mu.p;
    unsigned* xnm_h = w.sx_nm.p + 2 + i;
    short* xhi = (short*)const_cast<void*>(hx_->xhi) + t0 * 64 * W;
    float* xin = const_cast<float*>(hx_->xin) + t0 * 64;
    const int KT = dmlp_screen_kt(a->A);
    const int rc =
        a->Xr ? dmlp_host_ops_h2d_tiles_rows(a->Xr, a->N, t0, t1, nullptr, 0, a->A, mu, KT,
                                             w.sx_hi.p, w.sx_in.p, xnm_h, w.sq_hi.p, w.sq_n.p, xhi,
                                             xin, nullptr, w.dq_hi.p, w.dq_n.p, 1, w.side)
              : dmlp_host_ops_h2d_tiles(a->X, a->N, t0, t1, nullptr, 0, a->A, mu, KT, w.sx_hi.p,
                                        w.sx_in.p, xnm_h, w.sq_hi.p, w.sq_n.p, xhi, xin, nullptr,
                                        w.dq_hi.p, w.dq_n.p, 1, w.side);
    if (!(rc & 4)) {
      float nm;
      std::memcpy(&nm, xnm_h, 4);
      *xnm_h = ready_bits(nm);
      CK(dmlp::dma_copy(const_cast<unsigned*>(hx_->rdy) + i, xnm_h, 4, w.side));
    }
    return rc;
  }
  const HostOps* hx_ = nullptr;  // (run(): the host operands of the early start)
};

int drain_and_fail(Ctx* w, hipStream_t st, int code) {
  // every error path drains the streams before returning: nothing may still be writing the
  // caller's tensors or reading the page-locked staging when it frees or reuses them
  if (w && w->side) (void)hipStreamSynchronize(w->side);
  if (st) (void)hipStreamSynchronize(st);
  (void)hipGetLastError();
  return code;
}

}  // namespace

// ---------------------------------------------------------------- C API
extern "C" int dmlp_arena_reserve(int64_t dev_bytes, int64_t host_bytes) {
  int rc = 0;
  if (dev_bytes > 0 && !g_dev.base) {
    void* p = nullptr;
    if (hipMalloc(&p, (size_t)dev_bytes) == hipSuccess) {
      g_dev.base = (char*)p;
      g_dev.size = (size_t)dev_bytes;
      if (hipGetDevice(&g_dev.dev) != hipSuccess) g_dev.dev = -1;
    } else {
      rc |= 1;
    }
  }
  if (host_bytes > 0 && !g_host.base) {
    void* p = nullptr;
    if (hipHostMalloc(&p, (size_t)host_bytes, hipHostMallocDefault) == hipSuccess) {
      g_host.base = (char*)p;
      g_host.size = (size_t)host_bytes;
      // touch every page and move every byte once in each direction now, not inside the timed
      // call: the first DMA into a host range pays its mapping (~7 ms for 6 MB measured)
      for (size_t o = 0; o < g_host.size; o += 4096) g_host.base[o] = 0;
      const size_t chunk = std::min<size_t>(g_host.size, size_t(64) << 20);
      char* d = nullptr;
      if (hipMalloc((void**)&d, chunk) == hipSuccess) {
        for (size_t o = 0; o < g_host.size; o += chunk) {
          const size_t n = std::min(chunk, g_host.size - o);
          (void)hipMemcpy(d, g_host.base + o, n, hipMemcpyHostToDevice);
          (void)hipMemcpy(g_host.base + o, d, n, hipMemcpyDeviceToHost);
        }
        (void)hipFree(d);
      }
    } else {
      rc |= 2;
    }
  }
  return rc;
}
extern "C" void* dmlp_dev_alloc(int64_t bytes) { return dev_alloc((size_t)std::max<int64_t>(bytes, 1)); }
extern "C" void dmlp_dev_free(void* p) { dev_free(p); }
extern "C" void* dmlp_host_alloc(int64_t bytes) { return host_alloc((size_t)std::max<int64_t>(bytes, 1)); }
extern "C" void dmlp_host_free(void* p) { host_free(p); }

extern "C" int dmlp_knn_local(const double* X, int64_t N, int A, const double* Qx, int64_t Q,
                              const int* k, int kstride, double* out_d, int* out_i,
                              const int* labels, int label_lo, int label_hi, int* out_label,
                              uint64_t* out_cs, int exact, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  Ctx* wp = nullptr;
  try {
    if (Q < 0 || N < 0 || A < 1 || kstride < 1 || Q > (1 << 30)) return -1;
    if (Q == 0) return 0;
    // every query's list (min(k, N) entries) must fit its row of out_d / out_i (as dmlp_step)
    for (int64_t q = 0; q < Q; ++q)
      if (std::min<int64_t>(k[q], N) > kstride) return -3;
    Ctx& w = ctx();
    wp = &w;
    Local L(w);
    L.X = X; L.N = N; L.A = A; L.Qx = Qx; L.Q = Q; L.k_host = k; L.kstride = kstride;
    L.out_d = out_d; L.out_i = out_i; L.labels = labels; L.lo = label_lo; L.hi = label_hi;
    L.lab = out_label; L.cs = out_cs; L.exact = exact != 0; L.st = st;
    L.launch();
    int* h = w.small_h.get(8);
    CK(dmlp::dma_copy(h, L.ovf, sizeof(int), st));
    CK(hipStreamSynchronize(st));
    L.finish(h[0]);
    g_stats.n_exact = L.n_exact;
    g_stats.n_escalated = L.n_escalated;
    g_stats.path = 2;
    g_stats.early = 0;
    g_stats.device_render = 0;
    return 0;
  } catch (const Fail& f) {
    return drain_and_fail(wp, st, f.code);
  } catch (const std::bad_alloc&) {
    return drain_and_fail(wp, st, -(int)hipErrorOutOfMemory);
  }
}

extern "C" int dmlp_step(dmlp_step_args* a) {
  if (!a) return -1;
  hipStream_t st = (hipStream_t)a->stream;
  Ctx* wp = nullptr;
  try {
    Ctx& w = ctx();
    wp = &w;
    Step s(w, a);
    return s.run();
  } catch (const Fail& f) {
    return drain_and_fail(wp, st, f.code);
  } catch (const std::bad_alloc&) {
    return drain_and_fail(wp, st, -(int)hipErrorOutOfMemory);
  }
}

// The last dmlp_step's report bytes (report_mode 2: kept on the device) -> dst (page-locked or
// registered host memory), synchronously.
extern "C" int dmlp_step_emit(char* dst, int64_t bytes, void* stream) {
  try {
    Ctx& w = ctx();
    if (bytes < 0 || bytes > w.text_len) return -1;
    if (bytes == 0) return 0;
    CK(dmlp::dma_copy(dst, w.d_text.p, (size_t)bytes, (hipStream_t)stream));
    CK(hipStreamSynchronize((hipStream_t)stream));
    return 0;
  } catch (const Fail& f) {
    return f.code;
  }
}

// The last dmlp_step's report text on the device (report_mode 2) and its length: a caller that
// streams it out in pieces (the drop-in's chunked egress to stdout) copies the pieces itself.
extern "C" int dmlp_step_text(const char** dev, int64_t* len) {
  try {
    Ctx& w = ctx();
    *dev = w.d_text.p;
    *len = w.text_len;
    return 0;
  } catch (const Fail& f) {
    return f.code;
  }
}

// Right before a timed call after a long idle stretch (the reference harness parses its input
// for seconds, then constructs the Engine, untimed, and starts its clock: common.cpp:119-124):
// wake the render pool (its workers then spin into the call instead of sleeping on a futex),
// touch the page-locked staging of the last call, and keep the GPU busy for gpu_us so its clocks
// are up.  Synchronous.
extern "C" int dmlp_step_prewarm(int gpu_us) {
  try {
    Ctx& w = ctx();
    dmlp_host_pool_run([](void*, int, int) {}, nullptr);
    volatile char sink = 0;
    for (HBuf<int>* b : {&w.s_i32, &w.s_lab})
      if (b->p)
        for (size_t o = 0; o < b->n * sizeof(int); o += 4096) sink += ((volatile char*)b->p)[o];
    (void)sink;
    if (gpu_us > 0) {
      int dev = 0, khz = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0)
        khz = 100000;
      hipLaunchKernelGGL(k_busy, dim3(256), dim3(64), 0, w.side, (long long)gpu_us * khz / 1000);
      CK(hipGetLastError());
      CK(hipStreamSynchronize(w.side));
    }
    dmlp_host_pool_run([](void*, int, int) {}, nullptr);
    return 0;
  } catch (const Fail& f) {
    return f.code;
  }
}

// Early start of the following calls (1 on, 0 off, < 0: back to DMLP_FAST_EARLY); the host delay
// before each dataset image slice in microseconds (< 0: back to DMLP_FAST_EARLY_DELAY_US).
extern "C" void dmlp_step_early(int on) { g_early = on < 0 ? -1 : (on ? 1 : 0); }
extern "C" void dmlp_step_early_delay(int us) { g_early_delay_us = us < 0 ? -1 : us; }

// Step-timeline marks of dmlp_step (hipEvents with timing; off by default).
extern "C" int dmlp_step_events(int on) {
  try {
    Ctx& w = ctx();
    if (on && !w.marks[0])
      for (int i = 0; i < M_N; ++i)
        if (hipEventCreate(&w.marks[i]) != hipSuccess) return -1;
    w.marks_on = on != 0 && w.marks[0];
    return 0;
  } catch (const Fail& f) {
    return f.code;
  }
}

// The last call's marks as ms since it entered: names[i] / ms[i] for i < the returned count.
extern "C" int dmlp_step_timeline(double* ms, const char** names, int cap) {
  try {
    Ctx& w = ctx();
    if (!w.marks_valid) return 0;
    int n = 0;
    for (int i = 0; i < M_N && n < cap; ++i) {
      if (!(w.marks_rec & (1u << i))) continue;  // (never recorded: would leave a sticky error)
      float t = 0.0f;
      if (hipEventElapsedTime(&t, w.marks[M_ENTER], w.marks[i]) != hipSuccess) {
        (void)hipGetLastError();
        continue;
      }
      ms[n] = t;
      names[n] = kMarkNames[i];
      ++n;
    }
    return n;
  } catch (const Fail&) {
    return 0;
  }
}

// Tuning / A-B switches (see Tuning): "num_cus", "screen", "x1k", "host_ops", "device_render".
// Returns the previous value, or -1 for an unknown key.
extern "C" int dmlp_pipeline_set(const char* key, int value) {
  const std::string k = key ? key : "";
  int* f = k == "num_cus" ? &g_tune.num_cus : k == "screen" ? &g_tune.screen
           : k == "x1k" ? &g_tune.x1k : k == "host_ops" ? &g_tune.host_ops
           : k == "device_render" ? &g_tune.device_render : nullptr;
  if (!f) return -1;
  const int old = *f;
  *f = value;
  return old;
}

// What the last dmlp_step / dmlp_knn_local did: [0] queries on the exact fp64 path, [1] queries
// escalated from a single-term to a 3-term screen, [2] path (0 host-rendered operands, 2 device
// image), [3] early start.
extern "C" void dmlp_pipeline_stats(int64_t* out) {
  out[0] = g_stats.n_exact;
  out[1] = g_stats.n_escalated;
  out[2] = g_stats.path;
  out[3] = g_stats.early;
  out[4] = g_stats.n_exact_f64;
  out[5] = g_stats.n_exact_f64_redo;
  out[6] = g_stats.device_render;
}
