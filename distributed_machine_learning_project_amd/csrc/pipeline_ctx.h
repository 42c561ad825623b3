// pipeline_ctx.h — the native pipeline's shared state (pipeline.hip dmlp_step, local.hip
// dmlp_knn_local and the Local dispatcher of local.h): errors, the bump arenas and grow-only
// buffers, the environment switches and A/B tuning, the slice choice of the screens, the per-device
// workspace (Ctx) and the host-rendered operands handed to a local call (HostOps).
#pragma once

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

namespace dmlp_pipe {

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
inline Arena g_dev, g_host;

inline void* dev_alloc(size_t bytes) {
  // the arena lives on one device: a buffer for another device (a process driving two GPUs)
  // comes from hipMalloc on the current one
  int d = -1;
  void* p = nullptr;
  if (g_dev.base && hipGetDevice(&d) == hipSuccess && d == g_dev.dev) p = g_dev.take(bytes);
  if (!p && hipMalloc(&p, std::max<size_t>(bytes, 1)) != hipSuccess) p = nullptr;
  return p;
}
inline void dev_free(void* p) {
  if (p && !g_dev.owns(p)) (void)hipFree(p);
}
inline void* host_alloc(size_t bytes) {
  void* p = g_host.take(bytes);
  if (!p && hipHostMalloc(&p, std::max<size_t>(bytes, 1), hipHostMallocDefault) != hipSuccess)
    p = nullptr;
  return p;
}
inline void host_free(void* p) {
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
inline bool env_off(const char* name) {
  const char* e = std::getenv(name);
  return e && e[0] == '0';
}
inline int env_int(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e && *e ? std::atoi(e) : dflt;
}
// early start of dmlp_step (DMLP_FAST_EARLY=0: off, =1: on; dmlp_step_early); off for the rest
// of the process after a wait timed out.  Default: on, unless several ranks share this GPU
// (DMLP_DEVICE_RANKS > 1, set by both front ends): one rank's screen spinning on its slices
// then holds the CUs the other ranks' copies need — P = 3 on one MI355X measured 20.8 ms/step
// with it against 7.3 ms without (profiles/r7h_host_budget.md).
inline int g_early = -1;
inline bool early_on() {
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
inline bool rowmajor_on() {
  static const bool on = !(getenv("DMLP_PAIR_ROWMAJOR") && getenv("DMLP_PAIR_ROWMAJOR")[0] == '0');
  return on;
}
// query render slices under the early start (profiles/r6i: 4 is best)
inline int early_qchunks() {
  static const int q = std::min(16, std::max(1, env_int("DMLP_FAST_QCHUNKS", 4)));
  return q;
}
// Device render: the screen's fp16 operands rendered on the GPU (prep.hip k_render) from the rows
// that cross PCIe for the exact re-rank anyway (lossless int32): the host only packs int32 rows.
// On by the cost model at large N (dr_auto below: the chunked large-N pipeline); at the headline
// shape the operands would wait for the int32 rows, slower than the host render (profiles/r9r).
inline bool dr_on();  // (Tuning::device_render below)
// The render kernels (k_render: one-wave workgroups, 40 VGPRs, no LDS) would have to run beside
// an early-start screen that fills the GPU and spins on their ready words.  Measured
// (profiles/r9e-r9g): with 256-thread workgroups they never started beside it (every wave timed
// out); with one-wave workgroups beside the KT 1 / k <= 16 screen they ran in one session and
// never started in the next (same code and shape), and never beside the k > 16 variant.  The
// dispatcher does not reliably hand them slots, so an early-start step keeps the host render
// (host_prep.cpp: its copies do get through) and the device render serves the steps without
// an early start.
inline bool dr_early_ok(int, int) { return false; }
// The early start's copies (small ones run as blit kernels) need a wave slot beside the spinning
// screen: the screen variant must leave registers free (of 512 per SIMD lane; hipcc
// -Rpass-analysis=kernel-resource-usage, VGPR + AGPR): KT 1 SUB 16 2 x 223, KT 1 SUB 32 317,
// KT 2 SUB 32 350 — but KT 2 SUB 16 takes 2 x 256 (every wave timed out, profiles/r9h) and KT 8
// up to all 512.  KT 4 (SUB 16 322, SUB 32 414) has the room on paper, yet its copies found no
// slot in 2 of 7 test sessions (every wave timed out: profiles/r12a_kt4_early.txt), so KT 4
// runs without the early start too.
inline bool early_room(int KT, int kmax) {
  // (KT 2: only the SUB = 32 variant, the larger candidate lists)
  return KT == 1 || (KT == 2 && dmlp_screen_x1_cap_kt(2, kmax) > dmlp_screen_x1_cap_kt(2, 1));
}
// test knob: the host sleeps this long before each dataset image slice of an early-start call,
// so the screen provably waits mid-scan (tests/test_engine_gpu.py)
inline int g_early_delay_us = -1;
inline int early_delay_us() {
  if (g_early_delay_us < 0) g_early_delay_us = std::max(0, env_int("DMLP_FAST_EARLY_DELAY_US", 0));
  return g_early_delay_us;
}
// host render + H2D of the screen operands in pipelined slices (profiles/r2t: 2)
inline int host_slices() {
  static const int s = std::max(1, env_int("DMLP_HOST_OPS_CHUNKS", 2));
  return s;
}
// fp64 rows as lossless int32 when every value is a 6-decimal number (DMLP_ROWS_I32=0: fp64)
inline bool rows_i32_on() {
  static const bool on = !env_off("DMLP_ROWS_I32");
  return on;
}
// 3-term streaming screen for the escalation of k <= 32 (KNN_SCREEN=lds: the LDS screen)
inline bool stream_screen_on() {
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
  // report_mode 1 into page-locked memory the GPU can address: 1 the format kernel writes the
  // text straight across PCIe, 0 into device memory, then one D2H copy of the bound
  // (DMLP_REPORT_DIRECT)
  int report_direct = 1;
};
inline Tuning make_tuning() {
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
  if (env_off("DMLP_REPORT_DIRECT")) t.report_direct = 0;
  if (env_off("DMLP_HOST_OPS")) t.host_ops = 0;
  else if (const char* e = std::getenv("DMLP_HOST_OPS"); e && *e) t.host_ops = 2;  // forced on
  return t;
}
inline Tuning g_tune = make_tuning();
inline bool dr_on() { return g_tune.device_render > 0; }
// The device render's share of the work by the cost model: the host render ships 6 bytes per
// value (the fp16 image + the int32 rows) after a host pass that writes both, the device render 4
// (the int32 rows; the GPU renders the image from them) — at large N the step is bound by that
// host pass and PCIe (profiles/r10a_large_n_render_ab.jsonl: N = 1e6, A = 128: 21.1 / 22.4 vs
// 28.8 / 38.2 ms).  Below the early start's reach (one screen slice, nt <= 4096) the host render
// keeps the early start (the render kernels get no wave slots beside its spinning screen).
// It pays where the chunked large-N pipeline runs (every k in the one-pass class) and its extra
// slices cost the refine little: k <= 32 (the pair groups), or k <= 64 once the host pass is
// large (N A >= 2^26).  The two-pass class (k > 64) screens after all the rows landed, and the
// host render's overlap wins there (profiles/r11j_render_ab.txt: N = 1e6, A = 32, k = 200:
// 6.8-7.1 host vs 11.1-11.4 device; k 1-64: 5.7-6.3 vs 6.4-6.5; A = 128, k 1-64: 21-31 vs 16).
constexpr int64_t kDrMinValues = int64_t(1) << 23, kDrMinValuesK64 = int64_t(1) << 26;
inline bool dr_auto(int64_t N, int A, int kmin, int kmax) {
  if (g_tune.device_render >= 0 || kmin < 1) return false;
  const int64_t v = N * A;
  return (kmax <= 32 && v >= kDrMinValues) || (kmax <= 64 && v >= kDrMinValuesK64);
}
// Every small host <-> device copy of the step goes through the SDMA engines (dmlp::dma_copy: a
// copy below ~32 KiB would otherwise be a blit kernel, a memset a fill kernel) — its words are
// cleared by a DMA copy from this page-locked block of zeros.
constexpr int kZeroBytes = 4096;
inline const void* zero_block() {
  static void* z = [] {
    void* p = nullptr;
    if (hipHostMalloc(&p, kZeroBytes, hipHostMallocDefault) != hipSuccess) return (void*)nullptr;
    std::memset(p, 0, kZeroBytes);
    return p;
  }();
  return z;
}
inline hipError_t dma_zero(void* dst, size_t bytes, hipStream_t s) {
  const void* z = zero_block();
  if (!z || bytes > (size_t)kZeroBytes) return hipMemsetAsync(dst, 0, bytes, s);
  return dmlp::dma_copy(dst, z, bytes, s);
}
// memcpy on the render pool (large host staging copies: labels, k)
inline void pool_memcpy(void* dst, const void* src, int64_t bytes) {
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
inline unsigned ready_bits(float nm) {
  unsigned b = 0;
  std::memcpy(&b, &nm, 4);
  return b ? b : 1u;
}
// what the last call did (dmlp_pipeline_stats)
struct Stats {
  int64_t n_exact = 0, n_escalated = 0, path = 0, early = 0;
  int64_t n_exact_f64 = 0, n_exact_f64_redo = 0;  // exact-path queries on the fp64 MFMA screen
  int64_t device_render = 0;  // the screen operands were rendered on the device
  int64_t report_direct = 0;  // the report text went straight into the caller's host buffer
};
inline Stats g_stats;

// ---------------------------------------------------------------- slices of the screens
inline int slices_stream(int nq, int qw, int64_t n_tiles, int waves_per_cu, int64_t s_lo = 1) {
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
inline int slices_lds(int nq, int waves, int64_t n_tiles) {
  const int nqb = (nq + waves * 16 - 1) / (waves * 16);
  int S = 1;
  while ((int64_t)nqb * S < 2 * g_tune.num_cus && S * 2 <= std::max<int64_t>(1, n_tiles) && S < 256) S *= 2;
  return S;
}
// data slices of the single-term x1 pass over nq queries of class bound kcls.  Every (query,
// slice) keeps its slice's own top-k groups (all k may sit in one slice) in <= 120 entries, so a
// slice must hold many more groups than k: for k > 32 at least 32 k points per slice (a slice of
// a few hundred groups would keep most of them within 2 eps of its k-th key and overflow)
inline int x1_slices(int nq, int KT, int kcls, int64_t nt) {
  const int64_t smin = dmlp_screen_x1_min_slices(nt);
  int S = slices_stream(nq, dmlp_screen_x1_cols(KT, kcls), nt,
                        dmlp_screen_x1_waves_per_cu_kt(KT, kcls), smin);
  if (kcls > 32) S = (int)std::max<int64_t>(smin, std::min<int64_t>(S, nt * 64 / (32 * kcls)));
  return std::max(S, 1);
}

// sum of the decimal digit counts of v over [a, b)
inline int64_t digits_sum(int64_t a, int64_t b) {
  int64_t s = 0, lo = 0, hi = 10;
  for (int d = 1; d <= 19 && lo < b; ++d, lo = hi, hi = hi > INT64_MAX / 10 ? INT64_MAX : hi * 10) {
    const int64_t x = std::max(a, lo), y = std::min(b, hi);
    if (y > x) s += (y - x) * d;
  }
  return s;
}

// ---------------------------------------------------------------- per-device workspace
enum { M_ENTER, M_OPS, M_DATA, M_ROWS, M_SCREEN, M_REFINE, M_FORMAT, M_D2H, M_N };
inline constexpr const char* kMarkNames[M_N] = {"enter", "operands_landed", "data_landed", "rows_landed",
                                     "screen_done", "knn_done", "format_done",
                                     "report_d2h_done"};

struct Ctx {
  int dev = -1;
  hipStream_t side = nullptr;  // host->device copies of dmlp_step
  // the large-N device render's kernels (off the copies' stream), created on first use: another
  // stream changes how the process's streams share the runtime's hardware queues, and an
  // early-start step needs its copies' queue apart from its screen's (one on the same queue as
  // the spinning screen waits behind it: every wave timed out in a GPU test, r11m)
  hipStream_t rnd = nullptr;
  hipStream_t render_stream() {
    if (!rnd && hipStreamCreateWithPriority(&rnd, hipStreamNonBlocking, high_priority()) !=
                    hipSuccess)
      rnd = nullptr;
    return rnd ? rnd : side;
  }
  static int high_priority() {  // (DMLP_SIDE_PRIORITY=0: the default priority, A/B)
    if (env_off("DMLP_SIDE_PRIORITY")) return 0;
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) return 0;
    return greatest;
  }
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
  hipEvent_t ev_chunk[kEarlySlices] = {};  // the large-N pipeline's chunk events (rendered)
  hipEvent_t ev_copy[kEarlySlices] = {};   // ... and its chunks' rows landed
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

inline Ctx& ctx() {
  static Ctx c[16];
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= 16) d = 0;
  Ctx& w = c[d];
  if (!w.side) {
    w.dev = d;
    // the copies' stream at the high priority: the runtime keeps a separate pool of hardware
    // queues per priority, so it never shares one with a (normal-priority) stream whose screen
    // spins on the words these copies write (the early start)
    CK(hipStreamCreateWithPriority(&w.side, hipStreamNonBlocking, Ctx::high_priority()));
    CK(hipEventCreateWithFlags(&w.ev_ops, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&w.ev_rows, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&w.ev_done, hipEventDisableTiming));
    for (hipEvent_t& e : w.ev_chunk) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (hipEvent_t& e : w.ev_copy) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  return w;
}

// Wait for the step's last event by polling it (the host thread spins for the ~2 ms a step takes
// instead of sleeping in the runtime's blocking wait, whose wake-up sat on every step's tail).
inline void spin_wait(hipEvent_t e) {
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

inline int* identity(Ctx& w, int64_t n, hipStream_t st) {  // device 0, 1, ..., n-1 (grow-only)
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

inline int drain_and_fail(Ctx* w, hipStream_t st, int code) {
  // every error path drains the streams before returning: nothing may still be writing the
  // caller's tensors or reading the page-locked staging when it frees or reuses them
  if (w && w->side) (void)hipStreamSynchronize(w->side);
  if (w && w->rnd) (void)hipStreamSynchronize(w->rnd);
  if (st) (void)hipStreamSynchronize(st);
  (void)hipGetLastError();
  return code;
}

}  // namespace dmlp_pipe
