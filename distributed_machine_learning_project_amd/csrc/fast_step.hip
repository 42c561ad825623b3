// fast_step.hip — the single-GPU headline call in one native function (no Python between the
// phases): the host-operand pipeline of ops/knn.py knn_gpu_pipelined (+ _pipelined_parts with one
// part) for the common case, every k on the single-term class.  The Python path spends ~0.3 ms
// of interpreter time per call on the critical path (profiles/r5m: 0.19 ms between calls, 0.12
// ms before the first render, 0.12 ms of set-up between the data and query renders); here the
// whole step is host C++ around the same kernels:
//
//   side stream: dataset image + query fragments rendered on the host pool and copied in slices
//                (host_prep.cpp), k; then labels and the fp64 rows (lossless int32 when every
//                value is a 6-decimal number) behind the screen
//   main stream: single-term screen (screen_x1.hip) of each query part once its operands landed
//   tail stream: per part, group refine (refine.hip, waits for the rows and the part's screen)
//                -> the part's report text (GPU, at the previous part's device-side end) -> D2H
//                of its byte range; then the byte count and the overflow count -> one host sync
//                (one screen: the refine may run as R query ranges, DMLP_FAST_RPARTS, each
//                range's D2H on a copy stream of its own under the next range's refine)
//
// Returns 0 (report and results written), 1 when the call is not this path's (k outside
// [1, 32], data or queries outside the fp16 screen's range, no x1 variant for A: nothing the
// caller can observe was written), 2 when some query's single-term candidates overflowed (the
// caller reruns the call on the general path, whose per-query escalation handles it), < 0 on a
// HIP error.  out_lab / out_cs (device, Q each) are the caller's: the labels and checksums stay
// there; the report text goes to report_dst (page-locked, >= dmlp_format_bound(Q) bytes).  The
// internal device and page-locked buffers are grow-only and reused by the next call.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "dmlp.h"

namespace {

template <typename T>
struct DBuf {  // grow-only device buffer
  T* p = nullptr;
  size_t n = 0;
  T* get(size_t m) {
    if (m > n) {
      if (p) (void)hipFree(p);
      p = nullptr;
      n = 0;
      if (hipMalloc((void**)&p, std::max<size_t>(m, 1) * sizeof(T)) != hipSuccess) return nullptr;
      n = std::max<size_t>(m, 1);
    }
    return p;
  }
};

template <typename T>
struct HBuf {  // grow-only page-locked host buffer
  T* p = nullptr;
  size_t n = 0;
  T* get(size_t m) {
    if (m > n) {
      if (p) (void)hipHostFree(p);
      p = nullptr;
      n = 0;
      if (hipHostMalloc((void**)&p, std::max<size_t>(m, 1) * sizeof(T), hipHostMallocDefault) !=
          hipSuccess)
        return nullptr;
      n = std::max<size_t>(m, 1);
    }
    return p;
  }
};

// phase marks of the step timeline (dmlp_fast_step_events(1): hipEvents, read after the sync)
enum { M_ENTER, M_DATA, M_OPS, M_ROWS, M_SCREEN, M_REFINE, M_FORMAT, M_D2H, M_N };
const char* const kMarkNames[M_N] = {"enter", "data_landed", "operands_landed", "rows_landed",
                                     "screen_done", "refine_done", "format_done",
                                     "report_d2h_done"};

constexpr int kMaxParts = 4;

// query parts of a call (DMLP_FAST_PARTS, 1..4; default 1): part p's screen starts as soon as its
// operands landed, and its refine + report text + D2H run on the tail stream while the next
// part screens
int clamp_parts(int v) { return v < 1 ? 1 : v > kMaxParts ? kMaxParts : v; }
int g_parts = -1;  // -1: DMLP_FAST_PARTS (read once)
int fast_parts() {
  if (g_parts < 0) {
    const char* e = std::getenv("DMLP_FAST_PARTS");
    g_parts = clamp_parts(e ? std::atoi(e) : 1);
  }
  return g_parts;
}
// refine parts behind ONE screen (DMLP_FAST_RPARTS, 1..4; used when the screen is not split):
// the refine runs as R launches over query ranges on the tail stream, and each range's report
// text crosses PCIe on a stream of its own while the next range refines, so only the last
// range's D2H stays on the critical path
int g_rparts = -1;
int fast_rparts() {
  if (g_rparts < 0) {
    const char* e = std::getenv("DMLP_FAST_RPARTS");
    g_rparts = clamp_parts(e ? std::atoi(e) : 1);
  }
  return g_rparts;
}

// early start (default on, DMLP_FAST_EARLY=0 off; one part, one screen slice): the query operands
// cross first and the screen starts on them while the dataset image follows in kEarlySlices
// slices, each with a ready word the screen waits on (screen_x1.hip dmlp_screen_x1_early).
// profiles/r6f: 2.23-2.24 vs 2.35-2.38 ms/step (4 slices, interleaved on one box)
constexpr int kEarlySlices = 8;
int g_early = -1;
bool fast_early() {
  if (g_early < 0) {
    const char* e = std::getenv("DMLP_FAST_EARLY");
    g_early = (e && e[0] == '0') ? 0 : 1;
  }
  return g_early != 0;
}

// query render slices under the early start (DMLP_FAST_QCHUNKS, default 4): the query operands
// are the whole front of the step there, so their last slice's copy is exposed; profiles/r6i:
// 4 slices 2.29-2.40 ms/step vs 2.36-2.68 at 2 and 2.31-2.66 at 6, interleaved on one box
int early_qchunks(int ch) {
  static const int q = [] {
    const char* e = std::getenv("DMLP_FAST_QCHUNKS");
    return e ? std::atoi(e) : 4;
  }();
  return q > 0 ? std::min(q, 16) : ch;
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

struct Workspace {
  hipStream_t side = nullptr, tail = nullptr, d2h = nullptr;
  hipEvent_t ev_ops[kMaxParts] = {}, ev_scr[kMaxParts] = {}, ev_rows = nullptr, ev_k = nullptr;
  hipEvent_t ev_fmt[kMaxParts] = {};
  bool marks_on = false, marks_valid = false;
  hipEvent_t marks[M_N] = {};
  // device
  DBuf<short> xhi, qhi;
  DBuf<float> xin, qn, cand_h;
  DBuf<unsigned> words;  // [0] xnmax bits, [1] bad (0: the host checked the ranges)
  DBuf<int> kdev, ident, cand_ids, cand_cnt, status, ovf, lab_d, i32, out_i;
  DBuf<double> X, Qd, out_d;
  DBuf<int64_t> off;
  DBuf<char> text;
  // page-locked staging
  HBuf<uint16_t> xhi_h, qhi_h;
  HBuf<float> xin_h, qn_h;
  HBuf<unsigned> xnm_h;
  HBuf<int> k_h, i32_h, ident_h, small_h;  // small_h: [0] overflow count
  HBuf<int64_t> len_h;
  HBuf<double> mu_h;
  int64_t ident_len = 0;
};

Workspace& ws() {
  static Workspace w;
  return w;
}

// Data slices of the single-term screen (ops/knn.py _choose_slices_stream).
int slices(int nq, int qw, int64_t n_tiles, int waves_per_cu, int64_t s_lo) {
  const int nqb = (nq + qw - 1) / qw;
  const int slots = waves_per_cu * 256;
  const int s_min = (int)std::max<int64_t>(std::max<int64_t>(1, s_lo),
                                           (n_tiles * 64 + (1ll << 29) - 1) >> 29);
  if (nqb >= slots) return s_min;
  int best = s_min;
  double best_eff = 0.0;
  for (int S = s_min; S < s_min + 64 && S <= std::max<int64_t>(s_min, n_tiles / 4); ++S) {
    const double w = (double)nqb * S;
    const double eff = w / (double)(((int64_t)w + slots - 1) / slots * slots);
    if (eff >= 0.9) return S;
    if (eff > best_eff + 1e-9) {
      best = S;
      best_eff = eff;
    }
  }
  return best;
}

}  // namespace

extern "C" int dmlp_fast_step(const double* X, const int* labels, int64_t N, const double* Qx,
                              const int* k, int64_t Q, int A, int kmin, int kmax, int label_lo,
                              int label_hi, int64_t qid_base, int chunks, char* report_dst,
                              int64_t report_cap, int64_t* report_len, int* out_lab,
                              uint64_t* out_cs, void* stream) {
#define FS_CHK(x)                                         \
  do {                                                    \
    const hipError_t e_ = (x);                            \
    if (e_ != hipSuccess) return -(int)e_;                \
  } while (0)
#define FS_PTR(p)                                         \
  do {                                                    \
    if (!(p)) return -(int)hipErrorOutOfMemory;           \
  } while (0)
  if (N <= 0 || Q <= 0 || Q > (1 << 30) || A < 1 || kmin < 1 || kmax > 32 || kmax > N) return 1;
  const int KT = dmlp_screen_kt(A);
  if (dmlp_screen_x1_qw(KT) <= 0) return 1;
  const int64_t nt = (N + 63) / 64;
  if (report_cap < dmlp_format_bound((int)Q)) return 1;
  Workspace& w = ws();
  hipStream_t st = (hipStream_t)stream;
  if (!w.side) {
    FS_CHK(hipStreamCreateWithFlags(&w.side, hipStreamNonBlocking));
    FS_CHK(hipStreamCreateWithFlags(&w.tail, hipStreamNonBlocking));
    FS_CHK(hipStreamCreateWithFlags(&w.d2h, hipStreamNonBlocking));
    for (int p = 0; p < kMaxParts; ++p) {
      FS_CHK(hipEventCreateWithFlags(&w.ev_ops[p], hipEventDisableTiming));
      FS_CHK(hipEventCreateWithFlags(&w.ev_scr[p], hipEventDisableTiming));
      FS_CHK(hipEventCreateWithFlags(&w.ev_fmt[p], hipEventDisableTiming));
    }
    FS_CHK(hipEventCreateWithFlags(&w.ev_rows, hipEventDisableTiming));
    FS_CHK(hipEventCreateWithFlags(&w.ev_k, hipEventDisableTiming));
  }
  w.marks_valid = false;
  auto mark = [&](int i, hipStream_t s) -> hipError_t {
    return w.marks_on ? hipEventRecord(w.marks[i], s) : hipSuccess;
  };
  FS_CHK(mark(M_ENTER, w.side));
  const int64_t W = (int64_t)KT * 32;
  // page-locked staging + device buffers (grow-only)
  uint16_t* xhi_h = w.xhi_h.get(nt * 64 * W);
  float* xin_h = w.xin_h.get(nt * 64);
  unsigned* xnm_h = w.xnm_h.get(2 + kEarlySlices);
  uint16_t* qhi_h = w.qhi_h.get(Q * W);
  float* qn_h = w.qn_h.get(Q);
  double* mu = w.mu_h.get(A);
  int* k_h = w.k_h.get(Q);
  int* small_h = w.small_h.get(16);
  int64_t* len_h = w.len_h.get(2);
  short* xhi = w.xhi.get(nt * 64 * W);
  float* xin = w.xin.get(nt * 64);
  unsigned* words = w.words.get(2 + 2 * kEarlySlices);  // + early start: ready words, max norms
  short* qhi = w.qhi.get(Q * W);
  float* qn = w.qn.get(Q);
  int* kd = w.kdev.get(Q);
  FS_PTR(xhi_h); FS_PTR(xin_h); FS_PTR(xnm_h); FS_PTR(qhi_h); FS_PTR(qn_h); FS_PTR(mu);
  FS_PTR(k_h); FS_PTR(small_h); FS_PTR(len_h); FS_PTR(xhi); FS_PTR(xin); FS_PTR(words);
  FS_PTR(qhi); FS_PTR(qn); FS_PTR(kd);
  // the previous call's work on the main stream is complete (it ended with a sync); the side
  // stream may still hold nothing: no dependency needed
  dmlp_cpu_center(X, std::min<int64_t>(N, 4096), A, mu);
  // dataset image, then the query fragments part by part, rendered on the host pool and copied
  // in slices (side); a query call renders no tiles and writes its (zero) norm word into
  // words[1], the "bad" word, which the host-checked ranges leave at 0
  const int ch = chunks < 1 ? 1 : chunks;
  int rc = 0;
  std::memcpy(k_h, k, (size_t)Q * sizeof(int));
  FS_CHK(hipMemcpyAsync(kd, k_h, (size_t)Q * sizeof(int), hipMemcpyHostToDevice, w.side));
  // identity query list (grow-only, written once)
  if (w.ident_len < Q) {
    const int64_t n = std::max<int64_t>(Q, 1 << 16);
    int* h = w.ident_h.get(n);
    int* d = w.ident.get(n);
    FS_PTR(h); FS_PTR(d);
    for (int64_t i = 0; i < n; ++i) h[i] = (int)i;
    FS_CHK(hipMemcpyAsync(d, h, (size_t)n * sizeof(int), hipMemcpyHostToDevice, w.side));
    w.ident_len = n;
  }
  // parts: multiples of 64 queries (whole screen query blocks)
  const int P = (int)std::max<int64_t>(1, std::min<int64_t>(fast_parts(), (Q + 63) / 64));
  int64_t q0s[kMaxParts + 1];
  for (int p = 0; p <= P; ++p) q0s[p] = std::min<int64_t>(Q, (Q * p / P + 63) / 64 * 64);
  q0s[P] = Q;
  const int cap = dmlp_screen_x1_cap(kmax);
  int Sp[kMaxParts];
  int64_t coff[kMaxParts + 1] = {0};  // candidate slots before part p
  for (int p = 0; p < P; ++p) {
    const int64_t qp = q0s[p + 1] - q0s[p];
    Sp[p] = slices((int)qp, dmlp_screen_x1_cols(KT, kmax), nt,
                   dmlp_screen_x1_waves_per_cu_kt(KT, kmax), dmlp_screen_x1_min_slices(nt));
    coff[p + 1] = coff[p] + qp * Sp[p];
  }
  const bool early = fast_early() && P == 1 && Sp[0] == 1 && nt >= 2 && nt <= 4096;
  const int NS = early ? (int)std::min<int64_t>(kEarlySlices, nt) : 0;
  const int rt = early ? (int)((nt + NS - 1) / NS) : 1;  // image tiles per early slice
  unsigned* const rdy = words + 2;                         // [NS] ready words
  unsigned* const xnm_sl = words + 2 + kEarlySlices;       // [NS] slice max norms
  if (!early) {
    rc = dmlp_host_ops_h2d_tiles(X, N, 0, nt, Qx, 0, A, mu, KT, xhi_h, xin_h, xnm_h, qhi_h, qn_h,
                                 xhi, xin, words, qhi, qn, ch, w.side);
    FS_CHK(mark(M_DATA, w.side));
    if (rc & 4) return -(int)hipErrorUnknown;
  } else {
    FS_CHK(hipMemsetAsync(rdy, 0, (size_t)NS * sizeof(unsigned), w.side));
  }
  int* cand_ids = w.cand_ids.get((size_t)coff[P] * cap);
  int* cand_cnt = w.cand_cnt.get((size_t)coff[P]);
  float* cand_h = w.cand_h.get((size_t)coff[P] * 2);
  int* ovf = w.ovf.get(1);
  FS_PTR(cand_ids); FS_PTR(cand_cnt); FS_PTR(cand_h); FS_PTR(ovf);
  FS_CHK(hipMemsetAsync(ovf, 0, sizeof(int), st));
  for (int p = 0; p < P; ++p) {
    const int64_t q0 = q0s[p], qp = q0s[p + 1] - q0;
    rc |= dmlp_host_ops_h2d_tiles(X, N, nt, nt, Qx + q0 * A, qp, A, mu, KT, xhi_h, xin_h,
                                  xnm_h + 1, qhi_h + q0 * W, qn_h + q0, xhi, xin, words + 1,
                                  qhi + q0 * W, qn + q0, early ? early_qchunks(ch) : ch, w.side);
    if (rc & 4) return -(int)hipErrorUnknown;
    if (rc) {  // outside the fp16 screen's range: the caller's general path decides
      FS_CHK(hipStreamSynchronize(w.side));
      FS_CHK(hipStreamSynchronize(st));
      return 1;
    }
    if (p == P - 1) FS_CHK(mark(M_OPS, w.side));
    FS_CHK(hipMemsetAsync(words + 1, 0, sizeof(unsigned), w.side));
    FS_CHK(hipEventRecord(w.ev_ops[p], w.side));
    // ---- main: the part's screen as soon as its operands landed
    FS_CHK(hipStreamWaitEvent(st, w.ev_ops[p], 0));
    const int e =
        early ? dmlp_screen_x1_early(KT, A, xhi, xin, nt, N, qhi + q0 * W, qn + q0, w.ident.p,
                                     kd + q0, (int)qp, kmax, words + 1, rdy, rt, NS, xnm_sl,
                                     cand_ids + coff[p] * cap, cand_cnt + coff[p],
                                     cand_h + coff[p] * 2, st)
              : dmlp_screen_x1(KT, 1, A, xhi, xin, nt, N, qhi + q0 * W, qn + q0, w.ident.p,
                               kd + q0, (int)qp, kmax, words, words + 1, Sp[p],
                               cand_ids + coff[p] * cap, cand_cnt + coff[p],
                               cand_h + coff[p] * 2, st);
    if (e) return e < 0 ? e : -1;
    FS_CHK(hipEventRecord(w.ev_scr[p], st));
  }
  if (early) {
    // the dataset image behind the queries, slice by slice, each followed by its ready word (the
    // running screen waits on it); every word is written even when a slice is out of the fp16
    // range, so the screen always drains before the caller falls back
    small_h[8] = 1;
    for (int i = 0; i < NS; ++i) {
      const int64_t a = (int64_t)i * rt, b = std::min<int64_t>(nt, a + rt);
      rc |= dmlp_host_ops_h2d_tiles(X, N, a, b, Qx, 0, A, mu, KT, xhi_h, xin_h, xnm_h + 2 + i,
                                    qhi_h, qn_h, xhi + a * 64 * W, xin + a * 64, xnm_sl + i, qhi,
                                    qn, 1, w.side);
      FS_CHK(hipMemcpyAsync(rdy + i, small_h + 8, sizeof(unsigned), hipMemcpyHostToDevice,
                            w.side));
    }
    FS_CHK(mark(M_DATA, w.side));
    if (rc) {  // hip error or data outside the fp16 screen's range
      FS_CHK(hipStreamSynchronize(w.side));
      FS_CHK(hipStreamSynchronize(st));
      return (rc & 4) ? -(int)hipErrorUnknown : 1;
    }
  }
  FS_CHK(mark(M_SCREEN, st));
  // ---- side: labels and the fp64 rows behind the screen
  int* lab_d = w.lab_d.get(N);
  double* Xd = w.X.get((size_t)N * A);
  double* Qd = w.Qd.get((size_t)Q * A);
  FS_PTR(lab_d); FS_PTR(Xd); FS_PTR(Qd);
  FS_CHK(hipMemcpyAsync(lab_d, labels, (size_t)N * sizeof(int), hipMemcpyHostToDevice, w.side));
  {
    const int64_t nx = N * A, nqa = Q * A, at = (nx + 3) & ~int64_t(3);  // (16-B aligned)
    int* h32 = w.i32_h.get(at + nqa);
    int* d32 = w.i32.get(at + nqa);
    FS_PTR(h32); FS_PTR(d32);
    auto rows = [&](const double* src, int64_t n, double* dst, int64_t off) -> int {
      if (dmlp_cpu_rows_i32(src, n, h32 + off) == 0) {  // lossless 6-decimal: half the bytes
        if (hipMemcpyAsync(d32 + off, h32 + off, (size_t)n * 4, hipMemcpyHostToDevice, w.side) !=
            hipSuccess)
          return -1;
        return dmlp_rows_from_i32(d32 + off, n, dst, w.side);
      }
      return hipMemcpyAsync(dst, src, (size_t)n * 8, hipMemcpyHostToDevice, w.side) == hipSuccess
                 ? 0 : -1;
    };
    if (rows(X, nx, Xd, 0) || rows(Qx, nqa, Qd, at)) return -(int)hipErrorUnknown;
  }
  FS_CHK(hipEventRecord(w.ev_rows, w.side));
  FS_CHK(mark(M_ROWS, w.side));
  // ---- tail: per part, exact re-rank (+ vote, checksum), report text at the previous part's
  // end (device word), D2H of the part's byte range; then one sync
  double* out_d = w.out_d.get((size_t)Q * kmax);
  int* out_i = w.out_i.get((size_t)Q * kmax);
  int* status = w.status.get(Q);
  int64_t* off = w.off.get((size_t)dmlp_format_scratch((int)Q) + 2 * kMaxParts);
  char* text = w.text.get((size_t)dmlp_format_bound((int)Q));
  FS_PTR(out_d); FS_PTR(out_i); FS_PTR(out_lab); FS_PTR(out_cs); FS_PTR(status); FS_PTR(off);
  FS_PTR(text);
  FS_CHK(hipStreamWaitEvent(w.tail, w.ev_rows, 0));
  const int64_t bound = dmlp_format_bound((int)Q);
  // tail ranges: the screen parts, or (one screen) R query ranges of it
  const int R = P > 1 ? P : (int)std::max<int64_t>(1, std::min<int64_t>(fast_rparts(), (Q + 63) / 64));
  int64_t r0s[kMaxParts + 1];
  for (int r = 0; r <= R; ++r)
    r0s[r] = P > 1 ? q0s[r] : std::min<int64_t>(Q, (Q * r / R + 63) / 64 * 64);
  r0s[R] = Q;
  // the report bytes cross on their own stream when the refine is split (the next range refines
  // meanwhile); one range keeps them on the tail stream
  hipStream_t cp = R > 1 ? w.d2h : w.tail;
  int64_t lo = 0;           // a lower bound on the byte where range r's text starts
  const int64_t* base = nullptr;
  int64_t* off_p = off;     // range r's line offsets (scratch of its own: the next reads its end)
  for (int r = 0; r < R; ++r) {
    const int64_t q0 = r0s[r], qp = r0s[r + 1] - q0;
    const int sp = P > 1 ? r : 0;                              // the screen that served it
    const int64_t c0 = P > 1 ? coff[r] : q0 * Sp[0];           // its first candidate slot
    if (P > 1 || r == 0) FS_CHK(hipStreamWaitEvent(w.tail, w.ev_scr[sp], 0));
    int e = dmlp_refine_groups(cap, cand_ids + c0 * cap, cand_cnt + c0, cand_h + c0 * 2, Sp[sp],
                               Xd, A, Qd + q0 * A, xhi, xin, qhi + q0 * W, KT, 1, N, nullptr,
                               kd + q0, (int)qp, out_d + q0 * kmax, out_i + q0 * kmax, kmax,
                               lab_d, label_lo, label_hi, out_lab + q0, out_cs + q0, status + q0,
                               ovf, w.tail);
    if (e) return e < 0 ? e : -1;
    if (r == R - 1) FS_CHK(mark(M_REFINE, w.tail));
    e = dmlp_format_report_at(out_cs + q0, (int)qp, (int)(qid_base + q0), off_p, text, base,
                              w.tail);
    if (e) return e < 0 ? e : -1;
    if (r == R - 1) FS_CHK(mark(M_FORMAT, w.tail));
    if (cp != w.tail) {
      FS_CHK(hipEventRecord(w.ev_fmt[r], w.tail));
      FS_CHK(hipStreamWaitEvent(cp, w.ev_fmt[r], 0));
    }
    // bytes [lo, the range's upper bound): lines of at most 48 bytes; [lo, previous end) is the
    // previous range's text again (still intact on the device), copied after it in stream order
    // (bytes past this range's end that the next range's format may be writing meanwhile are
    // copied again, complete, by the next range's copy, later on the same stream)
    const int64_t hi = std::min<int64_t>(bound, 48 * (q0 + qp));
    FS_CHK(hipMemcpyAsync(report_dst + lo, text + lo, (size_t)(hi - lo), hipMemcpyDeviceToHost, cp));
    // the next range starts at or after this range's shortest text: "Query " qid " checksum: " d "\n"
    lo += 19 * qp + digits_sum(qid_base + q0, qid_base + q0 + qp);
    base = off_p + qp;
    off_p += qp + 1;  // (the next range's scratch: behind this range's offsets, below the bound)
  }
  FS_CHK(hipMemcpyAsync(len_h, base, sizeof(int64_t), hipMemcpyDeviceToHost, w.tail));
  FS_CHK(hipMemcpyAsync(small_h, ovf, sizeof(int), hipMemcpyDeviceToHost, w.tail));
  FS_CHK(mark(M_D2H, cp));
  FS_CHK(hipStreamSynchronize(w.tail));
  if (cp != w.tail) FS_CHK(hipStreamSynchronize(cp));
  FS_CHK(hipStreamSynchronize(st));
  w.marks_valid = w.marks_on;
  if (small_h[0]) return 2;  // some query's candidates overflowed: the general path escalates
  *report_len = len_h[0];
  return 0;
#undef FS_CHK
#undef FS_PTR
}

// Query parts of the following calls (1..4; <= 0: back to DMLP_FAST_PARTS / 1).
extern "C" void dmlp_fast_step_parts(int parts) { g_parts = parts <= 0 ? -1 : clamp_parts(parts); }
// Refine ranges behind one screen (1..4; <= 0: back to DMLP_FAST_RPARTS / 1).
extern "C" void dmlp_fast_step_rparts(int parts) { g_rparts = parts <= 0 ? -1 : clamp_parts(parts); }
// Early start of the following calls (1 on, 0 off, < 0: back to DMLP_FAST_EARLY).
extern "C" void dmlp_fast_step_early(int on) { g_early = on < 0 ? -1 : (on ? 1 : 0); }

// Step-timeline marks of dmlp_fast_step (hipEvents with timing; off by default).
extern "C" int dmlp_fast_step_events(int on) {
  Workspace& w = ws();
  if (on && !w.marks[0])
    for (int i = 0; i < M_N; ++i)
      if (hipEventCreate(&w.marks[i]) != hipSuccess) return -1;
  w.marks_on = on != 0 && w.marks[0];
  return 0;
}

// The last call's marks as ms since it entered (the previous call having synchronized, every
// event is complete): names[i] / ms[i] for i < the returned count (0: no timeline).
extern "C" int dmlp_fast_step_timeline(double* ms, const char** names, int cap) {
  Workspace& w = ws();
  if (!w.marks_valid) return 0;
  int n = 0;
  for (int i = 0; i < M_N && n < cap; ++i) {
    float t = 0.0f;
    if (hipEventElapsedTime(&t, w.marks[M_ENTER], w.marks[i]) != hipSuccess) continue;
    ms[n] = t;
    names[n] = kMarkNames[i];
    ++n;
  }
  return n;
}
