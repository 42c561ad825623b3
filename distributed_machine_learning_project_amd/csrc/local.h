// local.h — the dispatcher of one local k-NN call (struct Local): every query class's screen,
// refine and escalation queued on one stream (pipeline.hip header comment: the classes).
#pragma once

#include "pipeline_ctx.h"

namespace dmlp_pipe {

// (dmlp_step) the rows crossed PCIe as lossless int32 and their fp64 conversion is deferred: the
// refines read X as int32 (the pair refine Q too: half the gathered bytes); anything else that
// reads the fp64 rows converts them first — to_f64(need): bit 0 X, bit 1 Q, each queued on the
// call's stream once and cleared
struct I32Rows {
  const int* X = nullptr;
  const int* Q = nullptr;
  std::function<void(int)> to_f64;
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
  I32Rows* i32 = nullptr;  // (dmlp_step) rows still int32 on the device, or none
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
  // need: the rows the caller reads as fp64 (bit 0 X, bit 1 Q); the others it reads as int32
  // (I32Rows) when they are
  void wait_rows(int need = 3) {
    launch_rows();
    if (!rows_waited) {
      if (rows) CK(hipStreamWaitEvent(st, rows, 0));
      rows_waited = true;
    }
    if (i32 && i32->to_f64 && (((need & 1) && i32->X) || ((need & 2) && i32->Q)))
      i32->to_f64(need);
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
      const int cap = dmlp_screen_x1_cap_kt(KT, kcls);
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
      // (issues the row copies first) the re-rank reads the rows: the pair refine as int32 when
      // they crossed that way, the others as fp64
      // (the pair refine reads both as int32, the group refine the dataset's rows only)
      const bool pair = dmlp_refine_pair_path(S, hl, KT, fin, cap, kcls) != 0;
      wait_rows(pair ? 0 : 2);
      CKL(dmlp_refine_groups_rm(cap, ci, cc, ch, S, X, A, Qx, xf, hx ? hx->xrow : nullptr, xi,
                                qh, KT, hl, N, idx ? qi : nullptr, kd, nq, out_d, out_i, kstride,
                                fin ? labels : nullptr, lo, hi, lab, cs, stat, ovf, kcls,
                                i32 ? i32->X : nullptr, pair && i32 ? i32->Q : nullptr, st));
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
      const int cap1 = dmlp_screen_x1_cap_kt(KT, kmax1);
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

}  // namespace dmlp_pipe
