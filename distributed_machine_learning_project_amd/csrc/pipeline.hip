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
//                   exact re-rank + vote + FNV checksum, the report text rendered on the GPU
//                   straight into the caller's page-locked buffer (host_device_view; staged and
//                   copied for pageable memory), or kept on the device for a multi-rank egress
//                   (dmlp_step_emit).  One host sync in the common case; an
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
//
// Files: pipeline_ctx.h (arenas, buffers, switches, slices, the per-device workspace), local.h
// (the dispatcher, struct Local), local.hip (dmlp_knn_local, arenas, switches), this file
// (dmlp_step: struct Step, the host operands, the early start, the large-N pipeline).
#include "local.h"

namespace dmlp_pipe {

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

// The device's address for [p, p + bytes) of page-locked host memory (hipHostMalloc'd or
// registered, the whole range inside one allocation), or nullptr when the GPU cannot address it
// there (pageable memory: the step then stages the report on the device and copies it).  Both ends
// must map with one offset, and the allocation's address range (hipMemGetAddressRange) must hold
// the whole range — for registered memory this runtime reports the range's size with a null base
// (tools/probe/host_view_probe.py), so there both ends must lie in ranges of that one size.  Asked
// per call, never cached: a freed buffer's address can come back as pageable memory.
char* host_device_view(char* p, size_t bytes, int64_t* info = nullptr) {
  if (info) std::memset(info, 0, 8 * sizeof(int64_t));
  if (!p || bytes == 0) return nullptr;
  struct End {
    hipPointerAttribute_t at{};
    hipError_t e1 = hipErrorInvalidValue, e2 = hipErrorInvalidValue;
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
  } lo, hi;
  auto query = [](char* q, End& e) {
    e.e1 = hipPointerGetAttributes(&e.at, q);
    if (e.e1 == hipSuccess && e.at.devicePointer)
      e.e2 = hipMemGetAddressRange(&e.base, &e.size, (hipDeviceptr_t)e.at.devicePointer);
    if (e.e1 != hipSuccess || e.e2 != hipSuccess) (void)hipGetLastError();
    return e.e1 == hipSuccess && e.e2 == hipSuccess && e.at.type == hipMemoryTypeHost &&
           e.at.devicePointer && e.at.hostPointer == q;
  };
  const bool ok_lo = query(p, lo);
  const bool ok_hi = ok_lo && query(p + bytes - 1, hi);
  if (info) {
    const int64_t v[8] = {(int64_t)lo.e1, (int64_t)lo.at.type, (int64_t)(intptr_t)lo.at.devicePointer,
                          (int64_t)(intptr_t)lo.at.hostPointer, (int64_t)lo.e2,
                          (int64_t)(intptr_t)lo.base, (int64_t)lo.size, (int64_t)(intptr_t)p};
    std::memcpy(info, v, sizeof v);
  }
  if (!ok_hi) return nullptr;
  const char* d = (const char*)lo.at.devicePointer;
  if ((const char*)hi.at.devicePointer - d != (ptrdiff_t)(bytes - 1)) return nullptr;
  if (lo.base) {
    const char* b = (const char*)lo.base;
    return d >= b && d + bytes <= b + lo.size ? (char*)lo.at.devicePointer : nullptr;
  }
  return !hi.base && hi.size == lo.size && lo.size >= bytes ? (char*)lo.at.devicePointer : nullptr;
}

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
  I32Rows i32_;  // rows int32 on the device until something needs them as fp64 (I32Rows)
  // the conversions i32_ defers, queued when a reader needs them (after the rows' event, on the
  // call's stream)
  void defer_f64(double* Xd, double* Qd, int64_t nx, int64_t nqa) {
    if (!i32_.X && !i32_.Q) return;
    i32_.to_f64 = [this, Xd, Qd, nx, nqa](int need) {
      if ((need & 1) && i32_.X) {
        CKL(dmlp_rows_from_i32(i32_.X, nx, Xd, st));
        i32_.X = nullptr;
      }
      if ((need & 2) && i32_.Q) {
        CKL(dmlp_rows_from_i32(i32_.Q, nqa, Qd, st));
        i32_.Q = nullptr;
      }
    };
  }

  void issue_rows_now(double* Xd, double* Qd, int* lab_d) {
    const int64_t N = a->N, Q = a->Q, A = a->A;
    if (a->labels && N) {
      int* lh = w.s_lab.get(N);
      pool_memcpy(lh, a->labels, N * sizeof(int));
      CK(dmlp::dma_copy(lab_d, lh, N * sizeof(int), w.side));
    }
    const int64_t nx = N * A, nqa = Q * A, at = (nx + 3) & ~int64_t(3);  // (16-B aligned)
    // defer: keep 6-decimal rows int32 on the device (*defer = them) for the pair refine
    auto rows = [&](const double* src, const double* const* tab, int64_t nr, double* dst,
                    int64_t off, const int** defer = nullptr) {
      const int64_t n = nr * A;
      if (n == 0) return;
      if (rows_i32_on()) {
        int* h32 = w.s_i32.get(at + nqa) + off;
        if ((tab ? dmlp_cpu_rows_i32_rows(tab, nr, (int)A, h32) : dmlp_cpu_rows_i32(src, n, h32)) ==
            0) {
          int* d32 = w.d_i32.get(at + nqa) + off;
          CK(dmlp::dma_copy(d32, h32, n * 4, w.side));
          if (defer) {
            *defer = d32;
            return;
          }
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
      rows(a->X, a->Xr, N, Xd, 0, &i32_.X);
      rows(a->Qx, a->Qr, Q, Qd, at, &i32_.Q);
      defer_f64(Xd, Qd, nx, nqa);
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
                            (pl || dr_on() || dr_auto(N, A, kmin, kmax) || dmlp_host_threads() >= 2)));
    // device render (opt-in, DMLP_DEVICE_RENDER=1): the GPU renders the screen operands from the
    // landed rows.  With a plane every rank must render the same slice kinds, so a plane step
    // always renders on the host (a device-render rank never renders its image slices)
    bool dr = x1_front && !pl && (dr_on() || dr_auto(N, A, kmin, kmax));
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
    // The last chunk's screen is what the transfer does not hide: with F the slices one launch
    // needs to fill the GPU (one per query block and wave slot), a chunk of w < F slices runs at
    // w / F of the chip, so the exposed tail is T * max(1 / chunks, F / S) for a whole-scan screen
    // time T — 8 chunks of F slices each (S = 8 F) cut it to T / 8, and more slices only add
    // (query, slice) lists to the refine (profiles/r11a_large_n_pipeline.jsonl: N = 1e6 at S = F
    // ran every chunk at 1/8 of the chip, 11.4 ms; at S = 4 F 5.2 ms; N = 1e7 at 4 chunks 50 ms)
    int S_all = 0, n_chunks = 1;
    if (dr && x1_front && all_a) {
      const int S1 = x1_slices((int)Q, KT, kmax, nt);
      const int nqb = (int)((Q + dmlp_screen_x1_cols(KT, kmax) - 1) / dmlp_screen_x1_cols(KT, kmax));
      const int F = std::max(1, (dmlp_screen_x1_waves_per_cu_kt(KT, kmax) * g_tune.num_cus + nqb - 1) / nqb);
      int64_t S_cap = std::min<int64_t>(256, nt / 16);  // (refine: <= 256 slices; >= 16 tiles each)
      if (kmax > 32) S_cap = std::min<int64_t>(S_cap, nt * 64 / (32 * kmax));
      S_all = (int)std::max<int64_t>(S1, std::min<int64_t>((int64_t)kEarlySlices * F, S_cap));
      n_chunks = std::min(kEarlySlices, std::max(1, S_all / F));
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
    int rendered = -1;  // the last chunk issued
    std::vector<std::pair<int64_t, int64_t>> x_i32_rows;  // dataset rows rendered from int32
    bool x_f64_rows = false;                               // ... and some from fp64
    const int* x_i32_base = nullptr;                       // (the int32 rows' base: row 0)
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
          // the chunk's rows on the side stream, its render on the render stream behind them:
          // the copies run back to back on the SDMA engine while the renders overlap them (in
          // one stream each copy waited for the previous chunk's render)
          if (t1 > t0) {
            const int* s32 = a->X32d;  // (the xGMI replica: rendered straight from the device)
            const double* s64 = nullptr;
            if (!s32) ship(a->X, a->Xr, std::min(N, t0 * 64), std::min(N, t1 * 64), 0, Xd, &s32, &s64);
            // int32 rows stay int32 (the refines read them; fp64 only on demand, defer_f64)
            if (s32) x_i32_rows.emplace_back(std::min(N, t0 * 64), std::min(N, t1 * 64));
            else x_f64_rows = true;
            x_i32_base = s32 ? s32 : x_i32_base;
            hipStream_t rs = w.render_stream();
            CK(hipEventRecord(w.ev_copy[c], w.side));
            CK(hipStreamWaitEvent(rs, w.ev_copy[c], 0));
            CKL(dmlp_render_rows(KT, A, s32, s64 ? s64 : s32 ? nullptr : Xd, t0 * 64,
                                 (t1 - t0) * 64, N, mud, nullptr, 0, xhi_d, xin_d,
                                 const_cast<void*>(hx.xrow), words + kW_XNMAX, rbad, drw + c,
                                 nullptr, rs));
            CK(hipEventRecord(w.ev_chunk[c], rs));
          } else {
            CK(hipEventRecord(w.ev_chunk[c], w.side));
          }
          rendered = c;
          return;
        }
        if (!x_i32_rows.empty()) {
          if (!x_f64_rows) {  // every chunk int32: the refines read them, fp64 on demand
            i32_.X = x_i32_base;
            defer_f64(Xd, Qd, N * A, Q * A);
          } else {  // a chunk crossed as fp64: the int32 chunks' fp64 rows now, behind the renders
            hipStream_t rs = w.render_stream();
            for (auto& rg : x_i32_rows)
              CKL(dmlp_rows_from_i32(x_i32_base + rg.first * A, (rg.second - rg.first) * A,
                                     Xd + rg.first * A, rs));
            CK(hipEventRecord(w.ev_chunk[std::max(0, rendered)], rs));
          }
        }
        // (the renders are in order on their stream: the last chunk's event covers them all)
        if (rendered >= 0) CK(hipStreamWaitEvent(w.side, w.ev_chunk[rendered], 0));
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
    // report_mode 1 into page-locked memory the GPU addresses: the format kernel writes the text
    // there across PCIe, no device staging and no D2H copy of the whole bound on the tail
    char* direct = want_report && a->report_mode == 1 && g_tune.report_direct
                       ? host_device_view(a->report_dst, (size_t)dmlp_format_bound((int)Q))
                       : nullptr;
    char* text = !want_report ? nullptr
                 : direct     ? direct
                              : w.d_text.get((size_t)dmlp_format_bound((int)Q));
    // ---- dispatch: screens on `st`, the rows behind the first of them on the side stream
    auto run_local = [&](bool with_hx, bool rows_pending) {
      std::unique_ptr<Local> Lp(new Local(w));
      Local& L = *Lp;
      L.X = Xd; L.N = N; L.A = A; L.Qx = Qd; L.Q = Q; L.k_host = a->k; L.kstride = kst;
      L.out_d = od; L.out_i = oi; L.labels = lab_d; L.lo = a->label_lo; L.hi = a->label_hi;
      L.lab = olab; L.cs = ocs; L.exact = a->exact != 0; L.st = st;
      L.hx = with_hx ? &hx : nullptr;
      L.rows = w.ev_rows;
      L.i32 = &i32_;
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
    // (page-locked: the pack kernel writes the words straight there, no copy on the tail)
    int64_t* small_dev = (int64_t*)host_device_view((char*)small, 8 * sizeof(int64_t));
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
                         a->early ? estats : nullptr, dr_bad, small_dev ? small_dev : small_d);
      CK(hipGetLastError());
      if (!small_dev) CK(dmlp::dma_copy(small, small_d, 8 * sizeof(int64_t), st));
      if (want_report && a->report_mode == 1 && !direct)
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
    g_stats.report_direct = direct ? 1 : 0;
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
}  // namespace dmlp_pipe

using namespace dmlp_pipe;


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

// The device address the step would write a report_mode 1 text to for [p, p + bytes), or null
// (host_device_view); info (8 words, may be null): the attribute and address-range queries.
extern "C" void* dmlp_host_device_view(void* p, int64_t bytes, int64_t* info) {
  return host_device_view((char*)p, (size_t)std::max<int64_t>(bytes, 0), info);
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
