// local.hip — dmlp_knn_local (rows already on the device: the sharded strategies' shards, the
// ring's travelling shards, the out-of-core chunks) over the Local dispatcher (local.h), plus the
// pipeline's arenas and A/B switches (pipeline_ctx.h).  pipeline.hip: the dmlp_step front.
#include "local.h"

using namespace dmlp_pipe;

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
    g_stats.report_direct = 0;
    return 0;
  } catch (const Fail& f) {
    return drain_and_fail(wp, st, f.code);
  } catch (const std::bad_alloc&) {
    return drain_and_fail(wp, st, -(int)hipErrorOutOfMemory);
  }
}


// Tuning / A-B switches (see Tuning): "num_cus", "screen", "x1k", "host_ops", "device_render",
// "report_direct".
// Returns the previous value, or -1 for an unknown key.
extern "C" int dmlp_pipeline_set(const char* key, int value) {
  const std::string k = key ? key : "";
  int* f = k == "num_cus" ? &g_tune.num_cus : k == "screen" ? &g_tune.screen
           : k == "x1k" ? &g_tune.x1k : k == "host_ops" ? &g_tune.host_ops
           : k == "device_render" ? &g_tune.device_render
           : k == "report_direct" ? &g_tune.report_direct : nullptr;
  if (!f) return -1;
  const int old = *f;
  *f = value;
  return old;
}


// What the last dmlp_step / dmlp_knn_local did: [0] queries on the exact fp64 path, [1] queries
// escalated from a single-term to a 3-term screen, [2] path (0 host-rendered operands, 2 device
// image), [3] early start, [4] / [5] exact-path queries on the fp64 MFMA screen / those redone
// by the VALU kernel, [6] device render, [7] report written straight into host memory.
extern "C" void dmlp_pipeline_stats(int64_t* out) {
  out[0] = g_stats.n_exact;
  out[1] = g_stats.n_escalated;
  out[2] = g_stats.path;
  out[3] = g_stats.early;
  out[4] = g_stats.n_exact_f64;
  out[5] = g_stats.n_exact_f64_redo;
  out[6] = g_stats.device_render;
  out[7] = g_stats.report_direct;
}

extern "C" void* dmlp_dev_alloc(int64_t bytes) { return dev_alloc((size_t)std::max<int64_t>(bytes, 1)); }
extern "C" void dmlp_dev_free(void* p) { dev_free(p); }
extern "C" void* dmlp_host_alloc(int64_t bytes) { return host_alloc((size_t)std::max<int64_t>(bytes, 1)); }
extern "C" void dmlp_host_free(void* p) { host_free(p); }
