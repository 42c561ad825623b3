// engine_runtime.h — native runtime of the standalone `knn_engine` binary: MPI for process
// bootstrap and host-side control (like the reference's harness, common.cpp:82-133), RCCL over
// xGMI for the data plane, HIP streams, RAII device buffers, and the single-GPU k-NN pipeline
// that drives the libdmlp kernels (the C++ twin of ops/knn.py).
#pragma once
#include <hip/hip_runtime.h>
#include <mpi.h>
#include <rccl/rccl.h>

#include <dirent.h>
#include <sched.h>

#include <algorithm>
#include <cctype>
#include <chrono>
#include <thread>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <stdexcept>
#include <string>
#include <vector>

#include "dmlp.h"

namespace dmlp_rt {

#define HIPCHK(x)                                                                            \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      std::fprintf(stderr, "[knn_engine] HIP error %s at %s:%d\n", hipGetErrorString(e_),    \
                   __FILE__, __LINE__);                                                      \
      MPI_Abort(MPI_COMM_WORLD, 2);                                                          \
    }                                                                                        \
  } while (0)
#define NCCLCHK(x)                                                                           \
  do {                                                                                       \
    ncclResult_t r_ = (x);                                                                   \
    if (r_ != ncclSuccess) {                                                                 \
      std::fprintf(stderr, "[knn_engine] RCCL error %s at %s:%d\n", ncclGetErrorString(r_),  \
                   __FILE__, __LINE__);                                                      \
      MPI_Abort(MPI_COMM_WORLD, 3);                                                          \
    }                                                                                        \
  } while (0)
#define DMLPCHK(x)                                                                           \
  do {                                                                                       \
    int r_ = (x);                                                                            \
    if (r_ != 0) {                                                                           \
      std::fprintf(stderr, "[knn_engine] libdmlp call failed (%d) at %s:%d\n", r_, __FILE__, \
                   __LINE__);                                                                \
      MPI_Abort(MPI_COMM_WORLD, 4);                                                          \
    }                                                                                        \
  } while (0)

// Bump arenas reserved once, in the untimed Engine construction: the reference harness calls
// KNN once per process, so every hipMalloc / hipHostMalloc inside it would be paid in the timed
// region (a 25 MB hipMalloc costs milliseconds; the kernels themselves ~2 ms).  Device arena:
// KNN_POOL_MB (default min(free HBM / 4, 8 GiB)); pinned host arena: KNN_HOST_POOL_MB (default
// 1 GiB).  Allocations past the reservation fall back to hipMalloc / hipHostMalloc.
struct Arena {
  char* base = nullptr;
  size_t size = 0, used = 0;
  void* take(size_t bytes) {
    const size_t b = (bytes + 255) & ~size_t(255);
    if (!base || used + b > size) return nullptr;
    void* p = base + used;
    used += b;
    return p;
  }
  bool owns(const void* p) const { return base && p >= base && p < base + size; }
};
inline Arena& device_arena() { static Arena a; return a; }
inline Arena& host_arena() { static Arena a; return a; }

inline void reserve_arenas() {
  Arena& d = device_arena();
  if (!d.base) {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) fr = 0;
    size_t want = std::min<size_t>(fr / 4, size_t(8) << 30);
    if (const char* e = getenv("KNN_POOL_MB")) want = (size_t)std::atoll(e) << 20;
    if (want && hipMalloc((void**)&d.base, want) == hipSuccess) d.size = want;
    else d.base = nullptr;
  }
  Arena& h = host_arena();
  if (!h.base) {
    size_t want = size_t(1) << 30;
    if (const char* e = getenv("KNN_HOST_POOL_MB")) want = (size_t)std::atoll(e) << 20;
    if (want && hipHostMalloc((void**)&h.base, want, hipHostMallocDefault) == hipSuccess) {
      h.size = want;
      // touch every page now, not on the first copy inside the timed region
      for (size_t o = 0; o < want; o += 4096) h.base[o] = 0;
      // and move every byte once in each direction: the first DMA into a host range pays its
      // mapping (measured ~7 ms for a 6 MB report on the first D2H), untimed here
      const size_t chunk = std::min<size_t>(want, size_t(64) << 20);
      char* d = nullptr;
      if (hipMalloc((void**)&d, chunk) == hipSuccess) {
        for (size_t o = 0; o < want; o += chunk) {
          const size_t n = std::min(chunk, want - o);
          (void)hipMemcpy(d, h.base + o, n, hipMemcpyHostToDevice);
          (void)hipMemcpy(h.base + o, d, n, hipMemcpyDeviceToHost);
        }
        (void)hipFree(d);
      }
    } else {
      h.base = nullptr;
    }
  }
}

// Grow-only device buffer (reused across calls: no hipMalloc in steady state), carved from the
// device arena when it has room.
template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;
  T* get(size_t n) {
    if (n > cap) {
      if (p && !device_arena().owns(p)) HIPCHK(hipFree(p));
      cap = std::max<size_t>(n, 1);
      p = (T*)device_arena().take(cap * sizeof(T));
      if (!p) HIPCHK(hipMalloc(&p, cap * sizeof(T)));
    }
    return p;
  }
  ~DevBuf() {
    if (p && !device_arena().owns(p)) (void)hipFree(p);
  }
};

struct Runtime {
  int rank = 0, world = 1, local = 0, device = 0;
  ncclComm_t nccl = nullptr;
  hipStream_t stream = nullptr;

  bool gpu = false;
  // KNN_DATA_PLANE=host: no RCCL communicator; KnnCore stages transfers through host memory
  // and MPI (several ranks may then share one GPU — test mode)
  bool host_plane = getenv("KNN_DATA_PLANE") && std::string(getenv("KNN_DATA_PLANE")) == "host";

  int numa = -1;  // NUMA node this rank is bound to (bind_numa), -1 if none
  // Pin this rank to the CPUs of its GPU's NUMA node (within its affinity): first-touch then puts
  // the page-locked arenas, the parsed input and the render pool's threads next to the GPU's
  // PCIe root (the Python twin: parallel/comm.py Comm.bind_numa; profiles/r3m_numa.txt).
  // Every thread of the process is re-pinned (the HIP runtime's and MPI's, started before the
  // bind, too), and DMLP_NODE_RANKS tells the render pool how many of the node's `local_world`
  // ranks (local rank r drives GPU r % ndev) share the mask.  KNN_NUMA_BIND=0 disables it.
  static int numa_node(int dev) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), dev) != hipSuccess) return -1;
    for (char* c = bus; *c; ++c) *c = (char)std::tolower((unsigned char)*c);
    int node = -1;
    if (FILE* f = std::fopen((std::string("/sys/bus/pci/devices/") + bus + "/numa_node").c_str(), "r")) {
      if (std::fscanf(f, "%d", &node) != 1) node = -1;
      std::fclose(f);
    }
    return node;
  }
  static int bind_numa(int dev, int local_world = 1, int ndev = 1) {
    if (getenv("KNN_NUMA_BIND") && std::string(getenv("KNN_NUMA_BIND")) == "0") return -1;
    const int node = numa_node(dev);
    if (node < 0) return -1;
    FILE* f = std::fopen(("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist").c_str(), "r");
    if (!f) return -1;
    cpu_set_t want, have;
    CPU_ZERO(&want);
    int lo = 0, hi = 0;
    char sep = 0;
    while (std::fscanf(f, "%d", &lo) == 1) {
      hi = lo;
      sep = (char)std::fgetc(f);
      if (sep == '-') {
        if (std::fscanf(f, "%d", &hi) != 1) break;
        sep = (char)std::fgetc(f);
      }
      for (int c = lo; c <= hi && c < CPU_SETSIZE; ++c) CPU_SET(c, &want);
      if (sep != ',') break;
    }
    std::fclose(f);
    if (sched_getaffinity(0, sizeof(have), &have) != 0) return -1;
    CPU_AND(&want, &want, &have);
    if (CPU_COUNT(&want) == 0 || sched_setaffinity(0, sizeof(want), &want) != 0) return -1;
    if (DIR* d = opendir("/proc/self/task")) {
      while (dirent* e = readdir(d))
        if (e->d_name[0] != '.') (void)sched_setaffinity(std::atoi(e->d_name), sizeof(want), &want);
      closedir(d);
    }
    int share = 0;
    for (int r = 0; r < std::max(1, local_world); ++r) share += numa_node(r % std::max(1, ndev)) == node;
    setenv("DMLP_NODE_RANKS", std::to_string(std::max(1, share)).c_str(), 1);
    return node;
  }
  void init(bool need_gpu = true) {
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &world);
    MPI_Comm shm;
    MPI_Comm_split_type(MPI_COMM_WORLD, MPI_COMM_TYPE_SHARED, rank, MPI_INFO_NULL, &shm);
    MPI_Comm_rank(shm, &local);
    int local_world = 1;
    MPI_Comm_size(shm, &local_world);
    MPI_Comm_free(&shm);
    if (!need_gpu) return;  // serial KD-tree strategy (bench.debug): host only
    gpu = true;
    int ndev = 0;
    HIPCHK(hipGetDeviceCount(&ndev));
    if (ndev == 0) throw std::runtime_error("no HIP device");
    device = local % ndev;
    HIPCHK(hipSetDevice(device));
    numa = bind_numa(device, local_world, ndev);  // before the arenas: pages land next to the GPU
    HIPCHK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    reserve_arenas();
    if (world > 1 && !host_plane) {
      ncclUniqueId id;
      if (rank == 0) NCCLCHK(ncclGetUniqueId(&id));
      MPI_Bcast(&id, sizeof(id), MPI_BYTE, 0, MPI_COMM_WORLD);
      NCCLCHK(ncclCommInitRank(&nccl, world, id, rank));
    }
  }
  void finalize() {
    if (nccl) ncclCommDestroy(nccl);
    if (stream) (void)hipStreamDestroy(stream);
  }
  // Failure detection: with a communicator, wait for the stream by polling so a
  // dead or faulted peer surfaces as an RCCL async error (or a KNN_TIMEOUT_S watchdog expiry,
  // default 600 s) and the job aborts with a rank-tagged message instead of hanging in a
  // collective.  Without one, a plain stream synchronize.
  void sync() {
    if (!gpu) return;
    if (!nccl) {
      HIPCHK(hipStreamSynchronize(stream));
      return;
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (int spin = 0;; ++spin) {
      const hipError_t e = hipStreamQuery(stream);
      if (e == hipSuccess) return;
      if (e != hipErrorNotReady) HIPCHK(e);
      ncclResult_t ae = ncclSuccess;
      NCCLCHK(ncclCommGetAsyncError(nccl, &ae));
      const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (ae != ncclSuccess || s > timeout_s) {
        if (ae != ncclSuccess)
          std::fprintf(stderr, "[knn_engine] rank %d: RCCL async error: %s\n", rank,
                       ncclGetErrorString(ae));
        else
          std::fprintf(stderr, "[knn_engine] rank %d: watchdog: stream not drained after %.0f s "
                       "(peer failure?)\n", rank, s);
        ncclCommAbort(nccl);
        nccl = nullptr;
        MPI_Abort(MPI_COMM_WORLD, 5);
      }
      if (spin > 2000) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }
  double timeout_s = getenv("KNN_TIMEOUT_S") ? std::atof(getenv("KNN_TIMEOUT_S")) : 600.0;
};

// Opt-in per-phase tracer (KNN_TRACE=1): phase boundaries are hipEvents recorded
// on the engine stream (no host syncs inside the timed region), host clocks for CPU-only runs.
// Lines go to stderr as "[dmlp-trace] rank r <phase> <ms> ms" — never starting with "Time taken"
// (run_bench.sh:40 greps the first such line).
struct Trace {
  bool on = false;
  int rank = 0;
  hipStream_t st = nullptr;
  std::vector<std::string> names;
  std::vector<hipEvent_t> ev;
  std::vector<double> host_ms;
  std::chrono::steady_clock::time_point t0;

  void init(int r, hipStream_t s) {
    const char* e = getenv("KNN_TRACE");
    on = e && *e && std::string(e) != "0";
    rank = r;
    st = s;
  }
  void begin() {
    names.clear(); ev.clear(); host_ms.clear();
    t0 = std::chrono::steady_clock::now();
    if (on) mark("begin");
  }
  void mark(const char* name) {
    if (!on) return;
    names.emplace_back(name);
    host_ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    if (st) {
      hipEvent_t e;
      HIPCHK(hipEventCreate(&e));
      HIPCHK(hipEventRecord(e, st));
      ev.push_back(e);
    }
  }
  // Durations of the phases ending at each mark (after the run; synchronizes the stream).
  std::vector<std::pair<std::string, double>> finish() {
    std::vector<std::pair<std::string, double>> out;
    if (!on) return out;
    if (st) HIPCHK(hipStreamSynchronize(st));
    for (size_t i = 1; i < names.size(); ++i) {
      double ms = host_ms[i] - host_ms[i - 1];
      if (st) {
        float f = 0;
        HIPCHK(hipEventElapsedTime(&f, ev[i - 1], ev[i]));
        ms = f;
      }
      out.emplace_back(names[i], ms);
      std::fprintf(stderr, "[dmlp-trace] rank %d %s %.3f ms\n", rank, names[i].c_str(), ms);
    }
    for (auto e : ev) (void)hipEventDestroy(e);
    ev.clear();
    return out;
  }
};

// Balanced block partition (bench_1 @0xc5b2).
inline void block_partition(int64_t n, int parts, std::vector<int64_t>& cnt,
                            std::vector<int64_t>& off) {
  cnt.assign(parts, n / parts);
  off.assign(parts, 0);
  for (int i = 0; i < parts; ++i) cnt[i] += (i < n % parts) ? 1 : 0;
  for (int i = 1; i < parts; ++i) off[i] = off[i - 1] + cnt[i - 1];
}

// ---------------------------------------------------------------- single-GPU k-NN pipeline
struct LocalKnn {
  hipStream_t st = nullptr;
  Runtime* rt = nullptr;  // its sync() (watchdog) when set
  void wait() {
    if (rt) rt->sync();
    else HIPCHK(hipStreamSynchronize(st));
  }
  DevBuf<double> mu;
  DevBuf<char> xfrag;
  DevBuf<float> xinit;
  DevBuf<unsigned> words;  // [0] xnmax bits, [1] bad
  DevBuf<short> qhi, qlo;
  DevBuf<float> qn, cand_h;
  DevBuf<int> qidx_a, qidx_b, qidx_c, qidx_e, qidx_e2, qidx_f, kdev, cand_ids, cand_cnt, status;
  DevBuf<char> fb_ws;
  int KT = 1;
  int64_t N = 0;
  int A = 0;
  const double* X = nullptr;

  static float eps_rel(int A) {
    return 2.0f * (float)(3.0 * std::ldexp(1.0, -16) + (3 * A + 8) * std::ldexp(1.0, -24));
  }

  void prepare(const double* Xd, int64_t N_, int A_) {
    X = Xd;
    N = N_;
    A = A_;
    KT = dmlp_screen_kt(A);
    if (KT > 8 || N == 0) return;
    const int64_t nt = (N + 63) / 64;
    HIPCHK(hipMemsetAsync(words.get(2), 0, 2 * sizeof(unsigned), st));
    DMLPCHK(dmlp_center(Xd, N, A, mu.get(A), st));
    DMLPCHK(dmlp_prep_data(Xd, N, A, mu.p, KT, xfrag.get(nt * 64 * KT * 32 * 2 * sizeof(short)), xinit.get(nt * 64),
                           words.p, words.p + 1, st));
  }

  static int slices_stream(int nq, int qw, int64_t n_tiles, int waves_per_cu, int64_t s_lo = 1) {
    const int nqb = (nq + qw - 1) / qw;
    const int slots = waves_per_cu * 256;
    const int s_min = (int)std::max<int64_t>(std::max<int64_t>(1, s_lo),
                                             (n_tiles * 64 + (1ll << 29) - 1) >> 29);
    if (nqb >= slots) return s_min;
    int best = s_min;
    double best_eff = 0;
    for (int S = s_min; S < s_min + 64 && S <= std::max<int64_t>(s_min, n_tiles / 4); ++S) {
      const double w = (double)nqb * S;
      const double eff = w / (std::ceil(w / slots) * slots);
      if (eff >= 0.9) return S;
      if (eff > best_eff + 1e-9) { best = S; best_eff = eff; }
    }
    return best;
  }
  static int slices_lds(int nq, int waves, int64_t n_tiles) {
    const int nqb = (nq + waves * 16 - 1) / (waves * 16);
    int S = 1;
    while ((int64_t)nqb * S < 512 && S * 2 <= std::max<int64_t>(1, n_tiles) && S < 256) S *= 2;
    return S;
  }

  // The host-rendered single-term operands (host_prep.cpp, fp16, hl = 1), already on the device
  // (or in flight on the stream): the x1 class screens with them, so neither the dataset image
  // nor the query fragments are rendered on the device unless a query needs the 3-term screens.
  struct HostX1 {
    const void* xhi = nullptr;
    const float* xin = nullptr;
    unsigned* words = nullptr;  // [0] xnmax bits, [1] bad (0)
    const void* qhi = nullptr;
    const float* qn = nullptr;
  };
  // grow-only page-locked ints (arena-backed while the arena has room)
  struct PinnedInts {
    int* p = nullptr;
    size_t n = 0;
    int* get(int64_t m) {
      if ((size_t)m > n) {
        if (p && !host_arena().owns(p)) (void)hipHostFree(p);
        const size_t want = std::max<size_t>((size_t)m, 1024);
        p = (int*)host_arena().take(want * sizeof(int));
        if (!p && hipHostMalloc((void**)&p, want * sizeof(int), hipHostMallocDefault) != hipSuccess)
          throw std::runtime_error("page-locked allocation failed");
        n = want;
      }
      return p;
    }
    ~PinnedInts() {
      if (p && !host_arena().owns(p)) (void)hipHostFree(p);
    }
  } kk_h_, ident_h_, kp_h_;
  // the two-pass large-k x1 screen: first-pass lists / thresholds, per-query seeds, k'
  DevBuf<int> k1_ids_, k1_cnt_, kp_d_;
  DevBuf<float> k1_h_, k1_seed_;
  DevBuf<int> ident_, ovf_;
  int64_t ident_len_ = 0;
  int* identity(int64_t n) {  // device 0, 1, ..., n-1 (grow-only)
    int* p = ident_.get(std::max<int64_t>(n, 1));
    if (ident_len_ < n) {
      int* h = ident_h_.get(n);
      for (int64_t i = 0; i < n; ++i) h[i] = (int)i;
      HIPCHK(hipMemcpyAsync(p, h, n * sizeof(int), hipMemcpyHostToDevice, st));
      ident_len_ = n;
    }
    return p;
  }

  // Exact top-k (+ vote/checksum when labels != nullptr) of queries Qx [Q][A] (device).
  // k_host drives dispatch; out_* are [Q][kstride]; lab/cs may be null.  Per-query classes:
  // 1 <= k <= 32 the single-term x1 screen (host operands hx when given, else the device image
  // prepare() rendered), 32 < k <= 256 the 3-term LDS screen (cap 256 / 512), the rest the exact path; a query
  // whose x1 candidates overflow escalates alone (3-term screen, then exact).  With hx the
  // fp64 rows X / Qx may still be in flight: everything that reads them waits for `rows`, and
  // the device image (for 3-term work) is rendered on first need (prepare() was not called).
  void run(const double* Qx, int64_t Q, const int* k_host, int kstride, double* out_d,
           int* out_i, const int* labels, int lab_lo, int lab_hi, int* lab, uint64_t* cs,
           const HostX1* hx = nullptr, hipEvent_t rows = nullptr,
           const std::function<void()>& issue_rows = nullptr) {
    if (Q == 0) return;
    // issue_rows() enqueues the fp64 row copies (recording `rows`): right after the first
    // screen launch, so that this call's small copies never queue behind them on the copy
    // engine, or before the first wait on them if no screen runs
    bool rows_issued = !issue_rows;
    auto launch_rows = [&]() {
      if (!rows_issued) { issue_rows(); rows_issued = true; }
    };
    std::vector<int> a, b, c, f, rest;
    // page-locked k (a pageable source would make the copy wait for the stream)
    int* kk = kk_h_.get(Q);
    // A <= 256 (KT <= 8): every class on a screen (the LDS 3-term screen streams KT = 8 tiles
    // as two 32 KiB stages); wider rows take the exact path
    const bool lds_ok = KT <= 8;
    const bool x1_ok = dmlp_screen_x1_qw(KT) > 0;
    const bool screen = (lds_ok || x1_ok) && N > 0;
    // the common case (every k in [1, 32], k <= N, on the x1 class) needs no per-class lists
    bool all_a = screen && (x1_ok || !hx);
    for (int64_t q = 0; q < Q; ++q) {
      kk[q] = (int)std::min<int64_t>(k_host[q], N);
      all_a = all_a && k_host[q] >= 1 && k_host[q] <= 32 && k_host[q] <= N;
    }
    for (int64_t q = 0; q < Q && !all_a; ++q) {
      if (kk[q] < 1) { rest.push_back((int)q); all_a = false; continue; }
      if (screen && kk[q] <= 32 && (x1_ok || !hx)) a.push_back((int)q);
      else if (screen && lds_ok && kk[q] <= 128) { b.push_back((int)q); all_a = false; }
      else if (screen && lds_ok && kk[q] <= 256) { c.push_back((int)q); all_a = false; }
      else { f.push_back((int)q); all_a = false; }
      if (k_host[q] > N) rest.push_back((int)q);
    }
    bool rows_waited = rows == nullptr;
    auto wait_rows = [&]() {
      launch_rows();
      if (!rows_waited) { HIPCHK(hipStreamWaitEvent(st, rows, 0)); rows_waited = true; }
    };
    bool dev_ready = hx == nullptr;  // device image (prepare) + device query fragments
    bool qprep = false;
    auto need_dev = [&]() {
      if (!dev_ready) {
        wait_rows();
        prepare(X, N, A);
        dev_ready = true;
      }
      if (!qprep) {
        DMLPCHK(dmlp_prep_queries(Qx, Q, A, mu.p, KT, qhi.get(Q * KT * 32), qlo.get(Q * KT * 32),
                                  qn.get(Q), words.p + 1, st));
        qprep = true;
      }
    };
    int* kd = kdev.get(Q);
    HIPCHK(hipMemcpyAsync(kd, kk, Q * sizeof(int), hipMemcpyHostToDevice, st));
    int* stat = status.get(Q);
    const bool fin = labels != nullptr;
    // (the x1 refine writes every row's padding and status itself; the other paths need fills)
    bool filled = false;
    auto fill = [&]() {
      if (filled) return;
      // padding (+inf, -1) for k > N, like bench_2's {1e18, -1} sentinel
      HIPCHK(hipMemsetAsync(out_i, 0xff, (size_t)Q * kstride * sizeof(int), st));
      DMLPCHK(dmlp_fill_f64(out_d, (int64_t)Q * kstride, INFINITY, st));
      HIPCHK(hipMemsetAsync(stat, 0, Q * sizeof(int), st));
      filled = true;
    };
    int* ovf = ovf_.get(1);
    HIPCHK(hipMemsetAsync(ovf, 0, sizeof(int), st));
    // once, before any kernel writes results: every refine writes its queries' padding and
    // status itself, so the fill is only needed for rows no refine covers (exact path, k < 1)
    if (!all_a || !hx) fill();
    if (all_a || !a.empty() || !b.empty() || !c.empty()) {
      const float er = eps_rel(A);
      const int64_t nt = (N + 63) / 64;
      const int qw = dmlp_screen_stream_qw(KT);
      // default: single-term screen (screen_x1.hip); KNN_SCREEN=stream: 3-term streaming
      const char* impl = std::getenv("KNN_SCREEN");
      const bool use_x1 = x1_ok && (!lds_ok || !(impl && std::string(impl) == "stream" && !hx));
      // impl: 0 x1 (single-term), 1 stream (3-term, k <= 32), 2 LDS-shared (3-term, k <= 256),
      // 3 LDS-shared single-term on the host operands hx (k <= 256: no device image), 4 the
      // two-pass single-term x1 screen on hx (k <= 256; ops/knn.py _x1k_pass)
      auto pass = [&](const std::vector<int>* idx, int impl, DevBuf<int>& qbuf) {
        const int nq = idx ? (int)idx->size() : (int)Q;
        int* qi;
        if (idx) {
          qi = qbuf.get(nq);
          HIPCHK(hipMemcpyAsync(qi, idx->data(), nq * sizeof(int), hipMemcpyHostToDevice, st));
        } else {
          qi = identity(Q);
        }
        int kcls = 1;
        if (idx) for (int q : *idx) kcls = std::max(kcls, kk[q]);
        else for (int64_t q = 0; q < Q; ++q) kcls = std::max(kcls, kk[q]);
        const int cap = impl == 0 ? dmlp_screen_x1_cap(kcls)
                        : impl == 1 ? dmlp_screen_stream_cap(kcls)
                                    : (kcls <= 32 ? 128 : kcls <= 128 ? 256 : 512);
        const int S = impl == 0 ? slices_stream(nq, dmlp_screen_x1_cols(KT, kcls), nt,
                                                dmlp_screen_x1_waves_per_cu_kt(KT, kcls),
                                                dmlp_screen_x1_min_slices(nt))
                      : impl == 1 ? slices_stream(nq, qw, nt, dmlp_screen_stream_waves_per_cu(kcls))
                                  : slices_lds(nq, dmlp_screen_waves_hl(KT, cap, impl == 3 ? 1 : 2), nt);
        int* ci = cand_ids.get((size_t)nq * S * cap);
        int* cc = cand_cnt.get((size_t)nq * S);
        if (impl == 0) {
          float* ch = cand_h.get((size_t)nq * S * 2);
          const void* xf = hx ? hx->xhi : (const void*)xfrag.p;
          const float* xi = hx ? hx->xin : xinit.p;
          unsigned* wd = hx ? hx->words : words.p;
          const void* qh = hx ? hx->qhi : (const void*)qhi.p;
          const float* qnn = hx ? hx->qn : qn.p;
          const int hl = hx ? 1 : 2;
          DMLPCHK(dmlp_screen_x1(KT, hl, A, xf, xi, nt, N, qh, qnn, qi, kd, nq, kcls, wd, wd + 1, S,
                                 ci, cc, ch, st));
          wait_rows();  // (issues the row copies first) the re-rank reads the fp64 rows
          DMLPCHK(dmlp_refine_groups(cap, ci, cc, ch, S, X, A, Qx, xf, xi, qh, KT, hl, N,
                                     idx ? qi : nullptr, kd, nq, out_d, out_i, kstride,
                                     fin ? labels : nullptr, lab_lo, lab_hi, lab, cs, stat, ovf,
                                     st));
          return;
        }
        if (impl == 4) {
          // pass 1: S1 slices at k' = ceil(k / S1) -> per-query seeds; pass 2: COLLECT at the
          // seed into X1K_CCAP group ids per (query, slice); the large-k group refine
          constexpr int kCcap = 1024, kS1 = 16;
          const int S2 = slices_stream(nq, dmlp_screen_x1_cols(KT, 16), nt,
                                       dmlp_screen_x1_waves_per_cu_kt(KT, 16),
                                       dmlp_screen_x1_min_slices(nt));
          const int S1 = std::max(kS1, S2);
          int* kp = kp_h_.get(Q);
          for (int64_t q = 0; q < Q; ++q) kp[q] = (std::max(kk[q], 1) + S1 - 1) / S1;
          int kmax1 = 1;
          for (int q : *idx) kmax1 = std::max(kmax1, kp[q]);
          int* kpd = kp_d_.get(Q);
          HIPCHK(hipMemcpyAsync(kpd, kp, Q * sizeof(int), hipMemcpyHostToDevice, st));
          const int cap1 = dmlp_screen_x1_cap(kmax1);
          int* i1 = k1_ids_.get((size_t)nq * S1 * cap1);
          int* c1 = k1_cnt_.get((size_t)nq * S1);
          float* h1 = k1_h_.get((size_t)nq * S1 * 2);
          float* hs = k1_seed_.get(nq);
          int* i2 = cand_ids.get((size_t)nq * S2 * kCcap);
          int* c2 = cand_cnt.get((size_t)nq * S2);
          float* h2 = cand_h.get((size_t)nq * S2 * 2);
          DMLPCHK(dmlp_screen_x1(KT, 1, A, hx->xhi, hx->xin, nt, N, hx->qhi, hx->qn, qi, kpd, nq,
                                 kmax1, hx->words, hx->words + 1, S1, i1, c1, h1, st));
          DMLPCHK(dmlp_x1_seed(h1, c1, S1, nq, hs, st));
          DMLPCHK(dmlp_screen_x1_collect(KT, A, hx->xhi, hx->xin, nt, N, hx->qhi, hx->qn, qi, kd,
                                         nq, hx->words, hx->words + 1, hs, kCcap, S2, i2, c2, h2,
                                         st));
          wait_rows();
          DMLPCHK(dmlp_refine_groups2(kCcap, i2, c2, h2, S2, X, A, Qx, hx->xhi, hx->xin, hx->qhi,
                                      KT, 1, N, qi, kd, nq, out_d, out_i, kstride,
                                      fin ? labels : nullptr, lab_lo, lab_hi, lab, cs, stat, ovf,
                                      1, st));
          return;
        }
        if (impl == 3) {
          DMLPCHK(dmlp_screen_hl(KT, cap, 1, A, hx->xhi, hx->xin, nt, hx->qhi, nullptr, hx->qn, qi,
                                 kd, nq, hx->words, hx->words + 1, 0.0f, S, ci, cc, st));
          wait_rows();
          DMLPCHK(dmlp_refine(cap, ci, cc, S, X, A, Qx, qi, kd, nq, out_d, out_i, kstride,
                              fin ? labels : nullptr, lab_lo, lab_hi, lab, cs, stat, ovf, st));
          return;
        }
        need_dev();
        if (impl == 1)
          DMLPCHK(dmlp_screen_stream(KT, xfrag.p, xinit.p, nt, qhi.p, qlo.p, qn.p, qi, kd, nq, kcls,
                                     words.p, words.p + 1, er, S, ci, cc, st));
        else
          DMLPCHK(dmlp_screen(KT, cap, xfrag.p, xinit.p, nt, qhi.p, qlo.p, qn.p, qi, kd, nq,
                              words.p, words.p + 1, er, S, ci, cc, st));
        DMLPCHK(dmlp_refine(cap, ci, cc, S, X, A, Qx, qi, kd, nq, out_d, out_i, kstride,
                            fin ? labels : nullptr, lab_lo, lab_hi, lab, cs, stat, ovf, st));
      };
      if (!hx) need_dev();  // the device operands of every screen
      const int first_a = use_x1 ? 0 : (qw > 0 ? 1 : 2);
      if (all_a || !a.empty()) pass(all_a ? nullptr : &a, first_a, qidx_a);
      // k > 32 on the single-term LDS screen when the host operands are here (KNN_LDS_SINGLE=0:
      // always 3-term); its overflows escalate to the 3-term LDS screen below
      const char* ls = std::getenv("KNN_LDS_SINGLE");
      const int bc_impl = (hx && !(ls && std::string(ls) == "0") &&
                           dmlp_screen_waves_hl(KT, 128, 1) > 0) ? 3 : 2;
      // ... and by the two-pass x1 screen on the same operands (KNN_X1K=0: the LDS screen)
      const char* xk = std::getenv("KNN_X1K");
      const bool x1k = bc_impl == 3 && x1_ok && !(xk && std::string(xk) == "0");
      if (x1k && (!b.empty() || !c.empty())) {
        std::vector<int> bc(b);
        bc.insert(bc.end(), c.begin(), c.end());
        pass(&bc, 4, qidx_b);
      } else {
        if (!b.empty()) pass(&b, bc_impl, qidx_b);
        if (!c.empty()) pass(&c, bc_impl, qidx_c);
      }
      // one host sync: the overflow count (4 bytes); the per-query status only when some
      // screened query overflowed
      int novf = 0;
      HIPCHK(hipMemcpyAsync(&novf, ovf, sizeof(int), hipMemcpyDeviceToHost, st));
      wait();
      if (novf) {
        std::vector<int> sh(Q);
        HIPCHK(hipMemcpyAsync(sh.data(), stat, Q * sizeof(int), hipMemcpyDeviceToHost, st));
        wait();
        std::vector<int> esc, esc_bc;
        if (first_a == 0 && all_a) {
          for (int64_t q = 0; q < Q; ++q)
            if (sh[q]) esc.push_back((int)q);
        } else if (first_a == 0) {
          for (int q : a)
            if (sh[q]) esc.push_back(q);
        }
        if (bc_impl == 3) {
          for (int q : b)
            if (sh[q]) esc_bc.push_back(q);
          for (int q : c)
            if (sh[q]) esc_bc.push_back(q);
        }
        if (!(qw > 0 || lds_ok)) esc.clear();
        if (!esc.empty() || !esc_bc.empty()) {
          // single-term overflow (data too tight for its bound): those queries alone go to the
          // 3-term screen
          HIPCHK(hipMemsetAsync(ovf, 0, sizeof(int), st));
          for (int q : esc) HIPCHK(hipMemsetAsync(stat + q, 0, sizeof(int), st));
          for (int q : esc_bc) HIPCHK(hipMemsetAsync(stat + q, 0, sizeof(int), st));
          if (!esc.empty()) pass(&esc, qw > 0 ? 1 : 2, qidx_e);
          if (!esc_bc.empty()) pass(&esc_bc, 2, qidx_e2);
          HIPCHK(hipMemcpyAsync(&novf, ovf, sizeof(int), hipMemcpyDeviceToHost, st));
          wait();
          if (novf) {
            HIPCHK(hipMemcpyAsync(sh.data(), stat, Q * sizeof(int), hipMemcpyDeviceToHost, st));
            wait();
          } else {
            std::fill(sh.begin(), sh.end(), 0);
          }
        }
        for (int64_t q = 0; q < Q; ++q)
          if (sh[q]) f.push_back((int)q);
      }
    }
    if (!f.empty()) {
      wait_rows();
      std::sort(f.begin(), f.end());
      // k <= dmlp_exact_topk_kmax_for(N) (64, or 256 for large N): fused streaming exact kernel
      // (exact.hip); k <= 2048: radix select over exact rows; larger k: rows + segmented sort
      std::vector<int> fused, small, big;
      const int kf = dmlp_exact_topk_kmax_for(N), ksel = dmlp_fallback_select_kmax();
      int kfmax = 0;
      for (int q : f) {
        if (kk[q] <= kf) { fused.push_back(q); kfmax = std::max(kfmax, kk[q]); }
        else (kk[q] <= ksel ? small : big).push_back(q);
      }
      int* qi = qidx_f.get(f.size());
      size_t base = 0;
      if (!fused.empty()) {
        HIPCHK(hipMemcpyAsync(qi, fused.data(), fused.size() * sizeof(int), hipMemcpyHostToDevice, st));
        DMLPCHK(dmlp_exact_topk(X, N, A, Qx, qi, kd, (int)fused.size(), kfmax, out_d, out_i,
                                kstride, st));
        base += fused.size();
      }
      for (int pass = 0; pass < 2; ++pass) {
        const std::vector<int>& v = pass == 0 ? small : big;
        if (v.empty()) continue;
        HIPCHK(hipMemcpyAsync(qi + base, v.data(), v.size() * sizeof(int), hipMemcpyHostToDevice, st));
        const int rows_ = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)v.size(),
                                                                      (1ll << 27) / std::max<int64_t>(1, N)));
        const int64_t wsb = pass == 0 ? dmlp_fallback_select_bytes(rows_, N) : dmlp_fallback_bytes(rows_, N);
        char* ws = fb_ws.get(wsb);
        for (size_t c0 = 0; c0 < v.size(); c0 += rows_) {
          const int nb = (int)std::min<size_t>(rows_, v.size() - c0);
          if (pass == 0)
            DMLPCHK(dmlp_fallback_select(X, N, A, Qx, qi + base + c0, kd, nb, ws, wsb, out_d, out_i,
                                         kstride, st));
          else
            DMLPCHK(dmlp_fallback_topk(X, N, A, Qx, qi + base + c0, kd, nb, ws, wsb, out_d, out_i,
                                       kstride, st));
        }
        base += v.size();
      }
      rest.insert(rest.end(), f.begin(), f.end());
    }
    if (fin && !rest.empty()) {
      wait_rows();
      std::sort(rest.begin(), rest.end());
      rest.erase(std::unique(rest.begin(), rest.end()), rest.end());
      // the vote/checksum of k > N queries covers the padding, so use the unclamped k
      int* kfull = kdev.get(Q);  // safe: refine already consumed the clamped k on this stream
      HIPCHK(hipMemcpyAsync(kfull, k_host, Q * sizeof(int), hipMemcpyHostToDevice, st));
      int* qi = qidx_f.get(std::max<size_t>(rest.size(), f.size()));
      HIPCHK(hipMemcpyAsync(qi, rest.data(), rest.size() * sizeof(int), hipMemcpyHostToDevice, st));
      DMLPCHK(dmlp_finalize(out_d, out_i, kstride, kfull, qi, (int)rest.size(), labels, lab_lo,
                            lab_hi, lab, cs, st));
      wait();  // host vectors above die at scope exit
    }
  }
};

}  // namespace dmlp_rt
