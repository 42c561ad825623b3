// engine_runtime.h — native runtime of the standalone `knn_engine` binary and the engine.h
// drop-in: MPI for process bootstrap and host-side control (like the reference's harness,
// common.cpp:82-133), RCCL over xGMI for the data plane, HIP streams, RAII device buffers over the
// library's arenas.  The single-GPU k-NN itself is libdmlp's one pipeline (pipeline.hip).
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
// region (a 25 MB hipMalloc costs milliseconds; the kernels themselves ~2 ms).  They are the
// library's (pipeline.hip dmlp_arena_reserve), shared with the pipeline's own buffers.  Device:
// KNN_POOL_MB (default min(free HBM / 4, 8 GiB)); page-locked host: KNN_HOST_POOL_MB (default
// 1 GiB).  Allocations past the reservation fall back to hipMalloc / hipHostMalloc.
inline void reserve_arenas() {
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) fr = 0;
  size_t dev = std::min<size_t>(fr / 4, size_t(8) << 30);
  if (const char* e = getenv("KNN_POOL_MB")) dev = (size_t)std::atoll(e) << 20;
  size_t host = size_t(1) << 30;
  if (const char* e = getenv("KNN_HOST_POOL_MB")) host = (size_t)std::atoll(e) << 20;
  (void)dmlp_arena_reserve((int64_t)dev, (int64_t)host);
}

// Grow-only device buffer (reused across calls: no hipMalloc in steady state), carved from the
// device arena when it has room.
template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;
  T* get(size_t n) {
    if (n > cap) {
      dmlp_dev_free(p);
      cap = std::max<size_t>(n, 1);
      p = (T*)dmlp_dev_alloc((int64_t)(cap * sizeof(T)));
      if (!p) HIPCHK(hipErrorOutOfMemory);
    }
    return p;
  }
  ~DevBuf() { dmlp_dev_free(p); }
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
    // ranks of this node on the same GPU (a host-plane rehearsal): the native step's early start
    // stays off for them (pipeline.hip early_on; profiles/r7h_host_budget.md)
    {
      int same = 0;
      for (int r = 0; r < local_world; ++r) same += r % ndev == device;
      setenv("DMLP_DEVICE_RANKS", std::to_string(std::max(1, same)).c_str(), 1);
    }
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

}  // namespace dmlp_rt
