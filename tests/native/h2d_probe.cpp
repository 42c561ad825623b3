// H2D / D2H probe: API blocking time vs. completion time of hipMemcpyAsync for host memory that
// is (a) a sub-range of one large hipHostMalloc arena, (b) its own hipHostMalloc block, (c)
// pageable malloc.  Used to size the native engine's pinned staging (tools/gpu_h2d_probe.sh).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

static double ms(std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
  return std::chrono::duration<double, std::milli>(b - a).count();
}

static void run(const char* name, char* host, char* dev, size_t n, hipStream_t st, bool d2h) {
  for (int it = 0; it < 3; ++it) {
    auto t0 = std::chrono::steady_clock::now();
    CK(hipMemcpyAsync(d2h ? (void*)host : (void*)dev, d2h ? (void*)dev : (void*)host, n,
                      d2h ? hipMemcpyDeviceToHost : hipMemcpyHostToDevice, st));
    auto t1 = std::chrono::steady_clock::now();
    CK(hipStreamSynchronize(st));
    auto t2 = std::chrono::steady_clock::now();
    std::printf("%-28s %s %6.1f MB  api %7.3f ms  total %7.3f ms  (%5.1f GB/s)\n", name,
                d2h ? "D2H" : "H2D", n / 1e6, ms(t0, t1), ms(t0, t2), n / 1e6 / ms(t0, t2));
  }
}

int main() {
  const size_t n = 33554432;  // 32 MiB
  hipStream_t st;
  CK(hipSetDevice(0));
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  char* dev;
  CK(hipMalloc((void**)&dev, n));
  char* arena;
  const size_t asz = size_t(1) << 30;
  CK(hipHostMalloc((void**)&arena, asz, hipHostMallocDefault));
  for (size_t o = 0; o < asz; o += 4096) arena[o] = 1;
  char* own;
  CK(hipHostMalloc((void**)&own, n, hipHostMallocDefault));
  std::memset(own, 1, n);
  char* pg = (char*)std::malloc(n);
  std::memset(pg, 1, n);
  run("arena sub-range (+256 MB)", arena + (size_t(256) << 20), dev, n, st, false);
  run("arena sub-range (+256 MB)", arena + (size_t(256) << 20), dev, n, st, true);
  run("arena sub-range (+512 MB)", arena + (size_t(512) << 20), dev, n, st, false);
  run("arena sub-range (+768 MB)", arena + (size_t(768) << 20), dev, n, st, true);
  run("own hipHostMalloc", own, dev, n, st, false);
  run("own hipHostMalloc", own, dev, n, st, true);
  run("pageable malloc", pg, dev, n, st, false);
  run("pageable malloc", pg, dev, n, st, true);
  char* reg = (char*)std::aligned_alloc(4096, n);
  std::memset(reg, 1, n);
  CK(hipHostRegister(reg, n, hipHostRegisterDefault));
  run("hipHostRegister'd", reg, dev, n, st, false);
  run("hipHostRegister'd", reg, dev, n, st, true);
  return 0;
}
