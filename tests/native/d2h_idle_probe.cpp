// D2H start-up probe: does a device->host copy pay a start-up cost after the copy path idled,
// after a burst of host->device copies, or after a kernel?  (native engine report copy, r2)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

__global__ void k_touch(char* p, size_t n) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] = (char)i;
}

static double d2h(const char* what, char* h, char* d, size_t n, hipStream_t st) {
  auto t0 = std::chrono::steady_clock::now();
  CK(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, st));
  CK(hipStreamSynchronize(st));
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  std::printf("%-40s D2H %8zu B  %8.3f ms\n", what, n, ms);
  return ms;
}

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const size_t big = size_t(32) << 20, small = 140 << 10;
  char *d, *h;
  CK(hipMalloc((void**)&d, big));
  CK(hipHostMalloc((void**)&h, big, hipHostMallocDefault));
  for (size_t o = 0; o < big; o += 4096) h[o] = 0;
  CK(hipMemcpyAsync(d, h, big, hipMemcpyHostToDevice, st));
  CK(hipStreamSynchronize(st));
  d2h("warm-up", h, d, big, st);
  d2h("right after", h, d, small, st);
  for (int ms : {5, 50, 300}) {
    std::this_thread::sleep_for(std::chrono::milliseconds(ms));
    char what[64];
    std::snprintf(what, sizeof what, "after %d ms idle", ms);
    d2h(what, h, d, small, st);
  }
  CK(hipMemcpyAsync(d, h, big / 2, hipMemcpyHostToDevice, st));
  d2h("queued behind a 16 MB H2D (includes it)", h, d, small, st);
  k_touch<<<1024, 256, 0, st>>>(d, big);
  d2h("after a kernel", h, d, small, st);
  hipStream_t st2;
  CK(hipStreamCreateWithFlags(&st2, hipStreamNonBlocking));
  d2h("first copy on a new stream", h, d, small, st2);
  d2h("second copy on it", h, d, small, st2);
  std::this_thread::sleep_for(std::chrono::milliseconds(300));
  k_touch<<<1024, 256, 0, st>>>(d, big);
  CK(hipStreamSynchronize(st));
  d2h("300 ms idle, then kernel, then copy", h, d, small, st);
  return 0;
}
