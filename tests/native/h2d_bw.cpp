// Host -> device copy bandwidth from page-locked memory over 1 / 2 / 4 streams at once: does the
// runtime spread concurrent copies over several SDMA engines (the large-N step's dataset rows are
// one copy stream, pipeline.hip dr_part), and does the copy kind matter (hipMemcpyHostToDevice vs
// the forced-SDMA hipMemcpyDeviceToDeviceNoCU)?  Prints one JSON line per case.
//
//   hipcc --offload-arch=gfx950 -O2 tests/native/h2d_bw.cpp -o tools/bin/h2d_bw
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

int main() {
  CK(hipSetDevice(0));
  const size_t total = size_t(256) << 20;
  char *h = nullptr, *d = nullptr;
  CK(hipHostMalloc((void**)&h, total, hipHostMallocDefault));
  std::memset(h, 1, total);
  CK(hipMalloc((void**)&d, total));
  hipStream_t st[4];
  for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const hipMemcpyKind kinds[2] = {hipMemcpyHostToDevice, hipMemcpyDeviceToDeviceNoCU};
  const char* kname[2] = {"H2D", "NoCU"};
  for (int rep = 0; rep < 2; ++rep) {  // (the first round warms every path up)
    for (int ki = 0; ki < 2; ++ki) {
      for (int ns : {1, 2, 4}) {
        for (size_t piece : {size_t(4) << 20, size_t(16) << 20}) {
          CK(hipDeviceSynchronize());
          const auto t0 = std::chrono::steady_clock::now();
          size_t i = 0;
          for (size_t o = 0; o < total; o += piece, ++i)
            CK(hipMemcpyAsync(d + o, h + o, piece, kinds[ki], st[i % ns]));
          CK(hipDeviceSynchronize());
          const double ms =
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
          if (rep)
            std::printf("{\"kind\": \"%s\", \"streams\": %d, \"piece_MiB\": %zu, \"ms\": %.3f, "
                        "\"GBps\": %.2f}\n", kname[ki], ns, piece >> 20, ms, total / ms / 1e6);
        }
      }
    }
  }
  return 0;
}
