// Copy-engine probe: which hipMemcpyAsync / hipMemsetAsync / hipStreamWriteValue32 calls does
// this runtime run as a blit or fill KERNEL (a wave slot on the CUs) and which as an SDMA copy?
// Run under `rocprofv3 --kernel-trace --memory-copy-trace`: every operation is issued alone
// between two markers (a 1-wave marker kernel whose argument is the operation's index), so the
// kernel trace shows the blit kernels between markers and the memory-copy trace the SDMA copies.
//
//   hipcc --offload-arch=gfx950 -O2 tests/native/copy_kind_probe.cpp -o /tmp/copy_kind_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

__global__ void k_marker(int op, int* sink) {
  if (threadIdx.x == 0 && op < 0) *sink = op;  // never taken: the argument tags the dispatch
}

int main() {
  hipStream_t st;
  CK(hipSetDevice(0));
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const size_t big = size_t(8) << 20;
  char *dev, *dev2, *hm;
  int* sink;
  CK(hipMalloc((void**)&dev, big));
  CK(hipMalloc((void**)&dev2, big));
  CK(hipMalloc((void**)&sink, 64));
  CK(hipHostMalloc((void**)&hm, big, hipHostMallocDefault));
  std::memset(hm, 1, big);
  char* reg = (char*)std::aligned_alloc(4096, big);
  std::memset(reg, 1, big);
  CK(hipHostRegister(reg, big, hipHostRegisterDefault));
  const size_t sizes[] = {4, 8, 64, 256, 4096, 16384, 65536, 262144, 1 << 20, 6 << 20};
  int op = 0;
  auto mark = [&]() {
    hipLaunchKernelGGL(k_marker, dim3(1), dim3(64), 0, st, op, sink);
    CK(hipStreamSynchronize(st));
  };
  std::printf("op kind bytes\n");
  for (int pass = 0; pass < 2; ++pass) {  // (the first pass warms every path up)
    for (size_t n : sizes) {
      struct { const char* name; void* dst; const void* src; hipMemcpyKind k; } cs[] = {
          {"H2D_hostmalloc", dev, hm, hipMemcpyHostToDevice},
          {"D2H_hostmalloc", hm, dev, hipMemcpyDeviceToHost},
          {"H2D_registered", dev, reg, hipMemcpyHostToDevice},
          {"D2H_registered", reg, dev, hipMemcpyDeviceToHost},
          {"D2D", dev2, dev, hipMemcpyDeviceToDevice},
          // (the runtime's "no compute units" kind, and the pointer-inferred one, on page-locked
          // host memory)
          {"H2D_hostmalloc_NoCU", dev, hm, hipMemcpyDeviceToDeviceNoCU},
          {"D2H_hostmalloc_NoCU", hm, dev, hipMemcpyDeviceToDeviceNoCU},
          {"H2D_hostmalloc_Default", dev, hm, hipMemcpyDefault}};
      for (auto& c : cs) {
        mark();
        if (pass) std::printf("%d %s %zu\n", op, c.name, n);
        CK(hipMemcpyAsync(c.dst, c.src, n, c.k, st));
        ++op;
      }
      mark();
      if (pass) std::printf("%d memset %zu\n", op, n);
      CK(hipMemsetAsync(dev, 0, n, st));
      ++op;
    }
    mark();
    if (pass) std::printf("%d writevalue32 4\n", op);
    CK(hipStreamWriteValue32(st, dev, 1u, 0));
    ++op;
  }
  mark();
  CK(hipStreamSynchronize(st));
  return 0;
}
