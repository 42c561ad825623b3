// Cross-memory-attach probe: how fast can one process read another process's heap rows (the
// engine.h drop-in's query rows live in rank 0's heap as one std::vector per query)?  Reads a
// table of 131072 row pointers and the rows with process_vm_readv (a) one iovec per row, (b) one
// read of the rows' heap span, (c) the span in 4 threads; plus a plain in-process gather for scale.
//
//   g++ -O2 -pthread tests/native/cma_probe.cpp -o tools/bin/cma_probe
#include <sys/uio.h>
#include <sys/prctl.h>
#include <unistd.h>
#include <sys/wait.h>
#include <cstdio>
#include <cstring>
#include <vector>
#include <chrono>
#include <thread>
int main(int argc, char** argv) {
  const int Q = 131072, A = 32;
  std::vector<std::vector<double>> rows(Q);
  for (int i = 0; i < Q; ++i) { rows[i].resize(A); for (int a = 0; a < A; ++a) rows[i][a] = i + a; }
  std::vector<const double*> tab(Q);
  for (int i = 0; i < Q; ++i) tab[i] = rows[i].data();
  uintptr_t lo = (uintptr_t)tab[0], hi = lo;
  for (auto p : tab) { lo = std::min(lo, (uintptr_t)p); hi = std::max(hi, (uintptr_t)p + A * 8); }
  printf("span %.1f MB for %.1f MB of rows\n", (hi - lo) / 1e6, Q * A * 8 / 1e6);
  prctl(PR_SET_PTRACER, PR_SET_PTRACER_ANY, 0, 0, 0);
  pid_t parent = getpid();
    pid_t c = fork();
  if (c == 0) {
    // child: read the table then the rows (a) per-row iovecs (b) one span (c) span in T threads
    std::vector<const double*> t(Q);
    iovec l{t.data(), Q * 8}, r{(void*)tab.data(), Q * 8};
    ssize_t n = process_vm_readv(parent, &l, 1, &r, 1, 0);
    printf("table read %zd\n", n);
    std::vector<double> out((size_t)Q * A);
    std::vector<char> span(hi - lo);
    for (int rep = 0; rep < 3; ++rep) {
      auto t0 = std::chrono::steady_clock::now();
      for (int b = 0; b < Q; b += 1024) {
        iovec li{out.data() + (size_t)b * A, (size_t)1024 * A * 8};
        std::vector<iovec> ri(1024);
        for (int i = 0; i < 1024; ++i) ri[i] = {(void*)t[b + i], (size_t)A * 8};
        process_vm_readv(parent, &li, 1, ri.data(), 1024, 0);
      }
      auto t1 = std::chrono::steady_clock::now();
      iovec ls{span.data(), span.size()}, rs{(void*)lo, span.size()};
      ssize_t m = process_vm_readv(parent, &ls, 1, &rs, 1, 0);
      auto t2 = std::chrono::steady_clock::now();
      const int T = 4;
      std::vector<std::thread> th;
      for (int k = 0; k < T; ++k) th.emplace_back([&, k] {
        size_t a = span.size() * k / T, b = span.size() * (k + 1) / T;
        iovec l2{span.data() + a, b - a}, r2{(void*)(lo + a), b - a};
        process_vm_readv(parent, &l2, 1, &r2, 1, 0);
      });
      for (auto& x : th) x.join();
      auto t3 = std::chrono::steady_clock::now();
      printf("per-row iov %.2f ms | span %.2f ms (%zd B) | span x%d threads %.2f ms | check %d\n",
             std::chrono::duration<double, std::milli>(t1 - t0).count(),
             std::chrono::duration<double, std::milli>(t2 - t1).count(), m, T,
             std::chrono::duration<double, std::milli>(t3 - t2).count(), out[(size_t)77 * A + 3] == 80.0);
    }
    fflush(stdout); _exit(0);
  }
  int st; waitpid(c, &st, 0);
  std::vector<double> g((size_t)Q * A);
  for (int rep = 0; rep < 3; ++rep) {
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < Q; ++i) std::memcpy(g.data() + (size_t)i * A, tab[i], A * 8);
    auto t1 = std::chrono::steady_clock::now();
    printf("in-process gather (1 thread) %.2f ms\n", std::chrono::duration<double, std::milli>(t1 - t0).count());
  }
  return 0;
}
