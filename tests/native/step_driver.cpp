// Native step driver: dmlp_step (pipeline.hip) in a loop on synthetic data of generate_input.py's
// distribution, without Python or torch in the process — a clean target for rocprofv3 kernel /
// memory-copy traces (a torch process under --memory-copy-trace crashes in its exit handlers on
// this image) and a fast large-N A/B (no numpy generation of 1e7 x 32 rows per run).
//
//   step_driver [--n N] [--a A] [--q Q] [--kmin k] [--kmax k] [--steps S] [--warmup W]
//               [--rows table|flat] [--timeline]
// prints one JSON line: ms/step (mean and p50 of the timed steps), host issue ms, the step
// timeline (hipEvents) of the last step, path / early-start counters, report bytes.
//
//   hipcc --offload-arch=gfx950 -O2 tests/native/step_driver.cpp -I<pkg>/csrc -L<pkg> -ldmlp \
//       -Wl,-rpath,<pkg> -o tools/bin/step_driver       (tools/build_probes.sh)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "dmlp.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

int main(int argc, char** argv) {
  int64_t N = 100000, Q = 131072;
  int A = 32, kmin = 16, kmax = 16, steps = 50, warmup = 20;
  bool table = false, timeline = false;
  for (int i = 1; i < argc; ++i) {
    std::string s = argv[i];
    auto nxt = [&]() { return i + 1 < argc ? argv[++i] : (char*)"0"; };
    if (s == "--n") N = std::atoll(nxt());
    else if (s == "--a") A = std::atoi(nxt());
    else if (s == "--q") Q = std::atoll(nxt());
    else if (s == "--kmin") kmin = std::atoi(nxt());
    else if (s == "--kmax") kmax = std::atoi(nxt());
    else if (s == "--k") kmin = kmax = std::atoi(nxt());
    else if (s == "--steps") steps = std::atoi(nxt());
    else if (s == "--warmup") warmup = std::atoi(nxt());
    else if (s == "--rows") table = std::string(nxt()) == "table";
    else if (s == "--timeline") timeline = true;
    else { std::fprintf(stderr, "unknown arg %s\n", argv[i]); return 2; }
  }
  // generate_input.py's distribution: uniform [0, 1000) attributes with 6 decimals, 10 labels,
  // k uniform in [kmin, min(kmax, N)]
  std::mt19937_64 g(42);
  std::uniform_int_distribution<int64_t> um(0, 1000000000 - 1);
  auto attr = [&]() { return (double)um(g) / 1e6; };
  double *X = nullptr, *Qx = nullptr;
  int *lab = nullptr, *k = nullptr;
  CK(hipHostMalloc((void**)&X, sizeof(double) * N * A, hipHostMallocDefault));
  CK(hipHostMalloc((void**)&Qx, sizeof(double) * Q * A, hipHostMallocDefault));
  CK(hipHostMalloc((void**)&lab, sizeof(int) * N, hipHostMallocDefault));
  CK(hipHostMalloc((void**)&k, sizeof(int) * Q, hipHostMallocDefault));
  for (int64_t i = 0; i < N * A; ++i) X[i] = attr();
  for (int64_t i = 0; i < N; ++i) lab[i] = (int)(g() % 10);
  std::uniform_int_distribution<int> uk(kmin, (int)std::min<int64_t>(kmax, N));
  for (int64_t i = 0; i < Q; ++i) k[i] = uk(g);
  for (int64_t i = 0; i < Q * A; ++i) Qx[i] = attr();
  std::vector<const double*> xr(N), qr(Q);
  for (int64_t i = 0; i < N; ++i) xr[i] = X + i * A;
  for (int64_t i = 0; i < Q; ++i) qr[i] = Qx + i * A;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const int64_t bound = dmlp_format_bound((int)Q);
  char* rep = nullptr;
  CK(hipHostMalloc((void**)&rep, bound, hipHostMallocDefault));
  if (timeline) dmlp_step_events(1);
  std::vector<double> ms;
  double host_ms = 0.0;
  dmlp_step_args a;
  for (int it = 0; it < warmup + steps; ++it) {
    std::memset(&a, 0, sizeof a);
    a.X = table ? nullptr : X;
    a.Xr = table ? xr.data() : nullptr;
    a.N = N;
    a.A = A;
    a.labels = lab;
    a.Qx = table ? nullptr : Qx;
    a.Qr = table ? qr.data() : nullptr;
    a.k = k;
    a.Q = Q;
    a.kmin = 1;
    a.kmax = 0;  // scanned
    a.report_mode = 1;
    a.report_dst = rep;
    a.report_cap = bound;
    a.stream = st;
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = dmlp_step(&a);
    const auto t1 = std::chrono::steady_clock::now();
    if (rc != 0) {
      std::fprintf(stderr, "dmlp_step rc=%d\n", rc);
      return 1;
    }
    if (it >= warmup) {
      ms.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
      host_ms += a.host_ms;
    }
  }
  double sum = 0.0;
  for (double v : ms) sum += v;
  std::vector<double> srt = ms;
  std::sort(srt.begin(), srt.end());
  int64_t st_[8] = {0};
  dmlp_pipeline_stats(st_);
  std::printf("{\"N\": %lld, \"A\": %d, \"Q\": %lld, \"k\": \"%d-%d\", \"rows\": \"%s\", "
              "\"steps\": %d, \"ms_per_step\": %.4f, \"p50_ms\": %.4f, \"host_issue_ms\": %.4f, "
              "\"path\": %d, \"early\": %d, \"device_render\": %lld, \"escalated\": %d, "
              "\"report_bytes\": %lld",
              (long long)N, A, (long long)Q, kmin, kmax, table ? "table" : "flat", steps,
              sum / std::max<size_t>(1, ms.size()), srt.empty() ? 0.0 : srt[srt.size() / 2],
              host_ms / std::max(1, steps), a.path, a.early, (long long)st_[6], a.n_escalated,
              (long long)a.report_len);
  if (timeline) {
    double t[16];
    const char* nm[16];
    const int n = dmlp_step_timeline(t, nm, 16);
    std::printf(", \"timeline_ms\": {");
    for (int i = 0; i < n; ++i) std::printf("%s\"%s\": %.4f", i ? ", " : "", nm[i], t[i]);
    std::printf("}");
  }
  std::printf("}\n");
  return 0;
}
