// dropin_engine.cpp — Engine (include/engine.h) for the reference's own harness: packs the
// harness's AoS vectors (K1, timed like the reference's engines do), runs KnnCore::KNN, and
// hands every query's sorted (distance, id) list and label to the harness's reportResult
// (common.cpp:57-79), which formats the checksum / DEBUG lines itself.
#include <memory>
#include <thread>

#include "engine.h"
#include "engine_core.h"

struct Engine::Impl {
  dmlp_rt::Runtime rt;
  std::unique_ptr<dmlp_rt::KnnCore> core;
};

Engine::Engine() : impl_(new Impl) {
  const char* dev = getenv("KNN_DEVICE");
  const bool cpu = dev && std::string(dev) == "cpu";
  int ndev = 0;
  if (!cpu && hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
  const char* st = getenv("KNN_STRATEGY");
  std::string strategy = st ? st : (ndev > 0 && !cpu ? "farm" : "serial");
  if (cpu || ndev == 0) strategy = "serial";
  const char* ex = getenv("KNN_EXACT");
  impl_->rt.init(strategy != "serial");
  dmlp_rt::HostBuf<double>::use_pinned() = impl_->rt.gpu;
  // lists mode: the core returns every query's sorted list + label on rank 0
  impl_->core.reset(new dmlp_rt::KnnCore(impl_->rt, strategy, /*debug=*/true,
                                          ex && std::string(ex) == "1"));
}

Engine::~Engine() {
  impl_->core.reset();
  impl_->rt.finalize();
  delete impl_;
}

void Engine::KNN(Params& p, std::vector<DataPoint>& dataset, std::vector<Query>& queries) {
  const bool root = impl_->rt.rank == 0;
  dmlp_rt::Input in;
  dmlp_rt::Output out;
  if (root) {
    in.N = (int64_t)dataset.size();
    in.Q = (int64_t)queries.size();
    in.A = p.num_attrs;
    in.labels.resize(in.N);
    in.k.resize(in.Q);
    in.X.resize((size_t)in.N * in.A);
    in.Qx.resize((size_t)in.Q * in.A);
    // AoS -> row-major (K1); parallel over rows
    const int nt = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
      th.emplace_back([&, t] {
        for (int64_t i = t; i < in.N; i += nt) {
          in.labels[i] = dataset[i].label;
          std::memcpy(in.X.data() + i * in.A, dataset[i].attrs.data(), sizeof(double) * in.A);
        }
        for (int64_t i = t; i < in.Q; i += nt) {
          in.k[i] = queries[i].k;
          std::memcpy(in.Qx.data() + i * in.A, queries[i].attrs.data(), sizeof(double) * in.A);
        }
      });
    for (auto& x : th) x.join();
  }
  impl_->core->KNN(root ? &in : nullptr, root ? &out : nullptr);
  if (!root) return;
  const int ks = out.kstride;
  std::vector<std::pair<double, int>> res;
  for (int64_t q = 0; q < in.Q; ++q) {
    const int k = std::max(0, in.k[q]);
    res.resize(k);
    for (int j = 0; j < k; ++j)
      res[j] = {out.dist[(size_t)q * ks + j], out.ids[(size_t)q * ks + j]};
    reportResult(queries[q], res, out.label[q]);
  }
}
