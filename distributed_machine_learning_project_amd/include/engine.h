// Drop-in engine.h for the reference's fixed harness (common.cpp:81-135).
//
// Build the reference's own common.cpp against this header and the MI355X engine:
//     python -m distributed_machine_learning_project_amd.build --dropin /path/to/common.cpp
// produces an `engine` binary that behaves like the reference's (same stdin format, same
// reportResult output, same "Time taken" line), with Engine::KNN running on MI355X GPUs
// (RCCL over xGMI between ranks) or, with KNN_DEVICE=cpu, the serial KD-tree.
// API parity: engine.h:6-12 — default-constructible Engine, KNN called on every rank with
// rank 0 holding the parsed dataset/queries, a public (unused) `dataPoint` member.
// Engine knobs are environment variables (the harness is fixed): KNN_STRATEGY
// (farm|shard_gather|shard_reduce|grid2d|serial), KNN_DEVICE (auto|gpu|cpu), KNN_EXACT=1,
// KNN_TRACE=1, KNN_TIMEOUT_S.
#pragma once

// the harness's data-model header expects <vector> to be included before it
#include <vector>
#ifdef DMLP_COMMON_HEADER
#include DMLP_COMMON_HEADER
#else
#include "common.h"
#endif

class Engine {
 public:
  Engine();   // untimed in the harness: device binding, RCCL communicator, kernel warm-up
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  // Exact k-NN classification of `queries` against `dataset` (valid on rank 0 only; the
  // other ranks pass empty vectors).  Rank 0 calls reportResult once per query, in id order.
  void KNN(Params& p, std::vector<DataPoint>& dataset, std::vector<Query>& queries);

  std::vector<DataPoint> dataPoint;  // source compatibility only; never used

 private:
  struct Impl;
  Impl* impl_;
};
