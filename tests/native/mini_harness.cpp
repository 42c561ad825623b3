// Minimal re-implementation of the reference harness contract: rank 0 parses
// stdin, all ranks barrier, `Engine eng;` (untimed), rank 0 times eng.KNN + the closing barrier,
// reportResult prints "Query <id> checksum: <fnv>" (or the DEBUG listing with -DDEBUG), the time
// goes to stderr.  Used by tests/test_engine_native.py to exercise include/engine.h exactly the
// way the reference's common.cpp does.
#include <mpi.h>

#include <chrono>
#include <cstdio>
#include <iostream>
#include <sstream>
#include <stdexcept>
#include <string>

#include "engine.h"

static Params g_params;

void reportResult(Query& q, std::vector<std::pair<double, int>>& result, int label) {
#ifndef DEBUG
  unsigned long long h = 1469598103934665603ULL;
  h = (h ^ (unsigned long long)label) * 1099511628211ULL;
  for (const auto& pr : result) h = (h ^ (unsigned long long)(pr.second + 1)) * 1099511628211ULL;
  std::cout << "Query " << q.id << " checksum: " << h << "\n";
#else
  std::cout << "Label for Query " << q.id << " : " << label << "\n";
  std::cout << "Top-" << q.k << " neighbors:\n";
  for (const auto& pr : result) std::cout << pr.second << " : " << pr.first << "\n";
#endif
}

int main(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  std::ios::sync_with_stdio(false);
  int rank = 0;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  std::vector<DataPoint> data;
  std::vector<Query> qs;
  if (rank == 0) {
    std::string line;
    std::getline(std::cin, line);
    std::istringstream(line) >> g_params.num_data >> g_params.num_queries >> g_params.num_attrs;
    data.resize(g_params.num_data);
    for (int i = 0; i < g_params.num_data; ++i) {
      std::getline(std::cin, line);
      std::istringstream ss(line);
      data[i].id = i;
      ss >> data[i].label;
      data[i].attrs.resize(g_params.num_attrs);
      for (auto& v : data[i].attrs) ss >> v;
    }
    qs.resize(g_params.num_queries);
    for (int i = 0; i < g_params.num_queries; ++i) {
      std::getline(std::cin, line);
      if (line.empty() || line[0] != 'Q') throw std::runtime_error("bad query line");
      std::istringstream ss(line.substr(1));
      qs[i].id = i;
      ss >> qs[i].k;
      qs[i].attrs.resize(g_params.num_attrs);
      for (auto& v : qs[i].attrs) ss >> v;
    }
  }
  MPI_Barrier(MPI_COMM_WORLD);
  Engine eng;
  const auto t0 = std::chrono::steady_clock::now();
  eng.KNN(g_params, data, qs);
  MPI_Barrier(MPI_COMM_WORLD);
  if (rank == 0) {
    const auto ms =
        std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0)
            .count();
    std::cerr << "Time taken: " << ms << " ms\n";
  }
  MPI_Finalize();
  return 0;
}
