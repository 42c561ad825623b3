// Test-side data model with the reference harness's layout (common.h:4-25),
// so tests/native/mini_harness.cpp can drive include/engine.h without the reference sources.
#pragma once
#include <utility>
#include <vector>

struct Params {
  int num_data;
  int num_queries;
  int num_attrs;
};

struct DataPoint {
  int id;
  int label;
  std::vector<double> attrs;
};

struct Query {
  int id;
  int k;
  std::vector<double> attrs;
};

struct Update {
  int id;
  std::vector<double> new_attrs;
};

void reportResult(Query& q, std::vector<std::pair<double, int>>& result, int label);
