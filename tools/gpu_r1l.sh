#!/bin/bash
# One GPU session: native knn_engine strategies vs the oracle, verified bench, exact-path bench.
#   gpurun --timeout 600 -- bash tools/gpu_r1l.sh
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r1l
export TMPDIR=/tmp
timeout -k 10 300 bash tools/gpu_engine_check.sh > gpurun_out/r1l/engine_check.txt 2>&1; rc=$?
cat gpurun_out/r1l/engine_check.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --verify > gpurun_out/r1l/bench_verify.json 2> gpurun_out/r1l/bench_verify.err; rc=$?
cat gpurun_out/r1l/bench_verify.json; [ $rc -eq 0 ] || { tail gpurun_out/r1l/bench_verify.err; exit $rc; }
timeout -k 10 300 python bench.py --exact --steps 5 --warmup 1 > gpurun_out/r1l/bench_exact.json 2> gpurun_out/r1l/bench_exact.err; rc=$?
cat gpurun_out/r1l/bench_exact.json; [ $rc -eq 0 ] || { tail gpurun_out/r1l/bench_exact.err; exit $rc; }
