#!/bin/bash
# Quick GPU iteration: GPU tests, screen ablation/counters, default bench.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/quick_gpu_bench.py --q 131072 --modes 0,1,8 > gpurun_out/ablate.log 2>&1; rc=$?
cat gpurun_out/ablate.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err; rc=$?
cat gpurun_out/bench_default.json; [ $rc -eq 0 ] || { tail gpurun_out/bench_default.err; exit $rc; }
if [ -n "${ITER_EXTRA:-}" ]; then eval "$ITER_EXTRA"; fi
