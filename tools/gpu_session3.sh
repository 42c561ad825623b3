#!/bin/bash
# GPU: kernel tests, default bench, verified bench, harness run, rocprof of the bench step.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out profiles
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err; rc=$?
cat gpurun_out/bench_default.json; [ $rc -eq 0 ] || { tail gpurun_out/bench_default.err; exit $rc; }
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --verify > gpurun_out/bench_verify.json 2>&1; rc=$?
tail -1 gpurun_out/bench_verify.json; [ $rc -eq 0 ] || exit $rc
KNN_TRACE=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 > gpurun_out/bench_trace.log 2>&1; rc=$?
grep "dmlp-trace" gpurun_out/bench_trace.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 > gpurun_out/prof_bench.log 2>&1; rc=$?
echo "rocprof rc=$rc"
exit $rc
