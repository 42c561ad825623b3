#!/bin/bash
# First GPU session: kernel numerics tests, phase timing, rocprof kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/quick_gpu_bench.py --n 100000 --q 100000 > gpurun_out/qb_screen.log 2>&1; rc=$?
cat gpurun_out/qb_screen.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/quick_gpu_bench.py --n 100000 --q 20000 --exact --iters 2 > gpurun_out/qb_exact.log 2>&1; rc=$?
cat gpurun_out/qb_exact.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python3 tools/quick_gpu_bench.py --n 100000 --q 100000 --iters 2 --check 0 > gpurun_out/prof1.log 2>&1; rc=$?
echo "rocprof rc=$rc"
find gpurun_out/prof1 -name "*stats*" | head
exit $rc
