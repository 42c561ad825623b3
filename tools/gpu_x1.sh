#!/bin/bash
# Single-term screen session: kernel numerics, A/B vs the 3-term screen, ablation counters, bench.
set -u
TAG=${1:-x1}
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > gpurun_out/$TAG/pytest_kernels.log 2>&1; rc=$?
tail -15 gpurun_out/$TAG/pytest_kernels.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/quick_gpu_bench.py --q 131072 --modes 0,1,8 > gpurun_out/$TAG/ab_x1.log 2>&1; rc=$?
cat gpurun_out/$TAG/ab_x1.log; [ $rc -eq 0 ] || exit $rc
DMLP_SCREEN=stream timeout -k 10 200 python tools/quick_gpu_bench.py --q 131072 --modes 0 > gpurun_out/$TAG/ab_stream.log 2>&1; rc=$?
cat gpurun_out/$TAG/ab_stream.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/quick_gpu_bench.py --q 131072 --iters 5 > gpurun_out/$TAG/quick.log 2>&1; rc=$?
cat gpurun_out/$TAG/quick.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --verify > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err; rc=$?
cat gpurun_out/$TAG/bench.json; [ $rc -eq 0 ] || { tail gpurun_out/$TAG/bench.err; exit $rc; }
