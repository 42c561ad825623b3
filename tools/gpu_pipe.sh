#!/bin/bash
# Pipelined ingress session: kernel tests, bench with/without the chunked H2D, traced step.
set -u
TAG=${1:-pipe}
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > gpurun_out/$TAG/pytest_kernels.log 2>&1; rc=$?
tail -3 gpurun_out/$TAG/pytest_kernels.log; [ $rc -eq 0 ] || exit $rc
for pl in 0 1; do
  KNN_PIPELINE=$pl timeout -k 10 300 python bench.py --verify > gpurun_out/$TAG/bench_p$pl.json 2> gpurun_out/$TAG/bench_p$pl.err; rc=$?
  echo "pipeline=$pl"; cat gpurun_out/$TAG/bench_p$pl.json | cut -c1-200; [ $rc -eq 0 ] || { tail gpurun_out/$TAG/bench_p$pl.err; exit $rc; }
done
KNN_TRACE=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/$TAG/bench_trace.json 2> gpurun_out/$TAG/bench_trace.err; rc=$?
grep "dmlp-trace" gpurun_out/$TAG/bench_trace.err | tail -8; [ $rc -eq 0 ] || exit $rc
cd /tmp && cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/$TAG/prof -o run --output-format csv \
    -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/$TAG/prof.log 2>&1; rc=$?
[ $rc -eq 0 ] || { tail -5 gpurun_out/$TAG/prof.log; exit $rc; }
ls gpurun_out/$TAG/prof
