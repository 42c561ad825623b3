#!/bin/bash
set -u
TAG=${1:-pipe3}
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread -k "pipelined or bench_distribution" > gpurun_out/$TAG/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/$TAG/pytest.log; [ $rc -eq 0 ] || exit $rc
for pl in 0 1; do
  KNN_PIPELINE=$pl DMLP_PIPE_DEBUG=1 timeout -k 10 300 python bench.py --steps 10 > gpurun_out/$TAG/bench_p$pl.json 2> gpurun_out/$TAG/bench_p$pl.err; rc=$?
  echo "pipeline=$pl $(cut -c1-170 gpurun_out/$TAG/bench_p$pl.json)"; grep dmlp-pipe gpurun_out/$TAG/bench_p$pl.err | tail -3; [ $rc -eq 0 ] || { tail gpurun_out/$TAG/bench_p$pl.err; exit $rc; }
done
