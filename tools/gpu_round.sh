#!/bin/bash
# One GPU session: GPU test tier, default bench, rocprofv3 kernel stats of the bench.
#   gpurun --timeout 900 -- bash tools/gpu_round.sh [tag]
set -u
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/$TAG/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/$TAG/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err; rc=$?
cat gpurun_out/$TAG/bench.json; [ $rc -eq 0 ] || { tail gpurun_out/$TAG/bench.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run --output-format csv \
    -- python3 bench.py --steps 5 --warmup 1 > gpurun_out/$TAG/prof.log 2>&1; rc=$?
[ $rc -eq 0 ] || { tail gpurun_out/$TAG/prof.log; exit $rc; }
find gpurun_out/$TAG/prof -name '*kernel_stats.csv' -exec sh -c 'head -12 "$1" | cut -c1-160' _ {} \;
