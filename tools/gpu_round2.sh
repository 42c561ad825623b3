#!/bin/bash
# GPU session: GPU test tier, verified bench, default bench, step timeline.
#   gpurun --timeout 900 -- bash tools/gpu_round2.sh [tag]
set -u
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/$TAG/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/$TAG/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --verify > gpurun_out/$TAG/verify.json 2> gpurun_out/$TAG/verify.err; rc=$?
cat gpurun_out/$TAG/verify.json; [ $rc -eq 0 ] || { tail gpurun_out/$TAG/verify.err; exit $rc; }
timeout -k 10 300 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err; rc=$?
cat gpurun_out/$TAG/bench.json; [ $rc -eq 0 ] || { tail gpurun_out/$TAG/bench.err; exit $rc; }
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/$TAG/prof -o run --output-format csv \
    -- python3 bench.py --steps 4 --warmup 2 --no-busbw > gpurun_out/$TAG/prof.log 2>&1; rc=$?
[ $rc -eq 0 ] || { tail gpurun_out/$TAG/prof.log; exit $rc; }
python3 tools/timeline.py gpurun_out/$TAG/prof 7 > gpurun_out/$TAG/timeline.txt
find gpurun_out/$TAG/prof -name '*kernel_stats.csv' -exec sh -c 'head -6 "$1" | cut -c1-160' _ {} \;
