#!/bin/bash
# Kernel + memory-copy trace of a short bench run (timeline of the last steps).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/tl
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
DMLP_PIPE_DEBUG=${DMLP_PIPE_DEBUG:-0} timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/prof -o run --output-format csv \
    -- python3 bench.py --steps 4 --warmup 2 --no-busbw > $OUT/bench.log 2>&1; rc=$?
tail -1 $OUT/bench.log; [ $rc -eq 0 ] || exit $rc
python3 tools/timeline.py $OUT/prof 7 > $OUT/timeline.txt; tail -40 $OUT/timeline.txt
