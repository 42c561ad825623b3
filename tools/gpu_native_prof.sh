#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/nprof
mkdir -p $OUT
python3 tools/generate_input.py --fast --num_data 100000 --num_queries 131072 --num_attrs 32 \
    --min 0 --max 1000 --minK 16 --maxK 16 --num_labels 10 --output /tmp/bench4.in > /dev/null || exit 1
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --runtime-trace -d $OUT/p -o run --output-format csv \
    -- distributed_machine_learning_project_amd/knn_engine --strategy farm --input /tmp/bench4.in > $OUT/out.txt 2> $OUT/err.txt; rc=$?
grep "Time taken" $OUT/err.txt; ls $OUT/p; exit $rc
