#!/bin/bash
# PC sampling of the x1 screen kernel (instruction hotspots + stall reasons).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/pcs1
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 200 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 65536 -d gpurun_out/pcs1/st -o run --output-format csv -- python3 tools/quick_gpu_bench.py --q 131072 --iters 1 --check 0 > gpurun_out/pcs1/st.log 2>&1; rc=$?
echo "stochastic rc=$rc"; tail -3 gpurun_out/pcs1/st.log; find gpurun_out/pcs1/st -type f | head; exit $rc
