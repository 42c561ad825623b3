#!/bin/bash
# PC sampling of the screen kernel (instruction-level hotspots / stall reasons).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/pcs
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 120 rocprofv3 -L > gpurun_out/pcs/list_avail.txt 2>&1
grep -i -A12 "pc sampling\|PC_SAMPLING\|pc-sampling" gpurun_out/pcs/list_avail.txt | head -40
export DMLP_STREAM_GROUPS=${DMLP_STREAM_GROUPS:-0}
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 1048576 -d gpurun_out/pcs/st -o run --output-format csv -- python3 tools/quick_gpu_bench.py --q 131072 --modes 0 --iters 1 > gpurun_out/pcs/st.log 2>&1; rc=$?
echo "stochastic rc=$rc"; tail -3 gpurun_out/pcs/st.log; ls -la gpurun_out/pcs/st 2>/dev/null
if [ $rc -ne 0 ]; then
  timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 -d gpurun_out/pcs/ht -o run --output-format csv -- python3 tools/quick_gpu_bench.py --q 131072 --modes 0 --iters 1 > gpurun_out/pcs/ht.log 2>&1; rc=$?
  echo "host_trap rc=$rc"; tail -3 gpurun_out/pcs/ht.log; ls -la gpurun_out/pcs/ht 2>/dev/null
fi
exit $rc
