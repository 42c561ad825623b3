#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/d8
for c in 2 8; do
  DMLP_X1_CHECK=$c timeout -k 10 100 python tools/quick_gpu_bench.py --q 131072 --iters 5 > gpurun_out/d8/c$c.log 2>&1; rc=$?
  echo "check $c: $(grep -v amdgpu gpurun_out/d8/c$c.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
