#!/bin/bash
# One GPU session: native engine strategies vs the oracle, then the GPU pytest tier.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
bash tools/gpu_engine_check.sh > gpurun_out/engine_check.txt 2>&1; rc=$?
cat gpurun_out/engine_check.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
exit $rc
