#!/bin/bash
# A/B of streaming-screen variants (whole local pipeline, 131072 queries, N=1e5, A=32, k=16).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in "auto" "sub16" "nogroups"; do
  case $v in
    auto) E="" ;;
    sub16) E="DMLP_STREAM_SUB=16" ;;
    nogroups) E="DMLP_STREAM_GROUPS=0" ;;
  esac
  env $E timeout -k 10 300 python tools/quick_gpu_bench.py --q 131072 --modes 0,16,8 > gpurun_out/ab_$v.log 2>&1; rc=$?
  echo "== $v"; grep -v amdgpu.ids gpurun_out/ab_$v.log; [ $rc -eq 0 ] || exit $rc
done
