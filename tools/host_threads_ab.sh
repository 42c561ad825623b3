#!/bin/bash
# Host worker-pool A/B on the GPU box (cgroup CPU quota vs pool size / spin budget): interleaved
# bench runs, one line per run.  gpurun -- bash tools/host_threads_ab.sh
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/hv
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python3 -c "import os; print(len(os.sched_getaffinity(0)))"; } > gpurun_out/hv/env.txt 2>&1
timeout -k 10 120 python bench.py --steps 300 --warmup 20 > /dev/null 2>&1 || exit 1
i=0
for cfg in "16 40000" "8 40000" "16 2000" "8 2000" "4 2000" "16 40000" "8 40000" "16 2000" "8 2000" "4 2000"; do
  set -- $cfg
  i=$((i + 1))
  DMLP_HOST_THREADS=$1 DMLP_POOL_SPIN=$2 timeout -k 10 120 python bench.py --steps 300 --warmup 20 \
      > gpurun_out/hv/r$i.log 2>&1 || exit 1
  echo "threads $1 spin $2: $(tail -1 gpurun_out/hv/r$i.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
cat gpurun_out/hv/env.txt
