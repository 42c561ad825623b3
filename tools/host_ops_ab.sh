#!/bin/bash
# Host-ops phase clocks (DMLP_PIPE_DEBUG / DMLP_HOST_OPS_DEBUG) and bench ms/step for several
# slice counts of the host render + H2D pipeline, interleaved on one box.
#   gpurun -- bash tools/host_ops_ab.sh
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/hops
timeout -k 10 120 python bench.py --steps 300 --warmup 20 > /dev/null 2>&1 || exit 1
for round in 1 2; do
  for c in 1 2 4 8; do
    DMLP_HOST_OPS_CHUNKS=$c timeout -k 10 120 python bench.py --steps 400 --warmup 20 --no-busbw \
        > gpurun_out/hops/c$c.$round.log 2>&1 || exit 1
    echo "chunks $c round $round: $(tail -1 gpurun_out/hops/c$c.$round.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
for c in 1 4; do
  DMLP_HOST_OPS_CHUNKS=$c DMLP_PIPE_DEBUG=1 DMLP_HOST_OPS_DEBUG=1 timeout -k 10 120 python bench.py \
      --steps 6 --warmup 2 --no-busbw > gpurun_out/hops/dbg$c.log 2>&1 || exit 1
  echo "== chunks $c"; grep -E "dmlp-pipe|dmlp-hostops" gpurun_out/hops/dbg$c.log | tail -6
done
