#!/bin/bash
# Host-ops slice count A/B (DMLP_HOST_OPS_CHUNKS: host render + H2D of the screen operands in
# that many pipelined slices), interleaved bench runs on one box, plus phase clocks.
#   gpurun -- bash tools/host_ops_ab.sh [counts...] (default: 1 2)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/hops
counts=("$@")
[ ${#counts[@]} -eq 0 ] && counts=(1 2)
timeout -k 10 120 python bench.py --steps 300 --warmup 20 > /dev/null 2>&1 || exit 1
for round in 1 2 3; do
  for c in "${counts[@]}"; do
    DMLP_HOST_OPS_CHUNKS=$c timeout -k 10 120 python bench.py --steps 400 --warmup 20 --no-busbw \
        > gpurun_out/hops/c$c.$round.log 2>&1 || exit 1
    echo "chunks $c round $round: $(tail -1 gpurun_out/hops/c$c.$round.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
for c in "${counts[@]}"; do
  DMLP_HOST_OPS_CHUNKS=$c DMLP_PIPE_DEBUG=1 DMLP_HOST_OPS_DEBUG=1 timeout -k 10 120 python bench.py \
      --steps 6 --warmup 2 --no-busbw > gpurun_out/hops/dbg$c.log 2>&1 || exit 1
  echo "== chunks $c"; grep -E "dmlp-pipe|dmlp-hostops" gpurun_out/hops/dbg$c.log | tail -4
done
