#!/bin/bash
# Host-side timing of the host-rendered screen operands inside the bench (per-chunk marks),
# for 1 / 4 / 8 chunks.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/hod
for c in 1 4 8; do
DMLP_HOST_OPS_CHUNKS=$c DMLP_PIPE_DEBUG=1 DMLP_HOST_OPS_DEBUG=1 timeout -k 10 200 python bench.py --steps 20 --warmup 3 \
    > gpurun_out/hod/bench_c$c.json 2> gpurun_out/hod/bench_c$c.err || exit $?
tail -2 gpurun_out/hod/bench_c$c.err; cut -c1-140 gpurun_out/hod/bench_c$c.json
done
