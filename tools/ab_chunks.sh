# host-operand slices A/B on the native step: DMLP_HOST_OPS_CHUNKS = 2 4 6 3 2 4, then one run
# with the host render's own timestamps (DMLP_HOST_OPS_DEBUG)
set -e
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r5r
for C in 2 4 6 3 2 4; do
  DMLP_HOST_OPS_CHUNKS=$C timeout -k 10 200 python bench.py > gpurun_out/r5r/bench_c$C.log 2>&1
  echo "chunks=$C $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5r/bench_c$C.log | head -1) $(grep -o '"step_timeline_ms": {[^}]*}' gpurun_out/r5r/bench_c$C.log | head -1)"
done
DMLP_HOST_OPS_DEBUG=1 timeout -k 10 200 python bench.py --steps 5 --warmup 2 > gpurun_out/r5r/hostops_debug.log 2>&1
grep dmlp-hostops gpurun_out/r5r/hostops_debug.log | tail -6
