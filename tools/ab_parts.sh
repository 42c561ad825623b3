set -e
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r5p
export KTESTS="native_fast_step"
bash tools/gpu_session.sh r5p ktests
for P in 1 2 1 2 3 4; do
  DMLP_FAST_PARTS=$P timeout -k 10 200 python bench.py > gpurun_out/r5p/bench_p$P.log 2>&1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5p/bench_p$P.log | head -1
  cp gpurun_out/r5p/bench_p$P.log gpurun_out/r5p/bench_p${P}_$(date +%s).log
done
DMLP_FAST_PARTS=2 timeout -k 10 200 python bench.py --steps 20 --warmup 2 --verify > gpurun_out/r5p/verify_p2.log 2>&1
grep -o '"verify[a-z_]*": [a-zA-Z]*' gpurun_out/r5p/verify_p2.log
