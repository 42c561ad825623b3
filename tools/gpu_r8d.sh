# Pair refine survivors' phase: 4 lanes per exact row (8 rows per round) vs 8 (4 per round).
# Correctness of the 4-lane build first (bench --verify, native-step GPU tests), then kernel A/B.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r8d
rm -rf gpurun_out/ab
DMLP_LIB=ab/libdmlp_rl4.so timeout -k 10 300 python bench.py --steps 100 --verify > gpurun_out/r8d/verify_rl4.log 2>&1 || { tail -5 gpurun_out/r8d/verify_rl4.log; exit 1; }
echo "rl4 verify: $(grep -o '"verify_ok": [a-z]*' gpurun_out/r8d/verify_rl4.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r8d/verify_rl4.log | head -1)"
DMLP_LIB=ab/libdmlp_rl4.so timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_gpu_kernels.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r8d/tests_rl4.log 2>&1 || { tail -15 gpurun_out/r8d/tests_rl4.log; exit 1; }
tail -1 gpurun_out/r8d/tests_rl4.log
AB_PROF=1 AB_ROUNDS=2 AB_STEPS=30 bash tools/kernel_ab.sh rl8g rl4 || exit 1
python tools/ab_summary.py
AB_PROF=0 AB_ROUNDS=2 AB_STEPS=200 bash tools/kernel_ab.sh rl8g rl4
