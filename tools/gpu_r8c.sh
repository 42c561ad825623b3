# Pair refine survivors' phase: 8 lanes per exact row (4 rows per round) vs 16 (2 per round).
# Correctness of the 8-lane build first (bench --verify, native-step GPU tests), then kernel A/B.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r8c
rm -rf gpurun_out/ab
DMLP_LIB=ab/libdmlp_rl8.so timeout -k 10 300 python bench.py --steps 100 --verify > gpurun_out/r8c/verify_rl8.log 2>&1 || { tail -5 gpurun_out/r8c/verify_rl8.log; exit 1; }
echo "rl8 verify: $(grep -o '"verify_ok": [a-z]*' gpurun_out/r8c/verify_rl8.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r8c/verify_rl8.log | head -1)"
DMLP_LIB=ab/libdmlp_rl8.so timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_gpu_kernels.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r8c/tests_rl8.log 2>&1 || { tail -15 gpurun_out/r8c/tests_rl8.log; exit 1; }
tail -1 gpurun_out/r8c/tests_rl8.log
AB_PROF=1 AB_ROUNDS=2 AB_STEPS=30 bash tools/kernel_ab.sh rl16 rl8 || exit 1
python tools/ab_summary.py
AB_PROF=0 AB_ROUNDS=2 AB_STEPS=200 bash tools/kernel_ab.sh rl16 rl8
