# dot2 member scores (explicit word extraction): bench_4 lists vs base, --verify, GPU tests, A/B.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r8h
rm -rf gpurun_out/ab
DMLP_LIB=ab/libdmlp_base.so PYTHONPATH=. timeout -k 10 200 python tools/probe/refine_diff.py save /tmp/base > gpurun_out/r8h/diff.log 2>&1 || exit 1
DMLP_LIB=ab/libdmlp_dot2.so PYTHONPATH=. timeout -k 10 200 python tools/probe/refine_diff.py cmp /tmp/base >> gpurun_out/r8h/diff.log 2>&1 || exit 1
grep "queries differing" gpurun_out/r8h/diff.log
DMLP_LIB=ab/libdmlp_dot2.so timeout -k 10 300 python bench.py --steps 100 --verify > gpurun_out/r8h/verify_dot2.log 2>&1 || { tail -5 gpurun_out/r8h/verify_dot2.log; exit 1; }
echo "dot2 verify: $(grep -o '"verify_ok": [a-z]*' gpurun_out/r8h/verify_dot2.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r8h/verify_dot2.log | head -1)"
DMLP_LIB=ab/libdmlp_dot2.so timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_gpu_kernels.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r8h/tests_dot2.log 2>&1 || { tail -15 gpurun_out/r8h/tests_dot2.log; exit 1; }
tail -1 gpurun_out/r8h/tests_dot2.log
AB_PROF=1 AB_ROUNDS=2 AB_STEPS=30 bash tools/kernel_ab.sh base dot2 || exit 1
python tools/ab_summary.py
AB_PROF=0 AB_ROUNDS=2 AB_STEPS=200 bash tools/kernel_ab.sh base dot2
