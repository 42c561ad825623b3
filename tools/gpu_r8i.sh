# Pair refine members from a point-major copy of the fp16 image (DMLP_PAIR_ROWMAJOR=1) vs the
# tile image (default): --verify, GPU engine/kernel tests with it on, then kernel + step A/B.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r8i
rm -rf gpurun_out/ab
DMLP_PAIR_ROWMAJOR=1 timeout -k 10 300 python bench.py --steps 100 --verify > gpurun_out/r8i/verify.log 2>&1 || { tail -5 gpurun_out/r8i/verify.log; exit 1; }
echo "rowmajor verify: $(grep -o '"verify_ok": [a-z]*' gpurun_out/r8i/verify.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r8i/verify.log | head -1)"
DMLP_PAIR_ROWMAJOR=1 timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_gpu_kernels.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r8i/tests.log 2>&1 || { tail -15 gpurun_out/r8i/tests.log; exit 1; }
tail -1 gpurun_out/r8i/tests.log
AB_PROF=1 AB_ROUNDS=2 AB_STEPS=30 bash tools/kernel_ab.sh rm:DMLP_PAIR_ROWMAJOR=1 tile: | grep -v '^"ms' || exit 1
python tools/ab_summary.py
AB_PROF=0 AB_ROUNDS=3 AB_STEPS=200 bash tools/kernel_ab.sh rm:DMLP_PAIR_ROWMAJOR=1 tile: | grep -v '^"ms'
