# dot2 member scores: which results differ (native-step GPU tests on the dot2 build), and the
# base build's --verify as the control.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r8f
DMLP_LIB=ab/libdmlp_base.so timeout -k 10 300 python bench.py --steps 50 --verify > gpurun_out/r8f/verify_base.log 2>&1 || { tail -5 gpurun_out/r8f/verify_base.log; exit 1; }
echo "base verify: $(grep -o '"verify_ok": [a-z]*' gpurun_out/r8f/verify_base.log)"
DMLP_LIB=ab/libdmlp_dot2.so timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "native_step and not early" > gpurun_out/r8f/tests_dot2.log 2>&1
tail -40 gpurun_out/r8f/tests_dot2.log
