# Pair refine member scores: v_dot2c_f32_f16 (dot2) vs cvt + fma (base); verify first, then A/B.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r8e
rm -rf gpurun_out/ab
DMLP_LIB=ab/libdmlp_dot2.so timeout -k 10 300 python bench.py --steps 100 --verify > gpurun_out/r8e/verify_dot2.log 2>&1 || { tail -5 gpurun_out/r8e/verify_dot2.log; exit 1; }
echo "dot2 verify: $(grep -o '"verify_ok": [a-z]*' gpurun_out/r8e/verify_dot2.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r8e/verify_dot2.log | head -1)"
AB_PROF=1 AB_ROUNDS=3 AB_STEPS=30 bash tools/kernel_ab.sh base dot2 || exit 1
python tools/ab_summary.py
