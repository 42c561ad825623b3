# Pair refine with the lean member phase (dot2, point-major): U = 2 members per lane at 6 / 8
# waves per SIMD vs U = 1 at 8 (b); kernel trace A/B, then --verify of the fastest U = 2 build.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
rm -rf gpurun_out/ab
AB_PROF=1 AB_ROUNDS=2 AB_STEPS=30 bash tools/kernel_ab.sh b u2w6 u2w8 | grep -v '^"ms' || exit 1
python tools/ab_summary.py
DMLP_LIB=ab/libdmlp_u2w6.so timeout -k 10 300 python bench.py --steps 100 --verify > gpurun_out/ab/verify_u2w6.log 2>&1 || { tail -5 gpurun_out/ab/verify_u2w6.log; exit 1; }
echo "u2w6 verify: $(grep -o '"verify_ok": [a-z]*' gpurun_out/ab/verify_u2w6.log)"
