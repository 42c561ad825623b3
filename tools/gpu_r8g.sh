# dot2 member scores: which bench_4 queries differ from the base build (tools/probe/refine_diff.py)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r8g
DMLP_LIB=ab/libdmlp_base.so PYTHONPATH=. timeout -k 10 200 python tools/probe/refine_diff.py save /tmp/base || exit 1
DMLP_LIB=ab/libdmlp_dot2.so PYTHONPATH=. timeout -k 10 200 python tools/probe/refine_diff.py cmp /tmp/base
