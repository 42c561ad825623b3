# Early-start query render slices on the final tree: DMLP_FAST_QCHUNKS 2 / 4 (default) / 8,
# interleaved plain-bench rounds
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
rm -rf gpurun_out/ab
AB_PROF=0 AB_ROUNDS=3 AB_STEPS=200 bash tools/kernel_ab.sh q4: q2:DMLP_FAST_QCHUNKS=2 q8:DMLP_FAST_QCHUNKS=8 | grep -v '^"ms'
