#!/bin/bash
# Kernel A/B on one GPU box: alternative builds of libdmlp.so (ab/libdmlp_<X>.so, DMLP_LIB) run the
# headline bench under rocprofv3 --kernel-trace --stats, interleaved, one directory per run.
#   gpurun -- bash tools/kernel_ab.sh A B C
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for round in 1 2; do
  for X in "$@"; do
    DMLP_LIB=ab/libdmlp_$X.so timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/$X.$round \
        -o run --output-format csv -- python3 bench.py --steps 30 --warmup 3 --no-busbw \
        > gpurun_out/ab/$X.$round.log 2>&1 || { tail -20 gpurun_out/ab/$X.$round.log; exit 1; }
    echo "$X.$round done"
  done
done
