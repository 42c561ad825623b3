#!/bin/bash
# Kernel A/B on one GPU box, interleaved, one rocprofv3 --kernel-trace --stats run of the
# headline bench per variant and round.  A variant is either X (an alternative build of the
# library at ab/libdmlp_X.so, loaded through DMLP_LIB) or NAME:VAR=VAL[,VAR=VAL...] (the tree's
# library with those environment switches).
#   gpurun -- bash tools/kernel_ab.sh A B            # library builds
#   gpurun -- bash tools/kernel_ab.sh x1: x2:DMLP_X2=1
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for round in 1 2; do
  for V in "$@"; do
    NAME=${V%%:*}
    ENVS=()
    if [[ "$V" == *:* ]]; then
      IFS=',' read -ra kv <<< "${V#*:}"
      for e in "${kv[@]}"; do [ -n "$e" ] && ENVS+=("$e"); done
    else
      ENVS+=("DMLP_LIB=ab/libdmlp_$NAME.so")
    fi
    env "${ENVS[@]}" timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/$NAME.$round \
        -o run --output-format csv -- python3 bench.py --steps 30 --warmup 3 --no-busbw \
        > gpurun_out/ab/$NAME.$round.log 2>&1 || { tail -20 gpurun_out/ab/$NAME.$round.log; exit 1; }
    echo "$NAME.$round: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/$NAME.$round.log)"
  done
done
