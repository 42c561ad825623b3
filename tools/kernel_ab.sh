#!/bin/bash
# A/B on one GPU box, interleaved rounds of the headline bench per variant.  A variant is either
# X (an alternative build of the library at ab/libdmlp_X.so, loaded through DMLP_LIB) or
# NAME:VAR=VAL[,VAR=VAL...] (the tree's library with those environment switches).
#   gpurun -- bash tools/kernel_ab.sh A B                            # library builds, kernel trace
#   gpurun -- bash tools/kernel_ab.sh base: early0:DMLP_FAST_EARLY=0          # environment switches
#   AB_PROF=0 AB_ROUNDS=3 gpurun -- bash tools/kernel_ab.sh c1:DMLP_HOST_OPS_CHUNKS=1 c2:DMLP_HOST_OPS_CHUNKS=2
# AB_ARGS: extra bench.py arguments (e.g. "--q-per-gpu 32768").
# AB_PROF=1 (default): rocprofv3 --kernel-trace --stats per run (tools/ab_summary.py reads the
# kernel medians); AB_PROF=0: plain bench.py runs (host-side settings: no tracer overhead).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
export DMLP_BENCH_CONTRACT_RUNS=0  # no reference-contract processes after the timed steps
PROF=${AB_PROF:-1}
ROUNDS=${AB_ROUNDS:-2}
STEPS=${AB_STEPS:-30}
mkdir -p gpurun_out/ab
[ "$PROF" = 0 ] && { timeout -k 10 120 python bench.py --steps 100 --warmup 10 > /dev/null 2>&1 || exit 1; }
for round in $(seq 1 "$ROUNDS"); do
  for V in "$@"; do
    NAME=${V%%:*}
    ENVS=()
    if [[ "$V" == *:* ]]; then
      IFS=',' read -ra kv <<< "${V#*:}"
      for e in "${kv[@]}"; do [ -n "$e" ] && ENVS+=("$e"); done
    else
      ENVS+=("DMLP_LIB=ab/libdmlp_$NAME.so")
    fi
    LOG=gpurun_out/ab/$NAME.$round.log
    if [ "$PROF" = 0 ]; then
      env "${ENVS[@]}" timeout -k 10 120 python bench.py --steps "$STEPS" --warmup 20 --no-busbw \
          ${AB_ARGS:-} > "$LOG" 2>&1 || { tail -20 "$LOG"; exit 1; }
    else
      env "${ENVS[@]}" timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/$NAME.$round \
          -o run --output-format csv -- python3 bench.py --steps "$STEPS" --warmup 3 --no-busbw \
          > "$LOG" 2>&1 || { tail -20 "$LOG"; exit 1; }
    fi
    echo "$NAME.$round: $(grep -o '"ms_per_step": [0-9.]*' "$LOG")"
  done
done
