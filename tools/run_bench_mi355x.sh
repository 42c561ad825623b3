#!/bin/bash
# MI355X counterpart of the reference's run_bench.sh: CONFIG 1-4 run the matching strategy on
# 1/2/4/8 GPUs of one node (one MPI rank per GPU), CONFIG debug runs the serial KD-tree on the
# CPU; every run (debug: the GPU farm's DEBUG listing) is checked byte-for-byte against the serial
# oracle (a mismatch fails the script) and the "Time taken" lines
# are compared like run_bench.sh:29-72.  Inputs are generated (the reference's inputs.zip is
# absent) and cached under inputs/.
#
#   tools/run_bench_mi355x.sh <1|2|3|4|debug|all> [native|python|dropin]
#
# IMPL: native = knn_engine (this framework's own harness and parser); python = the torchrun
# front end; dropin = the reference's own harness: `make engine engine.debug` (top-level Makefile:
# the reference's unmodified common.cpp linked with include/engine.h + dropin_engine.cpp), then
# `mpiexec -n P ./engine < input` exactly as run_bench.sh:74,84 runs it (strategy from KNN_STRATEGY).
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
CONFIG="${1:-}"
IMPL="${2:-native}"
if [[ ! "$CONFIG" =~ ^(1|2|3|4|debug|all)$ ]]; then
  echo "Usage: $0 <1|2|3|4|debug|all> [native|python|dropin]"
  echo "  1 - shard_gather (bench_1) on 1 GPU      2 - shard_reduce (bench_2) on 2 GPUs"
  echo "  3 - shard_reduce batched (bench_3) on 4  4 - farm (bench_4) on 8 GPUs"
  echo "  debug - serial KD-tree (bench.debug) on the CPU"
  exit 1
fi
cd "$ROOT"
python3 -m distributed_machine_learning_project_amd.build >/dev/null
[[ "$IMPL" == "dropin" ]] && make -s engine engine.debug >/dev/null
mkdir -p inputs outputs
gen() {  # name N Q A kmin kmax
  [[ -f inputs/$1.in ]] || python3 tools/generate_input.py --fast --num_data $2 --num_queries $3 \
      --num_attrs $4 --min 0 --max 1000 --minK $5 --maxK $6 --num_labels 10 --output inputs/$1.in >/dev/null
}
gen input1 100000 20000 32 1 32
gen input2 200000 40000 32 1 64
gen input3 100000 100000 32 16 16
run() {  # config strategy gpus input [--debug]
  local cfg=$1 strat=$2 np=$3 in=inputs/$4.in dbg=${5:-}
  local ref=outputs/ref_$4${dbg:+_debug}
  if [[ ! -f $ref.out ]]; then
    timeout 3000 distributed_machine_learning_project_amd/knn_engine --strategy serial $dbg < $in \
        > $ref.out 2> $ref.err
  fi
  local launch=(/opt/conda/bin/mpiexec -n $np)
  [[ $np -eq 1 ]] && launch=()
  if [[ "$IMPL" == "dropin" ]]; then
    local exe=./engine
    [[ -n "$dbg" ]] && exe=./engine.debug
    # every rank opens the input as its stdin (only rank 0 reads it, common.cpp:93; MPICH's stdin
    # forwarding to rank 0 can die with SIGPIPE on large inputs)
    KNN_STRATEGY=$strat timeout 300 "${launch[@]}" sh -c "exec $exe < $in" \
        > outputs/tmp_$cfg.out 2> outputs/tmp_$cfg.err
  elif [[ "$IMPL" == "native" ]]; then
    timeout 300 "${launch[@]}" distributed_machine_learning_project_amd/knn_engine \
        --strategy $strat $dbg < $in > outputs/tmp_$cfg.out 2> outputs/tmp_$cfg.err
  else
    timeout 300 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node $np \
        --master-addr 127.0.0.1 --master-port $((29500 + np)) \
        -m distributed_machine_learning_project_amd.harness --strategy $strat --input $in $dbg \
        > outputs/tmp_$cfg.out 2> outputs/tmp_$cfg.err
  fi
  local ref_t eng_t
  ref_t=$(grep -oP 'Time taken:\s*\K[0-9]+' $ref.err)
  eng_t=$(grep -oP 'Time taken:\s*\K[0-9]+' outputs/tmp_$cfg.err)
  echo "=== CONFIG $cfg: $strat on $np GPU(s), $4 ==="
  echo "Serial KD-tree time: ${ref_t} ms"
  echo "Engine time:         ${eng_t} ms"
  if cmp -s $ref.out outputs/tmp_$cfg.out; then echo "Output: identical"; else echo "Output: MISMATCH"; return 1; fi
}
case "$CONFIG" in
  1) run 1 shard_gather 1 input1 ;;
  2) run 2 shard_reduce 2 input2 ;;
  3) run 3 shard_reduce 4 input2 ;;
  4) run 4 farm 8 input3 ;;
  # DEBUG listing (common.cpp:72-78): the GPU farm's listing byte-compared with the serial
  # KD-tree's (bench.debug), like the other configs
  debug) run debug farm 1 input1 --debug ;;
  all) for c in 1 2 3 4; do "$0" $c "$IMPL"; done ;;
esac
