#!/bin/bash
# Native knn_engine on one MI355X: every strategy (and the --exact path) must print the CPU
# oracle's bytes.   usage: tools/engine_check.sh [outdir]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/engine}
mkdir -p "$OUT"
E=distributed_machine_learning_project_amd/knn_engine
python3 - "$OUT" <<'PY'
import sys
import distributed_machine_learning_project_amd as dmlp
from distributed_machine_learning_project_amd.ops import knn as K
out = sys.argv[1]
# a, b: mixed k (general path); c, d: every k in [1, 32] (the single-GPU host-operand fast path)
for name, args in [("a", (20000, 3000, 32, 0, 1000, 1, 200, 10)), ("b", (5000, 700, 7, -5, 5, 1, 40, 3)),
                   ("c", (20000, 3000, 32, 0, 1000, 1, 32, 10)), ("d", (9000, 777, 50, 0, 100, 16, 16, 4))]:
    txt = dmlp.generate_text(*args, seed=5)
    open(f"{out}/{name}.in", "w").write(txt)
    inp = dmlp.parse_input(txt)
    d, i = K.knn_cpu(inp.X, inp.Qx, inp.k)
    _, cs = K.finalize_cpu(i, inp.k, inp.labels)
    open(f"{out}/{name}.expect", "wb").write(dmlp.format_report(cs))
PY
rc=0
for f in a b c d; do
  for s in farm shard_gather shard_reduce grid2d ring serial; do
    timeout -k 10 120 $E --strategy $s --input $OUT/$f.in > $OUT/$f.$s.out 2> $OUT/$f.$s.err; r=$?
    if [ $r -ne 0 ]; then echo "FAIL rc=$r $f $s"; cat $OUT/$f.$s.err; exit $r; fi
    if cmp -s $OUT/$f.$s.out $OUT/$f.expect; then echo "OK $f $s $(cat $OUT/$f.$s.err)"; else echo "MISMATCH $f $s"; rc=1; fi
  done
done
KNN_FAST=0 timeout -k 10 120 $E --strategy farm --input $OUT/c.in > $OUT/c.slow.out 2> $OUT/c.slow.err \
  && cmp -s $OUT/c.slow.out $OUT/c.expect && echo "OK c farm general path $(cat $OUT/c.slow.err)" \
  || { echo "c general-path mismatch"; rc=1; }
timeout -k 10 120 $E --strategy farm --exact --input $OUT/a.in > $OUT/a.exact.out 2> $OUT/a.exact.err \
  && cmp -s $OUT/a.exact.out $OUT/a.expect && echo "OK exact $(cat $OUT/a.exact.err)" \
  || { echo "exact mismatch"; head -3 $OUT/a.exact.out; rc=1; }
exit $rc
