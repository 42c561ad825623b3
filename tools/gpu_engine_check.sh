#!/bin/bash
# Native knn_engine on one MI355X: every strategy must print the CPU oracle's bytes.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/engine
E=distributed_machine_learning_project_amd/knn_engine
python3 - <<'PY'
import distributed_machine_learning_project_amd as dmlp
from distributed_machine_learning_project_amd.ops import knn as K
for name, args in [("a", (20000, 3000, 32, 0, 1000, 1, 200, 10)), ("b", (5000, 700, 7, -5, 5, 1, 40, 3))]:
    txt = dmlp.generate_text(*args, seed=5)
    open(f"gpurun_out/engine/{name}.in", "w").write(txt)
    inp = dmlp.parse_input(txt)
    d, i = K.knn_cpu(inp.X, inp.Qx, inp.k)
    _, cs = K.finalize_cpu(i, inp.k, inp.labels)
    open(f"gpurun_out/engine/{name}.expect", "wb").write(dmlp.format_report(cs))
PY
rc=0
for f in a b; do
  for s in farm shard_gather shard_reduce grid2d serial; do
    timeout -k 10 120 $E --strategy $s --input gpurun_out/engine/$f.in > gpurun_out/engine/$f.$s.out 2> gpurun_out/engine/$f.$s.err; r=$?
    if [ $r -ne 0 ]; then echo "FAIL rc=$r $f $s"; cat gpurun_out/engine/$f.$s.err; exit $r; fi
    if cmp -s gpurun_out/engine/$f.$s.out gpurun_out/engine/$f.expect; then echo "OK $f $s $(cat gpurun_out/engine/$f.$s.err)"; else echo "MISMATCH $f $s"; rc=1; fi
  done
done
timeout -k 10 120 $E --strategy farm --exact --input gpurun_out/engine/a.in > gpurun_out/engine/a.exact.out 2> gpurun_out/engine/a.exact.err && cmp -s gpurun_out/engine/a.exact.out gpurun_out/engine/a.expect && echo "OK exact" || { echo "exact mismatch"; head -3 gpurun_out/engine/a.exact.out; rc=1; }
exit $rc
