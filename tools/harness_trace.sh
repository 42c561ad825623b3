# Reference-contract runs on the bench shape with KNN_TRACE=1: knn_engine (its own parser, flat
# pinned rows) and the drop-in (the reference's common.cpp, rows read in place), one process per
# run: the engine phases and the step's hipEvent timeline of each cold call.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/harness_trace; mkdir -p $OUT
EXE=distributed_machine_learning_project_amd/_build/engine_dropin
[ -x $EXE ] || python -c "from distributed_machine_learning_project_amd import build; build.build_dropin(str(build.reference_harness()), out='$EXE')"
python - <<'PY'
from distributed_machine_learning_project_amd.utils.io import generate, to_text
inp = generate(100000, 131072, 32, 0.0, 1000.0, 16, 16, 10, seed=42)
open("/tmp/bench.in", "w").write(to_text(inp))
PY
for r in 1 2 3; do
  for H in native dropin; do
    if [ $H = native ]; then CMD="distributed_machine_learning_project_amd/knn_engine --input /tmp/bench.in"; else CMD="$EXE"; fi
    KNN_TRACE=1 KNN_METRICS=$OUT/$H$r.json timeout -k 10 120 $CMD < /tmp/bench.in > /tmp/out_$H.txt 2> $OUT/err_$H$r.txt || { tail -5 $OUT/err_$H$r.txt; exit 1; }
    echo "$H $r: $(cat $OUT/$H$r.json)"; grep -E "timeline|dmlp-trace" $OUT/err_$H$r.txt | tail -7
  done
done
cmp /tmp/out_native.txt /tmp/out_dropin.txt && echo "outputs identical"
