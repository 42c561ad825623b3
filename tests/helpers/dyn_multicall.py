"""torchrun worker for tests/test_distributed.py::test_dynamic_shared_farm_many_calls: several
KNN calls through two Engines on ONE node-shared segment with the dynamic schedule.  Every call
must give the oracle's report and the per-rank claimed query counts must add up to Q (a rank
claiming from an exhausted counter would compute nothing and return stale rows silently)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    from distributed_machine_learning_project_amd.ops import reference as ref
    from distributed_machine_learning_project_amd.parallel.comm import Comm
    from distributed_machine_learning_project_amd.parallel.engine import Engine
    from distributed_machine_learning_project_amd.utils.io import generate
    from distributed_machine_learning_project_amd.utils.shm import share_input

    comm = Comm.init("cpu")
    inp = generate(300, 41, 5, 0.0, 10.0, 1, 9, 4, seed=11) if comm.is_root else None
    expect = None
    if comm.is_root:
        _, _, cs = ref.knn(inp.X, inp.labels, inp.Qx, inp.k)
        expect = ref.report_lines(cs).encode()
    seg = share_input(comm, inp)
    results = []
    for calls, eng in ((3, Engine("farm", comm=comm, schedule="dynamic", warmup=False)),
                       (2, Engine("farm", comm=comm, schedule="dynamic", warmup=False))):
        for _ in range(calls):
            out = eng.KNN(None, seg, None)
            counts = [c[0] for c in comm.allgather_ints([seg.last_claimed])]
            rep = bytes(eng.report(out)) if out is not None else None
            if comm.is_root:
                results.append({"claimed": counts, "ok": rep == expect})
    if comm.is_root:
        print(json.dumps({"Q": int(seg.Qx.shape[0]), "calls": results}), flush=True)
    seg.close()
    comm.finalize()


if __name__ == "__main__":
    main()
