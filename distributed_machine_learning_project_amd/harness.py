"""Reference-compatible harness (common.cpp:81-135) on the MI355X engine.

    python -m distributed_machine_learning_project_amd.harness [--strategy S] [--debug] < input
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m distributed_machine_learning_project_amd.harness < input

Rank 0 reads and parses stdin (untimed), all ranks barrier, the Engine is constructed
(untimed: process group, device binding, kernel warm-up), rank 0 starts the clock, every rank
calls KNN, rank 0 renders the report, all ranks barrier, rank 0 stops the clock and prints
"Time taken: <ms> ms" on stderr.  stdout is written once, at the end (the reference's buffered
cout).  Malformed input raises like common.cpp:100-115.
"""
from __future__ import annotations

import argparse
import os
import sys
import time


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--strategy", default=os.environ.get("KNN_STRATEGY", "farm"))
    ap.add_argument("--device", default=os.environ.get("KNN_DEVICE", "auto"), choices=["auto", "gpu", "cpu"])
    ap.add_argument("--debug", action="store_true", help="DEBUG listing output (engine.debug)")
    ap.add_argument("--exact", action="store_true", help="skip the MFMA screen (fp64 only)")
    ap.add_argument("--schedule", default=os.environ.get("KNN_SCHEDULE", "static"),
                    choices=["static", "dynamic"])
    ap.add_argument("--input", default="-", help="input file (default: stdin)")
    ap.add_argument("--ingress", default=os.environ.get("KNN_INGRESS", "root"), choices=["root", "shm"],
                    help="root: rank 0 holds the parsed input (reference); shm: node-shared "
                         "segment, every GPU copies its own part (utils/shm.py)")
    a = ap.parse_args(argv)

    from .parallel.comm import Comm
    from .parallel.engine import Engine
    from .utils.io import read_input

    comm = Comm.init(a.device)
    inp = None
    if comm.is_root:
        inp = read_input(a.input)
    if a.ingress == "shm":  # part of ingest (untimed): the parsed arrays go to a shared segment
        from .utils.shm import share_input
        inp = share_input(comm, inp)
    elif comm.is_root and comm.on_gpu:
        import torch  # page-locked copies so the timed H2D runs at full PCIe speed
        for name in ("X", "labels", "Qx", "k"):
            setattr(inp, name + "_t", torch.from_numpy(getattr(inp, name)).pin_memory())
    comm.barrier()
    eng = Engine(a.strategy, comm=comm, exact=a.exact or None, debug=a.debug, schedule=a.schedule)
    t0 = time.perf_counter() if comm.is_root else 0.0
    out = eng.KNN(inp.params if inp is not None and comm.is_root else None, inp, None)
    rep = eng.report(out) if out is not None else b""
    comm.sync()
    comm.barrier()
    t1 = time.perf_counter()
    coll = None
    if comm.world > 1 and os.environ.get("DMLP_COLL_CHECK", "0") not in ("", "0"):
        # after the clock stopped: every rank's collective sequence compared on rank 0
        from .parallel import dist_api
        coll = dist_api.check_collective_sequence()
    if comm.is_root:
        ms = int((t1 - t0) * 1000)
        sys.stdout.buffer.write(rep)
        sys.stdout.flush()
        print(f"Time taken: {ms} ms", file=sys.stderr, flush=True)
        if coll is not None:
            print(f"[dmlp-coll] ok={coll['ok']} calls={coll['calls_per_rank']} "
                  f"problems={coll['problems']}", file=sys.stderr, flush=True)
            if not coll["ok"]:
                return 3
    if a.ingress == "shm":
        inp.close()
    eng.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
