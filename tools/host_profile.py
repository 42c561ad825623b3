#!/usr/bin/env python3
"""Host-side cost of the headline step: cProfile over bench.py's step loop (after warm-up) plus
per-phase wall clocks of one call (DMLP_PIPE_DEBUG).  Usage (GPU box):
    python tools/host_profile.py [--steps 100] [--top 30]"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    import torch
    from distributed_machine_learning_project_amd.parallel.comm import Comm
    from distributed_machine_learning_project_amd.parallel.engine import Engine
    from distributed_machine_learning_project_amd.utils.io import generate
    from distributed_machine_learning_project_amd.utils.shm import share_input

    comm = Comm.init("gpu")
    inp = share_input(comm, generate(100_000, 131_072, 32, 0.0, 1000.0, 16, 16, 10, seed=42))
    eng = Engine("farm", comm=comm)

    def step():
        out = eng.KNN(inp.params, inp, None)
        return eng.report(out)

    for _ in range(10):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    print(f"plain: {1e3 * (time.perf_counter() - t0) / a.steps:.3f} ms/step")
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    pr.disable()
    print(f"profiled: {1e3 * (time.perf_counter() - t0) / a.steps:.3f} ms/step")
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(a.top)
    print(s.getvalue())
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(a.top)
    print(s.getvalue())
    inp.close()
    eng.close()


if __name__ == "__main__":
    main()
