#!/usr/bin/env python3
"""Host-budget rehearsal of an 8-GPU node on ONE MI355X.

One GPU rank runs the headline step (bench_4 shape, its 131072-query block) while P - 1 CPU-only
"phantom" ranks do, concurrently and in lockstep, exactly the host work their GPU ranks would
do on a real node: the node render plane's protocol (their share of the dataset's rows, the
centre's handshake, the waits for every other slice) and their own query block's host work.
Every rank gets DMLP_HOST_THREADS threads (16 CPUs / 8 ranks = 2 on a node granting 16 per
GPU).  The GPU rank's ms/step against its solo run (same threads, no phantoms) is the contention
the host budget costs; --plane 0 makes every rank render the whole dataset (no plane);
--render sets the GPU rank's DMLP_DEVICE_RENDER (an early-start step renders on the host anyway).

    python tools/host_rehearsal.py --ranks 8 --threads 2 --plane 1 --render device --steps 100
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _phantom(path, rank, world, qblk, steps, plane_on, render, threads, ready):
    os.environ["DMLP_HOST_THREADS"] = str(threads)
    import ctypes as C
    import numpy as np
    from distributed_machine_learning_project_amd import _lib
    from distributed_machine_learning_project_amd.utils.shm import SharedInput
    L = _lib.lib()
    inp = SharedInput.attach(path)
    N, A = inp.X.shape
    q0, q1 = rank * qblk, (rank + 1) * qblk
    kt = 1 if A <= 32 else 2 if A <= 64 else 4 if A <= 128 else 8
    h32 = np.zeros((q1 - q0) * A, np.int32)
    x32 = np.zeros(N * A, np.int32)
    qhi = np.zeros((q1 - q0) * kt * 32, np.uint16)
    qn = np.zeros(q1 - q0, np.float32)
    mu = np.zeros(A)
    t0, t1 = C.c_int64(), C.c_int64()
    ns = L.dmlp_plane_slice(N, A, 0, C.byref(t0), C.byref(t1))
    nt = (N + 63) // 64
    img = np.zeros(nt * 64 * kt * 32, np.uint16)
    xin = np.zeros(nt * 64, np.float32)
    nm = C.c_float()
    Xp = inp.X.ctypes.data
    ready.put(rank)
    for _ in range(steps):
        # an early-start step's host work (the bench shape always starts early, and an early step
        # renders its screen operands on the host whatever DMLP_DEVICE_RENDER says: pipeline.hip
        # dr_early_ok): the centre, this rank's query operands, the image and the int32 rows
        pl = inp.plane(rank, world) if plane_on else None
        if pl is not None:
            assert L.dmlp_plane_get_mu(C.byref(pl), A, mu.ctypes.data) == 0
        else:
            L.dmlp_cpu_center(Xp, N, A, mu.ctypes.data)
        L.dmlp_cpu_prep_queries(inp.Qx[q0:q1].ctypes.data, q1 - q0, A, mu.ctypes.data, kt,
                                qhi.ctypes.data, qn.ctypes.data)
        if pl is not None:  # this rank's share of the node's slices, then every other slice
            for what in (1, 2):
                for i in range(rank, ns, world):
                    L.dmlp_plane_render(C.byref(pl), Xp, None, N, A, mu.ctypes.data, what, i)
        else:  # the whole dataset, this rank alone
            L.dmlp_cpu_prep_data_tiles(Xp, N, A, mu.ctypes.data, kt, 0, nt, img.ctypes.data,
                                       xin.ctypes.data, C.byref(nm))
            L.dmlp_cpu_rows_i32(Xp, N * A, x32.ctypes.data)
        L.dmlp_cpu_rows_i32(inp.Qx[q0:q1].ctypes.data, (q1 - q0) * A, h32.ctypes.data)
        if pl is not None:
            for what in (1, 2):
                for i in range(ns):
                    assert L.dmlp_plane_wait(C.byref(pl), what, i, None, None) == 0
        inp.barrier(world)  # the egress barrier of every front end
        inp.barrier(world)


def main():
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--threads", type=int, default=2)
    ap.add_argument("--plane", type=int, default=1)
    ap.add_argument("--render", default="device", choices=["device", "host"])
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--n-data", type=int, default=100_000)
    ap.add_argument("--q-per-gpu", type=int, default=131_072)
    a = ap.parse_args()
    os.environ["DMLP_HOST_THREADS"] = str(a.threads)
    os.environ["DMLP_DEVICE_RENDER"] = "1" if a.render == "device" else "0"
    import numpy as np
    import torch
    from distributed_machine_learning_project_amd.ops import knn as K
    from distributed_machine_learning_project_amd.utils.io import generate
    from distributed_machine_learning_project_amd.utils.shm import SharedInput
    P = a.ranks
    inp0 = generate(a.n_data, a.q_per_gpu * P, 32, 0.0, 1000.0, 16, 16, 10, seed=42)
    inp = SharedInput.create(inp0, plane=a.plane and P > 1)
    inp.pin()
    total = a.warmup + a.steps
    ctx = mp.get_context("spawn")
    ready = ctx.Queue()
    procs = [ctx.Process(target=_phantom, args=(inp.path, r, P, a.q_per_gpu, total, a.plane,
                                                a.render, a.threads, ready))
             for r in range(1, P)]
    for p in procs:
        p.start()
    for _ in procs:
        ready.get(timeout=300)
    inp.unlink()
    q1 = a.q_per_gpu
    dst = torch.empty(48 * q1 + 64, dtype=torch.uint8).pin_memory().numpy()
    times, iters = [], []
    for s in range(total):
        pl = inp.plane(0, P) if a.plane and P > 1 else None
        t = time.perf_counter()
        r = K.step(inp.X, inp.labels, (0, 10), inp.Qx[:q1], inp.k[:q1], report=dst, plane=pl)
        times.append(time.perf_counter() - t)
        if P > 1:
            inp.barrier(P)
            inp.barrier(P)
        iters.append(time.perf_counter() - t)  # + the wait for the slowest phantom
    for p in procs:
        p.join(60)
    st = np.array(times[a.warmup:]) * 1e3
    out = {"ranks": P, "threads": a.threads, "plane": a.plane, "render": a.render,
           "gpu_rank_step_ms_mean": round(float(st.mean()), 4),
           "p50": round(float(np.percentile(st, 50)), 4),
           "p90": round(float(np.percentile(st, 90)), 4),
           "iteration_ms_mean": round(float(np.mean(iters[a.warmup:]) * 1e3), 4),
           "device_render": K.pipeline_stats()["device_render"], "early": r.early}
    print(json.dumps(out), flush=True)
    inp.close()


if __name__ == "__main__":
    main()
