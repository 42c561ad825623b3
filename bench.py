#!/usr/bin/env python3
"""Headline benchmark: bench_4-style distributed exact k-NN classification on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--strategy farm] ...
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Metric (BASELINE.json): "samples/sec (whole node) on bench_4" = classified queries per second
over all GPUs.  One step = one full Engine::KNN call exactly as the reference times it
(common.cpp:122-131): rank 0 holds the parsed input in host memory; the step moves it to the
GPUs, broadcasts the dataset (bench_4 replicates it), distributes the queries, runs the exact
k-NN (bf16 MFMA screen + exact fp64 re-rank), votes, checksums, gathers the results to rank 0
and renders the "Query <id> checksum: <u64>" report bytes on rank 0.

Config: the reference's inputs (inputs.zip) are not in the repository, so the workload is
synthetic data with generate_input.py's distribution at the only shape BASELINE.md quotes a
number for: N=100000 points, A=32 attributes in [0,1000] (6 decimals), k=16, 10 labels, seed 42;
Q = --q-per-gpu queries per GPU (default 2^17: whole rounds of 64-query waves on the 1024 SIMDs;
weak scaling: per-GPU work is fixed).
vs_baseline is null: BASELINE.md publishes no number for any bench_N.  The only number it quotes
at this shape is the student engine.cpp on an 8-vCPU CPU sandbox (np=4: 1000 queries in 2255 ms);
the ratio to that is reported under its own name, vs_student_engine_cpu_np4.

Ranks: `python bench.py --gpus N` with N > 1 and no torchrun environment launches N ranks itself
(torch.distributed.run as a child process, before this process makes any GPU call) and exits with
their exit code; it refuses to run when fewer than N GPUs are visible, unless DMLP_DATA_PLANE=host
(the one-GPU rehearsal: N ranks share the GPU over the host-staged gloo plane).  Under torchrun,
--gpus must equal WORLD_SIZE.  Rank 0's JSON then carries the world the process group really had
(rccl_world / data_plane), an RCCL all-reduce check and its bus bandwidth, and per rank: ms/step,
NUMA node, phase times and PCIe / collective bytes from an untimed traced pass after the timed
steps, plus a rank-by-rank comparison of the collective sequence (parallel/dist_api.py).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

BASELINE_QPS = 1000.0 / 2.255  # engine.cpp np=4, N=1e5 Q=1e3 A=32 k=16 -> 2255 ms


def _launch_ranks(a, argv):
    """`python bench.py --gpus N` outside torchrun: start N ranks (one per GPU) and return their
    exit code; None when this process is itself the (only) rank.  Nothing here initialises HIP
    (torch.cuda.device_count() does not), so the children own the GPUs."""
    if "WORLD_SIZE" in os.environ or a.gpus <= 1 or a.harness != "python":
        return None
    import subprocess
    import torch
    host_plane = os.environ.get("DMLP_DATA_PLANE", "") == "host"
    ndev = torch.cuda.device_count()
    if ndev < a.gpus and not host_plane:
        print(f"[bench] --gpus {a.gpus} but only {ndev} GPU(s) visible; refusing to bench fewer "
              f"ranks than asked (DMLP_DATA_PLANE=host rehearses {a.gpus} ranks on one GPU)",
              file=sys.stderr, flush=True)
        return 2
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={a.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    print(f"[bench] launching {a.gpus} ranks: {' '.join(cmd[1:6])} ...", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env)


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    # >= 200 steps: the timed region is >= 0.5 s at the bench shape (a driver-side busy sampler
    # sees the GPU working), and per-step jitter averages out
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--min-warmup-s", type=float, default=3.0,
                    help="keep running untimed warm-up steps (at least --warmup of them) until this "
                         "much time has passed: a fresh process runs its first seconds up to 40 %% "
                         "slower (profiles/r3k_warmup.txt; r6b: 2.77 ms/step after 0.6 s of warm-up "
                         "vs 2.36 after 3 s on the same box), which a 10-step warm-up does not "
                         "cover; the JSON's warmup_curve_ms shows the per-window means")
    ap.add_argument("--strategy", default="farm")
    ap.add_argument("--schedule", default="static", choices=["static", "dynamic"])
    ap.add_argument("--n-data", type=int, default=100_000)
    ap.add_argument("--q-per-gpu", type=int, default=131_072)
    ap.add_argument("--attrs", type=int, default=32)
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--kmin", type=int, default=None, help="per-query k drawn from [kmin, kmax] "
                    "(generate_input.py's minK/maxK; default: every k = --k)")
    ap.add_argument("--kmax", type=int, default=None)
    ap.add_argument("--labels", type=int, default=10)
    ap.add_argument("--exact", action="store_true", help="fp64-only path (no MFMA screen)")
    ap.add_argument("--ingress", default="shm", choices=["shm", "root"],
                    help="shm: parsed input in a node-shared page-locked segment, every GPU "
                         "copies its own part inside the timed step; root: rank 0 holds it and "
                         "funnels it through GPU 0 (reference layout)")
    ap.add_argument("--verify", action="store_true",
                    help="compare a SHA-256 digest of the WHOLE rank-0 report (every query line) "
                         "with the CPU oracle's (C++ fp64 brute force, outside the timed region)")
    ap.add_argument("--no-busbw", action="store_true")
    ap.add_argument("--diag-steps", type=int, default=3,
                    help="untimed traced steps after the timed ones: per-rank phase times, PCIe "
                         "and collective bytes, collective-sequence check (0: skip)")
    ap.add_argument("--contract-runs", type=int,
                    default=int(os.environ.get("DMLP_BENCH_CONTRACT_RUNS", "3")),
                    help="one GPU: after the timed steps, this many fresh processes of the engine.h "
                         "drop-in linked with the reference's own common.cpp at this config (the "
                         "reference's contract: one Engine::KNN call per process, parse untimed, "
                         "the report written to a redirected stdout) -> reference_contract in the "
                         "JSON (0: skip; default DMLP_BENCH_CONTRACT_RUNS or 3)")
    ap.add_argument("--harness", default="python", choices=["python", "native", "dropin"],
                    help="native: time the reference-contract binary (knn_engine: parse untimed, "
                         "'Time taken' = KNN + report + barrier, common.cpp:121-131) at this "
                         "config AND at BASELINE.md's Q = 1000, one process per run")
    a = ap.parse_args(argv)
    if a.harness in ("native", "dropin"):
        return _bench_native(a)
    rc = _launch_ranks(a, argv)
    if rc is not None:
        return rc

    import numpy as np
    import torch

    from distributed_machine_learning_project_amd.parallel.comm import Comm
    from distributed_machine_learning_project_amd.parallel.engine import Engine
    from distributed_machine_learning_project_amd.utils.io import generate

    host_plane = os.environ.get("DMLP_DATA_PLANE", "") == "host"
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus != world_env:
        print(f"[bench] --gpus {a.gpus} but WORLD_SIZE={world_env}: refusing to label a "
              f"{world_env}-rank run as {a.gpus} GPUs", file=sys.stderr, flush=True)
        return 2
    ndev = torch.cuda.device_count()
    if world_env > 1 and ndev and ndev < world_env and not host_plane:
        print(f"[bench] WORLD_SIZE={world_env} but only {ndev} GPU(s) visible (one rank per GPU; "
              f"DMLP_DATA_PLANE=host rehearses several ranks on one GPU)", file=sys.stderr,
              flush=True)
        return 2
    comm = Comm.init("gpu" if torch.cuda.is_available() else "cpu")
    world = comm.world
    if world != a.gpus:
        print(f"[bench] process group has {world} ranks, --gpus {a.gpus}", file=sys.stderr)
        return 2
    Q = a.q_per_gpu * world
    kmin = a.k if a.kmin is None else a.kmin
    kmax = max(kmin, a.k if a.kmax is None else a.kmax)

    inp = None
    if comm.is_root:
        inp = generate(a.n_data, Q, a.attrs, 0.0, 1000.0, kmin, kmax, a.labels, seed=42)
    # the "parsed input" lives in page-locked host memory (untimed, like parsing)
    if a.ingress == "shm":
        from distributed_machine_learning_project_amd.utils.shm import share_input
        inp = share_input(comm, inp)
    elif comm.is_root and comm.on_gpu:
        for name in ("X", "labels", "Qx", "k"):
            setattr(inp, name + "_t", torch.from_numpy(getattr(inp, name)).pin_memory())
    eng = Engine(a.strategy, comm=comm, exact=a.exact, schedule=a.schedule)

    def step():
        out = eng.KNN(inp.params if comm.is_root else None, inp, None)
        return eng.report(out) if out is not None else None

    import torch as _t
    t_w = time.perf_counter()
    warm = 0
    curve, t_win, n_win = [], time.perf_counter(), 0  # mean ms/step of each ~0.25 s window
    while True:
        if warm >= a.warmup:
            # every rank takes the same decision (rank 0's clock), so all run the same step count
            flag = _t.tensor([1.0 if time.perf_counter() - t_w >= a.min_warmup_s else 0.0],
                             dtype=_t.float64, device=comm.device)
            if world > 1:
                from distributed_machine_learning_project_amd.parallel import dist_api as dist
                dist.broadcast(flag, 0)
            if flag.item() > 0:
                break
        rep = step()
        warm += 1
        n_win += 1
        if time.perf_counter() - t_win >= 0.25:
            now = time.perf_counter()
            curve.append(round((now - t_win) / n_win * 1e3, 3))
            t_win, n_win = now, 0
    comm.sync()
    comm.barrier()
    thr0 = _cgroup_cpu_stat()
    from distributed_machine_learning_project_amd.ops import knn as K
    K.step_stats(reset=True)
    t0 = time.perf_counter()
    marks = [0.0] * a.steps  # host return time of each step (a perf_counter read per step)
    for j in range(a.steps):
        rep = step()
        marks[j] = time.perf_counter()
    comm.sync()
    comm.barrier()
    elapsed = time.perf_counter() - t0
    thr1 = _cgroup_cpu_stat()
    steps_native = K.step_stats()  # this rank's timed steps served by the native step
    elapsed_mine = elapsed
    # max over ranks
    el = torch.tensor([elapsed], dtype=torch.float64, device=comm.device)
    if world > 1:
        from distributed_machine_learning_project_amd.parallel import dist_api as dist
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    ms = elapsed / max(1, a.steps) * 1e3
    my_ms = elapsed_mine / max(1, a.steps) * 1e3  # this rank's own clock

    extra = _world_report(comm, host_plane, a)
    # the timed steps' spread and the CPU quota throttling the cgroup saw meanwhile: a slow run
    # with uniformly slow steps points at the device side, one with a few very slow steps and
    # throttled time at the host's CPU quota (the render pool + main thread spinning)
    if a.steps:
        st = np.diff(np.array([t0] + marks)) * 1e3
        extra["timed_step_ms"] = {"p10": round(float(np.percentile(st, 10)), 4),
                                  "p50": round(float(np.percentile(st, 50)), 4),
                                  "p90": round(float(np.percentile(st, 90)), 4),
                                  "max": round(float(st.max()), 4)}
    # the timed region, as the native pipeline saw it (a silent fallback or a stalled early start
    # would show here, not only as a slower ms_per_step): steps served by the native step, steps
    # whose screen started before the dataset image landed, early-start waits / timeouts, queries
    # escalated after a screen overflow, steps on the device-image path (data outside fp16)
    if comm.on_gpu:
        extra["native_step"] = {"step_calls": steps_native["calls"], "timed_steps": a.steps,
                                "early_start_calls": steps_native["early"],
                                "early_waits": steps_native["early_waits"],
                                "early_timeouts": steps_native["early_timeouts"],
                                # host time per step until everything was issued (render / int32
                                # pack, plane waits): the per-rank host budget
                                "host_issue_ms_per_step": round(
                                    steps_native["host_ms"] / max(1, steps_native["calls"]), 4),
                                "escalated_queries": steps_native["escalated"],
                                "device_path_calls": steps_native["device_path"]}
    if thr0 and thr1:
        extra["cgroup_cpu_during_timed"] = {
            "usage_ms": round((thr1.get("usage_usec", 0) - thr0.get("usage_usec", 0)) / 1e3, 1),
            "nr_throttled": thr1.get("nr_throttled", 0) - thr0.get("nr_throttled", 0),
            "throttled_ms": round((thr1.get("throttled_usec", 0) - thr0.get("throttled_usec", 0)) / 1e3, 1)}
    if a.diag_steps > 0:
        extra.update(_diagnostics(comm, eng, step, a.diag_steps, my_ms, steps_native))
    if world > 1 and comm.backend == "nccl" and not a.no_busbw:
        # a diagnostic beside the headline: a failure records itself instead of losing the line
        try:
            extra["allreduce_busbw_GBps"] = round(_allreduce_busbw(comm), 1)
        except Exception as e:  # noqa: BLE001
            extra["allreduce_busbw_GBps"] = {"error": f"{type(e).__name__}: {e}"[-300:]}
    if a.verify and comm.is_root:
        import hashlib
        from distributed_machine_learning_project_amd.ops import knn as K
        from distributed_machine_learning_project_amd.utils.io import format_report
        t_v = time.perf_counter()
        d, i = K.knn_cpu(inp.X, inp.Qx, inp.k)
        _, cs = K.finalize_cpu(i, inp.k, inp.labels)
        ref = format_report(cs)
        got = bytes(rep)
        extra["verified_queries"] = Q
        extra["report_sha256"] = hashlib.sha256(got).hexdigest()
        extra["oracle_sha256"] = hashlib.sha256(ref).hexdigest()
        extra["verify_ok"] = got == ref
        extra["verify_s"] = round(time.perf_counter() - t_v, 1)

    if (world == 1 and comm.on_gpu and not a.exact
            and os.environ.get("DMLP_BENCH_LARGE_N", "1") != "0"):
        # the large-N regime beside the headline (after its timed steps; a failure records itself)
        try:
            extra["large_n"] = _large_n(a)
        except Exception as e:  # noqa: BLE001
            extra["large_n"] = {"error": f"{type(e).__name__}: {e}"[-300:]}

    if a.contract_runs > 0 and comm.on_gpu:
        # the same config through the reference's own contract (bench_4's binary is timed this
        # way by run_bench.sh:114-120): fresh processes, median of their Engine::KNN clocks.  One
        # GPU: the drop-in run directly with stdout to a file, and as run_bench.sh:84 launches it
        # (mpiexec, stdout a pipe to the launcher, which writes the file).  P GPUs: rank 0 runs
        # the drop-in at P ranks through the node window (mpiexec -n P), the others wait.
        if comm.is_root:
            runs = ((("reference_contract", 1, "direct", a.contract_runs),
                     ("reference_contract_mpiexec", 1, "mpiexec", a.contract_runs)) if world == 1
                    else (("reference_contract_node", world, "mpiexec",
                           min(2, a.contract_runs)),))
            for key, P, launcher, nrun in runs:
                extra[key] = _contract_entry(a, Q, P, launcher, nrun)
        if world > 1:
            # the other ranks wait on the host (a GPU collective would keep a kernel spinning on
            # every other GPU the contract's processes use), sleeping between polls
            if a.ingress == "shm":
                inp.barrier(world, timeout_s=1800.0, idle_s=0.01)
            else:
                comm.barrier()
    if comm.is_root:
        value = Q / (ms / 1e3)
        line = {
            "metric": "samples/sec (whole node) on bench_4",
            "value": round(value, 1),
            "unit": "queries/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "warmup_steps_run": warm,
            "warmup_curve_ms": curve,
            "numa_node": Comm._numa,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "vs_student_engine_cpu_np4": round(value / BASELINE_QPS, 1),
            "dtype": "fp64",
            "screen": "none" if a.exact else "single-term fp16 MFMA screen (3-term escalation), "
                                             "exact fp64 re-rank (results bit-identical to the "
                                             "fp64 reference)",
            "data": "synthetic (generate_input.py distribution, seed 42; reference inputs absent)",
            "config": {
                "model": f"bench_4 exact k-NN classifier N={a.n_data} A={a.attrs} k={a.k} "
                         f"labels={a.labels}",
                "global_batch": Q,
                "seq_len": a.attrs,
                "parallelism": f"{a.strategy}{world}" + ("" if a.schedule == "static" else "-dynamic"),
                "num_data": a.n_data,
                "queries_per_gpu": a.q_per_gpu,
                "ingress": a.ingress,
                "k": a.k if kmin == kmax else f"{kmin}-{kmax}",
            },
        }
        line.update(extra)
        print(json.dumps(line), flush=True)
    if a.ingress == "shm":
        inp.close()
    eng.close()
    return 0


def _large_n(a, shapes=((1_000_000, 32), (1_000_000, 128)), q=16384, warmup=2, steps=5):
    """The native step on larger datasets than the headline's, one GPU: N x A per shape, q
    queries at the headline's k and labels, synthetic data of the generator's distribution.  The
    step picks its own render (the cost model: above 2^23 values the device render and the chunked
    screen pipeline) — per shape the mean ms of `steps` steps after `warmup`, and which render
    ran."""
    import torch
    from distributed_machine_learning_project_amd import _lib
    from distributed_machine_learning_project_amd.ops import knn as K
    from distributed_machine_learning_project_amd.utils.io import generate
    out = {}
    for N, A in shapes:
        inp = generate(N, q, A, 0.0, 1000.0, a.k, a.k, a.labels, seed=7)
        rep = torch.empty(int(_lib.lib().dmlp_format_bound(q)), dtype=torch.uint8).pin_memory().numpy()
        for _ in range(warmup):
            K.step(inp.X, inp.labels, (0, a.labels), inp.Qx, inp.k, report=rep)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            K.step(inp.X, inp.labels, (0, a.labels), inp.Qx, inp.k, report=rep)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
        out[f"N{N}_A{A}"] = {"ms_per_step": round(ms, 3), "queries": q, "k": a.k, "steps": steps,
                             "device_render": bool(K.pipeline_stats()["device_render"])}
        del inp, rep
    return out


def _cgroup_cpu_stat():
    """cgroup v2 cpu.stat counters of this process's cgroup (usage_usec, nr_throttled,
    throttled_usec), or {} when unreadable."""
    try:
        with open("/proc/self/cgroup") as f:
            rel = next((ln.split(":", 2)[2].strip() for ln in f if ln.startswith("0::")), None)
        for path in ([f"/sys/fs/cgroup{rel}/cpu.stat"] if rel else []) + [
                "/sys/fs/cgroup/cpu.stat", "/sys/fs/cgroup/cpu/cpu.stat"]:  # v2, then v1
            if os.path.exists(path):
                with open(path) as f:
                    d = {k: int(v) for k, v in (ln.split() for ln in f if len(ln.split()) == 2)}
                if "throttled_time" in d:  # v1: ns
                    d["throttled_usec"] = d["throttled_time"] // 1000
                return d
    except (OSError, ValueError, StopIteration):
        pass
    return {}


def _contract_entry(a, Q, P, launcher, nrun):
    """One reference-contract record for the bench JSON (never fatal: an error is recorded)."""
    try:
        t_c = time.perf_counter()
        res, src = _contract_runs(a, True, (("bench", Q),), nrun, 0, P=P, launcher=launcher)
        b = res["bench"]
        how = ("one process per run, stdout to a file" if launcher == "direct" else
               f"mpiexec -n {P} per run (run_bench.sh:84,120), stdout a pipe to the launcher "
               f"which writes a file")
        out = {"harness": f"engine.h drop-in + {src}, {how}", "ranks": P,
               "runs": b["runs"], "time_ms_median": b["time_ms_median"],
               "time_ms_min": b["time_ms_min"],
               "knn_ms_median": b.get("knn_ms_median"), "emit_ms_median": b.get("emit_ms_median"),
               "harness_time_taken_ms": b.get("harness_time_taken_ms"),
               "queries_per_s": round(Q / (b["time_ms_median"] / 1e3), 1),
               "wall_s": round(time.perf_counter() - t_c, 1)}
        for key in ("window", "stdout_fifo", "vmsplice_bytes"):
            if key in b:
                out[key] = b[key]
        return out
    except Exception as e:  # noqa: BLE001 — a diagnostic beside the headline, never fatal
        return {"error": str(e)[-300:], "ranks": P}


def _world_report(comm, host_plane, a):
    """What the process group really is: its size, the data plane, and (RCCL) one all-reduce
    whose result proves every rank took part."""
    import torch
    out = {"rccl_world": None, "data_plane": "none (1 rank)" if comm.world == 1 else None}
    if comm.world == 1:
        return out
    from distributed_machine_learning_project_amd.parallel import dist_api as dist
    out["rccl_world"] = dist.get_world_size()
    out["data_plane"] = ("RCCL over xGMI" if comm.backend == "nccl" else
                         "host-staged gloo (DMLP_DATA_PLANE=host rehearsal)"
                         if host_plane and comm.on_gpu else "gloo (CPU)")
    t = torch.ones(1, dtype=torch.float32, device=comm.device)
    dist.all_reduce(t)
    out["allreduce_check"] = int(t.item())
    # the farm's dataset replication (parallel/strategies.py probe_replication, untimed): every
    # GPU over its own PCIe link ("h2d") or 1/P each + an all-gather over xGMI ("xgmi")
    out["replication_probe"] = getattr(comm, "replication", None)
    from distributed_machine_learning_project_amd.parallel.strategies import replication_mode
    ingress = os.environ.get("KNN_DATA_INGRESS", "auto")
    out["replication_mode"] = (ingress if ingress != "auto" else
                               replication_mode(getattr(comm, "replication", None),
                                                a.n_data * a.attrs * 4))
    if out["allreduce_check"] != comm.world:
        raise RuntimeError(f"all-reduce of ones gave {out['allreduce_check']} on {comm.world} ranks")
    return out


def _diagnostics(comm, eng, step, n, my_ms, steps_native=None):
    """Untimed traced steps after the timed ones (the tracer syncs around every phase, so they
    never run inside the timed region): per rank the mean phase times, the host<->device bytes
    the pipeline issued and the collective bytes, gathered on rank 0 together with the
    rank-by-rank comparison of the collective sequence.  Every rank runs the same steps and the
    same one gather whatever happens locally: a rank whose own bookkeeping fails (timeline reads,
    summaries) reports the error in its row instead, and the sequence check is skipped.
    DMLP_DIAG_FAIL=<ranks>|all (tests): that bookkeeping fails on those ranks."""
    import torch
    from distributed_machine_learning_project_amd.ops import knn as K
    from distributed_machine_learning_project_amd.parallel import dist_api as dist
    err = []

    def local(f, *args):
        try:
            return f(*args)
        except Exception as e:  # noqa: BLE001
            err.append(f"{type(e).__name__}: {e}"[-300:])
            return None
    tr = eng.tracer
    # GPU-timestamped phase boundaries of the pipeline (hipEvents, no syncs) over n steps
    tl = []
    if comm.on_gpu:
        local(K.set_pipe_events, True)
        for _ in range(n + 1):
            step()
            tl.append(local(K.pipe_timeline) or [])
        local(K.set_pipe_events, False)
        tl = tl[1:]  # the first has no previous call to measure the gap from
    was = tr.enabled
    tr.enabled, tr.records = True, []
    K.io_bytes(reset=True)
    if comm.world > 1:
        dist.coll_log_start()
    import contextlib
    import io
    with contextlib.redirect_stderr(io.StringIO()):  # the tracer's per-phase lines
        for _ in range(n):
            step()
    comm.sync()
    log = dist.coll_log_stop() if comm.world > 1 else []
    tr.enabled = was

    def summary():
        inj = os.environ.get("DMLP_DIAG_FAIL", "")
        if inj == "all" or str(comm.rank) in inj.split(","):
            raise RuntimeError("injected diagnostics failure")
        phases = {}
        for name, v in tr.records:
            phases[name] = phases.get(name, 0.0) + v / n
        io_b = {k: v // n for k, v in K.io_bytes().items()}
        coll_b = {}
        for op, _, nb, _, _ in log:
            coll_b[op] = coll_b.get(op, 0) + nb // n
        timeline = {}
        for row in tl:
            for name, ms in row:
                timeline[name] = timeline.get(name, 0.0) + ms / max(1, len(tl))
        return {"rank": comm.rank, "device": str(comm.device), "numa_node": type(comm)._numa,
                "ms_per_step": round(my_ms, 4),
                "timed_native_step_calls": (steps_native or {}).get("calls"),
                "host_issue_ms_per_step": round((steps_native or {}).get("host_ms", 0.0) /
                                                max(1, (steps_native or {}).get("calls") or 1), 4),
                "host_threads": _host_threads(),
                "step_timeline_ms": {k: round(v, 4) for k, v in timeline.items()},
                "phases_ms": {k: round(v, 4) for k, v in phases.items()},
                "pcie_bytes_per_step": io_b, "collective_bytes_per_step": coll_b}
    mine = local(summary) or {"rank": comm.rank}
    if err:
        mine["error"] = err[0]
    rows = [mine]
    check = None
    if comm.world > 1:
        rows = [None] * comm.world
        torch.distributed.all_gather_object(rows, mine)
        if all("error" not in r for r in rows):
            check = dist.check_collective_sequence(log)
    if not comm.is_root:
        return {}
    out = {"per_rank": rows, "diag_steps": n}
    if check is not None:
        out["collective_check"] = check
        if not check["ok"]:
            print(f"[bench] collective sequences differ between ranks: {check['problems']}",
                  file=sys.stderr, flush=True)
    return out


def _host_threads():
    from distributed_machine_learning_project_amd import _lib
    return int(_lib.lib().dmlp_host_threads())


def _bench_native(a):
    """knn_engine through the reference's harness contract: the input text is written once
    (untimed), then each run is a fresh `mpiexec -n P knn_engine --input F` process that parses
    (untimed), builds the engine (untimed warm-up) and times KNN + report + barrier; the
    KNN_METRICS sidecar carries that time with microsecond resolution ("Time taken" on stderr is
    whole milliseconds).  --steps runs per config (median reported), --warmup runs discarded.
    Rank 0's stdout is checked byte-for-byte against the Python engine's CPU oracle for Q = 1000."""
    P = max(1, a.gpus)
    steps = a.steps if a.steps != 200 else 5  # one process per run: 5 by default
    res, harness_src = _contract_runs(a, a.harness == "dropin", (("bench", a.q_per_gpu * P),
                                                                  ("q1000", 1000)), steps, a.warmup)
    dropin = a.harness == "dropin"
    kmin = a.k if a.kmin is None else a.kmin
    _print_native(a, res, harness_src, dropin, P, steps, kmin)


def _contract_runs(a, dropin, shapes, steps, warmup, P=None, launcher="direct"):
    """Fresh processes through the reference contract at each (tag, Q) of shapes: the drop-in
    (engine.h + the reference's common.cpp) or knn_engine, at P ranks (default --gpus) — one
    rank run directly ("direct") or under mpiexec ("mpiexec", as run_bench.sh launches it: the
    engine's stdout is then a pipe to the launcher).  Returns ({tag: entry}, harness)."""
    import json as _json
    import statistics
    import subprocess
    import tempfile

    from distributed_machine_learning_project_amd import build
    from distributed_machine_learning_project_amd.utils.io import generate, write_input

    harness_src = None
    if dropin:
        # engine.h + dropin_engine.cpp linked with the reference's own common.cpp (its parse,
        # timing and reportResult through cout) when available, else tests/native/mini_harness.cpp
        # (the same contract re-implemented)
        out_exe = os.path.join(ROOT, "distributed_machine_learning_project_amd", "_build",
                               "engine_dropin")
        ref_common = build.reference_harness()
        if ref_common is not None:
            harness_src = "reference common.cpp"
            exe = build.build_dropin(str(ref_common), out=out_exe)
        else:
            harness_src = "tests/native/mini_harness.cpp"
            exe = build.build_dropin(os.path.join(ROOT, "tests", "native", "mini_harness.cpp"),
                                     out=out_exe,
                                     extra_flags=['-DDMLP_COMMON_HEADER="contract_types.h"'])
    else:
        exe = build.build_engine()
    P = max(1, a.gpus if P is None else P)
    mpi = P > 1 or launcher == "mpiexec"
    kmin = a.k if a.kmin is None else a.kmin
    kmax = max(kmin, a.k if a.kmax is None else a.kmax)
    res = {}
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        for tag, q in shapes:
            inp = generate(a.n_data, q, a.attrs, 0.0, 1000.0, kmin, kmax, a.labels, seed=42)
            path = os.path.join(td, f"{tag}.in")
            write_input(path, inp)
            times, out0, harness_ms, parts, extra_last = [], None, [], {}, {}
            for r in range(warmup + steps):
                met = os.path.join(td, f"{tag}_{r}.json")
                env = dict(os.environ, KNN_METRICS=met, KNN_STRATEGY=a.strategy,
                           KNN_INGRESS=a.ingress)  # shm: per-GPU ingress from a shared window
                cmd = ([] if not mpi else ["/opt/conda/bin/mpiexec", "-n", str(P)]) + [str(exe)]
                if dropin and mpi:  # each rank opens the input (MPICH stdin forwarding: H5)
                    import shlex
                    cmd = cmd[:-1] + ["sh", "-c", f"exec {shlex.quote(str(exe))} < "
                                                  f"{shlex.quote(path)}"]
                if not dropin:
                    cmd += ["--input", path]
                    if a.schedule == "dynamic":
                        cmd += ["--schedule", "dynamic"]
                # stdout to a file, as run_bench.sh redirects it (run_bench.sh:82-84): a pipe would
                # time this process's reader draining 6 MB of report, not the engine
                outp, errp = os.path.join(td, "out.txt"), os.path.join(td, "err.txt")
                with open(path, "rb") as fin, open(outp, "wb") as fo, open(errp, "wb") as fe:
                    rc = subprocess.run(cmd, stdin=fin if dropin and not mpi else None,
                                        stdout=fo, stderr=fe, env=env,
                                        timeout=600 if P == 1 else 300).returncode
                pr = subprocess.CompletedProcess(cmd, rc, open(outp, "rb").read(),
                                                 open(errp, "rb").read())
                if pr.returncode != 0:
                    raise RuntimeError(pr.stderr.decode()[-2000:])
                if r >= warmup:
                    # KNN_METRICS: the engine's own microsecond clock (the harness prints whole
                    # milliseconds; the drop-in's covers Engine::KNN, pack and report included)
                    with open(met) as f:
                        mj = _json.load(f)
                    times.append(float(mj["time_ms"]))
                    for key in ("pack_ms", "knn_ms", "emit_ms", "step_ms"):
                        if key in mj:
                            parts.setdefault(key, []).append(float(mj[key]))
                    for key in ("window", "stdout_fifo", "vmsplice_bytes"):  # (the last run's)
                        if key in mj:
                            extra_last[key] = mj[key]
                    for rk in range(1, P):  # the drop-in's node window: each rank's phases
                        rp = f"{met}.r{rk}"
                        if os.path.exists(rp):
                            with open(rp) as f:
                                rj = _json.load(f)
                            for key in ("step_ms", "fetch_ms", "fetch_rows_ms", "fetch_share_ms"):
                                if key in rj:
                                    parts.setdefault(f"rank{rk}_{key}", []).append(float(rj[key]))
                            if "fetch_rows_span" in rj:
                                extra_last[f"rank{rk}_fetch_rows_span"] = rj["fetch_rows_span"]
                    if dropin:
                        import re as _re
                        m = _re.search(rb"Time taken: (\d+) ms", pr.stderr)
                        harness_ms.append(int(m.group(1)))
                out0 = pr.stdout
            entry = {"Q": q, "time_ms_median": round(statistics.median(times), 3),
                     "time_ms_min": round(min(times), 3), "runs": len(times)}
            if harness_ms:
                entry["harness_time_taken_ms"] = harness_ms
            entry.update(extra_last)
            for key, v in parts.items():
                entry[key + "_median"] = round(statistics.median(v), 3)
            if tag == "q1000":
                from distributed_machine_learning_project_amd.ops import knn as K
                from distributed_machine_learning_project_amd.utils.io import format_report
                _, i = K.knn_cpu(inp.X, inp.Qx, inp.k)
                _, cs = K.finalize_cpu(i, inp.k, inp.labels)
                entry["verify_ok"] = bytes(out0) == format_report(cs)
            res[tag] = entry
    return res, harness_src


def _print_native(a, res, harness_src, dropin, P, steps, kmin):
    ms = res["bench"]["time_ms_median"]
    Q = res["bench"]["Q"]
    value = Q / (ms / 1e3)
    line = {
        "metric": "samples/sec (whole node) on bench_4", "value": round(value, 1),
        "unit": "queries/s", "n_gpus": P, "steps": steps, "warmup": a.warmup,
        "ms_per_step": ms, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "vs_student_engine_cpu_np4": round(value / BASELINE_QPS, 1),
        "dtype": "fp64",
        "harness": (f"engine.h drop-in linked with {harness_src} (AoS pack + KNN + report to "
                    "cout; time = Engine::KNN on the engine's clock, the harness's whole-ms "
                    "'Time taken' alongside)" if dropin else
                    "native knn_engine (reference contract: Time taken = KNN + report + barrier)"),
        "data": "synthetic (generate_input.py distribution, seed 42; reference inputs absent)",
        "config": {"model": f"bench_4 exact k-NN classifier N={a.n_data} A={a.attrs} "
                            f"k={a.k if a.kmax is None or kmin == a.kmax else f'{kmin}-{a.kmax}'} "
                            f"labels={a.labels}",
                   "global_batch": Q, "seq_len": a.attrs,
                   "parallelism": f"{a.strategy}{P}", "num_data": a.n_data},
        "q1000": res["q1000"], "bench_runs": res["bench"],
    }
    print(json.dumps(line), flush=True)


def _allreduce_busbw(comm, nbytes=256 << 20, iters=10):
    """RCCL all-reduce bus bandwidth over xGMI (the BASELINE metric's second half; the k-NN
    itself needs no all-reduce).  busbw = bytes * 2(P-1)/P / time."""
    import torch
    import torch.distributed as dist
    x = torch.ones(nbytes // 4, dtype=torch.float32, device=comm.device)
    for _ in range(3):
        dist.all_reduce(x)
    comm.sync()
    t0 = time.perf_counter()
    for _ in range(iters):
        dist.all_reduce(x)
    comm.sync()
    dt = (time.perf_counter() - t0) / iters
    P = comm.world
    return nbytes * 2 * (P - 1) / P / dt / 1e9


if __name__ == "__main__":
    sys.exit(main())
