"""Multi-rank GPU data plane on ONE MI355X (SURVEY.md §4 level 4).

Several ranks share cuda:0, which RCCL refuses, so the data plane is host-staged: gloo over
host copies of the device tensors in the Python front end (DMLP_DATA_PLANE=host,
parallel/dist_api.py) and blocking MPI point-to-point over host copies in knn_engine
(KNN_DATA_PLANE=host, engine_core.h).  Everything else is the production multi-rank code on the
real HIP kernels: partitions, offsets, the x1 / 3-term screens, K4 merge kernels, the binomial
tree, the ring, the grid's column merge, the dynamic farm.  Output bytes must equal the NumPy
fp64 oracle's; knn_engine additionally checks that every send has a matching receive of the
same size (KNN_P2P_CHECK=1, logged per rank and compared on rank 0).
References: bench_2 @0xc844 (tree reduce), engine.cpp:283-309 (grid merge), bench_4 @0xd80c.
"""
import os
import socket
import subprocess
import sys

import pytest

import distributed_machine_learning_project_amd as dmlp
from distributed_machine_learning_project_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MPIEXEC = "/opt/conda/bin/mpiexec"
ENGINE = os.path.join(ROOT, "distributed_machine_learning_project_amd", "knn_engine")


def _port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


@pytest.fixture(scope="module")
def case(tmp_path_factory):
    """k in 1..40: the single-term x1 class (k <= 32) and the 3-term LDS class in one input."""
    d = tmp_path_factory.mktemp("mr")
    txt = dmlp.generate_text(3000, 301, 16, 0, 1000, 1, 40, 5, seed=11)
    p = d / "mr.in"
    p.write_text(txt)
    inp = dmlp.parse_input(txt)
    _, _, cs = ref.knn(inp.X, inp.labels, inp.Qx, inp.k)
    return str(p), ref.report_lines(cs).encode()


def _python(path, np_, strategy, env_extra=None):
    # DMLP_COLL_CHECK: every rank logs its collective sequence (parallel/dist_api.py) and the
    # harness compares them on rank 0 after the timed call (exit 3 on any divergence)
    env = dict(os.environ, PYTHONPATH=ROOT, DMLP_DATA_PLANE="host", OMP_NUM_THREADS="2",
               DMLP_COLL_CHECK="1")
    env.update(env_extra or {})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node",
           str(np_), "--master-addr", "127.0.0.1", "--master-port", str(_port()), "-m",
           "distributed_machine_learning_project_amd.harness", "--strategy", strategy,
           "--device", "gpu", "--input", path]
    r = subprocess.run(cmd, capture_output=True, env=env, timeout=180, cwd=ROOT)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    assert b"[dmlp-coll] ok=True" in r.stderr, r.stderr.decode()[-2000:]
    return r.stdout


@pytest.mark.parametrize("strategy", ["farm", "shard_gather", "shard_reduce", "grid2d", "ring"])
@pytest.mark.parametrize("np_", [2, 3])
def test_python_front_end(case, strategy, np_):
    path, expect = case
    assert _python(path, np_, strategy) == expect


def test_python_dynamic_farm_and_shm_ingress(case):
    path, expect = case
    assert _python(path, 3, "farm", {"KNN_SCHEDULE": "dynamic"}) == expect
    assert _python(path, 2, "farm", {"KNN_INGRESS": "shm"}) == expect


@pytest.mark.parametrize("np_", [2, 3])
def test_python_dynamic_farm_shared_counter(case, np_):
    """Chunks claimed by an atomic fetch-and-add in the node-shared segment (utils/shm.py),
    results written back into it; 7 chunks per rank so ranks interleave."""
    path, expect = case
    env = {"KNN_INGRESS": "shm", "KNN_SCHEDULE": "dynamic", "KNN_CHUNKS_PER_RANK": "7"}
    assert _python(path, np_, "farm", env) == expect


def _native(path, np_, strategy, extra=(), env_extra=None, want_err=False):
    if not os.path.exists(ENGINE):
        pytest.skip("knn_engine not built")
    if not os.path.exists(MPIEXEC):
        pytest.skip("no mpiexec")
    env = dict(os.environ, KNN_DATA_PLANE="host", KNN_P2P_CHECK="1", KNN_POOL_MB="256",
               KNN_HOST_POOL_MB="64")
    env.update(env_extra or {})
    cmd = [MPIEXEC, "-n", str(np_), ENGINE, "--strategy", strategy, "--input", path, *extra]
    r = subprocess.run(cmd, capture_output=True, env=env, timeout=180, cwd=ROOT)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    assert b"p2p check OK" in r.stderr, r.stderr.decode()[-2000:]
    return (r.stdout, r.stderr) if want_err else r.stdout


@pytest.mark.parametrize("strategy", ["farm", "shard_gather", "shard_reduce", "grid2d", "ring"])
@pytest.mark.parametrize("np_", [2, 3])
def test_native_front_end(case, strategy, np_):
    path, expect = case
    assert _native(path, np_, strategy) == expect


@pytest.mark.parametrize("np_", [2, 3])
def test_native_dynamic_farm(case, np_):
    """knn_engine --schedule dynamic: chunks claimed by MPI_Fetch_and_op on rank 0's window."""
    path, expect = case
    env_save = os.environ.get("KNN_CHUNKS_PER_RANK")
    os.environ["KNN_CHUNKS_PER_RANK"] = "7"
    try:
        assert _native(path, np_, "farm", ("--schedule", "dynamic")) == expect
    finally:
        if env_save is None:
            os.environ.pop("KNN_CHUNKS_PER_RANK")
        else:
            os.environ["KNN_CHUNKS_PER_RANK"] = env_save


def test_native_ring_debug_listing(case):
    """knn_engine --strategy ring --debug (lists gathered to rank 0) == the serial listing."""
    path, _ = case
    ring = _native(path, 3, "ring", ("--debug",))
    env = dict(os.environ)
    r = subprocess.run([ENGINE, "--strategy", "serial", "--debug", "--input", path],
                       capture_output=True, env=env, timeout=180, cwd=ROOT)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    assert ring == r.stdout


@pytest.mark.parametrize("np_", [1, 2, 3])
def test_native_out_of_core_farm(case, np_):
    """KNN_MAX_DEVICE_ROWS=700 (N=3000 -> 5 chunks): rank 0 streams double-buffered chunks,
    each broadcast; running lists merged per chunk; == oracle bytes (and the DEBUG listing)."""
    path, expect = case
    env = {"KNN_MAX_DEVICE_ROWS": "700"}
    assert _native(path, np_, "farm", env_extra=env) == expect
    if np_ == 2:
        dbg = _native(path, 2, "farm", ("--debug",), env_extra=env)
        r = subprocess.run([ENGINE, "--strategy", "serial", "--debug", "--input", path],
                           capture_output=True, timeout=180, cwd=ROOT)
        assert dbg == r.stdout


@pytest.fixture(scope="module")
def case_x1(tmp_path_factory):
    """k in 1..32 (every query on the single-term screen, so the host-ops pipeline runs) and
    N = 3000 -> 47 tiles: uneven per-rank image shards at np 2 and 3.  Plus the same input with
    one point outside the screen's range (|x| > 1e15) in the LAST rank's shard."""
    d = tmp_path_factory.mktemp("mrx1")
    inp = dmlp.parse_input(dmlp.generate_text(3000, 301, 16, 0, 1000, 1, 32, 5, seed=12))
    out = []
    for tag, big in (("ok", False), ("bad", True)):
        if big:
            inp.X[2990, 3] = 3.0e15
        p = d / f"{tag}.in"
        p.write_text(dmlp.to_text(inp))
        _, _, cs = ref.knn(inp.X, inp.labels, inp.Qx, inp.k)
        out.append((str(p), ref.report_lines(cs).encode()))
    return out


@pytest.mark.parametrize("np_", [2, 3])
def test_python_shared_step_farm(case_x1, np_):
    """Static farm over the node-shared segment: each rank runs libdmlp's native step on its own
    query block straight from the segment, keeps its report lines on its GPU and copies them to
    its byte offset in the segment (lengths through the segment's slots) == oracle bytes; with
    out-of-range data each rank's step takes the device-image path by itself (no collective);
    KNN_DATA_INGRESS=allgather (fp64 replica all-gathered over the data plane, then the
    device-rows pipeline) == oracle bytes too."""
    (path, expect), (bad_path, bad_expect) = case_x1
    env = {"KNN_INGRESS": "shm"}
    assert _python(path, np_, "farm", env) == expect
    assert _python(bad_path, np_, "farm", env) == bad_expect
    assert _python(path, np_, "farm", dict(env, KNN_DATA_INGRESS="allgather")) == expect
    # the xGMI replica: each rank ships 1/P of the int32 rows, one all-gather completes them
    # (here over the host-staged plane), the native step renders from the device replica
    assert _python(path, np_, "farm", dict(env, KNN_DATA_INGRESS="xgmi")) == expect
    assert _python(bad_path, np_, "farm", dict(env, KNN_DATA_INGRESS="xgmi")) == bad_expect


@pytest.mark.parametrize("np_", [2, 3])
def test_native_shared_ingress_farm(case, case_x1, np_):
    """knn_engine KNN_INGRESS=shm: the parsed input in an MPI-3 node-shared window, every rank
    runs the library's native step on its own query block over its own link and writes its
    report lines into the window (one 8-byte all-gather of the lengths); out-of-range data and
    k > 32 stay in the step too (device-image path / two-pass screen).  == oracle bytes in all
    cases, and the general farm (its "distribute" phase) never runs."""
    (path, expect), (bad_path, bad_expect) = case_x1
    env = {"KNN_INGRESS": "shm", "KNN_TRACE": "1"}
    for p, e in ((path, expect), (bad_path, bad_expect), case):
        out, err = _native(p, np_, "farm", env_extra=env, want_err=True)
        assert out == e
        for r in range(np_):  # the step ran on every rank
            assert f"rank {r} step ".encode() in err, err.decode()[-2000:]
        assert b"distribute" not in err


@pytest.mark.parametrize("np_", [2, 3])
def test_bench_self_launch_rehearsal(np_):
    """bench.py --gpus N launches its own N ranks (no torchrun in front of it) and reports the
    process group it really had; on one GPU the ranks share it over the host-staged plane.
    The whole rank-0 report is checked against the fp64 oracle (--verify) and the ranks'
    collective sequences are compared (root ingress: broadcast + scatter + gather)."""
    import json
    env = dict(os.environ, DMLP_DATA_PLANE="host", OMP_NUM_THREADS="2")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(np_), "--steps", "3",
           "--warmup", "1", "--min-warmup-s", "0", "--n-data", "20000", "--q-per-gpu", "2048",
           "--verify", "--ingress", "root", "--no-busbw"]
    r = subprocess.run(cmd, capture_output=True, env=env, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    res = json.loads(r.stdout.decode().strip().splitlines()[-1])
    assert res["n_gpus"] == np_ and res["rccl_world"] == np_
    assert res["verify_ok"] and res["allreduce_check"] == np_
    assert res["collective_check"]["ok"]
    assert len(res["per_rank"]) == np_
    assert all(c > 0 for c in res["collective_check"]["calls_per_rank"])


def test_bench_driver_path_eight_ranks():
    """The driver's N = 8 command line in miniature: bench.py --gpus 8 (its default node-shared
    ingress, the node render plane with 8 renderers, the native step on every rank) on the one
    GPU over the host-staged plane, small Q, --verify of the whole report against the fp64
    oracle; the JSON reports 8 ranks and every rank's row."""
    import json
    env = dict(os.environ, DMLP_DATA_PLANE="host", OMP_NUM_THREADS="2", DMLP_HOST_THREADS="2",
               DMLP_BENCH_CONTRACT_RUNS="0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "3",
           "--warmup", "1", "--min-warmup-s", "0", "--n-data", "20000", "--q-per-gpu", "2048",
           "--verify", "--no-busbw"]
    r = subprocess.run(cmd, capture_output=True, env=env, timeout=400, cwd=ROOT)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    res = json.loads(r.stdout.decode().strip().splitlines()[-1])
    assert res["n_gpus"] == 8 and res["verify_ok"]
    assert len(res["per_rank"]) == 8


# ---------------------------------------------------------------- wider worlds: P = 4 (2x2) and 8 (4x2)
@pytest.mark.parametrize("strategy", ["farm", "grid2d", "shard_reduce", "shard_gather", "ring"])
@pytest.mark.parametrize("np_", [4, 8])
def test_native_front_end_wide(case, strategy, np_):
    """knn_engine at the world sizes the target node runs: P = 4 makes
    grid2d a 2 x 2 grid and P = 8 a 4 x 2 grid (column split, column merge, row-0 gather with
    C > 1); 8 ranks share the one GPU over the host-staged plane.  == oracle bytes, every send
    matched by a receive."""
    path, expect = case
    env = {"KNN_POOL_MB": "128", "KNN_HOST_POOL_MB": "32", "DMLP_HOST_THREADS": "2"}
    assert _native(path, np_, strategy, env_extra=env) == expect


@pytest.mark.parametrize("np_", [4, 8])
def test_native_shared_farm_wide(case_x1, np_):
    """knn_engine KNN_INGRESS=shm at P = 4 / 8: every rank's native step, the dataset's image and
    rows rendered once for the node through the render plane (1/P per rank), == oracle bytes;
    with the plane off (KNN_PLANE=0: every rank renders everything) the same bytes."""
    (path, expect), (bad_path, bad_expect) = case_x1
    env = {"KNN_INGRESS": "shm", "KNN_TRACE": "1", "KNN_POOL_MB": "128", "KNN_HOST_POOL_MB": "32",
           "DMLP_HOST_THREADS": "2"}
    out, err = _native(path, np_, "farm", env_extra=env, want_err=True)
    assert out == expect
    for r in range(np_):
        assert f"rank {r} step ".encode() in err, err.decode()[-2000:]
    assert _native(bad_path, np_, "farm", env_extra=env) == bad_expect
    assert _native(path, np_, "farm", env_extra=dict(env, KNN_PLANE="0")) == expect


@pytest.mark.parametrize("np_", [4])
@pytest.mark.parametrize("strategy", ["farm", "grid2d"])
def test_python_front_end_wide(case, case_x1, strategy, np_):
    path, expect = case
    env = {"DMLP_HOST_THREADS": "2"}
    assert _python(path, np_, strategy, env) == expect
    if strategy == "farm":  # the node-shared farm with the render plane at P = 4
        (p1, e1), _ = case_x1
        assert _python(p1, np_, "farm", dict(env, KNN_INGRESS="shm")) == e1


# ---------------------------------------------------------------- the engine.h drop-in at P > 1
@pytest.fixture(scope="module")
def dropin_exe(tmp_path_factory):
    from distributed_machine_learning_project_amd import build
    d = tmp_path_factory.mktemp("dropin")
    ref_common = build.reference_harness()
    try:
        if ref_common is not None:
            return str(build.build_dropin(str(ref_common), str(d / "engine")))
        return str(build.build_dropin(os.path.join(ROOT, "tests", "native", "mini_harness.cpp"),
                                      str(d / "engine"),
                                      extra_flags=['-DDMLP_COMMON_HEADER="contract_types.h"']))
    except RuntimeError as e:
        pytest.skip(f"drop-in build unavailable: {e}")


@pytest.fixture(scope="module")
def case_dec9(tmp_path_factory):
    """9-decimal attributes: no lossless int32 rows, so the render plane ships fp64 rows."""
    import numpy as np
    d = tmp_path_factory.mktemp("dec9")
    rng = np.random.default_rng(5)
    N, Q, A = 3000, 301, 16
    X, Qx = rng.uniform(0, 1000, (N, A)), rng.uniform(0, 1000, (Q, A))
    k = rng.integers(1, 33, Q).astype(np.int32)
    labels = rng.integers(0, 5, N).astype(np.int32)
    lines = [f"{N} {Q} {A}"]
    lines += [f"{int(l)} " + " ".join("%.9f" % v for v in row) for l, row in zip(labels, X)]
    lines += [f"Q {int(kk)} " + " ".join("%.9f" % v for v in row) for kk, row in zip(k, Qx)]
    txt = "\n".join(lines) + "\n"
    p = d / "dec9.in"
    p.write_text(txt)
    inp = dmlp.parse_input(txt)
    _, _, cs = ref.knn(inp.X, inp.labels, inp.Qx, inp.k)
    return str(p), ref.report_lines(cs).encode()


def _dropin_run(exe, path, np_, env_extra=None):
    import shlex
    env = dict(os.environ, KNN_DATA_PLANE="host", KNN_TRACE="1", KNN_POOL_MB="128",
               KNN_HOST_POOL_MB="32", KNN_WINDOW_MB="8", DMLP_HOST_THREADS="2")
    env.update(env_extra or {})
    cmd = [MPIEXEC, "-n", str(np_), "sh", "-c", f"exec {shlex.quote(exe)} < {shlex.quote(path)}"]
    r = subprocess.run(cmd, stdin=subprocess.DEVNULL, capture_output=True, env=env, timeout=180,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    return r.stdout, r.stderr.decode()


@pytest.mark.parametrize("np_", [2, 3, 4, 8])
def test_dropin_node_window_gpu(dropin_exe, case, case_x1, case_dec9, np_):
    """The reference's own common.cpp + the drop-in at P > 1 (run_bench.sh config 4's
    `mpirun ./engine < input`): the node window joined in the MPI_Init hook, rank 0's labels / k /
    query rows in it, rank 0's native step rendering the dataset into the render plane from the
    harness's vectors, EVERY rank's native step on its own block ([dmlp-step] rank r), report
    lines through the window.  Inputs: k 1-40 (two screen classes), k 1-32 with an out-of-range
    point (the device-image path), 9-decimal data (fp64 rows through the plane); the 8 MiB
    window grows on first use; P = 8 is the target node's world size (eight ranks on the one
    GPU here).  stdout == the fp64 oracle's bytes."""
    (p1, e1), (p2, e2) = case_x1
    for path, expect in (case, (p1, e1), (p2, e2), case_dec9):
        out, err = _dropin_run(dropin_exe, path, np_)
        assert out == expect, err[-2000:]
        for r in range(np_):
            assert f"[dmlp-step] rank {r} path" in err, err[-2000:]
        assert "[dmlp-trace] rank 0 window" in err
