"""Multi-process strategy tests on CPU (gloo), SURVEY.md §4 levels 3-5: every strategy, several
(non-square, non-power-of-two) world sizes, the §2.2 defect scenarios (varying k, duplicate
points, N/P < k shards, Q < P, k = N), byte-identical stdout against the NumPy oracle, each
query printed exactly once in id order."""
import os
import subprocess
import sys

import numpy as np
import pytest

import distributed_machine_learning_project_amd as dmlp
from distributed_machine_learning_project_amd.ops import reference as ref

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    """A port the OS just handed out (safe under pytest-xdist, unlike a counter)."""
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _oracle_report(inp):
    _, _, cs = ref.knn(inp.X, inp.labels, inp.Qx, inp.k)
    return ref.report_lines(cs).encode()


def _run(path, np_, strategy, extra=(), env_extra=None):
    # DMLP_COLL_CHECK: the harness compares every rank's collective sequence on rank 0
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", DMLP_COLL_CHECK="1")
    env.update(env_extra or {})
    if np_ == 1:
        cmd = [sys.executable, "-m", "distributed_machine_learning_project_amd.harness"]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node",
               str(np_), "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "-m",
               "distributed_machine_learning_project_amd.harness"]
    cmd += ["--strategy", strategy, "--device", "cpu", "--input", path, *extra]
    r = subprocess.run(cmd, capture_output=True, env=env, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    assert b"Time taken:" in r.stderr
    if np_ > 1:
        assert b"[dmlp-coll] ok=True" in r.stderr, r.stderr.decode()[-2000:]
    return r.stdout


@pytest.fixture(scope="module")
def workload(tmp_path_factory):
    d = tmp_path_factory.mktemp("knn")
    txt = dmlp.generate_text(257, 23, 6, 0, 100, 1, 40, 5, seed=7)  # varying k (D2)
    p = d / "gen.in"
    p.write_text(txt)
    inp = dmlp.parse_input(txt)
    return str(p), _oracle_report(inp)


@pytest.mark.parametrize("strategy", ["farm", "shard_gather", "shard_reduce", "grid2d", "serial",
                                      "ring"])
@pytest.mark.parametrize("np_", [1, 2, 3])
def test_strategy_matches_oracle(workload, strategy, np_):
    path, expect = workload
    assert _run(path, np_, strategy) == expect


@pytest.mark.parametrize("strategy", ["grid2d", "shard_gather", "shard_reduce", "ring"])
def test_four_and_six_ranks(workload, strategy):
    path, expect = workload
    assert _run(path, 4, strategy) == expect
    assert _run(path, 6, strategy) == expect  # non-square grid (D1: heap overflow in engine.cpp)


@pytest.mark.parametrize("strategy", ["farm", "shard_gather", "shard_reduce", "grid2d", "serial",
                                      "ring"])
def test_eight_ranks(workload, strategy):
    """World size 8, the MI355X node's GPU count: grid2d is a 4 x 2 grid
    (MPI_Dims_create), shards of 32 points against k up to 40 (N/P < k, defect D4), Q = 23 over 8
    ranks; the dynamic farm at 8 claims from the shared counter."""
    path, expect = workload
    assert _run(path, 8, strategy) == expect
    if strategy == "farm":
        assert _run(path, 8, "farm", env_extra={"KNN_SCHEDULE": "dynamic"}) == expect


def test_dynamic_farm(workload):
    path, expect = workload
    assert _run(path, 3, "farm", env_extra={"KNN_SCHEDULE": "dynamic"}) == expect


@pytest.mark.parametrize("schedule", ["static", "dynamic"])
def test_shared_ingress_farm(workload, schedule):
    """Node-shared input segment (utils/shm.py): every rank copies its own query block."""
    path, expect = workload
    env = {"KNN_INGRESS": "shm", "KNN_SCHEDULE": schedule}
    assert _run(path, 3, "farm", env_extra=env) == expect
    assert _run(path, 1, "farm", env_extra=env) == expect


@pytest.mark.parametrize("data_ingress", ["allgather", "h2d", "bcast"])
def test_shared_ingress_dataset_modes(workload, data_ingress):
    """Replicated dataset over the node-shared segment: sharded H2D + all-gather (uneven
    row blocks at P = 3), full per-rank H2D, or root H2D + broadcast."""
    path, expect = workload
    env = {"KNN_INGRESS": "shm", "KNN_DATA_INGRESS": data_ingress}
    assert _run(path, 3, "farm", env_extra=env) == expect


@pytest.mark.parametrize("np_", [1, 2])
def test_out_of_core_farm(workload, np_):
    """Dataset larger than the device budget (KNN_MAX_DEVICE_ROWS): streamed from the node-
    shared segment in 50-row chunks, running top-k lists merged after every chunk."""
    path, expect = workload
    env = {"KNN_INGRESS": "shm", "KNN_MAX_DEVICE_ROWS": "50"}
    assert _run(path, np_, "farm", env_extra=env) == expect


def test_shared_ingress_other_strategies(workload):
    path, expect = workload
    for strategy in ("shard_reduce", "grid2d", "ring"):
        assert _run(path, 2, strategy, env_extra={"KNN_INGRESS": "shm"}) == expect


def test_edge_cases(tmp_path):
    """Duplicates (ties broken by larger id), shards smaller than k (D4), Q < P, k = N."""
    rng = np.random.default_rng(3)
    base = np.round(rng.uniform(0, 3, size=(6, 3)), 0)
    X = np.ascontiguousarray(base[rng.integers(0, 6, size=20)])
    labels = rng.integers(0, 3, size=20).astype(np.int32)
    Qx = np.round(rng.uniform(0, 3, size=(2, 3)), 0)
    k = np.array([20, 13], np.int32)  # k = N and k > N/P
    inp = dmlp.KNNInput(labels, X, k, Qx)
    p = tmp_path / "edge.in"
    p.write_text(dmlp.to_text(inp))
    expect = _oracle_report(dmlp.parse_input(p.read_text()))
    for s in ["farm", "shard_gather", "shard_reduce", "grid2d", "ring"]:
        assert _run(str(p), 4, s) == expect, s


def test_debug_output(workload):
    """DEBUG build listing (common.cpp:72-78) from every strategy is identical."""
    path, _ = workload
    outs = {s: _run(path, 2, s, extra=["--debug"])
            for s in ["farm", "shard_reduce", "grid2d", "ring"]}
    assert len(set(outs.values())) == 1
    first = list(outs.values())[0].decode().splitlines()
    assert first[0].startswith("Label for Query 0 : ")
    assert first[1].startswith("Top-")


def test_dynamic_shared_farm_many_calls():
    """the dynamic farm over the node-shared segment keeps its call generation in the
    segment, so five calls through two Engines on one segment each compute every query exactly
    once (per-rank claimed counts add up to Q) and print the oracle's bytes."""
    import json
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", KNN_CHUNKS_PER_RANK="3")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "3",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "helpers", "dyn_multicall.py")]
    r = subprocess.run(cmd, capture_output=True, env=env, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    res = json.loads(r.stdout.decode().strip().splitlines()[-1])
    assert len(res["calls"]) == 5
    for c in res["calls"]:
        assert c["ok"]
        assert sum(c["claimed"]) == res["Q"], c


def _segment_worker(path, rank, world, rounds, q):
    from distributed_machine_learning_project_amd.utils.shm import SharedInput
    s = SharedInput.attach(path)
    seen = []
    for r in range(rounds):
        s.slots[rank] = 1000 * r + rank   # a value per rank and round
        s.barrier(world)
        seen.append([int(v) for v in s.slots[:world]])
        s.barrier(world)                  # nobody overwrites a slot before everyone read it
    q.put((rank, seen))


def test_segment_barrier_and_slots(tmp_path):
    """The node-shared segment's control plane (utils/shm.py): per-rank slots published before
    a barrier are seen by every rank after it, round after round (the static farm's report
    lengths); 4 processes, 25 rounds."""
    import multiprocessing as mp
    from distributed_machine_learning_project_amd.utils.io import generate
    from distributed_machine_learning_project_amd.utils.shm import SharedInput
    s = SharedInput.create(generate(64, 16, 4, 0.0, 1.0, 1, 4, 3, seed=1), directory=str(tmp_path))
    world, rounds = 4, 25
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_segment_worker, args=(s.path, r, world, rounds, q))
          for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    s.close()
    for rank in range(world):
        for r, row in enumerate(got[rank]):
            assert row == [1000 * r + i for i in range(world)]


def test_segment_plane_only_when_shared(tmp_path):
    """The node-shared segment reserves the render plane only when asked (P > 1 with the plane on,
    utils/shm.py share_input): a one-rank segment is the plane's bytes smaller and hands out no
    plane; an attach reads the flag from the header and lays the segment out the same way."""
    from distributed_machine_learning_project_amd.utils import shm
    from distributed_machine_learning_project_amd.utils.io import generate
    inp = generate(4096, 64, 32, 0.0, 1.0, 1, 8, 5, seed=4)
    plain = shm.SharedInput.create(inp, directory=str(tmp_path))
    shared = shm.SharedInput.create(inp, directory=str(tmp_path), plane=True)
    pb = shm._plane_bytes(4096, 32)
    assert pb > 0 and shared.nbytes - plain.nbytes == shm._up(pb) - shm._ALIGN  # (a 1-page stub)
    assert plain.plane(0, 2) is None
    for s in (shared, shm.SharedInput.attach(shared.path)):
        assert s._plane_bytes == pb and s.plane(0, 2) is not None
        assert np.array_equal(s.X, inp.X) and np.array_equal(s.k, inp.k)
    assert shm.SharedInput.attach(plain.path)._plane_bytes == 0
    plain.close()
    shared.close()


def test_segment_numa_placement(tmp_path, monkeypatch):
    """NUMA placement of the node-shared segment (utils/shm.py _place/_mbind) is best effort and
    never changes what is stored: a segment created with per-block query nodes holds the same
    bytes as one created without, and an attach sees them.  Also: KNN_NUMA_BIND=0 turns the
    per-rank binding off (parallel/comm.py Comm.bind_numa) and _mbind refuses empty / huge masks."""
    from distributed_machine_learning_project_amd.parallel.comm import Comm
    from distributed_machine_learning_project_amd.utils import shm
    from distributed_machine_learning_project_amd.utils.io import generate
    inp = generate(2048, 3000, 16, 0.0, 1.0, 1, 8, 5, seed=3)
    (tmp_path / "a").mkdir()
    (tmp_path / "b").mkdir()
    plain = shm.SharedInput.create(inp, directory=str(tmp_path / "a"))
    placed = shm.SharedInput.create(inp, directory=str(tmp_path / "b"),
                                    query_nodes=[(0, 1500, 0), (1500, 3000, 0)])
    again = shm.SharedInput.attach(placed.path)
    for s in (placed, again):
        assert s.N == plain.N and s.Q == plain.Q and s.A == plain.A
        for name in ("X", "labels", "Qx", "k"):
            assert np.array_equal(getattr(s, name), getattr(plain, name)), name
    for s in (again, placed, plain):
        s.close()
    buf = np.zeros(1 << 16, np.uint8)
    assert not shm._mbind(buf.ctypes.data, buf.nbytes, [], 2)
    assert not shm._mbind(buf.ctypes.data, buf.nbytes, [64], 2)
    monkeypatch.setenv("KNN_NUMA_BIND", "0")
    assert Comm.bind_numa(0) == -1


def _bench(args, env_extra=None):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args],
                          capture_output=True, env=env, timeout=300, cwd=ROOT)


def test_bench_refuses_missing_gpus():
    """`bench.py --gpus 2` must not silently bench one rank: with fewer GPUs
    than asked (none here) and no host-plane rehearsal it exits non-zero with a message."""
    r = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0"],
               {"DMLP_DATA_PLANE": ""})
    assert r.returncode != 0
    assert b"GPU(s) visible" in r.stderr
    assert not r.stdout.strip()


@pytest.mark.parametrize("ingress", ["shm", "root"])
def test_bench_launches_its_ranks(ingress):
    """`bench.py --gpus 3` with no torchrun in front launches 3 ranks itself (here on gloo/CPU:
    DMLP_DATA_PLANE=host allows fewer devices than ranks); rank 0's JSON reports the real world
    size, per-rank rows, an identical collective sequence on every rank, and a whole-report
    verify against the oracle."""
    import json
    r = _bench(["--gpus", "3", "--steps", "2", "--warmup", "1", "--min-warmup-s", "0",
                "--n-data", "1500", "--q-per-gpu", "200", "--verify", "--ingress", ingress],
               {"DMLP_DATA_PLANE": "host"})
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    res = json.loads(r.stdout.decode().strip().splitlines()[-1])
    assert res["n_gpus"] == 3 and res["rccl_world"] == 3 and res["allreduce_check"] == 3
    assert res["verify_ok"] and res["vs_baseline"] is None
    assert [row["rank"] for row in res["per_rank"]] == [0, 1, 2]
    assert res["collective_check"]["ok"]
    if ingress == "root":  # broadcast / scatter / gather on every rank
        assert all(c > 0 for c in res["collective_check"]["calls_per_rank"])
    # the timed steps' spread and the warm-up curve travel with the mean
    ts = res["timed_step_ms"]
    assert 0 < ts["p10"] <= ts["p50"] <= ts["p90"] <= ts["max"]
    assert isinstance(res["warmup_curve_ms"], list)


@pytest.mark.parametrize("inject", ["1", "all"])
def test_bench_survives_replication_probe_failure(inject):
    """the replication probe run at Engine construction (P > 1) must not cost
    the headline line when it fails — on one rank before its first collective, or on every rank —
    at np 3: every rank agrees on the failure, takes the "h2d" replication, and rank 0's JSON
    carries the probe's error beside a valid, verified headline."""
    import json
    r = _bench(["--gpus", "3", "--steps", "2", "--warmup", "1", "--min-warmup-s", "0",
                "--n-data", "1500", "--q-per-gpu", "200", "--verify", "--diag-steps", "0"],
               {"DMLP_DATA_PLANE": "host", "DMLP_PROBE_FAIL": inject})
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    res = json.loads(r.stdout.decode().strip().splitlines()[-1])
    assert res["n_gpus"] == 3 and res["verify_ok"] and res["value"] > 0
    assert "error" in res["replication_probe"] and res["replication_probe"]["mode"] == "h2d"
    assert res["replication_mode"] == "h2d"


def test_bench_survives_diagnostics_failure():
    """The untimed diagnostic steps after the timed ones (per-rank phases, collective-sequence
    check) must not cost the headline line when one rank's part fails: every rank still takes
    part in the one gather, the failing rank's row carries its error, the sequence check is
    skipped, and rank 0 prints a valid, verified line (np 3)."""
    import json
    r = _bench(["--gpus", "3", "--steps", "2", "--warmup", "1", "--min-warmup-s", "0",
                "--n-data", "1500", "--q-per-gpu", "200", "--verify", "--diag-steps", "1"],
               {"DMLP_DATA_PLANE": "host", "DMLP_DIAG_FAIL": "1"})
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    res = json.loads(r.stdout.decode().strip().splitlines()[-1])
    assert res["n_gpus"] == 3 and res["verify_ok"] and res["value"] > 0
    rows = res["per_rank"]
    assert "error" in rows[1] and "error" not in rows[0] and "error" not in rows[2]
    assert "collective_check" not in res


def test_collective_log_compare():
    """The collective-sequence comparison (parallel/dist_api.py compare_logs) flags a rank that
    enters a different collective, a different size, a missing call and an unmatched send."""
    from distributed_machine_learning_project_amd.parallel.dist_api import compare_logs
    ok = [("broadcast", None, 64, "float64", 0), ("gather", None, 16, "int64", 0)]
    assert compare_logs([ok, list(ok), list(ok)])["ok"]
    bad_size = [("broadcast", None, 64, "float64", 0), ("gather", None, 32, "int64", 0)]
    res = compare_logs([ok, bad_size, list(ok)])
    assert not res["ok"] and res["problems"][0]["rank"] == 1 and res["problems"][0]["index"] == 1
    assert not compare_logs([ok, ok[:1], ok])["ok"]
    p2p = [[("send", None, 8, "float64", 1)], [("recv", None, 8, "float64", 0)]]
    assert compare_logs(p2p)["ok"]
    p2p_bad = [[("send", None, 8, "float64", 1)], [("recv", None, 16, "float64", 0)]]
    assert not compare_logs(p2p_bad)["ok"]
    sub = [("broadcast", (0, 2), 8, "int32", 0)]
    assert compare_logs([sub, [], sub])["ok"]  # rank 1 is not in the group
    assert not compare_logs([sub, [], []])["ok"]


def _recv_any_worker(rank, world, port, q):
    import torch
    import torch.distributed as td
    from distributed_machine_learning_project_amd.parallel import dist_api as dist
    td.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                          world_size=world)
    dist.coll_log_start()
    g = dist.new_group([0, 1])  # logged by creation order, not id(group)
    t = torch.zeros(4)
    if rank == 1:
        dist.send(torch.ones(4), 0)
    elif rank == 0:
        dist.recv(t, None)  # from any rank: logged with the real source
    dist.barrier(group=g) if rank in (0, 1) else None
    res = dist.check_collective_sequence(dist.coll_log_stop())
    q.put((rank, res["ok"] if res else None, res["problems"] if res else None))
    td.destroy_process_group()


def test_collective_log_recv_any_source():
    """a recv(src=None) is logged with the sender's rank (its pair matches the send),
    and sub-groups are keyed by a rank-independent id."""
    import multiprocessing as mp
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_recv_any_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in ps:
        p.start()
    out = {}
    for _ in ps:
        r, ok, probs = q.get(timeout=120)
        out[r] = (ok, probs)
    for p in ps:
        p.join(timeout=60)
    assert out[0][0] is True, out[0][1]


def test_replication_mode_rule():
    """The farm's dataset replication (parallel/strategies.py replication_mode): the rows cross
    each GPU's own link behind the screen unless that concurrent copy would outlast what the
    screen hides (~1 ms) and the all-gather route is faster; no probe: h2d."""
    from distributed_machine_learning_project_amd.parallel.strategies import replication_mode
    rows = 100_000 * 32 * 4  # bench_4's int32 rows, 12.8 MB
    fast = {"world": 8, "h2d_GBps_per_gpu_concurrent": 50.0, "allgather_GBps": 300.0}
    slow = {"world": 8, "h2d_GBps_per_gpu_concurrent": 5.0, "allgather_GBps": 300.0}
    assert replication_mode(fast, rows) == "h2d"          # 0.26 ms: hidden behind the screen
    assert replication_mode(slow, rows) == "xgmi"         # 2.6 ms of rows vs 0.3 + 0.04 ms
    assert replication_mode(dict(slow, allgather_GBps=1.0), rows) == "h2d"  # a slower gather
    assert replication_mode(None, rows) == "h2d"
    assert replication_mode(fast, 10 * rows) == "xgmi"    # 2.6 ms of rows again
