"""Standalone native `knn_engine` binary (csrc/engine_main.cpp) — host-only paths on the CPU
(serial KD-tree strategy = bench.debug, under 1 and 2 MPI ranks), every GPU strategy on a GPU.
Output is compared byte-for-byte with the float64 oracle's report (SURVEY.md §4 level 3/5)."""
import json
import os
import subprocess

import numpy as np
import pytest

import distributed_machine_learning_project_amd as dmlp
from distributed_machine_learning_project_amd import build
from distributed_machine_learning_project_amd.ops import reference as ref

MPIEXEC = "/opt/conda/bin/mpiexec"


def _engine():
    e = build.build_engine()
    if e is None or not os.path.exists(e):
        pytest.skip("knn_engine not built (no MPI headers)")
    return str(e)


def _case(tmp_path, N=1500, Q=120, A=6, kmin=1, kmax=60, seed=9):
    txt = dmlp.generate_text(N, Q, A, -20, 20, kmin, kmax, 5, seed=seed)
    path = tmp_path / "in.txt"
    path.write_text(txt)
    inp = dmlp.parse_input(txt)
    res, lab, cs = ref.knn(inp.X, inp.labels, inp.Qx, inp.k)
    return path, inp, res, lab, cs


def _run(args, path, env=None, np_=1, timeout=120):
    cmd = ([MPIEXEC, "-n", str(np_)] if np_ > 1 else []) + [_engine(), *args, "--input", str(path)]
    e = dict(os.environ)
    e.update(env or {})
    r = subprocess.run(cmd, capture_output=True, timeout=timeout, env=e)
    assert r.returncode == 0, r.stderr.decode()
    return r.stdout, r.stderr.decode()


def test_serial_matches_oracle(tmp_path):
    path, inp, res, lab, cs = _case(tmp_path)
    out, err = _run(["--strategy", "serial"], path)
    assert out == dmlp.format_report(cs)
    assert err.startswith("Time taken: ") and err.rstrip().endswith(" ms")


@pytest.mark.skipif(not os.path.exists(MPIEXEC), reason="no mpiexec")
def test_serial_two_ranks_prints_once(tmp_path):
    path, inp, res, lab, cs = _case(tmp_path, N=800, Q=50)
    out, _ = _run(["--strategy", "serial"], path, np_=2)
    assert out == dmlp.format_report(cs)


def test_serial_debug_listing(tmp_path):
    path, inp, res, lab, cs = _case(tmp_path, N=300, Q=12, kmax=9)
    out, _ = _run(["--strategy", "serial", "--debug"], path)
    K = max(int(k) for k in inp.k)
    d = np.full((inp.Q, K), np.inf)
    i = np.full((inp.Q, K), -1, np.int32)
    for q, (dq, iq) in enumerate(res):
        d[q, :len(dq)] = dq
        i[q, :len(iq)] = iq
    assert out == dmlp.format_debug(d, i, inp.k, lab)


def test_trace_and_metrics_sidecar(tmp_path):
    path, *_ = _case(tmp_path, N=500, Q=40)
    mpath = tmp_path / "m.json"
    out, err = _run(["--strategy", "serial"], path, env={"KNN_TRACE": "1", "KNN_METRICS": str(mpath)})
    lines = err.splitlines()
    assert lines[0].startswith("Time taken: ")           # run_bench.sh greps the first match
    assert any(l.startswith("[dmlp-trace] rank 0 kdtree") for l in lines)
    m = json.loads(mpath.read_text())
    assert m["strategy"] == "serial" and m["N"] == 500 and m["Q"] == 40 and m["queries_per_s"] > 0


def test_malformed_input_fails_loudly(tmp_path):
    p = tmp_path / "bad.txt"
    p.write_text("3 1 2\n0 1.0 2.0\n1 oops 2.0\n0 1 1\nQ 1 0 0\n")
    r = subprocess.run([_engine(), "--strategy", "serial", "--input", str(p)], capture_output=True,
                       timeout=60)
    assert r.returncode != 0 and b"wrongly formatted" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("strategy", ["farm", "shard_gather", "shard_reduce", "grid2d"])
def test_gpu_strategies_match_oracle(tmp_path, strategy):
    path, inp, res, lab, cs = _case(tmp_path, N=6000, Q=700, A=20, kmax=150)
    out, _ = _run(["--strategy", strategy], path)
    assert out == dmlp.format_report(cs)
    out, _ = _run(["--strategy", strategy, "--exact"], path)
    assert out == dmlp.format_report(cs)


# ---------------------------------------------------------------- include/engine.h drop-in
NATIVE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")


def _dropin(tmp_path, debug=False):
    try:
        return str(build.build_dropin(os.path.join(NATIVE, "mini_harness.cpp"),
                                      str(tmp_path / ("engine.debug" if debug else "engine")),
                                      debug=debug,
                                      extra_flags=['-DDMLP_COMMON_HEADER="contract_types.h"']))
    except RuntimeError as e:
        pytest.skip(f"drop-in build unavailable: {e}")


def _run_dropin(exe, path, env, np_=1):
    e = dict(os.environ)
    e.update(env)
    if np_ > 1:
        # every rank opens the file as its stdin (only rank 0 reads it, common.cpp:93): MPICH's
        # stdin forwarding to rank 0 can die with SIGPIPE on larger inputs
        import shlex
        cmd = [MPIEXEC, "-n", str(np_), "sh", "-c",
               f"exec {shlex.quote(exe)} < {shlex.quote(str(path))}"]
        r = subprocess.run(cmd, stdin=subprocess.DEVNULL, capture_output=True, timeout=180, env=e)
    else:
        with open(path, "rb") as f:
            r = subprocess.run([exe], stdin=f, capture_output=True, timeout=180, env=e)
    assert r.returncode == 0, r.stderr.decode()
    assert b"Time taken: " in r.stderr
    return r.stdout


def test_dropin_engine_h_cpu(tmp_path):
    """engine.h + dropin_engine.cpp driven by a harness with the reference's contract."""
    path, inp, res, lab, cs = _case(tmp_path, N=900, Q=70)
    exe = _dropin(tmp_path)
    assert _run_dropin(exe, path, {"KNN_DEVICE": "cpu"}) == dmlp.format_report(cs)
    if os.path.exists(MPIEXEC):
        assert _run_dropin(exe, path, {"KNN_DEVICE": "cpu"}, np_=2) == dmlp.format_report(cs)


def test_dropin_engine_h_debug_cpu(tmp_path):
    path, inp, res, lab, cs = _case(tmp_path, N=200, Q=9, kmax=7)
    out = _run_dropin(_dropin(tmp_path, debug=True), path, {"KNN_DEVICE": "cpu"})
    lines = out.decode().splitlines()
    assert lines[0] == f"Label for Query 0 : {lab[0]}"
    assert lines[1] == f"Top-{inp.k[0]} neighbors:"
    assert lines[2].split(" : ")[0] == str(res[0][1][0])


@pytest.mark.gpu
@pytest.mark.parametrize("strategy", ["farm", "shard_reduce"])
def test_dropin_engine_h_gpu(tmp_path, strategy):
    """One rank on the MI355X: stdout == the oracle's bytes.  The farm's report streams to
    stdout in pieces as their copies land (KnnCore::emit_chunks): 4 (default), 7 (uneven
    pieces) and 1 (the whole text after the step)."""
    path, inp, res, lab, cs = _case(tmp_path, N=5000, Q=400, A=12, kmax=150)
    exe = _dropin(tmp_path)
    out = _run_dropin(exe, path, {"KNN_STRATEGY": strategy})
    assert out == dmlp.format_report(cs)
    if strategy == "farm":
        for chunks in ("7", "1"):
            out = _run_dropin(exe, path, {"KNN_STRATEGY": strategy, "KNN_EMIT_CHUNKS": chunks})
            assert out == dmlp.format_report(cs), chunks


# ---------------------------------------------------------------- the reference's own harness
def _ref_dropin(tmp_path, debug=False, inplace=False):
    """Build from the reference's unmodified common.cpp: staged next to this
    package's engine.h, or in place against the reference's own engine.h (a copy of the tree,
    so nothing is written into the reference).  The reference tree, or on a GPU box the
    untracked copy build() staged in _refharness."""
    ref_common = build.reference_harness()
    if ref_common is None:
        pytest.skip("reference common.cpp not present")
    REF_COMMON = str(ref_common)
    import shutil
    src = REF_COMMON
    if inplace:
        tree = tmp_path / "reftree"
        tree.mkdir(exist_ok=True)
        for f in ("common.cpp", "common.h", "engine.h"):
            if not (tree / f).exists():  # (copyfile: the sources may be read-only)
                shutil.copyfile(os.path.join(os.path.dirname(REF_COMMON), f), tree / f)
        src = str(tree / "common.cpp")
    name = f"engine{'.debug' if debug else ''}{'.inplace' if inplace else ''}"
    try:
        return str(build.build_dropin(src, str(tmp_path / name), debug=debug, inplace=inplace))
    except RuntimeError as e:
        pytest.skip(f"drop-in build unavailable: {e}")


def _debug_expect(inp, res, lab):
    K = max(1, max(int(k) for k in inp.k))
    d = np.full((inp.Q, K), np.inf)
    i = np.full((inp.Q, K), -1, np.int32)
    for q, (dq, iq) in enumerate(res):
        d[q, :len(dq)] = dq
        i[q, :len(iq)] = iq
    return dmlp.format_debug(d, i, inp.k, lab)


@pytest.mark.parametrize("inplace", [False, True])
@pytest.mark.parametrize("debug", [False, True])
def test_reference_common_cpp_dropin_cpu(tmp_path, debug, inplace):
    """The reference's own common.cpp + dropin_engine.cpp, built staged (this engine.h) and in
    place (the reference's engine.h: the Engine object holds no state, the engine singleton
    starts at MPI_Init), release and -DDEBUG, np 1 and 2: stdout == the fp64 oracle's bytes."""
    path, inp, res, lab, cs = _case(tmp_path, N=700, Q=45, kmax=25)
    exe = _ref_dropin(tmp_path, debug=debug, inplace=inplace)
    expect = _debug_expect(inp, res, lab) if debug else dmlp.format_report(cs)
    assert _run_dropin(exe, path, {"KNN_DEVICE": "cpu"}) == expect
    if os.path.exists(MPIEXEC):
        assert _run_dropin(exe, path, {"KNN_DEVICE": "cpu"}, np_=2) == expect


@pytest.mark.gpu
@pytest.mark.parametrize("inplace", [False, True])
def test_reference_common_cpp_dropin_gpu(tmp_path, inplace):
    """Same on the MI355X: release build (GPU-rendered report written to std::cout) and the
    DEBUG listing (lists through the harness's reportResult); np 2 over the host-staged plane."""
    path, inp, res, lab, cs = _case(tmp_path, N=5000, Q=400, A=12, kmax=150)
    exe = _ref_dropin(tmp_path, inplace=inplace)
    assert _run_dropin(exe, path, {}) == dmlp.format_report(cs)
    assert _run_dropin(exe, path, {"KNN_DATA_PLANE": "host"}, np_=2) == dmlp.format_report(cs)
    dbg = _ref_dropin(tmp_path, debug=True, inplace=inplace)
    assert _run_dropin(dbg, path, {}) == _debug_expect(inp, res, lab)


@pytest.mark.gpu
def test_fast_path_serves_any_k_and_escalates_per_query(tmp_path):
    """knn_engine's single-GPU host-operand pipeline no longer gives up on the
    whole call — k in [1, 64] (the x1 class plus the 3-term class on a device image rendered from
    the landed rows) and one query among 600 duplicate points (its single-term candidates
    overflow: that query alone escalates to the 3-term screen / exact path) stay on the fast
    path (its KNN_TRACE phases), and print the oracle's bytes."""
    rng = np.random.default_rng(17)
    N, Q, A = 6000, 300, 16
    X = np.round(rng.uniform(0, 1000, (N, A)), 6)
    X[:600] = X[0]                      # 600 identical points: ties far beyond any buffer
    Qx = np.round(rng.uniform(0, 1000, (Q, A)), 6)
    Qx[7] = X[0]
    k = rng.integers(1, 65, Q).astype(np.int32)
    k[7] = 12
    labels = rng.integers(0, 5, N).astype(np.int32)
    inp = dmlp.KNNInput(labels, X, k, Qx)
    path = tmp_path / "tight.in"
    path.write_text(dmlp.to_text(inp))
    inp = dmlp.parse_input(path.read_text())
    _, _, cs = ref.knn(inp.X, inp.labels, inp.Qx, inp.k)
    out, err = _run(["--strategy", "farm"], path, env={"KNN_TRACE": "1"})
    assert out == dmlp.format_report(cs)
    phases = [l.split()[3] for l in err.splitlines() if l.startswith("[dmlp-trace]")]
    assert "step" in phases, phases  # the library's native step, not the general farm
    assert "distribute" not in phases and "compute" not in phases
    st = [l.split() for l in err.splitlines()
          if l.startswith("[dmlp-step]") and " path " in l][-1]  # (the call; not its timeline)
    assert st[st.index("path") + 1] == "0"            # host-rendered operands
    assert int(st[st.index("escalated") + 1]) >= 1    # the tied query escalated alone
    # k > 32 on the 3-term LDS screen over the device image instead of the default two-pass
    # single-term screen (KNN_X1K=0), and the 3-term streaming first screen (KNN_SCREEN=stream):
    # the same bytes
    for env in ({"KNN_X1K": "0"}, {"KNN_SCREEN": "stream"}):
        out, _ = _run(["--strategy", "farm"], path, env=env)
        assert out == dmlp.format_report(cs)


# ---------------------------------------------------------------- the reference runner's `make`
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_make_engine_targets_cpu(tmp_path):
    """run_bench.sh:74,84 runs `make` and then `mpirun ./engine < input`: the top-level Makefile's
    engine / engine.debug targets (the reference's unmodified common.cpp + the drop-in) build and
    print the fp64 oracle's bytes at np 1 and 2, release and DEBUG listing."""
    if build.reference_harness() is None:
        pytest.skip("reference common.cpp not present")
    r = subprocess.run(["make", "-C", ROOT, "engine", "engine.debug"], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    path, inp, res, lab, cs = _case(tmp_path, N=800, Q=50, kmax=30, seed=4)
    rel, dbg = os.path.join(ROOT, "engine"), os.path.join(ROOT, "engine.debug")
    assert _run_dropin(rel, path, {"KNN_DEVICE": "cpu"}) == dmlp.format_report(cs)
    assert _run_dropin(dbg, path, {"KNN_DEVICE": "cpu"}) == _debug_expect(inp, res, lab)
    if os.path.exists(MPIEXEC):
        assert _run_dropin(rel, path, {"KNN_DEVICE": "cpu"}, np_=2) == dmlp.format_report(cs)
    # up to date: a second `make` rebuilds nothing
    r = subprocess.run(["make", "-C", ROOT, "-q", "engine", "engine.debug"], capture_output=True,
                       timeout=60)
    assert r.returncode == 0


# ---------------------------------------------------------------- the drop-in's node window (P > 1)
def _text_with_decimals(inp, decimals):
    """The input as the reference's text format, attributes printed with `decimals` digits (9:
    values the lossless int32 row transfer cannot carry, so the render plane ships fp64 rows)."""
    f = f"%.{decimals}f"
    lines = [f"{inp.X.shape[0]} {inp.Qx.shape[0]} {inp.X.shape[1]}"]
    for lab, row in zip(inp.labels, inp.X):
        lines.append(f"{int(lab)} " + " ".join(f % v for v in row))
    for k, row in zip(inp.k, inp.Qx):
        lines.append(f"Q {int(k)} " + " ".join(f % v for v in row))
    return "\n".join(lines) + "\n"


@pytest.mark.skipif(not os.path.exists(MPIEXEC), reason="no mpiexec")
@pytest.mark.parametrize("np_,decimals", [(2, 6), (2, 9), (3, 6), (3, 9), (8, 6)])
@pytest.mark.parametrize("front", ["cma", "fill"])
def test_dropin_node_window_cpu(tmp_path, np_, decimals, front):
    """engine.h drop-in at P > 1 through the node window (KNN_DEVICE=cpu KNN_STRATEGY=farm runs
    the GPU path's protocol on the CPU), both fronts:
      cma  — rank 0 only publishes the addresses of its row tables, k and labels; every rank
             reads its own query block and its share of the dataset's rows straight from rank 0's
             address space (process_vm_readv) and renders 1/P of the render plane;
      fill — rank 0's pool gathers every rank's block into the MPI-3 shared window, releasing
             each as it lands, and renders the whole plane (int32 rows, or fp64 for 9-decimal
             data).
    Every rank rebuilds the dataset from the plane, answers its own query block and copies its
    report lines into the window at its offset.  The window starts at 1 MiB and grows
    collectively.  stdout == the fp64 oracle's bytes; every rank took part; the KNN_METRICS
    sidecar names the front and every rank's release time."""
    import json
    rng = np.random.default_rng(np_ * 10 + decimals)
    N, Q, A = 2100, 203, 7
    X = rng.uniform(-20, 20, (N, A))
    Qx = rng.uniform(-20, 20, (Q, A))
    k = rng.integers(1, 61, Q).astype(np.int32)
    labels = rng.integers(0, 5, N).astype(np.int32)
    txt = _text_with_decimals(dmlp.KNNInput(labels, X, k, Qx), decimals)
    path = tmp_path / "w.in"
    path.write_text(txt)
    inp = dmlp.parse_input(txt)
    _, _, cs = ref.knn(inp.X, inp.labels, inp.Qx, inp.k)
    exe = _ref_dropin(tmp_path) if build.reference_harness() is not None else _dropin(tmp_path)
    met = tmp_path / "m.json"
    env = {"KNN_DEVICE": "cpu", "KNN_STRATEGY": "farm", "KNN_WINDOW_MB": "1", "KNN_TRACE": "1",
           "KNN_WINDOW_FRONT": front, "KNN_METRICS": str(met)}
    e = dict(os.environ, **env)
    import shlex
    cmd = [MPIEXEC, "-n", str(np_), "sh", "-c", f"exec {shlex.quote(exe)} < {shlex.quote(str(path))}"]
    r = subprocess.run(cmd, stdin=subprocess.DEVNULL, capture_output=True, timeout=180, env=e)
    assert r.returncode == 0, r.stderr.decode()
    assert r.stdout == dmlp.format_report(cs)
    err = r.stderr.decode()
    for rank in range(np_):  # the window protocol ran on every rank (not the serial fallback)
        assert f"[dmlp-trace] rank {rank} window " in err, err[-2000:]
    m = json.loads(met.read_text())
    w = m["window"]
    if front == "cma":
        assert w["cma_ok"], "process_vm_readv on rank 0 was refused"
    assert w["front"] == front
    assert len(w["release_ms"]) == np_


@pytest.mark.skipif(not os.path.exists(MPIEXEC), reason="no mpiexec")
@pytest.mark.parametrize("np_", [1, 3])
@pytest.mark.parametrize("vms", ["1", "0"])
def test_dropin_report_egress_pipe(tmp_path, np_, vms):
    """the report egress as run_bench.sh launches the engine (mpiexec, the
    engine's stdout a pipe to the launcher): the pipe is widened and the report's pages are
    vmspliced into it (KNN_VMSPLICE=0: write()), the buffers stay untouched until the pipe
    drained; a redirected file gets write().  stdout == the oracle's bytes every way, and the
    KNN_METRICS sidecar says which path ran."""
    import json
    import shlex
    path, inp, res, lab, cs = _case(tmp_path, N=1500, Q=3000)
    exe = _ref_dropin(tmp_path) if build.reference_harness() is not None else _dropin(tmp_path)
    met = tmp_path / "m.json"
    e = dict(os.environ, KNN_DEVICE="cpu", KNN_STRATEGY="farm", KNN_VMSPLICE=vms,
             KNN_METRICS=str(met))
    cmd = [MPIEXEC, "-n", str(np_), "sh", "-c", f"exec {shlex.quote(exe)} < {shlex.quote(str(path))}"]
    r = subprocess.run(cmd, stdin=subprocess.DEVNULL, capture_output=True, timeout=180, env=e)
    assert r.returncode == 0, r.stderr.decode()
    assert r.stdout == dmlp.format_report(cs)
    m = json.loads(met.read_text())
    assert m["stdout_fifo"] is True
    assert (m["vmsplice_bytes"] > 0) == (vms == "1")
    # stdout redirected to a file (the direct run): write(), same bytes
    out = tmp_path / "o.txt"
    with open(path, "rb") as fin, open(out, "wb") as fo:
        r = subprocess.run([exe], stdin=fin, stdout=fo, stderr=subprocess.PIPE, timeout=180,
                           env=dict(e, KNN_STRATEGY="serial"))
    assert r.returncode == 0, r.stderr.decode()
    assert out.read_bytes() == dmlp.format_report(cs)
    m = json.loads(met.read_text())
    assert m["stdout_fifo"] is False and m["vmsplice_bytes"] == 0
