"""Python Engine (engine.h API) on one MI355X, in-process (world size 1): every strategy, the
node-shared ingress, the out-of-core streamed farm and the debug listing print the CPU oracle's
bytes.  The multi-rank versions of the same paths run on CPU (gloo) in test_distributed.py."""
import numpy as np
import pytest

import distributed_machine_learning_project_amd as dmlp
from distributed_machine_learning_project_amd.ops import knn as K

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def workload():
    inp = dmlp.generate(6000, 700, 32, 0.0, 1000.0, 1, 40, 10, seed=31)
    d, i = K.knn_cpu(inp.X, inp.Qx, inp.k)
    _, cs = K.finalize_cpu(i, inp.k, inp.labels)
    return inp, dmlp.format_report(cs), d, i


def _engine(strategy, **kw):
    from distributed_machine_learning_project_amd.parallel.engine import Engine
    return Engine(strategy, device="gpu", **kw)


@pytest.mark.parametrize("strategy", ["farm", "shard_gather", "shard_reduce", "grid2d", "ring"])
def test_strategies_match_oracle(gpu, workload, strategy):
    inp, expect, _, _ = workload
    eng = _engine(strategy)
    out = eng.KNN(inp.params, inp, None)
    assert bytes(eng.report(out)) == expect
    eng.close()


@pytest.mark.parametrize("max_rows", ["0", "2500"])
def test_shared_ingress_and_out_of_core(gpu, workload, monkeypatch, max_rows):
    """Node-shared page-locked segment; with KNN_MAX_DEVICE_ROWS=2500 the dataset is streamed
    from it in 3 chunks instead of being copied whole."""
    from distributed_machine_learning_project_amd.utils.shm import share_input
    inp, expect, _, _ = workload
    monkeypatch.setenv("KNN_MAX_DEVICE_ROWS", max_rows)
    eng = _engine("farm")
    sh = share_input(eng.comm, inp)
    out = eng.KNN(sh.params, sh, None)
    assert bytes(eng.report(out)) == expect
    sh.close()
    eng.close()


@pytest.mark.parametrize("kmax,A", [(32, 32), (24, 32), (40, 32), (64, 32), (200, 32), (16, 100)])
def test_native_step(gpu, kmax, A):
    """One rank over the node-shared segment: the whole call runs in libdmlp's native step
    (pipeline.hip dmlp_step) for EVERY k — k <= 64 on the one-pass single-term screen, k in
    (64, 256] on the two-pass single-term screen — report, labels and checksums == the oracle's, three calls in
    a row (reused buffers), each served by the step."""
    from distributed_machine_learning_project_amd.utils.shm import share_input
    inp = dmlp.generate(7000, 9000 + kmax, A, 0.0, 1000.0, 1, kmax, 8, seed=kmax + A)
    d, i = K.knn_cpu(inp.X, inp.Qx, inp.k)
    lab_ref, cs = K.finalize_cpu(i, inp.k, inp.labels)
    eng = _engine("farm")
    sh = share_input(eng.comm, inp)
    for _ in range(3):
        n0 = K.STEP_STATS["calls"]
        out = eng.KNN(sh.params, sh, None)
        assert bytes(eng.report(out)) == dmlp.format_report(cs)
        np.testing.assert_array_equal(out.labels_np(), lab_ref)
        np.testing.assert_array_equal(out.checksums_np(), cs)
        assert K.STEP_STATS["calls"] == n0 + 1
        st = K.pipeline_stats()
        assert st["path"] == 0
        if A == 32 and kmax <= 64:
            # uniform data: no query may overflow the one-pass screen's refine (k near 64 once
            # overflowed the two-queries-per-wave kernel's 64 member slots and escalated)
            assert st["n_escalated"] == 0 and st["n_exact"] == 0, st
    sh.close()
    eng.close()


@pytest.mark.parametrize("escalate", [False, True])
def test_native_step_report_direct(gpu, escalate):
    """report_mode 1 into page-locked memory (pipeline.hip host_device_view): the format kernels
    write the text straight into the caller's buffer across PCIe (report_direct 1); pageable
    memory, or the switch off, is staged on the device and copied (0).  Every case == the oracle's
    bytes, labels and checksums, at qid_base 0 and 123456789 (wider ids).  escalate: a duplicated
    point cluster hands a query back from the refine, so the report is rendered a second time in
    the call, after the escalation."""
    import torch
    from distributed_machine_learning_project_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(5)
    N, Q, A = 6000, 5000, 32
    X = np.round(rng.uniform(0.0, 1000.0, (N, A)), 6)
    Qx = np.round(rng.uniform(0.0, 1000.0, (Q, A)), 6)
    if escalate:
        X[:80] = X[0]
        Qx[0] = X[0]
    k = rng.integers(1, 33, Q).astype(np.int32)
    k[0] = 32
    labels = rng.integers(0, 8, N).astype(np.int32)
    d, i = K.knn_cpu(X, Qx, k)
    lab_ref, cs = K.finalize_cpu(i, k, labels)
    bound = L.dmlp_format_bound(Q)
    pinned = torch.empty(bound + 4096, dtype=torch.uint8).pin_memory().numpy()
    # name, buffer, report_direct, qid_base, expected report_direct stat
    cases = [("pinned", pinned, 1, 0, 1), ("pinned view", pinned[4096:], 1, 0, 1),
             ("pinned qid_base", pinned, 1, 123456789, 1),
             ("pageable", np.empty(bound, np.uint8), 1, 0, 0), ("staged", pinned, 0, 0, 0),
             ("staged qid_base", pinned, 0, 123456789, 0)]
    old_cus = L.dmlp_pipeline_set(b"num_cus", 4)  # (one screen slice: the pair refine's case)
    try:
        for name, dst, direct, base, want in cases:
            od = L.dmlp_pipeline_set(b"report_direct", direct)
            try:
                dst[:] = 0
                r = K.step(X, labels, (0, 8), Qx, k, report=dst, qid_base=base)
            finally:
                L.dmlp_pipeline_set(b"report_direct", od)
            assert bytes(dst[:r.report_len]) == dmlp.format_report(cs, base), name
            np.testing.assert_array_equal(r.label.cpu().numpy(), lab_ref)
            np.testing.assert_array_equal(r.checksum.cpu().numpy().view(np.uint64), cs)
            st = K.pipeline_stats()
            assert (st["n_escalated"] + st["n_exact"] >= 1) == escalate, (name, st)
            assert st["report_direct"] == want, (name, st)
    finally:
        L.dmlp_pipeline_set(b"num_cus", old_cus)


@pytest.mark.parametrize("decimals", [6, None])
def test_native_step_pair_refine_row_forms(gpu, decimals):
    """The pair refine (k <= 32, one slice of host operands) reads the dataset rows as they crossed
    PCIe: lossless int32 for 6-decimal data (each value divided back on the device, no fp64 copy
    made unless another pass needs it) or fp64 for full-precision data.  Both == the oracle's
    report, labels and checksums, with an escalated query in the same call (a duplicated point
    cluster) forcing the deferred fp64 conversion after the refine."""
    from distributed_machine_learning_project_amd.utils.shm import share_input
    rng = np.random.default_rng(11)
    N, Q, A = 9000, 6000, 32
    X = rng.uniform(0.0, 1000.0, (N, A))
    Qx = rng.uniform(0.0, 1000.0, (Q, A))
    if decimals is not None:
        X, Qx = np.round(X, decimals), np.round(Qx, decimals)
    X[:80] = X[0]  # 80 identical points: a query on them ties past the 64 member slots
    Qx[0] = X[0]
    k = rng.integers(1, 33, Q).astype(np.int32)
    k[0] = 32
    labels = rng.integers(0, 6, N).astype(np.int32)
    inp = dmlp.KNNInput(labels, X, k, Qx)
    d, i = K.knn_cpu(inp.X, inp.Qx, inp.k)
    lab_ref, cs = K.finalize_cpu(i, inp.k, inp.labels)
    from distributed_machine_learning_project_amd import _lib
    L = _lib.lib()
    # (one screen slice, the pair refine's case, needs a full round of waves: shrink the CUs the
    # slice choice fills so 6000 queries make one)
    old_cus = L.dmlp_pipeline_set(b"num_cus", 4)
    eng = _engine("farm")
    sh = share_input(eng.comm, inp)
    try:
        for _ in range(2):
            out = eng.KNN(sh.params, sh, None)
            assert bytes(eng.report(out)) == dmlp.format_report(cs)
            np.testing.assert_array_equal(out.labels_np(), lab_ref)
            np.testing.assert_array_equal(out.checksums_np(), cs)
            st = K.pipeline_stats()
            assert st["path"] == 0 and st["n_escalated"] + st["n_exact"] >= 1, st
    finally:
        L.dmlp_pipeline_set(b"num_cus", old_cus)
        sh.close()
        eng.close()


def _early_inputs(n, A, kmax, Q, seed):
    """Two different inputs of one shape (alternated through one engine, so a screen that read a
    slice before its ready word, or a stale line, would read the OTHER input's bytes), each with
    its farthest point in the last rows: the last image slice raises every column's eps."""
    out = []
    for s in (seed, seed + 1):
        inp = dmlp.generate(n, Q, A, 0.0, 1000.0, 1, kmax, 8, seed=s)
        inp.X[-1] = 1000.0 if s % 2 else 0.0  # a corner of the box: the largest |x - mu|
        d, i = K.knn_cpu(inp.X, inp.Qx, inp.k)
        lab_ref, cs = K.finalize_cpu(i, inp.k, inp.labels)
        out.append((inp, lab_ref, cs, dmlp.format_report(cs)))
    return out


@pytest.mark.parametrize("render", ["device", "host"])
@pytest.mark.parametrize("n,A,kmax", [(2000, 32, 16), (5000, 32, 32), (3000, 64, 64),
                                        (3000, 64, 32), (3000, 64, 16), (3000, 128, 32),
                                        (3000, 256, 32)])
def test_native_step_early_start(gpu, n, A, kmax, render):
    """Early start: the screen starts on the query operands while the dataset image crosses
    PCIe in slices with ready words.  The host sleeps 400 us before each image slice
    (dmlp_step_early_delay), so the screen provably waits mid-scan; the device counters then show
    waits > 0, eps growths > 0 (the far point sits in the last slice) and no timeout.  Two
    different inputs of equal shape alternate A, B, A, B (early on), then once with the early
    start off.  Each slice's ready word is one DMA copy carrying the slice's max norm; every
    report, label and checksum == its own oracle's.  A = 64 / k = 64 runs the KT = 2 screen on its
    32-entry variant with the early start; A = 64 / k <= 32 its 16-entry variant (2 x 256
    registers), which leaves no slot for the copies: no early start there.  A = 128 (KT = 4) and A = 256 (KT = 8): the step refuses the early start
    there — its image copies (blit kernels in this process) found no wave slot beside the spinning
    KT 4 screen in 2 of 7 sessions (profiles/r12a_kt4_early.txt), KT 8 takes all 512 registers —
    and the results stay exact.  One screen slice needs a full round of waves (>= 131072 queries
    at KT = 1, >= 65536 at KT >= 4).  render: the device
    render switch on or off — an early-start step renders on the host either way
    (pipeline.hip dr_early_ok); without the early start the switch's render runs."""
    from distributed_machine_learning_project_amd import _lib
    L = _lib.lib()
    old_dr = L.dmlp_pipeline_set(b"device_render", 1 if render == "device" else 0)
    # an early-start step renders on the host whatever the switch says (the device render's
    # kernels get no reliable wave slots beside the spinning screen: pipeline.hip dr_early_ok)
    dr_used = False
    # KT 2 / k <= 32 (the 16-entry screen): no registers for the early start's copies
    # (pipeline.hip early_room): no early start there
    no_room = A > 32 and A <= 64 and kmax <= 32
    Q = 131072 + 64 * 3 if A <= 64 else 65536 + 64
    cases = _early_inputs(n, A, kmax, Q, seed=n + A + kmax)
    dsts = []
    import torch
    for inp, _, _, _ in cases:
        dsts.append(torch.empty(48 * Q + 64, dtype=torch.uint8).pin_memory().numpy())
    try:
        L.dmlp_step_early_delay(400)
        for rnd, early in enumerate((1, 1, 1, 1, 0)):
            L.dmlp_step_early(early)
            inp, lab_ref, cs, expect = cases[rnd % 2]
            dst = dsts[rnd % 2]
            r = K.step(inp.X, inp.labels, (0, 8), inp.Qx, inp.k, report=dst)
            assert bytes(dst[:r.report_len]) == expect, f"round {rnd}"
            np.testing.assert_array_equal(r.label.cpu().numpy(), lab_ref)
            np.testing.assert_array_equal(r.checksum.cpu().numpy().view(np.uint64), cs)
            assert r.early == (early if A <= 64 and not no_room else 0)
            if r.early:
                assert K.pipeline_stats()["device_render"] == (1 if dr_used else 0)
            if A <= 64:
                assert r.n_escalated == 0, f"round {rnd}: {r.n_escalated} queries escalated"
            if not r.early and early and render == "device":
                assert K.pipeline_stats()["device_render"] == 1  # (no early start: rendered first)
            if r.early:
                assert r.early_timeouts == 0
                assert r.early_waits > 0, "the screen never waited for a slice"
                assert r.early_grows > 0, "no column's eps grew with a later slice"
    finally:
        L.dmlp_step_early(-1)
        L.dmlp_step_early_delay(-1)
        L.dmlp_pipeline_set(b"device_render", old_dr)


@pytest.mark.parametrize("n,A,Q,kmin,kmax,auto", [(300_000, 32, 4096, 1, 32, 1),
                                                   (110_000, 100, 2048, 16, 16, 1),
                                                   (270_000, 48, 3000, 40, 64, 0)])
def test_native_step_large_n_pipeline(gpu, n, A, Q, kmin, kmax, auto):
    """at large N the step picks the device render by its cost model (the host
    render's fp16 image + int32 rows vs the int32 rows alone) and runs the screen as a pipeline
    over up to 8 dataset chunks of its slices — chunk c's screen while chunk c + 1 crosses PCIe,
    each chunk's eps from the image's max norm seen so far (the refine takes the largest over the
    slices).  Two alternated inputs, then the host render forced (DMLP_DEVICE_RENDER=0 by the
    switch) and an input whose last row lies outside the fp16 range (the whole call redone on the
    device image): every report, label and checksum == the oracle's.  The device render is forced
    (DMLP_DEVICE_RENDER=1 by the switch) so every shape runs the pipeline; a last call checks the
    cost model's own choice (auto: 1 device, 0 host — k in (32, 64] below 2^26 values renders on
    the host)."""
    from distributed_machine_learning_project_amd import _lib
    import torch
    L = _lib.lib()
    cases = []
    for seed in (11, 12, 13):
        inp = dmlp.generate(n, Q, A, 0.0, 1000.0, kmin, kmax, 8, seed=seed + n)
        if seed == 13:
            inp.X[-1, 0] = 5.0e6  # far outside the fp16 screen's range, in the last chunk
        else:
            inp.X[-1] = 1000.0  # the largest |x - mu| sits in the last chunk: eps grows there
        _, i = K.knn_cpu(inp.X, inp.Qx, inp.k)
        lab_ref, cs = K.finalize_cpu(i, inp.k, inp.labels)
        cases.append((inp, lab_ref, cs, dmlp.format_report(cs)))
    dst = torch.empty(48 * Q + 64, dtype=torch.uint8).pin_memory().numpy()
    old = L.dmlp_pipeline_set(b"device_render", -1)
    try:
        for rnd, (ci, dr) in enumerate(((0, 1), (1, 1), (0, 1), (1, 0), (2, 1), (0, -1))):
            L.dmlp_pipeline_set(b"device_render", dr)
            inp, lab_ref, cs, expect = cases[ci]
            r = K.step(inp.X, inp.labels, (0, 8), inp.Qx, inp.k, report=dst)
            assert bytes(dst[:r.report_len]) == expect, f"round {rnd}"
            np.testing.assert_array_equal(r.label.cpu().numpy(), lab_ref)
            np.testing.assert_array_equal(r.checksum.cpu().numpy().view(np.uint64), cs)
            assert r.early == 0
            if ci == 2:
                assert r.path == 2  # (the device image path after the out-of-range render)
            else:
                assert r.path == 0
                want = auto if dr < 0 else dr
                assert K.pipeline_stats()["device_render"] == want, f"round {rnd}"
    finally:
        L.dmlp_pipeline_set(b"device_render", old)


def test_debug_listing(gpu, workload):
    inp, _, d, i = workload
    eng = _engine("ring", debug=True)
    out = eng.KNN(inp.params, inp, None)
    lab, _ = K.finalize_cpu(i, inp.k, inp.labels)
    assert bytes(eng.report(out)) == dmlp.format_debug(d, i, inp.k, lab)
    eng.close()


_POLICY_CHILD = r"""
import sys
import numpy as np
import distributed_machine_learning_project_amd as dmlp
from distributed_machine_learning_project_amd import _lib
from distributed_machine_learning_project_amd.ops import knn as K
inp = dmlp.generate(3000, 4096, 32, 0.0, 1000.0, 1, 16, 8, seed=5)
_, i = K.knn_cpu(inp.X, inp.Qx, inp.k)
_, cs = K.finalize_cpu(i, inp.k, inp.labels)
r = K.step(inp.X, inp.labels, (0, 8), inp.Qx, inp.k, report="device")
ok = np.array_equal(r.checksum.cpu().numpy().view(np.uint64), cs)
print("POLICY", _lib.lib().dmlp_host_threads(), r.path, int(ok))
"""


def test_step_policy_host_budget_and_shared_device(gpu, monkeypatch):
    """The step's automatic choices (profiles/r7h_host_budget.md): (1) ranks sharing one GPU
    (DMLP_DEVICE_RANKS > 1, set by Comm.init / knn_engine) run without the early start, which
    made P = 3 on one MI355X 2.8x slower; DMLP_FAST_EARLY=1 still forces it.  (2) With the host
    render (DMLP_DEVICE_RENDER=0) a render pool of one thread takes the device-image path
    (measured faster there); DMLP_HOST_OPS=1 forces the host operands.  Results == the oracle's
    either way."""
    import os
    import subprocess
    import sys
    from distributed_machine_learning_project_amd import _lib
    L = _lib.lib()
    (inp, lab_ref, cs, expect), _ = _early_inputs(2000, 32, 16, 131072 + 64, seed=77)
    import torch
    dst = torch.empty(48 * len(inp.k) + 64, dtype=torch.uint8).pin_memory().numpy()
    monkeypatch.delenv("DMLP_FAST_EARLY", raising=False)
    try:
        for ranks, force, want in (("2", None, 0), ("1", None, 1), ("3", "1", 1)):
            monkeypatch.setenv("DMLP_DEVICE_RANKS", ranks)
            if force:
                monkeypatch.setenv("DMLP_FAST_EARLY", force)
            L.dmlp_step_early(-1)  # re-read the environment
            r = K.step(inp.X, inp.labels, (0, 8), inp.Qx, inp.k, report=dst)
            assert bytes(dst[:r.report_len]) == expect
            assert r.early == want, (ranks, force)
    finally:
        monkeypatch.delenv("DMLP_DEVICE_RANKS", raising=False)
        monkeypatch.delenv("DMLP_FAST_EARLY", raising=False)
        L.dmlp_step_early(-1)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    # (3) with the device render (DMLP_DEVICE_RENDER=1) the host only packs int32 rows: a
    # one-thread pool keeps the single-term fp16 operands (path 0) as well; the default is the host
    # render (the device render measured slower: profiles/r9r_device_render_ab.txt)
    for env, want_path in (({"DMLP_HOST_THREADS": "1", "DMLP_DEVICE_RENDER": "0"}, 2),
                           ({"DMLP_HOST_THREADS": "1", "DMLP_HOST_OPS": "1",
                             "DMLP_DEVICE_RENDER": "0"}, 0),
                           ({"DMLP_HOST_THREADS": "2", "DMLP_DEVICE_RENDER": "0"}, 0),
                           ({"DMLP_HOST_THREADS": "1"}, 2),
                           ({"DMLP_HOST_THREADS": "1", "DMLP_DEVICE_RENDER": "1"}, 0)):
        e = dict(os.environ, **env)
        e.pop("DMLP_HOST_OPS", None) if "DMLP_HOST_OPS" not in env else None
        e.pop("DMLP_DEVICE_RENDER", None) if "DMLP_DEVICE_RENDER" not in env else None
        out = subprocess.run([sys.executable, "-c", _POLICY_CHILD], cwd=root, env=e,
                             capture_output=True, text=True, timeout=100)
        line = [x for x in out.stdout.splitlines() if x.startswith("POLICY")]
        assert line, out.stderr[-2000:]
        _, threads, path, ok = line[-1].split()
        assert int(threads) == int(env["DMLP_HOST_THREADS"])
        assert int(path) == want_path, env
        assert ok == "1"
