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


@pytest.mark.parametrize("kmax,fast,parts,rparts", [(32, True, 1, 1), (32, True, 2, 1),
                                                    (24, True, 3, 1), (40, False, 1, 1),
                                                    (32, True, 1, 2), (20, True, 1, 3)])
def test_native_fast_step(gpu, kmax, fast, parts, rparts):
    """One rank over the node-shared segment, every k on the single-term class: the whole call
    runs in one native function (fast_step.hip) — report, labels and checksums == the oracle's,
    three calls in a row (reused buffers), in 1-3 query parts (each part's report text placed at
    the previous part's device-side end) or one screen with 2-3 refine ranges (each range's text
    copied on the D2H stream while the next refines); k > 32 falls through to the Python
    pipeline."""
    from distributed_machine_learning_project_amd import _lib
    from distributed_machine_learning_project_amd.utils.shm import share_input
    _lib.lib().dmlp_fast_step_parts(parts)
    _lib.lib().dmlp_fast_step_rparts(rparts)
    inp = dmlp.generate(7000, 9000 + 37 * parts + 101 * rparts, 32, 0.0, 1000.0, 1, kmax, 8,
                        seed=kmax + parts + 10 * rparts)
    d, i = K.knn_cpu(inp.X, inp.Qx, inp.k)
    lab_ref, cs = K.finalize_cpu(i, inp.k, inp.labels)
    eng = _engine("farm")
    sh = share_input(eng.comm, inp)
    for _ in range(3):
        n0 = K.FAST_STEP_CALLS[0]
        out = eng.KNN(sh.params, sh, None)
        assert bytes(eng.report(out)) == dmlp.format_report(cs)
        np.testing.assert_array_equal(out.labels_np(), lab_ref)
        np.testing.assert_array_equal(out.checksums_np(), cs)
        assert (K.FAST_STEP_CALLS[0] == n0 + 1) == fast
    sh.close()
    eng.close()
    _lib.lib().dmlp_fast_step_parts(0)
    _lib.lib().dmlp_fast_step_rparts(0)


@pytest.mark.parametrize("n,kmax", [(2000, 16), (5000, 32)])
def test_native_fast_step_early(gpu, n, kmax):
    """Early start (DMLP_FAST_EARLY): the screen starts on the query operands while the dataset
    image crosses PCIe in 4 slices with ready words, each column's eps growing with the slices
    it has seen.  It needs one screen slice (>= 131072 queries fill the chip at S = 1); the
    report, labels and checksums == the oracle's over three calls, and == the default path."""
    from distributed_machine_learning_project_amd import _lib
    from distributed_machine_learning_project_amd.utils.shm import share_input
    inp = dmlp.generate(n, 131072 + 64 * 3, 32, 0.0, 1000.0, 1, kmax, 8, seed=n + kmax)
    d, i = K.knn_cpu(inp.X, inp.Qx, inp.k)
    lab_ref, cs = K.finalize_cpu(i, inp.k, inp.labels)
    expect = dmlp.format_report(cs)
    eng = _engine("farm")
    sh = share_input(eng.comm, inp)
    try:
        for early in (1, 0, 1):
            _lib.lib().dmlp_fast_step_early(early)
            for _ in range(2 if early else 1):
                n0 = K.FAST_STEP_CALLS[0]
                out = eng.KNN(sh.params, sh, None)
                assert bytes(eng.report(out)) == expect
                np.testing.assert_array_equal(out.labels_np(), lab_ref)
                np.testing.assert_array_equal(out.checksums_np(), cs)
                assert K.FAST_STEP_CALLS[0] == n0 + 1
    finally:
        _lib.lib().dmlp_fast_step_early(-1)
        sh.close()
        eng.close()


def test_debug_listing(gpu, workload):
    inp, _, d, i = workload
    eng = _engine("ring", debug=True)
    out = eng.KNN(inp.params, inp, None)
    lab, _ = K.finalize_cpu(i, inp.k, inp.labels)
    assert bytes(eng.report(out)) == dmlp.format_debug(d, i, inp.k, lab)
    eng.close()
