"""CPU implementations against the independent NumPy oracle (SURVEY.md §4 level 1) and the
input/output contract of the reference harness (common.cpp, generate_input.py)."""
import numpy as np
import pytest

import distributed_machine_learning_project_amd as dmlp
from distributed_machine_learning_project_amd.ops import reference as ref
from distributed_machine_learning_project_amd.ops import knn as K


def check_against_oracle(inp, method="brute"):
    d, i = K.knn_cpu(inp.X, inp.Qx, inp.k, method=method)
    lab, cs = K.finalize_cpu(i, inp.k, inp.labels)
    res, lab_o, cs_o = ref.knn(inp.X, inp.labels, inp.Qx, inp.k)
    for q, (do, io) in enumerate(res):
        kq = int(inp.k[q])
        n = min(kq, inp.N)
        np.testing.assert_array_equal(i[q, :n], io[:n])
        np.testing.assert_array_equal(d[q, :n], do[:n])
    np.testing.assert_array_equal(lab, lab_o)
    np.testing.assert_array_equal(cs, cs_o)


@pytest.mark.parametrize("method", ["brute", "kdtree"])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_generated_varying_k(method, seed):
    txt = dmlp.generate_text(300, 25, 6, 0, 100, 1, 40, 5, seed=seed)
    check_against_oracle(dmlp.parse_input(txt), method)


@pytest.mark.parametrize("method", ["brute", "kdtree"])
def test_duplicates_ties(method):
    rng = np.random.default_rng(0)
    base = np.round(rng.uniform(0, 3, size=(10, 3)), 0)
    X = np.ascontiguousarray(base[rng.integers(0, 10, size=400)])
    inp = dmlp.KNNInput(rng.integers(0, 3, 400).astype(np.int32), X,
                        rng.integers(1, 50, 30).astype(np.int32),
                        np.round(rng.uniform(0, 3, size=(30, 3)), 0))
    check_against_oracle(inp, method)


@pytest.mark.parametrize("method", ["brute", "kdtree"])
def test_k_equals_n(method):
    inp = dmlp.generate(60, 5, 4, 0, 1, 60, 60, 4, seed=3)
    check_against_oracle(inp, method)


def test_generate_text_matches_reference_generator():
    """Byte-identical to the reference's generate_input.py for the same arguments and seed."""
    import os
    import subprocess
    import sys
    import tempfile
    refgen = "/root/reference/generate_input.py"
    if not os.path.exists(refgen):
        pytest.skip("reference not mounted")
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "in.txt")
        subprocess.run([sys.executable, refgen, "--num_data", "50", "--num_queries", "7",
                        "--num_attrs", "3", "--min", "-5", "--max", "5", "--minK", "1",
                        "--maxK", "9", "--num_labels", "4", "--output", out, "--seed", "11"],
                       check=True, capture_output=True)
        ref_txt = open(out).read()
    assert dmlp.generate_text(50, 7, 3, -5, 5, 1, 9, 4, seed=11) == ref_txt


def test_parse_roundtrip_and_errors():
    inp = dmlp.generate(40, 6, 5, -3, 3, 1, 5, 3, seed=4)
    txt = dmlp.to_text(inp)
    back = dmlp.parse_input(txt)
    np.testing.assert_array_equal(back.X, inp.X)
    np.testing.assert_array_equal(back.Qx, inp.Qx)
    np.testing.assert_array_equal(back.k, inp.k)
    np.testing.assert_array_equal(back.labels, inp.labels)
    bad = txt.replace("Q ", "X ", 1)
    with pytest.raises(dmlp.utils.io.InputFormatError):
        dmlp.parse_input(bad)


def test_report_format():
    cs = np.array([0, 123, 2**64 - 1], dtype=np.uint64)
    assert dmlp.format_report(cs) == ref.report_lines(cs).encode()


def test_checksum_sentinel_and_empty():
    # label -1 (empty result) and id -1 padding follow common.cpp:59-70 exactly
    assert ref.checksum(-1, []) == ((ref.FNV_OFFSET ^ (2**64 - 1)) * ref.FNV_PRIME) % 2**64
    lab, cs = K.finalize_cpu(np.array([[-1, -1]], np.int32), np.array([2], np.int32),
                             np.array([0], np.int32))
    assert lab[0] == -1 and cs[0] == ref.checksum(-1, [-1, -1])
