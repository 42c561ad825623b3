"""Model front-end API (CPU path; the GPU path shares ops.knn, covered in test_gpu_kernels)."""
import numpy as np
import pytest

from distributed_machine_learning_project_amd.models import KDTree, KNNClassifier
from distributed_machine_learning_project_amd.ops import reference as ref


def test_classifier_cpu_matches_oracle():
    rng = np.random.default_rng(0)
    X = np.round(rng.uniform(0, 10, (300, 4)), 2)
    y = rng.integers(0, 4, 300)
    Q = np.round(rng.uniform(0, 10, (20, 4)), 2)
    k = rng.integers(1, 30, 20)
    clf = KNNClassifier(device="cpu").fit(X, y)
    d, i = clf.kneighbors(Q, k)
    lab = clf.predict(Q, k)
    cs = clf.checksums(Q, k)
    res, lab_o, cs_o = ref.knn(X, y.astype(np.int32), Q, k)
    for q in range(20):
        np.testing.assert_array_equal(i[q, :k[q]], res[q][1])
    np.testing.assert_array_equal(lab, lab_o)
    np.testing.assert_array_equal(cs, cs_o)
    dk, ik = KDTree(X).query(Q, 5)
    d5, i5 = clf.kneighbors(Q, 5)
    np.testing.assert_array_equal(ik, i5)
    np.testing.assert_array_equal(dk, d5)


def _update_case(device):
    from distributed_machine_learning_project_amd import Update, parse_update
    rng = np.random.default_rng(3)
    X = np.round(rng.uniform(0, 10, (500, 6)), 3)
    y = rng.integers(0, 5, 500).astype(np.int32)
    Q = np.round(rng.uniform(0, 10, (40, 6)), 3)
    k = rng.integers(1, 20, 40)
    clf = KNNClassifier(device=device).fit(X, y)
    # move 30 points onto the queries: they must become the nearest neighbours
    ups = [Update(int(i), list(Q[j % 40] + 1e-3)) for j, i in enumerate(rng.choice(500, 30, False))]
    ups.append(parse_update(f"7 {' '.join(['5.5'] * 6)}"))
    assert ups[-1].id == 7 and ups[-1].new_attrs == [5.5] * 6
    clf.update(ups)
    X2 = X.copy()
    for u in ups:
        X2[u.id] = u.new_attrs
    res, lab_o, cs_o = ref.knn(X2, y, Q, k)
    np.testing.assert_array_equal(clf.checksums(Q, k), cs_o)
    np.testing.assert_array_equal(clf.predict(Q, k), lab_o)
    with pytest.raises(ValueError):
        clf.update([Update(10**6, [0.0] * 6)])


def test_classifier_update_cpu():
    _update_case("cpu")


@pytest.mark.gpu
def test_classifier_update_gpu():
    _update_case("gpu")


@pytest.mark.gpu
def test_classifier_gpu_matches_oracle():
    rng = np.random.default_rng(1)
    X = np.round(rng.uniform(-50, 50, (3000, 20)), 4)
    y = rng.integers(0, 7, 3000).astype(np.int32)
    Q = np.round(rng.uniform(-50, 50, (500, 20)), 4)
    k = rng.integers(1, 150, 500)
    clf = KNNClassifier(device="gpu").fit(X, y)
    res, lab_o, cs_o = ref.knn(X, y, Q, k)
    np.testing.assert_array_equal(clf.checksums(Q, k), cs_o)
    d, i = clf.kneighbors(Q, k)
    for q in range(0, 500, 37):
        np.testing.assert_array_equal(i[q, :k[q]], res[q][1])
        np.testing.assert_array_equal(d[q, :k[q]], res[q][0])


def test_shared_segment_summary(tmp_path):
    """The node-shared segment's header carries (label lo, label hi, k min, k max), written once
    with the arrays and read by every KNN call instead of scanning them."""
    import numpy as np
    from distributed_machine_learning_project_amd.utils.io import generate
    from distributed_machine_learning_project_amd.utils.shm import SharedInput
    inp = generate(500, 300, 4, 0.0, 10.0, 2, 9, 5, seed=3)
    s = SharedInput.create(inp, directory=str(tmp_path))
    try:
        assert s.summary == (int(inp.labels.min()), int(inp.labels.max()) + 1,
                             int(inp.k.min()), int(inp.k.max()))
        t = SharedInput.attach(s.path)
        assert t.summary == s.summary
        s.k[7] = 31
        s.refresh_summary()
        assert t.summary[3] == 31
        np.testing.assert_array_equal(t.X, inp.X)
    finally:
        s.close()
