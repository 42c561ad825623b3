"""Model front-end API (CPU path; the GPU path shares ops.knn, covered in test_gpu_kernels)."""
import numpy as np

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
