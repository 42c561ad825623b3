"""Pure NumPy float64 oracle of the reference semantics (test pyramid level 1).

Independent of the native library: used by the tests to pin the C++/HIP implementations.
  distance: s = 0; for a: d = q[a] - X[:, a]; s = s + d*d   (sequential, separately rounded;
            NumPy elementwise ops never contract into FMA)        — engine.cpp:12-18
  order:    lexsort by (dist asc, id desc)                         — bench_1 @0xe018
  vote:     max count, ties -> larger label, empty -> -1           — engine.cpp:319-332
  checksum: FNV-1a 64 over label then id+1                          — common.cpp:59-70
"""
from __future__ import annotations

import numpy as np

FNV_OFFSET = 1469598103934665603
FNV_PRIME = 1099511628211
MASK = (1 << 64) - 1


def distances(X: np.ndarray, q: np.ndarray) -> np.ndarray:
    s = np.zeros(X.shape[0], dtype=np.float64)
    for a in range(X.shape[1]):
        d = q[a] - X[:, a]
        s = s + d * d
    return s


def topk(X: np.ndarray, q: np.ndarray, k: int):
    d = distances(X, q)
    ids = np.arange(X.shape[0])
    order = np.lexsort((-ids, d))[:k]
    return d[order], ids[order].astype(np.int64)


def vote(ids, labels) -> int:
    if len(ids) == 0:
        return -1
    vals, counts = np.unique(labels[np.asarray(ids)], return_counts=True)
    best = counts.max()
    return int(vals[counts == best].max())


def checksum(label: int, ids) -> int:
    h = FNV_OFFSET
    h = ((h ^ (label & MASK)) * FNV_PRIME) & MASK
    for i in ids:
        h = ((h ^ ((int(i) + 1) & MASK)) * FNV_PRIME) & MASK
    return h


def knn(X, labels, Qx, ks):
    """Returns (list of (dists, ids)), labels_pred [Q], checksums [Q] (uint64)."""
    res, lab, cs = [], [], []
    for qi in range(Qx.shape[0]):
        d, ids = topk(X, Qx[qi], int(ks[qi]))
        lb = vote(ids, labels)
        res.append((d, ids))
        lab.append(lb)
        cs.append(checksum(lb, ids))
    return res, np.array(lab, dtype=np.int32), np.array(cs, dtype=np.uint64)


def report_lines(checksums) -> str:
    return "".join(f"Query {i} checksum: {int(c)}\n" for i, c in enumerate(checksums))
