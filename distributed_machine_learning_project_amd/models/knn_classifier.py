"""Model front-ends: an estimator-style exact k-NN classifier and the serial KD-tree.

    clf = KNNClassifier().fit(X, y)          # X [N, A] float64, y [N] int
    dist, ids = clf.kneighbors(Q, k)         # k: int or per-query array
    labels = clf.predict(Q, k)               # majority vote, ties -> larger label
    cs = clf.checksums(Q, k)                 # reference FNV-1a report checksums

Semantics are the reference's: exact fp64 squared-L2 distances summed left to
right without FMA, neighbours ordered by (distance asc, id desc).  On a GPU the dataset is
prepared once at fit() (fp64 copy + bf16x3 MFMA fragments) and reused by every query batch;
on a CPU the native threaded brute force (or the KD-tree) runs.
"""
from __future__ import annotations

import numpy as np

from ..ops import knn as K


def _torch():
    import torch
    return torch


class KNNClassifier:
    def __init__(self, device: str = "auto", exact: bool = False, cpu_method: str = "brute"):
        torch = _torch()
        self.on_gpu = device == "gpu" or (device == "auto" and torch.cuda.is_available())
        self.exact = exact
        self.cpu_method = cpu_method
        self._ds = None

    def fit(self, X, y):
        self.X = np.ascontiguousarray(X, np.float64)
        self.y = np.ascontiguousarray(y, np.int32)
        if self.X.ndim != 2 or self.y.shape[0] != self.X.shape[0]:
            raise ValueError("X must be [N, A] and y [N]")
        if self.on_gpu:
            torch = _torch()
            lo = int(self.y.min()) if len(self.y) else 0
            hi = int(self.y.max()) + 1 if len(self.y) else 1
            self._ds = K.prepare_dataset(torch.from_numpy(self.X).cuda(),
                                         torch.from_numpy(self.y).cuda(), (lo, hi))
        return self

    def update(self, updates):
        """Apply Update records (common.h:22-25) to the fitted dataset: rows are replaced in the
        host copy and, on a GPU, scattered into the device copy, after which the screen layout
        (centering, bf16 fragments, norms) is rebuilt so later queries stay exact."""
        updates = list(updates)
        if not updates:
            return self
        for u in updates:
            if not 0 <= u.id < self.X.shape[0] or len(u.new_attrs) != self.X.shape[1]:
                raise ValueError(f"update {u.id}: id out of range or wrong attribute count")
            self.X[u.id] = np.asarray(u.new_attrs, np.float64)
        if self.on_gpu:
            torch = _torch()
            ids = np.array(sorted({u.id for u in updates}), np.int64)
            Xd = self._ds.X
            Xd[torch.from_numpy(ids).to(Xd.device)] = torch.from_numpy(self.X[ids]).to(Xd.device)
            self._ds = K.prepare_dataset(Xd, self._ds.labels, (self._ds.label_lo, self._ds.label_hi))
        return self

    def _k(self, Q, k):
        if np.isscalar(k):
            return np.full(Q.shape[0], int(k), np.int32)
        return np.ascontiguousarray(k, np.int32)

    def _run(self, Q, k, finalize):
        Q = np.ascontiguousarray(Q, np.float64)
        kk = self._k(Q, k)
        if self.on_gpu:
            torch = _torch()
            r = K.knn_gpu(self._ds, torch.from_numpy(Q).cuda(), kk, finalize=finalize,
                          exact=self.exact)
            d, i = r.dist.cpu().numpy(), r.ids.cpu().numpy()
            lab = r.label.cpu().numpy() if r.label is not None else None
            cs = r.checksum.cpu().numpy().view(np.uint64) if r.checksum is not None else None
            return d, i, lab, cs, kk
        d, i = K.knn_cpu(self.X, Q, kk, method=self.cpu_method)
        lab = cs = None
        if finalize:
            lab, cs = K.finalize_cpu(i, kk, self.y)
        return d, i, lab, cs, kk

    def kneighbors(self, Q, k):
        """(dist [Q, kmax], ids [Q, kmax]); row q is valid up to k_q, padded with (+inf, -1)."""
        d, i, _, _, _ = self._run(Q, k, finalize=False)
        return d, i

    def predict(self, Q, k):
        return self._run(Q, k, finalize=True)[2]

    def checksums(self, Q, k):
        return self._run(Q, k, finalize=True)[3]


class KDTree:
    """Serial exact KD-tree (bench.debug B0): median split on axis depth % A, near side first,
    far side visited when the split-plane bound can still tie the current k-th distance."""

    def __init__(self, X):
        self.X = np.ascontiguousarray(X, np.float64)

    def query(self, Q, k):
        Q = np.ascontiguousarray(Q, np.float64)
        kk = np.full(Q.shape[0], int(k), np.int32) if np.isscalar(k) else np.asarray(k, np.int32)
        return K.knn_cpu(self.X, Q, kk, method="kdtree")
