"""Per-rank compute backend used by the strategies: the HIP pipeline on MI355X, the native C++
pipeline on CPU.  Same API, torch tensors on the rank's device in and out."""
from __future__ import annotations

import numpy as np

from ..ops import knn as K


def _torch():
    import torch
    return torch


class Backend:
    def __init__(self, device, exact: bool = False, cpu_method: str = "brute"):
        self.device = device
        self.exact = exact
        self.cpu_method = cpu_method

    @property
    def on_gpu(self):
        return self.device.type == "cuda"

    def tensor(self, a, dtype=None):
        torch = _torch()
        if isinstance(a, np.ndarray):
            t = torch.from_numpy(np.ascontiguousarray(a))
        else:
            t = a
        if dtype is not None and t.dtype != dtype:
            t = t.to(dtype)
        return t.to(self.device, non_blocking=True)

    # ------------------------------------------------------------------ local k-NN
    def knn(self, X, Qx, k_host: np.ndarray, labels=None, label_range=(0, 1), kstride=None,
            finalize=True):
        """Exact local top-k.  Returns (dist [Q,ks] f64, ids [Q,ks] i32, label [Q] | None,
        checksum [Q] i64 | None) as tensors on this rank's device.  ids are row indices of X."""
        torch = _torch()
        if self.on_gpu:
            ds = K.prepare_dataset(X, labels if finalize else None, label_range)
            r = K.knn_gpu(ds, Qx, k_host, finalize=finalize, exact=self.exact, kstride=kstride)
            return r.dist, r.ids, r.label, r.checksum
        Xn = X.numpy()
        Qn = Qx.numpy()
        d, i = K.knn_cpu(Xn, Qn, k_host, kstride=kstride, method=self.cpu_method)
        lab = cs = None
        if finalize and labels is not None:
            l, c = K.finalize_cpu(i, k_host, labels.numpy())
            lab, cs = torch.from_numpy(l), torch.from_numpy(c.view(np.int64))
        return torch.from_numpy(d), torch.from_numpy(i), lab, cs

    def step(self, X_host, labels_host, label_range, Q_host, k_host, **kw):
        """One rank's whole call from host rows on the GPU (ops.knn.step: libdmlp's native
        pipeline, report text included)."""
        if not self.on_gpu:
            raise RuntimeError("the native step needs a GPU")
        return K.step(X_host, labels_host, label_range, Q_host, k_host, exact=self.exact, **kw)

    def knn_streamed(self, X_host, labels_host, label_range, Qx, k_host: np.ndarray,
                     chunk_rows: int, kstride=None):
        """Exact k-NN with the dataset left in host memory and processed chunk_rows rows at a
        time (out-of-core: datasets beyond one device's memory), running top-k lists merged
        after every chunk.  Returns (dist, ids, label, checksum) like knn()."""
        torch = _torch()
        if self.on_gpu:
            return K.knn_gpu_streamed(X_host, labels_host, label_range, Qx, k_host, chunk_rows,
                                      kstride=kstride, exact=self.exact)
        N = X_host.shape[0]
        dr = ir = None
        ks = kstride or max(1, int(np.max(k_host)) if len(k_host) else 1)
        for a0 in range(0, max(N, 1), max(1, chunk_rows)):
            a1 = min(N, a0 + chunk_rows)
            d, i, _, _ = self.knn(torch.from_numpy(np.ascontiguousarray(X_host[a0:a1])), Qx,
                                  k_host, finalize=False, kstride=ks)
            i = torch.where(i >= 0, i + a0, i)
            if dr is None:
                dr, ir = d, i
            else:
                dr, ir = self.merge(torch.stack([dr, d]), torch.stack([ir, i]), k_host, ks)
        lab, cs = self.finalize(torch.from_numpy(np.ascontiguousarray(labels_host)), label_range,
                                dr, ir, k_host)
        return dr, ir, lab, cs

    def merge(self, lists_d, lists_i, k_host: np.ndarray, kout: int):
        torch = _torch()
        if self.on_gpu:
            kd = torch.from_numpy(np.ascontiguousarray(k_host, np.int32)).to(self.device)
            return K.merge_gpu(lists_d, lists_i, kd, kout)
        d, i = K.merge_cpu(lists_d.numpy(), lists_i.numpy(), k_host, kout)
        return torch.from_numpy(d), torch.from_numpy(i)

    def finalize(self, labels, label_range, dist, ids, k_host: np.ndarray):
        torch = _torch()
        if self.on_gpu:
            kd = torch.from_numpy(np.ascontiguousarray(k_host, np.int32)).to(self.device)
            return K.finalize_gpu(labels, label_range, dist, ids, kd)
        l, c = K.finalize_cpu(ids.numpy(), k_host, labels.numpy())
        return torch.from_numpy(l), torch.from_numpy(c.view(np.int64))

    def report(self, cs, qid_base: int = 0) -> bytes:
        from ..utils.io import format_report
        if self.on_gpu:
            return K.format_report_gpu(cs, qid_base)
        return format_report(cs.numpy().view(np.uint64), qid_base)
