#!/usr/bin/env python3
"""Candidate-count diagnostics of the single-term screen on a few input shapes.

    python tools/debug_x1.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import distributed_machine_learning_project_amd as dmlp  # noqa: E402
from distributed_machine_learning_project_amd import _lib  # noqa: E402
from distributed_machine_learning_project_amd.ops import knn as K  # noqa: E402


def run(name, inp):
    L = _lib.lib()
    X = torch.from_numpy(inp.X).cuda()
    Qx = torch.from_numpy(inp.Qx).cuda()
    ds = K.prepare_dataset(X, None)
    Q, A = inp.Qx.shape
    KT = ds.KT
    kk = np.minimum(inp.k, ds.N).astype(np.int32)
    qhi = torch.empty(Q * KT * 32, dtype=torch.int16, device="cuda")
    qlo = torch.empty_like(qhi)
    qn = torch.empty(Q, dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    _lib.check(L.dmlp_prep_queries(Qx.data_ptr(), Q, A, ds.mu.data_ptr(), KT, qhi.data_ptr(),
                                   qlo.data_ptr(), qn.data_ptr(), ds.bad.data_ptr(), s), "prep")
    kmax = int(kk.max())
    cap = L.dmlp_screen_x1_cap(kmax)
    S = 1
    qidx = torch.arange(Q, dtype=torch.int32, device="cuda")
    kd = torch.from_numpy(kk).cuda()
    ci = torch.empty(Q * S * cap, dtype=torch.int32, device="cuda")
    cc = torch.empty(Q * S, dtype=torch.int32, device="cuda")
    _lib.check(L.dmlp_screen_x1(KT, A, ds.xfrag.data_ptr(), ds.xinit.data_ptr(), ds.n_tiles, ds.N,
                                qhi.data_ptr(), qn.data_ptr(), qidx.data_ptr(), kd.data_ptr(), Q,
                                kmax, ds.xnmax_bits.data_ptr(), ds.bad.data_ptr(), S,
                                ci.data_ptr(), cc.data_ptr(), s), "x1")
    torch.cuda.synchronize()
    import ctypes
    r1, r2 = ctypes.c_float(), ctypes.c_float()
    L.dmlp_screen_x1_bound(A, ctypes.byref(r1), ctypes.byref(r2))
    xn = ds.xnmax_bits.view(torch.float32).item()
    c = cc.cpu().numpy()
    print(f"{name}: N={ds.N} A={A} Q={Q} cap={cap} r1={r1.value:.3g} r2={r2.value:.3g} "
          f"xnmax={xn:.4g} qn[0]={qn[0].item():.4g}")
    print(f"   cand_cnt: min {c.min()} mean {c[c >= 0].mean() if (c >= 0).any() else -1:.1f} "
          f"max {c.max()} overflow {(c < 0).sum()}")
    # true candidates within the bound for query 0
    Xc = inp.X - ds.mu.cpu().numpy()
    q0 = inp.Qx[0] - ds.mu.cpu().numpy()
    a = Xc @ q0 - (Xc ** 2).sum(1) / 2
    ak = np.sort(a)[-kk[0]]
    eps = r1.value * np.sqrt(qn[0].item()) * np.sqrt(xn) + r2.value * xn
    print(f"   q0: k={kk[0]} a_k={ak:.6g} eps={eps:.4g} points >= a_k-2eps: "
          f"{(a >= ak - 2 * eps).sum()}  got {c[0]}")


def main():
    run("bench", dmlp.generate(20000, 512, 32, 0.0, 1000.0, 16, 16, 10, seed=12))
    run("dense1d", dmlp.generate(20000, 128, 1, 0.0, 1000.0, 8, 16, 4, seed=2))


if __name__ == "__main__":
    main()
