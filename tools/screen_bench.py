"""Micro-benchmark of the single-term screen (screen_x1.hip k_screen_x1) exactly as the native
step runs it at the bench shape: the host's fp16 operands (host_prep.cpp), one data slice,
every query in one launch — timed alone with hipEvents over rounds, and checked end to end: the
native step's whole report == the fp64 oracle's.

    python tools/screen_bench.py --rounds 3 --iters 20
"""
import argparse
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import distributed_machine_learning_project_amd as dmlp  # noqa: E402
from distributed_machine_learning_project_amd import _lib  # noqa: E402
from distributed_machine_learning_project_amd.ops import knn as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100000)
    ap.add_argument("--q", type=int, default=131072)
    ap.add_argument("--a", type=int, default=32)
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--verify", type=int, default=1)
    ap.add_argument("--early", type=int, default=0,
                    help="1: the early-start entry (dmlp_screen_x1_early) with every slice ready")
    a = ap.parse_args()
    L = _lib.lib()
    inp = dmlp.generate(a.n, a.q, a.a, 0.0, 1000.0, a.k, a.k, 10, seed=42)
    N, Q, A = a.n, a.q, a.a
    KT = K.screen_kt(A)
    W = KT * 32
    nt = (N + 63) // 64
    mu = np.empty(A)
    L.dmlp_cpu_center(inp.X.ctypes.data, min(N, 4096), A, mu.ctypes.data)
    xhi = np.zeros(nt * 64 * W, np.uint16)
    xin = np.zeros(nt * 64, np.float32)
    xnm = np.zeros(1, np.uint32)
    assert L.dmlp_cpu_prep_data(inp.X.ctypes.data, N, A, mu.ctypes.data, KT, xhi.ctypes.data,
                                xin.ctypes.data, xnm.ctypes.data) == 0
    qhi = np.zeros(Q * W, np.uint16)
    qn = np.zeros(Q, np.float32)
    assert L.dmlp_cpu_prep_queries(inp.Qx.ctypes.data, Q, A, mu.ctypes.data, KT, qhi.ctypes.data,
                                   qn.ctypes.data) == 0
    dev = "cuda"
    d_xhi = torch.from_numpy(xhi.view(np.int16)).to(dev)
    d_xin = torch.from_numpy(xin).to(dev)
    d_words = torch.from_numpy(np.array([xnm[0], 0], np.uint32).view(np.int32)).to(dev)
    d_qhi = torch.from_numpy(qhi.view(np.int16)).to(dev)
    d_qn = torch.from_numpy(qn).to(dev)
    d_k = torch.from_numpy(inp.k).to(dev)
    d_qi = torch.arange(Q, dtype=torch.int32, device=dev)
    cap = L.dmlp_screen_x1_cap_kt(KT, a.k)
    S = 1
    ci = torch.empty(Q * S * cap, dtype=torch.int32, device=dev)
    cc = torch.empty(Q * S, dtype=torch.int32, device=dev)
    ch = torch.empty(Q * S * 2, dtype=torch.float32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    wp = d_words.data_ptr()

    NS = 8
    rt = (nt + NS - 1) // NS
    # every slice "landed": its ready word carries the image's max norm bits (nonzero)
    rdy = torch.from_numpy(np.full(NS, max(int(xnm[0]), 1), np.uint32).view(np.int32)).to(dev)
    est = torch.zeros(4, dtype=torch.int32, device=dev)

    def launch():
        if a.early:
            rc = L.dmlp_screen_x1_early(KT, A, d_xhi.data_ptr(), d_xin.data_ptr(), nt, N,
                                        d_qhi.data_ptr(), d_qn.data_ptr(), d_qi.data_ptr(),
                                        d_k.data_ptr(), Q, a.k, wp + 4, rdy.data_ptr(), rt, NS,
                                        ci.data_ptr(), cc.data_ptr(), ch.data_ptr(),
                                        est.data_ptr(), s)
        else:
            rc = L.dmlp_screen_x1(KT, 1, A, d_xhi.data_ptr(), d_xin.data_ptr(), nt, N,
                                  d_qhi.data_ptr(), d_qn.data_ptr(), d_qi.data_ptr(),
                                  d_k.data_ptr(), Q, a.k, wp, wp + 4, S, ci.data_ptr(),
                                  cc.data_ptr(), ch.data_ptr(), s)
        assert rc == 0, rc

    res = []
    expect = None
    if a.verify:
        _, i = K.knn_cpu(inp.X, inp.Qx, inp.k)
        _, cs = K.finalize_cpu(i, inp.k, inp.labels)
        expect = dmlp.format_report(cs)
        dst = torch.empty(48 * Q + 64, dtype=torch.uint8).pin_memory().numpy()
    for rnd in range(a.rounds):
        launch()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.iters)]
        for it in range(a.iters):
            ev[2 * it].record()
            launch()
            ev[2 * it + 1].record()
        torch.cuda.synchronize()
        res += [ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(a.iters)]
        if a.verify and rnd == 0:
            r = K.step(inp.X, inp.labels, (0, 10), inp.Qx, inp.k, report=dst)
            ok = bytes(dst[:r.report_len]) == expect
            print(f"native step report == oracle: {ok} (path {r.path}, early {r.early}, "
                  f"escalated {r.n_escalated})", flush=True)
            assert ok
    v = np.array(res)
    print(f"k_screen_x1 median {np.median(v):.4f} ms  p10 {np.percentile(v, 10):.4f}"
          f"  p90 {np.percentile(v, 90):.4f}  (n={len(v)})", flush=True)


if __name__ == "__main__":
    main()
