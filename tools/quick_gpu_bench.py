"""Single-GPU micro benchmark of the local KNN pipeline phases (no distribution).

    python tools/quick_gpu_bench.py --n 100000 --q 100000 --a 32 --k 16
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import distributed_machine_learning_project_amd as dmlp  # noqa: E402
from distributed_machine_learning_project_amd.ops import knn as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100000)
    ap.add_argument("--q", type=int, default=100000)
    ap.add_argument("--a", type=int, default=32)
    ap.add_argument("--kmin", type=int, default=16)
    ap.add_argument("--kmax", type=int, default=16)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--exact", action="store_true")
    ap.add_argument("--check", type=int, default=200, help="queries to verify against CPU")
    ap.add_argument("--modes", type=str, default="",
                    help="comma list of screen ablation modes to time (profiling only)")
    a = ap.parse_args()
    if a.modes:
        from distributed_machine_learning_project_amd import _lib
        inp = dmlp.generate(a.n, a.q, a.a, 0.0, 1000.0, a.kmin, a.kmax, 10, seed=42)
        X = torch.from_numpy(inp.X).cuda()
        lab = torch.from_numpy(inp.labels).cuda()
        Qx = torch.from_numpy(inp.Qx).cuda()
        for m in [int(x) for x in a.modes.split(",")]:
            _lib.lib().dmlp_set_screen_mode(m)
            _lib.lib().dmlp_set_stream_mode(m)
            ts = []
            for it in range(a.iters + 1):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                ds = K.prepare_dataset(X, lab, (0, 10))
                K.knn_gpu(ds, Qx, inp.k)
                e1.record()
                torch.cuda.synchronize()
                if it:
                    ts.append(e0.elapsed_time(e1))
            print(f"mode {m}: {np.median(ts):.3f} ms")
            if m & 16:
                c2 = np.zeros(8, np.uint64)
                _lib.lib().dmlp_stream_debug_counters(c2.ctypes.data, 1)
                calls = a.iters + 1
                tl, tcp, tap = (float(x) / calls for x in c2[4:7])
                print("  cycles/call (summed over waves): loop %.4g  compaction %.4g (%.1f%%)  "
                      "appends %.4g (%.1f%%)" % (tl, tcp, 100 * tcp / max(tl, 1), tap,
                                                 100 * tap / max(tl, 1)))
            if m & 8:
                cnt = np.zeros(8, np.uint64)
                _lib.lib().dmlp_screen_debug_counters(cnt.ctypes.data, 1)
                c2 = np.zeros(8, np.uint64)
                _lib.lib().dmlp_stream_debug_counters(c2.ctypes.data, 1)
                cnt += c2
                calls = a.iters + 1
                print("  per call: wave-steps %.4g  cand-path %.4g  appends %.4g  compactions %.4g"
                      % tuple(float(x) / calls for x in cnt[:4]))
        _lib.lib().dmlp_set_screen_mode(0)
        _lib.lib().dmlp_set_stream_mode(0)
        return
    inp = dmlp.generate(a.n, a.q, a.a, 0.0, 1000.0, a.kmin, a.kmax, 10, seed=42)
    X = torch.from_numpy(inp.X).cuda()
    lab = torch.from_numpy(inp.labels).cuda()
    Qx = torch.from_numpy(inp.Qx).cuda()
    times = []
    for it in range(a.iters + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ds = K.prepare_dataset(X, lab, (0, 10))
        r = K.knn_gpu(ds, Qx, inp.k, exact=a.exact)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if it:
            times.append(t1 - t0)
    ms = 1e3 * float(np.median(times))
    print(f"N={a.n} Q={a.q} A={a.a} k=[{a.kmin},{a.kmax}] exact={a.exact}: {ms:.3f} ms "
          f"-> {a.q / ms * 1e3:.0f} queries/s  fallback={r.n_fallback} "
          f"escalated={r.n_escalated}")
    if a.check:
        nc = min(a.check, a.q)
        d_ref, i_ref = K.knn_cpu(inp.X, inp.Qx[:nc], inp.k[:nc], kstride=r.ids.shape[1])
        ids = r.ids[:nc].cpu().numpy()
        ok = all((ids[q, :inp.k[q]] == i_ref[q, :inp.k[q]]).all() for q in range(nc))
        print("check vs CPU:", "OK" if ok else "MISMATCH")


if __name__ == "__main__":
    main()
