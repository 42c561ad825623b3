#!/usr/bin/env python3
"""K4 merge micro-benchmark: P sorted top-k lists per query -> merged top-k.

    rocprofv3 --kernel-trace --stats -d <dir> -- python3 tools/merge_bench.py [--p 8] [--q 131072]

Lists are random but realistic (sorted by (dist asc, id desc), disjoint ids, as shard lists
are); the first 4096 queries are checked against the CPU merge (ops/knn.py merge_cpu).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from distributed_machine_learning_project_amd.ops import knn as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--p", type=int, default=8)
    ap.add_argument("--q", type=int, default=131072)
    ap.add_argument("--ks", default="16,128")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    for k in (int(x) for x in a.ks.split(",")):
        g = torch.Generator(device="cuda").manual_seed(k)
        d = torch.rand((a.p, a.q, k), generator=g, device="cuda", dtype=torch.float64) * 1e6
        d, _ = torch.sort(d, dim=2)
        ids = (torch.arange(a.p * a.q * k, device="cuda", dtype=torch.int32)
               .reshape(a.p, a.q, k))
        kd = torch.full((a.q,), k, dtype=torch.int32, device="cuda")
        for _ in range(2):
            K.merge_gpu(d, ids, kd, k)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            od, oi = K.merge_gpu(d, ids, kd, k)
        e1.record()
        torch.cuda.synchronize()
        nc = min(a.q, 4096)
        dc, ic = K.merge_cpu(d[:, :nc].cpu().numpy(), ids[:, :nc].cpu().numpy(),
                             kd[:nc].cpu().numpy(), kout=k)
        ok = np.array_equal(ic, oi[:nc].cpu().numpy()) and np.array_equal(dc, od[:nc].cpu().numpy())
        print(f"merge P={a.p} Q={a.q} k={k}: {e0.elapsed_time(e1) / a.iters:.4f} ms/call "
              f"(incl. output fill)  check {'OK' if ok else 'MISMATCH'}", flush=True)


if __name__ == "__main__":
    main()
