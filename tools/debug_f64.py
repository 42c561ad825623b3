"""Debug the exact path's fp64 screen: run it screen-only on a small case and compare each
query's candidates with the true top-k (numpy fp64)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["DMLP_EXACT_F64_SCREEN_ONLY"] = "1"
import numpy as np  # noqa: E402
import torch  # noqa: E402

import distributed_machine_learning_project_amd as dmlp  # noqa: E402
from distributed_machine_learning_project_amd import _lib  # noqa: E402
from distributed_machine_learning_project_amd.ops import knn as K  # noqa: E402

L = _lib.lib()
N, Q, A, kmin, kmax = [int(v) for v in (sys.argv[1:6] if len(sys.argv) > 5 else (3000, 130, 32, 1, 16))]
inp = dmlp.generate(N, Q, A, 0.0, 1000.0, kmin, kmax, 5, seed=N + A + kmax)
lay = (C.c_int64 * 8)()
L.dmlp_exact_f64_layout(N, A, Q, kmax, lay)
S, tps, cap = lay[0], lay[1], lay[2]
print("S", S, "tps", tps, "cap", cap)
nb = int(L.dmlp_exact_f64_bytes(N, A, Q, kmax))
ws = torch.zeros(nb, dtype=torch.uint8, device="cuda")
X = torch.from_numpy(inp.X).cuda()
Qx = torch.from_numpy(inp.Qx).cuda()
qi = torch.arange(Q, dtype=torch.int32, device="cuda")
kd = torch.from_numpy(inp.k).cuda()
od = torch.zeros(Q * kmax, dtype=torch.float64, device="cuda")
oi = torch.zeros(Q * kmax, dtype=torch.int32, device="cuda")
st = torch.zeros(Q, dtype=torch.int32, device="cuda")
ov = torch.zeros(1, dtype=torch.int32, device="cuda")
rc = L.dmlp_exact_f64(X.data_ptr(), N, A, Qx.data_ptr(), qi.data_ptr(), kd.data_ptr(), Q, kmax,
                      od.data_ptr(), oi.data_ptr(), kmax, st.data_ptr(), ov.data_ptr(),
                      ws.data_ptr(), nb, torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
print("rc", rc)
w = ws.cpu().numpy()
ids = w[lay[3]:lay[3] + Q * S * cap * 4].view(np.int32).reshape(Q, S, cap)
cnt = w[lay[4]:lay[4] + Q * S * 4].view(np.int32).reshape(Q, S)
ch = w[lay[5]:lay[5] + Q * S * 8].view(np.float32).reshape(Q, S, 2)
xn = w[lay[6]:lay[6] + 8].view(np.float64)[0]
mu = w[lay[7]:lay[7] + A * 8].view(np.float64)
print("xnmax", xn, "mu[:3]", mu[:3])
xs = inp.X - mu
qs = inp.Qx - mu
print("xn check", (xs ** 2).sum(1).max())
_, iref = K.knn_cpu(inp.X, inp.Qx, inp.k)
bad = 0
for q in range(min(Q, 40)):
    k = int(inp.k[q])
    sc = qs[q] @ xs.T - 0.5 * (xs ** 2).sum(1)
    true = iref[q, :k]
    groups = set()
    for s in range(S):
        n = cnt[q, s]
        for j in range(max(n, 0)):
            e = int(ids[q, s, j]) & 0xffffffff
            groups.add(s * tps * 16 + (e & 0xffff))
    miss = [int(t) for t in true if (t // 4) not in groups]
    if miss or q < 2:
        print(f"q{q} k{k} cnt {cnt[q].tolist()[:8]}... h {ch[q, :4, 0]} eps {ch[q, 0, 1]:.3g} "
              f"groups {len(groups)} missing {miss} true-scores-min {sc[true].min():.6g} "
              f"kth-score {np.sort(sc)[-k]:.6g}")
        if miss:
            for t in miss[:3]:
                s_ = (t // 64) // tps
                print(f"   point {t} score {sc[t]:.6g} slice {s_} cnt {cnt[q, s_]} h {ch[q, s_, 0]:.6g}")
        bad += bool(miss)
print("queries with missing true neighbours:", bad)
