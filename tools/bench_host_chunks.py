"""Host-side cost of the chunked screen-operand rendering (host_prep.cpp), no GPU:
python tools/bench_host_chunks.py  -> ms per full render at 1 / 4 / 8 chunks."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from distributed_machine_learning_project_amd import _lib  # noqa: E402

L = _lib.lib()
N, Q, A, KT = 100000, 131072, 32, 1
rng = np.random.default_rng(0)
X = rng.uniform(0, 1000, (N, A))
Qx = rng.uniform(0, 1000, (Q, A))
mu = np.empty(A)
nt = (N + 63) // 64
img = np.zeros(nt * 64 * 32, np.uint16)
xin = np.zeros(nt * 64, np.float32)
m = np.zeros(1, np.float32)
qhi = np.zeros((Q, 32), np.uint16)
qn = np.zeros(Q, np.float32)
ts = []
for _ in range(20):
    t0 = time.perf_counter()
    L.dmlp_cpu_center(X.ctypes.data, N, A, mu.ctypes.data)
    ts.append(time.perf_counter() - t0)
print("threads", L.dmlp_host_threads(), "center %.3f ms" % (1e3 * np.median(ts)))
for C in (1, 4, 8):
    ts = []
    for _ in range(20):
        t0 = time.perf_counter()
        for c in range(C):
            L.dmlp_cpu_prep_data_tiles(X.ctypes.data, N, A, mu.ctypes.data, KT, nt * c // C,
                                       nt * (c + 1) // C, img.ctypes.data, xin.ctypes.data,
                                       m.ctypes.data)
        for c in range(C):
            q0, q1 = Q * c // C, Q * (c + 1) // C
            L.dmlp_cpu_prep_queries(Qx[q0:].ctypes.data, q1 - q0, A, mu.ctypes.data, KT,
                                    qhi[q0:].ctypes.data, qn[q0:].ctypes.data)
        ts.append(time.perf_counter() - t0)
    print(C, "chunks: %.3f ms" % (1e3 * np.median(ts)))
