"""Host query-prep throughput (host_prep.cpp): python tools/bench_host_prep.py"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, time, os
from distributed_machine_learning_project_amd import _lib
L=_lib.lib()
rng=np.random.default_rng(0)
Q,A,KT=131072,32,1
Qx=rng.uniform(0,1000,(Q,A)); mu=np.full(A,500.0)
qhi=np.zeros((Q,KT*32),np.uint16); qn=np.zeros(Q,np.float32)
ts=[]
for _ in range(10):
    t=time.perf_counter(); L.dmlp_cpu_prep_queries(Qx.ctypes.data,Q,A,mu.ctypes.data,KT,qhi.ctypes.data,qn.ctypes.data); ts.append(time.perf_counter()-t)
print(os.environ.get("DMLP_HOST_THREADS"), "threads", L.dmlp_host_threads(), "min ms %.3f med %.3f" % (min(ts)*1e3, np.median(ts)*1e3))
