"""Node render plane (csrc/plane.cpp) on the CPU: P processes map one node-shared segment, each
renders its 1/P of the dataset slices (fp16 tile image + xinit + max norm, lossless int32 rows,
fp64 rows where the int32 check fails) and publishes them with generation flags; every process
then waits for all slices.  The segment must hold exactly what ONE process rendering the whole
dataset produces (host_prep.cpp), for P = 1, 2, 3 and 8 renderers and across calls with new data
(generations), and a rank whose partner never renders must time out, not hang."""
import ctypes as C
import multiprocessing as mp
import os

import numpy as np
import pytest

from distributed_machine_learning_project_amd import _lib


def _plane(base, nbytes, rank, renderers, gen, with_f64, wait_s=30.0):
    from distributed_machine_learning_project_amd.ops.knn import Plane
    return Plane(base=base, bytes=nbytes, rank=rank, renderers=renderers, with_f64=with_f64,
                 gen=gen, wait_s=wait_s)


def _worker(path, nbytes, rank, renderers, world, N, A, with_f64, calls, q):
    """One rank: per call (new data each call, seeded by the call), render this rank's slices
    (rank 0 also publishes mu), then wait for every slice and report what it saw."""
    L = _lib.lib()
    mm = np.memmap(path, np.uint8, "r+", shape=(nbytes,))
    base = mm.ctypes.data
    out = []
    for gen in range(1, calls + 1):
        X = _data(N, A, gen)
        pl = _plane(base, nbytes, rank, renderers, gen, with_f64)
        mu = np.zeros(A)
        if rank == 0:
            L.dmlp_cpu_center(X.ctypes.data, N, A, mu.ctypes.data)
            assert L.dmlp_plane_put_mu(C.byref(pl), A, mu.ctypes.data) == 0
        else:
            assert L.dmlp_plane_get_mu(C.byref(pl), A, mu.ctypes.data) == 0
        t0, t1 = C.c_int64(), C.c_int64()
        ns = L.dmlp_plane_slice(N, A, 0, C.byref(t0), C.byref(t1))
        if rank < renderers:
            for what in (1, 2):
                for i in range(rank, ns, renderers):
                    assert L.dmlp_plane_render(C.byref(pl), X.ctypes.data, None, N, A,
                                               mu.ctypes.data, what, i) >= 0
        bits = []
        for what in (1, 2):
            for i in range(ns):
                b, nm = C.c_int(), C.c_float()
                assert L.dmlp_plane_wait(C.byref(pl), what, i, C.byref(b), C.byref(nm)) == 0
                bits.append((what, i, b.value, nm.value))
        out.append((gen, bits, mu.tobytes()))
        # the callers separate calls by a barrier of all plane ranks
        q.put(("arrive", rank, gen))
        while True:
            with open(path + f".bar{gen}", "a+") as f:
                f.seek(0)
                if len(f.read()) >= world:
                    break
            import time
            time.sleep(0.001)
    q.put(("done", rank, out))


def _data(N, A, gen):
    rng = np.random.default_rng(100 + gen)
    X = np.round(rng.uniform(0, 1000, (N, A)), 6)
    if gen % 2 == 0:
        X[N // 3] += 1e-7  # one value that is not a 6-decimal number: that slice ships fp64
    return X


def _expected(N, A, gen):
    """One process rendering everything (host_prep.cpp)."""
    L = _lib.lib()
    X = _data(N, A, gen)
    mu = np.zeros(A)
    L.dmlp_cpu_center(X.ctypes.data, N, A, mu.ctypes.data)
    kt = 1 if A <= 32 else 2 if A <= 64 else 4 if A <= 128 else 8
    nt = (N + 63) // 64
    img = np.zeros(nt * 64 * kt * 32, np.uint16)
    xin = np.zeros(nt * 64, np.float32)
    bits = C.c_uint()
    L.dmlp_cpu_prep_data(X.ctypes.data, N, A, mu.ctypes.data, kt, img.ctypes.data,
                         xin.ctypes.data, C.byref(bits))
    return X, mu, img, xin


@pytest.mark.parametrize("N,A,renderers,world", [(5000, 32, 1, 2), (7001, 32, 3, 3),
                                                 (6400, 48, 2, 3), (9000, 32, 8, 8)])
@pytest.mark.parametrize("with_f64", [0, 1])
def test_plane_matches_single_render(tmp_path, N, A, renderers, world, with_f64):
    L = _lib.lib()
    nbytes = int(L.dmlp_plane_bytes(N, A, with_f64))
    path = str(tmp_path / "plane.seg")
    mm = np.memmap(path, np.uint8, "w+", shape=(nbytes,))
    assert L.dmlp_plane_init(mm.ctypes.data, nbytes, N, A, with_f64) == 0
    mm.flush()
    calls = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(path, nbytes, r, renderers, world, N, A, with_f64,
                                               calls, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    arrived = {}
    while len(results) < world:
        kind, rank, val = q.get(timeout=120)
        if kind == "arrive":
            arrived.setdefault(val, 0)
            arrived[val] += 1
            if arrived[val] == world:
                # every rank saw call `val` complete: check the segment, then release the barrier
                _check_segment(L, mm, nbytes, N, A, val, renderers, with_f64)
                with open(path + f".bar{val}", "w") as f:
                    f.write("x" * world)
        else:
            results[rank] = val
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    # every rank saw the same flags, norms and mu each call
    for gen in range(calls):
        views = {r: results[r][gen] for r in range(world)}
        assert len({repr(v[1]) for v in views.values()}) == 1
        assert len({v[2] for v in views.values()}) == 1
        fp64 = [b for what, _, b, _ in views[0][1] if what == 2 and b & 2]
        assert len(fp64) == (1 if (gen + 1) % 2 == 0 else 0)


def _check_segment(L, mm, nbytes, N, A, gen, renderers, with_f64):
    X, mu, img, xin = _expected(N, A, gen)
    pl = _plane(mm.ctypes.data, nbytes, 0, renderers, gen, with_f64)
    pi, px, p32, p64 = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_void_p()
    assert L.dmlp_plane_regions(C.byref(pl), N, A, C.byref(pi), C.byref(px), C.byref(p32),
                                C.byref(p64)) == 0
    seg_img = np.ctypeslib.as_array((C.c_uint16 * img.size).from_address(pi.value))
    seg_xin = np.ctypeslib.as_array((C.c_float * xin.size).from_address(px.value))
    np.testing.assert_array_equal(seg_img, img)
    np.testing.assert_array_equal(seg_xin, xin)
    r32 = np.ctypeslib.as_array((C.c_int32 * (N * A)).from_address(p32.value)).reshape(N, A)
    t0, t1 = C.c_int64(), C.c_int64()
    ns = L.dmlp_plane_slice(N, A, 0, C.byref(t0), C.byref(t1))
    for i in range(ns):
        L.dmlp_plane_slice(N, A, i, C.byref(t0), C.byref(t1))
        r0, r1 = min(N, t0.value * 64), min(N, t1.value * 64)
        b = C.c_int()
        assert L.dmlp_plane_wait(C.byref(pl), 2, i, C.byref(b), None) == 0
        if b.value & 2:
            if with_f64:
                r64 = np.ctypeslib.as_array((C.c_double * (N * A)).from_address(p64.value))
                np.testing.assert_array_equal(r64.reshape(N, A)[r0:r1], X[r0:r1])
        else:
            np.testing.assert_array_equal(r32[r0:r1] / 1e6, X[r0:r1])


def test_plane_wait_times_out(tmp_path):
    """A consumer whose renderer never publishes (or publishes a later generation) fails within
    the plane's wait bound instead of hanging."""
    import time
    L = _lib.lib()
    N, A = 3000, 32
    nbytes = int(L.dmlp_plane_bytes(N, A, 0))
    buf = np.zeros(nbytes, np.uint8)
    assert L.dmlp_plane_init(buf.ctypes.data, nbytes, N, A, 0) == 0
    pl = _plane(buf.ctypes.data, nbytes, 1, 2, gen=1, with_f64=0, wait_s=0.3)
    t = time.monotonic()
    assert L.dmlp_plane_wait(C.byref(pl), 1, 0, None, None) == -4
    assert time.monotonic() - t < 5
    mu = np.zeros(A)
    assert L.dmlp_plane_get_mu(C.byref(pl), A, mu.ctypes.data) == -4
    # a flag of a LATER call (ranks out of step) fails at once
    X = _data(N, A, 1)
    ahead = _plane(buf.ctypes.data, nbytes, 0, 2, gen=5, with_f64=0)
    assert L.dmlp_plane_render(C.byref(ahead), X.ctypes.data, None, N, A, mu.ctypes.data, 1, 0) >= 0
    t = time.monotonic()
    assert L.dmlp_plane_wait(C.byref(pl), 1, 0, None, None) == -4
    assert time.monotonic() - t < 1
    assert L.dmlp_plane_bytes(N, 300, 0) == -1  # beyond the screen's 256 attributes: no plane


def test_shared_segment_falls_back_from_a_small_dev_shm(tmp_path, monkeypatch):
    """utils/shm.py: a segment that does not fit the requested directory (a container's 64 MiB
    /dev/shm) goes to the first roomy candidate ($TMPDIR here) instead of dying of SIGBUS when its
    pages are first written; a segment that fits stays where it was asked."""
    import os
    from distributed_machine_learning_project_amd.utils import shm
    small = tmp_path / "small"
    small.mkdir()
    roomy = tmp_path / "roomy"
    roomy.mkdir()
    real = os.statvfs

    class _St:
        def __init__(self, free):
            self.f_bavail, self.f_frsize = free, 1

    def fake(d):
        if str(d) == str(small):
            return _St(1 << 20)  # 1 MiB free
        if str(d) == str(roomy):
            return _St(1 << 40)
        return real(d)

    monkeypatch.setattr(shm.os, "statvfs", fake)
    monkeypatch.setenv("TMPDIR", str(roomy))
    assert shm._roomy_dir(str(small), 512 << 20) == str(roomy)
    assert shm._roomy_dir(str(roomy), 512 << 20) == str(roomy)
