"""Host-side screen operands (csrc/host_prep.cpp) against a NumPy rendering of the same bits:
c = q - mu in fp64, hi = fp16_rn(fp32_rn(c)) (subnormals included), |c|^2 in fp64 rounded to
fp32, rows outside the fp16 range flagged.  Both the AVX2/F16C path (A % 8 == 0) and the
portable path (other A) run."""
import numpy as np
import pytest

from distributed_machine_learning_project_amd import _lib


def _f16_ref(c):
    # numpy's float32 -> float16 cast rounds to nearest even, subnormals included
    return c.astype(np.float32).astype(np.float16).view(np.uint16)


@pytest.mark.parametrize("A", [32, 40, 7, 64])
def test_cpu_prep_queries_bits(A):
    L = _lib.lib()
    rng = np.random.default_rng(A)
    X = rng.uniform(-1000, 1000, (6000, A))
    Qx = rng.uniform(-1000, 1000, (20000, A))
    KT = (A + 31) // 32
    mu = np.empty(A)
    L.dmlp_cpu_center(X.ctypes.data, len(X), A, mu.ctypes.data)
    np.testing.assert_allclose(mu, X[:4096].mean(0), rtol=1e-12, atol=1e-9)
    hh = np.full((len(Qx), KT * 32), 7, np.uint16)
    qn = np.zeros(len(Qx), np.float32)
    rc = L.dmlp_cpu_prep_queries(Qx.ctypes.data, len(Qx), A, mu.ctypes.data, KT, hh.ctypes.data,
                                 qn.ctypes.data)
    assert rc == 0
    c = Qx - mu
    np.testing.assert_array_equal(hh[:, :A], _f16_ref(c))
    assert (hh[:, A:] == 0).all()
    np.testing.assert_allclose(qn, (c * c).sum(1), rtol=1e-6)


@pytest.mark.parametrize("A", [32, 7])
def test_cpu_prep_fp16_rounding_edges(A):
    """Ties, subnormals, the largest finite fp16 range and signed zeros, both code paths."""
    L = _lib.lib()
    rng = np.random.default_rng(1)
    vals = np.concatenate([
        rng.uniform(-65000, 65000, 4000),
        rng.uniform(-1e-4, 1e-4, 4000),                       # fp16 subnormals
        (np.arange(-2000, 2000) + 0.5) * 2.0 ** -10,          # ties at the mantissa LSB
        np.ldexp(rng.integers(1, 2 ** 12, 2000).astype(np.float64), -24),  # subnormal ties
        [0.0, -0.0, 65503.0, -65503.0, 2.0 ** -14, 2.0 ** -25, 3 * 2.0 ** -26]])
    Q = len(vals) // A
    Qx = vals[:Q * A].reshape(Q, A).copy()
    KT = (A + 31) // 32
    mu = np.zeros(A)
    hh = np.zeros((Q, KT * 32), np.uint16)
    qn = np.zeros(Q, np.float32)
    assert L.dmlp_cpu_prep_queries(Qx.ctypes.data, Q, A, mu.ctypes.data, KT, hh.ctypes.data,
                                   qn.ctypes.data) == 0
    np.testing.assert_array_equal(hh[:, :A], _f16_ref(Qx))


def test_cpu_prep_queries_flags_range():
    L = _lib.lib()
    A = 32
    Qx = np.ones((5000, A))
    Qx[1234, 5] = 70000.0  # beyond the fp16 range
    mu = np.zeros(A)
    hh = np.zeros((5000, 32), np.uint16)
    qn = np.zeros(5000, np.float32)
    assert L.dmlp_cpu_prep_queries(Qx.ctypes.data, 5000, A, mu.ctypes.data, 1, hh.ctypes.data,
                                   qn.ctypes.data) == 1
    Qx[1234, 5] = 1e16
    assert L.dmlp_cpu_prep_queries(Qx.ctypes.data, 5000, A, mu.ctypes.data, 1, hh.ctypes.data,
                                   qn.ctypes.data) == 1
    Qx[1234, 5] = np.nan
    assert L.dmlp_cpu_prep_queries(Qx.ctypes.data, 5000, A, mu.ctypes.data, 1, hh.ctypes.data,
                                   qn.ctypes.data) == 1


def _hi_image_ref(X, mu, KT):
    """prep.hip's tile layout, hi halves only, as fp16: uint16 [n_tiles][4][KT][64 lanes][8],
    lane = r + 16 * kg holds attributes kt*32 + kg*8 .. +7 of point t*64 + rt*16 + r."""
    N, A = X.shape
    n_tiles = (N + 63) // 64
    c = np.zeros((n_tiles * 64, KT * 32))
    c[:N, :A] = X - mu
    h = _f16_ref(c)  # zero rows / columns render as 0
    img = h.reshape(n_tiles, 4, 16, KT, 4, 8)          # t, rt, r, kt, kg, j
    return img.transpose(0, 1, 3, 4, 2, 5).reshape(-1)  # t, rt, kt, kg, r, j


@pytest.mark.parametrize("N,A", [(6000, 32), (1000, 40), (130, 7), (4097, 64)])
def test_cpu_prep_data_image(N, A):
    L = _lib.lib()
    rng = np.random.default_rng(N + A)
    X = rng.uniform(-1000, 1000, (N, A))
    KT = (A + 31) // 32
    mu = np.empty(A)
    L.dmlp_cpu_center(X.ctypes.data, N, A, mu.ctypes.data)
    n_tiles = (N + 63) // 64
    img = np.full(n_tiles * 64 * KT * 32, 7, np.uint16)
    xinit = np.zeros(n_tiles * 64, np.float32)
    nmax = np.zeros(1, np.uint32)
    assert L.dmlp_cpu_prep_data(X.ctypes.data, N, A, mu.ctypes.data, KT, img.ctypes.data,
                                xinit.ctypes.data, nmax.ctypes.data) == 0
    np.testing.assert_array_equal(img, _hi_image_ref(X, mu, KT))
    ss = ((X - mu) ** 2).sum(1)
    np.testing.assert_allclose(xinit[:N], -0.5 * ss, rtol=1e-6)
    assert np.isneginf(xinit[N:]).all()
    m = nmax.view(np.float32)[0]
    assert ss.max() * (1 + 5e-7) <= m <= ss.max() * (1 + 3e-6)


def test_cpu_prep_data_flags_range():
    L = _lib.lib()
    X = np.ones((3000, 32))
    X[2999, 31] = np.inf
    mu = np.zeros(32)
    img = np.zeros(3008 * 32, np.uint16)
    xinit = np.zeros(3008, np.float32)
    nmax = np.zeros(1, np.uint32)
    assert L.dmlp_cpu_prep_data(X.ctypes.data, 3000, 32, mu.ctypes.data, 1, img.ctypes.data,
                                xinit.ctypes.data, nmax.ctypes.data) == 1


def test_pool_splits_mask_among_node_ranks():
    """The render pool divides its CPU mask among the local ranks bound to the same NUMA node
    (DMLP_NODE_RANKS, set by the NUMA binding), not among every rank of the machine."""
    import os
    import subprocess
    import sys

    def threads(**env):
        e = {k: v for k, v in os.environ.items()
             if k not in ("LOCAL_WORLD_SIZE", "DMLP_NODE_RANKS", "DMLP_HOST_THREADS")}
        e.update(env)
        r = subprocess.run([sys.executable, "-c", "from distributed_machine_learning_project_amd "
                            "import _lib; print(_lib.lib().dmlp_host_threads())"],
                           capture_output=True, text=True, env=e, check=True)
        return int(r.stdout.strip())

    alone = threads()
    if alone < 8:
        pytest.skip("needs >= 8 CPUs in the affinity mask")
    all_local = threads(LOCAL_WORLD_SIZE="4")
    node_pair = threads(LOCAL_WORLD_SIZE="4", DMLP_NODE_RANKS="2")
    node_one = threads(LOCAL_WORLD_SIZE="4", DMLP_NODE_RANKS="1")
    assert all_local <= node_pair <= node_one
    assert node_one > all_local


def test_rows_i32_lossless_check():
    """6-decimal inputs (generate_input.py's "%.6f") travel as int32 m with x == fl(m / 1e6) bit
    for bit; anything else (more digits, -0.0, |x| >= 2^31 / 1e6, NaN) is refused."""
    from distributed_machine_learning_project_amd import _lib
    import distributed_machine_learning_project_amd as dmlp
    L = _lib.lib()
    inp = dmlp.generate(5000, 10, 32, -1000.0, 1000.0, 1, 4, 3, seed=9)
    x = np.ascontiguousarray(inp.X.reshape(-1))
    m = np.empty(len(x), np.int32)
    assert L.dmlp_cpu_rows_i32(x.ctypes.data, len(x), m.ctypes.data) == 0
    back = m.astype(np.float64) / 1.0e6
    assert np.array_equal(back.view(np.uint64), x.view(np.uint64))
    for bad in (0.1234567, -0.0, 2147.483648, float("nan"), 1e300):
        y = x[:1001].copy()  # odd length: the scalar tail too
        y[np.random.default_rng(1).integers(0, 1001)] = bad
        assert L.dmlp_cpu_rows_i32(y.ctypes.data, len(y), m.ctypes.data) == 1, bad
        y[-1] = bad
        y[:-1] = x[:1000]
        assert L.dmlp_cpu_rows_i32(y.ctypes.data, len(y), m.ctypes.data) == 1, bad


def test_row_table_render_matches_flat():
    """The drop-in's in-place path (tables of row pointers into separately allocated rows) renders
    the same screen operands, centre, int32 pack and fp64 pack as the row-major path."""
    import ctypes
    from distributed_machine_learning_project_amd import _lib
    import distributed_machine_learning_project_amd as dmlp
    L = _lib.lib()
    inp = dmlp.generate(3000, 2100, 40, -500.0, 500.0, 1, 4, 3, seed=13)
    A, KT = 40, 2
    W = KT * 32
    # every row its own allocation, in shuffled address order, like vector<DataPoint>::attrs
    rows = [np.array(r, np.float64) for r in inp.X]
    order = np.random.default_rng(0).permutation(len(rows))
    keep = [rows[i] for i in order]  # (allocation order differs from row order)
    tab = (ctypes.c_void_p * len(rows))(*[r.ctypes.data for r in rows])
    qrows = [np.array(r, np.float64) for r in inp.Qx]
    qtab = (ctypes.c_void_p * len(qrows))(*[r.ctypes.data for r in qrows])
    N, Q = len(rows), len(qrows)
    mu_f, mu_t = np.empty(A), np.empty(A)
    L.dmlp_cpu_center(inp.X.ctypes.data, N, A, mu_f.ctypes.data)
    L.dmlp_cpu_center_rows(tab, N, A, mu_t.ctypes.data)
    assert np.array_equal(mu_f, mu_t)
    qh_f, qh_t = np.empty(Q * W, np.uint16), np.empty(Q * W, np.uint16)
    qn_f, qn_t = np.empty(Q, np.float32), np.empty(Q, np.float32)
    assert L.dmlp_cpu_prep_queries(inp.Qx.ctypes.data, Q, A, mu_f.ctypes.data, KT,
                                   qh_f.ctypes.data, qn_f.ctypes.data) == 0
    assert L.dmlp_cpu_prep_queries_rows(qtab, Q, A, mu_f.ctypes.data, KT, qh_t.ctypes.data,
                                        qn_t.ctypes.data) == 0
    assert np.array_equal(qh_f, qh_t) and np.array_equal(qn_f, qn_t)
    nt = (N + 63) // 64
    xh_f, xh_t = np.empty(nt * 64 * W, np.uint16), np.empty(nt * 64 * W, np.uint16)
    xi_f, xi_t = np.empty(nt * 64, np.float32), np.empty(nt * 64, np.float32)
    m_f, m_t = np.zeros(1, np.float32), np.zeros(1, np.float32)
    assert L.dmlp_cpu_prep_data_tiles(inp.X.ctypes.data, N, A, mu_f.ctypes.data, KT, 0, nt,
                                      xh_f.ctypes.data, xi_f.ctypes.data, m_f.ctypes.data) == 0
    assert L.dmlp_cpu_prep_data_tiles_rows(tab, N, A, mu_f.ctypes.data, KT, 0, nt,
                                           xh_t.ctypes.data, xi_t.ctypes.data, m_t.ctypes.data) == 0
    assert np.array_equal(xh_f, xh_t) and np.array_equal(xi_f, xi_t) and m_f[0] == m_t[0]
    i_f, i_t = np.empty(N * A, np.int32), np.empty(N * A, np.int32)
    assert L.dmlp_cpu_rows_i32(inp.X.ctypes.data, N * A, i_f.ctypes.data) == 0
    assert L.dmlp_cpu_rows_i32_rows(tab, N, A, i_t.ctypes.data) == 0
    assert np.array_equal(i_f, i_t)
    rows[17][3] += 1e-7  # not 6-decimal any more
    assert L.dmlp_cpu_rows_i32_rows(tab, N, A, i_t.ctypes.data) == 1
    g = np.empty(N * A)
    L.dmlp_cpu_gather_rows(tab, N, A, g.ctypes.data)
    assert np.array_equal(g.reshape(N, A), np.stack(rows))
    del keep


@pytest.mark.parametrize("n", [0, 1, 1000, 65535, 65536, 300001])
def test_host_i32_range_matches_numpy(n):
    """The native step's label / k scans (dmlp_host_i32_range: on the render pool above 64K
    values) == numpy's min / max, negative values and both ends included; (0, -1) when empty."""
    import ctypes as C
    from distributed_machine_learning_project_amd import _lib
    rng = np.random.default_rng(n)
    a = rng.integers(-(2 ** 31), 2 ** 31 - 1, size=n, dtype=np.int64).astype(np.int32)
    if n > 2:
        a[0], a[-1] = np.int32(2 ** 31 - 1), np.int32(-(2 ** 31))
    lo, hi = C.c_int(), C.c_int()
    _lib.lib().dmlp_host_i32_range(a.ctypes.data, a.size, C.byref(lo), C.byref(hi))
    if n == 0:
        assert (lo.value, hi.value) == (0, -1)
    else:
        assert (lo.value, hi.value) == (int(a.min()), int(a.max()))


def test_build_records_source_identity(tmp_path):
    """build() (what __graft_entry__.build runs) records what it did, and the library's identity is
    the hash of its sources: the srchash beside libdmlp.so matches a fresh hash of the tree, and
    build_info says whether anything was compiled."""
    import json
    from distributed_machine_learning_project_amd import build
    build.build(engine=False)
    info = build.build_info()
    assert info["lib_matches_sources"] is True
    srcs = sum(build._sources(), [])
    want = build._source_hash(srcs)
    assert build.SRCHASH.read_text().strip() == want
    assert info["source_hash_16"] == want[:16]
    rec = json.loads((build.BUILD / "build_info.json").read_text())
    assert rec["mode"] in ("up-to-date", "rebuilt") and rec["arch"] == "gfx950"
    # the headers a library object depends on are the ones its sources include, not every csrc
    # header (engine_core.h changes relink knn_engine only)
    names = {h.name for h in build._included(srcs)}
    assert "dmlp.h" in names and "engine_core.h" not in names
