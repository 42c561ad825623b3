"""HIP kernel numerics: every GPU result is compared with the exact CPU path (itself pinned to
the NumPy float64 oracle in test_cpu_oracle.py).  Exact equality is required: distances,
neighbour ids and order, labels and checksums must be bit-identical."""
import numpy as np
import pytest

import distributed_machine_learning_project_amd as dmlp
from distributed_machine_learning_project_amd.ops import knn as K

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import distributed_machine_learning_project_amd._lib as L
    L.lib()
    return torch


def run_both(torch, inp, exact=False, finalize=True):
    X = torch.from_numpy(inp.X).cuda()
    lab = torch.from_numpy(inp.labels).cuda()
    Qx = torch.from_numpy(inp.Qx).cuda()
    ds = K.prepare_dataset(X, lab, (int(inp.labels.min()), int(inp.labels.max()) + 1))
    r = K.knn_gpu(ds, Qx, inp.k, finalize=finalize, exact=exact)
    torch.cuda.synchronize()
    d_ref, i_ref = K.knn_cpu(inp.X, inp.Qx, inp.k, kstride=r.dist.shape[1])
    lab_ref, cs_ref = K.finalize_cpu(i_ref, inp.k, inp.labels)
    return r, (d_ref, i_ref, lab_ref, cs_ref)


def assert_same(r, refs):
    d_ref, i_ref, lab_ref, cs_ref = refs
    d = r.dist.cpu().numpy()
    i = r.ids.cpu().numpy()
    for q in range(len(r.k)):
        k = int(r.k[q])
        np.testing.assert_array_equal(i[q, :k], i_ref[q, :k], err_msg=f"ids q={q}")
        np.testing.assert_array_equal(d[q, :k], d_ref[q, :k], err_msg=f"dist q={q}")
    if r.label is not None:
        np.testing.assert_array_equal(r.label.cpu().numpy(), lab_ref)
        np.testing.assert_array_equal(r.checksum.cpu().numpy().view(np.uint64), cs_ref)


@pytest.mark.parametrize("A", [1, 5, 32, 33, 64, 100, 128])
def test_screen_small_k(torch_cuda, A):
    inp = dmlp.generate(3000, 200, A, 0.0, 1000.0, 1, 32, 7, seed=A)
    r, refs = run_both(torch_cuda, inp)
    assert r.n_fallback == 0
    assert_same(r, refs)


def test_screen_mid_k(torch_cuda):
    inp = dmlp.generate(5000, 150, 32, -50.0, 50.0, 33, 128, 5, seed=3)
    r, refs = run_both(torch_cuda, inp)
    assert r.n_fallback == 0
    assert_same(r, refs)


def test_large_k_fallback(torch_cuda):
    inp = dmlp.generate(2000, 40, 16, 0.0, 10.0, 100, 2000, 3, seed=4)
    r, refs = run_both(torch_cuda, inp)
    assert_same(r, refs)


def test_select_and_sort_fallback_paths(torch_cuda):
    """k <= 2048 -> radix-select path, k > 2048 -> segmented-sort path; duplicate-heavy data so
    the k-th distance is tied across the selection boundary."""
    rng = np.random.default_rng(11)
    base = np.round(rng.uniform(0, 3, size=(300, 5)), 1)
    X = base[rng.integers(0, 300, size=6000)]
    labels = rng.integers(0, 6, size=6000).astype(np.int32)
    Qx = np.round(rng.uniform(0, 3, size=(60, 5)), 1)
    k = np.concatenate([rng.integers(129, 2049, 40), rng.integers(2049, 6001, 20)]).astype(np.int32)
    inp = dmlp.KNNInput(labels, np.ascontiguousarray(X), k, Qx)
    r, refs = run_both(torch_cuda, inp)
    # k in (128, 256] is screened (cap-512 LDS screen); every larger k takes the exact path
    assert r.n_fallback == int((k > K.SCREEN_KMAX_C).sum())
    assert_same(r, refs)


def test_select_tie_overflow(torch_cuda):
    """Every distance equal: the select keeps the LARGEST ids among the ties (id desc order)."""
    X = np.full((7000, 3), 2.0)
    X[::97] = 5.0  # a few farther points
    labels = (np.arange(7000) % 4).astype(np.int32)
    Qx = np.zeros((9, 3))
    k = np.array([129, 500, 1000, 2048, 2047, 3000, 6900, 7000, 1500], np.int32)
    inp = dmlp.KNNInput(labels, X, k, Qx)
    r, refs = run_both(torch_cuda, inp)
    assert_same(r, refs)


def test_k_zero_and_k_gt_n(torch_cuda):
    inp = dmlp.generate(50, 20, 8, 0.0, 10.0, 1, 10, 3, seed=5)
    inp.k[:5] = 0
    inp.k[5:10] = 70  # > N: padded with (+inf, -1)
    r, refs = run_both(torch_cuda, inp)
    assert_same(r, refs)


def test_ties_duplicates(torch_cuda):
    rng = np.random.default_rng(0)
    base = np.round(rng.uniform(0, 5, size=(40, 6)), 1)
    X = base[rng.integers(0, 40, size=4000)]  # heavy duplication -> massive distance ties
    labels = rng.integers(0, 4, size=4000).astype(np.int32)
    Qx = np.round(rng.uniform(0, 5, size=(100, 6)), 1)
    k = rng.integers(1, 60, size=100).astype(np.int32)
    inp = dmlp.KNNInput(labels, np.ascontiguousarray(X), k, Qx)
    r, refs = run_both(torch_cuda, inp)
    assert_same(r, refs)


def test_all_identical_points(torch_cuda):
    X = np.ones((5000, 4))
    labels = (np.arange(5000) % 3).astype(np.int32)
    Qx = np.zeros((17, 4))
    k = np.full(17, 16, np.int32)
    inp = dmlp.KNNInput(labels, X, k, Qx)
    r, refs = run_both(torch_cuda, inp)
    assert r.n_fallback == 17
    assert_same(r, refs)


def test_huge_values_use_exact(torch_cuda):
    inp = dmlp.generate(1000, 50, 8, 0.0, 1.0, 1, 16, 3, seed=6)
    inp.X[3, 2] = 1e200
    r, refs = run_both(torch_cuda, inp)
    assert r.n_fallback == 50
    assert_same(r, refs)


def test_exact_mode(torch_cuda):
    inp = dmlp.generate(3000, 64, 32, 0.0, 1000.0, 1, 40, 10, seed=7)
    r, refs = run_both(torch_cuda, inp, exact=True)
    assert_same(r, refs)


@pytest.mark.parametrize("N,Q,A,kmin,kmax,lo,hi", [
    (3000, 130, 32, 1, 16, 0, 1000),       # k <= 16 variant, two workgroups' worth of queries
    (4097, 70, 7, 17, 64, -5, 5),          # k in (16, 64], odd A, ragged last tile
    (5000, 40, 33, 65, 256, 0, 1000),      # the 16-query, 384-slot variant
    (700, 33, 3, 200, 256, 0, 2),          # heavy exact ties (3 attrs in {0, 1, 2}); k near N/3
    (300, 20, 16, 250, 256, 0, 1000),      # k close to N
])
def test_fused_exact_kernel(torch_cuda, N, Q, A, kmin, kmax, lo, hi, monkeypatch):
    """exact.hip (the --exact path and the fallback for k <= 256) == the CPU path, bit for bit:
    every variant, ties broken by larger id, per-query k mixed within a workgroup.  Forced for
    every k (DMLP_EXACT_FUSED=2): at these small N the dispatch would pick rows + select for
    k > 64."""
    monkeypatch.setenv("DMLP_EXACT_FUSED", "2")
    monkeypatch.setenv("DMLP_EXACT_F64", "0")  # (A <= 32, k <= 64 would take the fp64 screen)
    inp = dmlp.generate(N, Q, A, lo, hi, kmin, kmax, 5, seed=N + A)
    r, refs = run_both(torch_cuda, inp, exact=True)
    assert_same(r, refs)
    assert K.pipeline_stats()["n_exact_f64"] == 0


@pytest.mark.parametrize("A", [32, 7, 1, 48, 64])
def test_exact_f64_mfma_layout(torch_cuda, A):
    """The fp64 screen's operand / result maps (v_mfma_f64_16x16x4_f64, screen_f64.hip) on exact
    integer data: 16 queries x the first 16 points, every score q'.x' - |x'|^2/2 exact."""
    from distributed_machine_learning_project_amd import _lib
    L = _lib.lib()
    torch = torch_cuda
    rng = np.random.default_rng(A)
    X = rng.integers(-8, 9, size=(64, A)).astype(np.float64)
    Qh = rng.integers(-8, 9, size=(16, A)).astype(np.float64)
    mu = X.mean(0)  # dyadic (N = 64): exact, as dmlp_center computes it
    xs, qs = X - mu, Qh - mu
    expect = qs @ xs[:16].T - 0.5 * (xs[:16] ** 2).sum(1)[None, :]
    dX, dQ = torch.from_numpy(X).cuda(), torch.from_numpy(Qh).cuda()
    out = torch.zeros(256, dtype=torch.float64, device="cuda")
    nb = int(L.dmlp_exact_f64_bytes(64, A, 64, 16))
    ws = torch.empty(nb, dtype=torch.uint8, device="cuda")
    rc = L.dmlp_exact_f64_probe(dX.data_ptr(), 64, A, dQ.data_ptr(), out.data_ptr(), ws.data_ptr(),
                                nb, torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy().reshape(16, 16), expect)


@pytest.mark.parametrize("N,Q,A,kmin,kmax,lo,hi", [
    (3000, 130, 32, 1, 16, 0, 1000),        # SUB 16, 2 query blocks, many slices
    (4097, 70, 7, 17, 64, -5, 5),           # SUB 32, odd A (padded to 8), ragged last tile
    (20000, 700, 32, 1, 64, 0, 1000),       # mixed k in one wave
    (9000, 64, 16, 16, 16, 1e6, 1e6 + 1),   # offset data: centring keeps the keys tight
    (700, 33, 3, 1, 40, 0, 2),              # heavy exact ties: overflow -> VALU kernel
    (1000, 20, 1, 1, 64, 0, 10),            # A = 1
    (6000, 150, 48, 1, 16, 0, 1000),        # A in (32, 64]: 12 fragments, one wave per SIMD
    (5000, 90, 64, 8, 64, -50, 50),         # A = 64, mixed k up to 64
    (3000, 70, 37, 1, 32, 0, 1000),         # odd A padded to 40 -> 12 fragments
])
def test_exact_f64_screen(torch_cuda, N, Q, A, kmin, kmax, lo, hi):
    """The exact path's fp64 MFMA screen (screen_f64.hip) + exact group re-rank == the CPU path
    bit for bit; queries whose candidates overflow (ties) are re-ranked by exact.hip, and the
    stats say how many took which."""
    inp = dmlp.generate(N, Q, A, lo, hi, kmin, kmax, 5, seed=N + A + kmax)
    r, refs = run_both(torch_cuda, inp, exact=True)
    assert_same(r, refs)
    st = K.pipeline_stats()
    assert st["n_exact_f64"] == Q
    if hi - lo > 100:
        assert st["n_exact_f64_redo"] == 0


def test_exact_f64_huge_and_duplicates(torch_cuda):
    """Magnitudes past the fp32 key range and all-identical points: every query overflows the
    fp64 screen and the VALU kernel answers it, still exact."""
    inp = dmlp.generate(1000, 50, 8, 0.0, 1.0, 1, 16, 3, seed=6)
    inp.X[3, 2] = 1e200
    r, refs = run_both(torch_cuda, inp, exact=True)
    assert_same(r, refs)
    assert K.pipeline_stats()["n_exact_f64_redo"] == 50
    X = np.ones((5000, 4))
    labels = (np.arange(5000) % 3).astype(np.int32)
    inp = dmlp.KNNInput(labels, X, np.full(17, 16, np.int32), np.zeros((17, 4)))
    r, refs = run_both(torch_cuda, inp, exact=True)
    assert_same(r, refs)


def test_many_slices_small_q(torch_cuda):
    inp = dmlp.generate(200000, 8, 32, 0.0, 1000.0, 16, 16, 10, seed=8)
    r, refs = run_both(torch_cuda, inp)
    assert r.n_fallback == 0
    assert_same(r, refs)


@pytest.mark.parametrize("impl", ["x1", "stream", "lds"])
def test_screen_impls_bench_distribution(torch_cuda, impl):
    """Every screen implementation is exact on the bench distribution (generate_input.py,
    A=32, k=16); the single-term screen needs no 3-term escalation there."""
    inp = dmlp.generate(20000, 700, 32, 0.0, 1000.0, 16, 16, 10, seed=12)
    with K.pipeline_options(screen=impl):
        r, refs = run_both(torch_cuda, inp)
    assert r.n_fallback == 0
    if impl == "x1":
        assert r.n_escalated == 0
    assert_same(r, refs)


@pytest.mark.parametrize("A,kmax", [(8, 16), (32, 32), (64, 16), (40, 30), (32, 64), (20, 48)])
def test_x1_screen_shapes(torch_cuda, A, kmax):
    """Single-term screen: KT 1/2, both sub-buffer depths (k <= 16 / <= 64), ragged tails."""
    inp = dmlp.generate(7777, 333, A, -100.0, 100.0, 1, kmax, 6, seed=A + kmax)
    r, refs = run_both(torch_cuda, inp)
    assert r.n_fallback == 0
    assert_same(r, refs)


@pytest.mark.parametrize("A,kmin,kmax,N,Q,lo,hi", [(8, 1, 16, 7777, 333, -100.0, 100.0),
                                                  (32, 16, 16, 20000, 700, 0.0, 1000.0),
                                                  (64, 1, 16, 9001, 260, -5.0, 5.0),
                                                  (32, 1, 1, 3000, 129, 0.0, 1000.0),
                                                  (20, 1, 12, 300000, 64, 0.0, 1000.0)])
def test_single_term_screens(torch_cuda, A, kmin, kmax, N, Q, lo, hi):
    """k <= 16 single-term class (screen_x1.hip, 16x16x32): KT 1/2, ragged query blocks and
    tiles, k = 1, and many slices (few queries, N = 3e5 > one slice's 16-bit group range)."""
    inp = dmlp.generate(N, Q, A, lo, hi, kmin, kmax, 6, seed=A + kmax + N)
    r, refs = run_both(torch_cuda, inp)
    assert r.n_fallback == 0
    assert_same(r, refs)


def test_x1_escalates_tight_data(torch_cuda):
    """Dense 1-D data: the single-term bound admits ~900 points per query (> its 60-group
    buffer), so queries escalate to the 3-term screen (or on to the exact path) and stay exact."""
    inp = dmlp.generate(20000, 100, 1, 0.0, 1000.0, 8, 16, 4, seed=2)
    # few slices: ~5000 points per query block and slice
    with K.pipeline_options(num_cus=1):
        r, refs = run_both(torch_cuda, inp)
    assert r.n_escalated > 0
    assert_same(r, refs)


@pytest.mark.parametrize("kmin", [1, 0])
def test_pipelined_chunks_match(torch_cuda, kmin):
    """Host-array entry (the native step) == the exact CPU path: the host renders the screen's
    operands and copies the fp64 rows behind the screen; kmin=0 adds k = 0 queries (no neighbour,
    label -1) to the per-query dispatch."""
    torch = torch_cuda
    inp = dmlp.generate(30000, 9000, 32, 0.0, 1000.0, kmin, 24, 10, seed=21)
    Xp = torch.from_numpy(inp.X).pin_memory().numpy()
    Qp = torch.from_numpy(inp.Qx).pin_memory().numpy()
    ds, d, i, lab, cs, nfb = K.knn_gpu_pipelined(Xp, inp.labels, (0, 10), Qp, inp.k)
    torch.cuda.synchronize()
    d_ref, i_ref = K.knn_cpu(inp.X, inp.Qx, inp.k, kstride=d.shape[1])
    lab_ref, cs_ref = K.finalize_cpu(i_ref, inp.k, inp.labels)
    np.testing.assert_array_equal(i.cpu().numpy(), i_ref)
    np.testing.assert_array_equal(d.cpu().numpy(), d_ref)
    np.testing.assert_array_equal(lab.cpu().numpy(), lab_ref)
    np.testing.assert_array_equal(cs.cpu().numpy().view(np.uint64), cs_ref)


@pytest.mark.parametrize("case", ["escalate", "slices", "ragged"])
def test_pipelined_host_image_paths(torch_cuda, case):
    """The host's fp16 hi-only dataset image (hl = 1) through the x1 screen and group refine:
    tight 1-D data escalates to the 3-term screen (device hi/lo image rendered on demand from
    the fp64 rows), few queries split the data into many slices, and A = 40 / N % 64 != 0
    exercises KT = 2 and a ragged last tile."""
    torch = torch_cuda
    ncus = 256
    if case == "escalate":
        ncus = 1
        inp = dmlp.generate(20000, 100, 1, 0.0, 1000.0, 8, 16, 4, seed=2)
    elif case == "slices":
        inp = dmlp.generate(60000, 64, 32, 0.0, 1000.0, 1, 32, 10, seed=4)
    else:
        inp = dmlp.generate(9001, 700, 40, -100.0, 100.0, 1, 30, 7, seed=6)
    Xp = torch.from_numpy(inp.X).pin_memory().numpy()
    Qp = torch.from_numpy(inp.Qx).pin_memory().numpy()
    with K.pipeline_options(num_cus=ncus):
        ds, d, i, lab, cs, nfb = K.knn_gpu_pipelined(Xp, inp.labels,
                                                     (0, int(inp.labels.max()) + 1), Qp, inp.k)
    torch.cuda.synchronize()
    if case == "escalate":
        assert ds.n_escalated > 0  # (1-D data this dense takes the device image: hl = 2)
    else:
        assert ds.hl == 1
    d_ref, i_ref = K.knn_cpu(inp.X, inp.Qx, inp.k, kstride=d.shape[1])
    lab_ref, cs_ref = K.finalize_cpu(i_ref, inp.k, inp.labels)
    np.testing.assert_array_equal(i.cpu().numpy(), i_ref)
    np.testing.assert_array_equal(d.cpu().numpy(), d_ref)
    np.testing.assert_array_equal(lab.cpu().numpy(), lab_ref)
    np.testing.assert_array_equal(cs.cpu().numpy().view(np.uint64), cs_ref)


def test_host_data_image_matches_device(torch_cuda):
    """dmlp_cpu_prep_data's fp16 hi-only image is the fp16 rounding of the same centred values
    prep.hip renders (in prep.hip's tile layout); xinit and the max norm agree with the device
    prep to fp32 rounding of differently ordered fp64 sums."""
    torch = torch_cuda
    from distributed_machine_learning_project_amd import _lib
    L = _lib.lib()
    inp = dmlp.generate(5000, 10, 40, -50.0, 1000.0, 1, 8, 10, seed=5)
    N, A, KT = 5000, 40, 2
    n_tiles = (N + 63) // 64
    mu = np.empty(A)
    L.dmlp_cpu_center(inp.X.ctypes.data, N, A, mu.ctypes.data)
    img = np.zeros(n_tiles * 64 * KT * 32, np.uint16)
    xin_h = np.zeros(n_tiles * 64, np.float32)
    nm_h = np.zeros(1, np.uint32)
    assert L.dmlp_cpu_prep_data(inp.X.ctypes.data, N, A, mu.ctypes.data, KT, img.ctypes.data,
                                xin_h.ctypes.data, nm_h.ctypes.data) == 0
    c = np.zeros((n_tiles * 64, KT * 32))
    c[:N, :A] = inp.X - mu
    ref = c.astype(np.float32).astype(np.float16).view(np.uint16)
    ref = ref.reshape(n_tiles, 4, 16, KT, 4, 8).transpose(0, 1, 3, 4, 2, 5).reshape(-1)
    np.testing.assert_array_equal(img, ref)
    X = torch.from_numpy(inp.X).cuda()
    mu_d = torch.from_numpy(mu).cuda()
    xfrag = torch.empty(n_tiles * 64 * KT * 32 * 2, dtype=torch.int16, device="cuda")
    xinit = torch.empty(n_tiles * 64, dtype=torch.float32, device="cuda")
    xnmax = torch.zeros(1, dtype=torch.int32, device="cuda")
    bad = torch.zeros(1, dtype=torch.int32, device="cuda")
    _lib.check(L.dmlp_prep_data(X.data_ptr(), N, A, mu_d.data_ptr(), KT, xfrag.data_ptr(),
                                xinit.data_ptr(), xnmax.data_ptr(), bad.data_ptr(),
                                torch.cuda.current_stream().cuda_stream), "prep_data")
    torch.cuda.synchronize()
    np.testing.assert_allclose(xinit.cpu().numpy()[:N], xin_h[:N], rtol=1e-6)
    assert np.isneginf(xinit.cpu().numpy()[N:]).all()
    np.testing.assert_allclose(xnmax.cpu().numpy().view(np.float32), nm_h.view(np.float32),
                               rtol=1e-6)


def test_host_prep_matches_device_prep(torch_cuda):
    """dmlp_cpu_prep_queries renders the fp16 rounding of the centred queries whose bf16 split
    the device prep renders (hi + lo of the device = the fp32 value to 16 bits), and the same
    qn (within fp64 summation order, rounded to fp32)."""
    torch = torch_cuda
    from distributed_machine_learning_project_amd import _lib
    L = _lib.lib()
    inp = dmlp.generate(5000, 3000, 40, -50.0, 1000.0, 1, 8, 10, seed=5)
    A, KT, Q = 40, 2, 3000
    mu = np.empty(A)
    L.dmlp_cpu_center(inp.X.ctypes.data, len(inp.X), A, mu.ctypes.data)
    hh = np.zeros((Q, KT * 32), np.uint16)
    qn_h = np.zeros(Q, np.float32)
    assert L.dmlp_cpu_prep_queries(inp.Qx.ctypes.data, Q, A, mu.ctypes.data, KT, hh.ctypes.data,
                                   qn_h.ctypes.data) == 0
    c = inp.Qx - mu
    np.testing.assert_array_equal(hh[:, :A], c.astype(np.float32).astype(np.float16).view(np.uint16))
    Qx = torch.from_numpy(inp.Qx).cuda()
    mu_d = torch.from_numpy(mu).cuda()
    qhi = torch.empty(Q * KT * 32, dtype=torch.int16, device="cuda")
    qlo = torch.empty_like(qhi)
    qn = torch.empty(Q, dtype=torch.float32, device="cuda")
    bad = torch.zeros(1, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    _lib.check(L.dmlp_prep_queries(Qx.data_ptr(), Q, A, mu_d.data_ptr(), KT, qhi.data_ptr(),
                                   qlo.data_ptr(), qn.data_ptr(), bad.data_ptr(), s), "prep")
    torch.cuda.synchronize()
    hi = qhi.cpu().numpy().view(np.uint16).reshape(Q, -1)[:, :A].astype(np.uint32) << 16
    lo = qlo.cpu().numpy().view(np.uint16).reshape(Q, -1)[:, :A].astype(np.uint32) << 16
    dev = hi.view(np.float32).astype(np.float64) + lo.view(np.float32).astype(np.float64)
    np.testing.assert_allclose(dev, c.astype(np.float32), rtol=2 ** -15, atol=1e-30)
    np.testing.assert_allclose(qn.cpu().numpy(), qn_h, rtol=1e-6)


def test_streamed_out_of_core_matches(torch_cuda):
    """Dataset streamed from pinned host memory in 3 chunks (double-buffered H2D), running
    top-k lists merged per chunk == the exact CPU path."""
    torch = torch_cuda
    inp = dmlp.generate(25000, 3000, 32, 0.0, 1000.0, 1, 30, 10, seed=23)
    Xp = torch.from_numpy(inp.X).pin_memory().numpy()
    Qx = torch.from_numpy(inp.Qx).cuda()
    d, i, lab, cs = K.knn_gpu_streamed(Xp, inp.labels, (0, 10), Qx, inp.k, chunk_rows=9000)
    torch.cuda.synchronize()
    d_ref, i_ref = K.knn_cpu(inp.X, inp.Qx, inp.k, kstride=d.shape[1])
    lab_ref, cs_ref = K.finalize_cpu(i_ref, inp.k, inp.labels)
    np.testing.assert_array_equal(i.cpu().numpy(), i_ref)
    np.testing.assert_array_equal(d.cpu().numpy(), d_ref)
    np.testing.assert_array_equal(cs.cpu().numpy().view(np.uint64), cs_ref)


def test_merge_and_finalize(torch_cuda):
    torch = torch_cuda
    rng = np.random.default_rng(1)
    Lists, Q, kin = 4, 300, 24
    d = np.sort(rng.integers(0, 50, size=(Lists, Q, kin)).astype(np.float64), axis=2)
    ids = rng.permutation(Lists * Q * kin).reshape(Lists, Q, kin).astype(np.int32) % 1000
    # make each list sorted under (d asc, id desc)
    for l in range(Lists):
        for q in range(Q):
            o = np.lexsort((-ids[l, q], d[l, q]))
            d[l, q], ids[l, q] = d[l, q][o], ids[l, q][o]
    k = rng.integers(0, kin + 1, size=Q).astype(np.int32)
    dc, ic = K.merge_cpu(d, ids, k, kout=kin)
    kd = torch.from_numpy(k).cuda()
    dg, ig = K.merge_gpu(torch.from_numpy(d).cuda(), torch.from_numpy(ids).cuda(), kd, kin)
    np.testing.assert_array_equal(ic, ig.cpu().numpy())
    np.testing.assert_array_equal(dc, dg.cpu().numpy())
    labels = rng.integers(0, 7, size=1000).astype(np.int32)
    lab_c, cs_c = K.finalize_cpu(ic, k, labels)
    lab_g, cs_g = K.finalize_gpu(torch.from_numpy(labels).cuda(), (0, 7), dg, ig, kd)
    np.testing.assert_array_equal(lab_c, lab_g.cpu().numpy())
    np.testing.assert_array_equal(cs_c, cs_g.cpu().numpy().view(np.uint64))
    # wide label range -> O(k^2) vote path
    labels2 = (rng.integers(0, 5, size=1000) * 100000 - 7).astype(np.int32)
    lab_c, cs_c = K.finalize_cpu(ic, k, labels2)
    lab_g, cs_g = K.finalize_gpu(torch.from_numpy(labels2).cuda(), (-7, 400000 - 6), dg, ig, kd)
    np.testing.assert_array_equal(lab_c, lab_g.cpu().numpy())
    np.testing.assert_array_equal(cs_c, cs_g.cpu().numpy().view(np.uint64))


@pytest.mark.parametrize("Lists,kin,kout", [(8, 16, 16), (8, 128, 128), (3, 40, 64), (64, 4, 8),
                                             (2, 24, 32), (1, 8, 12), (12, 16, 16),
                                             (5, 13, 16), (2, 7, 9)])
def test_merge_rank_shapes(torch_cuda, Lists, kin, kout):
    """K4 merge at shard-merge shapes (kin % 4 == 0 and L <= 8: the windowed register kernel;
    other kin: the one-load-per-output register kernel; L > 8: the LDS merge path): disjoint
    ids, padded (+inf, -1) suffixes of random length, per-query k in [0, kout] (bench_2 @0xbc70
    custom op semantics via merge_cpu)."""
    torch = torch_cuda
    rng = np.random.default_rng(Lists * 1000 + kin)
    Q = 777
    d = np.sort(rng.integers(0, 400, size=(Lists, Q, kin)).astype(np.float64), axis=2)
    ids = rng.permutation(Lists * Q * kin).reshape(Lists, Q, kin).astype(np.int32)
    for l in range(Lists):
        for q in range(Q):
            o = np.lexsort((-ids[l, q], d[l, q]))
            d[l, q], ids[l, q] = d[l, q][o], ids[l, q][o]
            npad = int(rng.integers(0, kin + 1)) if rng.random() < 0.3 else 0
            if npad:
                d[l, q, kin - npad:] = np.inf
                ids[l, q, kin - npad:] = -1
    k = rng.integers(0, kout + 1, size=Q).astype(np.int32)
    dc, ic = K.merge_cpu(d, ids, k, kout=kout)
    kd = torch.from_numpy(k).cuda()
    dg, ig = K.merge_gpu(torch.from_numpy(d).cuda(), torch.from_numpy(ids).cuda(), kd, kout)
    np.testing.assert_array_equal(ic, ig.cpu().numpy())
    np.testing.assert_array_equal(dc, dg.cpu().numpy())


def test_format_report_gpu(torch_cuda):
    torch = torch_cuda
    rng = np.random.default_rng(2)
    cs = rng.integers(0, 2**63, size=5000, dtype=np.int64).view(np.uint64)
    cs[:3] = [0, 1, 2**64 - 1]
    g = K.format_report_gpu(torch.from_numpy(cs.view(np.int64)).cuda(), qid_base=7)
    assert g == dmlp.format_report(cs, qid_base=7)


def test_pipelined_host_operands_any_k(torch_cuda):
    """knn_gpu_pipelined keeps the host's fp16 x1 operands for the k <= 32 queries when other
    queries need the 3-term class (k in (32, 128]) or the exact path (k > 128), and when one
    query's candidates overflow (600 duplicate points): per-query dispatch, bit-exact."""
    torch = torch_cuda
    rng = np.random.default_rng(23)
    N, Q, A = 8000, 500, 32
    X = np.round(rng.uniform(0, 1000, (N, A)), 6)
    X[:600] = X[0]
    Qx = np.round(rng.uniform(0, 1000, (Q, A)), 6)
    Qx[3] = X[0]
    k = rng.integers(1, 160, Q).astype(np.int32)
    k[3] = 10
    labels = rng.integers(0, 7, N).astype(np.int32)
    Xp = torch.from_numpy(X).pin_memory().numpy()
    Qp = torch.from_numpy(Qx).pin_memory().numpy()
    ds, d, i, lab, cs, nfb = K.knn_gpu_pipelined(Xp, labels, (0, 7), Qp, k)
    torch.cuda.synchronize()
    d_ref, i_ref = K.knn_cpu(X, Qx, k, kstride=d.shape[1])
    lab_ref, cs_ref = K.finalize_cpu(i_ref, k, labels)
    np.testing.assert_array_equal(i.cpu().numpy(), i_ref)
    np.testing.assert_array_equal(d.cpu().numpy(), d_ref)
    np.testing.assert_array_equal(lab.cpu().numpy(), lab_ref)
    np.testing.assert_array_equal(cs.cpu().numpy().view(np.uint64), cs_ref)


@pytest.mark.parametrize("A,dup,x1k", [(32, 0, False), (100, 0, False), (256, 0, False),
                                        (32, 700, False), (32, 0, True), (100, 0, True),
                                        (256, 0, True), (32, 700, True)])
def test_pipelined_single_term_lds(torch_cuda, A, dup, x1k):
    """k in (32, 256] on the two-pass single-term x1 screen over the host's fp16 operands (seeds
    from 16 slices at k' = ceil(k / 16), one COLLECT pass, the large-k group refine) — with `dup`
    copies of one point, the queries sitting on it overflow the single-term bound and escalate to
    the 3-term LDS screen; x1k=False is the 3-term-only A/B path on the device image.
    Bit-exact."""
    torch = torch_cuda
    rng = np.random.default_rng(A + dup)
    N, Q = 9000, 400
    X = np.round(rng.uniform(0, 1000, (N, A)), 6)
    if dup:
        X[:dup] = X[0]
    Qx = np.round(rng.uniform(0, 1000, (Q, A)), 6)
    Qx[5] = X[0]
    k = rng.integers(33, 257, Q).astype(np.int32)
    labels = rng.integers(0, 9, N).astype(np.int32)
    Xp = torch.from_numpy(X).pin_memory().numpy()
    Qp = torch.from_numpy(Qx).pin_memory().numpy()
    with K.pipeline_options(x1k=int(x1k)):
        ds, d, i, lab, cs, nfb = K.knn_gpu_pipelined(Xp, labels, (0, 9), Qp, k)
    torch.cuda.synchronize()
    d_ref, i_ref = K.knn_cpu(X, Qx, k, kstride=d.shape[1])
    lab_ref, cs_ref = K.finalize_cpu(i_ref, k, labels)
    np.testing.assert_array_equal(i.cpu().numpy(), i_ref)
    np.testing.assert_array_equal(d.cpu().numpy(), d_ref)
    np.testing.assert_array_equal(lab.cpu().numpy(), lab_ref)
    np.testing.assert_array_equal(cs.cpu().numpy().view(np.uint64), cs_ref)
    # (700 tied points may overflow the 3-term screen's buffers too: that query alone goes exact)
    assert nfb <= (1 if dup else 0)


def test_pipelined_x1k_small_block(torch_cuda):
    """Few k > 32 queries against a small dataset (N = 3000, A = 16): the two-pass x1 screen's
    COLLECT lists span many data slices (S2 > 1), where the refine must take each query's own
    seed (slice 0 of its lists) — reading another list's seed dropped true neighbours."""
    torch = torch_cuda
    inp = dmlp.parse_input(dmlp.generate_text(3000, 301, 16, 0, 1000, 1, 40, 5, seed=11))
    for a, b in ((0, 151), (151, 301)):
        Qx, k = np.ascontiguousarray(inp.Qx[a:b]), np.ascontiguousarray(inp.k[a:b])
        Xp = torch.from_numpy(inp.X).pin_memory().numpy()
        Qp = torch.from_numpy(Qx).pin_memory().numpy()
        ds, d, i, lab, cs, nfb = K.knn_gpu_pipelined(Xp, inp.labels, (0, 5), Qp, k)
        torch.cuda.synchronize()
        d_ref, i_ref = K.knn_cpu(inp.X, Qx, k, kstride=d.shape[1])
        _, cs_ref = K.finalize_cpu(i_ref, k, inp.labels)
        np.testing.assert_array_equal(i.cpu().numpy(), i_ref)
        np.testing.assert_array_equal(cs.cpu().numpy().view(np.uint64), cs_ref)


@pytest.mark.parametrize("A,kmax", [(65, 16), (100, 32), (128, 16), (129, 16), (200, 30),
                                    (256, 16)])
def test_x1_wide_rows(torch_cuda, A, kmax):
    """Single-term screen for A > 64 (KT = 4 and 8, one wave per SIMD) with the group refine
    staging hi(q') in LDS."""
    inp = dmlp.generate(6000, 300, A, 0.0, 1000.0, 1, kmax, 6, seed=A + kmax)
    r, refs = run_both(torch_cuda, inp)
    assert r.n_fallback == 0
    assert_same(r, refs)


@pytest.mark.parametrize("A", [32, 64, 100, 128, 200, 256])
def test_screen_k_up_to_256(torch_cuda, A):
    """128 < k <= 256 on the cap-512 LDS screen (3-term) and the P = 512 refine, mixed with the
    cap-256 class in one call; A in (128, 256] streams each tile as two LDS stages."""
    inp = dmlp.generate(20000, 300, A, 0.0, 1000.0, 100, 256, 8, seed=A)
    r, refs = run_both(torch_cuda, inp)
    assert r.n_fallback == 0
    assert_same(r, refs)


@pytest.mark.parametrize("A", [160, 256])
def test_wide_rows_every_class(torch_cuda, A):
    """A in (128, 256] with k over all three screen classes (x1 for k <= 32, cap-256 and
    cap-512 LDS screens above): nothing takes the exact path."""
    inp = dmlp.generate(12000, 400, A, 0.0, 1000.0, 1, 200, 7, seed=A + 1)
    r, refs = run_both(torch_cuda, inp)
    assert r.n_fallback == 0
    assert_same(r, refs)


@pytest.mark.parametrize("case", ["plain", "out_of_range", "data_out_of_range", "wide",
                                  "fp64_rows"])
def test_step_front_cases(torch_cuda, case):
    """The native step's front: out_of_range puts one query outside the fp16 range (the step
    takes the device image path for the whole call before anything is screened);
    data_out_of_range puts one point of the last image slice outside it (with the early start
    on, the screen already runs: it drains and the call continues on the device image path);
    wide runs KT = 8; fp64_rows has dataset values with more than 6 decimals, so its rows cross
    as fp64 while the queries' cross as lossless int32."""
    torch = torch_cuda
    A = 256 if case == "wide" else 32
    # (data_out_of_range: one full round of query waves, so the early start runs)
    inp = dmlp.generate(8000 if case == "wide" else 20000,
                        65536 + 64 if case == "data_out_of_range" else 32768, A, 0.0, 1000.0, 1,
                        32, 10, seed=31)
    if case == "out_of_range":
        inp.Qx[-5, 3] = 1.0e6
    if case == "data_out_of_range":
        inp.X[-3, 3] = 1.0e7
    if case == "fp64_rows":
        inp.X[7, 5] += 1e-9
    Xp = torch.from_numpy(inp.X).pin_memory().numpy()
    Qp = torch.from_numpy(inp.Qx).pin_memory().numpy()
    ds, d, i, lab, cs, nfb = K.knn_gpu_pipelined(Xp, inp.labels, (0, 10), Qp, inp.k)
    torch.cuda.synchronize()
    assert ds.hl == (2 if "out_of_range" in case else 1)
    d_ref, i_ref = K.knn_cpu(inp.X, inp.Qx, inp.k, kstride=d.shape[1])
    lab_ref, cs_ref = K.finalize_cpu(i_ref, inp.k, inp.labels)
    np.testing.assert_array_equal(i.cpu().numpy(), i_ref)
    np.testing.assert_array_equal(d.cpu().numpy(), d_ref)
    np.testing.assert_array_equal(lab.cpu().numpy(), lab_ref)
    np.testing.assert_array_equal(cs.cpu().numpy().view(np.uint64), cs_ref)


@pytest.mark.parametrize("A", [32, 100])
def test_step_mixed_k_one_pass(torch_cuda, A):
    """The generator's k distribution (minK = 1, maxK = 64: generate_input.py:19) screened in ONE
    single-term pass with per-column k (no class split, no second scan), one query sitting on
    600 duplicate points (its candidates overflow the single-term bound: it alone escalates
    inside the native step) — report, labels, checksums == the oracle's, served by the step."""
    torch = torch_cuda
    rng = np.random.default_rng(A)
    N, Q = 9000, 4000
    X = np.round(rng.uniform(0, 1000, (N, A)), 6)
    X[:600] = X[0]
    Qx = np.round(rng.uniform(0, 1000, (Q, A)), 6)
    Qx[11] = X[0]
    k = rng.integers(1, 65, Q).astype(np.int32)
    k[11] = 40
    labels = rng.integers(0, 6, N).astype(np.int32)
    _, i_ref = K.knn_cpu(X, Qx, k)
    lab_ref, cs_ref = K.finalize_cpu(i_ref, k, labels)
    dst = torch.empty(48 * Q + 64, dtype=torch.uint8).pin_memory().numpy()
    n0 = K.STEP_STATS["calls"]
    r = K.step(X, labels, (0, 6), Qx, k, report=dst)
    assert K.STEP_STATS["calls"] == n0 + 1
    assert bytes(dst[:r.report_len]) == dmlp.format_report(cs_ref)
    np.testing.assert_array_equal(r.label.cpu().numpy(), lab_ref)
    assert r.path == 0 and r.n_escalated >= 1


@pytest.mark.parametrize("N,Q,A", [(6000, 700, 32), (1000, 300, 40), (130, 65, 7), (4097, 129, 64)])
def test_device_render_matches_host_render(torch_cuda, N, Q, A):
    """dmlp_render_rows (prep.hip k_render): the screen's fp16 operands rendered on the device
    from the lossless int32 rows (or fp64 rows) are bit for bit host_prep.cpp's render — tile
    image, xinit, point-major copy, max norm, query fragments and norms — and the int32 path
    writes back the exact fp64 rows.  Two dataset slices and two query blocks, each publishing its
    ready word from its last workgroup."""
    import ctypes as C
    torch = torch_cuda
    from distributed_machine_learning_project_amd import _lib
    L = _lib.lib()
    inp = dmlp.generate(N, Q, A, 0.0, 1000.0, 1, 8, 5, seed=N + A)
    kt = 1 if A <= 32 else 2 if A <= 64 else 4 if A <= 128 else 8
    W = kt * 32
    nt = (N + 63) // 64
    mu = np.zeros(A)
    L.dmlp_cpu_center(inp.X.ctypes.data, N, A, mu.ctypes.data)
    img_h = np.zeros(nt * 64 * W, np.uint16)
    xin_h = np.zeros(nt * 64, np.float32)
    nmax_h = C.c_uint()
    assert L.dmlp_cpu_prep_data(inp.X.ctypes.data, N, A, mu.ctypes.data, kt, img_h.ctypes.data,
                                xin_h.ctypes.data, C.byref(nmax_h)) == 0
    qhi_h = np.zeros(Q * W, np.uint16)
    qn_h = np.zeros(Q, np.float32)
    assert L.dmlp_cpu_prep_queries(inp.Qx.ctypes.data, Q, A, mu.ctypes.data, kt,
                                   qhi_h.ctypes.data, qn_h.ctypes.data) == 0
    x32 = np.zeros(N * A, np.int32)
    q32 = np.zeros(Q * A, np.int32)
    assert L.dmlp_cpu_rows_i32(inp.X.ctypes.data, N * A, x32.ctypes.data) == 0
    assert L.dmlp_cpu_rows_i32(inp.Qx.ctypes.data, Q * A, q32.ctypes.data) == 0
    dev = torch.device("cuda")
    p = lambda t: t.data_ptr()
    mu_d = torch.from_numpy(mu).to(dev)
    for src in ("i32", "f64"):
        img = torch.zeros(nt * 64 * W, dtype=torch.int16, device=dev)
        xin = torch.zeros(nt * 64, dtype=torch.float32, device=dev)
        xrow = torch.zeros(nt * 64 * W, dtype=torch.int16, device=dev)
        words = torch.zeros(16, dtype=torch.int32, device=dev)  # nmax, bad, done[4], rdy[4]
        Xd = torch.zeros(N * A, dtype=torch.float64, device=dev)
        qhi = torch.zeros(Q * W, dtype=torch.int16, device=dev)
        qn = torch.zeros(Q, dtype=torch.float32, device=dev)
        Qd = torch.zeros(Q * A, dtype=torch.float64, device=dev)
        xs = torch.from_numpy(x32).to(dev) if src == "i32" else torch.from_numpy(inp.X.ravel()).to(dev)
        qs = torch.from_numpy(q32).to(dev) if src == "i32" else torch.from_numpy(inp.Qx.ravel()).to(dev)
        w0 = p(words)
        half_t = nt // 2
        for j, (t0, t1) in enumerate(((0, half_t), (half_t, nt))):
            args = (p(xs), None) if src == "i32" else (None, p(xs))
            assert L.dmlp_render_rows(kt, A, *args, t0 * 64, (t1 - t0) * 64, N, p(mu_d), p(Xd), 0,
                                      p(img), p(xin), p(xrow), w0, w0 + 4, w0 + 8 + 4 * j,
                                      w0 + 24 + 4 * j, None) == 0
        hq = Q // 2
        for j, (q0, q1) in enumerate(((0, hq), (hq, Q))):
            args = (p(qs), None) if src == "i32" else (None, p(qs))
            assert L.dmlp_render_rows(kt, A, *args, q0, q1 - q0, Q, p(mu_d), p(Qd), 1, p(qhi),
                                      p(qn), None, None, w0 + 4, w0 + 16 + 4 * j, w0 + 32 + 4 * j,
                                      None) == 0
        torch.cuda.synchronize()
        np.testing.assert_array_equal(img.cpu().numpy().view(np.uint16), img_h)
        np.testing.assert_array_equal(xin.cpu().numpy(), xin_h)
        # the point-major copy: each point's W fp16 values in attribute order
        ref_row = np.zeros((nt * 64, W), np.uint16)
        t = np.arange(nt * 64)
        for a0 in range(0, W, 8):
            kt_, kg = a0 // 32, (a0 // 8) % 4
            idx = (((t >> 6) * 4 + ((t & 63) >> 4)) * kt + kt_) * 64 + kg * 16 + (t & 15)
            ref_row[:, a0:a0 + 8] = img_h.reshape(-1, 8)[idx]
        np.testing.assert_array_equal(xrow.cpu().numpy().view(np.uint16).reshape(-1, W), ref_row)
        np.testing.assert_array_equal(qhi.cpu().numpy().view(np.uint16), qhi_h)
        np.testing.assert_array_equal(qn.cpu().numpy(), qn_h)
        w = words.cpu().numpy().view(np.uint32)
        assert w[0] == nmax_h.value and w[1] == 0
        assert list(w[6:8]) == [1, 1] and list(w[8:10]) == [1, 1]  # every ready word published
        if src == "i32":
            np.testing.assert_array_equal(Xd.cpu().numpy(), inp.X.ravel())
            np.testing.assert_array_equal(Qd.cpu().numpy(), inp.Qx.ravel())
    # an fp64 value outside the fp16 range flags *bad
    X2 = inp.X.copy()
    X2[N // 2, 0] = 1.0e6
    xs = torch.from_numpy(X2.ravel()).to(dev)
    words = torch.zeros(4, dtype=torch.int32, device=dev)
    img = torch.zeros(nt * 64 * W, dtype=torch.int16, device=dev)
    xin = torch.zeros(nt * 64, dtype=torch.float32, device=dev)
    assert L.dmlp_render_rows(kt, A, None, p(xs), 0, nt * 64, N, p(mu_d), None, 0, p(img), p(xin),
                              None, p(words), p(words) + 4, None, None, None) == 0
    torch.cuda.synchronize()
    assert int(words[1]) == 1
