"""Local (single-device) exact k-NN: the compute backend every parallel strategy calls.

GPU path (MI355X, HIP kernels in libdmlp.so), per KNN call:
  prepare_dataset  : fp64 rows -> centred bf16 hi/lo MFMA fragments + fp32 norms   (K1)
  screen           : bf16x3 MFMA scores, streaming per-query threshold, candidates  (K2+K3)
  refine           : exact fp64 re-rank (reference order, no FMA), exact top-k,
                     fused vote + FNV checksum                                      (K2,K3,K5,K6,K7)
  fallback         : exact fp64 distance rows + stable sort, for k beyond the screen's
                     capacity, pathological ties, or data outside the screen's range (K2, K8-free)
CPU path: libdmlp's threaded brute force (or the KD-tree of bench.debug).

Screen error bound (per query q, fp32 score a = <q',x'> - |x'|^2/2 with q' = q - mu):
  bf16 split residual |c - hi - lo| <= 2^-16 |c| per operand, the dropped lo*lo term, and
  (3*A + 8) fp32 roundings of partial sums bounded by |q'|^2 + |x'|^2 give
      |a - a_exact| <= (3*2^-16 + (3A+8)*2^-24) * (|q'|^2 + max|x'|^2)
  which is doubled for safety: eps_rel below.  Everything within 2*eps of the k-th best buffered
  score survives, so the exact re-rank sees every point of the exact top-k (ties included).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import numpy as np

from .. import _lib

SCREEN_KMAX_A = 32      # cap 128 class
SCREEN_KMAX_B = 128     # cap 256 class
SCREEN_MAX_KT = 4       # A <= 128 on the screen path
NUM_CUS = 256
# "x1": single-term bf16 screen (default) | "stream": 3-term streaming screen | "lds": LDS-shared
SCREEN_IMPL = os.environ.get("DMLP_SCREEN", "x1")


def eps_rel(A: int) -> float:
    return 2.0 * (3.0 * 2.0 ** -16 + (3 * A + 8) * 2.0 ** -24)


# ======================================================================= CPU backend
def knn_cpu(X: np.ndarray, Qx: np.ndarray, k: np.ndarray, kstride: int | None = None,
            nthreads: int = 0, method: str = "brute"):
    """Exact top-k on the host.  Returns (dist [Q,kstride] f64, ids [Q,kstride] i32)."""
    X = np.ascontiguousarray(X, np.float64)
    Qx = np.ascontiguousarray(Qx, np.float64)
    k = np.ascontiguousarray(k, np.int32)
    Q = Qx.shape[0]
    ks = max(1, int(k.max()) if Q else 1) if kstride is None else kstride
    d = np.full((Q, ks), np.inf, np.float64)
    i = np.full((Q, ks), -1, np.int32)
    L = _lib.lib()
    if method == "kdtree":
        rc = L.dmlp_kdtree_knn(X.ctypes.data, X.shape[0], X.shape[1], Qx.ctypes.data, Q,
                               k.ctypes.data, ks, d.ctypes.data, i.ctypes.data)
    else:
        rc = L.dmlp_cpu_knn(X.ctypes.data, X.shape[0], X.shape[1], Qx.ctypes.data, Q,
                            k.ctypes.data, ks, d.ctypes.data, i.ctypes.data, nthreads)
    _lib.check(rc, "cpu knn")
    return d, i


def finalize_cpu(ids: np.ndarray, k: np.ndarray, labels: np.ndarray):
    ids = np.ascontiguousarray(ids, np.int32)
    k = np.ascontiguousarray(k, np.int32)
    labels = np.ascontiguousarray(labels, np.int32)
    Q = len(k)
    lab = np.empty(Q, np.int32)
    cs = np.empty(Q, np.uint64)
    _lib.check(_lib.lib().dmlp_cpu_finalize(None, ids.ctypes.data, ids.shape[1] if Q else 0,
                                            k.ctypes.data, Q, labels.ctypes.data,
                                            lab.ctypes.data, cs.ctypes.data), "cpu finalize")
    return lab, cs


def merge_cpu(lists_d: np.ndarray, lists_i: np.ndarray, k: np.ndarray, kout: int | None = None):
    """lists_*: [L, Q, kin] sorted per-shard top-k lists -> merged [Q, kout]."""
    Ld = np.ascontiguousarray(lists_d, np.float64)
    Li = np.ascontiguousarray(lists_i, np.int32)
    k = np.ascontiguousarray(k, np.int32)
    L, Q, kin = Ld.shape
    kout = kout or max(1, int(k.max()) if Q else 1)
    d = np.full((Q, kout), np.inf, np.float64)
    i = np.full((Q, kout), -1, np.int32)
    _lib.check(_lib.lib().dmlp_cpu_merge(Ld.ctypes.data, Li.ctypes.data, L, Q * kin, kin,
                                         k.ctypes.data, Q, d.ctypes.data, i.ctypes.data, kout),
               "cpu merge")
    return d, i


# ======================================================================= GPU backend
def _torch():
    import torch
    return torch


def _stream():
    torch = _torch()
    return torch.cuda.current_stream().cuda_stream


def _p(t):
    if t is None:
        return None
    if not t.is_contiguous():
        raise ValueError("native kernels need contiguous tensors")
    return t.data_ptr()


@dataclass
class DeviceDataset:
    """A dataset resident on one GPU, prepared once per KNN call (timed, like the reference's
    pack/scatter) and reusable across query batches."""
    X: "object"            # torch f64 [N, A] (cuda)
    labels: "object"       # torch i32 [N] or None
    label_lo: int
    label_hi: int
    KT: int
    mu: "object"
    xfrag: "object"
    xinit: "object"
    xnmax_bits: "object"   # torch i32 [1] (fp32 bits)
    bad: "object"          # torch i32 [1]
    screen_ok: bool

    @property
    def N(self):
        return self.X.shape[0]

    @property
    def A(self):
        return self.X.shape[1]

    @property
    def n_tiles(self):
        return (self.N + 63) // 64


def prepare_dataset(X, labels=None, label_range=None) -> DeviceDataset:
    torch = _torch()
    L = _lib.lib()
    X = X.contiguous()
    assert X.is_cuda and X.dtype == torch.float64 and X.dim() == 2
    N, A = X.shape
    KT = max(1, (A + 31) // 32)
    screen_ok = KT <= SCREEN_MAX_KT and N > 0
    dev = X.device
    mu = torch.empty(max(A, 1), dtype=torch.float64, device=dev)
    xnmax = torch.zeros(1, dtype=torch.int32, device=dev)
    bad = torch.zeros(1, dtype=torch.int32, device=dev)
    n_tiles = (N + 63) // 64
    if screen_ok:
        xfrag = torch.empty(n_tiles * 64 * KT * 32 * 2, dtype=torch.int16, device=dev)
        xinit = torch.empty(n_tiles * 64, dtype=torch.float32, device=dev)
        s = _stream()
        _lib.check(L.dmlp_center(_p(X), N, A, _p(mu), s), "center")
        _lib.check(L.dmlp_prep_data(_p(X), N, A, _p(mu), KT, _p(xfrag), _p(xinit), _p(xnmax),
                                    _p(bad), s), "prep_data")
    else:
        xfrag = xinit = None
    if labels is not None:
        labels = labels.to(device=dev, dtype=torch.int32).contiguous()
        if label_range is None:
            lo = int(labels.min().item()) if N else 0
            hi = int(labels.max().item()) + 1 if N else 1
        else:
            lo, hi = label_range
    else:
        lo, hi = 0, 1
    return DeviceDataset(X, labels, lo, hi, KT, mu, xfrag, xinit, xnmax, bad, screen_ok)


@dataclass
class DeviceResult:
    dist: "object"     # torch f64 [Q, kstride]
    ids: "object"      # torch i32 [Q, kstride]
    label: "object"    # torch i32 [Q] or None
    checksum: "object"  # torch i64 [Q] (uint64 bits) or None
    k: np.ndarray
    n_fallback: int = 0
    n_escalated: int = 0   # single-term screen overflows re-screened with the 3-term kernel


def _choose_slices_stream(nq: int, qw: int, n_tiles: int, waves_per_cu: int = 4,
                          s_min: int = 1) -> int:
    """Data slices for the streaming screens: one wave per (query block, slice).
    Pick the smallest S whose last round of waves is >= 90 % full (the tail), else the best;
    never fewer than needed to keep a slice inside the kernel's group-index range (s_min)."""
    nqb = (nq + qw - 1) // qw
    slots = waves_per_cu * NUM_CUS
    s_min = max(1, s_min, -(-n_tiles * 64 // (1 << 29)))
    if nqb >= slots:
        # every extra slice repeats each query's threshold warm-up (candidate work grows ~S):
        # with a full round of waves already, a partial last round is cheaper than S > 1
        return s_min
    best, best_eff = s_min, 0.0
    for S in range(s_min, s_min + 64):
        if S > max(s_min, n_tiles // 4):
            break
        w = nqb * S
        eff = w / (math.ceil(w / slots) * slots)
        if eff >= 0.9:
            return S
        if eff > best_eff + 1e-9:
            best, best_eff = S, eff
    return best

def _choose_slices(nq: int, waves: int, n_tiles: int) -> int:
    nqb = (nq + waves * 16 - 1) // (waves * 16)
    S = 1
    while nqb * S < 2 * NUM_CUS and S * 2 <= max(1, n_tiles) and S < 256:
        S *= 2
    return S


def knn_gpu(ds: DeviceDataset, Qx, k_host: np.ndarray, finalize: bool = True,
            exact: bool = False, kstride: int | None = None) -> DeviceResult:
    """Exact top-k of every query row of Qx (torch f64 cuda [Q, A]) against ds.

    k_host: numpy int32 [Q] (host copy of the per-query k; drives the dispatch)."""
    torch = _torch()
    L = _lib.lib()
    Qx = Qx.contiguous()
    Q, A = Qx.shape
    assert A == ds.A
    dev = Qx.device
    k_host = np.ascontiguousarray(k_host, np.int32)
    ks = max(1, int(k_host.max()) if Q else 1) if kstride is None else kstride
    k_dev = torch.from_numpy(k_host).to(dev, non_blocking=True)
    out_d = torch.full((Q, ks), float("inf"), dtype=torch.float64, device=dev)
    out_i = torch.full((Q, ks), -1, dtype=torch.int32, device=dev)
    want_fin = finalize and ds.labels is not None
    lab = torch.empty(Q, dtype=torch.int32, device=dev) if want_fin else None
    cs = torch.empty(Q, dtype=torch.int64, device=dev) if want_fin else None
    s = _stream()
    N = ds.N
    kk = np.minimum(k_host, N)  # k > N: pad with (+inf,-1) like bench_2's sentinel

    _apply_env_switches(L)
    use_screen = ds.screen_ok and not exact and Q > 0
    cls_a = np.nonzero((kk >= 1) & (kk <= SCREEN_KMAX_A))[0] if use_screen else np.empty(0, np.int64)
    cls_b = (np.nonzero((kk > SCREEN_KMAX_A) & (kk <= SCREEN_KMAX_B))[0]
             if use_screen else np.empty(0, np.int64))
    on_screen = np.zeros(Q, bool)
    on_screen[cls_a] = True
    on_screen[cls_b] = True
    status = torch.zeros(Q, dtype=torch.int32, device=dev)

    if use_screen and (len(cls_a) or len(cls_b)):
        KT = ds.KT
        qhi = torch.empty(Q * KT * 32, dtype=torch.int16, device=dev)
        qlo = torch.empty(Q * KT * 32, dtype=torch.int16, device=dev)
        qn = torch.empty(Q, dtype=torch.float32, device=dev)
        _lib.check(L.dmlp_prep_queries(_p(Qx), Q, A, _p(ds.mu), KT, _p(qhi), _p(qlo), _p(qn),
                                       _p(ds.bad), s), "prep_queries")
        kdev_eff = torch.from_numpy(kk.astype(np.int32)).to(dev, non_blocking=True)
        er = eps_rel(A)
        # k <= 32 and A <= 64: single-term (x1) or 3-term barrier-free streaming kernel;
        # otherwise the LDS-shared 3-term kernel.  x1 queries whose candidates overflow (data
        # too tight for the single-term bound) escalate to the 3-term screen, and only what
        # overflows there takes the exact fallback.
        x1_ok = SCREEN_IMPL == "x1" and L.dmlp_screen_x1_qw(KT) > 0
        stream_ok = SCREEN_IMPL != "lds" and L.dmlp_screen_stream_qw(KT) > 0

        def screen_pass(idx, impl):
            nq = len(idx)
            kcls = int(kk[idx].max())
            if impl == "x1":
                cap = L.dmlp_screen_x1_cap(kcls)
                S = _choose_slices_stream(nq, L.dmlp_screen_x1_qw(KT), ds.n_tiles,
                                          L.dmlp_screen_x1_waves_per_cu(kcls),
                                          int(L.dmlp_screen_x1_min_slices(ds.n_tiles)))
            elif impl == "stream":
                cap = L.dmlp_screen_stream_cap(kcls)
                S = _choose_slices_stream(nq, L.dmlp_screen_stream_qw(KT), ds.n_tiles,
                                          L.dmlp_screen_stream_waves_per_cu(kcls))
            else:
                cap = 128 if kcls <= SCREEN_KMAX_A else 256
                S = _choose_slices(nq, L.dmlp_screen_waves(KT, cap), ds.n_tiles)
            qidx = torch.from_numpy(idx.astype(np.int32)).to(dev, non_blocking=True)
            cand_ids = torch.empty(nq * S * cap, dtype=torch.int32, device=dev)
            cand_cnt = torch.empty(nq * S, dtype=torch.int32, device=dev)
            if impl == "x1":
                cand_h = torch.empty(nq * S, dtype=torch.float32, device=dev)
                _lib.check(L.dmlp_screen_x1(KT, A, _p(ds.xfrag), _p(ds.xinit), ds.n_tiles, N,
                                            _p(qhi), _p(qn), _p(qidx), _p(kdev_eff), nq, kcls,
                                            _p(ds.xnmax_bits), _p(ds.bad), S, _p(cand_ids),
                                            _p(cand_cnt), _p(cand_h), s), "screen_x1")
                _lib.check(L.dmlp_refine_groups(
                    cap, _p(cand_ids), _p(cand_cnt), _p(cand_h), S, _p(ds.X), A, _p(Qx),
                    _p(ds.xfrag), _p(ds.xinit), _p(qhi), KT, N, _p(qidx), _p(kdev_eff), nq,
                    _p(out_d), _p(out_i), ks, _p(ds.labels) if want_fin else None, ds.label_lo,
                    ds.label_hi, _p(lab), _p(cs), _p(status), s), "refine_groups")
                return
            elif impl == "stream":
                _lib.check(L.dmlp_screen_stream(KT, _p(ds.xfrag), _p(ds.xinit), ds.n_tiles,
                                                _p(qhi), _p(qlo), _p(qn), _p(qidx), _p(kdev_eff),
                                                nq, kcls, _p(ds.xnmax_bits), _p(ds.bad), er, S,
                                                _p(cand_ids), _p(cand_cnt), s), "screen_stream")
            else:
                _lib.check(L.dmlp_screen(KT, cap, _p(ds.xfrag), _p(ds.xinit), ds.n_tiles,
                                         _p(qhi), _p(qlo), _p(qn), _p(qidx), _p(kdev_eff), nq,
                                         _p(ds.xnmax_bits), _p(ds.bad), er, S, _p(cand_ids),
                                         _p(cand_cnt), s), "screen")
            _lib.check(L.dmlp_refine(cap, _p(cand_ids), _p(cand_cnt), S, _p(ds.X), A, _p(Qx),
                                     _p(qidx), _p(kdev_eff), nq, _p(out_d), _p(out_i), ks,
                                     _p(ds.labels) if want_fin else None, ds.label_lo,
                                     ds.label_hi, _p(lab), _p(cs), _p(status), s), "refine")

        n_esc = 0
        first_a = "x1" if x1_ok else ("stream" if stream_ok else "lds")
        if len(cls_a):
            screen_pass(cls_a, first_a)
        if len(cls_b):
            screen_pass(cls_b, "lds")
        # one host sync: which screened queries overflowed?
        n_ovf = int(status.sum().item())
        if n_ovf and first_a == "x1":
            st = status.cpu().numpy()
            esc = cls_a[st[cls_a] != 0]
            n_esc = len(esc)
            if n_esc:
                screen_pass(esc, "stream" if stream_ok else "lds")
                n_ovf = int(status.sum().item())
    else:
        n_ovf = n_esc = 0

    fb = np.nonzero(~on_screen & (kk >= 1))[0]
    if n_ovf:
        ovf = np.nonzero(status.cpu().numpy())[0]
        fb = np.union1d(fb, ovf)
    if len(fb):
        _fallback_exact(ds, Qx, fb, kk, out_d, out_i)
    if want_fin:
        # queries not (correctly) finalized by refine: fallback ones, k == 0, and k > N (the
        # checksum then also covers the (+inf, -1) padding, as the CPU path does)
        rest = np.union1d(fb, np.nonzero((kk < 1) | (k_host > N))[0]).astype(np.int32)
        if len(rest):
            ridx = torch.from_numpy(rest).to(dev, non_blocking=True)
            _lib.check(L.dmlp_finalize(_p(out_d), _p(out_i), ks, _p(k_dev), _p(ridx), len(rest),
                                       _p(ds.labels), ds.label_lo, ds.label_hi, _p(lab), _p(cs),
                                       s), "finalize")
    return DeviceResult(out_d, out_i, lab, cs, k_host, int(len(fb)), int(n_esc))


_ENV_APPLIED = [False]


def _apply_env_switches(L):
    """DMLP_STREAM_GROUPS=0 switches the streaming screen to per-point appends (A/B only)."""
    if not _ENV_APPLIED[0]:
        if os.environ.get("DMLP_STREAM_GROUPS", "1") == "0":
            L.dmlp_set_stream_groups(0)
        if os.environ.get("DMLP_X1_CHECK"):
            L.dmlp_set_x1_check(int(os.environ["DMLP_X1_CHECK"]))
        if os.environ.get("DMLP_STREAM_SUB"):
            L.dmlp_set_stream_sub(int(os.environ["DMLP_STREAM_SUB"]))
        _ENV_APPLIED[0] = True


def _fallback_exact(ds: DeviceDataset, Qx, fb: np.ndarray, kk: np.ndarray, out_d, out_i):
    """Native exact path (fallback.hip) in row chunks that keep nb*N < 2^27: k <= 2048 by a
    per-row radix select over the exact distance bits (+ LDS bitonic sort of the survivors);
    larger k by exact rows in descending-id order + a stable segmented radix sort."""
    torch = _torch()
    L = _lib.lib()
    N, A = ds.N, ds.A
    dev = Qx.device
    s = _stream()
    kdev = torch.from_numpy(np.ascontiguousarray(kk, np.int32)).to(dev, non_blocking=True)
    ksel = L.dmlp_fallback_select_kmax()
    small = fb[kk[fb] <= ksel]
    big = fb[kk[fb] > ksel]
    for rows_idx, sel in ((small, True), (big, False)):
        if len(rows_idx) == 0:
            continue
        rows = max(1, min(len(rows_idx), (1 << 27) // max(1, N)))
        ws_bytes = L.dmlp_fallback_select_bytes(rows, N) if sel else L.dmlp_fallback_bytes(rows, N)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        fn = L.dmlp_fallback_select if sel else L.dmlp_fallback_topk
        for c0 in range(0, len(rows_idx), rows):
            sub = rows_idx[c0:c0 + rows]
            qidx = torch.from_numpy(sub.astype(np.int32)).to(dev, non_blocking=True)
            _lib.check(fn(_p(ds.X), N, A, _p(Qx), _p(qidx), _p(kdev), len(sub), _p(ws), ws_bytes,
                          _p(out_d), _p(out_i), out_d.shape[1], s),
                       "fallback_select" if sel else "fallback_topk")


def merge_gpu(lists_d, lists_i, k_dev, kout: int):
    """lists_*: torch [L, Q, kin] sorted lists on one GPU -> merged [Q, kout] (K4)."""
    torch = _torch()
    Ld = lists_d.contiguous()
    Li = lists_i.contiguous()
    Lc, Q, kin = Ld.shape
    out_d = torch.full((Q, kout), float("inf"), dtype=torch.float64, device=Ld.device)
    out_i = torch.full((Q, kout), -1, dtype=torch.int32, device=Ld.device)
    _lib.check(_lib.lib().dmlp_merge(_p(Ld), _p(Li), Lc, Q * kin, kin, _p(k_dev), Q, _p(out_d),
                                     _p(out_i), kout, _stream()), "merge")
    return out_d, out_i


def finalize_gpu(ds_labels, label_range, dist, ids, k_dev):
    torch = _torch()
    Q, ks = ids.shape
    lab = torch.empty(Q, dtype=torch.int32, device=ids.device)
    cs = torch.empty(Q, dtype=torch.int64, device=ids.device)
    _lib.check(_lib.lib().dmlp_finalize(_p(dist), _p(ids), ks, _p(k_dev), None, Q, _p(ds_labels),
                                        label_range[0], label_range[1], _p(lab), _p(cs),
                                        _stream()), "finalize")
    return lab, cs


def format_report_dev(cs, qid_base: int = 0):
    """Render "Query <id> checksum: <u64>\\n" lines on the GPU.  Returns (device uint8 tensor,
    byte count); one host sync for the count."""
    torch = _torch()
    L = _lib.lib()
    cs = cs.contiguous()
    nq = cs.numel()
    if nq == 0:
        return torch.empty(0, dtype=torch.uint8, device=cs.device), 0
    off = torch.empty(L.dmlp_format_scratch(nq), dtype=torch.int64, device=cs.device)
    out = torch.empty(L.dmlp_format_bound(nq), dtype=torch.uint8, device=cs.device)
    _lib.check(L.dmlp_format_report(_p(cs), nq, qid_base, _p(off), _p(out), _stream()), "format")
    return out, int(off[nq].item())


_PINNED = {}


def _pinned_bytes(n: int):
    """Grow-only page-locked host staging buffer (D2H at DMA rate, no per-call pinning)."""
    torch = _torch()
    buf = _PINNED.get("report")
    if buf is None or buf.numel() < n:
        buf = torch.empty(max(n, 1 << 20), dtype=torch.uint8).pin_memory()
        _PINNED["report"] = buf
    return buf


def format_report_gpu(cs, qid_base: int = 0):
    """Report bytes on the host: GPU formatter + one D2H into a pinned staging buffer.
    Returns a read-only memoryview valid until the next call (write it out or copy it)."""
    dev_text, n = format_report_dev(cs, qid_base)
    if n == 0:
        return memoryview(b"")
    host = _pinned_bytes(n)
    host[:n].copy_(dev_text[:n])
    return memoryview(host.numpy())[:n].toreadonly()