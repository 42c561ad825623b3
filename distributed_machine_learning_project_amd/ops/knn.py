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
import time
from dataclasses import dataclass

import numpy as np

from .. import _lib

SCREEN_KMAX_A = 32      # cap 128 class
SCREEN_KMAX_B = 128     # cap 256 class
SCREEN_KMAX_C = 256     # cap 512 class
SCREEN_MAX_KT = 8       # A <= 256 on the screen path: the single-term screen and the LDS 3-term
LDS_MAX_KT = 8          # screen (KT = 8 tiles stream through LDS as two 32 KiB stages)
NUM_CUS = 256
# "x1": single-term screen (fp16 operands on the host-operand path) (default) | "stream": 3-term streaming screen | "lds": LDS-shared
SCREEN_IMPL = os.environ.get("DMLP_SCREEN", "x1")
# slices of the host-rendered screen operands, each copied as soon as it is converted (1: measured
# best on the bench shape — every extra slice costs ~20 us of copy-API time on the host)
# host render + H2D of the screen operands in 2 pipelined slices: the first copy starts after half
# the render (profiles/r2t_host_ops_chunks.txt: median 2.63 vs 2.74 and 3.03 vs 3.18 ms/step on two boxes)
HOST_OPS_CHUNKS = int(os.environ.get("DMLP_HOST_OPS_CHUNKS", "2"))
# query parts of the host-operand pipeline (knn_gpu_pipelined): each part's screen starts as soon
# as its operands land, on its own stream, while the host renders the next part.  1 (one screen
# after the whole query image) is the default: 2 / 4 parts measured 2.76 / 4.29 ms against 2.58
# (profiles/r4j_query_parts_ab.txt) — concurrent part screens cost more than the front they hide
HOST_OPS_PARTS = int(os.environ.get("DMLP_HOST_OPS_PARTS", "1"))
# fp64 rows of the host-operand pipeline cross PCIe as lossless int32 when every value is a
# 6-decimal number (knn._issue_rows)
ROWS_I32 = os.environ.get("DMLP_ROWS_I32", "1") != "0"
# k in (32, 256] (the cap-256 / cap-512 classes) on the single-term LDS screen over the host's
# fp16 operands when the host rendered them (no device hi/lo image, a third of the MFMA work);
# its overflows escalate to the 3-term LDS screen.  DMLP_LDS_SINGLE=0: always 3-term (A/B)
LDS_SINGLE = os.environ.get("DMLP_LDS_SINGLE", "1") != "0"
# ... and, on the same operands, by the two-pass single-term x1 screen instead (screen_x1.hip:
# per-query seeds from S1 slices at k' = ceil(k / S1), then one COLLECT pass at that fixed
# threshold; refine over <= X1K_CCAP groups per query and slice).  DMLP_X1K=0: the LDS screen
X1K = os.environ.get("DMLP_X1K", "1") != "0"
X1K_S1 = 16        # first-pass slices: k' = ceil(k / 16) <= 16 for k <= 256 (the SUB = 16 variant)
X1K_CCAP = 1024    # COLLECT group ids per (query, slice)


def screen_kt(A: int) -> int:
    """32-attribute fragments per row of the screen images (dmlp.h dmlp_screen_kt): A <= 256
    rounds up to 1, 2, 4 or 8, the single-term screen's variants."""
    kt = max(1, (A + 31) // 32)
    return kt if kt > 8 else 1 << (kt - 1).bit_length()


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


_RAW_STREAM = []


def _stream():
    """The current stream's raw handle, without building a torch Stream object (a per-call hot
    path: ~15 uses per pipelined call)."""
    torch = _torch()
    if not _RAW_STREAM:
        f = getattr(torch._C, "_cuda_getCurrentRawStream", None)
        _RAW_STREAM.append(f)
    f = _RAW_STREAM[0]
    if f is not None:
        return f(torch.cuda.current_device())
    return torch.cuda.current_stream().cuda_stream


_SCRATCH = {}


def _scratch(name, numel, dtype, dev):
    """Grow-only device scratch reused across calls (never returned to callers): every
    pipelined call has completed on the device before it returns, so the next call may reuse
    its buffers.  Saves the per-call allocator round trips of the operand images."""
    torch = _torch()
    key = (name, str(dev), dtype)
    t = _SCRATCH.get(key)
    if t is None or t.numel() < numel:
        t = _SCRATCH[key] = torch.empty(max(numel, 1), dtype=dtype, device=dev)
    return t[:numel]


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
    hl: int = 2            # fragment halves in xfrag: 2 = prep.hip's hi/lo, 1 = host hi-only image

    def ensure_full_frags(self):
        """The 3-term screens read the lo halves too: render prep.hip's hi/lo image on the device
        from the (landed) fp64 rows when the dataset arrived as the host's hi-only image."""
        if self.hl == 2 or not self.screen_ok:
            return
        torch = _torch()
        L = _lib.lib()
        dev = self.X.device
        n_tiles = self.n_tiles
        xfrag = torch.empty(n_tiles * 64 * self.KT * 32 * 2, dtype=torch.int16, device=dev)
        xinit = torch.empty(n_tiles * 64, dtype=torch.float32, device=dev)
        xnmax = torch.zeros(1, dtype=torch.int32, device=dev)
        bad = torch.zeros(1, dtype=torch.int32, device=dev)
        _lib.check(L.dmlp_prep_data(_p(self.X), self.N, self.A, _p(self.mu), self.KT, _p(xfrag),
                                    _p(xinit), _p(xnmax), _p(bad), _stream()), "prep_data")
        self.xfrag, self.xinit, self.xnmax_bits, self.bad, self.hl = xfrag, xinit, xnmax, bad, 2

    @property
    def N(self):
        return self.X.shape[0]

    @property
    def A(self):
        return self.X.shape[1]

    @property
    def n_tiles(self):
        return (self.N + 63) // 64


def prepare_dataset(X, labels=None, label_range=None, mu=None) -> DeviceDataset:
    """mu (device f64 [A]), if given, is the centre to use instead of dmlp_center's (the
    host-prepared query operands of knn_gpu_pipelined were centred on it)."""
    torch = _torch()
    L = _lib.lib()
    X = X.contiguous()
    assert X.is_cuda and X.dtype == torch.float64 and X.dim() == 2
    N, A = X.shape
    KT = screen_kt(A)
    screen_ok = KT <= SCREEN_MAX_KT and N > 0
    dev = X.device
    mu_given = mu is not None
    if not mu_given:
        mu = torch.empty(max(A, 1), dtype=torch.float64, device=dev)
    xnmax = torch.zeros(1, dtype=torch.int32, device=dev)
    bad = torch.zeros(1, dtype=torch.int32, device=dev)
    n_tiles = (N + 63) // 64
    if screen_ok:
        xfrag = torch.empty(n_tiles * 64 * KT * 32 * 2, dtype=torch.int16, device=dev)
        xinit = torch.empty(n_tiles * 64, dtype=torch.float32, device=dev)
        s = _stream()
        if not mu_given:
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
                          s_min: int = 1, cus: int = NUM_CUS) -> int:
    """Data slices for the streaming screens: one wave per (query block, slice).
    Pick the smallest S whose last round of waves is >= 90 % full (the tail), else the best;
    never fewer than needed to keep a slice inside the kernel's group-index range (s_min)."""
    nqb = (nq + qw - 1) // qw
    slots = waves_per_cu * cus
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
    _ARENA.reset()
    r = _KnnCall(ds, Qx, k_host, finalize, exact, kstride).launch().finish()
    _ARENA.mark()
    return r


class _KnnCall:
    """One local k-NN call split into an asynchronous launch (prep + screen + refine on the
    current stream, no host sync) and a finish (one sync for the overflow status, then the
    3-term escalation / exact fallback / finalize of the few queries that need it).  The split
    lets knn_gpu_pipelined keep several query chunks in flight on their own streams."""

    def __init__(self, ds, Qx, k_host, finalize=True, exact=False, kstride=None, gpu_share=1.0,
                 out=None, prepped=None, qx_event=None, k_range=None):
        """prepped = (qhi, qn) device tensors rendered by the host (dmlp_cpu_prep_queries) with
        ds.mu; qx_event: the fp64 query rows are only complete once it fires (they are copied
        behind the screen) — everything that reads Qx waits for it."""
        torch = _torch()
        self.ds = ds
        self.Qx = Qx.contiguous()
        self.Q, self.A = self.Qx.shape
        assert self.A == ds.A
        self.dev = self.Qx.device
        self.k_host = np.ascontiguousarray(k_host, np.int32)
        Q = self.Q
        if k_range is not None and Q:  # (lower bound of min k, upper bound of max k)
            self.kmin, self.kmax = int(k_range[0]), int(k_range[1])
        else:
            self.kmin = int(self.k_host.min()) if Q else 0
            self.kmax = int(self.k_host.max()) if Q else 0
        self.ks = max(1, self.kmax) if kstride is None else kstride
        self.exact = exact
        self.gpu_share = gpu_share
        self.prepped = prepped
        self.pre_screen = None  # (cand_ids, cand_cnt, cand_h, S): x1 screen queued elsewhere
        self.qx_event = qx_event
        self.want_fin = finalize and ds.labels is not None
        # k > N: pad with (+inf,-1) like bench_2
        self.kk = self.k_host if self.kmax <= ds.N else np.minimum(self.k_host, ds.N)
        dev = self.dev
        self.k_dev = _h2d(self.k_host, dev)
        if out is not None:  # rows of caller-owned result tensors (pipelined chunks)
            self.out_d, self.out_i, self.lab, self.cs = out
        else:
            self.out_d = torch.empty((Q, self.ks), dtype=torch.float64, device=dev)
            self.out_i = torch.empty((Q, self.ks), dtype=torch.int32, device=dev)
            self.lab = torch.empty(Q, dtype=torch.int32, device=dev) if self.want_fin else None
            self.cs = torch.empty(Q, dtype=torch.int64, device=dev) if self.want_fin else None
        self.status = torch.empty(Q, dtype=torch.int32, device=dev)
        self._filled = False
        self._ovf = _ovf_counters(dev)
        self._ovf_slot = self._ovf.slot()

    def _fill_outputs(self):
        """(+inf, -1) padding of the result rows and a zero status, issued once, right before the
        first kernel that writes results — i.e. after the first screen is already queued, so
        these fills are not on the screen's critical path."""
        if not self._filled:
            self.out_d.fill_(float("inf"))
            self.out_i.fill_(-1)
            self.status.zero_()
            self._filled = True

    # ------------------------------------------------------------------ launch (async)
    def launch(self):
        torch = _torch()
        L = _lib.lib()
        _apply_env_switches(L)
        ds, kk, Q, A = self.ds, self.kk, self.Q, self.A
        # A <= 256 (KT <= 8): every class on a screen; wider rows take the exact path
        self.lds_ok = ds.KT <= LDS_MAX_KT
        self.use_screen = (ds.screen_ok and not self.exact and Q > 0 and
                           (self.lds_ok or (SCREEN_IMPL == "x1" and L.dmlp_screen_x1_qw(ds.KT) > 0)))
        empty = np.empty(0, np.int64)
        # common case (every k in [1, 32], k <= N): one class, identity query index, no per-query
        # host scans — this host path runs while the GPU waits for its first kernel
        self.all_a = self.use_screen and self.kmin >= 1 and self.kmax <= min(SCREEN_KMAX_A, ds.N)
        if self.all_a:
            self.cls_a, self.cls_b, self.cls_c = None, empty, empty
        else:
            self.cls_a = (np.nonzero((kk >= 1) & (kk <= SCREEN_KMAX_A))[0] if self.use_screen
                          else empty)
            self.cls_b = (np.nonzero((kk > SCREEN_KMAX_A) & (kk <= SCREEN_KMAX_B))[0]
                          if self.use_screen and self.lds_ok else empty)
            self.cls_c = (np.nonzero((kk > SCREEN_KMAX_B) & (kk <= SCREEN_KMAX_C))[0]
                          if self.use_screen and self.lds_ok else empty)
            self.on_screen = np.zeros(Q, bool)
            self.on_screen[self.cls_a] = True
            self.on_screen[self.cls_b] = True
            self.on_screen[self.cls_c] = True
        self.screened = self.use_screen and (self.all_a or len(self.cls_a) or len(self.cls_b)
                                             or len(self.cls_c))
        self.stream = _torch().cuda.current_stream()
        if not self.screened:
            return self
        KT = ds.KT
        dev = self.dev
        # k <= 32 and A <= 64: single-term (x1) or 3-term barrier-free streaming kernel;
        # otherwise the LDS-shared 3-term kernel.  x1 queries whose candidates overflow (data
        # too tight for the single-term bound) escalate to the 3-term screen, and only what
        # overflows there takes the exact fallback.
        x1_ok = SCREEN_IMPL == "x1" and L.dmlp_screen_x1_qw(KT) > 0
        self.stream_ok = SCREEN_IMPL != "lds" and L.dmlp_screen_stream_qw(KT) > 0
        self.first_a = "x1" if x1_ok else ("stream" if self.stream_ok else "lds")
        self.qhi = self.qlo = self.qn = None  # device (bf16) query operands, rendered on need
        if not (self.prepped is not None and ds.hl == 1 and self.first_a == "x1"):
            self._prep_on_device()
        self.kdev_eff = self.k_dev if kk is self.k_host else _h2d(kk.astype(np.int32), dev)
        if self.all_a or len(self.cls_a):
            self._screen_pass(self.cls_a, self.first_a)
        # k > 32: the single-term LDS screen on the host operands when they are here
        self.single_bc = (LDS_SINGLE and ds.hl == 1 and self.prepped is not None
                          and L.dmlp_screen_waves_hl(KT, 128, 1) > 0)
        lds_impl = "lds1" if self.single_bc else "lds"
        if self.single_bc and X1K and L.dmlp_screen_x1_qw(KT) > 0 and (len(self.cls_b)
                                                                       or len(self.cls_c)):
            # both k > 32 classes in one two-pass x1 screen
            self._screen_pass(np.concatenate([self.cls_b, self.cls_c]), "x1k")
            return self
        if len(self.cls_b):
            self._screen_pass(self.cls_b, lds_impl)
        if len(self.cls_c):
            self._screen_pass(self.cls_c, lds_impl)
        return self

    def _wait_qx(self):
        if self.qx_event is not None:
            _torch().cuda.current_stream().wait_event(self.qx_event)
            self.qx_event = None

    def _prep_on_device(self):
        torch = _torch()
        L = _lib.lib()
        ds, Q, A, KT, dev = self.ds, self.Q, self.A, self.ds.KT, self.dev
        self._wait_qx()
        self.qhi = torch.empty(Q * KT * 32, dtype=torch.int16, device=dev)
        self.qlo = torch.empty(Q * KT * 32, dtype=torch.int16, device=dev)
        self.qn = torch.empty(Q, dtype=torch.float32, device=dev)
        _lib.check(L.dmlp_prep_queries(_p(self.Qx), Q, A, _p(ds.mu), KT, _p(self.qhi),
                                       _p(self.qlo), _p(self.qn), _p(ds.bad), _stream()),
                   "prep_queries")

    def x1_buffers(self, slot: int = 0):
        """Candidate buffers + slice count of this call's all-queries x1 pass, for a screen that
        dmlp_host_ops_x1_parts queues natively; launch() then only adds the refine."""
        torch = _torch()
        L = _lib.lib()
        KT, kcls, nq = self.ds.KT, self.kmax, self.Q
        cap = L.dmlp_screen_x1_cap(kcls)
        cus = max(1, int(round(NUM_CUS * self.gpu_share)))
        S = _choose_slices_stream(nq, L.dmlp_screen_x1_cols(KT, kcls), self.ds.n_tiles,
                                  L.dmlp_screen_x1_waves_per_cu_kt(KT, kcls),
                                  int(L.dmlp_screen_x1_min_slices(self.ds.n_tiles)), cus)
        # (scratch: one all-queries x1 pass per pipelined call, complete before it returns)
        self.pre_screen = (_scratch(f"x1_ids{slot}", nq * S * cap, torch.int32, self.dev),
                           _scratch(f"x1_cnt{slot}", nq * S, torch.int32, self.dev),
                           _scratch(f"x1_h{slot}", nq * S * 2, torch.float32, self.dev), S)
        return self.pre_screen

    def _screen_pass(self, idx, impl):
        torch = _torch()
        if impl not in ("x1", "lds1", "x1k") and self.qlo is None:
            self._prep_on_device()  # 3-term class / escalation after a host-prepared x1 pass
        L = _lib.lib()
        ds, kk, A, KT, dev = self.ds, self.kk, self.A, self.ds.KT, self.dev
        N = ds.N
        s = _stream()
        if idx is None:  # every query
            nq, kcls = self.Q, self.kmax
            qidx = _identity(nq, dev)
        else:
            nq = len(idx)
            kcls = int(kk[idx].max())
            qidx = _h2d(idx.astype(np.int32), dev)
        cus = max(1, int(round(NUM_CUS * self.gpu_share)))
        pre = self.pre_screen if impl == "x1" and idx is None else None
        self.pre_screen = None
        if pre is not None:
            cap = L.dmlp_screen_x1_cap(kcls)
            cand_ids, cand_cnt, cand_h, S = pre
        elif impl == "x1":
            cap = L.dmlp_screen_x1_cap(kcls)
            S = _choose_slices_stream(nq, L.dmlp_screen_x1_cols(KT, kcls), ds.n_tiles,
                                      L.dmlp_screen_x1_waves_per_cu_kt(KT, kcls),
                                      int(L.dmlp_screen_x1_min_slices(ds.n_tiles)), cus)
        elif impl == "x1k":
            cap = S = 0  # (_x1k_pass sizes its own buffers)
        elif impl == "stream":
            cap = L.dmlp_screen_stream_cap(kcls)
            S = _choose_slices_stream(nq, L.dmlp_screen_stream_qw(KT), ds.n_tiles,
                                      L.dmlp_screen_stream_waves_per_cu(kcls), 1, cus)
        else:
            cap = (128 if kcls <= SCREEN_KMAX_A else 256 if kcls <= SCREEN_KMAX_B else 512)
            S = _choose_slices(nq, L.dmlp_screen_waves_hl(KT, cap, 1 if impl == "lds1" else 2),
                               ds.n_tiles)
        if pre is None and impl != "x1k":
            cand_ids = torch.empty(nq * S * cap, dtype=torch.int32, device=dev)
            cand_cnt = torch.empty(nq * S, dtype=torch.int32, device=dev)
        fin = (_p(ds.labels) if self.want_fin else None, ds.label_lo, ds.label_hi, _p(self.lab),
               _p(self.cs), _p(self.status), self._ovf.ptr(self._ovf_slot), s)
        if impl == "x1":
            if pre is None:
                cand_h = torch.empty(nq * S * 2, dtype=torch.float32, device=dev)
            # the host's fp16 image (hl = 1) pairs with the host's fp16 query fragments, prep.hip's
            # bf16 image (hl = 2) with the device's bf16 ones
            if ds.hl == 1:
                if self.prepped is None:
                    raise RuntimeError("x1 on the host fp16 image needs the host query operands")
                x1_qhi, x1_qn = self.prepped
            else:
                if self.qhi is None:
                    self._prep_on_device()
                x1_qhi, x1_qn = self.qhi, self.qn
            if pre is None:
                _mark("screen_start")
                _lib.check(L.dmlp_screen_x1(KT, ds.hl, A, _p(ds.xfrag), _p(ds.xinit), ds.n_tiles, N,
                              _p(x1_qhi), _p(x1_qn), _p(qidx), _p(self.kdev_eff),
                              nq, kcls, _p(ds.xnmax_bits), _p(ds.bad), S,
                              _p(cand_ids), _p(cand_cnt), _p(cand_h), s),
                           "screen_x1")
            _mark("screen_done")
            if idx is None:
                # every query goes through this refine: it writes each row's (+inf, -1) padding
                # and each status itself, so no fill pass at all
                self._filled = True
            self._fill_outputs()
            self._wait_qx()
            _lib.check(L.dmlp_refine_groups(
                cap, _p(cand_ids), _p(cand_cnt), _p(cand_h), S, _p(ds.X), A, _p(self.Qx),
                _p(ds.xfrag), _p(ds.xinit), _p(x1_qhi), KT, ds.hl, N,
                _p(qidx) if idx is not None else None, _p(self.kdev_eff), nq,
                _p(self.out_d), _p(self.out_i), self.ks, *fin), "refine_groups")
            _mark("refine_done")
            self._keep = (qidx, cand_ids, cand_cnt, cand_h)
            return
        if impl == "x1k":
            self._x1k_pass(idx, qidx, nq, kcls, cus, fin, s)
            return
        if impl == "lds1":
            # single term on the host's fp16 image + query fragments: nothing rendered on the
            # device, the refine alone waits for the fp64 rows
            x1_qhi, x1_qn = self.prepped
            self._fill_outputs()
            _lib.check(L.dmlp_screen_hl(KT, cap, 1, A, _p(ds.xfrag), _p(ds.xinit), ds.n_tiles,
                                        _p(x1_qhi), None, _p(x1_qn), _p(qidx), _p(self.kdev_eff),
                                        nq, _p(ds.xnmax_bits), _p(ds.bad), 0.0, S, _p(cand_ids),
                                        _p(cand_cnt), s), "screen_hl")
            self._wait_qx()
            _lib.check(L.dmlp_refine(cap, _p(cand_ids), _p(cand_cnt), S, _p(ds.X), A,
                                     _p(self.Qx), _p(qidx), _p(self.kdev_eff), nq, _p(self.out_d),
                                     _p(self.out_i), self.ks, *fin), "refine")
            self._keep = (qidx, cand_ids, cand_cnt)
            return
        if ds.hl != 2:
            self._wait_qx()  # the device image is rendered from the fp64 rows
            ds.ensure_full_frags()
        self._fill_outputs()
        er = eps_rel(A)
        if impl == "stream":
            _lib.check(L.dmlp_screen_stream(KT, _p(ds.xfrag), _p(ds.xinit), ds.n_tiles,
                                            _p(self.qhi), _p(self.qlo), _p(self.qn), _p(qidx),
                                            _p(self.kdev_eff), nq, kcls, _p(ds.xnmax_bits),
                                            _p(ds.bad), er, S, _p(cand_ids), _p(cand_cnt), s),
                       "screen_stream")
        else:
            _lib.check(L.dmlp_screen(KT, cap, _p(ds.xfrag), _p(ds.xinit), ds.n_tiles,
                                     _p(self.qhi), _p(self.qlo), _p(self.qn), _p(qidx),
                                     _p(self.kdev_eff), nq, _p(ds.xnmax_bits), _p(ds.bad), er, S,
                                     _p(cand_ids), _p(cand_cnt), s), "screen")
        self._wait_qx()
        _lib.check(L.dmlp_refine(cap, _p(cand_ids), _p(cand_cnt), S, _p(ds.X), A, _p(self.Qx),
                                 _p(qidx), _p(self.kdev_eff), nq, _p(self.out_d), _p(self.out_i),
                                 self.ks, *fin), "refine")
        self._keep = (qidx, cand_ids, cand_cnt)

    def _x1k_pass(self, idx, qidx, nq, kcls, cus, fin, s):
        """k in (32, 256] on the single-term screen in two passes over the host's fp16 operands
        (screen_x1.hip dmlp_x1_seed / dmlp_screen_x1_collect) and the large-k group refine;
        overflowing queries report status 1 (finish() escalates them to the 3-term screen)."""
        torch = _torch()
        L = _lib.lib()
        ds, A, KT, dev, N = self.ds, self.A, self.ds.KT, self.dev, self.ds.N
        x1_qhi, x1_qn = self.prepped
        n_tiles = ds.n_tiles
        s_min = int(L.dmlp_screen_x1_min_slices(n_tiles))
        S2 = _choose_slices_stream(nq, L.dmlp_screen_x1_cols(KT, 16), n_tiles,
                                   L.dmlp_screen_x1_waves_per_cu_kt(KT, 16), s_min, cus)
        S1 = max(X1K_S1, S2)
        kp = -(-np.maximum(self.kk, 1) // S1)  # k' = ceil(k / S1) per query row (<= 16)
        kp_dev = _h2d(kp.astype(np.int32), dev)
        kmax1 = int(kp[idx].max()) if idx is not None else int(kp.max())
        cap1 = L.dmlp_screen_x1_cap(kmax1)
        ids1 = torch.empty(nq * S1 * cap1, dtype=torch.int32, device=dev)
        cnt1 = torch.empty(nq * S1, dtype=torch.int32, device=dev)
        h1 = torch.empty(nq * S1 * 2, dtype=torch.float32, device=dev)
        hseed = torch.empty(nq, dtype=torch.float32, device=dev)
        ids2 = torch.empty(nq * S2 * X1K_CCAP, dtype=torch.int32, device=dev)
        cnt2 = torch.empty(nq * S2, dtype=torch.int32, device=dev)
        h2 = torch.empty(nq * S2 * 2, dtype=torch.float32, device=dev)
        self._fill_outputs()
        _lib.check(L.dmlp_screen_x1(KT, 1, A, _p(ds.xfrag), _p(ds.xinit), n_tiles, N, _p(x1_qhi),
                                    _p(x1_qn), _p(qidx), _p(kp_dev), nq, kmax1, _p(ds.xnmax_bits),
                                    _p(ds.bad), S1, _p(ids1), _p(cnt1), _p(h1), s), "screen_x1 seed pass")
        _lib.check(L.dmlp_x1_seed(_p(h1), _p(cnt1), S1, nq, _p(hseed), s), "x1_seed")
        _lib.check(L.dmlp_screen_x1_collect(KT, A, _p(ds.xfrag), _p(ds.xinit), n_tiles, N,
                                            _p(x1_qhi), _p(x1_qn), _p(qidx), _p(self.kdev_eff), nq,
                                            _p(ds.xnmax_bits), _p(ds.bad), _p(hseed), X1K_CCAP, S2,
                                            _p(ids2), _p(cnt2), _p(h2), s), "screen_x1_collect")
        self._wait_qx()
        _lib.check(L.dmlp_refine_groups2(
            X1K_CCAP, _p(ids2), _p(cnt2), _p(h2), S2, _p(ds.X), A, _p(self.Qx), _p(ds.xfrag),
            _p(ds.xinit), _p(x1_qhi), KT, 1, N, _p(qidx), _p(self.kdev_eff), nq, _p(self.out_d),
            _p(self.out_i), self.ks, *fin[:-1], 1, fin[-1]), "refine_groups2")
        self._keep = (qidx, kp_dev, ids1, cnt1, h1, hseed, ids2, cnt2, h2)

    # ------------------------------------------------------------------ finish (one sync)
    def finish(self) -> DeviceResult:
        torch = _torch()
        L = _lib.lib()
        ds, kk, dev = self.ds, self.kk, self.dev
        N = ds.N
        if torch.cuda.current_stream() != self.stream:
            # finishing on another stream (pipelined chunks): keep the allocator from recycling
            # this call's buffers before that stream's escalation / finalize work has run
            cur = torch.cuda.current_stream()
            for t in (self.Qx, self.k_dev, self.out_d, self.out_i, self.lab, self.cs, self.status,
                      getattr(self, "qhi", None), getattr(self, "qlo", None),
                      getattr(self, "qn", None), getattr(self, "kdev_eff", None)):
                if t is not None:
                    t.record_stream(cur)
        self._wait_qx()
        self._fill_outputs()  # no screen ran (exact / fallback-only calls)
        n_ovf = n_esc = 0
        self.cs_modified = False  # set when work after launch() rewrites labels / checksums
        if self.screened:
            # the refine kernels count overflowed queries into this call's counter slot: one
            # 4-byte read (and the call's one host sync) instead of a reduce over the status
            n_ovf = self._ovf.read(self._ovf_slot, self.stream)
            esc_a = esc_bc = np.empty(0, np.int64)
            if n_ovf and (self.first_a == "x1" or self.single_bc):
                st = self.status.cpu().numpy()
                if self.first_a == "x1" and (self.stream_ok or self.lds_ok):
                    esc_a = np.nonzero(st)[0] if self.all_a else self.cls_a[st[self.cls_a] != 0]
                if self.single_bc and not self.all_a:
                    # single-term k > 32 classes: their overflows get the 3-term LDS screen
                    esc_bc = np.concatenate([self.cls_b[st[self.cls_b] != 0],
                                             self.cls_c[st[self.cls_c] != 0]])
            n_esc = len(esc_a) + len(esc_bc)
            if n_esc:
                self.cs_modified = True
                if len(esc_a):
                    self._screen_pass(esc_a, "stream" if self.stream_ok else "lds")
                if len(esc_bc):
                    self._screen_pass(esc_bc, "lds")
                # (the escalation ran on this stream, which may not be the launch stream)
                n_ovf = self._ovf.read(self._ovf_slot, torch.cuda.current_stream())
        fb = (np.empty(0, np.int64) if self.all_a
              else np.nonzero(~self.on_screen & (kk >= 1))[0])
        if n_ovf:
            fb = np.union1d(fb, np.nonzero(self.status.cpu().numpy())[0])
        if len(fb):
            self.cs_modified = True
            _fallback_exact(ds, self.Qx, fb, kk, self.out_d, self.out_i)
        if self.want_fin and (len(fb) or self.kmin < 1 or self.kmax > N):
            # queries not (correctly) finalized by refine: fallback ones, k == 0, and k > N
            # (the checksum then also covers the (+inf, -1) padding, as the CPU path does)
            rest = np.union1d(fb, np.nonzero((kk < 1) | (self.k_host > N))[0]).astype(np.int32)
            if len(rest):
                self.cs_modified = True
                ridx = _h2d(rest, dev)
                _lib.check(L.dmlp_finalize(_p(self.out_d), _p(self.out_i), self.ks,
                                           _p(self.k_dev), _p(ridx), len(rest), _p(ds.labels),
                                           ds.label_lo, ds.label_hi, _p(self.lab), _p(self.cs),
                                           _stream()), "finalize")
        return DeviceResult(self.out_d, self.out_i, self.lab, self.cs, self.k_host,
                            int(len(fb)), int(n_esc))


class _OvfCounters:
    """Per-device running counters of overflowed queries (refine.hip atomically adds one per
    handed-back query).  Each call owns a slot (round robin over 256, far more than the calls
    ever in flight); the host keeps the value it last read per slot, so nothing is zeroed."""

    SLOTS = 256

    def __init__(self, dev):
        torch = _torch()
        self.dev_t = torch.zeros(self.SLOTS, dtype=torch.int32, device=dev)
        self.host = torch.zeros(self.SLOTS, dtype=torch.int32).pin_memory()
        self.seen = [0] * self.SLOTS
        self.next = 0

    def slot(self):
        i = self.next
        self.next = (i + 1) % self.SLOTS
        return i

    def ptr(self, i):
        return self.dev_t.data_ptr() + 4 * i

    def read(self, i, stream):
        """Overflows counted in slot i since the last read (synchronizes `stream`)."""
        torch = _torch()
        with torch.cuda.stream(stream):
            self.host[i:i + 1].copy_(self.dev_t[i:i + 1], non_blocking=True)
        stream.synchronize()
        v = int(self.host[i])
        d, self.seen[i] = v - self.seen[i], v
        return d


_OVF = {}


def _ovf_counters(dev):
    key = str(dev)
    c = _OVF.get(key)
    if c is None:
        c = _OVF[key] = _OvfCounters(dev)
    return c


class _PinnedArena:
    """Grow-only page-locked staging for the small per-call host arrays (k, query index lists):
    a pageable source would make the runtime wait for the stream (i.e. for every kernel queued
    before the copy), and a fresh pinned allocation per copy can synchronize the device.
    Reset at the start of each top-level call, after the previous call's copies completed."""

    def __init__(self):
        self.buf = None
        self.off = 0
        self.events = []
        self.old = []

    def reset(self):
        for e in self.events:
            e.synchronize()
        self.events = []
        self.old = []
        self.off = 0

    def alloc(self, n: int):
        """n uninitialised page-locked bytes (torch uint8), valid until the next reset()."""
        torch = _torch()
        if self.buf is None or self.off + n > self.buf.numel():
            if self.buf is not None:
                self.old.append(self.buf)  # in-flight copies may still read it
            self.buf = torch.empty(max(4 << 20, 2 * (self.off + n)), dtype=torch.uint8).pin_memory()
            self.off = 0
        view = self.buf[self.off:self.off + n]
        self.off = (self.off + n + 255) & ~255
        return view

    def put(self, a: np.ndarray):
        torch = _torch()
        a = np.ascontiguousarray(a)
        view = self.alloc(a.nbytes)
        view.numpy()[:] = a.view(np.uint8).reshape(-1)
        return view.view(torch.from_numpy(a[:0]).dtype)

    def mark(self):
        torch = _torch()
        e = torch.cuda.Event()
        e.record()
        self.events.append(e)


_ARENA = _PinnedArena()


def _h2d(a: np.ndarray, dev):
    """Small host array -> device as a real async DMA from the pinned arena."""
    return _ARENA.put(a).to(dev, non_blocking=True)


_IDENTITY = {}


def _identity(n: int, dev):
    """Device arange(n) int32 (grow-only cache): the query index list of an all-queries pass."""
    torch = _torch()
    key = str(dev)
    t = _IDENTITY.get(key)
    if t is None or t.numel() < n:
        t = _IDENTITY[key] = torch.arange(max(n, 1 << 16), dtype=torch.int32, device=dev)
    return t[:n]


# host <-> device bytes issued by the pipelined path (bench.py's per-rank diagnostics)
_IO = {"h2d": 0, "d2h": 0}


def io_bytes(reset: bool = False):
    out = dict(_IO)
    if reset:
        _IO["h2d"] = _IO["d2h"] = 0
    return out


_SIDE_STREAMS = {}
_PIPE_DEBUG = os.environ.get("DMLP_PIPE_DEBUG") == "1"
_HT = []  # DMLP_PIPE_DEBUG: host-side (phase, perf_counter) stamps of the current call
_HT_PREV = [None]  # the previous call's "synced" stamp (the host gap between calls)


def _ht(name):
    if _PIPE_DEBUG:
        _HT.append((name, time.perf_counter()))

# DMLP_PIPE_EVENTS=1: GPU timestamps (hipEvents) at the phase boundaries of knn_gpu_pipelined,
# read after the call's sync — a step timeline without a profiler (no host syncs added).
# pipe_timeline() returns the last call's [(phase, ms since the call entered)].
_EVENTS = os.environ.get("DMLP_PIPE_EVENTS") == "1"
_MARKS = []
_LAST_TIMELINE = []
_PREV_END = [None]  # the previous call's last mark: the gap between calls


def set_pipe_events(on: bool):
    global _EVENTS
    _EVENTS = bool(on)
    _PREV_END[0] = None
    try:  # the native step's own marks (fast_step.hip)
        _lib.lib().dmlp_fast_step_events(1 if on else 0)
    except Exception:  # noqa: BLE001 (a library without the native step)
        pass


def _mark(name, stream=None):
    if not _EVENTS:
        return
    torch = _torch()
    e = torch.cuda.Event(enable_timing=True)
    e.record(stream if stream is not None else torch.cuda.current_stream())
    _MARKS.append((name, e))


def _close_marks():
    global _LAST_TIMELINE
    if not _EVENTS or not _MARKS:
        return
    _MARKS[-1][1].synchronize()
    t0 = _MARKS[0][1]
    out = []
    if _PREV_END[0] is not None:
        out.append(("prev_call_done", round(-_PREV_END[0].elapsed_time(t0), 4)))
    for name, e in _MARKS:
        e.synchronize()
        out.append((name, round(t0.elapsed_time(e), 4)))
    _LAST_TIMELINE = out
    _PREV_END[0] = _MARKS[-1][1]
    _MARKS.clear()


def pipe_timeline():
    return list(_LAST_TIMELINE)


def _side_stream(name):
    torch = _torch()
    key = (name, torch.cuda.current_device())
    st = _SIDE_STREAMS.get(key)
    if st is None:
        st = _SIDE_STREAMS[key] = torch.cuda.Stream()
    return st


def knn_gpu_pipelined(X_host, labels_host, label_range, Q_host, k_host, kstride=None,
                      chunks: int = 1, finalize: bool = True, exact: bool = False, gather=None,
                      mu_rows=None, X_full_host=None, report=None, k_range=None,
                      image_shard=None, _host_ops=True):
    """Host arrays in (page-locked for real overlap), device results out, with the fp64 rows
    copied behind the screen ("H2D overlapped with compute").

    chunks == 1 (default): the host renders the single-term screen's operands — the dataset's
    hi-only bf16 tile image + norms and the queries' bf16 fragments + norms (host_prep.cpp:
    15.7 MB instead of the 59 MB of fp64 rows for the bench shape).  The screen starts once they
    have landed; the fp64 dataset and query rows (and the labels) cross PCIe behind the screen,
    and only the exact re-rank waits for them.  chunks > 1: query chunks each screened once they
    land (measured slower on the bench shape: two half-size screens have a worse tail than one).

    gather(X_dev, lab_dev) -> (X, lab), if given, completes a dataset shard into the replica (the
    RCCL all-gather ingress); it is issued on the copy stream, so it too runs behind the screen.
    X_full_host: the whole dataset when X_host is a shard (the host renders the full screen
    image from it); mu_rows: the dataset's first rows (the centre is their mean).
    report: {"qid_base": b[, "dst": page-locked uint8 numpy view of >= 48 Q + 64 bytes]} renders
    the report lines right behind the re-rank, before the one host sync (and, with "dst", copies
    the 48-byte-per-line bound of it there too); on return report["valid"] says whether nothing
    rewrote the checksums afterwards (escalation / fallback), report["text"] = (device bytes,
    pinned int64 byte count) and report["copied"] whether dst already holds them.
    k_range: (a lower bound of the smallest k, an upper bound of the largest k), e.g. from a
    segment header, instead of scanning k_host (bounds only steer the dispatch).
    image_shard: (rank, world, allgather(out, chunk), allreduce_max(t)) — every rank renders
    only its 1/world of the dataset's screen image (host memory reads and CPU time per rank drop
    by world) and one all-gather over xGMI completes the image before the screen; the max norm
    is max-reduced (+inf from a rank whose rows are outside the screen's range: every rank then
    takes the device path's exact fallbacks together, no rank-dependent branch).
    Returns (DeviceDataset, dist, ids, label, checksum, n_fallback); the DeviceDataset's device
    arrays (operand images, fp64 rows) are scratch reused by the next pipelined call, the
    result tensors are the caller's."""
    torch = _torch()
    L = _lib.lib()
    dev = torch.device("cuda", torch.cuda.current_device())
    main = torch.cuda.current_stream()
    copy = _side_stream("h2d")
    t_enter = time.perf_counter()
    if _PIPE_DEBUG:
        _HT.clear()
        _HT.append(("enter", t_enter))
        if _HT_PREV[0] is not None:
            _HT.append(("since_prev_sync", t_enter - _HT_PREV[0] + t_enter))
    _ARENA.reset()
    copy.wait_stream(main)  # buffers recycled from the previous call
    _MARKS.clear()
    _mark("enter", copy)
    Q = len(Q_host)
    A = X_host.shape[1]
    KT = screen_kt(A)
    k_host = np.ascontiguousarray(k_host, np.int32)
    chunks = max(1, min(chunks, Q // 2048 if Q >= 4096 else 1))
    bounds = [Q * c // chunks for c in range(chunks + 1)]
    Xf = X_host if X_full_host is None else X_full_host
    N = len(Xf)
    Qh = np.ascontiguousarray(Q_host, np.float64)
    if Q and k_range is None:
        k_range = (int(k_host.min()), int(k_host.max()))
    # the host renders the single-term (x1) operands whenever x1 serves this A; queries with k
    # outside [1, 32] (3-term class, exact path) and escalations get device operands on need
    host_ops = (_host_ops and chunks == 1 and not exact and SCREEN_IMPL == "x1" and Q > 0 and N > 0
                and L.dmlp_screen_x1_qw(KT) > 0)
    # every k on the x1 class and one local replica: the screen(s) are queued natively right
    # behind the query operands and before the host packs the fp64 rows (_pipelined_parts),
    # in HOST_OPS_PARTS query parts
    split = (host_ops and gather is None and k_range[0] >= 1
             and k_range[1] <= min(SCREEN_KMAX_A, N))
    parts = max(1, HOST_OPS_PARTS) if split and Q >= HOST_OPS_PARTS * 8192 else 1
    dsops = prepped = mu_d = None
    if host_ops:
        src = np.ascontiguousarray((Xf if mu_rows is None else mu_rows)[:4096], np.float64)
        mu_h = np.empty(A, np.float64)
        L.dmlp_cpu_center(src.ctypes.data, len(src), A, mu_h.ctypes.data)
        mu_d = _h2d(mu_h, dev)
        n_tiles = (N + 63) // 64
        Xc = np.ascontiguousarray(Xf, np.float64)
        hb = [_ARENA.alloc(n) for n in (n_tiles * 64 * KT * 64, n_tiles * 64 * 4, 4, Q * KT * 64,
                                        Q * 4)]
        sh = image_shard if image_shard is not None and image_shard[1] > 1 else None
        if sh is not None:
            tpr = (n_tiles + sh[1] - 1) // sh[1]  # tiles per rank (the last ranks' tails pad)
            t0 = min(sh[0] * tpr, n_tiles)
            t1 = min(t0 + tpr, n_tiles)
        else:
            tpr, t0, t1 = n_tiles, 0, n_tiles
        # the operand images: device scratch reused across calls (internal, never returned)
        W = 64 * KT * 32
        xhi = _scratch("xhi", (n_tiles if sh is None else sh[1] * tpr) * W, torch.int16, dev)
        xin = _scratch("xin", (n_tiles if sh is None else sh[1] * tpr) * 64, torch.float32, dev)
        xhi_c, xin_c = ((xhi, xin) if sh is None else
                        (_scratch("xhi_c", tpr * W, torch.int16, dev),
                         _scratch("xin_c", tpr * 64, torch.float32, dev)))
        xnm = _scratch("xnm", 1, torch.int32, dev)
        qhi = _scratch("qhi", Q * KT * 32, torch.int16, dev)
        qn = _scratch("qn", Q, torch.float32, dev)
        t_ops = t_ops0 = time.perf_counter()
        if split:
            def render_data(bad):
                """The dataset image (+ the sharded image's collectives) on `copy`."""
                rc = L.dmlp_host_ops_h2d_tiles(Xc.ctypes.data, N, t0, t1, Qh.ctypes.data, 0, A,
                                               mu_h.ctypes.data, KT, *[b.data_ptr() for b in hb],
                                               _p(xhi_c), _p(xin_c), _p(xnm), _p(qhi), _p(qn),
                                               HOST_OPS_CHUNKS, copy.cuda_stream)
                if sh is not None:
                    # the image collectives, on every rank whatever its own verdict (the same
                    # sequence as the path below)
                    with torch.cuda.stream(copy):
                        sh[2](xhi.view(torch.int32), xhi_c.view(torch.int32))
                        sh[2](xin, xin_c)
                        sh[3](xnm)
                        bad.copy_((xnm >= 0x7f800000).to(torch.int32))
                    rc &= ~1  # the data verdict is the reduced one, on the device
                if rc & 4:
                    raise RuntimeError("dmlp_host_ops_h2d: hipMemcpyAsync failed")
                return rc

            r = _pipelined_parts(parts, X_host, labels_host, label_range, Qh, k_host, kstride,
                                 finalize, k_range, KT, mu_h, mu_d, hb, xhi, xin, xnm, qhi, qn,
                                 copy, main, render_data)
            if r is None:
                # data or a query outside the screen's range: the device path decides (no
                # collective on it; the pinned staging is reused only once its copies are done)
                copy.synchronize()
                return knn_gpu_pipelined(X_host, labels_host, label_range, Q_host, k_host,
                                         kstride, chunks, finalize, exact, gather, mu_rows,
                                         X_full_host, report, k_range, image_shard,
                                         _host_ops=False)
            ds, od, oi, ol, oc, calls = r
            t_ops = time.perf_counter() - t_ops
            _IO["h2d"] += (t1 - t0) * 64 * (KT * 64 + 4) + 4 + Q * (KT * 64 + 4)
            return _pipelined_tail(ds, od, oi, ol, oc, calls, report, Q, finalize, t_enter,
                                   t_ops0, t_ops, True)
        # host conversion of each slice overlaps the PCIe copy of the previous one
        rc = L.dmlp_host_ops_h2d_tiles(Xc.ctypes.data, N, t0, t1, Qh.ctypes.data, Q, A,
                                       mu_h.ctypes.data, KT, *[b.data_ptr() for b in hb],
                                       _p(xhi_c), _p(xin_c), _p(xnm), _p(qhi), _p(qn),
                                       HOST_OPS_CHUNKS, copy.cuda_stream)
        t_ops = time.perf_counter() - t_ops
        _IO["h2d"] += (t1 - t0) * 64 * (KT * 64 + 4) + 4 + Q * (KT * 64 + 4)
        if rc & 4:
            raise RuntimeError("dmlp_host_ops_h2d: hipMemcpyAsync failed")
        bad_d = None
        if sh is not None:
            # every rank runs these collectives whatever its own rc (no divergent branch)
            with torch.cuda.stream(copy):
                sh[2](xhi.view(torch.int32), xhi_c.view(torch.int32))  # (no 16-bit int in RCCL)
                sh[2](xin, xin_c)
                sh[3](xnm)
                # +inf (0x7f800000) from any rank: rows outside the screen's range somewhere
                bad_d = (xnm >= 0x7f800000).to(torch.int32)
            rc &= ~1  # the data verdict is the reduced one, on the device
        if rc == 0:
            dsops, prepped = (xhi, xin, xnm, bad_d), (qhi, qn)
        else:
            mu_d = None  # outside the screen's range: the device path decides
    _mark("operands_landed", copy)
    with torch.cuda.stream(copy):
        ev_p = torch.cuda.Event()
        ev_p.record(copy)
        X = torch.from_numpy(np.ascontiguousarray(X_host)).to(dev, non_blocking=True)
        lab = (torch.from_numpy(np.ascontiguousarray(labels_host, np.int32)).to(
            dev, non_blocking=True) if labels_host is not None else None)
        if dsops is not None and gather is not None:
            X, lab = gather(X, lab)  # RCCL all-gather behind the screen
        ev_x = torch.cuda.Event()
        ev_x.record(copy)
    _IO["h2d"] += X.numel() * 8 + (lab.numel() * 4 if lab is not None else 0) + Q * A * 8
    ev = []
    with torch.cuda.stream(copy):
        Qd = torch.empty((Q, A), dtype=torch.float64, device=dev)
        for c in range(chunks):
            a, b = bounds[c], bounds[c + 1]
            Qd[a:b].copy_(torch.from_numpy(Qh[a:b]), non_blocking=True)
            e = torch.cuda.Event()
            e.record(copy)
            ev.append(e)
    _mark("rows_landed", copy)
    for t in (X, Qd) + ((lab,) if lab is not None else ()) + (prepped or ()) + (dsops or ()):
        if t is not None:
            t.record_stream(main)
    ks = max(1, k_range[1] if Q else 1) if kstride is None else kstride
    if dsops is not None:
        # the screen operands are on their way; X / labels / Qd complete with ev[-1]
        if lab is not None and finalize:
            lo, hi = label_range
            lab_ds = lab
        else:
            lo, hi, lab_ds = 0, 1, None
        ds = DeviceDataset(X, lab_ds, lo, hi, KT, mu_d, dsops[0], dsops[1], dsops[2],
                           dsops[3] if dsops[3] is not None
                           else torch.zeros(1, dtype=torch.int32, device=dev), True, hl=1)
    else:
        main.wait_event(ev_x)
        if gather is not None:
            X, lab = gather(X, lab)
        ds = prepare_dataset(X, lab if finalize else None, label_range, mu=mu_d)
    fin = finalize and ds.labels is not None
    od = torch.empty((Q, ks), dtype=torch.float64, device=dev)
    oi = torch.empty((Q, ks), dtype=torch.int32, device=dev)
    ol = torch.empty(Q, dtype=torch.int32, device=dev) if fin else None
    oc = torch.empty(Q, dtype=torch.int64, device=dev) if fin else None
    calls = []
    for c in range(chunks):
        a, b = bounds[c], bounds[c + 1]
        out = (od[a:b], oi[a:b], ol[a:b] if fin else None, oc[a:b] if fin else None)
        if prepped is not None:
            main.wait_event(ev_p)  # screen operands landed; the fp64 rows may still be in flight
            call = _KnnCall(ds, Qd, k_host, finalize, exact, ks, out=out, prepped=prepped,
                            qx_event=ev[-1], k_range=k_range)
        else:
            main.wait_event(ev[c])
            call = _KnnCall(ds, Qd[a:b], k_host[a:b], finalize, exact, ks, out=out)
        calls.append(call.launch())
    return _pipelined_tail(ds, od, oi, ol, oc, calls, report, Q, finalize, t_enter,
                           t_ops0 if host_ops else t_enter, t_ops if host_ops else 0.0,
                           prepped is not None)


# the single-GPU call in one native function (fast_step.hip) when every k is on the single-term
# class; DMLP_FAST_STEP=0: always the Python pipeline (knn_gpu_pipelined)
FAST_STEP = os.environ.get("DMLP_FAST_STEP", "1") != "0"
FAST_STEP_CALLS = [0]  # calls the native step served (tests, diagnostics)


def fast_step(X_host, labels_host, label_range, Q_host, k_host, k_range, dst, qid_base=0):
    """One rank's whole call natively (dmlp_fast_step): host render + copies, single-term screen,
    fp64 rows behind it, exact re-rank, vote, checksum, report text into the page-locked `dst`,
    one host sync.  Returns (label, checksum device tensors, report byte count), or None when
    the call is not this path's (k outside [1, 32], data outside the fp16 screen's range, a
    query that overflowed its single-term candidates): the caller then runs the general
    pipeline (knn_gpu_pipelined), whose per-query dispatch and escalation handle it."""
    torch = _torch()
    L = _lib.lib()
    Q, A = Q_host.shape
    N = len(X_host)
    if not FAST_STEP or Q == 0 or N == 0:
        return None
    dev = torch.device("cuda", torch.cuda.current_device())
    lab = torch.empty(Q, dtype=torch.int32, device=dev)
    cs = torch.empty(Q, dtype=torch.int64, device=dev)
    n = np.zeros(1, np.int64)
    rc = L.dmlp_fast_step(X_host.ctypes.data, labels_host.ctypes.data, N, Q_host.ctypes.data,
                          k_host.ctypes.data, Q, A, int(k_range[0]), int(k_range[1]),
                          int(label_range[0]), int(label_range[1]), qid_base, HOST_OPS_CHUNKS,
                          dst.ctypes.data, len(dst), n.ctypes.data, _p(lab), _p(cs), _stream())
    if rc in (1, 2):
        return None
    _lib.check(rc, "fast_step")
    FAST_STEP_CALLS[0] += 1
    if _EVENTS:
        import ctypes
        global _LAST_TIMELINE
        ms = (ctypes.c_double * 16)()
        names = (ctypes.c_char_p * 16)()
        m = L.dmlp_fast_step_timeline(ms, names, 16)
        _LAST_TIMELINE = [(names[i].decode(), round(ms[i], 4)) for i in range(m)]
    _IO["h2d"] += ((N + 63) // 64 * 64 * (screen_kt(A) * 64 + 4) + Q * (screen_kt(A) * 64 + 4)
                   + (N + Q) * A * 4 + N * 4)
    _IO["d2h"] += L.dmlp_format_bound(Q)
    return lab, cs, int(n[0])


def _pipelined_parts(parts, X_host, labels_host, label_range, Qh, k_host, kstride, finalize,
                     k_range, KT, mu_h, mu_d, hb, xhi, xin, xnm, qhi, qn, copy, main,
                     render_data):
    """knn_gpu_pipelined's front when every k is on the single-term class: the calls of the
    query parts are set up first (their own streams), then render_data(bad) queues the dataset
    image on `copy`, dmlp_host_ops_x1_parts renders each query part and queues its screen behind
    its copy, and only then does the host pack the fp64 rows (lossless int32 when it can) — the
    screens run meanwhile; every part's refine waits for the rows.  None when the data or a query
    is outside the screen's range (the streams are drained).  One part is the default: 2 and 4
    parts measured slower (profiles/r4j_query_parts_ab.txt)."""
    import ctypes
    torch = _torch()
    L = _lib.lib()
    dev = qhi.device
    Q, A = Qh.shape
    N = len(X_host)
    W = KT * 32
    with torch.cuda.stream(copy):
        bad = torch.zeros(1, dtype=torch.int32, device=dev)  # (sharded: the reduced verdict)
    # the dataset image first: its render and copy start before any of the Python set-up below
    # (~0.1 ms), which then runs while the image crosses PCIe
    _ht("render_data")
    if render_data(bad):
        copy.synchronize()
        return None
    _mark("data_landed", copy)
    _ht("setup")
    # the fp64 rows: device scratch reused across calls (internal, never returned)
    X = _scratch("X", N * A, torch.float64, dev).view(N, A)
    lab = _scratch("lab", N, torch.int32, dev) if labels_host is not None else None
    Qd = _scratch("Qd", Q * A, torch.float64, dev).view(Q, A)
    if lab is not None and finalize:
        lo, hi = label_range
        lab_ds = lab
    else:
        lo, hi, lab_ds = 0, 1, None
    ds = DeviceDataset(X, lab_ds, lo, hi, KT, mu_d, xhi, xin, xnm, bad, True, hl=1)
    fin = finalize and ds.labels is not None
    ks = max(1, k_range[1]) if kstride is None else kstride
    od = torch.empty((Q, ks), dtype=torch.float64, device=dev)
    oi = torch.empty((Q, ks), dtype=torch.int32, device=dev)
    ol = torch.empty(Q, dtype=torch.int32, device=dev) if fin else None
    oc = torch.empty(Q, dtype=torch.int64, device=dev) if fin else None
    pss = [_side_stream(f"part{p}") for p in range(parts)]
    bounds = [Q * p // parts for p in range(parts + 1)]
    shared = [t for t in (X, lab, Qd, bad, xhi, xin, xnm, qhi, qn, mu_d, od, oi, ol, oc)
              if t is not None]
    # (created on main before the part streams wait for it)
    qidx = _identity(max(bounds[p + 1] - bounds[p] for p in range(parts)), dev)
    calls, bufs = [], []
    for p, ps in enumerate(pss):
        a, b = bounds[p], bounds[p + 1]
        ps.wait_stream(main)
        ps.wait_stream(copy)
        for t in shared:
            t.record_stream(ps)
        with torch.cuda.stream(ps):
            out = (od[a:b], oi[a:b], ol[a:b] if fin else None, oc[a:b] if fin else None)
            call = _KnnCall(ds, Qd[a:b], k_host[a:b], finalize, False, ks,
                            gpu_share=1.0 / parts, out=out, prepped=(qhi[a * W:b * W], qn[a:b]),
                            k_range=k_range)
            bufs.append(call.x1_buffers(p))  # one scratch slot per query part
        calls.append(call)
    S = bufs[0][3]
    if any(bf[3] != S for bf in bufs):
        raise RuntimeError("query parts disagree on the slice count")
    arr = lambda xs: (ctypes.c_void_p * parts)(*xs)
    _ht("query_render")
    rc = L.dmlp_host_ops_x1_parts(
        Qh.ctypes.data, Q, A, mu_h.ctypes.data, KT, hb[3].data_ptr(), hb[4].data_ptr(), _p(qhi),
        _p(qn), parts, copy.cuda_stream, arr([ps.cuda_stream for ps in pss]), _p(xhi), _p(xin),
        ds.n_tiles, N, _p(qidx), arr([c.k_dev.data_ptr() for c in calls]), k_range[1], _p(xnm),
        _p(bad), S, arr([bf[0].data_ptr() for bf in bufs]), arr([bf[1].data_ptr() for bf in bufs]),
        arr([bf[2].data_ptr() for bf in bufs]), HOST_OPS_CHUNKS)
    if rc & 4:
        raise RuntimeError("dmlp_host_ops_x1_parts: copy or launch failed")
    if rc:
        for ps in pss:
            ps.synchronize()
        copy.synchronize()
        return None
    _mark("operands_landed", copy)
    _ht("rows")
    with torch.cuda.stream(copy):
        if lab is not None:
            lab.copy_(torch.from_numpy(np.ascontiguousarray(labels_host, np.int32)),
                      non_blocking=True)
        _issue_rows(((np.ascontiguousarray(X_host, np.float64), X), (Qh, Qd)), copy)
        ev_rows = torch.cuda.Event()
        ev_rows.record(copy)
    _mark("rows_landed", copy)
    _IO["h2d"] += lab.numel() * 4 if lab is not None else 0
    for call, ps in zip(calls, pss):
        call.qx_event = ev_rows
        with torch.cuda.stream(ps):
            call.launch()
        main.wait_stream(ps)
        # the call's one host sync (finish: the overflow count) goes on main, behind the report
        # kernels and the report D2H that _pipelined_tail queues there: the call returns with
        # its byte count and text complete (a sync on the part stream alone left them racing
        # the caller's reads)
        call.stream = main
    return ds, od, oi, ol, oc, calls


def _issue_rows(pairs, copy):
    """Queue the H2D of fp64 host rows into device tensors on `copy`, each (host, device) pair
    as lossless int32 when every value is a 6-decimal number (x == fl(m / 1e6), checked bit for
    bit on the host: half the PCIe bytes, the device divides back — prep.hip
    dmlp_rows_from_i32), else as fp64.  The host packs pair i + 1 while pair i crosses PCIe.
    DMLP_ROWS_I32=0 always ships fp64."""
    torch = _torch()
    L = _lib.lib()
    for host, dev_t in pairs:
        n = host.size
        if n == 0:
            continue
        if ROWS_I32:
            hb = _ARENA.alloc(n * 4)
            if L.dmlp_cpu_rows_i32(host.ctypes.data, n, hb.data_ptr()) == 0:
                db = torch.empty(n, dtype=torch.int32, device=dev_t.device)
                db.copy_(hb.view(torch.int32), non_blocking=True)
                _lib.check(L.dmlp_rows_from_i32(_p(db), n, _p(dev_t), copy.cuda_stream),
                           "rows_from_i32")
                _IO["h2d"] += n * 4
                continue
        dev_t.copy_(torch.from_numpy(host).view(dev_t.shape), non_blocking=True)
        _IO["h2d"] += n * 8


def _pipelined_tail(ds, od, oi, ol, oc, calls, report, Q, finalize, t_enter, t_ops0, t_ops,
                    host_ops):
    """Report render + D2H behind the re-rank, then each call's finish (the one host sync)."""
    L = _lib.lib()
    fin = finalize and ds.labels is not None
    spec = None
    _mark("knn_queued")
    if report is not None and fin and Q > 0:
        spec = format_report_dev_async(oc, report.get("qid_base", 0))
        _mark("format_done")
        dst = report.get("dst")
        if dst is not None and len(dst) >= L.dmlp_format_bound(Q):
            _lib.check(L.dmlp_d2h_async(dst.ctypes.data, _p(spec[0]), L.dmlp_format_bound(Q),
                                        _stream()), "d2h report")
            _IO["d2h"] += L.dmlp_format_bound(Q)
            report["copied"] = True
            _mark("report_d2h_done")
        else:
            report["copied"] = False
    t_launched = time.perf_counter()
    _ht("finish")
    n_fb = sum(call.finish().n_fallback for call in calls)
    _ht("synced")
    _HT_PREV[0] = time.perf_counter()
    _close_marks()
    if report is not None:
        report["valid"] = spec is not None and not any(c.cs_modified for c in calls)
        report["text"] = spec
    _ARENA.mark()
    if _PIPE_DEBUG:
        import sys
        t0 = _HT[0][1] if _HT else t_enter
        print("[dmlp-pipe] host stamps (ms): " + " ".join(f"{n}={1e3 * (t - t0):.3f}"
                                                           for n, t in _HT), file=sys.stderr)
        print(f"[dmlp-pipe] host launch {1e3 * (t_launched - t_enter):.3f} ms (before host ops "
              f"{1e3 * (t_ops0 - t_enter):.3f} ms), finish "
              f"{1e3 * (time.perf_counter() - t_launched):.3f} ms, host ops "
              f"{host_ops} ({1e3 * t_ops:.3f} ms), calls {len(calls)}", file=sys.stderr)
    return ds, od, oi, ol, oc, n_fb


_ENV_APPLIED = [False]


def _apply_env_switches(L):
    """DMLP_STREAM_GROUPS=0 switches the streaming screen to per-point appends (A/B only)."""
    if not _ENV_APPLIED[0]:
        if os.environ.get("DMLP_STREAM_GROUPS", "1") == "0":
            L.dmlp_set_stream_groups(0)
        if os.environ.get("DMLP_X1_CT"):
            L.dmlp_set_x1_ct(int(os.environ["DMLP_X1_CT"]))
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
    kdev = _h2d(np.ascontiguousarray(kk, np.int32), dev)
    # the fused streaming kernel (exact.hip: no distance rows, no workspace) for k <= 64, and for
    # k <= 256 once N is large enough that the rows' HBM traffic dominates
    mode = os.environ.get("DMLP_EXACT_FUSED", "1")  # 0: never, 2: for every k it supports
    kf = 0 if mode == "0" else (L.dmlp_exact_topk_kmax() if mode == "2"
                                else L.dmlp_exact_topk_kmax_for(N))
    fused = fb[kk[fb] <= kf]
    if len(fused):
        qidx = _h2d(fused.astype(np.int32), dev)
        _lib.check(L.dmlp_exact_topk(_p(ds.X), N, A, _p(Qx), _p(qidx), _p(kdev), len(fused),
                                     int(kk[fused].max()), _p(out_d), _p(out_i), out_d.shape[1],
                                     s), "exact_topk")
    fb = fb[kk[fb] > kf]
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
            qidx = _h2d(sub.astype(np.int32), dev)
            _lib.check(fn(_p(ds.X), N, A, _p(Qx), _p(qidx), _p(kdev), len(sub), _p(ws), ws_bytes,
                          _p(out_d), _p(out_i), out_d.shape[1], s),
                       "fallback_select" if sel else "fallback_topk")


def knn_gpu_streamed(X_host, labels_host, label_range, Qx, k_host, chunk_rows: int,
                     kstride=None, exact: bool = False):
    """Out-of-core exact k-NN ("stream from host memory beyond HBM"): the dataset
    stays in (page-locked) host memory and crosses PCIe in chunks of chunk_rows rows, double
    buffered on a copy stream so chunk c+1 is in flight while chunk c is screened; each chunk's
    top-k lists (global ids) are merged into the running lists by the K-way merge kernel, and
    the vote / checksum run once at the end.  Device memory: 2 chunks + queries + labels.
    Returns (dist, ids, label, checksum) on the current device."""
    torch = _torch()
    dev = Qx.device
    main = torch.cuda.current_stream()
    copy = _side_stream("h2d")
    N, A = X_host.shape
    Q = Qx.shape[0]
    k_host = np.ascontiguousarray(k_host, np.int32)
    ks = max(1, int(k_host.max()) if Q else 1) if kstride is None else kstride
    chunk_rows = max(1, min(int(chunk_rows), N))
    nchunks = (N + chunk_rows - 1) // chunk_rows
    bufs = [torch.empty((chunk_rows, A), dtype=torch.float64, device=dev) for _ in range(2)]
    ready = [torch.cuda.Event() for _ in range(2)]
    freed = [None, None]
    labels = None
    copy.wait_stream(main)
    with torch.cuda.stream(copy):
        if labels_host is not None:
            labels = torch.from_numpy(np.ascontiguousarray(labels_host)).to(dev, non_blocking=True)
    def issue(c):
        b = c % 2
        a0, a1 = c * chunk_rows, min(N, (c + 1) * chunk_rows)
        if freed[b] is not None:
            copy.wait_event(freed[b])  # chunk c-2's screen is done with this buffer
        with torch.cuda.stream(copy):
            bufs[b][: a1 - a0].copy_(torch.from_numpy(np.ascontiguousarray(X_host[a0:a1])),
                                     non_blocking=True)
            ready[b].record(copy)
    issue(0)
    dr = ir = None
    kd = torch.from_numpy(k_host).to(dev)
    for c in range(nchunks):
        b = c % 2
        a0, a1 = c * chunk_rows, min(N, (c + 1) * chunk_rows)
        if c + 1 < nchunks:
            issue(c + 1)
        main.wait_event(ready[b])
        ds = prepare_dataset(bufs[b][: a1 - a0])
        r = knn_gpu(ds, Qx, k_host, finalize=False, exact=exact, kstride=ks)
        d, i = r.dist, torch.where(r.ids >= 0, r.ids + a0, r.ids)
        if dr is None:
            dr, ir = d, i
        else:
            dr, ir = merge_gpu(torch.stack([dr, d]), torch.stack([ir, i]), kd, ks)
        freed[b] = main.record_event()
    main.wait_stream(copy)
    lab = cs = None
    if labels is not None:
        lab, cs = finalize_gpu(labels, label_range, dr, ir, kd)
    return dr, ir, lab, cs


def merge_gpu(lists_d, lists_i, k_dev, kout: int):
    """lists_*: torch [L, Q, kin] sorted lists on one GPU -> merged [Q, kout] (K4)."""
    torch = _torch()
    Ld = lists_d.contiguous()
    Li = lists_i.contiguous()
    Lc, Q, kin = Ld.shape
    if Lc <= 8:  # the register merge writes every slot, padding included
        out_d = torch.empty((Q, kout), dtype=torch.float64, device=Ld.device)
        out_i = torch.empty((Q, kout), dtype=torch.int32, device=Ld.device)
    else:
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


def format_report_dev_async(cs, qid_base: int = 0):
    """format_report_dev without the host sync: (device uint8 text, pinned int64 [1] byte count
    valid once the current stream has reached this point)."""
    torch = _torch()
    L = _lib.lib()
    cs = cs.contiguous()
    nq = cs.numel()
    off = torch.empty(L.dmlp_format_scratch(nq), dtype=torch.int64, device=cs.device)
    out = torch.empty(L.dmlp_format_bound(nq), dtype=torch.uint8, device=cs.device)
    _lib.check(L.dmlp_format_report(_p(cs), nq, qid_base, _p(off), _p(out), _stream()), "format")
    n_h = _ARENA.alloc(8).view(torch.int64)
    n_h.copy_(off[nq:nq + 1], non_blocking=True)
    return out, n_h


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