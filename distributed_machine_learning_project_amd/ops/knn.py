"""Local (single-device) exact k-NN: the compute backend every parallel strategy calls.

GPU: libdmlp's ONE native pipeline (csrc/pipeline.hip), which the standalone knn_engine and the
engine.h drop-in run as well — no part of a call is orchestrated from Python:
  knn_gpu  (dmlp_knn_local)  rows already on the device (shards, ring shards, out-of-core chunks):
           per-query classes — single-term MFMA screen (k <= 64), 3-term LDS screen (k <= 256),
           exact fp64 (k > 256, A > 256) — a device-rendered bf16 image, exact re-rank (reference
           order, no FMA), per-query escalation of overflowed screens, fused vote + FNV checksum
  step     (dmlp_step)       one rank's whole Engine::KNN call from host rows: the host renders
           the screen's fp16 operands while the GPU screens (early start), the fp64 rows cross
           PCIe behind the screen as lossless int32, exact re-rank, vote, checksum, the report
           text rendered on the GPU into page-locked host memory, one host sync
CPU: libdmlp's threaded brute force (or the KD-tree of bench.debug).

Exactness contract (common.cpp:57-79, engine.cpp:12-18): distances are the
reference's left-to-right fp64 sums without FMA; the MFMA screens only filter candidates, with a
rigorous error bound, so results are bit-identical to the fp64 oracle.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

from .. import _lib

SCREEN_KMAX_A = 64      # single-term one-pass screen class
SCREEN_KMAX_B = 128     # 3-term cap-256 class
SCREEN_KMAX_C = 256     # 3-term cap-512 class: larger k take the exact path
SCREEN_MAX_KT = 8       # A <= 256 on the screens


def screen_kt(A: int) -> int:
    """32-attribute fragments per row of the screen images (dmlp.h dmlp_screen_kt): A <= 256
    rounds up to 1, 2, 4 or 8, the single-term screen's variants."""
    kt = max(1, (A + 31) // 32)
    return kt if kt > 8 else 1 << (kt - 1).bit_length()


def eps_rel(A: int) -> float:
    """Relative error bound of the 3-term bf16 screen (pipeline.hip passes the same value)."""
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
    """The current stream's raw handle, without building a torch Stream object."""
    torch = _torch()
    if not _RAW_STREAM:
        _RAW_STREAM.append(getattr(torch._C, "_cuda_getCurrentRawStream", None))
    f = _RAW_STREAM[0]
    if f is not None:
        return f(torch.cuda.current_device())
    return torch.cuda.current_stream().cuda_stream


def _p(t):
    if t is None:
        return None
    if not t.is_contiguous():
        raise ValueError("native kernels need contiguous tensors")
    return t.data_ptr()


def _np_ptr(a):
    return None if a is None else a.ctypes.data


# ---------------------------------------------------------------- pipeline switches + stats
@contextlib.contextmanager
def pipeline_options(**kw):
    """Tuning / A-B switches of the native pipeline for the duration of a block (pipeline.hip
    Tuning): num_cus (CUs the slice choice fills), screen (first screen of the k <= 32 class on
    the device image: 0 single-term, 1 3-term streaming, 2 3-term LDS; != 0 also turns the host
    operands off), x1k (two-pass single-term screen for k in (32, 256]), host_ops."""
    L = _lib.lib()
    names = {"screen": {"x1": 0, "stream": 1, "lds": 2}}
    old = {}
    try:
        for key, v in kw.items():
            v = names.get(key, {}).get(v, v)
            prev = L.dmlp_pipeline_set(key.encode(), int(v))
            if prev < 0:
                raise KeyError(key)
            old[key] = prev
        yield
    finally:
        for key, v in old.items():
            L.dmlp_pipeline_set(key.encode(), v)


def pipeline_stats():
    """What the last native call did: {"n_exact", "n_escalated", "path", "early", "n_exact_f64",
    "n_exact_f64_redo", "device_render", "report_direct"} (exact-path queries on the fp64 MFMA
    screen, and those of them that overflowed to the fused VALU kernel; whether the GPU rendered
    the screen operands; whether the report text went straight into the caller's page-locked
    buffer)."""
    out = (C.c_int64 * 8)()
    _lib.lib().dmlp_pipeline_stats(out)
    return {"n_exact": out[0], "n_escalated": out[1], "path": out[2], "early": out[3],
            "n_exact_f64": out[4], "n_exact_f64_redo": out[5], "device_render": out[6],
            "report_direct": out[7]}


# ---------------------------------------------------------------- rows on the device
@dataclass
class DeviceDataset:
    """A dataset resident on one GPU (fp64 rows + labels); the native pipeline renders its
    screen image inside each call (timed, like the reference's pack/scatter)."""
    X: "object"            # torch f64 [N, A] (cuda)
    labels: "object"       # torch i32 [N] or None
    label_lo: int
    label_hi: int

    @property
    def N(self):
        return self.X.shape[0]

    @property
    def A(self):
        return self.X.shape[1]

    @property
    def KT(self):
        return screen_kt(self.A)


def prepare_dataset(X, labels=None, label_range=None) -> DeviceDataset:
    torch = _torch()
    X = X.contiguous()
    assert X.is_cuda and X.dtype == torch.float64 and X.dim() == 2
    N = X.shape[0]
    if labels is not None:
        labels = labels.to(device=X.device, dtype=torch.int32).contiguous()
        if label_range is None:
            lo = int(labels.min().item()) if N else 0
            hi = int(labels.max().item()) + 1 if N else 1
        else:
            lo, hi = label_range
    else:
        lo, hi = 0, 1
    return DeviceDataset(X, labels, lo, hi)


@dataclass
class DeviceResult:
    dist: "object"     # torch f64 [Q, kstride]
    ids: "object"      # torch i32 [Q, kstride]
    label: "object"    # torch i32 [Q] or None
    checksum: "object"  # torch i64 [Q] (uint64 bits) or None
    k: np.ndarray
    n_fallback: int = 0    # queries answered by the exact fp64 path
    n_escalated: int = 0   # single-term screen overflows re-screened with a 3-term screen


def knn_gpu(ds: DeviceDataset, Qx, k_host: np.ndarray, finalize: bool = True,
            exact: bool = False, kstride: int | None = None) -> DeviceResult:
    """Exact top-k of every query row of Qx (torch f64 cuda [Q, A]) against ds
    (dmlp_knn_local).  k_host: numpy int32 [Q]; returns once the results are complete."""
    torch = _torch()
    Qx = Qx.contiguous()
    Q = Qx.shape[0]
    k_host = np.ascontiguousarray(k_host, np.int32)
    ks = max(1, int(k_host.max()) if Q else 1) if kstride is None else kstride
    dev = Qx.device
    od = torch.empty((Q, ks), dtype=torch.float64, device=dev)
    oi = torch.empty((Q, ks), dtype=torch.int32, device=dev)
    fin = finalize and ds.labels is not None
    lab = torch.empty(Q, dtype=torch.int32, device=dev) if fin else None
    cs = torch.empty(Q, dtype=torch.int64, device=dev) if fin else None
    _lib.check(_lib.lib().dmlp_knn_local(
        _p(ds.X), ds.N, ds.A, _p(Qx), Q, k_host.ctypes.data, ks, _p(od), _p(oi),
        _p(ds.labels) if fin else None, ds.label_lo, ds.label_hi, _p(lab), _p(cs),
        1 if exact else 0, _stream()), "knn_local")
    st = pipeline_stats()
    return DeviceResult(od, oi, lab, cs, k_host, int(st["n_exact"]), int(st["n_escalated"]))


# ---------------------------------------------------------------- one rank's call from host rows
class StepArgs(C.Structure):
    """dmlp.h dmlp_step_args."""
    _fields_ = [("X", C.c_void_p), ("Xr", C.c_void_p), ("N", C.c_int64), ("A", C.c_int),
                ("labels", C.c_void_p), ("label_lo", C.c_int), ("label_hi", C.c_int),
                ("Qx", C.c_void_p), ("Qr", C.c_void_p), ("k", C.c_void_p), ("Q", C.c_int64),
                ("kmin", C.c_int), ("kmax", C.c_int), ("qid_base", C.c_int64),
                ("exact", C.c_int), ("out_lab", C.c_void_p), ("out_cs", C.c_void_p),
                ("out_d", C.c_void_p), ("out_i", C.c_void_p), ("kstride", C.c_int),
                ("report_mode", C.c_int), ("report_dst", C.c_void_p), ("report_cap", C.c_int64),
                ("stream", C.c_void_p), ("plane", C.c_void_p), ("report_len", C.c_int64),
                ("path", C.c_int),
                ("early", C.c_int), ("n_escalated", C.c_int), ("early_waits", C.c_int),
                ("early_grows", C.c_int), ("early_timeouts", C.c_int),
                ("host_ms", C.c_float), ("X32d", C.c_void_p)]


class Plane(C.Structure):
    """dmlp.h dmlp_plane: the node render plane (csrc/plane.cpp)."""
    _fields_ = [("base", C.c_void_p), ("bytes", C.c_int64), ("rank", C.c_int),
                ("renderers", C.c_int), ("with_f64", C.c_int), ("pad_", C.c_int),
                ("gen", C.c_int64), ("wait_s", C.c_double)]


@dataclass
class StepResult:
    label: "object"        # torch i32 [Q] (device)
    checksum: "object"     # torch i64 [Q] (device, uint64 bits)
    dist: "object"         # torch f64 [Q, kstride] or None (lists=False)
    ids: "object"
    report_len: int        # report bytes (in dst, or on the device for step_emit)
    path: int              # 0 host-rendered screen operands, 2 device image
    early: int             # the screen started before the dataset image landed
    n_escalated: int
    n_fallback: int
    early_waits: int = 0
    early_grows: int = 0
    early_timeouts: int = 0


# calls the native step served and its early-start counters (bench.py reports them for the timed
# region; tests check that the early start ran)
STEP_STATS = {"calls": 0, "early": 0, "early_waits": 0, "early_grows": 0, "early_timeouts": 0,
              "escalated": 0, "device_path": 0, "host_ms": 0.0}
_IO = {"h2d": 0, "d2h": 0}  # host <-> device bytes the steps issued (bench.py diagnostics)


def step_stats(reset: bool = False):
    out = dict(STEP_STATS)
    if reset:
        for key in STEP_STATS:
            STEP_STATS[key] = 0
    return out


def step(X_host, labels_host, label_range, Q_host, k_host, *, k_range=None, qid_base=0,
         exact=False, report=None, lists=False, kstride=None, plane=None,
         x32=None) -> StepResult:
    """One rank's whole Engine::KNN call from host arrays (dmlp_step): X_host [N, A] /
    Q_host [Q, A] fp64, labels_host [N] int32 (page-locked or registered memory for real
    overlap; a node-shared segment is), k_host [Q] int32.
      report: None — no text; a page-locked uint8 numpy array of >= dmlp_format_bound(Q) bytes —
              the "Query <id> checksum: <u64>" lines land there (ids from qid_base); "device" —
              kept on the GPU for step_emit (the multi-rank egress).
      lists:  also return the sorted (dist, id) lists [Q, kstride] (the DEBUG listing).
      k_range: (a lower bound of min k, an upper bound of max k) when known, else scanned.
      plane:  a Plane (node render plane): the dataset's image and rows are rendered once per
              node, slice by slice, by the plane's renderers into a node-shared segment.
      x32:    the dataset's rows already on this GPU as lossless int32 [N * A] (a torch tensor:
              the xGMI replica, parallel/strategies.py): no dataset rows cross PCIe.
    Returns once everything is complete (one host sync in the common case)."""
    torch = _torch()
    L = _lib.lib()
    X_host = np.ascontiguousarray(X_host, np.float64)
    Q_host = np.ascontiguousarray(Q_host, np.float64)
    k_host = np.ascontiguousarray(k_host, np.int32)
    labels_host = None if labels_host is None else np.ascontiguousarray(labels_host, np.int32)
    N, A = X_host.shape
    Q = Q_host.shape[0]
    if Q and k_range is None and lists and not kstride:
        k_range = _lib.i32_range(k_host)  # (the lists' stride)
    if k_range is None:  # the native step scans k on its render pool
        kmin, kmax = (1, 0) if Q else (1, 1)
    else:
        kmin, kmax = (int(k_range[0]), int(k_range[1])) if Q else (1, 1)
    ks = kstride or (max(1, kmax) if kmax >= kmin else 0)
    dev = torch.device("cuda", torch.cuda.current_device())
    lab = torch.empty(max(Q, 1), dtype=torch.int32, device=dev)[:Q]
    cs = torch.empty(max(Q, 1), dtype=torch.int64, device=dev)[:Q]
    od = oi = None
    if lists:
        od = torch.empty((Q, ks), dtype=torch.float64, device=dev)
        oi = torch.empty((Q, ks), dtype=torch.int32, device=dev)
    a = StepArgs()
    a.X, a.N, a.A = _np_ptr(X_host), N, A
    a.labels = _np_ptr(labels_host)
    # (label_range None: the native step scans the labels on its render pool)
    a.label_lo, a.label_hi = (int(label_range[0]), int(label_range[1])) if label_range else (0, 0)
    a.Qx, a.k, a.Q = _np_ptr(Q_host), _np_ptr(k_host), Q
    a.kmin, a.kmax = kmin, kmax
    a.qid_base = int(qid_base)
    a.exact = 1 if exact else 0
    a.out_lab, a.out_cs = _p(lab), _p(cs)
    a.out_d, a.out_i = _p(od), _p(oi)
    a.kstride = ks
    if report is None or labels_host is None:
        a.report_mode = 0
    elif isinstance(report, str):
        if report != "device":
            raise ValueError(report)
        a.report_mode = 2
    else:
        a.report_mode = 1
        a.report_dst, a.report_cap = report.ctypes.data, report.nbytes
    a.stream = _stream()
    a.plane = C.cast(C.pointer(plane), C.c_void_p) if plane is not None else None
    a.X32d = x32.data_ptr() if x32 is not None else None
    _lib.check(L.dmlp_step(C.byref(a)), "dmlp_step")
    st = pipeline_stats()
    STEP_STATS["calls"] += 1
    STEP_STATS["early"] += a.early
    STEP_STATS["early_waits"] += a.early_waits
    STEP_STATS["early_grows"] += a.early_grows
    STEP_STATS["early_timeouts"] += a.early_timeouts
    STEP_STATS["host_ms"] += a.host_ms
    STEP_STATS["escalated"] += a.n_escalated
    STEP_STATS["device_path"] += 1 if a.path == 2 else 0
    kt = screen_kt(A)
    _IO["h2d"] += ((N + 63) // 64 * 64 * (kt * 64 + 4) + Q * (kt * 64 + 4) if a.path == 0 else 0)
    _IO["h2d"] += (Q if x32 is not None else N + Q) * A * 4 + N * 4  # (lossless int32 rows)
    if a.report_mode == 1:  # (written straight across PCIe: the text; else the staged bound)
        _IO["d2h"] += int(a.report_len) if st["report_direct"] else L.dmlp_format_bound(Q)
    if _EVENTS[0]:
        _read_timeline()
    return StepResult(lab, cs, od, oi, int(a.report_len), a.path, a.early, a.n_escalated,
                      int(st["n_exact"]), a.early_waits, a.early_grows, a.early_timeouts)


def step_emit(dst, nbytes: int):
    """The last step's report bytes (report="device") -> dst (page-locked / registered uint8
    numpy view of >= nbytes), synchronously."""
    if nbytes:
        _lib.check(_lib.lib().dmlp_step_emit(dst.ctypes.data, int(nbytes), _stream()), "step_emit")
        _IO["d2h"] += int(nbytes)


def knn_gpu_pipelined(X_host, labels_host, label_range, Q_host, k_host, kstride=None,
                      finalize=True, exact=False, k_range=None):
    """step() with the sorted lists out (the DEBUG listing, tests): returns (info, dist, ids,
    label, checksum, n_fallback); info.hl is 1 when the host rendered the screen operands, 2 for
    the device image path."""
    r = step(X_host, labels_host if finalize else None, label_range, Q_host, k_host,
             k_range=k_range, exact=exact, lists=True, kstride=kstride)

    @dataclass
    class _Info:
        hl: int
        early: int
        n_escalated: int
    return (_Info(1 if r.path == 0 else 2, r.early, r.n_escalated), r.dist, r.ids,
            r.label if finalize else None, r.checksum if finalize else None, r.n_fallback)


def io_bytes(reset: bool = False):
    out = dict(_IO)
    if reset:
        _IO["h2d"] = _IO["d2h"] = 0
    return out


# ---------------------------------------------------------------- step timeline (hipEvents)
_EVENTS = [os.environ.get("DMLP_PIPE_EVENTS") == "1"]
_LAST_TIMELINE = []


def set_pipe_events(on: bool):
    _EVENTS[0] = bool(on)
    _lib.lib().dmlp_step_events(1 if on else 0)


def _read_timeline():
    global _LAST_TIMELINE
    ms = (C.c_double * 16)()
    names = (C.c_char_p * 16)()
    m = _lib.lib().dmlp_step_timeline(ms, names, 16)
    _LAST_TIMELINE = [(names[i].decode(), round(ms[i], 4)) for i in range(m)]


def pipe_timeline():
    return list(_LAST_TIMELINE)


# ---------------------------------------------------------------- out-of-core, merge, finalize
def _side_stream(name, _cache={}):
    torch = _torch()
    key = (name, torch.cuda.current_device())
    st = _cache.get(key)
    if st is None:
        st = _cache[key] = torch.cuda.Stream()
    return st


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


# ---------------------------------------------------------------- report text on the GPU
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
