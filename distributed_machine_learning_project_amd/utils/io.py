"""Input/output contract of the reference (common.cpp:12-79, generate_input.py:6-23).

Input text:  "<N> <Q> <A>\\n", N lines "<label> a_0 .. a_{A-1}", Q lines "Q <k> a_0 .. a_{A-1}".
Output text: "Query <id> checksum: <u64>\\n" per query in id order (release), or the DEBUG
listing "Label for Query <id> : <label>" / "Top-<k> neighbors:" / "<id> : <dist>".

Parsing and formatting run in the native library (multi-threaded C++), with strtod so parsed
doubles are bit-identical to `std::stringstream >> double` in the reference harness.
"""
from __future__ import annotations

import ctypes as C
import random
import sys
from dataclasses import dataclass, field

import numpy as np

from .. import _lib


@dataclass
class Params:
    """common.h:4-8."""
    num_data: int = 0
    num_queries: int = 0
    num_attrs: int = 0


@dataclass
class DataPoint:
    """common.h:10-14 (AoS form; the framework itself works on the flat arrays below)."""
    id: int
    label: int
    attrs: list = field(default_factory=list)


@dataclass
class Query:
    """common.h:16-20."""
    id: int
    k: int
    attrs: list = field(default_factory=list)


@dataclass
class Update:
    """common.h:22-25: replace the attributes of data point `id` (dead code in the reference's
    harness; here it drives KNNInput.apply_updates / KNNClassifier.update)."""
    id: int
    new_attrs: list = field(default_factory=list)


def parse_update(line: str) -> Update:
    """common.cpp:46-55: "<id> <a_0> <a_1> ..." (every remaining token is an attribute)."""
    tok = line.split()
    if not tok:
        raise InputFormatError("empty update line")
    try:
        return Update(int(tok[0]), [float(t) for t in tok[1:]])
    except ValueError as e:
        raise InputFormatError(f"malformed update line: {line!r}") from e


@dataclass
class KNNInput:
    """Parsed workload in flat, device-friendly form (ids are the row indices)."""
    labels: np.ndarray  # int32 [N]
    X: np.ndarray       # float64 [N, A], C-contiguous
    k: np.ndarray       # int32 [Q]
    Qx: np.ndarray      # float64 [Q, A]

    @property
    def params(self) -> Params:
        return Params(self.X.shape[0], self.Qx.shape[0], self.X.shape[1])

    @property
    def N(self):
        return self.X.shape[0]

    @property
    def Q(self):
        return self.Qx.shape[0]

    @property
    def A(self):
        return self.X.shape[1]

    def datapoints(self):
        return [DataPoint(i, int(self.labels[i]), list(self.X[i])) for i in range(self.N)]

    def queries(self):
        return [Query(i, int(self.k[i]), list(self.Qx[i])) for i in range(self.Q)]

    def apply_updates(self, updates) -> None:
        """Apply Update records in order (later updates of the same id win)."""
        for u in updates:
            if not 0 <= u.id < self.N or len(u.new_attrs) != self.A:
                raise ValueError(f"update {u.id}: id out of range or wrong attribute count")
            self.X[u.id] = np.asarray(u.new_attrs, np.float64)

    @staticmethod
    def from_aos(dataset, queries) -> "KNNInput":
        A = len(dataset[0].attrs) if dataset else (len(queries[0].attrs) if queries else 0)
        X = np.array([p.attrs for p in dataset], dtype=np.float64).reshape(len(dataset), A)
        labels = np.array([p.label for p in dataset], dtype=np.int32)
        Qx = np.array([q.attrs for q in queries], dtype=np.float64).reshape(len(queries), A)
        k = np.array([q.k for q in queries], dtype=np.int32)
        return KNNInput(labels, np.ascontiguousarray(X), k, np.ascontiguousarray(Qx))


class InputFormatError(RuntimeError):
    pass


def parse_input(data: bytes | str, nthreads: int = 0) -> KNNInput:
    if isinstance(data, str):
        data = data.encode()
    L = _lib.lib()
    buf = C.create_string_buffer(data, len(data))
    N, Q, body = C.c_int64(), C.c_int64(), C.c_int64()
    A = C.c_int()
    if L.dmlp_parse_header(buf, len(data), C.byref(N), C.byref(Q), C.byref(A), C.byref(body)) != 0:
        raise InputFormatError("malformed header line")
    N, Q, A = N.value, Q.value, A.value
    labels = np.empty(N, np.int32)
    X = np.empty((N, A), np.float64)
    k = np.empty(Q, np.int32)
    Qx = np.empty((Q, A), np.float64)
    rc = L.dmlp_parse_body(buf, len(data), body.value, N, Q, A, labels.ctypes.data,
                           X.ctypes.data, k.ctypes.data, Qx.ctypes.data, nthreads)
    if rc != 0:
        line = -rc
        kind = "data" if line <= N else "query"
        raise InputFormatError(f"malformed {kind} line {line + 1} (reference: common.cpp:100-115)")
    return KNNInput(labels, X, k, Qx)


def read_input(path: str | None = None) -> KNNInput:
    if path is None or path == "-":
        data = sys.stdin.buffer.read()
    else:
        with open(path, "rb") as f:
            data = f.read()
    return parse_input(data)


def format_report(checksums: np.ndarray, qid_base: int = 0) -> bytes:
    cs = np.ascontiguousarray(checksums, dtype=np.uint64)
    out = C.create_string_buffer(48 * len(cs) + 64)
    n = _lib.lib().dmlp_cpu_format_report(cs.ctypes.data, len(cs), qid_base, out)
    return out.raw[:n]


def format_debug(dist: np.ndarray, ids: np.ndarray, k: np.ndarray, labels_pred: np.ndarray) -> bytes:
    d = np.ascontiguousarray(dist, np.float64)
    i = np.ascontiguousarray(ids, np.int32)
    kk = np.ascontiguousarray(k, np.int32)
    lp = np.ascontiguousarray(labels_pred, np.int32)
    cap = 64 * len(kk) + 48 * int(kk.sum()) + 64
    out = C.create_string_buffer(cap)
    n = _lib.lib().dmlp_cpu_format_debug(d.ctypes.data, i.ctypes.data, d.shape[1] if d.ndim == 2 else 0,
                                         kk.ctypes.data, lp.ctypes.data, len(kk), out, cap)
    if n < 0:
        raise RuntimeError("debug report buffer overflow")
    return out.raw[:n]


# ------------------------------------------------------------------ workload generation
def generate_text(num_data, num_queries, num_attrs, vmin, vmax, minK, maxK, num_labels,
                  seed=42) -> str:
    """Byte-identical to generate_input.py (same `random` call sequence, generate_input.py:6-23)."""
    rng = random.Random(seed)
    lines = [f"{num_data} {num_queries} {num_attrs}"]
    for _ in range(num_data):
        label = rng.randint(0, num_labels - 1)
        attrs = " ".join(f"{rng.uniform(vmin, vmax):.6f}" for _ in range(num_attrs))
        lines.append(f"{label} {attrs}")
    for _ in range(num_queries):
        kq = rng.randint(minK, min(maxK, num_data))
        attrs = " ".join(f"{rng.uniform(vmin, vmax):.6f}" for _ in range(num_attrs))
        lines.append(f"Q {kq} {attrs}")
    return "\n".join(lines) + "\n"


def generate(num_data, num_queries, num_attrs, vmin=0.0, vmax=1000.0, minK=16, maxK=16,
             num_labels=10, seed=42) -> KNNInput:
    """Fast vectorised generator with generate_input.py's distribution (numpy PCG64 stream, not
    Python's Mersenne Twister): uniform attributes quantised to 6 decimals exactly as the text
    round trip would give, uniform labels, per-query k ~ U{minK, min(maxK, N)}."""
    g = np.random.default_rng(seed)
    scale = 1_000_000.0

    def attrs(n):
        u = g.uniform(vmin, vmax, size=(n, num_attrs))
        return np.rint(u * scale) / scale  # == strtod("%.6f")

    X = np.ascontiguousarray(attrs(num_data))
    labels = g.integers(0, num_labels, size=num_data, dtype=np.int64).astype(np.int32)
    k = g.integers(minK, min(maxK, num_data) + 1, size=num_queries, dtype=np.int64).astype(np.int32)
    Qx = np.ascontiguousarray(attrs(num_queries))
    return KNNInput(labels, X, k, Qx)


def write_input(path, inp: KNNInput) -> None:
    """inp as the reference's input file at `path` — the bytes of to_text(inp), formatted by the
    native library on its render pool (hundreds of MB for the multi-rank contract runs)."""
    from .. import _lib
    lab = np.ascontiguousarray(inp.labels, np.int32)
    X = np.ascontiguousarray(inp.X, np.float64)
    k = np.ascontiguousarray(inp.k, np.int32)
    Qx = np.ascontiguousarray(inp.Qx, np.float64)
    rc = _lib.lib().dmlp_cpu_write_input(str(path).encode(), lab.ctypes.data, X.ctypes.data,
                                         X.shape[0], k.ctypes.data, Qx.ctypes.data, Qx.shape[0],
                                         X.shape[1])
    if rc != 0:
        raise OSError(f"cannot write {path}")


def to_text(inp: KNNInput) -> str:
    """Serialise a KNNInput in the reference input format (6 decimals, like generate_input.py)."""
    out = [f"{inp.N} {inp.Q} {inp.A}"]
    for i in range(inp.N):
        out.append(f"{int(inp.labels[i])} " + " ".join(f"{v:.6f}" for v in inp.X[i]))
    for i in range(inp.Q):
        out.append(f"Q {int(inp.k[i])} " + " ".join(f"{v:.6f}" for v in inp.Qx[i]))
    return "\n".join(out) + "\n"
