"""Node-shared input segment: the parsed workload placed in one /dev/shm mapping that every
rank of the node maps, so each GPU pulls ITS part of the input over its own PCIe link.

The reference harness parses stdin on rank 0 only (common.cpp:93-117) and every engine then
pushes all data out of rank 0 (bench_4 @0xc199 broadcasts the dataset, @0xd64c hands out
queries).  On one MI355X node the 8 GPUs hang off separate PCIe x16 links: funnelling every
byte through GPU 0's link serialises 8x the H2D volume (≈300 MB at 8 GPUs for the bench),
while per-rank copies from a node-shared page-locked segment run all 8 links concurrently
("per-GPU H2D from shared pinned host memory").  Placing the parsed arrays
in the segment is part of ingest (untimed, like parsing); every byte that moves host->GPU is
still moved inside the timed KNN call.

Egress is symmetric: with the static farm each rank renders the report lines of its own query
block on its GPU and copies them over its own PCIe link into the segment's output region at its
byte offset, so rank 0 ends up holding the whole report in host memory without a funnel.

Control plane: with every rank mapping the segment, the static farm's per-call bookkeeping
between the ranks of a node (report lengths, the "every block is written" barrier, the per-query
(label, checksum) rows) goes through it — atomics and plain stores on shared memory instead of
RCCL collectives with a host sync each.

Layout: 64-byte header (magic, N, Q, A, label lo, label hi, k min, k max — a summary for tools;
the KNN strategies re-scan the labels and k inside every timed call), two int64 work counters at
byte 64 (the dynamic farm's chunk claims, alternating per call), a barrier counter at byte 96,
a call generation at byte 80 (the dynamic farm: which counter a call claims from), the render
plane flag at byte 112 (1: the segment reserves the plane region),
per-rank int64 slots from byte 128 (report lengths), then labels i32[N], k i32[Q],
X f64[N*A], Qx f64[Q*A], out u8[48*Q + 64] (report text), res i64[2*Q] (the dynamic farm's
(label, checksum) per query), plane (the node render plane, csrc/plane.cpp: the dataset's fp16
image and int32 rows, rendered once per call by all ranks together, 1/P each), each section
4096-byte aligned.
"""
from __future__ import annotations

import os
import uuid

import numpy as np

from .io import KNNInput

_MAGIC = 0x444D4C50534D4831  # "DMLPSMH1"
_ALIGN = 4096
_PLANE_FLAG = 112  # header word: 1 when the segment reserves the render plane


def _up(x):
    return (x + _ALIGN - 1) // _ALIGN * _ALIGN


def _plane_bytes(N, A):
    """Bytes of the node render plane for this dataset (0: none — A beyond the screen's 256)."""
    from .. import _lib
    b = int(_lib.lib().dmlp_plane_bytes(N, A, 0))
    return max(b, 0)


def _layout(N, Q, A, plane):
    """Offsets of the segment's arrays; the render plane region only when the segment carries one
    (a one-rank job, or KNN_PLANE=0, maps no plane: it would be N * A * 2 bytes of tmpfs unused)."""
    off = {}
    o = _ALIGN
    for name, nbytes in (("labels", 4 * N), ("k", 4 * Q), ("X", 8 * N * A), ("Qx", 8 * Q * A),
                         ("out", 48 * Q + 64), ("res", 16 * Q),
                         ("plane", _plane_bytes(N, A) if plane else 0)):
        off[name] = o
        o += _up(max(nbytes, 1))
    return off, o


def _roomy_dir(directory: str, need: int) -> str:
    """directory when its filesystem has room for need bytes, else the first of $TMPDIR / /tmp /
    /var/tmp that has (a small /dev/shm — a container's 64 MiB default — would otherwise end in
    SIGBUS when the segment's pages are first written); the file-backed mapping is shared and
    page-locked the same way."""
    import tempfile

    def room(d):
        try:
            st = os.statvfs(d)
        except OSError:
            return 0
        return st.f_bavail * st.f_frsize

    for d in (directory, os.environ.get("TMPDIR") or "", tempfile.gettempdir(), "/tmp", "/var/tmp"):
        if d and os.path.isdir(d) and os.access(d, os.W_OK) and room(d) >= need + (64 << 20):
            return d
    return directory


class SharedInput(KNNInput):
    """KNNInput whose arrays are views of a node-shared mapping (same on every rank)."""
    shared = True

    def __init__(self, mm, path, N, Q, A, owner, plane):
        off, total = _layout(N, Q, A, plane)
        labels = np.frombuffer(mm, np.int32, N, off["labels"])
        k = np.frombuffer(mm, np.int32, Q, off["k"])
        X = np.frombuffer(mm, np.float64, N * A, off["X"]).reshape(N, A)
        Qx = np.frombuffer(mm, np.float64, Q * A, off["Qx"]).reshape(Q, A)
        super().__init__(labels, X, k, Qx)
        self.out = np.frombuffer(mm, np.uint8, 48 * Q + 64, off["out"])
        self.res = np.frombuffer(mm, np.int64, 2 * Q, off["res"]).reshape(Q, 2)
        self.counters = np.frombuffer(mm, np.int64, 2, 64)
        self._gen = np.frombuffer(mm, np.int64, 1, 80)
        self.slots = np.frombuffer(mm, np.int64, (_ALIGN - 128) // 8, 128)
        self._bar = np.frombuffer(mm, np.int64, 1, 96)
        self._nbar = 0  # barriers this process has entered
        self._mm, self.path, self.owner, self.nbytes = mm, path, owner, total
        self._pinned = False
        self._plane_off, self._plane_bytes = off["plane"], _plane_bytes(N, A) if plane else 0
        self._plane_gen = 0  # node render plane calls this process made (same on every rank)

    def plane(self, rank: int, renderers: int):
        """The node render plane for this call (ops.knn.Plane), or None when the segment has
        none: every rank calls it once per farm call, so the generations agree."""
        if not self._plane_bytes:
            return None
        from ..ops.knn import Plane
        self._plane_gen += 1
        return Plane(base=self._mm.ctypes.data + self._plane_off, bytes=self._plane_bytes,
                     rank=rank, renderers=renderers, with_f64=0, gen=self._plane_gen,
                     wait_s=float(os.environ.get("DMLP_PLANE_WAIT_S", "60")))

    @staticmethod
    def create(inp: KNNInput, directory: str = "/dev/shm", query_nodes=None,
               plane: bool = False) -> "SharedInput":
        """query_nodes: [(first query, end query, NUMA node), ...] — the query rows (and their
        report bytes) of each block are placed on that node before they are written (the GPU
        that reads them hangs off it); the dataset is interleaved over the nodes named.
        plane: reserve the node render plane (P > 1 ranks share the segment's dataset render)."""
        N, A = inp.X.shape
        Q = inp.Qx.shape[0]
        off, total = _layout(N, Q, A, plane)
        directory = _roomy_dir(directory, total)
        path = os.path.join(directory, f"dmlp_input_{os.getpid()}_{uuid.uuid4().hex[:8]}")
        mm = np.memmap(path, np.uint8, "w+", shape=(total,))
        if query_nodes:
            _place(mm, off, N, Q, A, query_nodes, plane)
        np.frombuffer(mm, np.int64, 4, 0)[:] = [_MAGIC, N, Q, A]
        np.frombuffer(mm, np.int64, 1, _PLANE_FLAG)[0] = int(bool(plane))
        s = SharedInput(mm, path, N, Q, A, owner=True, plane=plane)
        if s._plane_bytes:
            from .. import _lib
            _lib.check(_lib.lib().dmlp_plane_init(mm.ctypes.data + off["plane"], s._plane_bytes,
                                                  N, A, 0), "dmlp_plane_init")
        s.labels[:] = inp.labels
        s.k[:] = inp.k
        s.X[:] = inp.X
        s.Qx[:] = inp.Qx
        s.refresh_summary()
        mm.flush()
        return s

    def refresh_summary(self):
        """Recompute the header summary (call after writing the arrays in place)."""
        N, Q = len(self.labels), len(self.k)
        np.frombuffer(self._mm, np.int64, 4, 32)[:] = [
            int(self.labels.min()) if N else 0, int(self.labels.max()) + 1 if N else 1,
            int(self.k.min()) if Q else 0, int(self.k.max()) if Q else 0]

    def claim(self, slot: int) -> int:
        """Atomically take the next work item from counter `slot` (0 or 1): 0, 1, 2, ... across
        every process that maps the segment (a fetch-and-add on shared memory, no server)."""
        from .. import _lib
        return int(_lib.lib().dmlp_atomic_fetch_add_i64(self.counters.ctypes.data + 8 * slot, 1))

    def barrier(self, world: int, timeout_s: float = 600.0, idle_s: float = 0.0):
        """Barrier of the `world` processes mapping the segment: one atomic add on a monotonic
        counter, then a spin until every rank's add of this round has landed (the atomic is
        sequentially consistent, so stores before it are visible to every rank after it).
        idle_s > 0: a long wait sleeps that long between polls instead of yielding (ranks that
        wait seconds for rank 0 leave the CPUs to the work it runs)."""
        import time
        from .. import _lib
        L = _lib.lib()
        p = self._bar.ctypes.data
        self._nbar += 1
        target = self._nbar * world
        L.dmlp_atomic_fetch_add_i64(p, 1)
        t0 = None
        spins = 0
        while L.dmlp_atomic_fetch_add_i64(p, 0) < target:
            spins += 1
            if spins > 2000:
                if t0 is None:
                    t0 = time.monotonic()
                elif time.monotonic() - t0 > timeout_s:
                    raise TimeoutError("node-shared barrier: a rank did not arrive")
                time.sleep(idle_s)

    def reset_counter(self, slot: int):
        from .. import _lib
        _lib.lib().dmlp_atomic_store_i64(self.counters.ctypes.data + 8 * slot, 0)

    def begin_claims(self, world: int, is_root: bool) -> int:
        """Collective over the ranks mapping the segment: start a new round of claim() calls and
        return the counter slot every rank claims from.  The call generation lives in the
        segment (not in any one Engine), so a fresh Engine, or any caller whose call count does
        not match the segment's history, still starts on a zeroed counter: rank 0 bumps the
        generation and zeroes that generation's counter, then a segment barrier publishes both
        (and keeps every rank out of the round until rank 0 is done with the previous one)."""
        from .. import _lib
        L = _lib.lib()
        if is_root:
            g = int(L.dmlp_atomic_fetch_add_i64(self._gen.ctypes.data, 0)) + 1
            L.dmlp_atomic_store_i64(self.counters.ctypes.data + 8 * (g & 1), 0)
            L.dmlp_atomic_store_i64(self._gen.ctypes.data, g)
        if world > 1:
            self.barrier(world)
        return int(L.dmlp_atomic_fetch_add_i64(self._gen.ctypes.data, 0)) & 1

    @property
    def summary(self):
        """(label lo, label hi (exclusive), k min, k max) from the header."""
        return tuple(int(v) for v in np.frombuffer(self._mm, np.int64, 4, 32))

    @staticmethod
    def attach(path: str) -> "SharedInput":
        mm = np.memmap(path, np.uint8, "r+")
        magic, N, Q, A = (int(v) for v in np.frombuffer(mm, np.int64, 4, 0))
        if magic != _MAGIC:
            raise ValueError(f"{path}: not a dmlp input segment")
        plane = bool(np.frombuffer(mm, np.int64, 1, _PLANE_FLAG)[0])
        return SharedInput(mm, path, N, Q, A, owner=False, plane=plane)

    def pin(self) -> bool:
        """Page-lock the mapping for DMA (GPU ranks).  Returns False if HIP refused it (copies
        then fall back to staged pageable transfers; still correct)."""
        if self._pinned:
            return True
        from .. import _lib
        rc = _lib.lib().dmlp_host_register(self._mm.ctypes.data, self.nbytes)
        self._pinned = rc == 0
        return self._pinned

    def unlink(self):
        """Remove the name (mappings stay valid until closed): called once all ranks attached."""
        if self.owner and os.path.exists(self.path):
            os.unlink(self.path)

    def close(self):
        if self._pinned:
            from .. import _lib
            _lib.lib().dmlp_host_unregister(self._mm.ctypes.data)
            self._pinned = False
        self.unlink()


def _mbind(addr: int, length: int, nodes, mode: int) -> bool:
    """mbind(2) on [addr, addr + length) (page-aligned inward) — the policy of the shared tmpfs
    object, so it decides where the pages land when rank 0 writes them.  False on any failure."""
    import ctypes
    page = os.sysconf("SC_PAGE_SIZE")
    a0 = (addr + page - 1) // page * page
    a1 = (addr + length) // page * page
    if a1 <= a0 or not nodes or max(nodes) >= 64:
        return False
    import platform
    if platform.machine() != "x86_64":  # the syscall number below is x86_64's
        return False
    mask = ctypes.c_ulong(sum(1 << n for n in set(nodes)))
    libc = ctypes.CDLL(None, use_errno=True)
    SYS_mbind = 237  # x86_64
    rc = libc.syscall(SYS_mbind, ctypes.c_void_p(a0), ctypes.c_ulong(a1 - a0), ctypes.c_int(mode),
                      ctypes.byref(mask), ctypes.c_ulong(65), ctypes.c_uint(0))
    return rc == 0


def _place(mm, off, N, Q, A, query_nodes, plane):
    """NUMA placement of a fresh segment (best effort: any failure leaves the default policy).
    MPOL_PREFERRED, not MPOL_BIND: a node short of memory falls back to another node instead of
    failing rank 0's tmpfs writes with SIGBUS."""
    MPOL_PREFERRED, MPOL_INTERLEAVE = 1, 3
    base = mm.ctypes.data
    nodes = sorted({n for _, _, n in query_nodes if n >= 0})
    if not nodes:
        return
    if len(nodes) > 1:
        _mbind(base + off["X"], 8 * N * A, nodes, MPOL_INTERLEAVE)
        if plane:
            _mbind(base + off["plane"], _plane_bytes(N, A), nodes, MPOL_INTERLEAVE)
    for a, b, n in query_nodes:
        if n >= 0 and b > a:
            _mbind(base + off["Qx"] + 8 * A * a, 8 * A * (b - a), [n], MPOL_PREFERRED)
            _mbind(base + off["out"] + 48 * a, 48 * (b - a), [n], MPOL_PREFERRED)


def gpu_numa_node(dev_index: int) -> int:
    """NUMA node of GPU dev_index's PCIe root (sysfs), -1 if unknown."""
    try:
        import torch
        p = torch.cuda.get_device_properties(dev_index)
        bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as f:
            return int(f.read().strip())
    except (OSError, ValueError, AttributeError, RuntimeError, ImportError):
        return -1


def share_input(comm, inp: KNNInput | None, pin: bool | None = None) -> SharedInput:
    """Collective: rank 0 places `inp` in a node-shared segment, every rank maps it.  Single
    node only (all ranks must see the same /dev/shm)."""
    from ..parallel import dist_api as dist
    path = None
    s = None
    if comm.is_root:
        qn = None
        if comm.on_gpu and comm.world > 1 and os.environ.get("KNN_NUMA_BIND", "1") != "0":
            # each rank's query block next to its GPU (ranks r -> device r mod devices, as
            # Comm.init binds them; the static farm's balanced blocks)
            import torch
            from ..parallel.comm import block_partition
            ndev = max(1, torch.cuda.device_count())
            counts, displs = block_partition(inp.Qx.shape[0], comm.world)
            qn = [(displs[r], displs[r] + counts[r], gpu_numa_node(r % ndev))
                  for r in range(comm.world)]
        # the render plane only where ranks share a render (parallel/strategies.py farm)
        s = SharedInput.create(inp, query_nodes=qn,
                               plane=comm.world > 1 and os.environ.get("KNN_PLANE", "1") != "0")
        path = s.path
    if comm.world > 1:
        obj = [path]
        dist.broadcast_object_list(obj, 0, device=comm.device if comm.backend == "nccl" else None)
        path = obj[0]
        if not comm.is_root:
            s = SharedInput.attach(path)
        comm.barrier()
    s.unlink()  # every rank holds a mapping: drop the name so nothing leaks in /dev/shm
    if pin if pin is not None else comm.on_gpu:
        s.pin()
    return s
