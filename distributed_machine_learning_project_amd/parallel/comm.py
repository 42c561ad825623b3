"""Process/device runtime and collectives (SURVEY.md §2.6, §5 "Distributed communication backend").

One process per GPU.  On MI355X the data plane is RCCL over xGMI (torch.distributed backend
"nccl" == RCCL on ROCm); on CPU-only hosts the same code runs over gloo.  The reference's MPI
call sites map as follows (bench_* addresses from SURVEY.md §2.6):

  MPI_Bcast (params, dataset, k, queries)   -> Comm.bcast            (ncclBroadcast)
  MPI_Scatterv (shards)                     -> Comm.scatter_rows     (scatter, one xGMI hop each)
  MPI_Gather/Gatherv (per-query results)    -> Comm.gather_rows      (batched, once per call)
  (dataset replication, node-shared input)  -> Comm.allgather_rows   (all-gather of H2D shards)
  MPI_Reduce + user MPI_Op (bench_2/3)      -> strategies.tree_merge (send/recv + merge kernel)
  MPI_Cart_create/Cart_sub (engine.cpp)     -> Comm.grid_groups      (dist.new_group row/col)
  MPI_Send/Recv ANY_SOURCE farming (bench_4)-> Comm.claim            (TCPStore atomic counter)

Uneven splits are padded to the largest part (RCCL collectives need equal counts); padding
rows are never read back.
"""
from __future__ import annotations

import contextlib
import datetime
import os
from dataclasses import dataclass

import numpy as np


def _torch():
    import torch
    return torch


@contextlib.contextmanager
def quiet_stdout():
    """gloo prints connection banners on fd 1; the harness's stdout must carry only the report."""
    import sys
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        devnull = os.open(os.devnull, os.O_WRONLY)
        os.dup2(devnull, 1)
        os.close(devnull)
        yield
    finally:
        os.dup2(saved, 1)
        os.close(saved)


def dims_create(nprocs: int):
    """MPI_Dims_create(n, 2) equivalent: the most balanced factorisation, dims[0] >= dims[1]."""
    best = (nprocs, 1)
    r = 1
    while r * r <= nprocs:
        if nprocs % r == 0:
            best = (nprocs // r, r)
        r += 1
    return best


def block_partition(n: int, parts: int):
    """Balanced block partition (bench_1 @0xc5b2): counts[i] = n//p + (i < n%p), displs prefix."""
    base, rem = divmod(n, parts)
    counts = [base + (1 if i < rem else 0) for i in range(parts)]
    displs = [0] * parts
    for i in range(1, parts):
        displs[i] = displs[i - 1] + counts[i - 1]
    return counts, displs


@dataclass
class Comm:
    rank: int
    world: int
    local_rank: int
    device: "object"       # torch.device
    backend: str           # "nccl" (RCCL) or "gloo"
    initialized_here: bool = False
    _store: "object" = None

    # ------------------------------------------------------------------ setup
    _numa = -1  # NUMA node this process was bound to (bind_numa), -1 if none

    @staticmethod
    def _numa_node(dev_index: int) -> int:
        """NUMA node of a GPU's PCIe function (sysfs), -1 if unknown."""
        torch = _torch()
        try:
            p = torch.cuda.get_device_properties(dev_index)
            bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
            with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as f:
                return int(f.read().strip())
        except (OSError, ValueError, AttributeError, RuntimeError):
            return -1

    @staticmethod
    def bind_numa(dev_index: int, local_world: int = 1) -> int:
        """Pin this process to the CPUs of its GPU's NUMA node (within its current affinity),
        before any large host allocation: first-touch then places the input, the page-locked
        staging and the render pool's threads next to the GPU's PCIe root, so the host render
        and the H2D copies never cross the socket link (unpinned, ~1 run in 3 measured ~20 %
        slower: profiles/r3m_numa.txt).  Every thread of the process is re-pinned (the HIP
        runtime's and torch's, started before this call, too), and DMLP_NODE_RANKS tells the
        render pool how many of the node's local ranks (local rank r drives GPU r % ndev) share
        this mask.  KNN_NUMA_BIND=0 disables it.  Returns the node or -1."""
        if os.environ.get("KNN_NUMA_BIND", "1") == "0":
            return -1
        torch = _torch()
        node = Comm._numa_node(dev_index)
        if node < 0:
            return -1
        try:
            with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
                cpus = set()
                for part in f.read().strip().split(","):
                    lo, _, hi = part.partition("-")
                    cpus.update(range(int(lo), int(hi or lo) + 1))
            mine = os.sched_getaffinity(0) & cpus
            if not mine:
                return -1
            os.sched_setaffinity(0, mine)
            for tid in os.listdir("/proc/self/task"):
                try:
                    os.sched_setaffinity(int(tid), mine)
                except OSError:
                    pass  # a thread that just exited
        except (OSError, ValueError):
            return -1
        ndev = max(1, torch.cuda.device_count())
        nodes = {}
        share = sum(1 for r in range(max(1, local_world))
                    if nodes.setdefault(r % ndev, Comm._numa_node(r % ndev)) == node)
        os.environ["DMLP_NODE_RANKS"] = str(max(1, share))
        return node

    @staticmethod
    def init(device: str = "auto", timeout_s: int = 600) -> "Comm":
        """Initialise torch.distributed from the launcher environment (RANK/WORLD_SIZE/
        LOCAL_RANK/MASTER_ADDR/MASTER_PORT); a single process without them is world_size 1."""
        torch = _torch()
        import torch.distributed as dist
        use_gpu = device == "gpu" or (device == "auto" and torch.cuda.is_available())
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
        if use_gpu:
            ndev = torch.cuda.device_count()
            torch.cuda.set_device(local_rank % max(1, ndev))
            # ranks of this node on the same GPU (DMLP_DATA_PLANE=host rehearsals): the native
            # step's early start stays off for them (csrc/pipeline.hip early_on)
            lw = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
            same = sum(1 for r in range(max(1, lw)) if r % max(1, ndev) == local_rank % max(1, ndev))
            os.environ["DMLP_DEVICE_RANKS"] = str(max(1, same))
            dev = torch.device("cuda", torch.cuda.current_device())
            Comm._numa = Comm.bind_numa(dev.index, int(os.environ.get("LOCAL_WORLD_SIZE", "1")))
        else:
            dev = torch.device("cpu")
        # DMLP_DATA_PLANE=host: gloo over host-staged copies of the device tensors (dist_api.py)
        # so that several ranks can share one GPU — a test mode; RCCL is the MI355X data plane
        staged = use_gpu and os.environ.get("DMLP_DATA_PLANE", "") == "host"
        backend = "nccl" if use_gpu and not staged else "gloo"
        here = False
        if world > 1 and not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29511")
            kw = {}
            if backend == "nccl":
                kw["device_id"] = dev
            with quiet_stdout():
                dist.init_process_group(backend, rank=rank, world_size=world,
                                        timeout=datetime.timedelta(seconds=timeout_s), **kw)
                if backend == "gloo":
                    dist.barrier()
            here = True
        elif dist.is_initialized():
            rank, world = dist.get_rank(), dist.get_world_size()
            backend = dist.get_backend()
        return Comm(rank, world, local_rank, dev, backend, here)

    def finalize(self):
        from . import dist_api as dist
        if self.initialized_here and dist.is_initialized():
            dist.destroy_process_group()

    @property
    def is_root(self):
        return self.rank == 0

    @property
    def on_gpu(self):
        return self.device.type == "cuda"

    # ------------------------------------------------------------------ primitives
    def barrier(self):
        if self.world > 1:
            from . import dist_api as dist
            dist.barrier(device_ids=[self.device.index] if self.on_gpu else None)

    def sync(self):
        if self.on_gpu:
            _torch().cuda.synchronize(self.device)

    def bcast_ints(self, vals=None, n: int = 0):
        """Broadcast a small int64 vector from rank 0 (the 3 x MPI_Bcast of Params)."""
        torch = _torch()
        if self.world == 1:
            return list(vals)
        from . import dist_api as dist
        n = len(vals) if vals is not None else n
        t = torch.zeros(n, dtype=torch.int64, device=self.device)
        if self.is_root:
            t.copy_(torch.tensor(list(vals), dtype=torch.int64))
        dist.broadcast(t, 0)
        return [int(x) for x in t.cpu().tolist()]

    def allgather_ints(self, vals):
        """Every rank's small int vector, concatenated in rank order (host list)."""
        torch = _torch()
        if self.world == 1:
            return [list(vals)]
        from . import dist_api as dist
        t = torch.tensor(list(vals), dtype=torch.int64, device=self.device)
        out = torch.empty(self.world * t.numel(), dtype=torch.int64, device=self.device)
        dist.all_gather_into_tensor(out, t)
        flat = [int(x) for x in out.cpu().tolist()]
        n = t.numel()
        return [flat[r * n:(r + 1) * n] for r in range(self.world)]

    def bcast(self, t, shape, dtype):
        """Broadcast a tensor from rank 0 (allocated on the other ranks)."""
        torch = _torch()
        if self.world == 1:
            return t
        from . import dist_api as dist
        if not self.is_root:
            t = torch.empty(shape, dtype=dtype, device=self.device)
        if t.numel():
            dist.broadcast(t, 0)
        return t

    def scatter_rows(self, t, counts, row_shape, dtype):
        """Scatter row blocks [counts[i] rows -> rank i] from rank 0 (MPI_Scatterv)."""
        torch = _torch()
        if self.world == 1:
            return t[: counts[0]]
        from . import dist_api as dist
        mx = max(counts)
        out = torch.empty((mx, *row_shape), dtype=dtype, device=self.device)
        if mx == 0:
            return out[:0]
        chunks = None
        if self.is_root:
            chunks = []
            off = 0
            for c in counts:
                blk = t[off:off + c]
                if c < mx:
                    pad = torch.zeros((mx - c, *row_shape), dtype=dtype, device=self.device)
                    blk = torch.cat([blk, pad])
                chunks.append(blk.contiguous())
                off += c
        dist.scatter(out, chunks, src=0)
        return out[: counts[self.rank]]

    def allgather_rows(self, t, counts, row_shape, dtype):
        """Every rank contributes counts[rank] rows; every rank gets the concatenation in rank
        order (MPI_Allgatherv; one RCCL all-gather over xGMI, padded to the largest part)."""
        torch = _torch()
        if self.world == 1:
            return t
        from . import dist_api as dist
        mx = max(counts)
        if mx == 0:
            return torch.empty((0, *row_shape), dtype=dtype, device=self.device)
        src = t
        if t.shape[0] != mx:
            src = torch.zeros((mx, *row_shape), dtype=dtype, device=self.device)
            src[: t.shape[0]] = t
        out = torch.empty((self.world * mx, *row_shape), dtype=dtype, device=self.device)
        dist.all_gather_into_tensor(out, src.contiguous())
        if all(c == mx for c in counts):
            return out
        return torch.cat([out[r * mx:r * mx + c] for r, c in enumerate(counts)])

    def allgather_into(self, out, chunk):
        """out = the concatenation of every rank's equal-size `chunk` in rank order (one RCCL
        all-gather; out and chunk are flat device tensors, out.numel() = world * chunk.numel())."""
        if self.world == 1:
            out.copy_(chunk)
            return out
        from . import dist_api as dist
        dist.all_gather_into_tensor(out, chunk)
        return out

    def allreduce_max_(self, t):
        """In-place elementwise max over ranks."""
        if self.world > 1:
            from . import dist_api as dist
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return t

    def gather_rows(self, t, counts, row_shape, dtype):
        """Gather row blocks to rank 0 in rank order (MPI_Gatherv); returns the concatenation on
        rank 0 and None elsewhere."""
        torch = _torch()
        if self.world == 1:
            return t
        from . import dist_api as dist
        mx = max(counts)
        src = torch.zeros((mx, *row_shape), dtype=dtype, device=self.device)
        if t is not None and t.shape[0]:
            src[: t.shape[0]] = t
        bufs = [torch.empty_like(src) for _ in range(self.world)] if self.is_root else None
        dist.gather(src, bufs, dst=0)
        if not self.is_root:
            return None
        return torch.cat([b[:c] for b, c in zip(bufs, counts)])

    def send(self, t, dst):
        from . import dist_api as dist
        dist.send(t.contiguous(), dst)

    def recv(self, shape, dtype, src):
        torch = _torch()
        from . import dist_api as dist
        t = torch.empty(shape, dtype=dtype, device=self.device)
        dist.recv(t, src)
        return t

    def new_group(self, ranks):
        from . import dist_api as dist
        if self.world == 1:
            return None
        with quiet_stdout():
            g = dist.new_group(ranks=ranks)
            if not self.on_gpu and self.rank in ranks:
                dist.barrier(group=g)  # gloo connects (and prints) eagerly; finish it here
        return g

    # ------------------------------------------------------------------ dynamic farming
    def store(self):
        if self._store is None and self.world > 1:
            import torch.distributed as dist
            from torch.distributed import distributed_c10d as c10d
            self._store = c10d._get_default_store()
        return self._store

    def claim(self, key: str) -> int:
        """Atomically claim the next work item (the bench_4 master's ANY_SOURCE hand-out,
        without a master rank): returns 0, 1, 2, ... across all ranks."""
        st = self.store()
        if st is None:
            v = getattr(self, "_local_ctr", {}).get(key, 0)
            self.__dict__.setdefault("_local_ctr", {})[key] = v + 1
            return v
        return int(st.add(key, 1)) - 1
