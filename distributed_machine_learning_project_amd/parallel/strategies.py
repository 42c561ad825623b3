"""Distributed k-NN strategies — every parallelism of the reference,
re-designed for one process per MI355X with RCCL over xGMI.  All of them produce byte-identical
results (exact fp64 distances, (dist asc, id desc) order, vote tie -> larger label).

  farm          bench_4 (B4 @0xbe50): dataset replicated by broadcast, queries farmed out.
                schedule="static": one scatter of balanced query blocks (identical MI355Xs make
                static optimal); schedule="dynamic": ranks claim query chunks from a shared
                atomic counter (the master's ANY_SOURCE hand-out without a dedicated master),
                results combined by a sum-reduce of disjoint slots.
  shard_gather  bench_1 (B1 @0xc410): dataset sharded (scatter), all queries broadcast once,
                local top-k per shard, ONE batched gather of the [P, Q, k] lists (not 2 per
                query), K-way merge kernel at the root.
  shard_reduce  bench_2/bench_3 (B2 @0xbdc0 + MPI_Op @0xbc70): same sharding, lists combined
                by a log2(P) send/recv tree with the pairwise merge kernel at every interior
                node (RCCL has no user reductions), batched over all queries (B3 style).
  grid2d        engine.cpp (E2-E9, with defects D1-D6 fixed): R x C process grid
                (MPI_Dims_create), data sharded over grid rows, queries over grid columns,
                row/column sub-communicators (MPI_Cart_sub -> dist.new_group), column merge to
                row 0, results gathered to rank 0.
  serial        bench.debug (B0): KD-tree on rank 0's CPU, other ranks idle.
  ring          beyond the reference: dataset sharded, queries split, shards
                rotate around the xGMI ring while each rank merges its queries' running top-k —
                datasets larger than one GPU's HBM.
"""
from __future__ import annotations

import os

import numpy as np

from .comm import block_partition, dims_create

STRATEGIES = ("farm", "shard_gather", "shard_reduce", "grid2d", "serial", "ring")


def _torch():
    import torch
    return torch


def _offset_ids(ids, off):
    torch = _torch()
    if off == 0:
        return ids
    return torch.where(ids >= 0, ids + off, ids)


def _root_arrays(be, inp):
    """H2D of the root's host arrays (pinned torch tensors when the caller provided them)."""
    torch = _torch()
    g = lambda name, dt: be.tensor(getattr(inp, name + "_t", None) if getattr(inp, name + "_t", None)
                                   is not None else getattr(inp, name), dt)
    return (g("X", torch.float64), g("labels", torch.int32), g("Qx", torch.float64),
            g("k", torch.int32))


def _meta(comm, inp, with_shared=False):
    """Sizes, label range, kmax (engine.cpp:27-35) [+ whether the input is a node-shared
    segment that every rank has mapped].  With a node-shared segment (mapped by every rank by
    construction: share_input is collective) each rank scans it itself, no broadcast."""
    if getattr(inp, "shared", False):
        from .. import _lib
        N, A = inp.X.shape
        Q = inp.Qx.shape[0]
        lmin, lmax = _lib.i32_range(inp.labels)
        lo, hi = (lmin, lmax + 1) if N else (0, 1)
        kmin, kmx = _lib.i32_range(inp.k) if Q else (0, 0)
        kmax = max(1, kmx) if Q else 1
        inp.k_range_all = (kmin, kmx)  # this call's k bounds (the farm's world-1 dispatch)
        out = [N, Q, A, lo, hi, kmax, 1]
        return out if with_shared else out[:6]
    if comm.is_root:
        N, A = inp.X.shape
        Q = inp.Qx.shape[0]
        # scanned inside every call, like the reference engines' own passes over the input
        from .. import _lib
        lmin, lmax = _lib.i32_range(inp.labels)
        lo, hi = (lmin, lmax + 1) if N else (0, 1)
        kmax = max(1, _lib.i32_range(inp.k)[1]) if Q else 1
        vals = [N, Q, A, lo, hi, kmax, int(bool(getattr(inp, "shared", False)))]
    else:
        vals = None
    out = comm.bcast_ints(vals, 7)
    if out[6] and not getattr(inp, "shared", False):
        raise RuntimeError("rank 0 passed a node-shared input but this rank has none mapped")
    return out if with_shared else out[:6]


def _lib_range(k):
    from .. import _lib
    lo, hi = _lib.i32_range(k)
    return (lo, hi) if len(k) else (0, 0)


def _k_host(comm, k_dev_or_none, Q):
    """Every rank needs the per-query k on the host (it drives kernel dispatch)."""
    torch = _torch()
    k = comm.bcast(k_dev_or_none, (Q,), torch.int32)
    return k, k.cpu().numpy()


# ============================================================================ farm (bench_4)
def farm(comm, be, inp, tr, schedule="static", chunks_per_rank=4, call_id=0, debug=False, **_):
    torch = _torch()
    import os
    if (getattr(inp, "shared", False) and schedule == "static" and comm.world == 1 and not debug
            and be.on_gpu and not int(os.environ.get("KNN_MAX_DEVICE_ROWS", "0") or 0)):
        # one rank, the whole call in the native step: it scans the label and k ranges itself
        # (on its render pool, ~2 us instead of ~30 us of host scans on the critical path)
        N, A = inp.X.shape
        return _farm_shared(comm, be, inp, tr, N, inp.Qx.shape[0], A, None, None, None, debug)
    N, Q, A, lo, hi, kmax, shared = _meta(comm, inp, with_shared=True)
    if shared and schedule == "static":
        return _farm_shared(comm, be, inp, tr, N, Q, A, lo, hi, kmax, debug)
    if shared and not debug:
        return _farm_dynamic_shared(comm, be, inp, tr, N, Q, A, lo, hi, kmax, call_id,
                                    chunks_per_rank)
    with tr.phase("h2d"):
        X = lab = Qx = kd = None
        if shared:  # dynamic schedule over a node-shared segment: per-rank dataset H2D
            X, lab = be.tensor(inp.X), be.tensor(inp.labels)
        elif comm.is_root:
            X, lab, Qx, kd = _root_arrays(be, inp)
    if not shared:
        with tr.phase("bcast_data"):
            X = comm.bcast(X, (N, A), torch.float64)
            lab = comm.bcast(lab, (N,), torch.int32)
    if schedule == "static":
        counts, displs = block_partition(Q, comm.world)
        with tr.phase("scatter_queries"):
            Ql = comm.scatter_rows(Qx, counts, (A,), torch.float64)
            kl = comm.scatter_rows(kd, counts, (), torch.int32)
            kl_h = kl.cpu().numpy()
        with tr.phase("compute"):
            d, i, lb, cs = be.knn(X, Ql, kl_h, labels=lab, label_range=(lo, hi), kstride=kmax)
        with tr.phase("gather"):
            packed = torch.stack([lb.to(torch.int64), cs], dim=1)
            allp = comm.gather_rows(packed, counts, (2,), torch.int64)
            dd = ii = None
            if debug:
                dd = comm.gather_rows(d, counts, (kmax,), torch.float64)
                ii = comm.gather_rows(i, counts, (kmax,), torch.int32)
        if not comm.is_root:
            return None
        return allp[:, 0].to(torch.int32), allp[:, 1].contiguous(), dd, ii
    # dynamic: every rank holds all queries; chunks are claimed from an atomic counter
    with tr.phase("bcast_queries"):
        if shared:  # claimed chunks are copied straight from the segment
            k_h = np.array(inp.k)
        else:
            Qx = comm.bcast(Qx, (Q, A), torch.float64)
            kd, k_h = _k_host(comm, kd, Q)
    nchunks = max(1, min(Q, comm.world * chunks_per_rank))
    csz = (Q + nchunks - 1) // nchunks
    out = torch.zeros((Q, 2), dtype=torch.int64, device=be.device)
    dbg_d = torch.zeros((Q, kmax), dtype=torch.float64, device=be.device) if debug else None
    dbg_i = torch.zeros((Q, kmax), dtype=torch.int32, device=be.device) if debug else None
    with tr.phase("compute"):
        key = f"dmlp_farm_{call_id}"
        while True:
            c = comm.claim(key)
            if c >= nchunks:
                break
            a, b = c * csz, min(Q, (c + 1) * csz)
            if a >= b:
                continue
            Qc = be.tensor(inp.Qx[a:b]) if shared else Qx[a:b]
            d, i, lb, cs = be.knn(X, Qc, k_h[a:b], labels=lab, label_range=(lo, hi),
                                  kstride=kmax)
            out[a:b, 0] = lb.to(torch.int64)
            out[a:b, 1] = cs
            if debug:
                dbg_d[a:b] = d
                dbg_i[a:b] = i
    with tr.phase("reduce"):
        if comm.world > 1:
            from . import dist_api as dist
            dist.reduce(out, 0, op=dist.ReduceOp.SUM)
            if debug:
                dist.reduce(dbg_d, 0, op=dist.ReduceOp.SUM)
                dist.reduce(dbg_i, 0, op=dist.ReduceOp.SUM)
    if not comm.is_root:
        return None
    return out[:, 0].to(torch.int32), out[:, 1].contiguous(), dbg_d, dbg_i


def _farm_dynamic_shared(comm, be, inp, tr, N, Q, A, lo, hi, kmax, call_id, chunks_per_rank):
    """Dynamic farm over the node-shared segment (bench_4's master/worker hand-out, @0xd80c
    Recv ANY_SOURCE -> @0xd986 Send, without a master rank or a server round trip): query
    chunks are claimed with an atomic fetch-and-add on a counter word in the shared mapping,
    each rank copies its claimed chunk straight from the segment to its GPU and writes the
    chunk's (label, checksum) rows back into the segment's results region; one barrier, and
    rank 0 holds every result.  The counter is chosen by a call generation kept in the segment
    (SharedInput.begin_claims: rank 0 bumps it and zeroes that counter, a segment barrier
    publishes it), so a second Engine on the same segment, or ranks whose call counts differ,
    never claim from an exhausted counter.  Rank 0 finishes reading the results region before
    it enters the next call's barrier, so no rank overwrites rows still being collected."""
    import os
    torch = _torch()
    slot = inp.begin_claims(comm.world, comm.is_root)
    claimed = 0
    per_rank = int(os.environ.get("KNN_CHUNKS_PER_RANK", chunks_per_rank))
    nchunks = max(1, min(Q, comm.world * max(1, per_rank)))
    csz = (Q + nchunks - 1) // nchunks
    with tr.phase("h2d"):
        X, lab = be.tensor(inp.X), be.tensor(inp.labels)
    res = torch.from_numpy(inp.res)  # host view of the shared results rows
    with tr.phase("compute"):
        while True:
            c = inp.claim(slot)
            if c >= nchunks:
                break
            a, b = c * csz, min(Q, (c + 1) * csz)
            if a >= b:
                continue
            kc = inp.k[a:b]
            d, i, lb, cs = be.knn(X, be.tensor(inp.Qx[a:b]), kc, labels=lab,
                                  label_range=(lo, hi), kstride=kmax)
            res[a:b].copy_(torch.stack([lb.to(torch.int64), cs], dim=1))  # D2H into the segment
            claimed += b - a
    inp.last_claimed = claimed  # queries this rank computed in this call (tests, diagnostics)
    comm.barrier()
    if not comm.is_root:
        return None
    with tr.phase("collect"):
        out = be.tensor(inp.res)
        if be.on_gpu:  # the H2D reads the segment: done before the next call's barrier
            torch.cuda.current_stream().synchronize()
    return out[:, 0].to(torch.int32), out[:, 1].contiguous(), None, None


def _farm_shared(comm, be, inp, tr, N, Q, A, lo, hi, kmax, debug):
    """Static farm over a node-shared input segment (utils/shm.py): every rank runs the native
    step (ops/knn.py step: libdmlp's one pipeline, csrc/pipeline.hip) on its own query block,
    straight from the segment over its own PCIe link — no funnel through GPU 0; the replicated
    dataset (bench_4 @0xc199 broadcasts it) is read by every rank from the segment.  Report lines:
    one rank writes them straight into the segment's output region; with P ranks each keeps its
    lines on its GPU, the lengths go through the segment's per-rank slots, and each rank copies
    its lines to its byte offset (no RCCL collective, no per-call small collective).
    KNN_DATA_INGRESS (A/B, P > 1): allgather — each rank H2Ds 1/P of the fp64 rows and one RCCL
    all-gather over xGMI completes the replica; bcast — rank 0 H2Ds them and broadcasts; both then
    run the device-rows pipeline (knn_gpu) on the rank's block."""
    import os
    torch = _torch()
    counts, displs = block_partition(Q, comm.world)
    a, b = displs[comm.rank], displs[comm.rank] + counts[comm.rank]
    mode = os.environ.get("KNN_DATA_INGRESS", "auto") if comm.world > 1 else "h2d"
    if mode == "auto":  # from the untimed probe's measurements (Engine._warmup), for this N x A
        mode = replication_mode(getattr(comm, "replication", None), N * A * 4)
    max_rows = int(os.environ.get("KNN_MAX_DEVICE_ROWS", "0") or 0)
    kl_h = inp.k[a:b]  # a view of the node-shared segment (never written here)
    if max_rows and N > max_rows:
        # out-of-core: the replica does not fit the device budget, stream it from the segment
        with tr.phase("h2d"):
            Ql = be.tensor(inp.Qx[a:b])
        with tr.phase("h2d+compute"):
            d, i, lb, cs = be.knn_streamed(inp.X, inp.labels, (lo, hi), Ql, np.array(kl_h),
                                           max_rows, kstride=kmax)
        return _farm_shared_tail(comm, be, inp, tr, counts, a, kmax, d, i, lb, cs, debug)
    if mode in ("h2d", "xgmi") and be.on_gpu:
        x32 = None
        if mode == "xgmi" and not debug:
            with tr.phase("replica"):  # 1/P of the rows over PCIe, the rest over xGMI
                x32 = _x32_replica(comm, be, inp)
        with tr.phase("step"):
            # lo / hi / kmax None (one rank, farm()): the native step scans them
            k_range = (None if kmax is None else inp.k_range_all if comm.world == 1
                       else _lib_range(kl_h))
            rep = None if debug else (inp.out if comm.world == 1 else "device")
            # P > 1: the replicated dataset's image and rows are rendered once for the node, 1/P
            # by each rank, into the segment's render plane (KNN_PLANE=0: every rank renders all)
            # (the debug listing's gather is no barrier between calls: no plane there)
            plane = (inp.plane(comm.rank, comm.world) if comm.world > 1 and not debug
                     and os.environ.get("KNN_PLANE", "1") != "0" else None)
            r = be.step(inp.X, inp.labels, None if lo is None else (lo, hi), inp.Qx[a:b], kl_h,
                        k_range=k_range, qid_base=a, report=rep, lists=debug, kstride=kmax,
                        plane=plane, x32=x32)
        if debug:
            return _farm_shared_tail(comm, be, inp, tr, counts, a, kmax, r.dist, r.ids, r.label,
                                     r.checksum, True)
        with tr.phase("report"):
            text = _step_egress(comm, inp, r, a)
        if comm.world == 1:
            return r.label, r.checksum, None, None, text
        if not comm.is_root:
            return None
        res = torch.from_numpy(inp.res)  # copies: the segment is reused by the next call
        return res[:, 0].to(torch.int32), res[:, 1].contiguous(), None, None, text
    with tr.phase("h2d"):
        Ql = be.tensor(inp.Qx[a:b])
        X = lab = None
        if mode == "allgather":
            nc, nd = block_partition(N, comm.world)
            r0, r1 = nd[comm.rank], nd[comm.rank] + nc[comm.rank]
            Xs, ls = be.tensor(inp.X[r0:r1]), be.tensor(inp.labels[r0:r1])
        elif mode != "bcast" or comm.is_root:
            X, lab = be.tensor(inp.X), be.tensor(inp.labels)
    if mode == "allgather":
        with tr.phase("allgather_data"):
            X = comm.allgather_rows(Xs, nc, (A,), torch.float64)
            lab = comm.allgather_rows(ls, nc, (), torch.int32)
    elif mode == "bcast":
        with tr.phase("bcast_data"):
            X = comm.bcast(X, (N, A), torch.float64)
            lab = comm.bcast(lab, (N,), torch.int32)
    with tr.phase("compute"):
        d, i, lb, cs = be.knn(X, Ql, np.array(kl_h), labels=lab, label_range=(lo, hi),
                              kstride=kmax)
    return _farm_shared_tail(comm, be, inp, tr, counts, a, kmax, d, i, lb, cs, debug)


def _x32_replica(comm, be, inp):
    """The dataset's rows on every GPU as lossless int32, assembled over xGMI: each rank packs
    and copies over its own PCIe link only its 1/P shard (rows [r s, (r + 1) s), s = ceil(N / P),
    zero-padded), and one all-gather (RCCL) completes the replica — instead of every GPU pulling
    all N rows over its own link.  bench_4 replicates the dataset with one MPI_Bcast (@0xc199);
    this is its xGMI form.  None (every rank agrees, one 4-byte all-reduce) when some value is
    not a 6-decimal number: the rows then go through the render plane."""
    torch = _torch()
    from .. import _lib
    from . import dist_api as dist
    N, A = inp.X.shape
    P, r = comm.world, comm.rank
    s = -(-N // P)
    r0, r1 = min(N, r * s), min(N, (r + 1) * s)
    st = getattr(inp, "_x32_stage", None)
    if st is None or st.numel() != s * A:
        st = torch.zeros(s * A, dtype=torch.int32).pin_memory()
        inp._x32_stage = st
    h = st.numpy()
    bad = 0
    if r1 > r0:
        bad = int(_lib.lib().dmlp_cpu_rows_i32(inp.X[r0:r1].ctypes.data, (r1 - r0) * A,
                                               h.ctypes.data))
    flag = torch.tensor([bad], dtype=torch.int32, device=be.device)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX)
    if int(flag.item()):
        return None
    shard = st.to(be.device, non_blocking=True)
    full = torch.empty(P * s * A, dtype=torch.int32, device=be.device)
    dist.all_gather_into_tensor(full, shard)
    return full


# In "h2d" mode the dataset's int32 rows cross each GPU's own link BEHIND the screen (only the
# re-rank waits for them); in "xgmi" mode 1/P of them cross and an all-gather completes them
# BEFORE the step (plus one small all-reduce + host sync on the pack's range check).  So xgmi pays
# only when the rows could not hide behind the screen: their concurrent H2D takes longer than
# about the screen's own time.
_ROWS_HIDE_S = 1.0e-3


def replication_mode(probe, row_bytes: int) -> str:
    """"xgmi" when every GPU copying row_bytes over its own link (at the bandwidth the probe saw
    with all ranks copying at once) would outlast what the screen hides and the all-gather is
    faster than that copy; else "h2d".  No probe: "h2d"."""
    if not probe or not probe.get("h2d_GBps_per_gpu_concurrent"):
        return "h2d"
    t_h2d = row_bytes / (probe["h2d_GBps_per_gpu_concurrent"] * 1e9)
    ag = probe.get("allgather_GBps") or 0.0
    t_x = (t_h2d / max(1, probe.get("world", 1))) + (row_bytes / (ag * 1e9) if ag else float("inf"))
    return "xgmi" if t_h2d > _ROWS_HIDE_S and t_x < t_h2d else "h2d"


def probe_replication(comm, nbytes=32 << 20, iters=3):
    """Untimed, at Engine construction (P > 1 on GPUs): how the replicated dataset should reach
    every GPU.  Measures, with every rank at once, the page-locked H2D bandwidth of one GPU and
    an all-gather of nbytes (maxima over ranks: every rank sees the same numbers and takes the
    same decision); replication_mode turns them into the choice for a call's dataset."""
    import time
    torch = _torch()
    from . import dist_api as dist
    P = comm.world
    n = nbytes // 4 // P * P
    h = torch.zeros(n, dtype=torch.int32).pin_memory()
    d = torch.empty(n, dtype=torch.int32, device=comm.device)
    shard = torch.zeros(n // P, dtype=torch.int32, device=comm.device)

    def timed(fn):
        fn()
        comm.sync()
        comm.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        comm.sync()
        t = torch.tensor([(time.perf_counter() - t0) / iters], dtype=torch.float64,
                         device=comm.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    t_h2d = timed(lambda: d.copy_(h, non_blocking=True))
    t_ag = timed(lambda: dist.all_gather_into_tensor(d, shard))
    t_x = t_h2d / P + t_ag
    out = {"bytes": n * 4, "world": P,
           "h2d_GBps_per_gpu_concurrent": round(n * 4 / t_h2d / 1e9, 2),
           "allgather_GBps": round(n * 4 / t_ag / 1e9, 2),
           "est_ms_h2d": round(t_h2d * 1e3, 4), "est_ms_xgmi": round(t_x * 1e3, 4)}
    # the choice for the bench_4 dataset (1e5 x 32 int32 rows); each call decides for its own
    # N x A (replication_mode)
    out["mode"] = replication_mode(out, 100_000 * 32 * 4)
    return out


def probe_replication_safe(comm):
    """probe_replication that cannot take the run down with it (the first real 8-GPU run has no
    second chance): a failure on any rank — DMLP_PROBE_FAIL=<rank>|all injects one before the
    probe's first collective — is agreed on by one MAX all-reduce, and every rank then records
    {"error": ..., "mode": "h2d"} (the replication that needs no collective).  A failure inside
    the probe's collectives is bounded by the process group's timeout (KNN_TIMEOUT_S)."""
    torch = _torch()
    from . import dist_api as dist
    err = None
    inj = os.environ.get("DMLP_PROBE_FAIL", "")
    try:
        if inj and (inj == "all" or str(comm.rank) in inj.split(",")):
            raise RuntimeError(f"injected probe failure on rank {comm.rank} (DMLP_PROBE_FAIL)")
        if not comm.on_gpu:
            raise RuntimeError("replication probe needs GPUs")
    except Exception as e:  # noqa: BLE001 — recorded, never fatal
        err = f"{type(e).__name__}: {e}"
    flag = torch.tensor([1 if err else 0], dtype=torch.int32, device=comm.device)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX)
    if int(flag.item()):
        return {"error": err or "probe failed on another rank", "mode": "h2d", "world": comm.world}
    try:
        return probe_replication(comm)
    except Exception as e:  # noqa: BLE001
        return {"error": f"{type(e).__name__}: {e}"[-300:], "mode": "h2d", "world": comm.world}


def _step_egress(comm, inp, r, qid_base):
    """The native step's report lines into the segment's output region.  One rank: the step
    already copied them to offset 0.  P ranks: each length goes through the segment's per-rank
    slots, a segment barrier, each rank copies its lines (still on its GPU) to its byte offset
    and its (label, checksum) rows to the results region, a second barrier; rank 0 gets a view
    of the whole report."""
    torch = _torch()
    from ..ops import knn as K
    n = r.report_len
    if comm.world == 1:
        comm.barrier()
        return memoryview(inp.out)[:n].toreadonly()
    inp.slots[comm.rank] = n
    inp.barrier(comm.world)  # every length is in its slot
    lens = [int(v) for v in inp.slots[:comm.world]]
    off = sum(lens[:comm.rank])
    if off + n > len(inp.out):
        raise RuntimeError("shared output region too small")
    K.step_emit(inp.out[off:off + n], n)
    nq = r.checksum.shape[0]
    if nq:
        rows = torch.from_numpy(inp.res[qid_base:qid_base + nq])
        rows.copy_(torch.stack([r.label.to(torch.int64), r.checksum], dim=1))
    inp.barrier(comm.world)  # every block's text and rows are in the segment
    return memoryview(inp.out)[:sum(lens)].toreadonly() if comm.is_root else None


def _farm_shared_tail(comm, be, inp, tr, counts, a, kmax, d, i, lb, cs, debug):
    torch = _torch()
    text = None
    if not debug:
        with tr.phase("report"):
            text = _shared_egress(comm, be, inp, cs, a, lb=lb)
    if comm.world == 1:
        return lb, cs, d if debug else None, i if debug else None, text
    if not debug:
        # every rank's (label, checksum) rows already sit in the segment (_shared_egress)
        if not comm.is_root:
            return None
        res = torch.from_numpy(inp.res)  # copies: the segment is reused by the next call
        return res[:, 0].to(torch.int32), res[:, 1].contiguous(), None, None, text
    with tr.phase("gather"):
        packed = torch.stack([lb.to(torch.int64), cs], dim=1)
        allp = comm.gather_rows(packed, counts, (2,), torch.int64)
        dd = comm.gather_rows(d, counts, (kmax,), torch.float64)
        ii = comm.gather_rows(i, counts, (kmax,), torch.int32)
    if not comm.is_root:
        return None
    return allp[:, 0].to(torch.int32), allp[:, 1].contiguous(), dd, ii, text


def _shared_egress(comm, be, inp, cs, qid_base, lb=None):
    """Every rank renders its block's report lines (GPU formatter, or the host's on CPU) and
    copies them straight into the shared segment's output region at its byte offset; rank 0 gets
    a view of the whole report.  P > 1: the lengths go through the segment's per-rank slots and
    two segment barriers order the writes; with lb given, the block's (label, checksum) rows are
    copied into the segment's results region in the same pass."""
    torch = _torch()
    if be.on_gpu:
        from ..ops import knn as K
        dev_text, n = K.format_report_dev(cs, qid_base)
    else:
        from ..utils.io import format_report
        host = format_report(cs.numpy().view(np.uint64), qid_base)
        n = len(host)
    if comm.world > 1:
        inp.slots[comm.rank] = n
        inp.barrier(comm.world)  # every length is in its slot
        lens = [int(v) for v in inp.slots[:comm.world]]
    else:
        lens = [n]
    off = sum(lens[:comm.rank])
    nq = cs.shape[0]
    if n:
        dst = torch.from_numpy(inp.out[off:off + n])
        if be.on_gpu:
            dst.copy_(dev_text[:n], non_blocking=True)  # D2H into the page-locked segment
        else:
            dst.copy_(torch.frombuffer(bytearray(host), dtype=torch.uint8))
    if lb is not None and comm.world > 1 and nq:
        rows = torch.from_numpy(inp.res[qid_base:qid_base + nq])
        rows.copy_(torch.stack([lb.to(torch.int64), cs], dim=1), non_blocking=True)
    if be.on_gpu:
        torch.cuda.current_stream().synchronize()
    if comm.world > 1:
        inp.barrier(comm.world)  # every block's text and rows are in the segment
    else:
        comm.barrier()
    return memoryview(inp.out)[:sum(lens)].toreadonly() if comm.is_root else None


# ============================================================================ sharded data
def _shard_local(comm, be, inp, tr):
    """Scatter the dataset in balanced blocks, broadcast queries, local top-k lists with
    global ids.  Returns (meta, root labels tensor, k_host, d, i)."""
    torch = _torch()
    N, Q, A, lo, hi, kmax, shared = _meta(comm, inp, with_shared=True)
    counts, displs = block_partition(N, comm.world)
    if shared:  # node-shared segment: each rank copies its own shard and the queries
        with tr.phase("h2d"):
            a = displs[comm.rank]
            Xl = be.tensor(inp.X[a:a + counts[comm.rank]])
            Qx = be.tensor(inp.Qx)
            k_h = np.array(inp.k)
            lab = be.tensor(inp.labels) if comm.is_root else None
    else:
        with tr.phase("h2d"):
            X = lab = Qx = kd = None
            if comm.is_root:
                X, lab, Qx, kd = _root_arrays(be, inp)
        with tr.phase("scatter_data"):
            Xl = comm.scatter_rows(X, counts, (A,), torch.float64)
        with tr.phase("bcast_queries"):
            Qx = comm.bcast(Qx, (Q, A), torch.float64)
            kd, k_h = _k_host(comm, kd, Q)
    with tr.phase("compute"):
        d, i, _, _ = be.knn(Xl, Qx, k_h, finalize=False, kstride=kmax)
        i = _offset_ids(i, displs[comm.rank])
    return (N, Q, A, lo, hi, kmax), lab, k_h, d, i


def shard_gather(comm, be, inp, tr, debug=False, **_):
    torch = _torch()
    (N, Q, A, lo, hi, kmax), lab, k_h, d, i = _shard_local(comm, be, inp, tr)
    with tr.phase("gather"):
        P = comm.world
        if P > 1:
            from . import dist_api as dist
            bd = [torch.empty_like(d) for _ in range(P)] if comm.is_root else None
            bi = [torch.empty_like(i) for _ in range(P)] if comm.is_root else None
            dist.gather(d.contiguous(), bd, dst=0)
            dist.gather(i.contiguous(), bi, dst=0)
    if not comm.is_root:
        return None
    with tr.phase("merge"):
        if P > 1:
            d, i = be.merge(torch.stack(bd), torch.stack(bi), k_h, kmax)
        lb, cs = be.finalize(lab, (lo, hi), d, i, k_h)
    return lb, cs, d, i


def tree_merge(comm, be, d, i, k_h, kmax, group_ranks=None, tr=None):
    """Binomial-tree reduction of sorted top-k lists toward group_ranks[0] (the MPI_Reduce with
    bench_2's commutative merge op): log2(P) rounds of send/recv, pairwise merge kernel at each
    receiving node.  Returns the merged lists on the tree root, None elsewhere."""
    torch = _torch()
    ranks = group_ranks or list(range(comm.world))
    P = len(ranks)
    me = ranks.index(comm.rank)
    step = 1
    while step < P:
        if me % (2 * step) == step:
            comm.send(d, ranks[me - step])
            comm.send(i, ranks[me - step])
            return None
        if me % (2 * step) == 0 and me + step < P:
            od = comm.recv(d.shape, d.dtype, ranks[me + step])
            oi = comm.recv(i.shape, i.dtype, ranks[me + step])
            d, i = be.merge(torch.stack([d, od]), torch.stack([i, oi]), k_h, kmax)
        step *= 2
    return d, i


def shard_reduce(comm, be, inp, tr, debug=False, **_):
    (N, Q, A, lo, hi, kmax), lab, k_h, d, i = _shard_local(comm, be, inp, tr)
    with tr.phase("tree_reduce"):
        res = tree_merge(comm, be, d, i, k_h, kmax)
    if not comm.is_root:
        return None
    d, i = res
    with tr.phase("finalize"):
        lb, cs = be.finalize(lab, (lo, hi), d, i, k_h)
    return lb, cs, d, i


# ============================================================================ grid2d (engine.cpp)
class GridGroups:
    """Row/column sub-communicators of the R x C grid (MPI_Cart_create + MPI_Cart_sub).
    dist.new_group is collective over the world, so all groups are created once, in order."""

    def __init__(self, comm):
        self.R, self.C = dims_create(comm.world)
        self.row, self.col = divmod(comm.rank, self.C)
        self.row_ranks = [[r * self.C + c for c in range(self.C)] for r in range(self.R)]
        self.col_ranks = [[r * self.C + c for r in range(self.R)] for c in range(self.C)]
        self.row_groups = [comm.new_group(rk) for rk in self.row_ranks]
        self.col_groups = [comm.new_group(rk) for rk in self.col_ranks]


def _grp_scatter(comm, t, counts, row_shape, dtype, group, ranks, src_idx=0):
    """MPI_Scatterv inside a sub-communicator (equal-size padded chunks)."""
    torch = _torch()
    from . import dist_api as dist
    me = ranks.index(comm.rank)
    mx = max(counts)
    out = torch.empty((mx, *row_shape), dtype=dtype, device=be_device(comm))
    if len(ranks) == 1:
        return t[: counts[0]]
    chunks = None
    if me == src_idx:
        chunks, off = [], 0
        for c in counts:
            blk = t[off:off + c]
            if c < mx:
                blk = torch.cat([blk, torch.zeros((mx - c, *row_shape), dtype=dtype, device=t.device)])
            chunks.append(blk.contiguous())
            off += c
    if mx:
        dist.scatter(out, chunks, src=ranks[src_idx], group=group)
    return out[: counts[me]]


def _grp_bcast(comm, t, shape, dtype, group, ranks, src_idx=0):
    torch = _torch()
    from . import dist_api as dist
    if len(ranks) == 1:
        return t
    if ranks.index(comm.rank) != src_idx:
        t = torch.empty(shape, dtype=dtype, device=be_device(comm))
    if t.numel():
        dist.broadcast(t, ranks[src_idx], group=group)
    return t


def be_device(comm):
    return comm.device


def grid2d(comm, be, inp, tr, groups=None, debug=False, **_):
    torch = _torch()
    from . import dist_api as dist
    g = groups or GridGroups(comm)
    N, Q, A, lo, hi, kmax = _meta(comm, inp)
    dcounts, ddispl = block_partition(N, g.R)   # data over grid rows (engine.cpp:62-63)
    qcounts, qdispl = block_partition(Q, g.C)   # queries over grid columns (engine.cpp:136-137)
    with tr.phase("h2d"):
        X = lab = Qx = kd = None
        if comm.is_root:
            X, lab, Qx, kd = _root_arrays(be, inp)
    with tr.phase("distribute"):
        # data: scatter down column 0 to the row leaders, then broadcast along each row
        Xs = None
        if g.col == 0:
            Xs = _grp_scatter(comm, X, dcounts, (A,), torch.float64, g.col_groups[0], g.col_ranks[0])
        Xs = _grp_bcast(comm, Xs, (dcounts[g.row], A), torch.float64, g.row_groups[g.row],
                        g.row_ranks[g.row])
        # queries (+k): scatter along row 0 to the column leaders, broadcast down each column
        Qs = ks = None
        if g.row == 0:
            Qs = _grp_scatter(comm, Qx, qcounts, (A,), torch.float64, g.row_groups[0], g.row_ranks[0])
            ks = _grp_scatter(comm, kd, qcounts, (), torch.int32, g.row_groups[0], g.row_ranks[0])
        Qs = _grp_bcast(comm, Qs, (qcounts[g.col], A), torch.float64, g.col_groups[g.col],
                        g.col_ranks[g.col])
        ks = _grp_bcast(comm, ks, (qcounts[g.col],), torch.int32, g.col_groups[g.col],
                        g.col_ranks[g.col])
        k_h = ks.cpu().numpy()
        # labels: only the row-0 ranks (column mergers) vote
        if g.row == 0:
            lab = _grp_bcast(comm, lab, (N,), torch.int32, g.row_groups[0], g.row_ranks[0])
    with tr.phase("compute"):
        d, i, _, _ = be.knn(Xs, Qs, k_h, finalize=False, kstride=kmax)
        i = _offset_ids(i, ddispl[g.row])
    with tr.phase("column_merge"):
        cr = g.col_ranks[g.col]
        if g.R > 1:
            me = cr.index(comm.rank)
            bd = [torch.empty_like(d) for _ in cr] if me == 0 else None
            bi = [torch.empty_like(i) for _ in cr] if me == 0 else None
            dist.gather(d.contiguous(), bd, dst=cr[0], group=g.col_groups[g.col])
            dist.gather(i.contiguous(), bi, dst=cr[0], group=g.col_groups[g.col])
            if me == 0:
                d, i = be.merge(torch.stack(bd), torch.stack(bi), k_h, kmax)
    if g.row != 0:
        return None
    with tr.phase("finalize"):
        lb, cs = be.finalize(lab, (lo, hi), d, i, k_h)
    with tr.phase("gather"):
        rr = g.row_ranks[0]
        packed = torch.stack([lb.to(torch.int64), cs], dim=1)
        if g.C > 1:
            mx = max(qcounts)
            src = torch.zeros((mx, 2), dtype=torch.int64, device=be.device)
            src[: packed.shape[0]] = packed
            bufs = [torch.empty_like(src) for _ in rr] if comm.is_root else None
            dist.gather(src, bufs, dst=0, group=g.row_groups[0])
            dd = ii = None
            if debug:
                sd = torch.full((mx, kmax), float("inf"), dtype=torch.float64, device=be.device)
                si = torch.full((mx, kmax), -1, dtype=torch.int32, device=be.device)
                sd[: d.shape[0]] = d
                si[: i.shape[0]] = i
                bd = [torch.empty_like(sd) for _ in rr] if comm.is_root else None
                bi = [torch.empty_like(si) for _ in rr] if comm.is_root else None
                dist.gather(sd, bd, dst=0, group=g.row_groups[0])
                dist.gather(si, bi, dst=0, group=g.row_groups[0])
            if not comm.is_root:
                return None
            allp = torch.cat([b[:c] for b, c in zip(bufs, qcounts)])
            if debug:
                dd = torch.cat([b[:c] for b, c in zip(bd, qcounts)])
                ii = torch.cat([b[:c] for b, c in zip(bi, qcounts)])
            return allp[:, 0].to(torch.int32), allp[:, 1].contiguous(), dd, ii
    return lb, cs, d, i


# ============================================================================ serial (bench.debug)
def serial(comm, be, inp, tr, debug=False, **_):
    """KD-tree on rank 0 (exact search, tie-inclusive pruning), no communication at all."""
    torch = _torch()
    from ..ops import knn as K
    if not comm.is_root:
        return None
    with tr.phase("compute"):
        d, i = K.knn_cpu(inp.X, inp.Qx, inp.k, method="kdtree")
        lb, cs = K.finalize_cpu(i, inp.k, inp.labels)
    return (torch.from_numpy(lb), torch.from_numpy(cs.view(np.int64)), torch.from_numpy(d),
            torch.from_numpy(i))


# ============================================================================ ring (beyond-HBM datasets)
def ring(comm, be, inp, tr, debug=False, **_):
    """Ring k-NN — the SURVEY.md §5 "long-context" analog (ring-attention pattern over the
    dataset axis): the dataset is sharded N/P per GPU and never replicated, the queries are split
    in P blocks, and every rank keeps the running top-k of its own block while the data shards
    travel one hop per step around the xGMI ring (P - 1 grouped send/recv exchanges, each
    overlapped with the local screen + exact re-rank of the shard in hand, merged by the K-way
    merge kernel).  Memory per GPU: two shards + Q/P queries, so datasets up to P x the HBM of
    one MI355X (288 GB ~ 3.6e10 fp64 values) stay exact, with the farm's query parallelism."""
    torch = _torch()
    N, Q, A, lo, hi, kmax, shared = _meta(comm, inp, with_shared=True)
    P, r = comm.world, comm.rank
    nc, nd = block_partition(N, P)
    qc, qd = block_partition(Q, P)
    mx = max(nc)
    with tr.phase("h2d"):
        if shared:  # node-shared segment: every rank copies its shard, its query block, labels
            cur = torch.zeros((mx, A), dtype=torch.float64, device=be.device)
            if nc[r]:
                cur[: nc[r]] = be.tensor(inp.X[nd[r]:nd[r] + nc[r]])
            Ql = be.tensor(inp.Qx[qd[r]:qd[r] + qc[r]])
            kl_h = np.array(inp.k[qd[r]:qd[r] + qc[r]], np.int32)
            lab = be.tensor(inp.labels)
        else:
            X = lab = Qx = kd = None
            if comm.is_root:
                X, lab, Qx, kd = _root_arrays(be, inp)
    if not shared:
        with tr.phase("scatter"):
            cur = comm.scatter_rows(X, nc, (A,), torch.float64)
            if cur.shape[0] < mx:
                cur = torch.cat([cur, torch.zeros((mx - cur.shape[0], A), dtype=torch.float64,
                                                  device=be.device)])
            Ql = comm.scatter_rows(Qx, qc, (A,), torch.float64)
            kl_h = comm.scatter_rows(kd, qc, (), torch.int32).cpu().numpy()
            lab = comm.bcast(lab, (N,), torch.int32)
    dr = ir = None
    nxt = torch.empty_like(cur) if P > 1 else None
    for step in range(P):
        src = (r - step) % P  # the shard in hand started on rank src
        reqs = []
        if step < P - 1:
            from . import dist_api as dist
            ops = [dist.P2POp(dist.isend, cur, (r + 1) % P), dist.P2POp(dist.irecv, nxt, (r - 1) % P)]
            with tr.phase("ring_post"):
                reqs = dist.batch_isend_irecv(ops)
        with tr.phase("compute"):
            d, i, _, _ = be.knn(cur[: nc[src]], Ql, kl_h, finalize=False, kstride=kmax)
            i = _offset_ids(i, nd[src])
            if dr is None:
                dr, ir = d, i
            else:
                dr, ir = be.merge(torch.stack([dr, d]), torch.stack([ir, i]), kl_h, kmax)
        if reqs:
            with tr.phase("ring_wait"):
                for q_ in reqs:
                    q_.wait()
            cur, nxt = nxt, cur
    with tr.phase("finalize"):
        lb, cs = be.finalize(lab, (lo, hi), dr, ir, kl_h)
    with tr.phase("gather"):
        packed = torch.stack([lb.to(torch.int64), cs], dim=1)
        allp = comm.gather_rows(packed, qc, (2,), torch.int64)
        dd = ii = None
        if debug:
            dd = comm.gather_rows(dr, qc, (kmax,), torch.float64)
            ii = comm.gather_rows(ir, qc, (kmax,), torch.int32)
    if not comm.is_root:
        return None
    return allp[:, 0].to(torch.int32), allp[:, 1].contiguous(), dd, ii


FUNCS = {"farm": farm, "shard_gather": shard_gather, "shard_reduce": shard_reduce,
         "grid2d": grid2d, "serial": serial, "ring": ring}
