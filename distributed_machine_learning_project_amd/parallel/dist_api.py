"""torch.distributed facade used by every collective call site (comm.py, strategies.py, shm.py).

With an RCCL process group (the MI355X data plane) or gloo on CPU tensors every call goes
straight to torch.distributed.  With a gloo group and CUDA tensors — the host-staged data plane
(``DMLP_DATA_PLANE=host``, parallel/comm.py) that lets several ranks share ONE GPU in tests,
which RCCL cannot — each call stages its device tensors through host memory: device -> host
copy, the gloo collective on the host copies, host -> device copy into the caller's tensors.
Same semantics, same call sequence, so the multi-rank GPU code (offsets, merge kernel, tree,
ring) runs unchanged on real HIP kernels.
"""
from __future__ import annotations

import hashlib
import os

import torch
import torch.distributed as _d

ReduceOp = _d.ReduceOp
P2POp = _d.P2POp
isend = _d.isend
irecv = _d.irecv
is_initialized = _d.is_initialized
get_rank = _d.get_rank
get_world_size = _d.get_world_size
get_backend = _d.get_backend
destroy_process_group = _d.destroy_process_group
broadcast_object_list = _d.broadcast_object_list


# ---------------------------------------------------------------- collective-sequence log
# The Python twin of knn_engine's KNN_P2P_CHECK (csrc/engine_core.h): every call below appends
# (op, group members, bytes, dtype, peer) to a per-process list while logging is on
# (DMLP_COLL_CHECK=1 or coll_log_start()).  check_collective_sequence() then compares the lists
# of all ranks on rank 0: every collective must be entered by every member of its group with
# the same bytes in the same order, and every send must meet a receive of the same size — a
# rank-divergent sequence that would HANG at P = 8 fails here with the first mismatch instead.
_LOG = None if os.environ.get("DMLP_COLL_CHECK", "0") in ("", "0") else []


def coll_log_start():
    global _LOG
    _LOG = []


def coll_log_stop():
    global _LOG
    out, _LOG = _LOG, None
    return out or []


def coll_log():
    return list(_LOG or [])


# sub-groups by creation order: dist.new_group is collective (every rank creates every group in
# the same order), so the index is the same on every rank, unlike id(group)
_GROUPS = {}


def new_group(ranks=None, **kw):
    g = _d.new_group(ranks, **kw)
    _GROUPS[id(g)] = (len(_GROUPS), tuple(ranks) if ranks is not None else None)
    return g


def _members(group):
    if group is None or not _d.is_initialized():
        return None  # the world
    try:
        return tuple(_d.get_process_group_ranks(group))
    except Exception:  # noqa: BLE001 - older torch: no rank listing
        idx, ranks = _GROUPS.get(id(group), (-1, None))
        return ranks if ranks is not None else ("group", idx)


def _rec(op, t, group=None, peer=None, nbytes=None):
    if _LOG is None:
        return
    nb = nbytes if nbytes is not None else (t.numel() * t.element_size() if t is not None else 0)
    dt = str(t.dtype).replace("torch.", "") if t is not None else "-"
    _LOG.append((op, _members(group), int(nb), dt, peer))


def check_collective_sequence(log=None, group=None):
    """Collective: gather every rank's log on rank 0 and compare.  Returns a summary dict on
    rank 0 (``ok``, counts, bytes per rank and op, the first mismatch) and None elsewhere.
    The gather itself is not logged."""
    global _LOG
    mine = coll_log() if log is None else list(log)
    saved, _LOG = _LOG, None
    try:
        world = _d.get_world_size() if _d.is_initialized() else 1
        rank = _d.get_rank() if _d.is_initialized() else 0
        logs = [None] * world
        if world > 1:
            _d.all_gather_object(logs, mine, group=group)
        else:
            logs = [mine]
    finally:
        _LOG = saved
    if rank != 0:
        return None
    return compare_logs(logs)


def compare_logs(logs):
    """Pure comparison of per-rank logs (index = rank)."""
    world = len(logs)
    problems = []
    # collectives: per group, the members' sequences of (op, bytes, dtype) must be identical
    seqs = {}
    for r, lg in enumerate(logs):
        for op, grp, nb, dt, peer in lg:
            if op in ("send", "recv"):
                continue
            members = tuple(range(world)) if grp is None else grp
            seqs.setdefault(members, {}).setdefault(r, []).append((op, nb, dt, peer))
    for members, per in seqs.items():
        ranks = [m for m in members if isinstance(m, int)]
        ref_r = ranks[0] if ranks else min(per)
        ref = per.get(ref_r, [])
        for r in ranks:
            got = per.get(r, [])
            if got != ref:
                n = next((i for i, (x, y) in enumerate(zip(ref, got)) if x != y),
                         min(len(ref), len(got)))
                problems.append({"group": list(members), "rank": r, "ref_rank": ref_r,
                                 "index": n, "ref": list(ref[n]) if n < len(ref) else None,
                                 "got": list(got[n]) if n < len(got) else None,
                                 "ref_len": len(ref), "got_len": len(got)})
                break
    # point to point: for each ordered pair, the sizes sent must equal the sizes received
    sent, recvd = {}, {}
    for r, lg in enumerate(logs):
        for op, grp, nb, dt, peer in lg:
            if op == "send":
                sent.setdefault((r, peer), []).append((nb, dt))
            elif op == "recv":
                recvd.setdefault((peer, r), []).append((nb, dt))
    for pair in sorted(set(sent) | set(recvd), key=str):
        if sent.get(pair, []) != recvd.get(pair, []):
            problems.append({"p2p": list(pair), "sent": sent.get(pair, []),
                             "received": recvd.get(pair, [])})
    by_rank = []
    for lg in logs:
        b = {}
        for op, _, nb, _, _ in lg:
            b[op] = b.get(op, 0) + nb
        by_rank.append(b)
    digest = [hashlib.sha256(repr(lg).encode()).hexdigest()[:12] for lg in logs]
    return {"ok": not problems, "calls_per_rank": [len(lg) for lg in logs],
            "bytes_per_rank": by_rank, "digest_per_rank": digest, "problems": problems[:4]}


def staged(t=None) -> bool:
    """True when `t` (a tensor or None) must travel through host memory."""
    if not _d.is_initialized() or _d.get_backend() != "gloo":
        return False
    return t is None or (isinstance(t, torch.Tensor) and t.is_cuda)


def _host(t):
    return t.detach().to("cpu") if t.is_cuda else t


def barrier(group=None, device_ids=None):
    _rec("barrier", None, group)
    if _d.get_backend(group) == "gloo":
        return _d.barrier(group=group)
    return _d.barrier(group=group, device_ids=device_ids)


def broadcast(t, src, group=None):
    _rec("broadcast", t, group, peer=src)
    if not staged(t):
        return _d.broadcast(t, src, group=group)
    h = _host(t)
    _d.broadcast(h, src, group=group)
    t.copy_(h)


def all_reduce(t, op=ReduceOp.SUM, group=None):
    _rec("all_reduce", t, group)
    if not staged(t):
        return _d.all_reduce(t, op=op, group=group)
    h = _host(t)
    _d.all_reduce(h, op=op, group=group)
    t.copy_(h)


def reduce(t, dst, op=ReduceOp.SUM, group=None):
    _rec("reduce", t, group, peer=dst)
    if not staged(t):
        return _d.reduce(t, dst, op=op, group=group)
    h = _host(t)
    _d.reduce(h, dst, op=op, group=group)
    if _d.get_rank() == dst:
        t.copy_(h)


def gather(t, gather_list=None, dst=0, group=None):
    _rec("gather", t, group, peer=dst)
    if not staged(t):
        return _d.gather(t, gather_list, dst=dst, group=group)
    h = _host(t)
    hl = [torch.empty_like(h) for _ in gather_list] if gather_list is not None else None
    _d.gather(h, hl, dst=dst, group=group)
    if gather_list is not None:
        for g, x in zip(gather_list, hl):
            g.copy_(x)


def scatter(out, scatter_list=None, src=0, group=None):
    _rec("scatter", out, group, peer=src)
    if not staged(out):
        return _d.scatter(out, scatter_list, src=src, group=group)
    h = torch.empty(out.shape, dtype=out.dtype)
    hl = [_host(c) for c in scatter_list] if scatter_list is not None else None
    _d.scatter(h, hl, src=src, group=group)
    out.copy_(h)


def all_gather_into_tensor(out, t, group=None):
    _rec("all_gather", t, group)
    if not staged(t):
        return _d.all_gather_into_tensor(out, t, group=group)
    h = torch.empty(out.shape, dtype=out.dtype)
    _d.all_gather_into_tensor(h, _host(t).contiguous(), group=group)
    out.copy_(h)


def send(t, dst, group=None):
    _rec("send", t, None, peer=dst)
    if not staged(t):
        return _d.send(t, dst, group=group)
    _d.send(_host(t).contiguous(), dst, group=group)


def recv(t, src=None, group=None):
    # logged with the rank the message really came from (src=None receives from any rank: its
    # pair must match the sender's (sender, me) entry)
    if not staged(t):
        r = _d.recv(t, src, group=group)
    else:
        h = torch.empty(t.shape, dtype=t.dtype)
        r = _d.recv(h, src, group=group)
        t.copy_(h)
    _rec("recv", t, None, peer=src if src is not None else r)
    return r


class _StagedReq:
    """A gloo request on a host copy; wait() lands received bytes in the device tensor."""

    def __init__(self, req, dev_t=None, host_t=None):
        self.req, self.dev_t, self.host_t = req, dev_t, host_t

    def wait(self):
        self.req.wait()
        if self.dev_t is not None:
            self.dev_t.copy_(self.host_t)
        return True


def batch_isend_irecv(ops):
    for op in ops:
        _rec("send" if op.op is _d.isend else "recv", op.tensor, None, peer=op.peer)
    if not ops or not staged(ops[0].tensor):
        return _d.batch_isend_irecv(ops)
    reqs = []
    for op in ops:
        if op.op is _d.isend:
            reqs.append(_StagedReq(_d.isend(_host(op.tensor).contiguous(), op.peer,
                                            group=op.group)))
        else:
            h = torch.empty(op.tensor.shape, dtype=op.tensor.dtype)
            reqs.append(_StagedReq(_d.irecv(h, op.peer, group=op.group), op.tensor, h))
    return reqs
