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
new_group = _d.new_group
destroy_process_group = _d.destroy_process_group
broadcast_object_list = _d.broadcast_object_list


def staged(t=None) -> bool:
    """True when `t` (a tensor or None) must travel through host memory."""
    if not _d.is_initialized() or _d.get_backend() != "gloo":
        return False
    return t is None or (isinstance(t, torch.Tensor) and t.is_cuda)


def _host(t):
    return t.detach().to("cpu") if t.is_cuda else t


def barrier(group=None, device_ids=None):
    if _d.get_backend(group) == "gloo":
        return _d.barrier(group=group)
    return _d.barrier(group=group, device_ids=device_ids)


def broadcast(t, src, group=None):
    if not staged(t):
        return _d.broadcast(t, src, group=group)
    h = _host(t)
    _d.broadcast(h, src, group=group)
    t.copy_(h)


def all_reduce(t, op=ReduceOp.SUM, group=None):
    if not staged(t):
        return _d.all_reduce(t, op=op, group=group)
    h = _host(t)
    _d.all_reduce(h, op=op, group=group)
    t.copy_(h)


def reduce(t, dst, op=ReduceOp.SUM, group=None):
    if not staged(t):
        return _d.reduce(t, dst, op=op, group=group)
    h = _host(t)
    _d.reduce(h, dst, op=op, group=group)
    if _d.get_rank() == dst:
        t.copy_(h)


def gather(t, gather_list=None, dst=0, group=None):
    if not staged(t):
        return _d.gather(t, gather_list, dst=dst, group=group)
    h = _host(t)
    hl = [torch.empty_like(h) for _ in gather_list] if gather_list is not None else None
    _d.gather(h, hl, dst=dst, group=group)
    if gather_list is not None:
        for g, x in zip(gather_list, hl):
            g.copy_(x)


def scatter(out, scatter_list=None, src=0, group=None):
    if not staged(out):
        return _d.scatter(out, scatter_list, src=src, group=group)
    h = torch.empty(out.shape, dtype=out.dtype)
    hl = [_host(c) for c in scatter_list] if scatter_list is not None else None
    _d.scatter(h, hl, src=src, group=group)
    out.copy_(h)


def all_gather_into_tensor(out, t, group=None):
    if not staged(t):
        return _d.all_gather_into_tensor(out, t, group=group)
    h = torch.empty(out.shape, dtype=out.dtype)
    _d.all_gather_into_tensor(h, _host(t).contiguous(), group=group)
    out.copy_(h)


def send(t, dst, group=None):
    if not staged(t):
        return _d.send(t, dst, group=group)
    _d.send(_host(t).contiguous(), dst, group=group)


def recv(t, src=None, group=None):
    if not staged(t):
        return _d.recv(t, src, group=group)
    h = torch.empty(t.shape, dtype=t.dtype)
    r = _d.recv(h, src, group=group)
    t.copy_(h)
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
