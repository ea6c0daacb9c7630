"""Flat parameter/gradient storage — the memory layout every MI355X parallel mode shares.

A ``FlatGroup`` owns one contiguous HBM buffer for a list of same-dtype
parameters (padded to a multiple of ``align * world``) and one for their
gradients. Each ``Parameter`` is re-pointed to a leaf view of the flat param
buffer and gets a pre-set ``.grad`` view of the flat grad buffer, so autograd
accumulates in place and every collective (all-reduce, reduce-scatter,
all-gather) runs on ONE large contiguous slab per bucket — no pack/unpack
copies, few large RCCL calls (xGMI ring collectives are per-link bandwidth bound
and small messages are latency bound; 288 GB HBM makes the padding free).

Parity: the reference's fused-buffer storage
python/paddle/distributed/fleet/meta_parallel/sharding/group_sharded_storage.py
(ParamStorage/GradStorage) and the C++ Reducer buckets
(paddle/fluid/distributed/collective/reducer.cc).
"""
import torch

from ..framework.core import Parameter


def _round_up(n, m):
    return (n + m - 1) // m * m


class FlatGroup:
    def __init__(self, params, world=1, rank=0, align=128, grad_dtype=None):
        assert params, "empty FlatGroup"
        self.params = list(params)
        t0 = self.params[0]._t
        self.dtype = t0.dtype
        self.device = t0.device
        assert all(p._t.dtype == self.dtype for p in self.params), "FlatGroup needs one dtype"
        self.world, self.rank = world, rank
        self.offsets = []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            off += _round_up(p._t.numel(), align)
        self.numel = _round_up(max(off, 1), align * world)
        self.shard_numel = self.numel // world
        self.param_buf = torch.zeros(self.numel, dtype=self.dtype, device=self.device)
        self.grad_dtype = grad_dtype or self.dtype
        self.grad_buf = torch.zeros(self.numel, dtype=self.grad_dtype, device=self.device)
        with torch.no_grad():
            for p, o in zip(self.params, self.offsets):
                n = p._t.numel()
                self.param_buf[o:o + n].copy_(p._t.detach().reshape(-1))
        self.attach()

    # -- views -------------------------------------------------------------------------
    def attach(self):
        """(Re)point every param to its slice of the flat buffers."""
        for p, o in zip(self.params, self.offsets):
            shape = p._t.shape
            n = p._t.numel()
            rg = not p.stop_gradient
            v = self.param_buf[o:o + n].view(shape)
            leaf = v.detach()
            if rg:
                leaf.requires_grad_(True)
                leaf.grad = self.grad_buf[o:o + n].view(shape)
            object.__setattr__(p, '_t', leaf)

    def reattach_grads(self):
        for p, o in zip(self.params, self.offsets):
            t = p._t
            if t.requires_grad and (t.grad is None or t.grad.data_ptr() != self.grad_buf[o:].data_ptr()):
                n = t.numel()
                t.grad = self.grad_buf[o:o + n].view(t.shape)

    # -- shards ------------------------------------------------------------------------
    def shard(self, buf, rank=None):
        r = self.rank if rank is None else rank
        return buf[r * self.shard_numel:(r + 1) * self.shard_numel]

    @property
    def param_shard(self):
        return self.shard(self.param_buf)

    def params_in_shard(self, rank=None):
        """[(param, local_lo, local_hi, param_lo)] overlaps of params with a rank's shard."""
        r = self.rank if rank is None else rank
        lo, hi = r * self.shard_numel, (r + 1) * self.shard_numel
        out = []
        for p, o in zip(self.params, self.offsets):
            n = p._t.numel()
            a, b = max(o, lo), min(o + n, hi)
            if a < b:
                out.append((p, a - lo, b - lo, a - o))
        return out


def group_params_into_buckets(params, bucket_bytes, reverse=True):
    """Split params (same-dtype runs) into buckets of ~bucket_bytes, in backward order."""
    ps = list(reversed(params)) if reverse else list(params)
    buckets, cur, cur_b, cur_dt = [], [], 0, None
    for p in ps:
        nb = p._t.numel() * p._t.element_size()
        if cur and (p._t.dtype != cur_dt or cur_b + nb > bucket_bytes):
            buckets.append(cur)
            cur, cur_b = [], 0
        cur.append(p)
        cur_b += nb
        cur_dt = p._t.dtype
    if cur:
        buckets.append(cur)
    return buckets
