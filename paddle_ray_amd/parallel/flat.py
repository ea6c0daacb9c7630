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
        self.shapes = [tuple(p._t.shape) for p in self.params]
        self.numels = [p._t.numel() for p in self.params]
        off = 0
        for n in self.numels:
            self.offsets.append(off)
            off += _round_up(n, align)
        self.numel = _round_up(max(off, 1), align * world)
        self.shard_numel = self.numel // world
        self.param_buf = torch.zeros(self.numel, dtype=self.dtype, device=self.device)
        self.grad_dtype = grad_dtype or self.dtype
        self.grad_buf = torch.zeros(self.numel, dtype=self.grad_dtype, device=self.device)
        with torch.no_grad():
            for p, o in zip(self.params, self.offsets):
                n = p._t.numel()
                self.param_buf[o:o + n].copy_(p._t.detach().reshape(-1))
        self._shard_store = None
        self.params_released = False
        self.grads_released = False
        self.leaves = []
        self.attach()

    # -- views -------------------------------------------------------------------------
    def attach(self):
        """(Re)point every param to its slice of the flat buffers.

        Each leaf is built with ``set_`` on the flat storage instead of as a view, so it has
        its own autograd version counter: collectives writing into ``param_buf`` (the ZeRO-3
        re-gather in the middle of backward) do not invalidate tensors saved for backward."""
        self.leaves = []
        st = self.param_buf.untyped_storage()
        for p, o, shape, n in zip(self.params, self.offsets, self.shapes, self.numels):
            rg = not p.stop_gradient
            leaf = torch.empty(0, dtype=self.dtype, device=self.device)
            leaf.set_(st, o, shape, torch.empty(shape, device='meta').stride())
            if rg:
                leaf.requires_grad_(True)
                leaf.grad = self.grad_buf[o:o + n].view(shape)
            object.__setattr__(p, '_t', leaf)
            self.leaves.append(leaf)

    def reattach_grads(self):
        if self.grads_released:
            return
        for t, o in zip(self.leaves, self.offsets):
            if t.requires_grad and (t.grad is None or t.grad.data_ptr() != self.grad_buf[o:].data_ptr()):
                n = t.numel()
                t.grad = self.grad_buf[o:o + n].view(t.shape)

    def grads_missing(self):
        return any(t.grad is None for t in self.leaves if t.requires_grad)

    # -- ZeRO-3 residency (parity: group_sharded_stage3.py _release_param / _allgather_buffer) --
    def own_shard(self):
        """Move the owned parameter shard into its own storage so the full buffer can be freed."""
        if self._shard_store is None:
            self._shard_store = self.shard(self.param_buf).clone()

    def release_params(self):
        """Free the gathered full buffer. Parameters point at an empty placeholder (a use while
        released fails with a shape error on the host, never a device fault); tensors autograd
        saved keep the storage object and see the data again after ``materialize_params``."""
        if self.params_released:
            return
        assert self._shard_store is not None, "release_params needs own_shard() first"
        for p in self.params:
            object.__setattr__(p, '_t', torch.empty(0, dtype=self.dtype, device=self.device))
        self.param_buf.untyped_storage().resize_(0)
        self.params_released = True

    def materialize_params(self):
        """Re-allocate the full buffer (contents undefined until gathered); re-point params."""
        if not self.params_released:
            return
        self.param_buf.untyped_storage().resize_(self.numel * self.param_buf.element_size())
        for p, leaf in zip(self.params, self.leaves):
            object.__setattr__(p, '_t', leaf)
        self.params_released = False

    def release_grads(self):
        if not self.grads_released:
            self.grad_buf.untyped_storage().resize_(0)
            self.grads_released = True

    def materialize_grads(self):
        if self.grads_released:
            self.grad_buf.untyped_storage().resize_(self.numel * self.grad_buf.element_size())
            self.grad_buf.zero_()
            self.grads_released = False

    def resident_bytes(self):
        return self.param_buf.untyped_storage().nbytes() + self.grad_buf.untyped_storage().nbytes()

    # -- shards ------------------------------------------------------------------------
    def shard(self, buf, rank=None):
        r = self.rank if rank is None else rank
        return buf[r * self.shard_numel:(r + 1) * self.shard_numel]

    @property
    def param_shard(self):
        if self._shard_store is not None:
            return self._shard_store
        return self.shard(self.param_buf)

    def params_in_shard(self, rank=None):
        """[(param, local_lo, local_hi, param_lo)] overlaps of params with a rank's shard."""
        r = self.rank if rank is None else rank
        lo, hi = r * self.shard_numel, (r + 1) * self.shard_numel
        out = []
        for p, o, n in zip(self.params, self.offsets, self.numels):
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
