"""DataParallel: bucketed gradient all-reduce overlapped with backward.

Parity: python/paddle/distributed/parallel.py (DataParallel) +
paddle/fluid/distributed/collective/reducer.cc (EagerReducer: buckets, hooks,
FinalizeBackward).

MI355X design: gradients live in per-bucket flat buffers (``FlatGroup``), so a
bucket is all-reduced IN PLACE by one RCCL call the moment its last gradient is
accumulated (post-accumulate-grad hook) — RCCL runs on its own stream while the
backward keeps computing; one end-of-backward callback makes the compute stream
wait on the outstanding collectives (no host sync). Default bucket 64 MB: large
enough to run xGMI rings near link bandwidth, small enough that the first
bucket launches early in the backward.
"""
import contextlib

import torch
import torch.distributed as dist

from ..framework.core import Tensor
from ..nn.layer.layers import Layer
from .flat import FlatGroup, group_params_into_buckets


def _avg_supported(pg):
    try:
        return dist.get_backend(pg) == 'nccl'
    except Exception:
        return False


class GradBucketReducer:
    """Shared by DataParallel (all-reduce) and sharding stage 1 (all-reduce) / 2,3 (reduce-scatter)."""

    def __init__(self, groups, pg, world, mode='allreduce', shard_grads=None):
        self.groups = groups
        self.pg = pg
        self.world = world
        self.mode = mode
        self.shard_grads = shard_grads  # for reduce_scatter: per-group output buffers
        self.avg = _avg_supported(pg)
        self.counts = [0] * len(groups)
        self.launched = [False] * len(groups)
        self.works = []
        self.enabled = True
        self._cb_queued = False
        self._hooks = []
        for gi, g in enumerate(groups):
            for p in g.params:
                if p._t.requires_grad:
                    self._hooks.append(p._t.register_post_accumulate_grad_hook(
                        self._make_hook(gi)))
        self.n_req = [sum(1 for p in g.params if p._t.requires_grad) for g in groups]

    def _make_hook(self, gi):
        def hook(t):
            if not self.enabled:
                return
            if not self._cb_queued:
                self._cb_queued = True
                torch.autograd.Variable._execution_engine.queue_callback(self.finalize)
            self.counts[gi] += 1
            if self.counts[gi] == self.n_req[gi]:
                self._launch(gi)
        return hook

    def _launch(self, gi):
        if self.launched[gi] or self.world == 1:
            self.launched[gi] = True
            return
        g = self.groups[gi]
        op = dist.ReduceOp.AVG if self.avg else dist.ReduceOp.SUM
        if self.mode == 'allreduce':
            w = dist.all_reduce(g.grad_buf, op=op, group=self.pg, async_op=True)
        else:
            w = dist.reduce_scatter_tensor(self.shard_grads[gi], g.grad_buf, op=op, group=self.pg,
                                           async_op=True)
        self.works.append((gi, w))
        self.launched[gi] = True

    def finalize(self):
        for gi in range(len(self.groups)):
            if not self.launched[gi]:
                self._launch(gi)
        for gi, w in self.works:
            w.wait()
            if not self.avg and self.world > 1:
                (self.groups[gi].grad_buf if self.mode == 'allreduce'
                 else self.shard_grads[gi]).div_(self.world)
        if self.world == 1 and self.mode != 'allreduce':
            for gi, g in enumerate(self.groups):
                if self.shard_grads[gi].data_ptr() != g.grad_buf.data_ptr():
                    self.shard_grads[gi].copy_(g.grad_buf)
        self.works.clear()
        self.counts = [0] * len(self.groups)
        self.launched = [False] * len(self.groups)
        self._cb_queued = False

    def remove(self):
        for h in self._hooks:
            h.remove()


class DataParallel(Layer):
    """paddle.DataParallel — one process per GPU, RCCL all-reduce of flat gradient buckets."""

    def __init__(self, layers, strategy=None, comm_buffer_size=64, last_comm_buffer_size=1,
                 find_unused_parameters=False, group=None):
        super().__init__()
        self._layers = layers
        from ..distributed import collective as C
        self._group = group
        self._pg = None if group is None else group.process_group
        self._world = C.get_world_size(group)
        self._groups = []
        self._reducer = None
        self.find_unused_parameters = find_unused_parameters
        params = [p for p in layers.parameters() if not p.stop_gradient]
        if self._world > 1 and params:
            for p in layers.parameters() + [b for b in layers.buffers()]:
                src = group.ranks[0] if group is not None else 0
                dist.broadcast(p._t.data if p._t.requires_grad else p._t, src, group=self._pg)
            buckets = group_params_into_buckets(params, comm_buffer_size * 1024 * 1024)
            self._groups = [FlatGroup(b) for b in buckets]
            self._reducer = GradBucketReducer(self._groups, self._pg, self._world, 'allreduce')

    def forward(self, *inputs, **kwargs):
        for g in self._groups:
            if any(p._t.grad is None for p in g.params if p._t.requires_grad):
                g.grad_buf.zero_()
                g.reattach_grads()
        return self._layers(*inputs, **kwargs)

    @contextlib.contextmanager
    def no_sync(self):
        r = self._reducer
        if r is None:
            yield
            return
        r.enabled = False
        try:
            yield
        finally:
            r.enabled = True

    def scale_loss(self, loss):
        return loss

    def apply_collective_grads(self):
        pass

    def state_dict(self, *a, **k):
        return self._layers.state_dict(*a, **k)

    def set_state_dict(self, *a, **k):
        return self._layers.set_state_dict(*a, **k)

    set_dict = set_state_dict
    load_dict = set_state_dict

    def parameters(self, include_sublayers=True):
        return self._layers.parameters(include_sublayers)

    def named_parameters(self, prefix='', include_sublayers=True):
        return self._layers.named_parameters(prefix, include_sublayers)
