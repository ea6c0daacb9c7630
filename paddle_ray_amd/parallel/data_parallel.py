"""DataParallel: bucketed gradient all-reduce overlapped with backward.

Parity: python/paddle/distributed/parallel.py (DataParallel) +
paddle/fluid/distributed/collective/reducer.cc (EagerReducer: buckets, hooks,
FinalizeBackward).

MI355X design: gradients live in per-bucket flat buffers (``FlatGroup``), so a
bucket is all-reduced IN PLACE by one RCCL call the moment its last gradient is
accumulated (post-accumulate-grad hook) — RCCL runs on its own stream while the
backward keeps computing; one end-of-backward callback makes the compute stream
wait on the outstanding collectives (no host sync).

Bucket size (default 64 MB; the reference's EagerReducer uses 25 MB, written for NVLink
switches). The basis on an 8 x MI355X node, where every GPU reaches the other seven through
its own point-to-point xGMI link (7 x ~64 GB/s per direction) and RCCL runs one ring per
channel over those links, is a latency / bandwidth split of one ring all-reduce:

    t(B) = a + 2 (n-1)/n * B / BW_bus,   a ~= 25-40 us launch + ring pipeline fill,
                                          BW_bus ~= 250-350 GB/s (all 7 links busy)

* fixed-cost share a / t(B) at n = 8: 25 MB -> ~15-25 %, 64 MB -> ~7-11 %, 256 MB -> ~2-3 %:
  below ~32 MB the per-call cost is a visible fraction of the link time;
* the LAST bucket of the backward cannot overlap compute: its t(B) is exposed once per step
  (64 MB: ~0.35-0.45 ms; 256 MB: ~1.4-1.8 ms), and the FIRST bucket should launch early;
  a GPT-1.3B block's gradients are 100 MB bf16 (~4 ms of backward compute), so a 64 MB
  bucket launches within the first block's backward and every later bucket hides under the
  following blocks' compute (about 0.4 ms of link time per ~2.5 ms of compute).
64 MB keeps the per-call share under ~10 % and the exposed tail under half a millisecond.
ZeRO-2/3 reduce-scatters use one bucket per unit (a repeated block, 100 MB here) and 128 MB
for the resident remainder (``group_sharded_parallel(bucket_mb=128)``): a reduce-scatter
moves (n-1)/n * B per rank -- half the all-reduce bytes -- so the same call-overhead share
needs twice the bucket. These are derived numbers (no 8-GPU node in this build's test pool);
``fuse_grad_size_in_MB`` / ``bucket_mb`` override them.
"""
import contextlib

import torch
import torch.distributed as dist

from ..framework.core import Tensor
from ..nn.layer.layers import Layer
from .flat import FlatGroup, group_params_into_buckets
from ..distributed import watchdog as _watchdog


def _avg_supported(pg):
    try:
        return dist.get_backend(pg) == 'nccl'
    except Exception:
        return False


class GradBucketReducer:
    """Shared by DataParallel (all-reduce) and sharding stage 1 (all-reduce) / 2,3 (reduce-scatter).

    ``dp_pg``: in hybrid dp x sharding, the owned (already sharding-reduced) gradient shard
    is then averaged over the data-parallel group. On RCCL that all-reduce is issued per bucket
    as soon as the bucket's reduce-scatter is launched, from a side HIP stream that waits on the
    reduce-scatter's completion event, so the dp traffic overlaps the rest of the backward (the
    compute stream never waits for it until ``finalize``). ``on_launch(gi)`` / ``on_finalize()``
    let ZeRO-3 free a bucket's gathered parameters as soon as its gradients are complete.
    ``accumulate``: several backward passes before one optimizer step ADD into the shard
    gradients (ZeRO-3 frees and re-zeroes the full gradient buffer after every backward, so the
    reduce-scatter of pass k > 1 lands in a scratch shard that is then added; parity:
    group_sharded_stage3.py:675-694 adding into ``param.bw_storage``). ``reset_accumulation``
    (called from ``clear_grad``) makes the next pass write the shard directly again.
    Every RCCL work is registered with the collective watchdog until it is waited on.
    """

    def __init__(self, groups, pg, world, mode='allreduce', shard_grads=None, dp_pg=None,
                 dp_world=1, on_launch=None, on_finalize=None, name='dp_bucket',
                 accumulate=False):
        self.groups = groups
        self.pg = pg
        self.world = world
        self.mode = mode
        self.shard_grads = shard_grads  # for reduce_scatter: per-group output buffers
        self.avg = _avg_supported(pg)
        self.dp_pg, self.dp_world = dp_pg, dp_world
        self.dp_avg = _avg_supported(dp_pg) if dp_pg is not None else False
        self.on_launch, self.on_finalize = on_launch, on_finalize
        self.name = name
        self.accumulate = accumulate and mode != 'allreduce'
        self.fresh = [True] * len(groups)   # shard_grads[gi] holds nothing of this step yet
        self._scratch = [None] * len(groups)
        self.counts = [0] * len(groups)
        self.launched = [False] * len(groups)
        self.works = []
        self.dp_works = []
        self._side = None
        self.enabled = True
        self.auto_finalize = True  # finalize at the end of the backward that first fires a hook
        self._cb_queued = False
        self.finalize_count = 0
        self._hooks = []
        for gi, g in enumerate(groups):
            for t in g.leaves:
                if t.requires_grad:
                    self._hooks.append(t.register_post_accumulate_grad_hook(self._make_hook(gi)))
        self.n_req = [sum(1 for t in g.leaves if t.requires_grad) for g in groups]

    def _make_hook(self, gi):
        def hook(t):
            if not self.enabled:
                return
            if not self._cb_queued and self.auto_finalize:
                self._cb_queued = True
                from .recompute import queue_outer_callback
                queue_outer_callback(self.finalize)
            self.counts[gi] += 1
            if self.counts[gi] == self.n_req[gi]:
                self._launch(gi)
        return hook

    def reset_accumulation(self):
        self.fresh = [True] * len(self.groups)

    def _rs_target(self, gi):
        """Where this pass's reduce-scatter of bucket gi lands: the shard itself on the first
        pass of a step, else a scratch shard added at finalize."""
        if not self.accumulate or self.fresh[gi]:
            return self.shard_grads[gi]
        if self._scratch[gi] is None:
            self._scratch[gi] = torch.empty_like(self.shard_grads[gi])
        return self._scratch[gi]

    def _dp_overlap(self):
        return (self.dp_pg is not None and self.dp_world > 1 and self.world > 1 and
                torch.cuda.is_available() and _avg_supported(self.dp_pg) and self.avg)

    def _launch(self, gi):
        if self.launched[gi]:
            return
        self.launched[gi] = True
        if self.world > 1:
            g = self.groups[gi]
            op = dist.ReduceOp.AVG if self.avg else dist.ReduceOp.SUM
            if self.mode == 'allreduce':
                out = g.grad_buf
                w = dist.all_reduce(out, op=op, group=self.pg, async_op=True)
            else:
                out = self._rs_target(gi)
                w = dist.reduce_scatter_tensor(out, g.grad_buf, op=op, group=self.pg,
                                               async_op=True)
            w = _watchdog.track(f'{self.name}.{self.mode}[{gi}]', w, self.world)
            self.works.append((gi, w))
            if self._dp_overlap():
                # the side stream waits for this bucket's reduce-scatter, then the dp all-reduce
                # of the shard runs on the dp communicator's stream: the compute stream is free
                if self._side is None:
                    self._side = torch.cuda.Stream()
                self._side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(self._side):
                    w.wait()
                    w2 = dist.all_reduce(out, op=dist.ReduceOp.AVG, group=self.dp_pg,
                                         async_op=True)
                self.dp_works.append((gi, _watchdog.track(
                    f'{self.name}.dp_allreduce[{gi}]', w2, self.dp_world)))
        if self.on_launch is not None:
            self.on_launch(gi)

    def _shard_out(self, gi):
        return self.groups[gi].grad_buf if self.mode == 'allreduce' else self._rs_target(gi)

    def finalize(self):
        for gi in range(len(self.groups)):
            if not self.launched[gi]:
                self._launch(gi)
        for gi, w in self.works:
            w.wait()
            if not self.avg and self.world > 1:
                self._shard_out(gi).div_(self.world)
        if self.world == 1 and self.mode != 'allreduce':
            for gi, g in enumerate(self.groups):
                dst = self._rs_target(gi)
                if dst.data_ptr() != g.grad_buf.data_ptr():
                    dst.copy_(g.shard(g.grad_buf))
        if self.dp_pg is not None and self.dp_world > 1:
            if self.dp_works:  # issued during the backward (RCCL): only wait here
                for gi, w in self.dp_works:
                    w.wait()
            else:
                # hybrid dp x sharding: average the owned shard over the replicas
                op = dist.ReduceOp.AVG if self.dp_avg else dist.ReduceOp.SUM
                dws = []
                for gi, g in enumerate(self.groups):
                    out = self._shard_out(gi) if self.shard_grads is not None else g.grad_buf
                    dws.append((out, _watchdog.track(f'{self.name}.dp_allreduce[{gi}]', dist.all_reduce(
                        out, op=op, group=self.dp_pg, async_op=True), self.dp_world)))
                for out, w in dws:
                    w.wait()
                    if not self.dp_avg:
                        out.div_(self.dp_world)
        if self.accumulate:
            for gi in range(len(self.groups)):
                if not self.fresh[gi]:
                    self.shard_grads[gi].add_(self._scratch[gi])
                self.fresh[gi] = False
        self.works.clear()
        self.dp_works.clear()
        self.counts = [0] * len(self.groups)
        self.launched = [False] * len(self.groups)
        self._cb_queued = False
        self.finalize_count += 1
        if self.on_finalize is not None:
            self.on_finalize()

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
            if g.grads_missing():
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
