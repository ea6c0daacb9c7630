"""DistributedFusedLamb: LAMB with gradients reduce-scattered into 1/nranks shards and the
moments + fp32 master weights sharded (parity: python/paddle/incubate/optimizer/
distributed_fused_lamb.py; paddle/fluid/operators/optimizers/distributed_fused_lamb_op.cu:922-1000
reduce-scatter, :1595-1641 sharded state).

MI355X design:
* parameters and gradients live in FlatGroup buffers (parallel/flat.py): each parameter is a view
  of one flat slab and its ``.grad`` a view of the flat gradient slab, so autograd accumulates in
  place and nothing is packed per step;
* the reduce-scatter of each slab is launched from the backward itself (GradBucketReducer
  post-accumulate hooks) as soon as the slab's gradients are complete, on RCCL's stream;
* each rank keeps m, v and the fp32 master copy of ITS shard only (1/nranks of the state);
* the update is two HIP launches per slab on the contiguous shard (ops/csrc/lamb.hip): moments,
  r = m^/(sqrt(v^)+eps) + wd*w and per-parameter partial ||w||^2, ||r||^2; one all-reduce of the
  [2][P] partials; then w -= lr * (||w|| / ||r||) * r, written straight into the parameter-dtype
  shard that the all-gather distributes back into every rank's parameter slab;
* the global-norm clip (after the reduce-scatter by default) is one scalar all-reduce of the
  shards' sums of squares; its coefficient is read on the device by the stage-1 kernel;
* gradient accumulation keeps accumulating into the flat gradient slab; only the last micro-step's
  backward communicates.
"""
import torch
import torch.distributed as dist

from ...framework.core import Tensor, _u
from ...optimizer.optimizer import Optimizer

_PIECE = 8192   # elements per kernel block (a piece never crosses a parameter boundary)


class _Shard:
    """One FlatGroup's sharded LAMB state."""

    def __init__(self, group, wds, device):
        self.group = group
        self.n = group.shard_numel
        lo = group.rank * self.n
        self.master = group.param_buf[lo:lo + self.n].detach().float().clone()
        self.m = torch.zeros(self.n, dtype=torch.float32, device=device)
        self.v = torch.zeros_like(self.m)
        self.r = torch.empty_like(self.m)
        self.pshard = group.param_buf[lo:lo + self.n].detach().clone()
        self.grad_shard = torch.zeros(self.n, dtype=group.grad_dtype, device=device)
        self.P = len(group.params)
        self.norms = torch.zeros(2 * self.P, dtype=torch.float32, device=device)
        self.wd = torch.tensor(wds, dtype=torch.float32, device=device)
        idx = {id(p): i for i, p in enumerate(group.params)}
        pieces = []
        for p, a, b, _ in group.params_in_shard():
            for s in range(a, b, _PIECE):
                pieces.append((idx[id(p)], s, min(s + _PIECE, b)))
        self.pieces_list = pieces
        self.pieces = torch.tensor(pieces if pieces else [(0, 0, 0)], dtype=torch.int64, device=device)
        self.npieces = len(pieces)


class DistributedFusedLamb(Optimizer):
    def __init__(self, learning_rate=0.001, lamb_weight_decay=0.01, beta1=0.9, beta2=0.999,
                 epsilon=1e-6, parameters=None, grad_clip=None,
                 exclude_from_weight_decay_fn=None, clip_after_allreduce=True,
                 is_grad_scaled_by_nranks=True, alignment=128, use_master_param_norm=True,
                 gradient_accumulation_steps=1, use_master_acc_grad=True, nproc_per_node=None,
                 use_hierarchical_allreduce=False, name=None):
        super().__init__(learning_rate, parameters, None, None, name, True)
        self._wd, self._beta1, self._beta2, self._epsilon = lamb_weight_decay, beta1, beta2, epsilon
        self._exclude = exclude_from_weight_decay_fn
        self._dfl_clip = grad_clip
        self._clip_after_allreduce = clip_after_allreduce
        self._is_grad_scaled_by_nranks = is_grad_scaled_by_nranks
        self._alignment = max(1, int(alignment))
        self._acc_steps = max(1, int(gradient_accumulation_steps))
        self._acc_count = 0
        self._built = False
        self._shards = []
        self._reducer = None
        if self._parameter_list:
            self._build()

    # -- layout --------------------------------------------------------------------------------------
    def _world(self):
        if dist.is_available() and dist.is_initialized():
            return dist.get_world_size(), dist.get_rank()
        return 1, 0

    def _build(self):
        from ...parallel.flat import FlatGroup, group_params_into_buckets
        from ...parallel.data_parallel import GradBucketReducer
        params = [p for p in self._parameter_list if not p.stop_gradient]
        world, rank = self._world()
        self._world_size = world
        buckets = group_params_into_buckets(params, 256 << 20, reverse=True)
        self._groups = [FlatGroup(b, world=world, rank=rank, align=self._alignment) for b in buckets]
        dev = self._groups[0].device if self._groups else torch.device('cpu')
        self._shards = []
        for g in self._groups:
            wds = [0.0 if (self._exclude is not None and self._exclude(p)) else float(self._wd) for p in g.params]
            self._shards.append(_Shard(g, wds, dev))
        pg = dist.group.WORLD if world > 1 else None
        # the reduce-scatter of each slab starts inside the backward (disabled on accumulation
        # micro-steps and when the clip must see the local gradients first)
        self._reducer = GradBucketReducer(self._groups, pg, world, mode='reduce_scatter',
                                          shard_grads=[s.grad_shard for s in self._shards],
                                          name='dist_fused_lamb')
        self._reducer.enabled = self._comm_in_backward()
        self._last_finalize = self._reducer.finalize_count
        self._built = True

    def _comm_in_backward(self):
        return self._clip_after_allreduce and (self._acc_count == self._acc_steps - 1)

    def state_bytes(self):
        """Bytes of optimizer state this rank holds (moments + fp32 masters of its shards)."""
        return sum(s.m.numel() * 4 * 3 for s in self._shards)

    # -- the step ------------------------------------------------------------------------------------------
    def clear_grad(self, set_to_zero=True):
        if self._acc_count != 0:
            return          # gradient-accumulation micro-step: keep accumulating in the flat slabs
        from ...ops.fused import zero_tensors
        zero_tensors([g.grad_buf for g in self._groups])

    @torch.no_grad()
    def step(self):
        if not self._built:
            self._build()
        self._acc_count += 1
        if self._acc_count < self._acc_steps:
            self._reducer.enabled = self._comm_in_backward()
            return
        self._acc_count = 0
        world = self._world_size
        gscale = 1.0 / self._acc_steps
        if not self._clip_after_allreduce and self._dfl_clip is not None:
            # clip the LOCAL gradients before they are reduced
            sq = sum(g.grad_buf.float().pow(2).sum() for g in self._groups)
            coef = self._clip_coefficient(sq * (gscale * gscale))
            for g in self._groups:
                g.grad_buf.mul_(coef.to(g.grad_buf.dtype))
        if not self._reducer.enabled:
            for s in self._shards:       # communication not launched from the backward
                if world > 1:
                    dist.reduce_scatter_tensor(s.grad_shard, s.group.grad_buf)
                else:
                    s.grad_shard.copy_(s.group.grad_buf)
            if world > 1:
                for s in self._shards:
                    s.grad_shard.div_(world)
        elif self._reducer.finalize_count == self._last_finalize:
            self._reducer.finalize()      # (no hook fired in this backward: launch + wait here)
        if world > 1 and not self._is_grad_scaled_by_nranks:
            gscale *= world           # the reducer averaged; the caller wants the plain sum
        coef_t = None
        if self._clip_after_allreduce and self._dfl_clip is not None:
            sq = sum(s.grad_shard.float().pow(2).sum() for s in self._shards) * (gscale * gscale)
            if world > 1:
                dist.all_reduce(sq)
            coef_t = self._clip_coefficient(sq).reshape(1).float()
        self._step_count += 1
        t = self._step_count
        bc1, bc2 = 1 - self._beta1 ** t, 1 - self._beta2 ** t
        lr = float(self.get_lr())
        for s in self._shards:
            s.norms.zero_()
            self._stage1(s, gscale, coef_t, bc1, bc2)
            if world > 1:
                dist.all_reduce(s.norms)
            self._stage2(s, lr)
            if world > 1:
                dist.all_gather_into_tensor(s.group.param_buf, s.pshard)
            else:
                s.group.param_buf.copy_(s.pshard)
        self._reducer.reset_accumulation()
        self._reducer.enabled = self._comm_in_backward()
        self._last_finalize = self._reducer.finalize_count

    def _clip_coefficient(self, sq):
        clip_norm = float(getattr(self._dfl_clip, 'clip_norm', 1.0))
        norm = sq.sqrt()
        return clip_norm / torch.maximum(norm, torch.full_like(norm, clip_norm))

    def _hip(self, s):
        if not s.m.is_cuda:
            return None
        from ...ops import _native
        return _native.lib() if _native.available() else _native.require()

    def _stage1(self, s, gscale, coef_t, bc1, bc2):
        L = self._hip(s)
        g = s.grad_shard
        if L is not None:
            from ...ops.fused import _dt, _stream
            L.lamb_shard_stage1(s.pieces.data_ptr(), s.npieces, g.data_ptr(), _dt(g), s.master.data_ptr(),
                                s.m.data_ptr(), s.v.data_ptr(), s.r.data_ptr(), s.wd.data_ptr(), s.norms.data_ptr(),
                                s.P, self._beta1, self._beta2, self._epsilon, bc1, bc2, gscale,
                                coef_t.data_ptr() if coef_t is not None else 0, _stream())
            return
        lamb_stage1_ref(s.pieces_list, g, s.master, s.m, s.v, s.r, s.wd, s.norms, s.P, self._beta1, self._beta2,
                        self._epsilon, bc1, bc2, gscale * (float(coef_t) if coef_t is not None else 1.0))

    def _stage2(self, s, lr):
        L = self._hip(s)
        if L is not None:
            from ...ops.fused import _dt, _stream
            L.lamb_shard_stage2(s.pieces.data_ptr(), s.npieces, s.master.data_ptr(), s.r.data_ptr(),
                                s.norms.data_ptr(), s.P, lr, s.pshard.data_ptr(), _dt(s.pshard), _stream())
            # padding between parameters (and past the last one) keeps the old values
            return
        lamb_stage2_ref(s.pieces_list, s.master, s.r, s.norms, s.P, lr, s.pshard)

    # -- checkpoint ------------------------------------------------------------------------------------------
    def _gather(self, shard):
        world = self._world_size
        if world == 1:
            return shard
        out = torch.empty(shard.numel() * world, dtype=shard.dtype, device=shard.device)
        dist.all_gather_into_tensor(out, shard)
        return out

    def state_dict(self):
        """Per-parameter moments and master weights in the reference's naming (every rank
        gathers the shards: collective)."""
        sd = {}
        masters = {}
        for s in self._shards:
            fm, fv, fw = self._gather(s.m), self._gather(s.v), self._gather(s.master)
            for p, o, n, shape in zip(s.group.params, s.group.offsets, s.group.numels, s.group.shapes):
                sd[f'{p.name}_moment1_0'] = Tensor(fm[o:o + n].view(shape).clone())
                sd[f'{p.name}_moment2_0'] = Tensor(fv[o:o + n].view(shape).clone())
                masters[p.name] = Tensor(fw[o:o + n].view(shape).clone())
        sd['master_weights'] = masters
        sd['step'] = self._step_count
        return sd

    def set_state_dict(self, sd):
        if not self._built:
            self._build()
        masters = sd.get('master_weights', {})
        for s in self._shards:
            lo, hi = s.group.rank * s.n, (s.group.rank + 1) * s.n
            for p, o, n in zip(s.group.params, s.group.offsets, s.group.numels):
                a, b = max(o, lo), min(o + n, hi)
                if a >= b:
                    continue
                for key, dst in ((f'{p.name}_moment1_0', s.m), (f'{p.name}_moment2_0', s.v)):
                    if key in sd:
                        dst[a - lo:b - lo].copy_(_u(sd[key]).reshape(-1)[a - o:b - o].float())
                if p.name in masters:
                    s.master[a - lo:b - lo].copy_(_u(masters[p.name]).reshape(-1)[a - o:b - o].float())
        self._step_count = int(sd.get('step', self._step_count))


def lamb_stage1_ref(pieces, g, w, m, v, r, wd, norms, P, b1, b2, eps, bc1, bc2, gscale):
    """fp32 reference of the stage-1 kernel (host path and tests)."""
    for p, lo, hi in pieces:
        gi = g[lo:hi].float() * gscale
        m[lo:hi] = b1 * m[lo:hi] + (1 - b1) * gi
        v[lo:hi] = b2 * v[lo:hi] + (1 - b2) * gi * gi
        ri = (m[lo:hi] / bc1) / ((v[lo:hi] / bc2).sqrt() + eps) + wd[p] * w[lo:hi]
        r[lo:hi] = ri
        norms[p] += w[lo:hi].pow(2).sum()
        norms[P + p] += ri.pow(2).sum()


def lamb_stage2_ref(pieces, w, r, norms, P, lr, pout):
    for p, lo, hi in pieces:
        wn, rn = norms[p].sqrt(), norms[P + p].sqrt()
        trust = (wn / rn) if (wn > 0 and rn > 0) else torch.ones((), dtype=torch.float32, device=w.device)
        w[lo:hi] -= lr * trust * r[lo:hi]
        if pout is not None:
            pout[lo:hi] = w[lo:hi].to(pout.dtype)
