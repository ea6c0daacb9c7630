"""ZeRO sharding stages 1/2/3 over RCCL (parity:
python/paddle/distributed/sharding/group_sharded.py (group_sharded_parallel,
save_group_sharded_model), python/paddle/distributed/fleet/meta_parallel/sharding/
group_sharded_stage2.py, group_sharded_stage3.py, group_sharded_optimizer_stage2.py,
python/paddle/distributed/fleet/meta_optimizers/dygraph_optimizer/dygraph_sharding_optimizer.py).

One mechanism, three schedules (MI355X-first):
  * parameters of a bucket ("unit", default 128 MB) live in one flat buffer
    (``FlatGroup``); rank r OWNS the r-th contiguous shard of every bucket;
  * optimizer state (fp32 master, Adam moments) exists only for the owned shard;
    ONE fused multi-tensor AdamW launch updates every owned shard piece and
    writes the new bf16 values straight into the owned slice of the flat param
    buffer (the all-gather source, in place);
  * level 'os'    (stage 1): grads all-reduced (full), update own shard, all-gather params after step;
    level 'os_g'  (stage 2): grads reduce-scattered into the owner shard as each bucket completes
                             in backward, update, all-gather params after step;
    level 'p_g_os'(stage 3): as stage 2 but params are kept sharded after the step and all-gathered
                             lazily at the next forward: every bucket's all-gather is issued up front
                             on the RCCL stream and each layer waits only for its own bucket, so the
                             gather overlaps the forward compute. With 288 GB HBM the gathered
                             buffers stay resident through backward (no backward re-gather traffic).
"""
import contextlib
import math

import torch
import torch.distributed as dist

from ..framework.core import Tensor, Parameter, _u
from ..nn.layer.layers import Layer
from ..ops import fused as K
from ..ops import _native
from .data_parallel import GradBucketReducer, _avg_supported
from .flat import FlatGroup, group_params_into_buckets

LEVELS = {'os': 1, 'os_g': 2, 'p_g_os': 3}


class ShardedState:
    """Flat buckets + owned-shard optimizer state for one model."""

    def __init__(self, layer, level, group=None, segment_bytes=128 << 20, grad_fp32=False):
        from ..distributed import collective as C
        self.layer = layer
        self.stage = LEVELS[level] if isinstance(level, str) else int(level)
        self.group = group
        self.pg = None if group is None else group.process_group
        self.world = C.get_world_size(group)
        self.rank = C.get_rank(group)
        params = [p for p in layer.parameters() if not p.stop_gradient]
        if self.world > 1:
            src = group.ranks[0] if group is not None else 0
            for t in [p._t for p in layer.parameters()] + [b._t for b in layer.buffers()]:
                dist.broadcast(t.data, src, group=self.pg)
        buckets = group_params_into_buckets(params, segment_bytes)
        self.groups = [FlatGroup(b, self.world, self.rank) for b in buckets]
        self.shard_grads = [g.shard(g.grad_buf) if self.world == 1 else
                            torch.zeros(g.shard_numel, dtype=g.grad_dtype, device=g.device)
                            for g in self.groups]
        mode = 'allreduce' if self.stage == 1 else 'reduce_scatter'
        self.reducer = GradBucketReducer(self.groups, self.pg, self.world, mode,
                                         self.shard_grads) if self.stage > 1 or self.world > 1 \
            else None
        if self.stage == 1:
            # stage 1 reduces the full grad buffer; the owned slice of it is the shard grad
            self.shard_grads = [g.shard(g.grad_buf) for g in self.groups]
        self.gather_works = {}
        self.params_stale = False
        self._param_bucket = {}
        for gi, g in enumerate(self.groups):
            for p in g.params:
                self._param_bucket[id(p)] = gi
        self._pre_hooks = []
        if self.stage == 3 and self.world > 1:
            for sub in layer.sublayers(include_self=True):
                mine = sorted({self._param_bucket[id(p)] for p in sub._parameters.values()
                               if p is not None and id(p) in self._param_bucket})
                if mine:
                    self._pre_hooks.append(sub.register_forward_pre_hook(self._make_wait(mine)))

    # -- params all-gather -------------------------------------------------------------
    def _make_wait(self, gids):
        def hook(layer, inputs):
            for gi in gids:
                w = self.gather_works.pop(gi, None)
                if w is not None:
                    w.wait()
        return hook

    def launch_gathers(self, order=None):
        if self.world == 1:
            self.params_stale = False
            return
        order = range(len(self.groups) - 1, -1, -1) if order is None else order
        for gi in order:  # buckets are in backward order: gather forward-first buckets first
            g = self.groups[gi]
            self.gather_works[gi] = dist.all_gather_into_tensor(
                g.param_buf, g.param_shard, group=self.pg, async_op=True)
        self.params_stale = False

    def wait_gathers(self):
        for gi in list(self.gather_works):
            self.gather_works.pop(gi).wait()

    def before_forward(self):
        for g in self.groups:
            if any(p._t.grad is None for p in g.params if p._t.requires_grad):
                g.grad_buf.zero_()
                g.reattach_grads()
        if self.params_stale:
            self.launch_gathers()
            if self.stage != 3:
                self.wait_gathers()

    def after_step(self):
        self.params_stale = True
        if self.stage in (1, 2):
            self.launch_gathers()
            self.wait_gathers()

    def sync_params(self):
        if self.params_stale:
            self.launch_gathers()
        self.wait_gathers()

    def zero_grad(self):
        for g in self.groups:
            g.grad_buf.zero_()
            g.reattach_grads()
        if self.stage > 1 and self.world > 1:
            for s in self.shard_grads:
                s.zero_()


class ShardedOptimizer:
    """Owned-shard optimizer driving the fused multi-tensor HIP kernel.

    Hyper-parameters (lr / scheduler, betas, eps, weight decay incl.
    apply_decay_param_fun, grad_clip) are taken from the user's optimizer.
    """

    def __init__(self, optimizer, state: ShardedState):
        self._inner = optimizer
        self.state = state
        self._kind = type(optimizer).__name__
        if self._kind not in ('Adam', 'AdamW', 'Momentum', 'SGD'):
            raise NotImplementedError(f"sharding does not support {self._kind} yet")
        self._pieces = []
        self._masters, self._m, self._v = [], [], []
        for gi, g in enumerate(state.groups):
            shard = g.param_shard
            master = shard.detach().float().clone() if shard.dtype != torch.float32 else None
            self._masters.append(master)
            self._m.append(torch.zeros(g.shard_numel, dtype=torch.float32, device=g.device))
            self._v.append(torch.zeros(g.shard_numel, dtype=torch.float32, device=g.device)
                           if self._kind in ('Adam', 'AdamW') else None)
            for (p, lo, hi, plo) in g.params_in_shard():
                self._pieces.append((gi, p, lo, hi, plo))
        self._plan = None
        self._step = 0

    # -- paddle optimizer surface ----------------------------------------------------------
    def get_lr(self):
        return self._inner.get_lr()

    def set_lr(self, v):
        self._inner.set_lr(v)

    @property
    def _learning_rate(self):
        return self._inner._learning_rate

    @property
    def _parameter_list(self):
        return self._inner._parameter_list

    def clear_grad(self, set_to_zero=True):
        self.state.zero_grad()

    clear_gradients = clear_grad

    def _wd(self, p):
        o = self._inner
        wd = o._weight_decay
        wd = float(wd) if wd is not None else 0.0
        fn = getattr(o, '_apply_decay_param_fun', None)
        if fn is not None and not fn(p.name):
            return 0.0
        return wd

    def _clip_coef(self):
        from ..nn.clip import ClipGradByGlobalNorm
        clip = self._inner._grad_clip
        if clip is None:
            return None
        if not isinstance(clip, ClipGradByGlobalNorm):
            raise NotImplementedError("sharding supports ClipGradByGlobalNorm only")
        # owned shards partition the gradients: local sum of squares + one all-reduce
        sq = K.global_l2_norm_sq(self.state.shard_grads)
        if self.state.world > 1:
            dist.all_reduce(sq, group=self.state.pg)
        return clip.clip_norm / torch.clamp(torch.sqrt(sq), min=clip.clip_norm)

    @torch.no_grad()
    def step(self):
        st = self.state
        self._step += 1
        o = self._inner
        o._step_count = self._step
        coef = self._clip_coef()
        lr = o.get_lr()
        dev = st.groups[0].device if st.groups else None
        coupled = self._kind == 'Adam' and o._weight_decay
        if dev is not None and dev.type == 'cuda' and _native.available() and not coupled:
            # the clip coefficient is read by the update kernel: no extra pass over the grads
            self._step_hip(lr, None if coef is None else
                           coef.to(torch.float32).reshape(()).contiguous())
        else:
            if coef is not None:
                for s in st.shard_grads:
                    s.mul_(coef.to(s.dtype))
            if dev is not None and dev.type == 'cuda' and _native.available():
                self._step_hip(lr)
            else:
                self._step_ref(lr)
        st.after_step()

    def _piece_views(self, gi, lo, hi):
        g = self.state.groups[gi]
        shard = g.param_shard
        master = self._masters[gi]
        return (master[lo:hi] if master is not None else shard[lo:hi], self.state.shard_grads[gi][lo:hi],
                self._m[gi][lo:hi], None if self._v[gi] is None else self._v[gi][lo:hi],
                shard[lo:hi] if master is not None else None)

    def _step_ref(self, lr):
        o = self._inner
        for gi, p, lo, hi, plo in self._pieces:
            master, grad, m, v, lowp = self._piece_views(gi, lo, hi)
            lrm = p.optimize_attr.get('learning_rate', 1.0)
            if self._kind in ('Adam', 'AdamW'):
                wd = self._wd(p)
                if self._kind == 'Adam' and wd:
                    grad = grad.float() + wd * master.float()
                    wd = 0.0
                K.adamw_ref([master if lowp is None else lowp], [grad], [m], [v],
                            [None if lowp is None else master], lr, o._beta1, o._beta2, o._epsilon,
                            [wd], [lrm], self._step)
            else:
                mu = getattr(o, '_momentum', 0.0)
                K.momentum_ref([master if lowp is None else lowp], [grad], [m],
                               [None if lowp is None else master], lr * lrm, mu, [self._wd(p)],
                               getattr(o, '_use_nesterov', False))

    def _step_hip(self, lr, scale_t=None):
        o = self._inner
        if self._plan is None:
            cols = [[], [], [], [], [], [], [], []]
            wds, lrms = [], []
            for gi, p, lo, hi, plo in self._pieces:
                master, grad, m, v, lowp = self._piece_views(gi, lo, hi)
                cols[0].append(master.data_ptr())
                cols[1].append(grad.data_ptr())
                cols[2].append(m.data_ptr())
                cols[3].append(0 if v is None else v.data_ptr())
                cols[4].append(0 if lowp is None else lowp.data_ptr())
                cols[5].append(hi - lo)
                cols[6].append(K._DT[grad.dtype])
                cols[7].append(K._DT[(lowp if lowp is not None else master).dtype])
                wd = self._wd(p)
                if self._kind == 'Adam':
                    wd = 0.0  # coupled L2 handled below (rare); AdamW decoupled in-kernel
                wds.append(wd)
                lrms.append(p.optimize_attr.get('learning_rate', 1.0))
            self._plan = K._mt_table(cols, cols[5], [wds, lrms], self.state.groups[0].device)
        tab, ftab, ch, nch = self._plan
        if self._kind in ('Adam', 'AdamW'):
            if self._kind == 'Adam' and o._weight_decay:
                for gi, p, lo, hi, plo in self._pieces:
                    w = self._wd(p)
                    if w:
                        master, grad, m, v, lowp = self._piece_views(gi, lo, hi)
                        grad.add_(master.to(grad.dtype), alpha=w)
            b1, b2 = o._beta1, o._beta2
            _native.lib().adamw_mt(tab.data_ptr(), ftab.data_ptr(), ch.data_ptr(), nch, float(lr),
                                   float(b1), float(b2), float(o._epsilon),
                                   float(1 - b1 ** self._step), float(1 - b2 ** self._step), 1.0,
                                   K._stream(), 0 if scale_t is None else scale_t.data_ptr())
        else:
            _native.lib().momentum_mt(tab.data_ptr(), ftab.data_ptr(), ch.data_ptr(), nch, float(lr),
                                      float(getattr(o, '_momentum', 0.0)),
                                      int(getattr(o, '_use_nesterov', False)), 1.0, K._stream(),
                                      0 if scale_t is None else scale_t.data_ptr())

    def minimize(self, loss, *a, **k):
        loss.backward()
        self.step()

    # -- checkpoint ------------------------------------------------------------------------
    def state_dict(self):
        """Owned-shard state (each rank saves its own .pdopt shard)."""
        sd = {}
        for gi in range(len(self.state.groups)):
            sd[f'shard{gi}_moment1'] = Tensor(self._m[gi])
            if self._v[gi] is not None:
                sd[f'shard{gi}_moment2'] = Tensor(self._v[gi])
            if self._masters[gi] is not None:
                sd[f'shard{gi}_master'] = Tensor(self._masters[gi])
        sd['@step'] = self._step
        sd['@rank'] = self.state.rank
        sd['@world'] = self.state.world
        from ..optimizer.lr import LRScheduler
        if isinstance(self._inner._learning_rate, LRScheduler):
            sd['LR_Scheduler'] = self._inner._learning_rate.state_dict()
        return sd

    def set_state_dict(self, sd):
        for gi in range(len(self.state.groups)):
            for key, buf in ((f'shard{gi}_moment1', self._m[gi]), (f'shard{gi}_moment2', self._v[gi]),
                             (f'shard{gi}_master', self._masters[gi])):
                if key in sd and buf is not None:
                    buf.copy_(_u(sd[key]).to(buf.device))
        self._step = int(sd.get('@step', self._step))
        if 'LR_Scheduler' in sd:
            self._inner._learning_rate.set_state_dict(sd['LR_Scheduler'])
        # refresh the owned low-precision shard from the restored master
        for gi, g in enumerate(self.state.groups):
            if self._masters[gi] is not None:
                g.param_shard.copy_(self._masters[gi])
        self.state.params_stale = True
        self.state.sync_params()


class ShardedModel(Layer):
    """Model wrapper returned by group_sharded_parallel (GroupShardedStage2/3 parity)."""

    def __init__(self, layer, state: ShardedState):
        super().__init__()
        self._layer = layer
        self.__dict__['_state'] = state

    def forward(self, *inputs, **kwargs):
        self._state.before_forward()
        return self._layer(*inputs, **kwargs)

    def state_dict(self, *a, **k):
        self._state.sync_params()
        return self._layer.state_dict(*a, **k)

    def set_state_dict(self, sd, use_structured_name=True):
        r = self._layer.set_state_dict(sd, use_structured_name)
        return r

    set_dict = set_state_dict
    load_dict = set_state_dict

    def parameters(self, include_sublayers=True):
        return self._layer.parameters(include_sublayers)

    def named_parameters(self, prefix='', include_sublayers=True):
        return self._layer.named_parameters(prefix, include_sublayers)

    def get_all_parameters(self, convert2cpu=False):
        self._state.sync_params()
        return self._layer.parameters()


def group_sharded_parallel(model, optimizer, level, scaler=None, group=None, offload=False,
                           sync_buffers=False, buffer_max_size=2 ** 23, segment_size=2 ** 20,
                           sync_comm=False, dp_group=None, exclude_layer=None,
                           bucket_mb=128):
    if level not in LEVELS:
        raise ValueError(f"level must be one of {list(LEVELS)}")
    st = ShardedState(model, level, group, segment_bytes=bucket_mb << 20)
    # the (bucketed, flat) params were re-pointed in place: the inner optimizer's list stays valid
    return ShardedModel(model, st), ShardedOptimizer(optimizer, st), scaler


def save_group_sharded_model(model, output, optimizer=None):
    import os
    from ..framework.io import save
    from ..distributed import collective as C
    os.makedirs(output, exist_ok=True)
    sd = model.state_dict()
    if C.get_rank() == 0:
        save(sd, os.path.join(output, 'model.pdparams'))
    if optimizer is not None:
        save(optimizer.state_dict(), os.path.join(output, f'model.rank{C.get_rank()}.pdopt'))
