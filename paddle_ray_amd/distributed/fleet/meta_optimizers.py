"""Static-graph Fleet: the meta-optimizer chain behind ``fleet.distributed_optimizer(opt).minimize``
in static mode (parity: python/paddle/distributed/fleet/fleet.py:1216,1485 `minimize` ->
meta-optimizer chain; meta_optimizers/raw_program_optimizer.py:284 `_insert_allreduce_ops` and
its fused form :343; gradient_merge_optimizer.py; sharding_optimizer.py:672 (stage 1);
lamb_optimizer.py; lars_optimizer.py; localsgd_optimizer.py; amp_optimizer.py). DGC
(dgc_optimizer.py) is rejected with an error instead of being silently ignored.

Program rewrite (MI355X design, not the reference's op-by-op c_allreduce_sum insertion):

* the parameter gradients are grouped into flat buckets in the order the backward PRODUCES them
  (last layers first), ``strategy.fuse_grad_size_in_MB`` per bucket (the DataParallel bucket
  rule, sized for the per-link xGMI ring: parallel/data_parallel.py);
* one ``c_allreduce_coalesced`` op per bucket is placed right after the grad op that produces the
  bucket's last gradient: it packs the bucket and issues an ASYNCHRONOUS RCCL all_reduce, so the
  late layers' gradients travel on RCCL's stream while the earlier layers' backward still runs;
* one ``c_sync_comm_stream`` op joins every bucket (work.wait: a stream dependency on the device,
  not a host block), applies the 1/nranks (x 1/k_steps) average and hands per-parameter views of
  the reduced buckets to the ``fleet_optimize`` op.

Gradient merge accumulates each bucket into a persistent flat buffer and communicates only on the
k-th micro-step (the reference merges before its allreduce the same way); the optimizer runs once
per window. Sharding stage 1 keeps each parameter's optimizer state on one owner rank (greedy
by size, sharding/shard.py), the owner updates it and broadcasts the new value. LocalSGD skips the
gradient all-reduce and averages the parameters every k_steps. Lamb / LARS replace an Adam(W) /
Momentum inner optimizer as the reference's meta-optimizers do.
"""
import torch
import torch.distributed as dist

from ...framework.core import Tensor, _u

_DEFAULT_BUCKET_MB = 32


# -- optimizer swaps (lamb / lars), shared with dygraph -------------------------------------------
def _exclude_fn(names):
    names = list(names or [])
    if not names:
        return None
    return lambda p: any(n in getattr(p, 'name', '') for n in names)


def apply_optimizer_swaps(opt, strategy):
    """strategy.lamb / strategy.lars replace the inner optimizer (lamb_optimizer.py:40-70,
    lars_optimizer.py:38-66); strategy.dgc raises. Returns the optimizer to use."""
    from ... import optimizer as O
    if getattr(strategy, 'dgc', False):
        raise NotImplementedError(
            "DistributedStrategy.dgc (deep gradient compression) is not supported on this "
            "framework; disable strategy.dgc")
    if getattr(strategy, 'lamb', False) and getattr(strategy, 'lars', False):
        raise ValueError("strategy.lamb and strategy.lars cannot both be enabled")
    if getattr(strategy, 'lamb', False):
        if not isinstance(opt, O.Adam):
            raise TypeError(f"strategy.lamb needs an Adam/AdamW inner optimizer, got {type(opt).__name__}")
        cfg = dict(getattr(strategy, 'lamb_configs', {}) or {})
        lamb = O.Lamb(learning_rate=opt._learning_rate,
                      lamb_weight_decay=cfg.get('lamb_weight_decay', 0.01),
                      beta1=opt._beta1, beta2=opt._beta2, epsilon=opt._epsilon,
                      parameters=opt._parameter_list or None, grad_clip=opt._grad_clip,
                      exclude_from_weight_decay_fn=_exclude_fn(cfg.get('exclude_from_weight_decay')),
                      multi_precision=opt._multi_precision)
        return lamb
    if getattr(strategy, 'lars', False):
        if not isinstance(opt, O.Momentum):
            raise TypeError(f"strategy.lars needs a Momentum inner optimizer, got {type(opt).__name__}")
        cfg = dict(getattr(strategy, 'lars_configs', {}) or {})
        return O.LarsMomentum(learning_rate=opt._learning_rate, momentum=opt._momentum,
                              lars_coeff=cfg.get('lars_coeff', 0.001),
                              lars_weight_decay=cfg.get('lars_weight_decay', 0.0005),
                              epsilon=cfg.get('epsilon', 0.0),
                              exclude_from_weight_decay=cfg.get('exclude_from_weight_decay'),
                              parameters=opt._parameter_list or None, grad_clip=opt._grad_clip,
                              multi_precision=opt._multi_precision)
    return opt


# -- communication state of one rewritten program ---------------------------------------------------
class _CommState:
    def __init__(self, pg, nranks, k_steps=1, avg=True, rank_avg=True, extra_pgs=()):
        self.pg, self.nranks = pg, nranks
        self.k_steps, self.avg = max(1, int(k_steps)), avg
        self.rank_avg = rank_avg          # divide the all-reduced sum by nranks
        self.extra_pgs = list(extra_pgs)  # further groups reduced after the first (2-D meshes)
        self.works = {}
        self.merged = {}    # bucket -> persistent flat accumulation buffer (gradient merge)
        self.micro = 0      # completed runs
        self.buckets = []   # [[(param name, numel, shape)]] per bucket (introspection / tests)
        self.shard = None   # sharding stage 1: _ShardPlan
        self.localsgd = None
        self.steps = 0      # optimizer steps taken
        self.last_comm = 0  # localsgd: the step of the last parameter averaging
        self.linked = []    # bucket states whose merge window this (optimize) state drives

    def final_micro(self):
        """This run completes a gradient-merge window (always True without merging)."""
        return (self.micro + 1) % self.k_steps == 0


def _bucket_allreduce(state, b, *grads):
    """Pack one bucket and start its all_reduce (async). With gradient merge the bucket is
    accumulated into its persistent buffer and reduced only on the window's last micro-step."""
    gs = [_u(g) for g in grads]
    flat = torch.cat([g.reshape(-1) for g in gs]) if len(gs) > 1 else gs[0].reshape(-1).clone()
    if state.k_steps > 1:
        m = state.merged.get(b)
        if m is None or m.shape != flat.shape or m.dtype != flat.dtype or m.device != flat.device:
            m = state.merged[b] = torch.zeros_like(flat)
        m.add_(flat)
        flat = m
        if not state.final_micro():
            return Tensor(flat)
    if state.nranks > 1:
        state.works[b] = dist.all_reduce(flat, group=state.pg, async_op=True)
    return Tensor(flat)


def _sync_split(state, layout, *flats):
    """Join the buckets' collectives, average, and return per-parameter views (None on a
    gradient-merge micro-step that does not complete its window)."""
    n = sum(len(b) for b in layout)
    if not state.final_micro():
        for b in range(len(flats)):
            state.works.pop(b, None)
        return [None] * n
    scale = 1.0
    if state.nranks > 1 and state.rank_avg:
        scale /= state.nranks
    if state.k_steps > 1 and state.avg:
        scale /= state.k_steps
    outs = []
    for b, flat in enumerate(flats):
        f = _u(flat)
        w = state.works.pop(b, None)
        if w is not None:
            w.wait()
        for pg in state.extra_pgs:
            dist.all_reduce(f, group=pg)
        if scale != 1.0:
            f.mul_(scale)
        off = 0
        for _, numel, shape in layout[b]:
            outs.append(Tensor(f[off:off + numel].view(shape)))
            off += numel
    return outs


class _ShardPlan:
    """Sharding stage 1: parameter -> owner rank (greedy by size over the sharding group)."""

    def __init__(self, params, group):
        self.group = group
        self.pg = group.process_group if group is not None else None
        self.nranks = group.nranks if group is not None else dist.get_world_size()
        self.ranks = list(group.ranks) if group is not None else list(range(self.nranks))
        me = dist.get_rank()
        self.local = self.ranks.index(me)
        load = [0] * self.nranks
        self.owner = {}
        for p in sorted(params, key=lambda p: -_u(p).numel()):
            r = min(range(self.nranks), key=lambda i: (load[i], i))
            self.owner[p.name] = r
            load[r] += _u(p).numel()

    def owned(self, params):
        """This rank's parameters: the ones it owns plus any outside the plan (updated by every
        rank, e.g. parameters not replicated over the sharding group)."""
        return [p for p in params if self.owner.get(p.name, self.local) == self.local]

    def broadcast(self, params):
        """Every owner sends its updated parameters (one flat broadcast per owner)."""
        pend = []
        for r in range(self.nranks):
            ps = [p for p in params if self.owner.get(p.name) == r]
            if not ps:
                continue
            flat = torch.cat([_u(p).detach().reshape(-1) for p in ps])
            w = dist.broadcast(flat, src=self.ranks[r], group=self.pg, async_op=True)
            pend.append((w, flat, ps, r))
        for w, flat, ps, r in pend:
            w.wait()
            if r == self.local:
                continue
            off = 0
            with torch.no_grad():
                for p in ps:
                    t = _u(p)
                    t.copy_(flat[off:off + t.numel()].view(t.shape))
                    off += t.numel()


def _average_params(state, params):
    """LocalSGD communication: parameters <- their mean over the ranks (localsgd_optimizer.py:
    snapshot - allreduce_mean(snapshot - param), the snapshot being equal on every rank)."""
    ts = [_u(p) for p in params]
    flat = torch.cat([t.detach().reshape(-1) for t in ts])
    dist.all_reduce(flat, group=state.pg)
    flat.div_(state.nranks)
    off = 0
    with torch.no_grad():
        for t in ts:
            t.copy_(flat[off:off + t.numel()].view(t.shape))
            off += t.numel()


def _fleet_optimize(state, opt, params, *grads, scaler=None):
    from ...static.graph import _optimize_fn
    final = state.final_micro()
    state.micro += 1
    for s in state.linked:
        s.micro += 1
    if not final:
        return None
    if state.shard is not None:
        sh = state.shard
        owned = set(id(p) for p in sh.owned(params))
        own_p = [p for p in params if id(p) in owned]
        own_g = [g for p, g in zip(params, grads) if id(p) in owned]
        others = [(p, _u(g)) for p, g in zip(params, grads) if g is not None and id(p) not in owned]

        # Every rank holds EVERY reduced gradient. The loss-scale unscale / found_inf check and
        # the global clip norm must cover all of them (not just the owned ones): found_inf is
        # then identical on every rank (all skip or all step, the scales never drift apart, a
        # rank that owns nothing included) and the norm is taken over unscaled gradients.
        def every_grad(clip_only=False):
            gs = [p._t.grad for p in own_p if p._t.grad is not None and
                  (not clip_only or getattr(p, 'need_clip', True))]
            return gs + [g for p, g in others if not clip_only or getattr(p, 'need_clip', True)]
        clip = opt._grad_clip
        from ...nn.clip import ClipGradByGlobalNorm
        from ...ops.fused import global_l2_norm_sq
        prev_hook = None
        if isinstance(clip, ClipGradByGlobalNorm):
            prev_hook = clip._norm_hook
            if getattr(prev_hook, 'dist_norm', None) is not None:
                # a partitioned program's distributed clip: per parameter class over its mesh
                # axes, reading the owned gradients and the reduced ones of the other owners
                gmap = {id(p): g for p, g in others}
                clip._norm_hook = lambda sq: prev_hook.dist_norm(
                    lambda p: p._t.grad if id(p) in owned else gmap.get(id(p)), sq)
            else:
                clip._norm_hook = lambda sq: global_l2_norm_sq(every_grad(True)).reshape(())
        had_sg = '_scaler_grads' in opt.__dict__
        prev_sg = opt.__dict__.get('_scaler_grads')
        opt._scaler_grads = every_grad
        try:
            if own_p:
                _optimize_fn(opt, own_p, *own_g, scaler=scaler)
            elif scaler is not None:
                scaler.unscale_(opt)     # found_inf over the reduced gradients like every rank
                scaler.update()
        finally:
            if isinstance(clip, ClipGradByGlobalNorm):
                clip._norm_hook = prev_hook
            if had_sg:
                opt._scaler_grads = prev_sg
            else:
                del opt.__dict__['_scaler_grads']
        sh.broadcast(params)
    else:
        _optimize_fn(opt, params, *grads, scaler=scaler)
    state.steps += 1
    for s in [state] + state.linked:
        for m in s.merged.values():
            m.zero_()
    ls = state.localsgd
    if ls is not None:
        # localsgd_optimizer.py:206: cond(step > begin_step, begin_localsgd, communicate) --
        # average after EVERY step through begin_step, then k_steps after the last averaging
        k, begin = ls
        if state.steps <= begin or state.steps - state.last_comm >= k:
            _average_params(state, params)
            state.last_comm = state.steps
    return None


# -- the program rewrite ------------------------------------------------------------------------------
def _bucket_plan(blk, n_before, pg_items, bucket_bytes):
    """[(insert position, [(param, grad var)])]: gradients in production order, cut into buckets
    of about ``bucket_bytes`` (one dtype per bucket)."""
    producer = {}
    for i in range(n_before, len(blk.ops)):
        for v in blk.ops[i].all_outputs():
            producer[v] = i
    items = sorted(pg_items, key=lambda pg: producer.get(pg[1].vid, len(blk.ops)))
    buckets, cur, cur_bytes, cur_dt = [], [], 0, None
    for p, g in items:
        t = _u(p)
        nb = t.numel() * t.element_size()
        if cur and (cur_bytes + nb > bucket_bytes or t.dtype != cur_dt):
            buckets.append(cur)
            cur, cur_bytes = [], 0
        cur.append((p, g))
        cur_bytes += nb
        cur_dt = t.dtype
    if cur:
        buckets.append(cur)
    out = []
    for b in buckets:
        pos = max(producer.get(g.vid, len(blk.ops) - 1) for _, g in b) + 1
        out.append((pos, b))
    return out


def _insert_bucketed(blk, n_before, pg, state, bucket_bytes, tag=''):
    """Insert one async all-reduce op per gradient bucket (right after the bucket's last
    producer) and the joining sync op; returns (params, reduced grad vars) in bucket order."""
    from ...static import graph as G
    plan = _bucket_plan(blk, n_before, pg, bucket_bytes)
    layout, flat_vids, inserts = [], [], []
    for b, (pos, items) in enumerate(plan):
        fv = G._new_var(blk, [sum(_u(p).numel() for p, _ in items)], _u(items[0][0]).dtype,
                        f'coalesced_grad{tag}_{b}')
        op = G.OpDesc('c_allreduce_coalesced', _bucket_allreduce,
                      [state, b] + [G._VarRef(g.vid) for _, g in items], {},
                      [g.vid for _, g in items], [fv.vid], 'T', role='backward')
        inserts.append((pos, op))
        layout.append([(p.name, _u(p).numel(), tuple(_u(p).shape)) for p, _ in items])
        flat_vids.append(fv.vid)
    for pos, op in sorted(inserts, key=lambda x: -x[0]):   # back to front: positions stay valid
        blk.ops.insert(pos, op)
    state.buckets = layout
    order = [p for _, items in plan for p, _ in items]
    outs = [G._new_var(blk, list(_u(p).shape), _u(p).dtype, p.name + '@GRAD@REDUCED') for p in order]
    sync = G.OpDesc('c_sync_comm_stream', _sync_split, [state, layout] + [G._VarRef(v) for v in flat_vids],
                    {}, list(flat_vids), [g.vid for g in outs], ('list', ['T'] * len(outs)),
                    role='backward')
    blk.ops.append(sync)
    return order, outs


def insert_grad_sync(prog, n_before, pg, sync, bucket_mb=_DEFAULT_BUCKET_MB, k_steps=1, avg=True):
    """Static auto-parallel: the gradients of parameters replicated over mesh axes (data
    parallel) are SUMMED over those axes' groups (the loss's own 1/n already scales them) in
    flat buckets, asynchronously inside the backward (parity: auto_parallel_data_parallel_
    optimization.py:57,132 `_fuse_allreduce`, GradientsGroup :727). ``sync``: local parameter
    name -> [Group, ...]. With ``k_steps`` > 1 each bucket accumulates locally and is reduced on
    the merge window's last micro-step only. Returns (params, grad vars) for the optimize op;
    the bucket states are ``prog._ap_grad_states``."""
    blk = prog.global_block()
    byname = {p.name: (p, g) for p, g in pg}
    keyed = {}
    for name, groups in sync.items():
        if name in byname and groups:
            keyed.setdefault(tuple(id(g) for g in groups), (groups, []))[1].append(byname[name])
    states = []
    done = {}
    for t, (key, (groups, items)) in enumerate(sorted(keyed.items(), key=lambda kv: kv[0])):
        st = _CommState(groups[0].process_group, groups[0].nranks, k_steps, avg, rank_avg=False,
                        extra_pgs=[g.process_group for g in groups[1:]])
        ps, gs = _insert_bucketed(blk, n_before, items, st, int(bucket_mb * (1 << 20)), tag=f'_{t}')
        for p, g in zip(ps, gs):
            done[p.name] = g
        states.append(st)
    prog.__dict__['_ap_grad_states'] = states
    prog.__dict__['_no_graph'] = True
    params = [p for p, _ in pg]
    return params, [done.get(p.name, g) for p, g in pg]


def _majority_group(sync):
    """The group most parameters reduce over (the data-parallel axis of a partitioned program)."""
    count = {}
    for groups in (sync or {}).values():
        for g in groups:
            count.setdefault(id(g), [g, 0])[1] += 1
    return max(count.values(), key=lambda gc: gc[1])[0] if count else None


def build_sync_optimize(prog, n_before, pg, opt, scaler, sync, k_steps, avg, shard, bucket_mb):
    """The training tail of a program built by ``paddle.static`` minimize when a gradient all-reduce
    (auto-parallel ``sync``), a gradient-merge window or sharding stage 1 applies (the
    distributed passes auto_parallel_data_parallel_optimization / gradient_merge / sharding):
    bucketed reductions inside the backward, then one ``fleet_optimize`` op that steps on the
    window's last micro-step (the owners update, then broadcast, under sharding)."""
    from ...static import graph as G
    blk = prog.global_block()
    k_steps = max(1, int(k_steps))
    linked = []
    params = [p for p, _ in pg]
    gvars = [g for _, g in pg]
    if sync:
        params, gvars = insert_grad_sync(prog, n_before, pg, sync, bucket_mb, k_steps, avg)
        linked += prog.__dict__['_ap_grad_states']
    if k_steps > 1:
        # gradients no group reduces still accumulate over the window (a local bucket state)
        synced = {p.name for p in params if sync and p.name in sync and sync[p.name]}
        local = [(p, g) for p, g in zip(params, gvars) if p.name not in synced]
        if local:
            st = _CommState(None, 1, k_steps, avg, rank_avg=False)
            order, outs = _insert_bucketed(blk, n_before, local, st, int(bucket_mb * (1 << 20)),
                                           tag='_local')
            red = {p.name: g for p, g in zip(order, outs)}
            gvars = [red.get(p.name, g) for p, g in zip(params, gvars)]
            linked.append(st)
    state = _CommState(None, 1, k_steps, avg)
    state.linked = linked
    if shard is not None and dist.is_initialized() and dist.get_world_size() > 1:
        group = shard if shard != 'auto' else _majority_group(sync)
        if group is None and not sync:
            raise ValueError("sharding stage 1 needs the program's data-parallel gradient all-reduce "
                             "(a partitioned program with replicated parameters); none was found")
        members = [p for p in params if not sync or (p.name in sync and any(g is group for g in sync[p.name]))] \
            if group is not None else params
        state.shard = _ShardPlan(members, group)
        opt._param_groups = []
        opt._add_param_group({'params': state.shard.owned(params)})
    op = G.OpDesc('fleet_optimize', _fleet_optimize, [state, opt, params] + [G._VarRef(g.vid) for g in gvars],
                  {'scaler': scaler}, [g.vid for g in gvars], [], 'C', role='optimize')
    blk.ops.append(op)
    prog.__dict__['_no_graph'] = True
    prog.__dict__['_fleet_state'] = state


def _static_pipeline(opt, loss, strategy, hcg, parameters, scaler):
    """strategy.pipeline: the program split by device_guard into one stage per rank of the
    pipeline group (static/pipeline.py; reference meta_optimizers/pipeline_optimizer.py:198)."""
    from ...static.pipeline import build_pipeline
    ls = None
    if getattr(strategy, 'localsgd', False):
        if getattr(strategy, 'sharding', False):
            raise NotImplementedError("static pipeline: localsgd together with sharding is not supported")
        lcfg = strategy.localsgd_configs or {}
        ls = (int(lcfg.get('k_steps', 1)), int(lcfg.get('begin_step', 1)))
    shard = bool(getattr(strategy, 'sharding', False))
    if shard:
        stage = int((strategy.sharding_configs or {}).get('stage', 1))
        if stage != 1:
            raise NotImplementedError(f"static pipeline with sharding supports stage 1 (got stage {stage})")
    # (strategy.lamb / lars: fleet.distributed_optimizer already swapped the inner optimizer;
    # every stage steps it on its own parameters)
    if scaler is not None:
        raise NotImplementedError("static pipeline with fp16 loss scaling is not supported (use bf16)")
    cfg = dict(strategy.pipeline_configs or {})
    n_micro = int(cfg.get('accumulate_steps', 1))
    pp_group = dp_group = None
    if hcg is not None:
        if hcg.get_model_parallel_world_size() > 1:
            raise NotImplementedError("static pipeline with tensor parallelism is not supported")
        if hcg.get_pipe_parallel_world_size() > 1:
            pp_group = hcg.get_pipe_parallel_group()
        if hcg.get_data_parallel_world_size() > 1:
            dp_group = hcg.get_data_parallel_group()
    ckpts = None
    if getattr(strategy, 'recompute', False):
        ckpts = list((strategy.recompute_configs or {}).get('checkpoints') or [])
        if not ckpts:
            raise ValueError("strategy.recompute needs recompute_configs['checkpoints']")
    gm = None
    if getattr(strategy, 'gradient_merge', False):
        gcfg = strategy.gradient_merge_configs or {}
        gm = (int(gcfg.get('k_steps', 1)), bool(gcfg.get('avg', True)))
    return build_pipeline(opt, loss, n_micro, cfg.get('schedule_mode', '1F1B'), parameters, pp_group, dp_group,
                          checkpoints=ckpts, gradient_merge=gm, shard=shard, localsgd=ls)


def strategy_with_pass_cfg(strategy, cfg):
    """A copy of a fleet DistributedStrategy with the settings the distributed passes recorded."""
    import copy
    s = copy.copy(strategy)
    for k, v in list(vars(s).items()):
        if isinstance(v, dict):
            s.__dict__[k] = dict(v)
    if cfg.get('checkpoints'):
        s.__dict__['recompute'] = True
        s.__dict__['recompute_configs'] = {'checkpoints': list(cfg['checkpoints'])}
    amp = cfg.get('amp')
    if amp is not None:
        s.__dict__['amp'] = True
        s.__dict__['amp_configs'] = {
            'init_loss_scaling': amp.get('init_loss_scaling', 32768.0),
            'use_dynamic_loss_scaling': amp.get('use_dynamic_loss_scaling', True),
            'use_bf16': amp['dtype'] == 'bfloat16', 'use_pure_fp16': amp.get('level') == 'O2',
            'custom_white_list': list(amp.get('white') or ()),
            'custom_black_list': list(amp.get('black') or ())}
    k, avg = cfg.get('gradient_merge', (1, True))
    if k > 1:
        s.__dict__['gradient_merge'] = True
        s.__dict__['gradient_merge_configs'] = {'k_steps': k, 'avg': avg}
    if cfg.get('sharding') is not None:
        s.__dict__['sharding'] = True
        s.__dict__['sharding_configs'] = dict(s.sharding_configs, stage=1)
    if 'bucket_mb' in cfg:
        s.__dict__['fuse_grad_size_in_MB'] = cfg['bucket_mb']
    return s


def static_minimize(opt, loss, strategy, hcg, parameters=None):
    """Rewrite the program of ``loss`` for collective training (see the module docstring)."""
    from ...static import graph as G
    from ...static.amp import OptimizerWithMixedPrecision, decorate as amp_decorate
    prog = loss.block.program
    blk = prog.global_block()
    orig_opt, orig_strategy = opt, strategy
    if prog.__dict__.get('_pass_cfg'):
        strategy = strategy_with_pass_cfg(strategy, prog.__dict__['_pass_cfg'])
    fwd_vids = set(blk.vars)
    scaler, loss_scale = None, 1.0
    if getattr(strategy, 'amp', False) and not isinstance(opt, OptimizerWithMixedPrecision):
        cfg = dict(strategy.amp_configs or {})
        from ...static.amp import AutoMixedPrecisionLists
        lists = AutoMixedPrecisionLists(cfg.get('custom_white_list'), cfg.get('custom_black_list'))
        opt = amp_decorate(opt, lists, init_loss_scaling=cfg.get('init_loss_scaling', 32768),
                           use_pure_fp16=cfg.get('use_pure_fp16', False),
                           use_bf16=cfg.get('use_bf16', False),
                           use_dynamic_loss_scaling=cfg.get('use_dynamic_loss_scaling', True))
    if isinstance(opt, OptimizerWithMixedPrecision):
        opt._tag_program(prog)
        if opt._use_scaling:
            from ...static.amp import _ScaleRef
            scaler, loss_scale = opt._scaler, _ScaleRef(opt._scaler)
        opt = opt._optimizer
    if getattr(strategy, 'localsgd', False) and getattr(strategy, 'gradient_merge', False):
        raise ValueError("strategy.localsgd cannot be combined with gradient_merge")
    if getattr(strategy, 'adaptive_localsgd', False):
        raise NotImplementedError("strategy.adaptive_localsgd is not supported; use localsgd")
    if not opt._parameter_list:
        ps = parameters or [p for p in prog.all_parameters() if not p.stop_gradient]
        opt._param_groups = []
        opt._add_param_group({'params': list(ps)})
    groups = G.save_param_groups(opt)
    if getattr(strategy, 'pipeline', False):
        return _static_pipeline(opt, loss, strategy, hcg, parameters, scaler)
    if hcg is not None and (hcg.get_model_parallel_world_size() > 1 or
                            hcg.get_pipe_parallel_world_size() > 1):
        raise NotImplementedError(
            "static-mode fleet supports data parallel, pipeline (strategy.pipeline), sharding "
            "stage 1, gradient merge and localsgd; for tensor-parallel static programs use "
            "paddle.distributed.auto_parallel (static Engine)")
    world = dist.get_world_size() if dist.is_initialized() else 1
    k = 1
    avg = True
    if getattr(strategy, 'gradient_merge', False):
        gm = strategy.gradient_merge_configs or {}
        k, avg = int(gm.get('k_steps', 1)), bool(gm.get('avg', True))
    state = _CommState(None, world, k, avg)
    sharding = getattr(strategy, 'sharding', False) and world > 1
    if sharding:
        stage = int((strategy.sharding_configs or {}).get('stage', 1))
        if stage != 1:
            raise NotImplementedError(f"static-mode sharding supports stage 1 (got stage {stage}); "
                                      "use dygraph group_sharded_parallel for stages 2/3")
    G.check_single_device(prog, 'fleet.distributed_optimizer(...).minimize')
    ckpts = None
    if getattr(strategy, 'recompute', False):
        # recompute_optimizer.py:97 -> RecomputeOptimizer._set_checkpoints + backward with
        # forward recomputation between the checkpoints
        names = list((strategy.recompute_configs or {}).get('checkpoints') or [])
        if not names:
            raise ValueError("strategy.recompute needs recompute_configs['checkpoints'] (the "
                             "static Variables or their names to keep in memory)")
        ckpts = [blk.var(n) if isinstance(n, str) else n for n in names]
    pcfg = prog.__dict__.get('_pass_cfg') or {}
    segments_fn = None
    if ckpts is None and pcfg.get('recompute_annotated') is not None:
        skip = list(pcfg['recompute_annotated'])
        segments_fn = lambda fwd: G.annotated_segments(fwd, skip)  # noqa: E731
    n_before = len(blk.ops)
    pg = G.append_backward(loss, parameters, loss_scale=loss_scale, checkpoints=ckpts,
                           segments_fn=segments_fn)
    params = [p for p, _ in pg]
    prog.__dict__['_minimize_params'] = list(params)
    if sharding:
        state.shard = _ShardPlan(params, hcg.get_sharding_parallel_group()
                                 if hcg is not None and hcg.get_sharding_parallel_world_size() > 1
                                 else None)
        # the inner optimizer keeps state for the owned parameters only
        own = state.shard.owned(params)
        opt._param_groups = []
        opt._add_param_group({'params': own})
    localsgd = getattr(strategy, 'localsgd', False) and world > 1
    if localsgd:
        cfg = strategy.localsgd_configs or {}
        state.localsgd = (max(1, int(cfg.get('k_steps', 1))), max(1, int(cfg.get('begin_step', 1))))
    gvars = [g for _, g in pg]
    comm = (world > 1 and not localsgd) or k > 1
    if comm:
        mb = getattr(strategy, 'fuse_grad_size_in_MB', _DEFAULT_BUCKET_MB) or _DEFAULT_BUCKET_MB
        if not getattr(strategy, 'fuse_all_reduce_ops', True):
            mb = 0   # one bucket per gradient (reference: unfused c_allreduce_sum per grad)
        params, gvars = _insert_bucketed(blk, n_before, pg, state, int(mb * (1 << 20)))
    op = G.OpDesc('fleet_optimize', _fleet_optimize, [state, opt, params] + [G._VarRef(g.vid) for g in gvars],
                  {'scaler': scaler}, [g.vid for g in gvars], [], 'C', role='optimize')
    blk.ops.append(op)
    # collectives whose participation changes per run (merge windows, localsgd, owner
    # broadcasts) and async work handles are kept out of HIP-graph capture
    prog.__dict__['_no_graph'] = True
    prog.__dict__['_fleet_state'] = state
    for hook in pcfg.get('minimize_hooks', ()):
        hook(prog, opt)
    prog.__dict__['_train_meta'] = {
        'fwd_vids': fwd_vids, 'kind': 'fleet',
        'rebuild': lambda: (G.restore_param_groups(opt, groups),
                            static_minimize(orig_opt, loss, orig_strategy, hcg, parameters))}
    prog._bump()
    return None, pg
