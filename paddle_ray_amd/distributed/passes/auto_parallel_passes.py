"""Distributed-training passes over ``paddle.static`` programs (parity:
python/paddle/distributed/passes/auto_parallel_amp.py:663, auto_parallel_fp16.py:742,
auto_parallel_recompute.py:254, auto_parallel_gradient_merge.py:331,
auto_parallel_sharding.py:83, auto_parallel_grad_clip.py:288,
auto_parallel_data_parallel_optimization.py:56, fuse_all_reduce.py:353).

MI355X design, not the reference's op-by-op program surgery: this framework's static programs
replay eager ops (HIP kernels, RCCL collectives) per OpDesc, so the passes do not insert cast /
check_finite / c_allreduce ops one at a time. Each records what it changes in
``program._pass_cfg``; the program's minimize (static/graph.py ``_static_minimize``, fleet's
``static_minimize``) builds the training ops from it:

* amp / fp16: every forward op (and its grad op) is tagged with the AMP policy the Executor
  replays it under (O1 white/black lists, O2 = everything but the black list), a GradScaler
  with dynamic loss scaling seeds the backward and unscales / inf-checks the gradients inside
  the optimize op (float16; bfloat16 runs unscaled);
* recompute: explicit ``checkpoints`` or the ``auto_parallel.recompute`` regions of the program
  become recompute segments of the backward (RNG-exact re-forward, see graph._emit_recompute);
* gradient_merge: ``k_steps`` micro-steps accumulate in the flat gradient buckets, the bucket
  all-reduce and the optimizer run once per window (``avg``: mean over the window);
* sharding (stage 1): parameters are owned greedily by size over the data-parallel group, the
  owner updates (its optimizer state only) and broadcasts;
* data_parallel_optimization / fuse_all_reduce: the gradient bucket size of the bucketed async
  all-reduce issued inside the backward (size it for the per-link xGMI ring);
* grad_clip: the global-norm clip of a partitioned program sums each parameter's squared norm
  over the mesh axes the parameter is split on (replicated parameters count once).

A pass applied to a program that is already minimized strips its training ops and re-runs the
minimize (static/graph.py ``rebuild_training``), so passes compose in any order; applied before
minimize, the settings wait for it."""
import torch
import torch.distributed as dist

from .pass_base import PassBase, PassType, register_pass

__all__ = []


def _cfg(prog):
    return prog.__dict__.setdefault('_pass_cfg', {})


def _refresh(prog):
    from ...static.graph import rebuild_training
    if not rebuild_training(prog):
        prog._bump()


def _as_float(v, what):
    try:
        return float(v)
    except (TypeError, ValueError):
        raise TypeError(f"{what} must be a number, got {v!r}") from None


class _ProgramPass(PassBase):
    def _type(self):
        return PassType.PARALLEL_OPT

    def _apply_single_impl(self, main_program, startup_program, context):
        self._record(main_program, _cfg(main_program), context)
        _refresh(main_program)

    def _record(self, prog, cfg, context):
        raise NotImplementedError


# -- AMP ----------------------------------------------------------------------------------------
@register_pass('auto_parallel_amp')
class AMPPass(_ProgramPass):
    """O1 mixed precision. Attributes: dtype ('float16' | 'bfloat16'), custom_white_list,
    custom_black_list, custom_black_varnames, init_loss_scaling, incr_every_n_steps,
    decr_every_n_nan_or_inf, incr_ratio, decr_ratio, use_dynamic_loss_scaling (float16 only:
    bfloat16 has fp32's exponent range and runs unscaled)."""
    level = 'O1'

    def __init__(self):
        super().__init__()
        for k, v in (('dtype', ''), ('loss', None), ('dist_context', None), ('custom_white_list', None),
                     ('custom_black_list', None), ('custom_black_varnames', None),
                     ('init_loss_scaling', 32768.0), ('incr_every_n_steps', 1000),
                     ('decr_every_n_nan_or_inf', 2), ('incr_ratio', 2.0), ('decr_ratio', 0.8),
                     ('use_dynamic_loss_scaling', False), ('input_data', []), ('params_grads', [])):
            self.set_attr(k, v)

    def _check_self(self):
        if self.get_attr('dtype') not in ('float16', 'bfloat16'):
            return False
        for k in ('init_loss_scaling', 'incr_every_n_steps', 'decr_every_n_nan_or_inf', 'incr_ratio',
                  'decr_ratio'):
            if _as_float(self.get_attr(k), k) < 0:
                return False
        white = set(self.get_attr('custom_white_list') or ())
        black = set(self.get_attr('custom_black_list') or ())
        if white & black:
            raise ValueError(f"ops in both custom_white_list and custom_black_list: {sorted(white & black)}")
        return True

    def _check_conflict(self, other_pass):
        return not isinstance(other_pass, AMPPass)

    def _record(self, prog, cfg, context):
        from ...amp import GradScaler
        dtype = self.get_attr('dtype')
        amp = {'dtype': dtype, 'level': self.level,
               'white': set(self.get_attr('custom_white_list') or ()),
               'black': set(self.get_attr('custom_black_list') or ()),
               'init_loss_scaling': self.get_attr('init_loss_scaling'),
               'use_dynamic_loss_scaling': self.get_attr('use_dynamic_loss_scaling'),
               'scaler': None}
        scaling = dtype == 'float16' and (self.get_attr('use_dynamic_loss_scaling') or
                                          float(self.get_attr('init_loss_scaling')) != 1.0)
        if scaling:
            amp['scaler'] = GradScaler(
                init_loss_scaling=float(self.get_attr('init_loss_scaling')),
                incr_ratio=float(self.get_attr('incr_ratio')), decr_ratio=float(self.get_attr('decr_ratio')),
                incr_every_n_steps=int(self.get_attr('incr_every_n_steps')),
                decr_every_n_nan_or_inf=int(self.get_attr('decr_every_n_nan_or_inf')),
                use_dynamic_loss_scaling=bool(self.get_attr('use_dynamic_loss_scaling')))
        cfg['amp'] = amp
        from ...static.amp import tag_program
        tag_program(prog, amp)
        context.set_attr('amp_scaler', amp['scaler'])


@register_pass('auto_parallel_fp16')
class FP16Pass(AMPPass):
    """Pure low-precision (O2): every op but the black list runs in ``dtype``; the optimizer
    keeps fp32 master weights (multi_precision). ``use_optimizer_fp16`` / level 'o3' (optimizer
    state in low precision too) is refused: the fused multi-tensor optimizers here keep fp32
    moments."""
    level = 'O2'

    def _check_self(self):
        if self.get_attr('use_optimizer_fp16') or str(self.get_attr('level', '')).lower() == 'o3':
            raise NotImplementedError("auto_parallel_fp16 with use_optimizer_fp16 / level 'o3' is not "
                                      "supported: the optimizer keeps fp32 master weights and moments")
        return super()._check_self()


# -- recompute ------------------------------------------------------------------------------------
@register_pass('auto_parallel_recompute')
class RecomputePass(_ProgramPass):
    """Attributes: checkpoints (Variables or names kept in memory; the ops between them are
    re-run in the backward) -- or, without checkpoints, the program's ``auto_parallel.recompute``
    regions; no_recompute_segments (indices of annotated regions to keep); loss, dist_context,
    no_grad_set (accepted for API parity)."""

    def __init__(self):
        super().__init__()
        self.set_attr('loss', None)
        self.set_attr('dist_context', None)
        self.set_attr('no_grad_set', None)
        self.set_attr('no_recompute_segments', [])
        self.set_attr('checkpoints', None)

    def _check_self(self):
        ck = self.get_attr('checkpoints')
        if ck is not None and not isinstance(ck, (list, tuple)):
            raise TypeError("checkpoints must be a list of Variables or names")
        return True

    def _record(self, prog, cfg, context):
        ck = self.get_attr('checkpoints')
        cfg.pop('checkpoints', None)
        cfg.pop('recompute_annotated', None)
        if ck:
            blk = prog.global_block()
            cfg['checkpoints'] = [blk.var(c).name if isinstance(c, str) else c.name for c in ck]
            return
        if not any('recompute_id' in op.attrs for op in prog.global_block().ops):
            raise ValueError("auto_parallel_recompute: give `checkpoints` or wrap layers with "
                             "paddle.distributed.auto_parallel.recompute(...) in the program")
        cfg['recompute_annotated'] = list(self.get_attr('no_recompute_segments') or [])


# -- gradient merge ---------------------------------------------------------------------------------
@register_pass('auto_parallel_gradient_merge_pass')
class GradientMergePass(_ProgramPass):
    """Attributes: k_steps (micro-steps per optimizer step), avg (mean instead of sum)."""

    def __init__(self):
        super().__init__()
        self.set_attr('k_steps', -1)
        self.set_attr('avg', True)
        self.set_attr('dist_context', None)
        self.set_attr('params_grads', [])

    def _check_self(self):
        return int(self.get_attr('k_steps')) >= 1

    def _record(self, prog, cfg, context):
        cfg['gradient_merge'] = (int(self.get_attr('k_steps')), bool(self.get_attr('avg')))


# -- sharding stage 1 -----------------------------------------------------------------------------
@register_pass('auto_parallel_sharding')
class ShardingPass(_ProgramPass):
    """Attributes: stage (1; stages 2 / 3 shard gradients / parameters and live in dygraph
    ``group_sharded_parallel``), degree / sharding_degree (checked against the group), group
    (a communication Group; default: the group most gradients are all-reduced over -- the
    data-parallel axis of a partitioned program -- or the world)."""

    def __init__(self):
        super().__init__()
        for k, v in (('dist_context', None), ('stage', 1), ('sharding_degree', None), ('degree', None),
                     ('enable_overlap', False), ('params_grads', []), ('global_rank', -1), ('group', None)):
            self.set_attr(k, v)

    def _check_self(self):
        stage = int(self.get_attr('stage'))
        if stage not in (1, 2, 3):
            return False
        if stage != 1:
            raise NotImplementedError(
                f"auto_parallel_sharding stage {stage} is not supported for static programs; use "
                "paddle.distributed.sharding.group_sharded_parallel (dygraph) for stages 2 / 3")
        return True

    def _record(self, prog, cfg, context):
        group = self.get_attr('group')
        deg = self.get_attr('degree') or self.get_attr('sharding_degree')
        if deg and dist.is_initialized():
            have = group.nranks if group is not None else dist.get_world_size()
            if group is None and prog.__dict__.get('_ap_grad_sync'):
                from ..fleet.meta_optimizers import _majority_group
                g = _majority_group(prog._ap_grad_sync)
                have = g.nranks if g is not None else have
            if int(deg) != have:
                raise ValueError(f"auto_parallel_sharding: degree {deg} does not match the sharding "
                                 f"group's {have} ranks")
        cfg['sharding'] = group if group is not None else 'auto'


# -- gradient bucketing ------------------------------------------------------------------------------
@register_pass('auto_parallel_data_parallel_optimization')
class DataParallelOptimizationPass(_ProgramPass):
    """Attributes: fuse_grad_size_in_MB (flat gradient bucket size; default 32), dist_context,
    global_rank, use_sharding (accepted for API parity)."""

    def __init__(self):
        super().__init__()
        self.set_attr('dist_context', None)
        self.set_attr('global_rank', -1)
        self.set_attr('use_sharding', False)
        self.set_attr('fuse_grad_size_in_MB', 32)

    def _type(self):
        return PassType.COMM_OPT

    def _record(self, prog, cfg, context):
        cfg['bucket_mb'] = float(self.get_attr('fuse_grad_size_in_MB'))


@register_pass('fuse_all_reduce')
class FuseAllReducePass(_ProgramPass):
    """Attribute max_memory_size (bytes per fused all-reduce bucket; 0 = one per gradient)."""

    def __init__(self):
        super().__init__()
        self.set_attr('max_memory_size', -1)

    def _check_self(self):
        return int(self.get_attr('max_memory_size')) >= 0

    def _type(self):
        return PassType.COMM_OPT

    def _record(self, prog, cfg, context):
        cfg['bucket_mb'] = int(self.get_attr('max_memory_size')) / float(1 << 20)


# -- global-norm clip over a partitioned program -------------------------------------------------------
def install_dist_clip(prog, opt):
    """Make the optimizer's ClipGradByGlobalNorm see the norm of the WHOLE (unpartitioned)
    model: per parameter class (the mesh axes it is split over) the local squared norm is
    all-reduced over those axes' groups; replicated parameters count once."""
    from ...nn.clip import ClipGradByGlobalNorm
    from ...ops.fused import global_l2_norm_sq
    from ...static.graph import _inner_opt
    inner = _inner_opt(opt)
    clip = inner._grad_clip
    if not isinstance(clip, ClipGradByGlobalNorm):
        return
    dims = prog.__dict__.get('_ap_param_dims') or {}
    mesh = prog.__dict__.get('_ap_mesh')
    params = [p for p in (prog.__dict__.get('_minimize_params') or inner._parameter_list)
              if getattr(p, 'need_clip', True)]
    classes = {}
    for p in params:
        groups = []
        if mesh is not None:
            for d in sorted({d for d in dims.get(p.name, ()) if d >= 0}):
                g = mesh.axis_group(d)
                if g is not None:
                    groups.append(g)
        classes.setdefault(tuple(id(g) for g in groups), (groups, []))[1].append(p)
    order = sorted(classes)   # the same collective sequence on every rank

    def dist_norm(grad_of, sq):
        tot = None
        for key in order:
            groups, ps = classes[key]
            gs = [g for g in (grad_of(p) for p in ps) if g is not None]
            s = global_l2_norm_sq(gs) if gs else None
            s = s.reshape(()).float() if s is not None else torch.zeros((), device=sq.device)
            for g in groups:
                dist.all_reduce(s, group=g.process_group)
            tot = s if tot is None else tot + s
        return sq if tot is None else tot

    def hook(sq):
        return dist_norm(lambda p: p._t.grad, sq)
    hook.dist_norm = dist_norm
    clip._norm_hook = hook


@register_pass('auto_parallel_grad_clip')
class GradClipPass(_ProgramPass):
    """The distributed global-norm clip (see install_dist_clip); attributes dist_context and
    params_grads are accepted for API parity."""

    def __init__(self):
        super().__init__()
        self.set_attr('dist_context', None)
        self.set_attr('params_grads', [])

    def _record(self, prog, cfg, context):
        hooks = [h for h in cfg.get('minimize_hooks', []) if h is not install_dist_clip]
        cfg['minimize_hooks'] = hooks + [install_dist_clip]


def param_dims_of(prog):
    """{local parameter name: dims mapping} of a partitioned program (introspection)."""
    return dict(prog.__dict__.get('_ap_param_dims') or {})
