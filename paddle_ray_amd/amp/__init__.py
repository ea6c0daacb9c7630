"""paddle.amp (parity: python/paddle/amp/{auto_cast,grad_scaler}.py).

O1: per-op autocast (GEMM/conv in bf16/fp16, reductions/softmax/norm in fp32)
via PyTorch-ROCm's autocast dispatch; our HIP ops accept low-precision inputs
and accumulate in fp32 internally. O2: ``decorate`` casts parameters to the
low-precision dtype and switches optimizers to fp32 master weights.
GradScaler: dynamic loss scaling with on-device found_inf (no host sync
except the one read that decides whether to skip the step).
"""
import contextlib

import torch

from ..framework.core import Tensor, _u, convert_dtype, _default_device

WHITE_LIST = {'matmul', 'conv2d', 'linear', 'bmm', 'mul'}
BLACK_LIST = {'softmax', 'cross_entropy', 'layer_norm', 'exp', 'log', 'mean', 'sum'}

_amp_state = {'enabled': False, 'dtype': torch.float16, 'level': 'O1',
              'white': frozenset(), 'black': frozenset()}


def amp_state():
    return dict(_amp_state)


def _cast_args(args, kwargs, dt):
    def c(a):
        if isinstance(a, Tensor):
            t = a._t
            return Tensor(t.to(dt)) if t.is_floating_point() and t.dtype != dt else a
        if isinstance(a, torch.Tensor):
            return a.to(dt) if a.is_floating_point() and a.dtype != dt else a
        if isinstance(a, (list, tuple)):
            return type(a)(c(x) for x in a)
        return a
    return [c(a) for a in args], {k: c(v) for k, v in kwargs.items()}


def amp_op(name):
    """Per-op AMP policy for paddle ops (parity: auto_cast.py:135-161 custom lists, :450 O2).

    Inside ``auto_cast``: an op in the custom black list runs in fp32 (inputs up-cast,
    autocast off); an op in the custom white list runs in the AMP dtype (inputs down-cast,
    autocast off); anything else follows the default policy (PyTorch-ROCm autocast dispatch
    for O1; under O2 the parameters are already low precision)."""
    def deco(fn):
        def wrapped(*args, **kwargs):
            st = _amp_state
            if not st['enabled'] or (name not in st['black'] and name not in st['white']):
                return fn(*args, **kwargs)
            dt = torch.float32 if name in st['black'] else st['dtype']
            a, k = _cast_args(args, kwargs, dt)
            with torch.autocast(device_type=_default_device().type, enabled=False):
                return fn(*a, **k)
        wrapped.__name__ = fn.__name__
        wrapped.__doc__ = fn.__doc__
        wrapped.__wrapped__ = fn
        return wrapped
    return deco


@contextlib.contextmanager
def auto_cast(enable=True, custom_white_list=None, custom_black_list=None, level='O1',
              dtype='float16', use_promote=True):
    dt = convert_dtype(dtype)
    prev = dict(_amp_state)
    white = frozenset(custom_white_list or ())
    black = frozenset(custom_black_list or ())
    if white & black:
        raise ValueError(f"ops in both custom_white_list and custom_black_list: {sorted(white & black)}")
    _amp_state.update(enabled=bool(enable), dtype=dt, level=level, white=white, black=black)
    dev = _default_device().type
    try:
        if enable and level in ('O1', 'O2'):
            with torch.autocast(device_type=dev, dtype=dt if dev == 'cuda' else torch.bfloat16,
                                enabled=True):
                yield
        else:
            yield
    finally:
        _amp_state.clear()
        _amp_state.update(prev)


amp_guard = auto_cast


def decorate(models, optimizers=None, level='O1', dtype='float16', master_weight=None,
             save_dtype=None, master_grad=False, excluded_layers=None):
    dt = convert_dtype(dtype)
    if level == 'O2':
        from ..nn.layer.norm import _BatchNormBase, LayerNorm
        ms = models if isinstance(models, (list, tuple)) else [models]
        excl = tuple(excluded_layers) if excluded_layers else ()
        for m in ms:
            for sub in m.sublayers(include_self=True):
                if isinstance(sub, (_BatchNormBase, LayerNorm)) or (excl and isinstance(sub, excl)):
                    continue
                for n, p in list(sub._parameters.items()):
                    if p is not None and p._t.is_floating_point():
                        rg = p._t.requires_grad
                        object.__setattr__(p, '_t', p._t.detach().to(dt).requires_grad_(rg))
        if optimizers is not None:
            os_ = optimizers if isinstance(optimizers, (list, tuple)) else [optimizers]
            for o in os_:
                o._multi_precision = True if master_weight is None else bool(master_weight)
                o._fused_plan = None
    if optimizers is None:
        return models
    return models, optimizers


class AmpScaler:
    def __init__(self, enable=True, init_loss_scaling=2. ** 15, incr_ratio=2.0, decr_ratio=0.5,
                 incr_every_n_steps=1000, decr_every_n_nan_or_inf=2,
                 use_dynamic_loss_scaling=True):
        self._enable = enable
        self._scale = float(init_loss_scaling) if enable else 1.0
        self._incr_ratio, self._decr_ratio = incr_ratio, decr_ratio
        self._incr_every, self._decr_every = incr_every_n_steps, decr_every_n_nan_or_inf
        self._dynamic = use_dynamic_loss_scaling
        self._good, self._bad = 0, 0
        self._found_inf = False
        self._unscaled = set()
        self._extra_pgs = []

    def is_enable(self):
        return self._enable

    def is_use_dynamic_loss_scaling(self):
        return self._dynamic

    def get_loss_scaling(self):
        return self._scale

    def set_init_loss_scaling(self, v):
        self._scale = float(v)

    def scale(self, var):
        if not self._enable:
            return var
        return Tensor(_u(var) * self._scale)

    def unscale_(self, optimizer):
        """Unscale the gradients the optimizer will actually apply and decide found_inf.

        Sharded optimizers expose their owned gradient shards (``_scaler_grads``) — with
        stage 2/3 those, not ``p.grad``, are what the update reads. found_inf is MAX-reduced
        over every group the optimizer spans (``_found_inf_groups``: sharding, dp, mp, pp)
        so all ranks skip or take the step together (parity:
        hybrid_parallel_gradscaler.py:72-81, group_sharded_utils GroupShardedScaler)."""
        if not self._enable or id(optimizer) in self._unscaled:
            return
        get = getattr(optimizer, '_scaler_grads', None)
        grads = get() if get is not None else \
            [p._t.grad for p in optimizer._parameter_list if p._t.grad is not None]
        grads = [g for g in grads if g is not None and g.numel() > 0]
        pgs = list(getattr(optimizer, '_found_inf_groups', lambda: [])()) + list(self._extra_pgs)
        if not grads and not pgs:
            self._found_inf = False
            return
        dev = grads[0].device if grads else _default_device()
        found = torch.zeros(1, device=dev)
        inv = torch.full((1,), 1.0 / self._scale, device=dev)
        by_dt = {}
        for g in grads:
            by_dt.setdefault((g.device, g.dtype), []).append(g)
        for (gdev, _), gs in by_dt.items():
            f = found if gdev == dev else torch.zeros(1, device=gdev)
            torch._amp_foreach_non_finite_check_and_unscale_(gs, f, inv.to(gdev))
            if f is not found:
                found.add_(f.to(dev))
        if pgs:
            import torch.distributed as dist
            for pg in _uniq(pgs):
                dist.all_reduce(found, op=dist.ReduceOp.MAX, group=pg)
        self._found_inf = bool(found.item())
        self._unscaled.add(id(optimizer))

    def minimize(self, optimizer, *args, **kwargs):
        self.step(optimizer)
        self.update()
        return None, None

    def step(self, optimizer):
        if not self._enable:
            optimizer.step()
            return
        self.unscale_(optimizer)
        if not self._found_inf:
            optimizer.step()

    def update(self):
        if not (self._enable and self._dynamic):
            self._unscaled.clear()
            return
        if self._found_inf:
            self._bad += 1
            self._good = 0
            if self._bad >= self._decr_every:
                self._scale = max(self._scale * self._decr_ratio, 1.0)
                self._bad = 0
        else:
            self._good += 1
            self._bad = 0
            if self._good >= self._incr_every:
                self._scale *= self._incr_ratio
                self._good = 0
        self._found_inf = False
        self._unscaled.clear()

    def state_dict(self):
        return {'scale': self._scale, 'incr_ratio': self._incr_ratio,
                'decr_ratio': self._decr_ratio, 'incr_count': self._good,
                'decr_count': self._bad, 'use_dynamic_loss_scaling': self._dynamic}

    def load_state_dict(self, sd):
        self._scale = float(sd['scale'])
        self._good, self._bad = sd.get('incr_count', 0), sd.get('decr_count', 0)

    set_state_dict = load_state_dict


class GradScaler(AmpScaler):
    def __init__(self, enable=True, init_loss_scaling=2. ** 16, incr_ratio=2.0, decr_ratio=0.5,
                 incr_every_n_steps=2000, decr_every_n_nan_or_inf=1,
                 use_dynamic_loss_scaling=True):
        super().__init__(enable, init_loss_scaling, incr_ratio, decr_ratio, incr_every_n_steps,
                         decr_every_n_nan_or_inf, use_dynamic_loss_scaling)


def _uniq(pgs):
    out, seen = [], set()
    for pg in pgs:
        if id(pg) not in seen:
            seen.add(id(pg))
            out.append(pg)
    return out


class ShardedGradScaler(GradScaler):
    """GroupShardedScaler parity: a GradScaler bound to a ShardedState — unscales the owned
    gradient shards and MAX-reduces found_inf over the sharding (and dp) groups."""

    @staticmethod
    def wrap(scaler, state):
        pgs = [state.pg if state.world > 1 else None, state.dp_pg if state.dp_world > 1 else None]
        scaler._extra_pgs = _uniq(list(scaler._extra_pgs) + [p for p in pgs if p is not None])
        return scaler


GroupShardedScaler = ShardedGradScaler


def is_float16_supported(device=None):
    return True


def is_bfloat16_supported(device=None):
    return True
from . import debugging  # noqa: E402
