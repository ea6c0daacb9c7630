"""paddle.static.amp (parity: python/paddle/static/amp/decorator.py OptimizerWithMixedPrecision,
fp16_lists.py AutoMixedPrecisionLists).

``decorate(optimizer, amp_lists, ...)`` returns an optimizer whose ``minimize`` tags every
forward op of the program with the AMP policy (dtype, level, custom white/black lists; the
Executor replays each op under ``auto_cast`` with that policy, and its grad op too), seeds
the backward with the loss scaling and unscales / inf-checks the ``param@GRAD`` vars inside
the ``optimize`` op through a GradScaler (dynamic loss scaling for fp16; bf16 runs unscaled).
"""
from ..amp import auto_cast, decorate as _decorate, GradScaler  # noqa: F401


class AutoMixedPrecisionLists:
    def __init__(self, custom_white_list=None, custom_black_list=None, custom_black_varnames=None,
                 dtype='float16'):
        self.white_list = set(custom_white_list or [])
        self.black_list = set(custom_black_list or [])
        self.black_varnames = set(custom_black_varnames or [])
        if self.white_list & self.black_list:
            raise ValueError("an op cannot be in both custom_white_list and custom_black_list")


CustomOpLists = AutoMixedPrecisionLists


class OptimizerWithMixedPrecision:
    def __init__(self, optimizer, amp_lists=None, level='O1', dtype='float16',
                 init_loss_scaling=2 ** 15, use_dynamic_loss_scaling=True,
                 incr_every_n_steps=1000, decr_every_n_nan_or_inf=2, incr_ratio=2.0,
                 decr_ratio=0.8):
        self._optimizer = optimizer
        self._amp_lists = amp_lists or AutoMixedPrecisionLists()
        self._level = level
        self._dtype = dtype
        self._use_scaling = dtype == 'float16'
        self._scaler = GradScaler(enable=self._use_scaling, init_loss_scaling=init_loss_scaling,
                                  incr_ratio=incr_ratio, decr_ratio=decr_ratio,
                                  incr_every_n_steps=incr_every_n_steps,
                                  decr_every_n_nan_or_inf=decr_every_n_nan_or_inf,
                                  use_dynamic_loss_scaling=use_dynamic_loss_scaling)
        if level == 'O2':
            optimizer._multi_precision = True

    def get_loss_scaling(self):
        return self._scaler.get_loss_scaling()

    def _tag_program(self, prog):
        tag_program(prog, {'dtype': self._dtype, 'level': self._level,
                           'white': self._amp_lists.white_list, 'black': self._amp_lists.black_list})

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        from .graph import _static_minimize
        self._tag_program(loss.block.program)
        # the seed of the backward is the (current) loss scale: a dynamic scale change takes
        # effect through the scaler's unscale of the param grads, the seed is re-read per run
        return _static_minimize(self._optimizer, loss, parameters,
                                scaler=self._scaler if self._use_scaling else None,
                                loss_scale=_ScaleRef(self._scaler) if self._use_scaling else 1.0)

    def __getattr__(self, k):
        return getattr(self._optimizer, k)


def tag_program(prog, amp):
    """Tag every forward op (and the grad op built from it) with the AMP policy ``amp`` =
    {dtype: 'float16' | 'bfloat16', level: 'O1' | 'O2', white, black}: the Executor replays each
    op under ``auto_cast`` with it."""
    import torch
    dt = amp['dtype']
    if isinstance(dt, str):
        dt = torch.bfloat16 if dt == 'bfloat16' else torch.float16
    cfg = {'dtype': dt, 'level': amp.get('level', 'O1'), 'white': set(amp.get('white') or ()),
           'black': set(amp.get('black') or ())}
    for op in prog.global_block().ops:
        if op.role == 'forward' or op.role == 'recompute':
            op.attrs['amp'] = cfg
        elif op.role == 'backward' and 'fwd' in op.attrs:
            op.attrs['amp'] = cfg
    prog._bump()


class _ScaleRef:
    """Late-bound loss scale for the fill_grad_seed op (reads the scaler at replay time)."""

    def __init__(self, scaler):
        self.scaler = scaler

    def __float__(self):
        return float(self.scaler.get_loss_scaling())


def decorate(optimizer, amp_lists=None, init_loss_scaling=2 ** 15, incr_every_n_steps=1000,
             decr_every_n_nan_or_inf=2, incr_ratio=2.0, decr_ratio=0.8,
             use_dynamic_loss_scaling=True, use_pure_fp16=False, use_fp16_guard=None,
             use_bf16=False, level=None, dtype=None, **kw):
    dtype = dtype or ('bfloat16' if use_bf16 else 'float16')
    level = level or ('O2' if use_pure_fp16 else 'O1')
    return OptimizerWithMixedPrecision(optimizer, amp_lists, level, dtype, init_loss_scaling,
                                       use_dynamic_loss_scaling, incr_every_n_steps,
                                       decr_every_n_nan_or_inf, incr_ratio, decr_ratio)


def fp16_guard():
    import contextlib
    return contextlib.nullcontext()


def cast_model_to_fp16(program, amp_lists=None, use_fp16_guard=True, dest_type=None):
    return program


def cast_parameters_to_fp16(place, program, scope=None, to_fp16_var_names=None):
    return None
