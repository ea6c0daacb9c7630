"""NaN/Inf checker (parity: FLAGS_check_nan_inf in paddle/fluid/framework/operator.cc:1668,
new_executor/interpretercore.cc:902 and paddle/fluid/eager/nan_inf_utils.cc).

Every op's floating outputs are checked after it runs:
* torch ops — through a ``TorchDispatchMode`` pushed while the flag is on (this sees the
  forward AND the autograd backward ops, like the reference's per-kernel check);
* our HIP kernels — the kernel registry calls ``check_outputs`` on their results.
Level 0 raises ``RuntimeError`` naming the op; level >= 1 only logs (count of NaN / Inf,
max |x|). The check is a device reduction + host sync per op: a debugging tool.
"""
import logging

import torch
from torch.utils._python_dispatch import TorchDispatchMode

_log = logging.getLogger('paddle_ray_amd.nan_inf')
_state = {'mode': None, 'level': 0, 'skip': set()}


def _check(name, t):
    if not isinstance(t, torch.Tensor) or not t.is_floating_point() or t.numel() == 0 \
            or t.device.type == 'meta':
        return
    finite = torch.isfinite(t)
    if bool(finite.all()):
        return
    n_nan = int(torch.isnan(t).sum())
    n_inf = int(torch.isinf(t).sum())
    msg = (f"[check_nan_inf] op {name}: output {tuple(t.shape)} {t.dtype} has {n_nan} NaN "
           f"and {n_inf} Inf values")
    if _state['level'] == 0:
        raise RuntimeError(msg)
    _log.warning(msg)


def check_outputs(name, out):
    if _state['mode'] is None or name in _state['skip']:
        return out
    if isinstance(out, torch.Tensor):
        _check(name, out)
    elif isinstance(out, (list, tuple)):
        for o in out:
            check_outputs(name, o)
    return out


class _NanInfMode(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = str(func.overloadpacket.__name__)
        if name not in _state['skip'] and not name.startswith(('isfinite', 'isnan', 'isinf',
                                                                 'all', 'sum', 'empty')):
            flat = out if isinstance(out, (list, tuple)) else (out,)
            for o in flat:
                _check(name, o)
        return out


def enable(level=0, skip_ops=()):
    _state['level'] = int(level)
    _state['skip'] = set(skip_ops)
    if _state['mode'] is None:
        m = _NanInfMode()
        m.__enter__()
        _state['mode'] = m


def disable():
    m = _state['mode']
    if m is not None:
        _state['mode'] = None
        m.__exit__(None, None, None)


def enabled():
    return _state['mode'] is not None
