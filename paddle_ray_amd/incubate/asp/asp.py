"""Automatic SParsity for dygraph models (parity: python/paddle/incubate/asp/asp.py,
supported_layer_list.py).

prune_model() applies an n:m mask to every supported layer weight (Linear / Conv2D by
default, minus excluded names) and remembers the masks; decorate(optimizer) returns an
optimizer whose step() re-applies them so the sparsity pattern survives training.
"""
import logging
import threading

import numpy as np
import torch

from ...framework.core import _u
from . import utils as U

_logger = logging.getLogger(__name__)
_lock = threading.Lock()
supported_layers_and_prune_func_map = {}
_excluded = set()
_masks = {}  # id(param) -> (param, torch mask)


def _default_pruning(weight_nparray, m, n, func_name, param_name):
    shape = weight_nparray.shape
    if (len(shape) == 2 and shape[0] < m) or (len(shape) == 4 and shape[1] < m):
        _logger.warning(f"{param_name} is not pruned: its reduction dimension {shape} < {m}")
        return weight_nparray.copy(), np.ones_like(weight_nparray)
    # prune along the GEMM reduction dimension (rows of W^T for an [in, out] Linear weight)
    mask = U.create_mask(weight_nparray.T, func_name=func_name, n=n, m=m).T
    pruned = weight_nparray * mask
    assert U.check_sparsity(pruned.T, n=n, m=m,
                            func_name=U.CheckMethod.get_checking_method(func_name)), \
        f'Pruning {param_name} weight matrix failure!!!'
    return pruned, mask


def add_supported_layer(layer, pruning_func=None):
    """Register a Layer class (or a parameter-name prefix string) as prunable."""
    from ...nn import Layer
    if isinstance(layer, str):
        name = layer
    elif isinstance(layer, type) and issubclass(layer, Layer):
        name = layer.__name__
    elif isinstance(layer, Layer):
        name = type(layer).__name__
    else:
        raise TypeError("layer must be a str, a Layer subclass or a Layer instance")
    with _lock:
        supported_layers_and_prune_func_map[name] = pruning_func


def _init_defaults():
    if not supported_layers_and_prune_func_map:
        for n in ('Linear', 'Conv2D', 'ColumnParallelLinear', 'RowParallelLinear'):
            supported_layers_and_prune_func_map[n] = None


def set_excluded_layers(param_names, main_program=None):
    _excluded.update(param_names)


def reset_excluded_layers(main_program=None):
    _excluded.clear()


def _prunable(model):
    _init_defaults()
    for lname, layer in model.named_sublayers(include_self=True):
        kind = type(layer).__name__
        if kind not in supported_layers_and_prune_func_map:
            continue
        w = getattr(layer, 'weight', None)
        if w is None:
            continue
        full = f'{lname}.weight' if lname else 'weight'
        if full in _excluded or getattr(w, 'name', None) in _excluded or lname in _excluded:
            continue
        yield full, w, supported_layers_and_prune_func_map[kind]


def prune_model(model, n=2, m=4, mask_algo='mask_1d', with_mask=True):
    """Prune every supported weight of ``model`` in place; returns {param name: mask}."""
    algo = {'mask_1d': U.MaskAlgo.MASK_1D, 'mask_2d_greedy': U.MaskAlgo.MASK_2D_GREEDY,
            'mask_2d_best': U.MaskAlgo.MASK_2D_BEST}[mask_algo] \
        if isinstance(mask_algo, str) else mask_algo
    out = {}
    for name, w, fn in _prunable(model):
        t = _u(w)
        arr = t.detach().float().cpu().numpy()
        pruned, mask = (fn or _default_pruning)(arr, m, n, algo, name)
        with torch.no_grad():
            t.copy_(torch.from_numpy(np.asarray(pruned)).to(t.dtype))
        mt = torch.from_numpy(np.asarray(mask, np.float32)).to(t.device, t.dtype)
        if with_mask:
            _masks[id(w)] = (w, mt)
        out[name] = mask
    return out


class OptimizerWithSparsityGuarantee:
    """Wraps an optimizer: after every step the pruned weights are re-masked."""

    def __init__(self, optimizer):
        self._optimizer = optimizer

    def __getattr__(self, item):
        return getattr(self._optimizer, item)

    @torch.no_grad()
    def _apply_masks(self):
        for w, mask in _masks.values():
            _u(w).mul_(mask)

    def step(self):
        self._optimizer.step()
        self._apply_masks()

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        res = self._optimizer.minimize(loss, startup_program, parameters, no_grad_set)
        self._apply_masks()
        return res

    def state_dict(self):
        return self._optimizer.state_dict()

    def set_state_dict(self, sd):
        return self._optimizer.set_state_dict(sd)


def decorate(optimizer):
    return OptimizerWithSparsityGuarantee(optimizer)
