"""Pickling reductions for framework Tensors across processes (parity:
python/paddle/incubate/multiprocessing/reductions.py)."""
from multiprocessing.reduction import ForkingPickler

import torch.multiprocessing  # noqa: F401  (registers torch.Tensor shared-memory reductions)

from ...framework.core import Parameter, Tensor


def _rebuild_tensor(cls, data, stop_gradient, name):
    if issubclass(cls, Parameter):
        return cls(data, trainable=not stop_gradient, name=name)
    return cls(data, stop_gradient=stop_gradient, name=name)


def _reduce_tensor(t):
    data = t._t.detach()
    if not data.is_cuda:
        data = data.share_memory_()
    return _rebuild_tensor, (type(t), data, t.stop_gradient, getattr(t, 'name', None))


def init_reductions():
    for cls in (Tensor, Parameter):
        ForkingPickler.register(cls, _reduce_tensor)
