import torch.utils.dlpack as _dl

from ..framework.core import Tensor, _u


def to_dlpack(x):
    return _dl.to_dlpack(_u(x))


def from_dlpack(dlpack):
    return Tensor(_dl.from_dlpack(dlpack))
