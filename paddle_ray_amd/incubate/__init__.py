"""paddle.incubate (parity: python/paddle/incubate/__init__.py)."""
from . import nn  # noqa
from . import autograd  # noqa
from .nn.functional import fused_dropout_add  # noqa


def softmax_mask_fuse(x, mask, name=None):
    from ..framework.core import Tensor, _u
    from ..ops import fused as K
    return Tensor(K.softmax_lastdim(_u(x) + _u(mask)))


def softmax_mask_fuse_upper_triangle(x):
    import torch
    from ..framework.core import Tensor, _u
    from ..ops import fused as K
    t = _u(x)
    S = t.shape[-1]
    m = torch.triu(torch.full((S, S), float('-inf'), device=t.device, dtype=t.dtype), 1)
    return Tensor(K.softmax_lastdim(t + m))
