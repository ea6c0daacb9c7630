"""paddle.incubate (parity: python/paddle/incubate/__init__.py)."""
from . import nn  # noqa
from . import autograd  # noqa
from . import autotune  # noqa
from . import distributed  # noqa
from . import optimizer  # noqa
from .optimizer import LookAhead, ModelAverage, DistributedFusedLamb  # noqa
from .nn.functional import fused_dropout_add  # noqa
from ..geometric import (segment_sum, segment_mean, segment_max, segment_min,  # noqa
                         send_u_recv as graph_send_recv, reindex_graph as graph_reindex,
                         sample_neighbors as graph_sample_neighbors)


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
