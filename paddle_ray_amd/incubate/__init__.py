"""paddle.incubate (parity: python/paddle/incubate/__init__.py)."""
from . import nn  # noqa
from . import autograd  # noqa
from . import autotune  # noqa
from . import distributed  # noqa
from . import optimizer  # noqa
from . import asp, checkpoint, multiprocessing, passes  # noqa
from .checkpoint import auto_checkpoint  # noqa
from .passes import fuse_resnet_unit_pass  # noqa
from .nn.loss import identity_loss  # noqa
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


def graph_khop_sampler(row, colptr, input_nodes, sample_sizes, sorted_eids=None,
                       return_eids=False, name=None):
    """Multi-hop neighbor sampling over a CSC graph (parity: python/paddle/incubate/
    operators/graph_khop_sampler.py): hop h samples ``sample_sizes[h]`` neighbors of the
    previous hop's new nodes. Returns (edge_src, edge_dst, sample_index, reindex_nodes
    [, edge_eids]) with every node renumbered (input nodes first)."""
    import numpy as np
    import torch
    from ..framework.core import Tensor, _u
    from ..geometric import sample_neighbors
    frontier = _u(input_nodes)
    srcs, dsts, eids = [], [], []
    for size in sample_sizes:
        if frontier.numel() == 0:
            break
        res = sample_neighbors(row, colptr, Tensor(frontier), sample_size=size,
                               eids=sorted_eids, return_eids=return_eids)
        nb, cnt = _u(res[0]), _u(res[1])
        srcs.append(nb)
        dsts.append(torch.repeat_interleave(frontier, cnt.long()))
        if return_eids:
            eids.append(_u(res[2]))
        seen = set(torch.cat([_u(input_nodes)] + srcs[:-1]).tolist()) if len(srcs) > 1 \
            else set(_u(input_nodes).tolist())
        new = [v for v in dict.fromkeys(nb.tolist()) if v not in seen]
        frontier = torch.tensor(new, dtype=frontier.dtype, device=frontier.device)
    src = torch.cat(srcs) if srcs else torch.zeros(0, dtype=_u(row).dtype)
    dst = torch.cat(dsts) if dsts else torch.zeros(0, dtype=_u(row).dtype)
    order = {int(v): i for i, v in enumerate(_u(input_nodes).tolist())}
    for v in torch.cat([src, dst]).tolist():
        order.setdefault(int(v), len(order))
    remap = lambda t: torch.tensor([order[int(v)] for v in t.tolist()],  # noqa: E731
                                   dtype=torch.int64, device=t.device)
    sample_index = torch.tensor(list(order.keys()), dtype=torch.int64)
    out = (Tensor(remap(src)), Tensor(remap(dst)), Tensor(sample_index),
           Tensor(torch.arange(len(_u(input_nodes)), dtype=torch.int64)))
    if return_eids:
        out = out + (Tensor(torch.cat(eids) if eids else torch.zeros(0, dtype=torch.int64)),)
    return out


from . import operators  # noqa: E402  (re-exports the functions above)
from .operators import ResNetUnit, resnet_unit, unzip  # noqa: E402,F401
