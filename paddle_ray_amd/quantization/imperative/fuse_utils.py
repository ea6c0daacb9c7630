"""Conv+BN / Linear+BN folding for quantization (parity:
python/paddle/quantization/imperative/fuse_utils.py fuse_layers).

``layers_to_fuse`` is a list of [conv_name, bn_name] pairs of sublayer paths. The BN's
affine transform (running statistics, eval semantics) is folded into the conv/linear
weight and bias; the BN is replaced by Identity.
"""
import copy

import torch

from ... import nn
from ...framework.core import _u


def _get(model, path):
    cur = model
    for p in path.split('.'):
        cur = cur._sub_layers[p]
    return cur


def _set(model, path, layer):
    parts = path.split('.')
    parent = model
    for p in parts[:-1]:
        parent = parent._sub_layers[p]
    parent._sub_layers[parts[-1]] = layer


@torch.no_grad()
def _fold(layer, bn):
    w = _u(layer.weight)
    mean, var = _u(bn._mean).float(), _u(bn._variance).float()
    gamma = _u(bn.weight).float() if bn.weight is not None else torch.ones_like(mean)
    beta = _u(bn.bias).float() if bn.bias is not None else torch.zeros_like(mean)
    k = gamma / torch.sqrt(var + bn._epsilon)
    if isinstance(layer, nn.Linear):  # weight [in, out]: scale output columns
        w.copy_((w.float() * k.reshape(1, -1)).to(w.dtype))
    else:  # conv weight [out, in/g, kh, kw]
        w.copy_((w.float() * k.reshape(-1, *([1] * (w.dim() - 1)))).to(w.dtype))
    b0 = _u(layer.bias).float() if layer.bias is not None else torch.zeros_like(mean)
    nb = (b0 - mean) * k + beta
    if layer.bias is None:
        layer.bias = layer.create_parameter([nb.numel()], is_bias=True)
    _u(layer.bias).copy_(nb.to(_u(layer.bias).dtype))


def fuse_layers(model, layers_to_fuse, inplace=False):
    m = model if inplace else copy.deepcopy(model)
    for pair in layers_to_fuse:
        if len(pair) != 2:
            raise ValueError("each fuse item must be [conv_or_linear_name, bn_name]")
        a, b = _get(m, pair[0]), _get(m, pair[1])
        if not isinstance(a, (nn.Conv2D, nn.Linear)) or not isinstance(
                b, (nn.BatchNorm2D, nn.BatchNorm1D, nn.BatchNorm)):
            raise TypeError(f"cannot fuse {type(a).__name__} with {type(b).__name__}")
        _fold(a, b)
        _set(m, pair[1], nn.Identity())
    return m


def find_conv_bn_pairs(model, prefix=''):
    """Adjacent (Conv2D, BatchNorm2D) children of Sequential containers."""
    pairs = []
    kids = list(model.named_children())
    for (n1, l1), (n2, l2) in zip(kids, kids[1:]):
        if isinstance(l1, nn.Conv2D) and isinstance(l2, nn.BatchNorm2D):
            pairs.append([prefix + n1, prefix + n2])
    for n, l in kids:
        pairs += find_conv_bn_pairs(l, prefix + n + '.')
    return pairs
