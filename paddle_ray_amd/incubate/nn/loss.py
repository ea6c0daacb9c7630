"""identity_loss (parity: python/paddle/incubate/nn/loss.py): marks a tensor as the loss
(reduction 'sum'/0, 'mean'/1, 'none'/2)."""
from ...framework.core import Tensor, _u


def identity_loss(x, reduction='none'):
    if isinstance(reduction, str):
        reduction = {'sum': 0, 'mean': 1, 'none': 2}.get(reduction.lower())
    if reduction not in (0, 1, 2):
        raise ValueError("reduction must be 'sum', 'mean', 'none' or 0/1/2")
    t = _u(x)
    return Tensor(t.sum() if reduction == 0 else t.mean() if reduction == 1 else t)
