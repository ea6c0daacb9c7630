"""Gradient clipping (parity: python/paddle/nn/clip.py).

ClipGradByGlobalNorm computes the global norm with the fused multi-tensor
sum-of-squares kernel and folds the clip coefficient into the optimizer's
fused update (``grad_scale``) instead of rewriting every gradient.
"""
import torch

from ..framework.core import Tensor, _u
from ..ops import fused as K


class ClipGradBase:
    def __call__(self, params_grads):
        return self._dygraph_clip(params_grads)


class ClipGradByValue(ClipGradBase):
    def __init__(self, max, min=None):
        self.max = max
        self.min = -max if min is None else min

    def _dygraph_clip(self, params_grads):
        out = []
        for p, g in params_grads:
            if g is not None and getattr(p, 'need_clip', True):
                _u(g).clamp_(self.min, self.max)
            out.append((p, g))
        return out


class ClipGradByNorm(ClipGradBase):
    def __init__(self, clip_norm):
        self.clip_norm = clip_norm

    def _dygraph_clip(self, params_grads):
        for p, g in params_grads:
            if g is None or not getattr(p, 'need_clip', True):
                continue
            t = _u(g)
            n = t.float().norm()
            t.mul_((self.clip_norm / torch.maximum(n, torch.tensor(self.clip_norm,
                                                                   device=n.device))).to(t.dtype))
        return params_grads


class ClipGradByGlobalNorm(ClipGradBase):
    def __init__(self, clip_norm, group_name="default_group", auto_skip_clip=False):
        self.clip_norm = float(clip_norm)
        self.group_name = group_name
        self._norm_hook = None  # distributed wrappers install a cross-rank reduction here

    def global_norm_sq(self, grads):
        sq = K.global_l2_norm_sq(grads)
        if sq is None:
            return None
        if self._norm_hook is not None:
            sq = self._norm_hook(sq)
        return sq

    def coefficient(self, grads):
        """Returns a 0-d tensor = clip_norm / max(global_norm, clip_norm) (stays on device)."""
        sq = self.global_norm_sq(grads)
        if sq is None:
            return None
        gn = torch.sqrt(sq)
        return self.clip_norm / torch.clamp(gn, min=self.clip_norm)

    def _dygraph_clip(self, params_grads):
        grads = [_u(g) for p, g in params_grads if g is not None and getattr(p, 'need_clip', True)]
        c = self.coefficient(grads)
        if c is not None:
            for g in grads:
                g.mul_(c.to(g.dtype))
        return params_grads


def clip_grad_norm_(parameters, max_norm, norm_type=2.0, error_if_nonfinite=False):
    ps = [p for p in (parameters if isinstance(parameters, (list, tuple)) else [parameters])
          if p.grad is not None]
    gs = [_u(p)._t.grad if isinstance(p, Tensor) else p.grad for p in ps]
    gs = [p._t.grad for p in ps]
    total = torch.nn.utils.clip_grad_norm_([p._t for p in ps], max_norm, norm_type,
                                           error_if_nonfinite)
    return Tensor(total)


def clip_grad_value_(parameters, clip_value):
    ps = parameters if isinstance(parameters, (list, tuple)) else [parameters]
    torch.nn.utils.clip_grad_value_([p._t for p in ps], clip_value)
