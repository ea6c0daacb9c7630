"""ClipGradForMOEByGlobalNorm (parity: .../models/moe/grad_clip.py): global-norm clipping
where the expert parameters' squared norm is summed over the MoE group (each rank holds
different experts) before being added to the replicated parameters' norm."""
import torch
import torch.distributed as dist

from .....framework.core import _u
from .....nn.clip import ClipGradByGlobalNorm
from .....ops import fused as K


class ClipGradForMOEByGlobalNorm(ClipGradByGlobalNorm):
    def __init__(self, clip_norm, is_expert_param_func=None, moe_group=None,
                 group_name="default_moe_group"):
        super().__init__(clip_norm, group_name)
        self.moe_group = moe_group
        if moe_group is not None and moe_group.nranks > 1:
            assert is_expert_param_func is not None, \
                "When moe group size > 1, a function for selecting expert params must be specified."
        self.is_expert_param_func = is_expert_param_func

    def __str__(self):
        return "Gradient Clip By GlobalNorm, global_norm=%f" % (self.clip_norm)

    def _split(self, params_grads):
        normal, expert = [], []
        for p, g in params_grads:
            if g is None or not getattr(p, 'need_clip', True):
                continue
            if self.is_expert_param_func is not None and self.is_expert_param_func(p):
                expert.append(_u(g))
            else:
                normal.append(_u(g))
        return normal, expert

    def coefficient_from_params(self, params_grads):
        """0-d device tensor clip_norm / max(global_norm, clip_norm), or None."""
        normal, expert = self._split(params_grads)
        sq = K.global_l2_norm_sq(normal)
        esq = K.global_l2_norm_sq(expert)
        if esq is not None and self.moe_group is not None and self.moe_group.nranks > 1:
            esq = esq.clone()
            dist.all_reduce(esq, group=getattr(self.moe_group, 'process_group', None))
        tot = sq if esq is None else (esq if sq is None else sq + esq.to(sq.device))
        if tot is None:
            return None
        if self._norm_hook is not None:
            tot = self._norm_hook(tot)
        return self.clip_norm / torch.clamp(torch.sqrt(tot), min=self.clip_norm)

    def _dygraph_clip(self, params_grads):
        c = self.coefficient_from_params(params_grads)
        if c is not None:
            normal, expert = self._split(params_grads)
            for g in normal + expert:
                g.mul_(c.to(g.dtype))
        return params_grads
