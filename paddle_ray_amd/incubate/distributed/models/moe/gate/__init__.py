"""MoE gates (parity: .../models/moe/gate/{base,naive,gshard,switch}_gate.py)."""
import math

import torch

from ......framework.core import Tensor, _u
from ...... import nn
from ......distributed.models.moe import utils as U


class BaseGate(nn.Layer):
    def __init__(self, num_expert, world_size):
        super().__init__()
        self.world_size = world_size
        self.num_expert = num_expert
        self.tot_expert = world_size * num_expert
        self.loss = None

    def forward(self, x):
        raise NotImplementedError("Please implement the forward function.")

    def set_loss(self, loss):
        self.loss = loss

    def get_loss(self, clear=True):
        loss = self.loss
        if clear:
            self.loss = None
        return loss


class NaiveGate(BaseGate):
    """Linear router, top-k over the raw gate logits."""

    def __init__(self, d_model, num_expert, world_size, topk=2):
        super().__init__(num_expert, world_size)
        self.gate = nn.Linear(d_model, self.tot_expert)
        self.top_k = topk

    def forward(self, inp, return_all_scores=False):
        g = _u(self.gate(inp))
        val, idx = torch.topk(g, k=self.top_k, dim=-1, largest=True, sorted=False)
        if return_all_scores:
            return Tensor(val), Tensor(idx), Tensor(g)
        return Tensor(val), Tensor(idx)


def limit_by_capacity(topk_idx, num_expert, world_size, capacity, group=None):
    """Drop routes beyond each expert's capacity (lower ranks first); returns
    (new_local_count, new_global_count, pruned_topk_idx)."""
    from ......distributed.utils.moe_utils import _a2a
    with torch.no_grad():
        idx = _u(topk_idx)
        cap = torch.full((num_expert,), int(capacity), dtype=torch.int64, device=idx.device)
        lec = _u(U._number_count(idx, num_expert * world_size)).long()
        if world_size > 1:
            gec = _a2a(lec, lec.numel(), [num_expert] * world_size, [num_expert] * world_size,
                       group)
        else:
            gec = lec
        new_gec = _u(U._limit_by_capacity(gec, cap, world_size))
        if world_size > 1:
            new_lec = _a2a(new_gec, new_gec.numel(), [num_expert] * world_size,
                           [num_expert] * world_size, group)
        else:
            new_lec = new_gec
        pruned = _u(U._prune_gate_by_capacity(idx, new_lec, num_expert, world_size))
    return Tensor(new_lec), Tensor(new_gec), Tensor(pruned)


class GShardGate(NaiveGate):
    """Top-2 gate with the GShard load-balancing loss, capacity limit and random routing."""

    def __init__(self, d_model, num_expert, world_size, topk=2, capacity=(1.2, 2.4),
                 random_routing=True, group=None):
        assert topk == 2, "topk should be 2 in gshard"
        super().__init__(d_model, num_expert, world_size)
        self.capacity = capacity
        self.random_routing = random_routing
        self.group = group

    def forward(self, x):
        topk_val, topk_idx, gate_score = super().forward(x, return_all_scores=True)
        gs = _u(gate_score)
        s = gs.shape[0]
        top1 = _u(topk_idx).reshape(-1).long()
        c_e = torch.bincount(top1, minlength=self.tot_expert)[:self.tot_expert].float() / s
        m_e = torch.softmax(gs.float(), dim=1).mean(0)
        self.set_loss(Tensor((c_e * m_e).mean() * (self.num_expert ** 2)))
        cap_rate = self.capacity[0 if self.training else 1]
        capacity = math.ceil(cap_rate * x.shape[0])
        _, _, topk_idx = limit_by_capacity(topk_idx, self.num_expert, self.world_size, capacity,
                                           group=self.group)
        if self.random_routing:
            prob = torch.rand(gs.shape[0], device=gs.device)
            topk_idx = U._random_routing(topk_idx, topk_val, Tensor(prob))
        return topk_val, topk_idx


class SwitchGate(NaiveGate):
    """Top-1 Switch-Transformer gate (multiplicative jitter, capacity, balance loss)."""

    def __init__(self, d_model, num_expert, world_size, topk=1, switch_eps=0.1,
                 capacity=(1.2, 2.4), group=None):
        assert topk == 1, "topk should be 1 in switch"
        super().__init__(d_model, num_expert, world_size, topk=1)
        self.switch_eps = switch_eps
        self.capacity = capacity
        self.group = group

    def forward(self, inp):
        score = _u(self.gate(inp))
        if self.training:
            noise = torch.rand_like(score) * 2 * self.switch_eps + 1.0 - self.switch_eps
            score = score + noise
        score = torch.softmax(score.float(), dim=-1).to(score.dtype)
        top1_score, top1_idx = torch.topk(score, k=1, dim=-1, largest=True)
        cap_rate = self.capacity[0 if self.training else 1]
        capacity = math.ceil(cap_rate * inp.shape[0])
        _, _, top1_idx = limit_by_capacity(Tensor(top1_idx), self.num_expert, self.world_size,
                                           capacity, group=self.group)
        ti = _u(top1_idx)
        valid = ti[ti > -1]
        n = max(valid.numel(), 1)
        frac = torch.bincount(valid.long(), minlength=self.tot_expert)[:self.tot_expert].float() / n
        prob = score.float().sum(0) / n
        self.set_loss(Tensor((frac * prob).sum() * self.tot_expert))
        return Tensor(top1_score), top1_idx
