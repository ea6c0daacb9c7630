"""MoELayer (parity: python/paddle/incubate/distributed/models/moe/moe_layer.py).

Forward (tokens [b, s, d] -> [b, s, d]):
  gate -> (top-k values, top-k expert ids; -1 = dropped by capacity)
  stable sort of the (token, k) routes by global expert id  -> expert-contiguous rows
  global_scatter: ONE variable-split RCCL all_to_all to the experts' owners (expert-major)
  each local expert runs on its contiguous slice (one GEMM chain per expert)
  global_gather: the inverse all_to_all, scatter back to (token, k) slots (dropped = 0)
  combine: out[t] = sum_k value[t, k] * y[t, k]  (a batched [1 x k] @ [k x d] product)
The experts are ordinary Layers; with ``moe_group`` of size W each rank holds
``len(experts)`` experts and the global expert id is ``rank * len(experts) + e``.
``mp_group``: tokens are sliced across the model-parallel group before routing and
all-gathered after (as the reference does), so TP ranks do not duplicate expert work.
"""
import numpy as np
import torch
import torch.distributed as dist

from .....framework.core import Tensor, _u
from ..... import nn
from .....distributed.utils.moe_utils import _GlobalScatter, _GlobalGather
from .gate import BaseGate, NaiveGate, GShardGate, SwitchGate, limit_by_capacity  # noqa: F401


class _Slice(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, rank, world, group):
        ctx.args = (rank, world, group, x.shape[0])
        n = x.shape[0] // world
        return x[rank * n:(rank + 1) * n].contiguous()

    @staticmethod
    def backward(ctx, g):
        rank, world, group, rows = ctx.args
        parts = [torch.empty_like(g) for _ in range(world)]
        dist.all_gather(parts, g.contiguous(), group=getattr(group, 'process_group', None))
        return torch.cat(parts, 0), None, None, None


class _AllGather(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, rank, world, group):
        ctx.args = (rank, world)
        parts = [torch.empty_like(x) for _ in range(world)]
        dist.all_gather(parts, x.contiguous(), group=getattr(group, 'process_group', None))
        return torch.cat(parts, 0)

    @staticmethod
    def backward(ctx, g):
        rank, world = ctx.args
        n = g.shape[0] // world
        return g[rank * n:(rank + 1) * n].contiguous(), None, None, None


def prepare_forward(gate_idx, num_expert, world_size, moe_group=None):
    """Route bookkeeping: (pos, local_expert_count, global_expert_count, fwd_expert_count,
    fwd_batch_size). Counts are host lists (they size the all_to_all splits)."""
    from .....distributed.utils.moe_utils import _a2a
    g = _u(gate_idx).reshape(-1).long()
    E = num_expert * world_size
    with torch.no_grad():
        lec = torch.bincount(g[g >= 0], minlength=E)[:E]
        if world_size > 1:
            gec = _a2a(lec, E, [num_expert] * world_size, [num_expert] * world_size, moe_group)
        else:
            gec = lec
        key = torch.where(g >= 0, g, torch.full_like(g, torch.iinfo(torch.int64).max))
        pos = torch.sort(key, stable=True).indices[:int(lec.sum())]
    lec_l, gec_l = lec.tolist(), gec.tolist()
    fwd_expert_count = np.asarray(gec_l, dtype=np.int64).reshape(world_size, num_expert).sum(0)
    return pos, lec_l, gec_l, fwd_expert_count, int(sum(gec_l))


class MoELayer(nn.Layer):
    def __init__(self, d_model, experts, gate=None, moe_group=None, mp_group=None,
                 recompute_interval=0, recompute_ctx=None):
        super().__init__()
        self.recompute_ctx = recompute_ctx
        if gate is None:
            gate = {}
        if not isinstance(gate, (dict, BaseGate)):
            raise TypeError("gate config' type must be dict or an instance of BaseGate")
        self.group = moe_group
        self.world_size = moe_group.nranks if moe_group is not None else 1
        self.num_expert = len(experts)
        self.recompute_interval = recompute_interval
        self.experts = experts
        self.mp_group = mp_group
        self.d_model = d_model
        if isinstance(gate, dict):
            self.top_k = gate.get("top_k", 2)
            kind = gate.get("type", "gshard")
            if kind == "naive" or kind is None:
                gate = NaiveGate(d_model, num_expert=len(experts), world_size=self.world_size,
                                 topk=self.top_k)
            elif kind == "gshard":
                gate = GShardGate(d_model, num_expert=len(experts), world_size=self.world_size,
                                  topk=self.top_k, group=self.group)
            elif kind == "switch":
                gate = SwitchGate(d_model, num_expert=len(experts), world_size=self.world_size,
                                  topk=self.top_k, group=self.group)
            else:
                raise AssertionError(f"We only support naive gate, gshard gate and switch gate, "
                                     f"but you choose {kind} gate.")
        elif isinstance(gate, NaiveGate):
            self.top_k = gate.top_k
        else:
            raise TypeError("Unimplemented gate type: ", type(gate))
        self.gate = gate

    def _experts_fwd(self, x, fwd_expert_count):
        if x.shape[0] == 0:
            return x
        ys, start = [], 0
        for e, cnt in enumerate(fwd_expert_count.tolist()):
            if cnt <= 0:
                continue
            ys.append(_u(self.experts[e](Tensor(x[start:start + cnt]))))
            start += cnt
        return torch.cat(ys, 0)

    def forward(self, inp):
        t = _u(inp)
        assert t.dim() == 3, "MoELayer expects [batch, seq, d_model]"
        origin_shape = t.shape
        t = t.reshape(-1, origin_shape[2])
        mp_rank, mp_size = 0, 1
        if self.mp_group is not None:
            mp_rank, mp_size = self.mp_group.rank, self.mp_group.nranks
        if mp_size > 1:
            t = _Slice.apply(t, mp_rank, mp_size, self.mp_group)
        value, gate_idx = self.gate(Tensor(t))
        value, gate_idx = _u(value), _u(gate_idx)
        topk = gate_idx.shape[1] if gate_idx.dim() == 2 else 1
        assert topk == self.top_k
        pos, lec, gec, fwd_count, fwd_bs = prepare_forward(gate_idx, self.num_expert,
                                                           self.world_size, self.group)
        rows = t.index_select(0, pos // topk) if pos.numel() else t.new_zeros((0, t.shape[1]))
        x = _GlobalScatter.apply(rows, lec, gec, self.world_size, self.group)
        if self.recompute_interval > 0 and x.shape[0] > 0:
            from .....distributed.fleet.utils import recompute
            x = _u(recompute(lambda xx: Tensor(self._experts_fwd(_u(xx), fwd_count)), Tensor(x)))
        else:
            x = self._experts_fwd(x, fwd_count)
        x = _GlobalGather.apply(x, lec, gec, self.world_size, self.group)
        out_rows = t.shape[0] * topk
        full = x.new_zeros((out_rows, x.shape[-1]))
        if pos.numel():
            full = full.index_copy(0, pos, x)
        full = full.view(-1, self.top_k, self.d_model)
        w = value.reshape(full.shape[0], 1, self.top_k).to(full.dtype)
        y = torch.bmm(w, full).reshape(-1, self.d_model)
        if mp_size > 1:
            y = _AllGather.apply(y, mp_rank, mp_size, self.mp_group)
        return Tensor(y.reshape(origin_shape))
