"""MoE routing primitives (parity: python/paddle/distributed/models/moe/utils.py; the
reference's CUDA ops number_count / assign_pos / limit_by_capacity / prune_gate_by_capacity /
random_routing in paddle/fluid/operators/*.cu).

All are deterministic device-side tensor programs (bincount, stable argsort, cumsum) instead
of the reference's atomic-counter kernels: the same kept/dropped sets, a fixed order.
"""
import torch

from ....framework.core import Tensor, _u


def _w(t):
    return Tensor(t)


def _number_count(numbers, upper_range):
    """counts[e] = #entries equal to e (entries < 0 are dropped routes)."""
    n = _u(numbers).reshape(-1).long()
    n = n[n >= 0]
    return _w(torch.bincount(n, minlength=int(upper_range))[:int(upper_range)])


def _assign_pos(x, cum_count):
    """Positions of the routed entries grouped by expert id (expert-major, stable within an
    expert): pos[cum_count[e-1]:cum_count[e]] are the flat indices routed to expert e."""
    ids = _u(x).reshape(-1).long()
    total = int(_u(cum_count)[-1].item()) if _u(cum_count).numel() else 0
    key = torch.where(ids >= 0, ids, torch.full_like(ids, torch.iinfo(torch.int64).max))
    order = torch.sort(key, stable=True).indices
    return _w(order[:total])


def _random_routing(topk_idx, topk_value, prob, topk=2):
    """GShard random routing: drop the 2nd choice where 2 * its gate value < prob."""
    if topk != 2:
        raise ValueError("random routing only supports topk=2")
    idx = _u(topk_idx).clone()
    drop = 2 * _u(topk_value)[:, 1].float() < _u(prob).float()
    idx[:, 1] = torch.where(drop, torch.full_like(idx[:, 1], -1), idx[:, 1])
    return _w(idx)


def _limit_by_capacity(expert_count, capacity, n_worker):
    """expert_count: [n_worker * n_expert] counts worker w sends to local expert e (worker
    major). Lower ranks fill each expert's capacity first."""
    ec = _u(expert_count).long().view(int(n_worker), -1)
    cap = _u(capacity).long().view(1, -1)
    before = torch.cumsum(ec, 0) - ec                  # sent by lower ranks
    keep = torch.clamp(torch.minimum(ec, cap - before), min=0)
    return _w(keep.reshape(-1))


def _prune_gate_by_capacity(gate_idx, expert_count, n_expert, n_worker):
    """Keep, per global expert g, only the first expert_count[g] entries routed to g (in
    flat order); the rest become -1."""
    g = _u(gate_idx)
    flat = g.reshape(-1).long()
    E = int(n_expert) * int(n_worker)
    valid = flat >= 0
    onehot = torch.zeros(flat.numel(), E, dtype=torch.int64, device=flat.device)
    onehot[valid, flat[valid]] = 1
    rank_in_expert = (torch.cumsum(onehot, 0) - onehot)[torch.arange(flat.numel(),
                                                                    device=flat.device),
                                                       flat.clamp(min=0)]
    limit = _u(expert_count).long()[flat.clamp(min=0)]
    keep = valid & (rank_in_expert < limit)
    out = torch.where(keep, flat, torch.full_like(flat, -1))
    return _w(out.view(g.shape).to(g.dtype))
