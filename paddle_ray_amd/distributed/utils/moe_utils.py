"""Expert-parallel token exchange (parity: python/paddle/distributed/utils/moe_utils.py
``global_scatter`` / ``global_gather``; CUDA ops paddle/fluid/operators/collective/
global_scatter_op.cu.cc, global_gather_op.cu.cc).

MI355X design: ONE variable-split ``all_to_all_single`` per exchange over RCCL (xGMI is
point-to-point, so a single a2a keeps every link busy at once instead of the reference's
per-expert send/recv loop), plus an on-device permutation between the wire order
(worker-major) and the expert-major order the experts consume. Both are differentiable:
the backward of a scatter is the gather with the same counts and vice versa.
"""
import torch
import torch.distributed as dist

from ...framework.core import Tensor, _u


def _pg(group):
    return None if group is None else getattr(group, 'process_group', None)


def _world(group):
    if group is not None:
        return group.nranks
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def _a2a(x, out_rows, in_splits, out_splits, group):
    out = x.new_empty((out_rows,) + tuple(x.shape[1:]))
    pg = _pg(group)
    if dist.get_backend(pg) == 'gloo':  # gloo: pairwise exchange
        ranks = group.ranks if group is not None else list(range(dist.get_world_size()))
        me = ranks.index(dist.get_rank())
        ins = list(torch.split(x, in_splits))
        outs = list(torch.split(out, out_splits))
        ops = []
        for j, peer in enumerate(ranks):
            if j == me:
                outs[j].copy_(ins[j])
                continue
            if in_splits[j]:
                ops.append(dist.P2POp(dist.isend, ins[j].contiguous(), peer, pg))
            if out_splits[j]:
                buf = torch.empty_like(outs[j])
                ops.append(dist.P2POp(dist.irecv, buf, peer, pg))
                outs[j] = buf
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        return torch.cat(outs, 0) if outs else out
    dist.all_to_all_single(out, x.contiguous(), out_splits, in_splits, group=pg)
    return out


def _perm_worker_to_expert(counts_wm, n_worker, n_expert, device):
    """Index that reorders rows stored worker-major (w outer, e inner) into expert-major."""
    c = torch.as_tensor(counts_wm, dtype=torch.int64).view(n_worker, n_expert)
    start_wm = (torch.cumsum(c.reshape(-1), 0) - c.reshape(-1)).view(n_worker, n_expert)
    c_em = c.t().reshape(-1)
    s_em = start_wm.t().reshape(-1)
    total = int(c_em.sum())
    if total == 0:
        return torch.zeros(0, dtype=torch.int64, device=device)
    base_em = torch.cumsum(c_em, 0) - c_em
    idx = torch.repeat_interleave(s_em - base_em, c_em) + torch.arange(total)
    return idx.to(device)


def _scatter_impl(x, lc, gc, n_worker, group):
    n_expert = len(lc) // n_worker
    in_splits = [int(sum(lc[w * n_expert:(w + 1) * n_expert])) for w in range(n_worker)]
    out_splits = [int(sum(gc[w * n_expert:(w + 1) * n_expert])) for w in range(n_worker)]
    y = _a2a(x, sum(out_splits), in_splits, out_splits, group) if n_worker > 1 else x
    idx = _perm_worker_to_expert(gc, n_worker, n_expert, x.device)
    return y.index_select(0, idx)


def _gather_impl(x, lc, gc, n_worker, group):
    n_expert = len(lc) // n_worker
    idx = _perm_worker_to_expert(gc, n_worker, n_expert, x.device)
    y = torch.empty_like(x)
    y.index_copy_(0, idx, x)  # expert-major -> worker-major
    in_splits = [int(sum(gc[w * n_expert:(w + 1) * n_expert])) for w in range(n_worker)]
    out_splits = [int(sum(lc[w * n_expert:(w + 1) * n_expert])) for w in range(n_worker)]
    return _a2a(y, sum(out_splits), in_splits, out_splits, group) if n_worker > 1 else y


class _GlobalScatter(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, lc, gc, n_worker, group):
        ctx.args = (lc, gc, n_worker, group)
        return _scatter_impl(x, lc, gc, n_worker, group)

    @staticmethod
    def backward(ctx, g):
        lc, gc, n_worker, group = ctx.args
        return _gather_impl(g.contiguous(), lc, gc, n_worker, group), None, None, None, None


class _GlobalGather(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, lc, gc, n_worker, group):
        ctx.args = (lc, gc, n_worker, group)
        return _gather_impl(x, lc, gc, n_worker, group)

    @staticmethod
    def backward(ctx, g):
        lc, gc, n_worker, group = ctx.args
        return _scatter_impl(g.contiguous(), lc, gc, n_worker, group), None, None, None, None


def _counts(c):
    return [int(v) for v in (_u(c).tolist() if isinstance(c, Tensor) or torch.is_tensor(c)
                             else c)]


def global_scatter(x, local_count, global_count, group=None, use_calc_stream=True):
    """Send rows of ``x`` (ordered by global expert id = worker * n_expert + expert) to the
    workers owning those experts; the result is expert-major (expert outer, source worker
    inner), ready for the local experts."""
    n_worker = _world(group)
    return Tensor(_GlobalScatter.apply(_u(x), _counts(local_count), _counts(global_count),
                                       n_worker, group))


def global_gather(x, local_count, global_count, group=None, use_calc_stream=True):
    """Inverse of :func:`global_scatter`."""
    n_worker = _world(group)
    return Tensor(_GlobalGather.apply(_u(x), _counts(local_count), _counts(global_count),
                                      n_worker, group))
