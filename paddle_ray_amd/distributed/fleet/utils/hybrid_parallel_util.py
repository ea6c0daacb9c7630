"""Parameter/gradient sync helpers (parity: fleet/utils/hybrid_parallel_util.py)."""
import torch.distributed as dist


def fused_allreduce_gradients(parameter_list, hcg):
    g = hcg.get_data_parallel_group() if hcg is not None else None
    n = g.nranks if g is not None else (dist.get_world_size() if dist.is_initialized() else 1)
    if n <= 1:
        return
    grads = [p._t.grad for p in parameter_list if p._t.grad is not None]
    if not grads:
        return
    import torch
    flat = torch.cat([x.reshape(-1) for x in grads])
    dist.all_reduce(flat, group=None if g is None else g.process_group)
    flat.div_(n)
    off = 0
    for x in grads:
        x.copy_(flat[off:off + x.numel()].view_as(x))
        off += x.numel()


def broadcast_mp_parameters(model, hcg):
    g = hcg.get_model_parallel_group()
    for p in model.parameters():
        if not getattr(p, 'is_distributed', False) and g.nranks > 1:
            dist.broadcast(p._t.data, g.ranks[0], group=g.process_group)


def broadcast_dp_parameters(model, hcg):
    g = hcg.get_data_parallel_group()
    for p in model.parameters():
        if g.nranks > 1:
            dist.broadcast(p._t.data, g.ranks[0], group=g.process_group)


def broadcast_sharding_parameters(model, hcg):
    g = hcg.get_sharding_parallel_group()
    for p in model.parameters():
        if g.nranks > 1:
            dist.broadcast(p._t.data, g.ranks[0], group=g.process_group)
