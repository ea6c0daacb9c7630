"""DistributedFusedLamb (parity: python/paddle/incubate/optimizer/distributed_fused_lamb.py,
CUDA op distributed_fused_lamb_op.cu).

MI355X design: gradients live in one flat bf16/fp32 buffer per dtype; ONE RCCL all-reduce
of that buffer per step (or per ``gradient_accumulation_steps``), optional global-norm clip
before/after the all-reduce, then the LAMB update with fp32 master weights. The flat buffer
is sized for 288 GB HBM: no bucketing below the whole-model size is needed for LAMB-scale
models, and the single large collective is xGMI-link-bound rather than latency-bound."""
import torch
import torch.distributed as dist

from ...framework.core import _u
from ...optimizer.optimizer import Lamb


class DistributedFusedLamb(Lamb):
    def __init__(self, learning_rate=0.001, lamb_weight_decay=0.01, beta1=0.9, beta2=0.999,
                 epsilon=1e-6, parameters=None, grad_clip=None,
                 exclude_from_weight_decay_fn=None, clip_after_allreduce=True,
                 is_grad_scaled_by_nranks=True, alignment=128, use_master_param_norm=True,
                 gradient_accumulation_steps=1, use_master_acc_grad=True, nproc_per_node=None,
                 use_hierarchical_allreduce=False, name=None):
        super().__init__(learning_rate, lamb_weight_decay, beta1, beta2, epsilon, parameters,
                         None, exclude_from_weight_decay_fn, multi_precision=True, name=name)
        self._dfl_clip = grad_clip
        self._clip_after_allreduce = clip_after_allreduce
        self._is_grad_scaled_by_nranks = is_grad_scaled_by_nranks
        self._acc_steps = max(1, int(gradient_accumulation_steps))
        self._acc_count = 0
        self._acc_grads = None
        self._use_master_acc_grad = use_master_acc_grad

    def _nranks(self):
        return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1

    def _allreduce(self, grads):
        n = self._nranks()
        if n == 1 or not grads:
            return
        by_dtype = {}
        for g in grads:
            by_dtype.setdefault(g.dtype, []).append(g)
        for gs in by_dtype.values():
            flat = torch.cat([g.reshape(-1) for g in gs])
            dist.all_reduce(flat)
            if self._is_grad_scaled_by_nranks:
                flat.div_(n)
            off = 0
            for g in gs:
                g.copy_(flat[off:off + g.numel()].view_as(g))
                off += g.numel()

    def _clip(self, params):
        if self._dfl_clip is None:
            return
        self._dfl_clip._dygraph_clip([(p, p.grad) for p in params if p.grad is not None])

    @torch.no_grad()
    def step(self):
        params = [p for p in self._parameter_list if not p.stop_gradient and _u(p).grad is not None]
        grads = [_u(p).grad for p in params]
        if self._acc_steps > 1:
            if self._acc_grads is None:
                dt = torch.float32 if self._use_master_acc_grad else None
                self._acc_grads = [torch.zeros_like(g, dtype=dt or g.dtype) for g in grads]
            torch._foreach_add_(self._acc_grads, [g.to(a.dtype) for g, a in
                                                  zip(grads, self._acc_grads)])
            self._acc_count += 1
            if self._acc_count < self._acc_steps:
                return
            for g, a in zip(grads, self._acc_grads):
                g.copy_(a / self._acc_steps)
                a.zero_()
            self._acc_count = 0
        if not self._clip_after_allreduce:
            self._clip(params)
        self._allreduce(grads)
        if self._clip_after_allreduce:
            self._clip(params)
        super().step()
