"""Tensor (model) parallelism (parity: python/paddle/distributed/fleet/layers/mpu/{mp_layers,mp_ops,random}.py).

Megatron-style column/row split linear layers, vocab-parallel embedding and
vocab-parallel fused cross-entropy; communication is RCCL all-reduce /
all-gather inside the TP group (adjacent GPUs on xGMI — see topology.py).
"""
import contextlib

import numpy as np
import torch
import torch.distributed as dist

from ..framework.core import Tensor, Parameter, _u
from ..nn.layer.layers import Layer
from ..nn import functional as F
from ..nn import initializer as I
from ..distributed import collective as C
from ..ops import fused as K


def _pg(group):
    return None if group is None else group.process_group


def _ws(group):
    return 1 if group is None else group.nranks


def _rank(group):
    return 0 if group is None else group.rank


# -- autograd comm ops ----------------------------------------------------------------
class _Identity(torch.autograd.Function):
    """fwd identity / bwd all-reduce (Megatron 'f')."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x

    @staticmethod
    def backward(ctx, g):
        if _ws(ctx.group) > 1:
            g = g.contiguous()
            dist.all_reduce(g, group=_pg(ctx.group))
        return g, None


class _AllReduce(torch.autograd.Function):
    """fwd all-reduce / bwd identity (Megatron 'g')."""

    @staticmethod
    def forward(ctx, x, group):
        if _ws(group) > 1:
            x = x.contiguous().clone()
            dist.all_reduce(x, group=_pg(group))
        return x

    @staticmethod
    def backward(ctx, g):
        return g, None


class _Split(torch.autograd.Function):
    """fwd take own slice of last dim / bwd all-gather."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        n = _ws(group)
        if n == 1:
            return x
        return x.chunk(n, -1)[_rank(group)].contiguous()

    @staticmethod
    def backward(ctx, g):
        return _gather_last(g, ctx.group), None


def _gather_last(x, group):
    n = _ws(group)
    if n == 1:
        return x
    x = x.contiguous()
    outs = [torch.empty_like(x) for _ in range(n)]
    dist.all_gather(outs, x, group=_pg(group))
    return torch.cat(outs, -1)


class _Concat(torch.autograd.Function):
    """fwd all-gather along last dim / bwd split."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _gather_last(x, group)

    @staticmethod
    def backward(ctx, g):
        n = _ws(ctx.group)
        if n == 1:
            return g, None
        return g.chunk(n, -1)[_rank(ctx.group)].contiguous(), None


def _c_identity(x, group=None):
    return Tensor(_Identity.apply(_u(x), group))


def _mp_allreduce(x, group=None, use_calc_stream=True, use_model_parallel=True):
    return Tensor(_AllReduce.apply(_u(x), group))


def _c_split(x, group=None):
    return Tensor(_Split.apply(_u(x), group))


def _c_concat(x, group=None):
    return Tensor(_Concat.apply(_u(x), group))


def _default_mp_group():
    from ..distributed import fleet
    hcg = fleet.get_hybrid_communicate_group() if fleet.fleet._hcg is not None else None
    return hcg.get_model_parallel_group() if hcg is not None else None


# -- RNG tracker ------------------------------------------------------------------------
MODEL_PARALLEL_RNG = 'model_parallel_rng'


class RNGStatesTracker:
    def __init__(self):
        self.states_ = {}
        self.seeds_ = set()

    def reset(self):
        self.states_ = {}
        self.seeds_ = set()

    def add(self, name, seed):
        if seed in self.seeds_:
            raise ValueError(f'seed {seed} already exists')
        self.seeds_.add(seed)
        if name in self.states_:
            raise ValueError(f'state {name} already exists')
        cpu = torch.get_rng_state()
        dev = torch.cuda.get_rng_state() if torch.cuda.is_available() else None
        torch.manual_seed(seed)
        self.states_[name] = (torch.get_rng_state(),
                              torch.cuda.get_rng_state() if torch.cuda.is_available() else None)
        torch.set_rng_state(cpu)
        if dev is not None:
            torch.cuda.set_rng_state(dev)

    def get_states_tracker(self):
        return dict(self.states_)

    def set_states_tracker(self, states):
        self.states_ = dict(states)

    @contextlib.contextmanager
    def rng_state(self, name=MODEL_PARALLEL_RNG):
        if name not in self.states_:
            yield
            return
        cpu = torch.get_rng_state()
        dev = torch.cuda.get_rng_state() if torch.cuda.is_available() else None
        s_cpu, s_dev = self.states_[name]
        torch.set_rng_state(s_cpu)
        if s_dev is not None:
            torch.cuda.set_rng_state(s_dev)
        try:
            yield
        finally:
            self.states_[name] = (torch.get_rng_state(),
                                  torch.cuda.get_rng_state() if torch.cuda.is_available() else None)
            torch.set_rng_state(cpu)
            if dev is not None:
                torch.cuda.set_rng_state(dev)


_RNG_TRACKER = RNGStatesTracker()


def get_rng_state_tracker():
    return _RNG_TRACKER


def model_parallel_random_seed(seed=None):
    from ..distributed import fleet
    hcg = fleet.get_hybrid_communicate_group()
    rank = hcg.get_model_parallel_rank() if hcg else 0
    seed = 2048 if seed is None else seed
    _RNG_TRACKER.reset()
    _RNG_TRACKER.add(MODEL_PARALLEL_RNG, seed * 1024 + rank * 100 + 1)
    # the global stream stays identical across the TP group (random.py:104): dropout on the
    # replicated residual stream must draw the same mask on every mp rank
    torch.manual_seed(seed)


# -- layers -------------------------------------------------------------------------------
class VocabParallelEmbedding(Layer):
    def __init__(self, num_embeddings, embedding_dim, weight_attr=None, mp_group=None, name=None):
        super().__init__()
        self.model_parallel_group = mp_group if mp_group is not None else _default_mp_group()
        self.world_size = _ws(self.model_parallel_group)
        self.rank = _rank(self.model_parallel_group)
        self.origin_num_embeddings = num_embeddings
        assert num_embeddings % self.world_size == 0
        per = num_embeddings // self.world_size
        self.vocab_start_index = self.rank * per
        self._size = [per, embedding_dim]
        with get_rng_state_tracker().rng_state():
            self.weight = self.create_parameter(self._size, weight_attr)
        self.weight.is_distributed = self.world_size > 1

    def forward(self, x):
        ids = _u(x)
        if self.world_size == 1:
            return F.embedding(x, self.weight)
        # the lookup kernel reads ids outside [0, per) as zero rows and skips them in the
        # weight gradient: shifting by vocab_start_index IS the vocab-range mask
        out = K.embedding(ids - self.vocab_start_index, self.weight._t)
        return Tensor(_AllReduce.apply(out, self.model_parallel_group))


class ColumnParallelLinear(Layer):
    def __init__(self, in_features, out_features, weight_attr=None, has_bias=None,
                 gather_output=True, fuse_matmul_bias=False, mp_group=None, name=None):
        super().__init__()
        self.model_parallel_group = mp_group if mp_group is not None else _default_mp_group()
        self.world_size = _ws(self.model_parallel_group)
        assert out_features % self.world_size == 0
        self.output_size_per_partition = out_features // self.world_size
        self.gather_output = gather_output
        with get_rng_state_tracker().rng_state():
            self.weight = self.create_parameter([in_features, self.output_size_per_partition],
                                                weight_attr)
        self.weight.is_distributed = self.world_size > 1
        self.bias = self.create_parameter([self.output_size_per_partition], is_bias=True) \
            if has_bias in (None, True) else None
        if self.bias is not None:
            self.bias.is_distributed = self.world_size > 1

    def forward(self, x):
        xin = _c_identity(x, self.model_parallel_group) if self.world_size > 1 else x
        out = F.linear(xin, self.weight, self.bias)
        if self.gather_output and self.world_size > 1:
            out = _c_concat(out, self.model_parallel_group)
        return out


class RowParallelLinear(Layer):
    def __init__(self, in_features, out_features, weight_attr=None, has_bias=True,
                 input_is_parallel=False, fuse_matmul_bias=False, mp_group=None, name=None):
        super().__init__()
        self.model_parallel_group = mp_group if mp_group is not None else _default_mp_group()
        self.world_size = _ws(self.model_parallel_group)
        assert in_features % self.world_size == 0
        self.input_size_per_partition = in_features // self.world_size
        self.input_is_parallel = input_is_parallel
        with get_rng_state_tracker().rng_state():
            self.weight = self.create_parameter([self.input_size_per_partition, out_features],
                                                weight_attr)
        self.weight.is_distributed = self.world_size > 1
        self.bias = self.create_parameter([out_features], is_bias=True) if has_bias else None

    def forward(self, x):
        xin = x if (self.input_is_parallel or self.world_size == 1) else \
            _c_split(x, self.model_parallel_group)
        out = F.linear(xin, self.weight)
        if self.world_size > 1:
            out = _mp_allreduce(out, self.model_parallel_group)
        if self.bias is not None:
            out = out + self.bias
        return out


class ParallelCrossEntropy(Layer):
    def __init__(self, mp_group=None, name=None, ignore_index=-100):
        super().__init__()
        self.model_parallel_group = mp_group if mp_group is not None else _default_mp_group()
        self.ignore_index = ignore_index

    def forward(self, input, label):
        lab = _u(label)
        if lab.dim() == _u(input).dim():
            lab = lab.squeeze(-1)
        g = self.model_parallel_group
        loss = K.vocab_parallel_cross_entropy(_u(input), lab.long(), _pg(g), _ws(g), _rank(g),
                                              self.ignore_index)
        return Tensor(loss.unsqueeze(-1))


def split(x, size, operation, axis=0, num_partitions=1, gather_out=True, weight_attr=None,
          bias_attr=None, name=None):
    """paddle.distributed.split: build a parallel embedding/linear and apply it."""
    if operation == 'embedding':
        layer = VocabParallelEmbedding(size[0], size[1], weight_attr)
    elif operation == 'linear' and axis == 1:
        layer = ColumnParallelLinear(size[0], size[1], weight_attr, bias_attr is not False,
                                     gather_out)
    elif operation == 'linear':
        layer = RowParallelLinear(size[0], size[1], weight_attr, bias_attr is not False, False)
    else:
        raise ValueError(operation)
    return layer(x)
