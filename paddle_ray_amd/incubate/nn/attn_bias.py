"""Attention biases for memory_efficient_attention (parity:
python/paddle/incubate/nn/attn_bias.py; xformers-style semantics).

Structured biases (causal, block-diagonal over packed variable-length sequences) are kept
symbolic so the attention call can run the flash kernel per block instead of building an
[Mq, Mk] mask; ``materialize`` builds the dense additive mask for the reference path.
"""
from abc import ABC, abstractmethod
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import torch

from ...framework.core import Tensor, _u, convert_dtype


def _dt(dtype):
    return convert_dtype(dtype) if dtype is not None else torch.float32


class AttentionBias(ABC):
    @abstractmethod
    def materialize(self, shape, dtype='float32'):
        raise NotImplementedError


class LowerTriangularMask(AttentionBias):
    """Causal: query i attends keys j <= i."""

    def materialize(self, shape, dtype='float32'):
        m = torch.full(list(shape), float('-inf')).triu(diagonal=1)
        return Tensor(m.to(_dt(dtype)))

    def add_bias(self, bias):
        return LowerTriangularMaskWithTensorBias(bias)


class LowerTriangularMaskWithTensorBias(LowerTriangularMask):
    def __init__(self, bias):
        self._bias = bias

    def materialize(self, shape, dtype='float32'):
        return Tensor(_u(super().materialize(shape, dtype)) + _u(self._bias))


@dataclass
class SeqLenInfo:
    seqstart: object
    max_seqlen: int
    seqstart_py: List[int]

    def intervals(self):
        yield from zip(self.seqstart_py, self.seqstart_py[1:])

    @classmethod
    def from_seqlens(cls, seqlens):
        starts = [0]
        for s in seqlens:
            starts.append(starts[-1] + int(s))
        return cls(seqstart=Tensor(torch.tensor(starts, dtype=torch.int32)),
                   max_seqlen=max(int(s) for s in seqlens), seqstart_py=starts)

    def split(self, x, batch_sizes=None):
        xt = _u(x)
        assert self.seqstart_py[-1] == xt.shape[1] and xt.shape[0] == 1
        batch_sizes = batch_sizes or [1] * (len(self.seqstart_py) - 1)
        out, it = [], 0
        for bs in batch_sizes:
            a, b = self.seqstart_py[it], self.seqstart_py[it + bs]
            out.append(Tensor(xt[:, a:b].reshape(bs, -1, *xt.shape[2:])))
            it += bs
        return out


@dataclass
class PaddedSeqLenInfo(SeqLenInfo):
    seqlen: object = None
    seqlen_py: Sequence[int] = field(default_factory=list)

    def intervals(self):
        for (start, _), n in zip(super().intervals(), self.seqlen_py):
            yield start, start + n

    @classmethod
    def from_seqlens(cls, seqlens):
        raise NotImplementedError("use SeqLenInfo.from_seqlens or "
                                  "PaddedSeqLenInfo.from_seqlens_padded")

    @classmethod
    def from_seqlens_padded(cls, seqlens, padding):
        assert all(s <= padding for s in seqlens)
        starts = list(range(0, len(seqlens) * padding + 1, padding))
        return cls(seqstart=Tensor(torch.tensor(starts, dtype=torch.int32)),
                   max_seqlen=max(seqlens), seqstart_py=starts,
                   seqlen=Tensor(torch.tensor(list(seqlens), dtype=torch.int32)),
                   seqlen_py=list(seqlens))

    def split(self, x, batch_sizes=None):
        raise NotImplementedError


@dataclass
class BlockDiagonalMask(AttentionBias):
    """Packed sequences along dim 1 (batch 1): query block i attends key block i only."""
    q_seqinfo: SeqLenInfo
    k_seqinfo: SeqLenInfo
    _batch_sizes: Optional[Sequence[int]] = None
    causal = False

    def _block(self, nq, nk):
        if self.causal:
            return torch.full((nq, nk), float('-inf')).triu(diagonal=1)
        return torch.zeros(nq, nk)

    def materialize(self, shape, dtype='float32'):
        assert shape[-1] == self.k_seqinfo.seqstart_py[-1]
        assert shape[-2] == self.q_seqinfo.seqstart_py[-1]
        m = torch.full(list(shape[-2:]), float('-inf'))
        for (qa, qb), (ka, kb) in zip(self.q_seqinfo.intervals(), self.k_seqinfo.intervals()):
            m[qa:qb, ka:kb] = self._block(qb - qa, kb - ka)
        return Tensor(m.expand(list(shape)).to(_dt(dtype)))

    @classmethod
    def from_seqlens(cls, q_seqlen, kv_seqlen=None):
        assert kv_seqlen is None or len(q_seqlen) == len(kv_seqlen)
        q = SeqLenInfo.from_seqlens(q_seqlen)
        k = q if kv_seqlen is None or list(q_seqlen) == list(kv_seqlen) else \
            SeqLenInfo.from_seqlens(kv_seqlen)
        return cls(q_seqinfo=q, k_seqinfo=k)

    @classmethod
    def from_tensor_list(cls, tensors):
        seqlens = [x.shape[1] for x in tensors for _ in range(x.shape[0])]
        bd = cls.from_seqlens(seqlens)
        bd._batch_sizes = [x.shape[0] for x in tensors]
        cat = torch.cat([_u(x).reshape(1, -1, *x.shape[2:]) for x in tensors], 1)
        return bd, Tensor(cat)

    @classmethod
    def from_tensor_lists_qkv(cls, tensors_q, tensors_k, tensors_v=None):
        assert len(tensors_q) == len(tensors_k)
        qs = [q.shape[1] for q in tensors_q for _ in range(q.shape[0])]
        ks = [k.shape[1] for k in tensors_k for _ in range(k.shape[0])]
        bd = cls.from_seqlens(qs, ks)
        bd._batch_sizes = [x.shape[0] for x in tensors_q]
        cat = lambda ts: Tensor(torch.cat([_u(x).reshape(1, -1, *x.shape[2:])  # noqa: E731
                                           for x in ts], 1))
        return bd, cat(tensors_q), cat(tensors_k), \
            (cat(tensors_v) if tensors_v is not None else None)

    def split_queries(self, tensor):
        return self.q_seqinfo.split(tensor, self._batch_sizes)

    def split_kv(self, tensor):
        return self.k_seqinfo.split(tensor, self._batch_sizes)

    def split(self, tensor):
        assert self.q_seqinfo is self.k_seqinfo
        return self.q_seqinfo.split(tensor, self._batch_sizes)

    def make_causal(self):
        return BlockDiagonalCausalMask(q_seqinfo=self.q_seqinfo, k_seqinfo=self.k_seqinfo,
                                       _batch_sizes=self._batch_sizes)


@dataclass
class BlockDiagonalCausalMask(BlockDiagonalMask):
    causal = True


@dataclass
class BlockDiagonalCausalWithOffsetPaddedKeysMask(AttentionBias):
    """Causal blocks whose keys live in fixed-size padded slots (KV-cache decoding): query
    block i attends the first seqlen_i keys of slot i, causally aligned to their end."""
    q_seqinfo: SeqLenInfo
    k_seqinfo: PaddedSeqLenInfo
    causal_diagonal: object = None

    def materialize(self, shape, dtype='float32'):
        m = torch.full(list(shape[-2:]), float('-inf'))
        for i, ((qa, qb), (ka, kb)) in enumerate(zip(self.q_seqinfo.intervals(),
                                                     self.k_seqinfo.intervals())):
            nq, nk = qb - qa, kb - ka
            off = nk - nq
            if self.causal_diagonal is not None:
                off += int(_u(self.causal_diagonal)[i])
            m[qa:qb, ka:kb] = torch.full((nq, nk), float('-inf')).triu(diagonal=1 + off)
        return Tensor(m.expand(list(shape)).to(_dt(dtype)))

    @classmethod
    def from_seqlens(cls, q_seqlen, kv_padding, kv_seqlen, causal_diagonal=None):
        assert kv_seqlen is None or len(q_seqlen) == len(kv_seqlen)
        return cls(q_seqinfo=SeqLenInfo.from_seqlens(q_seqlen),
                   k_seqinfo=PaddedSeqLenInfo.from_seqlens_padded(kv_seqlen, kv_padding),
                   causal_diagonal=causal_diagonal)
