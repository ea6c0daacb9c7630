"""memory_efficient_attention (parity: python/paddle/incubate/nn/memory_efficient_attention.py).

q/k/v are [B, M, H, K] (xformers BMHK). Dispatch on MI355X: no bias / causal masks run
the in-tree MFMA flash-attention kernels directly; block-diagonal (packed variable-length)
masks run the flash kernel once per block on the contiguous slice -- nothing quadratic
is materialized; any other bias (tensor biases, padded-key masks) or dropout uses the
dense reference path with the materialized additive mask.
"""
import math

import torch
import torch.nn.functional as TF

from ...framework.core import Tensor, _u
from . import attn_bias as AB


def _flash_ok(q, k, p, training):
    return (q.is_cuda and q.dtype in (torch.bfloat16, torch.float16) and q.shape[-1] in (64, 128)
            and q.shape[-1] == k.shape[-1] and (p == 0.0 or not training))


def _dense(q, k, v, bias, p, scale, training):
    qt, kt, vt = (x.transpose(1, 2).float() for x in (q, k, v))  # [B, H, M, K]
    s = torch.matmul(qt, kt.transpose(-1, -2)) * scale
    if bias is not None:
        s = s + bias.float()
    a = torch.softmax(s, -1)
    if p > 0.0 and training:
        a = TF.dropout(a, p)
    return torch.matmul(a, vt).transpose(1, 2).to(q.dtype)


def memory_efficient_attention(query, key, value, attn_bias=None, p=0.0, scale=None,
                               training=True):
    from ...ops import fused as K
    q, k, v = _u(query), _u(key), _u(value)
    scale = (1.0 / math.sqrt(q.shape[-1])) if scale is None else float(scale)
    flash = _flash_ok(q, k, p, training)
    if attn_bias is None or type(attn_bias) is AB.LowerTriangularMask:
        causal = attn_bias is not None
        if flash:
            return Tensor(K.flash_attention(q, k, v, causal=causal, scale=scale))
        bias = _u(attn_bias.materialize([q.shape[1], k.shape[1]])).to(q.device) if causal \
            else None
        return Tensor(_dense(q, k, v, bias, p, scale, training))
    if isinstance(attn_bias, AB.BlockDiagonalMask) and flash and q.shape[0] == 1:
        # the packed blocks are independent sequences: ONE varlen flash launch over all of them
        qi, ki = list(attn_bias.q_seqinfo.intervals()), list(attn_bias.k_seqinfo.intervals())
        cu_q = torch.tensor([0] + [b for _, b in qi], dtype=torch.int32, device=q.device)
        cu_k = torch.tensor([0] + [b for _, b in ki], dtype=torch.int32, device=q.device)
        mq = max(b - a for a, b in qi)
        mk = max(b - a for a, b in ki)
        o = K.flash_attn_varlen(q[0], k[0], v[0], cu_q, cu_k, mq, mk, causal=attn_bias.causal,
                                scale=scale)
        return Tensor(o[None])
    if isinstance(attn_bias, AB.AttentionBias):
        bias = _u(attn_bias.materialize([q.shape[0], q.shape[2], q.shape[1], k.shape[1]],
                                        dtype='float32')).to(q.device)
    else:
        bias = _u(attn_bias)
    return Tensor(_dense(q, k, v, bias, p, scale, training))
