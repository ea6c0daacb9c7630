"""Fused ops with direct grad kernels, usable in dygraph AND as single static-graph ops.

Each public function here takes paddle Tensors. Eagerly it runs the fused HIP kernels of
``ops/fused.py`` (autograd Functions). Called with static ``Variable``s it records ONE op whose
forward is the Function's forward and whose ``<type>_grad`` op is the Function's backward, run
directly by the Executor (``static/graph.py`` `_FN_OPS`; parity: the reference's per-op grad
kernels, e.g. ``paddle/phi/kernels/fusion/gpu/fused_linear_param_grad_add_kernel.cu``,
``paddle/phi/kernels/gpu/flash_attn_grad_kernel.cu``,
``paddle/fluid/operators/fused/fused_bias_dropout_residual_layer_norm_op.cu`` grad,
``paddle/phi/kernels/gpu/cross_entropy_grad_kernel.cu``) instead of differentiating the op's
retained autograd graph.

    fused_linear(x, w, b=None)                     y = x·W (+ b), W [in, out]
    fused_linear_nt(x, w)                          y = x·Wᵀ, W [out, in] (tied LM head)
    fused_bias_gelu(x, b, approximate)             gelu(x + b)
    fused_mlp_gelu(x, w1, b1, w2, approximate)     gelu(x·W1 + b1)·W2
    fused_add_dropout_ln(x, h, hb, w, b, p, eps)   (r, LN(r)), r = x + dropout(h + hb)
    fused_flash_qkv(qkv, mask, heads, p)           packed-QKV flash attention [B, S, 3h] -> [B, S, h]
    fused_softmax_ce(logits, labels, ignore)       per-row softmax cross-entropy
"""
import math

import torch

from ..framework.core import Tensor, _u
from ..ops import fused as K
from . import graph as G

__all__ = ['fused_linear', 'fused_linear_nt', 'fused_bias_gelu', 'fused_mlp_gelu',
           'fused_add_dropout_ln', 'fused_flash_qkv', 'fused_softmax_ce']


def _wrap(out):
    if isinstance(out, tuple):
        return tuple(Tensor(o) for o in out)
    return Tensor(out)


def _op(name, fn_cls, eager, pred=None):
    """Register ``name``: eager = ``eager`` (torch args), static = one recorded op backed by
    ``fn_cls`` (``pred(torch args)`` decides at run time whether its kernels apply)."""
    G.register_fn_op(name, fn_cls, pred)

    def public(*args):
        return _wrap(eager(*[_u(a) if isinstance(a, Tensor) else a for a in args]))
    public.__name__ = name
    return G.static_op(name, public)


# -- linear --------------------------------------------------------------------------------------
def _lin_ok(x, w, b=None, *_):
    return isinstance(w, torch.Tensor) and w.requires_grad and w.is_leaf and x.dtype == w.dtype and \
        K._no_autocast_change(x, w)


fused_linear = _op('fused_linear', K.LinearFn, lambda x, w, b=None: K.linear(x, w, b), _lin_ok)


def _lin_nt_ok(x, w):
    return isinstance(w, torch.Tensor) and w.requires_grad and w.is_leaf and x.dtype == w.dtype and \
        K._no_autocast_change(x, w) and x.dim() == 2


fused_linear_nt = _op('fused_linear_nt', K.LinearNTFn, lambda x, w: K.linear_nt(x, w), _lin_nt_ok)


def _bias_gelu_ok(x, b, approximate=False):
    return x.dtype in K._DT


fused_bias_gelu = _op('fused_bias_gelu', K.BiasGeluFn,
                      lambda x, b, approximate=False: K.bias_gelu(x, b, approximate), _bias_gelu_ok)


# -- GELU MLP ------------------------------------------------------------------------------------
def _mlp_ok(x, w1, b1, w2, approximate=True):
    return all(isinstance(t, torch.Tensor) and t.requires_grad and t.is_leaf for t in (w1, b1, w2)) and \
        x.dtype == w1.dtype == w2.dtype == b1.dtype and x.is_cuda and K._no_autocast_change(x, w1)


fused_mlp_gelu = _op('fused_mlp_gelu', K.MlpGeluFn,
                     lambda x, w1, b1, w2, approximate=True: K.mlp_gelu(x, w1, b1, w2, approximate),
                     _mlp_ok)


# -- add + dropout + LayerNorm ---------------------------------------------------------------------
def _adl_ok(x, h, hb, w, b, p, eps):
    return not (p > 0 and x.is_cuda and torch.cuda.is_current_stream_capturing() and
                not K._adl_ok(x.shape[-1]))


fused_add_dropout_ln = _op(
    'fused_add_dropout_ln', K.AddDropoutLNFn,
    lambda x, h, hb, w, b, p=0.0, eps=1e-5: K.add_dropout_layer_norm(x, h, hb, w, b, p, eps),
    _adl_ok)


# -- packed-QKV flash attention -----------------------------------------------------------------
class FlashQKV3Fn(torch.autograd.Function):
    """[B, S, 3*H*D] QKV projection output -> attention context [B, S, H*D]: the packed-QKV flash
    kernels (plain, or the extended ones with an additive mask / dropout) on a view, and the
    packed gradient written back in the projection's layout."""

    @staticmethod
    def forward(ctx, qkv3, mask, heads, p):
        B, S, W = qkv3.shape
        D = W // (3 * heads)
        qkv = qkv3.view(B, S, 3, heads, D)
        ctx.plain = mask is None and p == 0.0
        ctx.shp3 = qkv3.shape
        if ctx.plain:
            o = K.FlashAttnQKVPackedFn.forward(ctx, qkv, False, 1.0 / math.sqrt(D))
        else:
            if mask is not None and mask.dtype not in (qkv.dtype, torch.float32):
                mask = mask.to(qkv.dtype)
            sd, off = K._fa_next_rng(None) if p > 0 else (0, 0)
            o = K.FlashAttnExtQKVFn.forward(ctx, qkv, mask, False, 1.0 / math.sqrt(D), float(p), sd, off)
        return o.reshape(B, S, heads * D)

    @staticmethod
    def backward(ctx, do2):
        B, S, W = ctx.shp3
        if ctx.plain:
            qkv = ctx.saved_tensors[0]   # [B, S, 3, H, D]
            do = do2.reshape(qkv.shape[0], qkv.shape[1], qkv.shape[3], qkv.shape[4])
            dqkv = K.FlashAttnQKVPackedFn.backward(ctx, do)[0]
        else:
            q = ctx.saved_tensors[0]     # [B, S, H, D]
            do = do2.reshape(q.shape[0], q.shape[1], q.shape[2], q.shape[3])
            dqkv = K.FlashAttnExtQKVFn.backward(ctx, do)[0]
        return dqkv.reshape(B, S, W), None, None, None


def _flash_ok(qkv3, mask, heads, p):
    D = qkv3.shape[-1] // (3 * heads)
    return qkv3.is_cuda and qkv3.dtype in (torch.bfloat16, torch.float16) and D in (64, 128) and \
        qkv3.is_contiguous()


def _flash_eager(qkv3, mask, heads, p):
    if _flash_ok(qkv3, mask, heads, p):
        return FlashQKV3Fn.apply(qkv3, mask, heads, p)
    B, S, W = qkv3.shape
    D = W // (3 * heads)
    q, k, v = qkv3.view(B, S, 3, heads, D).unbind(2)
    return K.flash_attention_ext(q, k, v, causal=False, attn_mask=mask, dropout=p).reshape(B, S, heads * D)


fused_flash_qkv = _op('fused_flash_qkv', FlashQKV3Fn, _flash_eager, _flash_ok)


# -- softmax cross-entropy ---------------------------------------------------------------------------
fused_softmax_ce = _op('fused_softmax_ce', K.SoftmaxCEFn,
                       lambda logits, labels, ignore_index=-100: K.softmax_cross_entropy(logits, labels,
                                                                                          ignore_index))
