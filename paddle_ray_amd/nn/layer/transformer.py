"""Transformer layers (parity: python/paddle/nn/layer/transformer.py).

MultiHeadAttention runs on the gfx950 flash-attention kernels: the plain kernel without a
mask or dropout, the extended kernel (additive / padding mask, in-kernel dropout) otherwise.
Only ``need_weights=True`` (the probabilities are returned) uses a composed softmax(QK^T)V.
"""
import collections
import copy

import torch

from ...framework.core import Tensor, _u
from .. import functional as F
from .common import Dropout, Linear, LayerList
from .layers import Layer
from .norm import LayerNorm
from ...ops import fused as K


def _convert_attention_mask(attn_mask, dtype):
    if attn_mask is None:
        return None
    m = _u(attn_mask)
    if m.dtype == torch.bool:
        return torch.where(m, torch.zeros((), dtype=dtype, device=m.device),
                           torch.full((), -1e9, dtype=dtype, device=m.device))
    if not m.is_floating_point():
        return (m.to(dtype) - 1.0) * 1e9
    return m.to(dtype)


class MultiHeadAttention(Layer):
    Cache = collections.namedtuple("Cache", ["k", "v"])
    StaticCache = collections.namedtuple("StaticCache", ["k", "v"])

    def __init__(self, embed_dim, num_heads, dropout=0., kdim=None, vdim=None, need_weights=False,
                 weight_attr=None, bias_attr=None):
        super().__init__()
        self.embed_dim, self.num_heads = embed_dim, num_heads
        self.kdim, self.vdim = kdim or embed_dim, vdim or embed_dim
        self.dropout, self.need_weights = dropout, need_weights
        self.head_dim = embed_dim // num_heads
        assert self.head_dim * num_heads == embed_dim
        self.q_proj = Linear(embed_dim, embed_dim, weight_attr, bias_attr)
        self.k_proj = Linear(self.kdim, embed_dim, weight_attr, bias_attr)
        self.v_proj = Linear(self.vdim, embed_dim, weight_attr, bias_attr)
        self.out_proj = Linear(embed_dim, embed_dim, weight_attr, bias_attr)

    def _split(self, x):
        t = _u(x)
        return t.reshape(t.shape[0], t.shape[1], self.num_heads, self.head_dim)

    def gen_cache(self, key, value=None, type=Cache):
        if type == MultiHeadAttention.StaticCache:
            return self.StaticCache(Tensor(self._split(self.k_proj(key))),
                                    Tensor(self._split(self.v_proj(value if value is not None
                                                                   else key))))
        k = _u(key)
        z = torch.zeros(k.shape[0], 0, self.num_heads, self.head_dim, dtype=k.dtype, device=k.device)
        return self.Cache(Tensor(z), Tensor(z.clone()))

    def forward(self, query, key=None, value=None, attn_mask=None, cache=None):
        key = query if key is None else key
        value = query if value is None else value
        q = self._split(self.q_proj(query))
        if isinstance(cache, self.StaticCache):
            k, v = _u(cache.k), _u(cache.v)
        else:
            k = self._split(self.k_proj(key))
            v = self._split(self.v_proj(value))
            if isinstance(cache, self.Cache):
                k = torch.cat([_u(cache.k), k], 1)
                v = torch.cat([_u(cache.v), v], 1)
                cache = self.Cache(Tensor(k), Tensor(v))
        drop = self.dropout if self.training else 0.0
        weights = None
        if self.need_weights:
            # the probabilities are an output: the composed softmax(QK^T)V path
            qt, kt, vt = (t.transpose(1, 2) for t in (q, k, v))
            s = torch.matmul(qt, kt.transpose(-1, -2)) * (self.head_dim ** -0.5)
            m = _convert_attention_mask(attn_mask, s.dtype)
            if m is not None:
                s = s + m
            p = torch.softmax(s, -1)
            weights = p
            if drop:
                p = torch.nn.functional.dropout(p, drop, True)
            o = torch.matmul(p, vt).transpose(1, 2)
        elif attn_mask is None and drop == 0.0 and q.is_cuda and \
                q.dtype in (torch.bfloat16, torch.float16):
            o = K.flash_attention(q, k, v, causal=False)
        else:
            # additive / boolean padding masks and attention dropout: the flash kernel's extended
            # path (mask added to the scaled scores, dropout bits drawn in-kernel); on the host
            # and for head dims the kernel does not cover, the same math in fp32 / torch SDPA
            m = _convert_attention_mask(attn_mask, q.dtype if q.is_cuda else torch.float32)
            o = K.flash_attention_ext(q, k, v, causal=False, attn_mask=m, dropout=drop).to(q.dtype)
        o = o.reshape(o.shape[0], o.shape[1], self.embed_dim)
        out = self.out_proj(Tensor(o))
        outs = [out]
        if self.need_weights:
            outs.append(Tensor(weights) if weights is not None else None)
        if cache is not None:
            outs.append(cache)
        return out if len(outs) == 1 else tuple(outs)


def _act_fn(name):
    return getattr(F, name)


class TransformerEncoderLayer(Layer):
    def __init__(self, d_model, nhead, dim_feedforward, dropout=0.1, activation="relu",
                 attn_dropout=None, act_dropout=None, normalize_before=False, weight_attr=None,
                 bias_attr=None, layer_norm_eps=1e-5):
        super().__init__()
        attn_dropout = dropout if attn_dropout is None else attn_dropout
        act_dropout = dropout if act_dropout is None else act_dropout
        self.normalize_before = normalize_before
        self.self_attn = MultiHeadAttention(d_model, nhead, attn_dropout, weight_attr=weight_attr,
                                            bias_attr=bias_attr)
        self.linear1 = Linear(d_model, dim_feedforward, weight_attr, bias_attr)
        self.dropout = Dropout(act_dropout, mode="upscale_in_train")
        self.linear2 = Linear(dim_feedforward, d_model, weight_attr, bias_attr)
        self.norm1 = LayerNorm(d_model, layer_norm_eps)
        self.norm2 = LayerNorm(d_model, layer_norm_eps)
        self.dropout1 = Dropout(dropout, mode="upscale_in_train")
        self.dropout2 = Dropout(dropout, mode="upscale_in_train")
        self.activation = _act_fn(activation)

    def forward(self, src, src_mask=None, cache=None):
        residual = src
        if self.normalize_before:
            src = self.norm1(src)
        if cache is None:
            src = self.self_attn(src, src, src, src_mask)
        else:
            src, incremental_cache = self.self_attn(src, src, src, src_mask, cache)
        src = residual + self.dropout1(src)
        if not self.normalize_before:
            src = self.norm1(src)
        residual = src
        if self.normalize_before:
            src = self.norm2(src)
        src = self.linear2(self.dropout(self.activation(self.linear1(src))))
        src = residual + self.dropout2(src)
        if not self.normalize_before:
            src = self.norm2(src)
        return src if cache is None else (src, incremental_cache)

    def gen_cache(self, src):
        return self.self_attn.gen_cache(src, type=self.self_attn.Cache)


class TransformerEncoder(Layer):
    def __init__(self, encoder_layer, num_layers, norm=None):
        super().__init__()
        self.layers = LayerList([encoder_layer if i == 0 else copy.deepcopy(encoder_layer)
                                 for i in range(num_layers)])
        self.num_layers = num_layers
        self.norm = norm

    def forward(self, src, src_mask=None, cache=None):
        out = src
        new_caches = []
        for i, mod in enumerate(self.layers):
            if cache is None:
                out = mod(out, src_mask)
            else:
                out, c = mod(out, src_mask, cache[i])
                new_caches.append(c)
        if self.norm is not None:
            out = self.norm(out)
        return out if cache is None else (out, new_caches)

    def gen_cache(self, src):
        return [l.gen_cache(src) for l in self.layers]


class TransformerDecoderLayer(Layer):
    def __init__(self, d_model, nhead, dim_feedforward, dropout=0.1, activation="relu",
                 attn_dropout=None, act_dropout=None, normalize_before=False, weight_attr=None,
                 bias_attr=None, layer_norm_eps=1e-5):
        super().__init__()
        attn_dropout = dropout if attn_dropout is None else attn_dropout
        act_dropout = dropout if act_dropout is None else act_dropout
        self.normalize_before = normalize_before
        self.self_attn = MultiHeadAttention(d_model, nhead, attn_dropout, weight_attr=weight_attr,
                                            bias_attr=bias_attr)
        self.cross_attn = MultiHeadAttention(d_model, nhead, attn_dropout, weight_attr=weight_attr,
                                             bias_attr=bias_attr)
        self.linear1 = Linear(d_model, dim_feedforward, weight_attr, bias_attr)
        self.dropout = Dropout(act_dropout)
        self.linear2 = Linear(dim_feedforward, d_model, weight_attr, bias_attr)
        self.norm1 = LayerNorm(d_model, layer_norm_eps)
        self.norm2 = LayerNorm(d_model, layer_norm_eps)
        self.norm3 = LayerNorm(d_model, layer_norm_eps)
        self.dropout1 = Dropout(dropout)
        self.dropout2 = Dropout(dropout)
        self.dropout3 = Dropout(dropout)
        self.activation = _act_fn(activation)

    def forward(self, tgt, memory, tgt_mask=None, memory_mask=None, cache=None):
        residual = tgt
        if self.normalize_before:
            tgt = self.norm1(tgt)
        if cache is None:
            tgt = self.self_attn(tgt, tgt, tgt, tgt_mask, None)
        else:
            tgt, inc = self.self_attn(tgt, tgt, tgt, tgt_mask, cache[0])
        tgt = residual + self.dropout1(tgt)
        if not self.normalize_before:
            tgt = self.norm1(tgt)
        residual = tgt
        if self.normalize_before:
            tgt = self.norm2(tgt)
        if cache is None:
            tgt = self.cross_attn(tgt, memory, memory, memory_mask, None)
        else:
            tgt, sc = self.cross_attn(tgt, memory, memory, memory_mask, cache[1])
        tgt = residual + self.dropout2(tgt)
        if not self.normalize_before:
            tgt = self.norm2(tgt)
        residual = tgt
        if self.normalize_before:
            tgt = self.norm3(tgt)
        tgt = self.linear2(self.dropout(self.activation(self.linear1(tgt))))
        tgt = residual + self.dropout3(tgt)
        if not self.normalize_before:
            tgt = self.norm3(tgt)
        return tgt if cache is None else (tgt, (inc, sc))

    def gen_cache(self, memory):
        inc = self.self_attn.gen_cache(memory, type=self.self_attn.Cache)
        st = self.cross_attn.gen_cache(memory, memory, type=self.cross_attn.StaticCache)
        return inc, st


class TransformerDecoder(Layer):
    def __init__(self, decoder_layer, num_layers, norm=None):
        super().__init__()
        self.layers = LayerList([decoder_layer if i == 0 else copy.deepcopy(decoder_layer)
                                 for i in range(num_layers)])
        self.num_layers = num_layers
        self.norm = norm

    def forward(self, tgt, memory, tgt_mask=None, memory_mask=None, cache=None):
        out = tgt
        new_caches = []
        for i, mod in enumerate(self.layers):
            if cache is None:
                out = mod(out, memory, tgt_mask, memory_mask, None)
            else:
                out, c = mod(out, memory, tgt_mask, memory_mask, cache[i])
                new_caches.append(c)
        if self.norm is not None:
            out = self.norm(out)
        return out if cache is None else (out, new_caches)

    def gen_cache(self, memory, do_zip=False):
        c = [l.gen_cache(memory) for l in self.layers]
        return list(zip(*c)) if do_zip else c


class Transformer(Layer):
    def __init__(self, d_model=512, nhead=8, num_encoder_layers=6, num_decoder_layers=6,
                 dim_feedforward=2048, dropout=0.1, activation="relu", attn_dropout=None,
                 act_dropout=None, normalize_before=False, weight_attr=None, bias_attr=None,
                 custom_encoder=None, custom_decoder=None):
        super().__init__()
        self.encoder = custom_encoder or TransformerEncoder(
            TransformerEncoderLayer(d_model, nhead, dim_feedforward, dropout, activation,
                                    attn_dropout, act_dropout, normalize_before, weight_attr,
                                    bias_attr), num_encoder_layers,
            LayerNorm(d_model) if normalize_before else None)
        self.decoder = custom_decoder or TransformerDecoder(
            TransformerDecoderLayer(d_model, nhead, dim_feedforward, dropout, activation,
                                    attn_dropout, act_dropout, normalize_before, weight_attr,
                                    bias_attr), num_decoder_layers,
            LayerNorm(d_model) if normalize_before else None)
        self.d_model, self.nhead = d_model, nhead

    def forward(self, src, tgt, src_mask=None, tgt_mask=None, memory_mask=None):
        memory = self.encoder(src, src_mask)
        return self.decoder(tgt, memory, tgt_mask, memory_mask)

    @staticmethod
    def generate_square_subsequent_mask(length):
        m = torch.triu(torch.full((length, length), float('-inf')), 1)
        return Tensor(m)
