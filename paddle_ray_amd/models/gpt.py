"""GPT-3 family (parity: PaddleNLP GPT used by the reference's Fleet benchmarks; layer
structure as in python/paddle/nn/layer/transformer.py pre-LN decoder).

MI355X mapping per block:
  LN (HIP row kernel) -> fused QKV GEMM (hipBLASLt, bias epilogue) -> causal flash
  attention (HIP MFMA kernel, reads Q/K/V as strided views of the QKV output, no
  transposes) -> out-proj GEMM -> residual; LN -> fc1 GEMM -> bias+GELU (HIP,
  fused) -> fc2 GEMM -> residual. Logits = h @ E^T (tied) -> fused one-pass
  softmax-CE (HIP) — the [tokens, vocab] probability matrix is never stored.
Tensor parallel (mp_degree > 1) swaps in Column/RowParallelLinear,
VocabParallelEmbedding and ParallelCrossEntropy and keeps every fusion: the block input
enters the TP region through an identity/all-reduce-grad op, the rank-local QKV GEMM +
flash attention + out-proj (and fc1 GEMM+bias+GELU + fc2) produce partial sums that are
all-reduced ONCE, and the fused add+dropout+LayerNorm kernel adds the replicated bias,
residual and next LN after the all-reduce. The embedding is the HIP lookup on shifted ids
and the loss is the one-pass vocab-parallel softmax-CE kernel.
"""
import math
from dataclasses import dataclass

import torch

from ..framework.core import Tensor, _u
from .. import nn
from ..nn import functional as F
from ..nn import initializer as I
from ..ops import fused as K


@dataclass
class GPTConfig:
    vocab_size: int = 50304
    hidden_size: int = 2048
    num_layers: int = 24
    num_heads: int = 16
    ffn_hidden_size: int = 8192
    max_seq_len: int = 1024
    hidden_dropout: float = 0.1
    attention_dropout: float = 0.0
    initializer_range: float = 0.02
    layer_norm_eps: float = 1e-5
    mp_degree: int = 1
    recompute: bool = False
    gelu_approximate: bool = True


GPT_CONFIGS = {
    'gpt3-tiny': dict(vocab_size=1024, hidden_size=128, num_layers=2, num_heads=4,
                      ffn_hidden_size=512, max_seq_len=128),
    'gpt3-125m': dict(hidden_size=768, num_layers=12, num_heads=12, ffn_hidden_size=3072,
                      max_seq_len=1024),
    'gpt3-350m': dict(hidden_size=1024, num_layers=24, num_heads=16, ffn_hidden_size=4096),
    'gpt3-1.3b': dict(hidden_size=2048, num_layers=24, num_heads=16, ffn_hidden_size=8192),
    'gpt3-2.7b': dict(hidden_size=2560, num_layers=32, num_heads=32, ffn_hidden_size=10240),
    'gpt3-6.7b': dict(hidden_size=4096, num_layers=32, num_heads=32, ffn_hidden_size=16384),
    'gpt3-13b': dict(hidden_size=5120, num_layers=40, num_heads=40, ffn_hidden_size=20480),
}


def gpt_config(name, **overrides):
    d = dict(GPT_CONFIGS[name])
    d.update(overrides)
    return GPTConfig(**d)


def _mp():
    from ..parallel import tensor_parallel as tp
    return tp


class GPTEmbeddings(nn.Layer):
    def __init__(self, cfg):
        super().__init__()
        init = I.Normal(0.0, cfg.initializer_range)
        if cfg.mp_degree > 1:
            self.word_embeddings = _mp().VocabParallelEmbedding(
                cfg.vocab_size, cfg.hidden_size, weight_attr=nn.ParamAttr(initializer=init))
        else:
            self.word_embeddings = nn.Embedding(cfg.vocab_size, cfg.hidden_size,
                                                weight_attr=nn.ParamAttr(initializer=init))
        self.position_embeddings = nn.Embedding(cfg.max_seq_len, cfg.hidden_size,
                                                weight_attr=nn.ParamAttr(initializer=init))
        self.dropout = nn.Dropout(cfg.hidden_dropout)

    def forward(self, input_ids, position_ids=None):
        ids = _u(input_ids)
        if position_ids is None:
            pos = torch.arange(ids.shape[-1], device=ids.device).unsqueeze(0)
        else:
            pos = _u(position_ids)
        x = self.word_embeddings(Tensor(ids))._t + self.position_embeddings(Tensor(pos))._t
        return self.dropout(Tensor(x))


class GPTAttention(nn.Layer):
    def __init__(self, cfg, layer_idx):
        super().__init__()
        h = cfg.hidden_size
        self.num_heads = cfg.num_heads // cfg.mp_degree
        self.head_dim = h // cfg.num_heads
        init = I.Normal(0.0, cfg.initializer_range)
        out_init = I.Normal(0.0, cfg.initializer_range / math.sqrt(2.0 * cfg.num_layers))
        if cfg.mp_degree > 1:
            tp = _mp()
            self.qkv_proj = tp.ColumnParallelLinear(h, 3 * h, nn.ParamAttr(initializer=init),
                                                    has_bias=True, gather_output=False)
            self.out_proj = tp.RowParallelLinear(h, h, nn.ParamAttr(initializer=out_init),
                                                 has_bias=True, input_is_parallel=True)
        else:
            self.qkv_proj = nn.Linear(h, 3 * h, nn.ParamAttr(initializer=init))
            self.out_proj = nn.Linear(h, h, nn.ParamAttr(initializer=out_init))
        self.attn_dropout = cfg.attention_dropout
        self.mp = cfg.mp_degree

    def _core(self, x, pair=None):
        if pair is not None:
            # QKV projection as a paired Linear: its backward also issues the output
            # projection's weight gradient, both in one grouped launch (ops/fused.py WgradPair)
            qp = self.qkv_proj
            qkv = K.linear(_u(x), qp.weight._t, qp.bias._t if qp.bias is not None else None, pair=pair,
                           w_dep=self.out_proj.weight._t)
        else:
            qkv = _u(self.qkv_proj(x))
        B, S = qkv.shape[0], qkv.shape[1]
        qkv = qkv.view(B, S, 3, self.num_heads, self.head_dim)
        if self.attn_dropout > 0 and self.training:
            # in-kernel dropout on the attention probabilities (flash kernel, same bits in bwd)
            q, k, v = qkv.unbind(2)
            o = K.flash_attention_ext(q, k, v, causal=True, dropout=self.attn_dropout)
        else:
            o = K.flash_attention_qkvpacked(qkv, causal=True)
        return o.reshape(B, S, self.num_heads * self.head_dim)

    def forward_nobias(self, x):
        """attention output projection WITHOUT its bias (fused into the next kernel). Under
        TP the row-parallel partial sums are all-reduced here (bias added after, once)."""
        pair = None
        if self.mp == 1 and _u(x).is_cuda and self.training:
            pair = K.WgradPair()
        a = K.linear(self._core(x, pair), self.out_proj.weight._t, pair=pair)
        if self.mp > 1:
            a = _mp()._AllReduce.apply(a, self.out_proj.model_parallel_group)
        return Tensor(a)

    def forward(self, x):
        qkv = _u(self.qkv_proj(x))
        B, S = qkv.shape[0], qkv.shape[1]
        qkv = qkv.view(B, S, 3, self.num_heads, self.head_dim)
        q, k, v = qkv.unbind(2)
        if self.attn_dropout > 0 and self.training:
            o = K.flash_attention_ext(q, k, v, causal=True, dropout=self.attn_dropout)
        else:
            o = K.flash_attention(q, k, v, causal=True)
        return self.out_proj(Tensor(o.reshape(B, S, self.num_heads * self.head_dim)))


class GPTMLP(nn.Layer):
    def __init__(self, cfg):
        super().__init__()
        h, f = cfg.hidden_size, cfg.ffn_hidden_size
        init = I.Normal(0.0, cfg.initializer_range)
        out_init = I.Normal(0.0, cfg.initializer_range / math.sqrt(2.0 * cfg.num_layers))
        self.approx = cfg.gelu_approximate
        if cfg.mp_degree > 1:
            tp = _mp()
            self.fc1 = tp.ColumnParallelLinear(h, f, nn.ParamAttr(initializer=init),
                                               has_bias=True, gather_output=False)
            self.fc2 = tp.RowParallelLinear(f, h, nn.ParamAttr(initializer=out_init),
                                            has_bias=True, input_is_parallel=True)
            self._fused = False
        else:
            self.fc1 = nn.Linear(h, f, nn.ParamAttr(initializer=init))
            self.fc2 = nn.Linear(f, h, nn.ParamAttr(initializer=out_init))
            self._fused = True
        self.mp = cfg.mp_degree

    def forward_nobias(self, x):
        """fc2(gelu(fc1 x)) without fc2's bias (fused into the next kernel). On the device the
        bias+GELU and its backward live in the GEMM epilogues (K.mlp_gelu). Under TP fc1/fc2
        are the rank's column/row shards: identity-in (grad all-reduce), all-reduce out."""
        t = _u(x)
        if self.mp > 1:
            t = _mp()._Identity.apply(t, self.fc1.model_parallel_group)
        if t.is_cuda:
            o = K.mlp_gelu(t, self.fc1.weight._t, self.fc1.bias._t, self.fc2.weight._t, self.approx)
        else:
            hdn = K.bias_gelu(K.linear(t, self.fc1.weight._t), self.fc1.bias._t, self.approx)
            o = K.linear(hdn, self.fc2.weight._t)
        if self.mp > 1:
            o = _mp()._AllReduce.apply(o, self.fc2.model_parallel_group)
        return Tensor(o)

    def forward(self, x):
        if self._fused:
            # GEMM without bias, then the fused bias+GELU HIP kernel (one pass over [T, 4h])
            t = _u(x)
            hdn = K.linear(t, self.fc1.weight._t)
            hdn = K.bias_gelu(hdn, self.fc1.bias._t, self.approx)
            return self.fc2(Tensor(hdn))
        return self.fc2(F.gelu(self.fc1(x), approximate=self.approx))


class GPTBlock(nn.Layer):
    def __init__(self, cfg, layer_idx):
        super().__init__()
        self.ln1 = nn.LayerNorm(cfg.hidden_size, cfg.layer_norm_eps)
        # the fused path applies ln1 at the end of the PREVIOUS block (add+dropout+LN): its
        # parameters are read outside this block's forward, so ZeRO-3 keeps them resident
        self.ln1._zero3_resident = True
        self.attn = GPTAttention(cfg, layer_idx)
        self.ln2 = nn.LayerNorm(cfg.hidden_size, cfg.layer_norm_eps)
        self.mlp = GPTMLP(cfg)
        self.p = cfg.hidden_dropout
        self.eps = cfg.layer_norm_eps
        self.fused = True

    def _drop(self, t):
        if self.p > 0 and self.training:
            return torch.nn.functional.dropout(t, self.p, True)
        return t

    def forward(self, x, y=None, next_ln=None):
        """Unfused reference path: x -> x + attn(ln1 x) -> + mlp(ln2 .). With ``y`` given this
        is the fused path ``forward_fused(x, y, next_ln)``; both are reached through
        ``__call__`` so forward hooks (ZeRO-3 gather/release, recompute) see every block."""
        if y is not None:
            return self.forward_fused(_u(x), _u(y), next_ln)
        t = _u(x)
        t = t + self._drop(_u(self.attn(self.ln1(Tensor(t)))))
        t = t + self._drop(_u(self.mlp(self.ln2(Tensor(t)))))
        return Tensor(t)

    def forward_fused(self, r, y, next_ln):
        """(r, y=ln1(r)) -> (r', next_ln(r')) with both residual adds, dropouts, out-proj /
        fc2 bias-adds and the following LayerNorms done by the fused HIP kernel."""
        p = self.p if self.training else 0.0
        a = _u(self.attn.forward_nobias(Tensor(y)))
        r1, y1 = K.add_dropout_layer_norm(r, a, self.attn.out_proj.bias._t, self.ln2.weight._t,
                                          self.ln2.bias._t, p, self.eps)
        m = _u(self.mlp.forward_nobias(Tensor(y1)))
        return K.add_dropout_layer_norm(r1, m, self.mlp.fc2.bias._t, next_ln.weight._t,
                                        next_ln.bias._t, p, self.eps)


class GPTModel(nn.Layer):
    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        self.embeddings = GPTEmbeddings(cfg)
        self.layers = nn.LayerList([GPTBlock(cfg, i) for i in range(cfg.num_layers)])
        self.final_norm = nn.LayerNorm(cfg.hidden_size, cfg.layer_norm_eps)

    def forward(self, input_ids, position_ids=None):
        x = self.embeddings(input_ids, position_ids)
        blocks = list(self.layers)
        if blocks and blocks[0].fused:
            r = _u(x)
            y = _u(blocks[0].ln1(x))
            for i, blk in enumerate(blocks):
                nxt = blocks[i + 1].ln1 if i + 1 < len(blocks) else self.final_norm
                if self.cfg.recompute and self.training:
                    from ..parallel.recompute import recompute
                    r, y = recompute(lambda a, b, blk=blk, nxt=nxt: tuple(
                        Tensor(t) for t in blk(a, b, nxt)), Tensor(r), Tensor(y))
                    r, y = _u(r), _u(y)
                else:
                    r, y = blk(r, y, nxt)
            return Tensor(y)
        if self.cfg.recompute and self.training:
            from ..parallel.recompute import recompute
            for blk in blocks:
                x = recompute(blk, x)
        else:
            for blk in blocks:
                x = blk(x)
        return self.final_norm(x)


class GPTForPretraining(nn.Layer):
    """Returns mean token loss when labels are given, else logits."""

    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        self.gpt = GPTModel(cfg)
        if cfg.mp_degree > 1:
            self._pce = _mp().ParallelCrossEntropy()

    def forward(self, input_ids, labels=None, position_ids=None):
        h = _u(self.gpt(input_ids, position_ids))
        w = self.gpt.embeddings.word_embeddings.weight._t
        if self.cfg.mp_degree > 1:
            h = _u(_mp()._c_identity(Tensor(h), self.gpt.embeddings.word_embeddings
                                     .model_parallel_group))
        B, S, H = h.shape
        logits = K.linear_nt(h.reshape(B * S, H), w)  # tied head, dW accumulated in place
        if labels is None:
            return Tensor(logits.view(B, S, -1))
        lab = _u(labels).reshape(-1)
        if self.cfg.mp_degree > 1:
            loss = self._pce(Tensor(logits), Tensor(lab))._t.mean()
        else:
            loss = K.softmax_cross_entropy(logits, lab, -100).mean()
        return Tensor(loss)


def gpt_flops_per_token(cfg, seq_len):
    """Model FLOPs per trained token (fwd+bwd = 3x fwd; causal attention counted full as in
    the usual 6N + 12·L·H·S convention)."""
    n = 12 * cfg.num_layers * cfg.hidden_size ** 2 + cfg.vocab_size * cfg.hidden_size
    return 6 * n + 12 * cfg.num_layers * cfg.hidden_size * seq_len
