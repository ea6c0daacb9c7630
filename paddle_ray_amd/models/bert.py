"""BERT / ERNIE encoders (parity: the reference's BERT test model
python/paddle/fluid/tests/unittests/prim/model/bert.py:59-460 — BertConfig, BertEmbeddings,
BertPooler, BertModel, BertPretrainingHeads, Bert(ForPretraining), BertPretrainingCriterion —
and the ERNIE-style hybrid-parallel configs used by the Fleet tests).

MI355X mapping per post-LN encoder layer:
  fused QKV GEMM (hipBLASLt) -> non-causal flash attention (HIP MFMA kernel, packed QKV
  read in place) when there is no padding mask, else SDPA with an additive mask ->
  out-proj GEMM WITHOUT bias -> ONE fused HIP kernel for (+bias, dropout, +residual,
  LayerNorm) -> fc1 GEMM -> fused bias+GELU (HIP) -> fc2 GEMM -> fused
  (+bias, dropout, +residual, LayerNorm).
Tensor parallel (mp_degree > 1): Column/RowParallelLinear + VocabParallelEmbedding.
"""
import math
from dataclasses import dataclass

import torch

from ..framework.core import Tensor, _u
from .. import nn
from ..nn import functional as F
from ..nn import initializer as I
from ..ops import fused as K
from ..static import fn_ops as FO
from ..static.graph import Variable as _Var, static_op as _static_op


def _pad_mask(ids, pad_token_id, dtype):
    """[B, S] token ids -> [B, 1, 1, S] additive key-padding mask (-1e4 at padding)."""
    return Tensor(((_u(ids) == pad_token_id).to(dtype) * -1e4)[:, None, None, :])


# one static op (no gradient) when the ids are a Program Variable: the mask is always built
# there, since a recorded program cannot test the fed values for padding
_pad_mask_op = _static_op('bert_pad_mask', _pad_mask)


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    hidden_act: str = 'gelu'
    hidden_dropout_prob: float = 0.1
    attention_probs_dropout_prob: float = 0.1
    max_position_embeddings: int = 512
    type_vocab_size: int = 2
    initializer_range: float = 0.02
    layer_norm_eps: float = 1e-12
    pad_token_id: int = 0
    pool_act: str = 'tanh'
    mp_degree: int = 1
    recompute: bool = False
    # ERNIE 3.0 extras
    task_type_vocab_size: int = 3
    use_task_id: bool = False


BERT_CONFIGS = {
    'bert-tiny': dict(vocab_size=1024, hidden_size=128, num_hidden_layers=2,
                      num_attention_heads=2, intermediate_size=512, max_position_embeddings=128),
    'bert-base-uncased': dict(),
    'bert-large-uncased': dict(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16,
                               intermediate_size=4096),
    'ernie-1.0': dict(vocab_size=18000, max_position_embeddings=513, type_vocab_size=2,
                      hidden_act='relu', layer_norm_eps=1e-5),
    'ernie-3.0-base-zh': dict(vocab_size=40000, max_position_embeddings=2048, type_vocab_size=4,
                              use_task_id=True, layer_norm_eps=1e-5),
    'ernie-3.0-medium-zh': dict(vocab_size=40000, num_hidden_layers=6,
                                max_position_embeddings=2048, type_vocab_size=4,
                                use_task_id=True, layer_norm_eps=1e-5),
    # BASELINE config 5: ERNIE-3.0 10B class dense encoder (48 x 4096, 64 heads, 16384 FFN:
    # 9.7B encoder + 0.16B embedding parameters) for the TP=2 x PP=4 Fleet hybrid run
    'ernie-3.0-10b': dict(vocab_size=40000, hidden_size=4096, num_hidden_layers=48,
                          num_attention_heads=64, intermediate_size=16384,
                          max_position_embeddings=2048, type_vocab_size=4, layer_norm_eps=1e-5),
}


def bert_config(name, **overrides):
    d = dict(BERT_CONFIGS[name])
    d.update(overrides)
    return BertConfig(**d)


def _tp():
    from ..parallel import tensor_parallel as tp
    return tp


def _init(cfg):
    return nn.ParamAttr(initializer=I.Normal(0.0, cfg.initializer_range))


class BertEmbeddings(nn.Layer):
    def __init__(self, cfg):
        super().__init__()
        if cfg.mp_degree > 1:
            self.word_embeddings = _tp().VocabParallelEmbedding(cfg.vocab_size, cfg.hidden_size,
                                                                weight_attr=_init(cfg))
        else:
            self.word_embeddings = nn.Embedding(cfg.vocab_size, cfg.hidden_size,
                                                padding_idx=None, weight_attr=_init(cfg))
        self.position_embeddings = nn.Embedding(cfg.max_position_embeddings, cfg.hidden_size,
                                                weight_attr=_init(cfg))
        self.token_type_embeddings = nn.Embedding(cfg.type_vocab_size, cfg.hidden_size,
                                                  weight_attr=_init(cfg))
        self.use_task_id = cfg.use_task_id
        if cfg.use_task_id:
            self.task_type_embeddings = nn.Embedding(cfg.task_type_vocab_size, cfg.hidden_size,
                                                     weight_attr=_init(cfg))
        self.layer_norm = nn.LayerNorm(cfg.hidden_size, cfg.layer_norm_eps)
        self.dropout = nn.Dropout(cfg.hidden_dropout_prob)

    def forward(self, input_ids, token_type_ids=None, position_ids=None, task_type_ids=None,
                past_key_values_length=None):
        ids = _u(input_ids)
        S = ids.shape[-1]
        x = _u(self.word_embeddings(Tensor(ids)))
        # default position / token-type ids index the SAME rows for every sequence: a broadcast
        # add of the table slice (its gradient is a sum over the batch) instead of a lookup whose
        # backward sorts 16K copies of a few ids (a 16K-long run for token type 0)
        off = int(past_key_values_length or 0)
        if position_ids is None and off + S <= self.position_embeddings.weight.shape[0]:
            x = x + _u(self.position_embeddings.weight)[off:off + S]
        else:
            pos = _u(position_ids) if position_ids is not None else \
                (torch.arange(S, device=ids.device) + off).unsqueeze(0)
            x = x + _u(self.position_embeddings(Tensor(pos)))
        if token_type_ids is None:
            x = x + _u(self.token_type_embeddings.weight)[0]
        else:
            x = x + _u(self.token_type_embeddings(Tensor(_u(token_type_ids))))
        if self.use_task_id:
            tk = torch.zeros_like(ids) if task_type_ids is None else _u(task_type_ids)
            x = x + _u(self.task_type_embeddings(Tensor(tk)))
        return self.dropout(self.layer_norm(Tensor(x)))


class BertSelfAttention(nn.Layer):
    def __init__(self, cfg):
        super().__init__()
        h = cfg.hidden_size
        self.num_heads = cfg.num_attention_heads // cfg.mp_degree
        self.head_dim = h // cfg.num_attention_heads
        if cfg.mp_degree > 1:
            tp = _tp()
            self.qkv_proj = tp.ColumnParallelLinear(h, 3 * h, _init(cfg), has_bias=True,
                                                    gather_output=False)
            self.out_proj = tp.RowParallelLinear(h, h, _init(cfg), has_bias=True,
                                                 input_is_parallel=True)
        else:
            self.qkv_proj = nn.Linear(h, 3 * h, _init(cfg))
            self.out_proj = nn.Linear(h, h, _init(cfg))
        self.attn_dropout = cfg.attention_probs_dropout_prob

    def context(self, x, attn_mask=None):
        """[B, S, h] -> attention context [B, S, heads*head_dim] (before out_proj)."""
        qkv = _u(self.qkv_proj(x))
        B, S = qkv.shape[0], qkv.shape[1]
        qkv = qkv.view(B, S, 3, self.num_heads, self.head_dim)
        drop = self.attn_dropout if self.training else 0.0
        if attn_mask is None and drop == 0.0:
            o = K.flash_attention_qkvpacked(qkv, causal=False)
        else:
            # padded batches (additive mask) / attention dropout: the flash kernel's extended path
            m = None if attn_mask is None else _u(attn_mask)
            o = K.flash_attention_ext_qkvpacked(qkv, causal=False, attn_mask=m, dropout=drop)
        return o.reshape(B, S, self.num_heads * self.head_dim)

    def forward(self, x, attn_mask=None):
        return self.out_proj(Tensor(self.context(x, attn_mask)))


class BertLayer(nn.Layer):
    """Post-LN encoder layer: y = LN(x + drop(attn(x))); out = LN(y + drop(ffn(y)))."""

    def __init__(self, cfg):
        super().__init__()
        h, f = cfg.hidden_size, cfg.intermediate_size
        self.attn = BertSelfAttention(cfg)
        self.ln1 = nn.LayerNorm(h, cfg.layer_norm_eps)
        if cfg.mp_degree > 1:
            tp = _tp()
            self.fc1 = tp.ColumnParallelLinear(h, f, _init(cfg), has_bias=True,
                                               gather_output=False)
            self.fc2 = tp.RowParallelLinear(f, h, _init(cfg), has_bias=True,
                                            input_is_parallel=True)
        else:
            self.fc1 = nn.Linear(h, f, _init(cfg))
            self.fc2 = nn.Linear(f, h, _init(cfg))
        self.ln2 = nn.LayerNorm(h, cfg.layer_norm_eps)
        self.act = cfg.hidden_act
        self.p = cfg.hidden_dropout_prob
        self.eps = cfg.layer_norm_eps
        self.fused = cfg.mp_degree == 1

    def _ffn_hidden(self, y):
        if self.act == 'gelu' and self.fused:
            return K.bias_gelu(K.linear(_u(y), self.fc1.weight._t), self.fc1.bias._t, False)
        return _u(getattr(F, self.act)(self.fc1(y)))

    def forward(self, x, attn_mask=None):
        p = self.p if self.training else 0.0
        if self.fused:
            # fused ops (static/fn_ops.py): the same HIP kernels eagerly, and ONE static op each
            # with a direct grad kernel inside a Program
            at = self.attn
            qkv = FO.fused_linear(x, at.qkv_proj.weight, at.qkv_proj.bias)
            c = FO.fused_flash_qkv(qkv, attn_mask, at.num_heads, at.attn_dropout if self.training else 0.0)
            a = FO.fused_linear(c, at.out_proj.weight)
            _, y1 = FO.fused_add_dropout_ln(x, a, at.out_proj.bias, self.ln1.weight, self.ln1.bias,
                                            p, self.eps)
            if self.act == 'gelu':
                # fc1 GEMM with the bias+GELU epilogue, fc2 GEMM (its bias goes to the ADL kernel)
                m = FO.fused_mlp_gelu(y1, self.fc1.weight, self.fc1.bias, self.fc2.weight, False)
            else:
                m = FO.fused_linear(getattr(F, self.act)(self.fc1(y1)), self.fc2.weight)
            _, y2 = FO.fused_add_dropout_ln(y1, m, self.fc2.bias, self.ln2.weight, self.ln2.bias,
                                            p, self.eps)
            return y2
        drop = (lambda t: torch.nn.functional.dropout(t, p, True)) if p > 0 else (lambda t: t)
        y1 = _u(self.ln1(Tensor(_u(x) + drop(_u(self.attn(x, attn_mask))))))
        m = _u(self.fc2(Tensor(self._ffn_hidden(Tensor(y1)))))
        return self.ln2(Tensor(y1 + drop(m)))


class BertPooler(nn.Layer):
    def __init__(self, cfg):
        super().__init__()
        self.dense = nn.Linear(cfg.hidden_size, cfg.hidden_size, _init(cfg))
        self.pool_act = cfg.pool_act

    def forward(self, hidden_states):
        first = Tensor(_u(hidden_states)[:, 0])
        out = self.dense(first)
        return F.tanh(out) if self.pool_act == 'tanh' else out


class BertModel(nn.Layer):
    def __init__(self, cfg):
        super().__init__()
        self.config = self.cfg = cfg
        self.pad_token_id = cfg.pad_token_id
        self.embeddings = BertEmbeddings(cfg)
        self.encoder = nn.LayerList([BertLayer(cfg) for _ in range(cfg.num_hidden_layers)])
        self.pooler = BertPooler(cfg)

    def get_input_embeddings(self):
        return self.embeddings.word_embeddings

    def _mask(self, input_ids, attention_mask, dtype):
        if attention_mask is None and isinstance(input_ids, _Var):
            return _pad_mask_op(input_ids, self.pad_token_id, dtype)
        if attention_mask is None:
            ids = _u(input_ids)
            pad = ids == self.pad_token_id
            capturing = ids.is_cuda and torch.cuda.is_current_stream_capturing()
            if not capturing and not bool(pad.any()):
                return None  # no padding: the flash kernel path (a HIP graph keeps the mask)
            return Tensor((pad.to(dtype) * -1e4)[:, None, None, :])
        m = _u(attention_mask)
        if m.dim() == 2:
            m = (1.0 - m[:, None, None, :].to(dtype)) * -1e4
        return Tensor(m.to(dtype))

    def forward(self, input_ids, token_type_ids=None, position_ids=None, attention_mask=None,
                task_type_ids=None, output_hidden_states=False):
        x = self.embeddings(input_ids, token_type_ids, position_ids, task_type_ids)
        mask = self._mask(input_ids, attention_mask, x.dtype if isinstance(x, _Var) else _u(x).dtype)
        hs = []
        for layer in self.encoder:
            if self.cfg.recompute and self.training:
                from ..parallel.recompute import recompute
                x = recompute(layer, x, mask)
            else:
                x = layer(x, mask)
            if output_hidden_states:
                hs.append(x)
        pooled = self.pooler(x)
        return (x, pooled, hs) if output_hidden_states else (x, pooled)


class BertLMPredictionHead(nn.Layer):
    def __init__(self, cfg, embedding_weights=None):
        super().__init__()
        self.transform = nn.Linear(cfg.hidden_size, cfg.hidden_size, _init(cfg))
        self.act = cfg.hidden_act
        self.layer_norm = nn.LayerNorm(cfg.hidden_size, cfg.layer_norm_eps)
        self.decoder_weight = embedding_weights if embedding_weights is not None else \
            self.create_parameter([cfg.vocab_size, cfg.hidden_size], _init(cfg))
        self.decoder_bias = self.create_parameter([cfg.vocab_size], is_bias=True)

    def forward(self, hidden_states, masked_positions=None):
        from .. import tensor as T
        h = hidden_states
        if masked_positions is not None:
            h = T.manipulation.index_select(T.manipulation.reshape(h, [-1, h.shape[-1]]),
                                            T.manipulation.reshape(masked_positions, [-1]), 0)
        if self.act == 'gelu':
            # transform GEMM with the bias+GELU epilogue (exact erf GELU)
            h = FO.fused_bias_gelu(FO.fused_linear(h, self.transform.weight), self.transform.bias, False)
        else:
            h = getattr(F, self.act)(self.transform(h))
        h = self.layer_norm(h)
        h2 = T.manipulation.reshape(h, [-1, h.shape[-1]])
        # decoder: logits = h·Eᵀ + b on the NT GEMM (the tied [vocab, hidden] word embedding)
        return T.math.add(FO.fused_linear_nt(h2, self.decoder_weight), self.decoder_bias)


class BertPretrainingHeads(nn.Layer):
    def __init__(self, cfg, embedding_weights=None):
        super().__init__()
        self.predictions = BertLMPredictionHead(cfg, embedding_weights)
        self.seq_relationship = nn.Linear(cfg.hidden_size, 2, _init(cfg))

    def forward(self, sequence_output, pooled_output, masked_positions=None):
        return (self.predictions(sequence_output, masked_positions),
                self.seq_relationship(pooled_output))


class BertForPretraining(nn.Layer):
    """MLM + NSP. With labels returns the summed loss (MLM over non-ignored positions via
    the fused one-pass softmax-CE kernel), else (prediction_scores, seq_relationship)."""

    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        self.bert = BertModel(cfg)
        emb = self.bert.embeddings.word_embeddings.weight if cfg.mp_degree == 1 else None
        self.cls = BertPretrainingHeads(cfg, emb)

    def forward(self, input_ids, token_type_ids=None, position_ids=None, attention_mask=None,
                masked_positions=None, labels=None, next_sentence_label=None):
        seq, pooled = self.bert(input_ids, token_type_ids, position_ids, attention_mask)[:2]
        scores, nsp = self.cls(seq, pooled, masked_positions)
        if labels is None:
            return scores, nsp
        from .. import tensor as T
        lab = T.manipulation.reshape(labels, [-1])
        mlm = FO.fused_softmax_ce(T.manipulation.reshape(scores, [-1, scores.shape[-1]]), lab, -1)
        valid = T.math.clip(T.math.sum(T.manipulation.cast(T.math.not_equal(lab, -1), 'float32')),
                            min=1.0)
        loss = T.math.divide(T.math.sum(T.manipulation.cast(mlm, 'float32')), valid)
        if next_sentence_label is not None:
            loss = T.math.add(loss, F.cross_entropy(T.manipulation.cast(nsp, 'float32'),
                                                    T.manipulation.reshape(next_sentence_label, [-1])))
        return loss


class BertPretrainingCriterion(nn.Layer):
    def __init__(self, vocab_size=30522):
        super().__init__()
        self.vocab_size = vocab_size

    def forward(self, prediction_scores, seq_relationship_score, masked_lm_labels,
                next_sentence_labels, masked_lm_scale=1.0):
        s = _u(prediction_scores)
        mlm = K.softmax_cross_entropy(s.reshape(-1, s.shape[-1]),
                                      _u(masked_lm_labels).reshape(-1), -1)
        mlm = mlm.sum() / masked_lm_scale
        nsp = torch.nn.functional.cross_entropy(_u(seq_relationship_score).float(),
                                                _u(next_sentence_labels).reshape(-1),
                                                reduction='none')
        return Tensor(mlm + nsp.mean())


class BertForSequenceClassification(nn.Layer):
    def __init__(self, cfg, num_classes=2, dropout=None):
        super().__init__()
        self.bert = BertModel(cfg)
        self.dropout = nn.Dropout(cfg.hidden_dropout_prob if dropout is None else dropout)
        self.classifier = nn.Linear(cfg.hidden_size, num_classes, _init(cfg))

    def forward(self, input_ids, token_type_ids=None, position_ids=None, attention_mask=None):
        _, pooled = self.bert(input_ids, token_type_ids, position_ids, attention_mask)[:2]
        return self.classifier(self.dropout(pooled))


class BertForTokenClassification(nn.Layer):
    def __init__(self, cfg, num_classes=2, dropout=None):
        super().__init__()
        self.bert = BertModel(cfg)
        self.dropout = nn.Dropout(cfg.hidden_dropout_prob if dropout is None else dropout)
        self.classifier = nn.Linear(cfg.hidden_size, num_classes, _init(cfg))

    def forward(self, input_ids, token_type_ids=None, position_ids=None, attention_mask=None):
        seq = self.bert(input_ids, token_type_ids, position_ids, attention_mask)[0]
        return self.classifier(self.dropout(seq))


class BertForQuestionAnswering(nn.Layer):
    def __init__(self, cfg):
        super().__init__()
        self.bert = BertModel(cfg)
        self.classifier = nn.Linear(cfg.hidden_size, 2, _init(cfg))

    def forward(self, input_ids, token_type_ids=None, position_ids=None, attention_mask=None):
        seq = self.bert(input_ids, token_type_ids, position_ids, attention_mask)[0]
        logits = _u(self.classifier(seq))
        return Tensor(logits[..., 0]), Tensor(logits[..., 1])


# ERNIE = BERT architecture + optional task-type embeddings (ERNIE 3.0)
ErnieConfig = BertConfig
ErnieModel = BertModel
ErnieForPretraining = BertForPretraining
ErnieForSequenceClassification = BertForSequenceClassification
ErnieForTokenClassification = BertForTokenClassification
ErnieForQuestionAnswering = BertForQuestionAnswering


def ernie_config(name='ernie-3.0-base-zh', **overrides):
    return bert_config(name, **overrides)


# ---------------------------------------------------------------------------------------
# Pipeline form (TP x PP hybrid): embeddings | encoder layers | MLM head as LayerDescs
# ---------------------------------------------------------------------------------------
class _PipeEmbeddings(BertEmbeddings):
    def forward(self, input_ids):
        return super().forward(input_ids)


class _PipeLayer(BertLayer):
    def forward(self, x):
        return super().forward(x, None)


class _PipeHead(nn.Layer):
    def __init__(self, cfg):
        super().__init__()
        self.transform = nn.Linear(cfg.hidden_size, cfg.hidden_size, _init(cfg))
        self.layer_norm = nn.LayerNorm(cfg.hidden_size, cfg.layer_norm_eps)
        self.decoder = nn.Linear(cfg.hidden_size, cfg.vocab_size, _init(cfg))

    def forward(self, x):
        return self.decoder(self.layer_norm(F.gelu(self.transform(x))))


class _PipeHeadTransform(nn.Layer):
    def __init__(self, cfg):
        super().__init__()
        self.transform = nn.Linear(cfg.hidden_size, cfg.hidden_size, _init(cfg))
        self.layer_norm = nn.LayerNorm(cfg.hidden_size, cfg.layer_norm_eps)

    def forward(self, x):
        return self.layer_norm(F.gelu(self.transform(x)))


def _tied_decoder(emb, x):
    """MLM logits against the (pipeline-shared) word-embedding matrix."""
    h = _u(x)
    w = emb.word_embeddings.weight._t
    return Tensor(K.linear_nt(h.reshape(-1, h.shape[-1]), w).view(*h.shape[:-1], w.shape[0]))


class _MLMLoss(nn.Layer):
    def forward(self, scores, labels):
        s = _u(scores)
        return Tensor(K.softmax_cross_entropy(s.reshape(-1, s.shape[-1]),
                                              _u(labels).reshape(-1), -1).mean())


def ernie_pipe(cfg, num_stages=None, topology=None, tie_word_embeddings=False, **kw):
    """ERNIE/BERT MLM model as a ``PipelineLayer`` (layers split over pipeline stages;
    TP inside each layer when ``cfg.mp_degree > 1``). ``tie_word_embeddings``: the MLM
    decoder reuses the input word embedding across the first and last stage
    (``SharedLayerDesc('embed')``: broadcast at build, gradient all-reduced per batch)."""
    from ..parallel.pipeline import LayerDesc, PipelineLayer, SharedLayerDesc
    if tie_word_embeddings and cfg.mp_degree == 1:
        attr = 'word_embeddings.weight'
        descs = [SharedLayerDesc('embed', _PipeEmbeddings, None, attr, cfg)]
        descs += [LayerDesc(_PipeLayer, cfg) for _ in range(cfg.num_hidden_layers)]
        descs += [LayerDesc(_PipeHeadTransform, cfg),
                  SharedLayerDesc('embed', _PipeEmbeddings, _tied_decoder, attr, cfg)]
        return PipelineLayer(descs, num_stages=num_stages, topology=topology,
                             loss_fn=_MLMLoss(), **kw)
    descs = [LayerDesc(_PipeEmbeddings, cfg)]
    descs += [LayerDesc(_PipeLayer, cfg) for _ in range(cfg.num_hidden_layers)]
    descs.append(LayerDesc(_PipeHead, cfg))
    return PipelineLayer(descs, num_stages=num_stages, topology=topology, loss_fn=_MLMLoss(),
                         **kw)


def bert_flops_per_token(cfg, seq_len):
    n = 12 * cfg.num_hidden_layers * cfg.hidden_size ** 2
    return 6 * n + 12 * cfg.num_hidden_layers * cfg.hidden_size * seq_len
