"""Fused layer classes (parity: python/paddle/incubate/nn/layer/*)."""
import math

from ...nn.layer.layers import Layer
from ...nn import initializer as I
from . import functional as FF


class FusedLinear(Layer):
    def __init__(self, in_features, out_features, weight_attr=None, bias_attr=None,
                 transpose_weight=False, name=None):
        super().__init__()
        shape = [out_features, in_features] if transpose_weight else [in_features, out_features]
        self.weight = self.create_parameter(shape, weight_attr)
        self.bias = self.create_parameter([out_features], bias_attr, is_bias=True)
        self.transpose_weight = transpose_weight

    def forward(self, x):
        return FF.fused_linear(x, self.weight, self.bias, self.transpose_weight)


class FusedDropoutAdd(Layer):
    def __init__(self, p=0.5, mode="upscale_in_train", name=None):
        super().__init__()
        self.p, self.mode = p, mode

    def forward(self, x, y):
        return FF.fused_dropout_add(x, y, self.p, self.training, self.mode)


class FusedBiasDropoutResidualLayerNorm(Layer):
    def __init__(self, embed_dim, dropout_rate=0.5, weight_attr=None, bias_attr=None,
                 epsilon=1e-5, name=None):
        super().__init__()
        self.linear_bias = self.create_parameter([embed_dim], bias_attr, is_bias=True)
        self.ln_scale = self.create_parameter([embed_dim], weight_attr,
                                              default_initializer=I.Constant(1.0))
        self.ln_bias = self.create_parameter([embed_dim], bias_attr, is_bias=True)
        self.dropout_rate, self.epsilon = dropout_rate, epsilon

    def forward(self, x, residual):
        return FF.fused_bias_dropout_residual_layer_norm(x, residual, self.linear_bias,
                                                         self.ln_scale, self.ln_bias,
                                                         self.dropout_rate, self.epsilon,
                                                         self.training)


class FusedMultiHeadAttention(Layer):
    def __init__(self, embed_dim, num_heads, dropout_rate=0.5, attn_dropout_rate=0.5, kdim=None,
                 vdim=None, normalize_before=False, need_weights=False, qkv_weight_attr=None,
                 qkv_bias_attr=None, linear_weight_attr=None, linear_bias_attr=None,
                 pre_ln_scale_attr=None, pre_ln_bias_attr=None, ln_scale_attr=None,
                 ln_bias_attr=None, epsilon=1e-5, nranks=1, ring_id=-1, transpose_qkv_wb=False,
                 name=None):
        super().__init__()
        self.embed_dim, self.num_heads = embed_dim, num_heads
        self.head_dim = embed_dim // num_heads
        self.normalize_before, self.epsilon = normalize_before, epsilon
        self.dropout_rate, self.attn_dropout_rate = dropout_rate, attn_dropout_rate
        self.transpose_qkv_wb = transpose_qkv_wb
        qshape = [embed_dim, 3 * embed_dim] if transpose_qkv_wb else \
            [3, num_heads, self.head_dim, embed_dim]
        self.qkv_weight = self.create_parameter(qshape, qkv_weight_attr)
        self.qkv_bias = self.create_parameter([3 * embed_dim] if transpose_qkv_wb else
                                              [3, num_heads, self.head_dim], qkv_bias_attr,
                                              is_bias=True)
        self.linear_weight = self.create_parameter([embed_dim, embed_dim], linear_weight_attr)
        self.linear_bias = self.create_parameter([embed_dim], linear_bias_attr, is_bias=True)
        one = I.Constant(1.0)
        self.pre_ln_scale = self.create_parameter([embed_dim], pre_ln_scale_attr,
                                                  default_initializer=one)
        self.pre_ln_bias = self.create_parameter([embed_dim], pre_ln_bias_attr, is_bias=True)
        self.ln_scale = self.create_parameter([embed_dim], ln_scale_attr, default_initializer=one)
        self.ln_bias = self.create_parameter([embed_dim], ln_bias_attr, is_bias=True)

    def forward(self, query, key=None, value=None, attn_mask=None, cache=None):
        return FF.fused_multi_head_attention(
            query, self.qkv_weight, self.linear_weight, self.normalize_before, self.pre_ln_scale,
            self.pre_ln_bias, self.ln_scale, self.ln_bias, self.epsilon, self.qkv_bias,
            self.linear_bias, cache, attn_mask, self.dropout_rate, self.attn_dropout_rate,
            self.epsilon, self.training, num_heads=self.num_heads,
            transpose_qkv_wb=self.transpose_qkv_wb)


class FusedFeedForward(Layer):
    def __init__(self, d_model, dim_feedforward, dropout_rate=0.1, epsilon=1e-05,
                 activation="relu", act_dropout_rate=None, normalize_before=False,
                 linear1_weight_attr=None, linear1_bias_attr=None, linear2_weight_attr=None,
                 linear2_bias_attr=None, ln1_scale_attr=None, ln1_bias_attr=None,
                 ln2_scale_attr=None, ln2_bias_attr=None, nranks=1, ring_id=-1, name=None):
        super().__init__()
        self.dropout_rate = dropout_rate
        self.act_dropout_rate = dropout_rate if act_dropout_rate is None else act_dropout_rate
        self.activation, self.normalize_before, self.epsilon = activation, normalize_before, \
            epsilon
        self.linear1_weight = self.create_parameter([d_model, dim_feedforward], linear1_weight_attr)
        self.linear1_bias = self.create_parameter([dim_feedforward], linear1_bias_attr,
                                                  is_bias=True)
        self.linear2_weight = self.create_parameter([dim_feedforward, d_model], linear2_weight_attr)
        self.linear2_bias = self.create_parameter([d_model], linear2_bias_attr, is_bias=True)
        one = I.Constant(1.0)
        self.ln1_scale = self.create_parameter([d_model], ln1_scale_attr, default_initializer=one)
        self.ln1_bias = self.create_parameter([d_model], ln1_bias_attr, is_bias=True)
        self.ln2_scale = self.create_parameter([d_model], ln2_scale_attr, default_initializer=one)
        self.ln2_bias = self.create_parameter([d_model], ln2_bias_attr, is_bias=True)

    def forward(self, src, cache=None):
        return FF.fused_feedforward(src, self.linear1_weight, self.linear2_weight,
                                    self.linear1_bias, self.linear2_bias, self.ln1_scale,
                                    self.ln1_bias, self.ln2_scale, self.ln2_bias,
                                    self.act_dropout_rate, self.dropout_rate, self.activation,
                                    self.epsilon, self.epsilon, self.normalize_before,
                                    self.training)


class FusedTransformerEncoderLayer(Layer):
    def __init__(self, d_model, nhead, dim_feedforward, dropout_rate=0.1, activation="relu",
                 attn_dropout_rate=None, act_dropout_rate=None, normalize_before=False,
                 weight_attr=None, bias_attr=None):
        super().__init__()
        adr = dropout_rate if attn_dropout_rate is None else attn_dropout_rate
        self.fused_attn = FusedMultiHeadAttention(d_model, nhead, dropout_rate, adr,
                                                  normalize_before=normalize_before)
        self.ffn = FusedFeedForward(d_model, dim_feedforward, dropout_rate, activation=activation,
                                    act_dropout_rate=act_dropout_rate,
                                    normalize_before=normalize_before)

    def forward(self, src, src_mask=None, cache=None):
        return self.ffn(self.fused_attn(src, attn_mask=src_mask))


class FusedMultiTransformer(Layer):
    """Stack of pre/post-LN transformer layers for inference and generation, parameters in
    the reference layout (parity: python/paddle/incubate/nn/layer/fused_transformer.py
    FusedMultiTransformer): qkv [3, H, D, E], linear [E, E], ffn1 [E, F], ffn2 [F, E].
    ``forward(src, attn_mask, caches, ..., time_step)`` runs the context phase (caches
    filled in place) or, with ``time_step``, one decode step on the HIP cache kernel."""

    def __init__(self, embed_dim, num_heads, dim_feedforward, dropout_rate=0.0, activation="gelu",
                 normalize_before=True, ln_scale_attrs=None, ln_bias_attrs=None,
                 qkv_weight_attrs=None, qkv_bias_attrs=None, linear_weight_attrs=None,
                 linear_bias_attrs=None, ffn_ln_scale_attrs=None, ffn_ln_bias_attrs=None,
                 ffn1_weight_attrs=None, ffn1_bias_attrs=None, ffn2_weight_attrs=None,
                 ffn2_bias_attrs=None, epsilon=1e-5, num_layers=-1, nranks=1,
                 trans_qkvw=True, ring_id=-1, name=None):
        super().__init__()
        if num_layers < 0:
            num_layers = len(qkv_weight_attrs) if isinstance(qkv_weight_attrs, (list, tuple)) else 1
        assert embed_dim % num_heads == 0
        self.embed_dim, self.num_heads = embed_dim, num_heads
        self.head_dim = embed_dim // num_heads
        self.normalize_before, self._epsilon = normalize_before, epsilon
        self.dropout_rate, self.activation, self._trans_qkvw = dropout_rate, activation, trans_qkvw
        one = I.Constant(1.0)

        def attr(a, i):
            return a[i] if isinstance(a, (list, tuple)) else a
        names = ('ln_scales', 'ln_biases', 'qkv_weights', 'qkv_biases', 'linear_weights',
                 'linear_biases', 'ffn_ln_scales', 'ffn_ln_biases', 'ffn1_weights', 'ffn1_biases',
                 'ffn2_weights', 'ffn2_biases')
        for n in names:
            setattr(self, n, [])
        E, H, D, F = embed_dim, num_heads, self.head_dim, dim_feedforward
        qkv_shape = [3, H, D, E] if trans_qkvw else [E, 3, H, D]
        for i in range(num_layers):
            specs = (
                ('ln_scales', [E], ln_scale_attrs, False, one),
                ('ln_biases', [E], ln_bias_attrs, True, None),
                ('qkv_weights', qkv_shape, qkv_weight_attrs, False, None),
                ('qkv_biases', [3, H, D], qkv_bias_attrs, True, None),
                ('linear_weights', [E, E], linear_weight_attrs, False, None),
                ('linear_biases', [E], linear_bias_attrs, True, None),
                ('ffn_ln_scales', [E], ffn_ln_scale_attrs, False, one),
                ('ffn_ln_biases', [E], ffn_ln_bias_attrs, True, None),
                ('ffn1_weights', [E, F], ffn1_weight_attrs, False, None),
                ('ffn1_biases', [F], ffn1_bias_attrs, True, None),
                ('ffn2_weights', [F, E], ffn2_weight_attrs, False, None),
                ('ffn2_biases', [E], ffn2_bias_attrs, True, None))
            for n, shp, a, is_bias, init in specs:
                p = self.create_parameter(shp, attr(a, i), is_bias=is_bias, default_initializer=init)
                self.add_parameter(f'{n}_{i}', p)
                getattr(self, n).append(p)

    def forward(self, src, attn_mask=None, caches=None, pre_caches=None, rotary_embs=None,
                rotary_emb_dims=0, seq_lens=None, time_step=None):
        return FF.fused_multi_transformer(
            src, self.ln_scales, self.ln_biases, self.qkv_weights, self.qkv_biases,
            self.linear_weights, self.linear_biases, self.ffn_ln_scales, self.ffn_ln_biases,
            self.ffn1_weights, self.ffn1_biases, self.ffn2_weights, self.ffn2_biases,
            pre_layer_norm=self.normalize_before, epsilon=self._epsilon, cache_kvs=caches,
            pre_caches=pre_caches, seq_lens=seq_lens, rotary_embs=rotary_embs,
            time_step=time_step, attn_mask=attn_mask, dropout_rate=self.dropout_rate,
            rotary_emb_dims=rotary_emb_dims, activation=self.activation, training=self.training,
            trans_qkvw=self._trans_qkvw)


class FusedMultiTransformerDecoder:
    """Serving loop for a ``FusedMultiTransformer``: persistent KV caches, a prefill call, and
    per-token decode steps replayed from ONE captured HIP graph (the decode-attention kernel
    reads the position from a device int32 counter that the graph itself advances), so a
    step costs one graph launch instead of ~10 kernel launches per layer.

        dec = FusedMultiTransformerDecoder(model, batch_size=8, max_seq_len=2048)
        h = dec.prefill(prompt_hidden)          # [B, S0, E], fills the caches
        for _ in range(n): h_t = dec.step(x_t)  # [B, 1, E] -> [B, 1, E]
    ``attn_mask`` (additive, [B, max_seq_len]) masks padded positions across all steps.
    """

    def __init__(self, model, batch_size, max_seq_len, use_graph=True):
        import torch
        self.model = model
        self.B, self.L = int(batch_size), int(max_seq_len)
        p0 = model.qkv_weights[0]._t
        self.dev, self.dtype = p0.device, p0.dtype
        H, D, E = model.num_heads, model.head_dim, model.embed_dim
        n = len(model.qkv_weights)
        self.caches = [torch.zeros(2, self.B, H, self.L, D, device=self.dev, dtype=self.dtype)
                       for _ in range(n)]
        self.t = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self.mask = torch.zeros(self.B, 1, 1, self.L, dtype=torch.float32, device=self.dev)
        self.x_buf = torch.zeros(self.B, 1, E, device=self.dev, dtype=self.dtype)
        self.use_graph = use_graph and self.dev.type == 'cuda'
        self._graph = None
        self._out = None

    def _caches(self):
        from ...framework.core import Tensor
        return [Tensor(c) for c in self.caches]

    def set_mask(self, attn_mask):
        import torch
        m = attn_mask._t if hasattr(attn_mask, '_t') else torch.as_tensor(attn_mask)
        self.mask.copy_(m.reshape(self.B, 1, 1, self.L).to(self.mask.dtype))

    def prefill(self, x, attn_mask=None):
        """Context phase over the prompt (caches filled in place); decode continues at S0."""
        from ...framework.core import Tensor
        import torch
        xt = x._t if hasattr(x, '_t') else x
        S0 = xt.shape[1]
        if attn_mask is None:
            m = torch.triu(torch.full((S0, S0), float('-inf'), device=self.dev), 1)
            attn_mask = Tensor(m.expand(self.B, 1, S0, S0).to(self.dtype))
        with torch.no_grad():
            out, _ = self.model(Tensor(xt), attn_mask=attn_mask, caches=self._caches())
        self.t.fill_(S0)
        return out

    def _step_eager(self):
        from ...framework.core import Tensor
        out, _ = self.model(Tensor(self.x_buf), attn_mask=Tensor(self.mask), caches=self._caches(),
                            time_step=Tensor(self.t))
        return out._t

    def step(self, x_tok):
        """One token for every sequence: returns [B, 1, E]; the position advances by one."""
        import torch
        from ...framework.core import Tensor
        xt = x_tok._t if hasattr(x_tok, '_t') else x_tok
        self.x_buf.copy_(xt.reshape(self.x_buf.shape))
        with torch.no_grad():
            if not self.use_graph:
                out = self._step_eager()
                self.t.add_(1)
                return Tensor(out)
            if self._graph is None:
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):  # warm-up (rewrites the same cache slot, t unchanged)
                    self._step_eager()
                torch.cuda.current_stream().wait_stream(s)
                self._graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self._graph):
                    self._out = self._step_eager()
                    self.t.add_(1)
            self._graph.replay()
        return Tensor(self._out.clone())


class FusedEcMoe(Layer):
    def __init__(self, hidden_size, inter_size, num_experts, act_type, weight_attr=None,
                 bias_attr=None):
        super().__init__()
        self.bmm_weight0 = self.create_parameter([num_experts, hidden_size, inter_size],
                                                 weight_attr)
        self.bmm_bias0 = self.create_parameter([num_experts, 1, inter_size], bias_attr,
                                               is_bias=True)
        self.bmm_weight1 = self.create_parameter([num_experts, inter_size, hidden_size],
                                                 weight_attr)
        self.bmm_bias1 = self.create_parameter([num_experts, 1, hidden_size], bias_attr,
                                               is_bias=True)
        self.act_type = act_type

    def forward(self, x, gate):
        return FF.fused_ec_moe(x, gate, self.bmm_weight0, self.bmm_bias0, self.bmm_weight1,
                               self.bmm_bias1, self.act_type)
