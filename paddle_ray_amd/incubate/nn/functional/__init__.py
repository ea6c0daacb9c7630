"""Fused transformer functionals (parity: python/paddle/incubate/nn/functional/fused_transformer.py,
fused_matmul_bias.py, fused_dropout_add.py, fused_ec_moe.py).

Mapped onto the gfx950 kernels: LayerNorm, bias+GELU, flash attention, and
hipBLASLt GEMMs with bias epilogue (addmm)."""
import math

import torch

from ....framework.core import Tensor, _u
from ....ops import fused as K


def _t(x):
    return None if x is None else _u(x)


def _drop(x, p, training, mode='upscale_in_train'):
    if not training or p == 0:
        return x if mode == 'upscale_in_train' or training else x * (1 - p)
    return torch.nn.functional.dropout(x, p, True) if mode == 'upscale_in_train' else \
        x * (torch.rand_like(x, dtype=torch.float32) >= p).to(x.dtype)


def _ln(x, w, b, eps):
    return K.layer_norm(x, _t(w), _t(b), eps)


def fused_matmul_bias(x, y, bias=None, transpose_x=False, transpose_y=False, name=None):
    a, b = _u(x), _u(y)
    if transpose_x:
        a = a.transpose(-1, -2)
    if transpose_y:
        b = b.transpose(-1, -2)
    if bias is not None and a.dim() == 2:
        return Tensor(torch.addmm(_u(bias), a, b))
    out = torch.matmul(a, b)
    return Tensor(out if bias is None else out + _u(bias))


def fused_linear(x, weight, bias=None, transpose_weight=False, name=None):
    return fused_matmul_bias(x, weight, bias, False, transpose_weight)


def fused_linear_activation(x, y, bias, trans_x=False, trans_y=False, activation=None):
    """act(x @ y + bias) with the epilogue fused into one gfx950 MFMA GEMM launch
    (ops/csrc/gemm.hip; parity: reference python/paddle/incubate/nn/functional/
    fused_matmul_bias.py `fused_linear_activation`, activation in {None, 'none', 'gelu', 'relu'})."""
    a, b = _u(x), _u(y)
    if trans_x:
        a = a.transpose(-1, -2)
    if trans_y:
        b = b.t().contiguous()
    if activation not in (None, 'none', 'gelu', 'gelu_tanh', 'relu'):
        raise ValueError(f"fused_linear_activation: unsupported activation {activation!r}")
    return Tensor(K.gemm_bias_act(a, b, _t(bias), activation))


def fused_dropout_add(x, y, p=0.5, training=True, mode='upscale_in_train', name=None):
    return Tensor(_drop(_u(x), p, training, mode) + _u(y))


def fused_bias_dropout_residual_layer_norm(x, residual, bias=None, ln_scale=None, ln_bias=None,
                                           dropout_rate=0.5, ln_epsilon=1e-5, training=True,
                                           mode='upscale_in_train', name=None):
    h = _u(x) if bias is None else _u(x) + _u(bias)
    h = _u(residual) + _drop(h, dropout_rate, training, mode)
    return Tensor(_ln(h, ln_scale, ln_bias, ln_epsilon))


def fused_multi_head_attention(x, qkv_weight, linear_weight, pre_layer_norm=False,
                               pre_ln_scale=None, pre_ln_bias=None, ln_scale=None, ln_bias=None,
                               pre_ln_epsilon=1e-05, qkv_bias=None, linear_bias=None, cache_kv=None,
                               attn_mask=None, dropout_rate=0.5, attn_dropout_rate=0.5,
                               ln_epsilon=1e-05, training=True, mode='upscale_in_train',
                               ring_id=-1, add_residual=True, num_heads=-1, transpose_qkv_wb=False,
                               name=None):
    t = _u(x)
    B, S, E = t.shape
    residual = t
    h = _ln(t, pre_ln_scale, pre_ln_bias, pre_ln_epsilon) if pre_layer_norm else t
    w = _u(qkv_weight)
    if transpose_qkv_wb:  # [E, 3E]
        qkv = h @ w
        nh = num_heads
        if qkv_bias is not None:
            qkv = qkv + _u(qkv_bias)
        qkv = qkv.view(B, S, 3, nh, E // nh)
    else:  # [3, nh, hd, E]
        _, nh, hd, _ = w.shape
        qkv = torch.einsum('bse,tnde->bstnd', h, w)
        if qkv_bias is not None:
            qkv = qkv + _u(qkv_bias)
    q, k, v = qkv.unbind(2)
    if cache_kv is not None:
        ck = _u(cache_kv)
        k = torch.cat([ck[0].transpose(1, 2), k], 1)
        v = torch.cat([ck[1].transpose(1, 2), v], 1)
    hd = q.shape[-1]
    if attn_mask is None and (attn_dropout_rate == 0 or not training) and t.is_cuda and \
            t.dtype in (torch.bfloat16, torch.float16):
        o = K.flash_attention(q, k, v, causal=False)
    else:
        s = torch.einsum('bqnd,bknd->bnqk', q, k) / math.sqrt(hd)
        if attn_mask is not None:
            s = s + _u(attn_mask)
        p = _drop(torch.softmax(s.float(), -1).to(s.dtype), attn_dropout_rate, training, mode)
        o = torch.einsum('bnqk,bknd->bqnd', p, v)
    o = o.reshape(B, S, -1)
    out = o @ _u(linear_weight)
    if linear_bias is not None:
        out = out + _u(linear_bias)
    out = _drop(out, dropout_rate, training, mode)
    if add_residual:
        out = residual + out
    if not pre_layer_norm:
        out = _ln(out, ln_scale, ln_bias, ln_epsilon)
    if cache_kv is not None:
        return Tensor(out), Tensor(torch.stack([k.transpose(1, 2), v.transpose(1, 2)]))
    return Tensor(out)


def fused_feedforward(x, linear1_weight, linear2_weight, linear1_bias=None, linear2_bias=None,
                      ln1_scale=None, ln1_bias=None, ln2_scale=None, ln2_bias=None,
                      dropout1_rate=0.5, dropout2_rate=0.5, activation="relu", ln1_epsilon=1e-5,
                      ln2_epsilon=1e-5, pre_layer_norm=False, training=True,
                      mode='upscale_in_train', ring_id=-1, add_residual=True, name=None):
    t = _u(x)
    residual = t
    h = _ln(t, ln1_scale, ln1_bias, ln1_epsilon) if pre_layer_norm else t
    h = h @ _u(linear1_weight)
    if activation == 'gelu':
        h = K.bias_gelu(h, _t(linear1_bias), False)
    else:
        if linear1_bias is not None:
            h = h + _u(linear1_bias)
        h = torch.relu(h)
    h = _drop(h, dropout1_rate, training, mode)
    h = h @ _u(linear2_weight)
    if linear2_bias is not None:
        h = h + _u(linear2_bias)
    h = _drop(h, dropout2_rate, training, mode)
    if add_residual:
        h = residual + h
    if not pre_layer_norm:
        h = _ln(h, ln2_scale, ln2_bias, ln2_epsilon)
    return Tensor(h)


def fused_multi_transformer(x, ln_scales, ln_biases, qkv_weights, qkv_biases, linear_weights,
                            linear_biases, ffn_ln_scales, ffn_ln_biases, ffn1_weights, ffn1_biases,
                            ffn2_weights, ffn2_biases, pre_layer_norm=True, epsilon=1e-05,
                            cache_kvs=None, time_step=None, attn_mask=None, dropout_rate=0.0,
                            activation="gelu", training=False, mode='upscale_in_train',
                            trans_qkvw=True, ring_id=-1, name=None):
    h = x
    for i in range(len(qkv_weights)):
        h = fused_multi_head_attention(h, qkv_weights[i], linear_weights[i], pre_layer_norm,
                                       ln_scales[i], ln_biases[i], None, None, epsilon,
                                       qkv_biases[i] if qkv_biases else None,
                                       linear_biases[i] if linear_biases else None, None,
                                       attn_mask, dropout_rate, dropout_rate, epsilon, training,
                                       mode)
        h = fused_feedforward(h, ffn1_weights[i], ffn2_weights[i],
                              ffn1_biases[i] if ffn1_biases else None,
                              ffn2_biases[i] if ffn2_biases else None, ffn_ln_scales[i],
                              ffn_ln_biases[i], None, None, dropout_rate, dropout_rate,
                              activation, epsilon, epsilon, pre_layer_norm, training, mode)
    return h


def fused_ec_moe(x, gate, bmm0_weight, bmm0_bias, bmm1_weight, bmm1_bias, act_type):
    t = _u(x)
    g = torch.softmax(_u(gate).float(), -1).to(t.dtype)  # [B,S,E]
    h = torch.einsum('bsd,edf->bsef', t, _u(bmm0_weight)) + _u(bmm0_bias).squeeze(1)
    h = torch.nn.functional.gelu(h) if act_type == 'gelu' else torch.relu(h)
    o = torch.einsum('bsef,efd->bsed', h, _u(bmm1_weight)) + _u(bmm1_bias).squeeze(1)
    return Tensor((o * g.unsqueeze(-1)).sum(2))
