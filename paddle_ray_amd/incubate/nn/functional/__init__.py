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
    """LayerNorm(residual + dropout(x + bias)) as ONE add_dropout_layer_norm kernel pass
    (upscale_in_train; the downscale_in_infer variant composes)."""
    t, r = _u(x), _u(residual)
    if mode != 'upscale_in_train':
        h = t if bias is None else t + _u(bias)
        return Tensor(_ln(r + _drop(h, dropout_rate, training, mode), ln_scale, ln_bias,
                          ln_epsilon))
    E = t.shape[-1]
    b = _u(bias) if bias is not None else torch.zeros(E, dtype=t.dtype, device=t.device)
    w = _u(ln_scale) if ln_scale is not None else torch.ones(E, dtype=t.dtype, device=t.device)
    lb = _u(ln_bias) if ln_bias is not None else torch.zeros(E, dtype=t.dtype, device=t.device)
    _, y = K.add_dropout_layer_norm(r, t, b, w, lb, dropout_rate, ln_epsilon, training)
    return Tensor(y)


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
    elif mode == 'upscale_in_train':
        # masked / dropout attention: fused SDPA (no [B, H, S, S] fp32 score tensor)
        am = None if attn_mask is None else _u(attn_mask).to(q.dtype)
        o = torch.nn.functional.scaled_dot_product_attention(
            q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), am,
            attn_dropout_rate if training else 0.0).transpose(1, 2)
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


def _rotary(x, cos, sin, dims):
    """Half-split rotation inside each of ``dims`` chunks of the head dim (reference
    RotrayKernel / mmha rotary): x [B, S, H, D], cos/sin [B, S, D]."""
    B, S, H, D = x.shape
    last = D // dims
    half = last // 2
    xv = x.float().view(B, S, H, dims, last)
    c = cos.float().view(B, S, 1, dims, last)
    sn = sin.float().view(B, S, 1, dims, last)
    left, right = xv[..., :half], xv[..., half:]
    out = torch.cat([left * c[..., :half] - right * sn[..., :half],
                     right * c[..., half:] + left * sn[..., half:]], -1)
    return out.view(B, S, H, D).to(x.dtype)


def _qkv(y, w, b, trans_qkvw):
    B, S, E = y.shape
    if trans_qkvw:                       # [3, H, D, E]
        _, H, D, _ = w.shape
        out = K.linear_nt(y.reshape(B * S, E), w.reshape(3 * H * D, E))
    else:                                # [E, 3, H, D]
        _, _, H, D = w.shape
        out = K.linear(y.reshape(B * S, E), w.reshape(E, 3 * H * D))
    if b is not None:
        out = out + b.reshape(-1).to(out.dtype)
    return out.view(B, S, 3, H, D)


def _ones_zeros(t, n, like):
    return t if t is not None else (torch.ones(n, dtype=like.dtype, device=like.device) if n
                                     else None)


def fused_multi_transformer(x, ln_scales, ln_biases, qkv_weights, qkv_biases, linear_weights,
                            linear_biases, ffn_ln_scales, ffn_ln_biases, ffn1_weights, ffn1_biases,
                            ffn2_weights, ffn2_biases, pre_layer_norm=True, epsilon=1e-05,
                            cache_kvs=None, pre_caches=None, seq_lens=None, rotary_embs=None,
                            time_step=None, attn_mask=None, dropout_rate=0.0, rotary_emb_dims=0,
                            activation="gelu", training=False, mode='upscale_in_train',
                            trans_qkvw=True, ring_id=-1, name=None):
    """N transformer layers for inference / generation (parity: reference
    incubate/nn/functional/fused_transformer.py:872 and fused_multi_transformer_op.cu.h).

    * context phase (``time_step`` None): QKV GEMM, optional rotary, attention over
      [pre_cache ; prompt] (flash kernel when unmasked, else masked SDPA), and with
      ``cache_kvs`` ([2, B, H, max_len, D] per layer) the prompt's K/V written in place.
    * decode phase (``time_step`` = t, x [B, 1, E]): the HIP decode-attention kernel streams
      cache positions [0, t) split-K across the chip and appends the token's K/V at t.
    * every residual add + dropout + following LayerNorm is ONE add_dropout_layer_norm
      kernel; FFN1 runs with its bias+activation in the GEMM epilogue.
    Returns ``out`` or ``(out, cache_kvs)`` when caches are given (updated in place)."""
    if mode not in ('downscale_in_infer', 'upscale_in_train'):
        raise ValueError("mode argument should be 'downscale_in_infer' or 'upscale_in_train'")
    h = _u(x)
    B, S, E = h.shape
    n = len(qkv_weights)
    p = dropout_rate if training else 0.0
    decode = time_step is not None
    if decode and not isinstance(time_step, int):
        ts = _u(time_step)
        # a device int32 step stays on the device (graph-capturable decode); host -> int
        t = ts.reshape(-1)[:1] if (ts.is_cuda and ts.dtype == torch.int32) else int(ts.reshape(-1)[0])
    else:
        t = int(time_step) if decode else None
    if decode and S != 1:
        raise ValueError("fused_multi_transformer: decode phase (time_step given) takes one token")
    rot = None
    if rotary_embs is not None and rotary_emb_dims:
        re = _u(rotary_embs)                          # [2, B, 1, S, D]
        rot = (re[0].reshape(B, S, -1), re[1].reshape(B, S, -1))
    mask = _t(attn_mask)
    sl = _t(seq_lens)
    zero_b = torch.zeros(E, dtype=h.dtype, device=h.device)
    one_w = torch.ones(E, dtype=h.dtype, device=h.device)

    def lnp(lst, i, default):
        return _u(lst[i]) if lst is not None and lst[i] is not None else default

    r = h
    y = K.layer_norm(h, lnp(ln_scales, 0, one_w), lnp(ln_biases, 0, zero_b), epsilon) \
        if pre_layer_norm else h
    for i in range(n):
        qkv = _qkv(y, _u(qkv_weights[i]), _t(qkv_biases[i]) if qkv_biases else None, trans_qkvw)
        H, D = qkv.shape[3], qkv.shape[4]
        if rot is not None:
            q = _rotary(qkv[:, :, 0], rot[0], rot[1], rotary_emb_dims)
            k = _rotary(qkv[:, :, 1], rot[0], rot[1], rotary_emb_dims)
            qkv = torch.stack([q, k, qkv[:, :, 2]], 2)
        cache = _u(cache_kvs[i]) if cache_kvs is not None else None
        if decode:
            if cache is None:
                raise ValueError("fused_multi_transformer: time_step needs cache_kvs")
            o = K.mmha_decode(qkv[:, 0].contiguous(), cache, t, mask).reshape(B, 1, H * D)
        else:
            q, k, v = qkv.unbind(2)                  # [B, S, H, D]
            P = 0
            if pre_caches is not None and pre_caches[i] is not None:
                pc = _u(pre_caches[i])               # [2, B, H, P, D]
                P = pc.shape[3]
                k = torch.cat([pc[0].transpose(1, 2).to(k.dtype), k], 1)
                v = torch.cat([pc[1].transpose(1, 2).to(v.dtype), v], 1)
            if cache is not None:
                cache[0, :, :, :P + S] = k.transpose(1, 2)
                cache[1, :, :, :P + S] = v.transpose(1, 2)
            if mask is None and sl is None and h.is_cuda and h.dtype in (torch.bfloat16,
                                                                         torch.float16):
                o = K.flash_attention(q.contiguous(), k.contiguous(), v.contiguous(), causal=False)
            else:
                am = None if mask is None else mask.to(torch.float32)
                if sl is not None:
                    pad = torch.arange(P + S, device=h.device)[None, :] >= \
                        (sl.reshape(-1, 1).to(h.device) + P)
                    pm = torch.zeros(B, 1, 1, P + S, device=h.device).masked_fill(
                        pad[:, None, None, :], float('-inf'))
                    am = pm if am is None else am + pm
                o = torch.nn.functional.scaled_dot_product_attention(
                    q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                    None if am is None else am.to(q.dtype), p)
                o = o.transpose(1, 2)
            o = o.reshape(B, S, H * D)
        a = K.linear(o, _u(linear_weights[i]))
        lb = _t(linear_biases[i]) if linear_biases else None
        lb = zero_b if lb is None else lb
        if pre_layer_norm:
            r, y = K.add_dropout_layer_norm(r, a, lb, lnp(ffn_ln_scales, i, one_w),
                                            lnp(ffn_ln_biases, i, zero_b), p, epsilon, training)
        else:
            _, r = K.add_dropout_layer_norm(r, a, lb, lnp(ln_scales, i, one_w),
                                            lnp(ln_biases, i, zero_b), p, epsilon, training)
            y = r
        b1 = _t(ffn1_biases[i]) if ffn1_biases else None
        w1 = _u(ffn1_weights[i])
        if decode and y.is_cuda:
            # skinny decode rows: hipBLASLt + the activation (3.0 vs 3.6 ms per 24-layer graph
            # decode step at batch 8); the 256-row MFMA tile would idle
            f = y.reshape(-1, E) @ w1 if b1 is None else torch.addmm(b1, y.reshape(-1, E), w1)
            f = (torch.nn.functional.gelu(f) if activation == 'gelu' else torch.relu(f)
                 ).view(B, S, -1)
        else:
            f = K.gemm_bias_act(y, w1, b1, 'gelu' if activation == 'gelu' else activation)
        if p:
            f = torch.nn.functional.dropout(f, p, True)
        f = K.linear(f, _u(ffn2_weights[i]))
        b2 = _t(ffn2_biases[i]) if ffn2_biases else None
        b2 = zero_b if b2 is None else b2
        if pre_layer_norm:
            if i + 1 < n:
                r, y = K.add_dropout_layer_norm(r, f, b2, lnp(ln_scales, i + 1, one_w),
                                                lnp(ln_biases, i + 1, zero_b), p, epsilon,
                                                training)
            else:
                r = r + _drop(f + b2, p, training, mode)
        else:
            _, r = K.add_dropout_layer_norm(r, f, b2, lnp(ffn_ln_scales, i, one_w),
                                            lnp(ffn_ln_biases, i, zero_b), p, epsilon, training)
            y = r
    out = Tensor(r)
    if cache_kvs is not None:
        return out, cache_kvs
    return out


def fused_ec_moe(x, gate, bmm0_weight, bmm0_bias, bmm1_weight, bmm1_bias, act_type):
    t = _u(x)
    g = torch.softmax(_u(gate).float(), -1).to(t.dtype)  # [B,S,E]
    h = torch.einsum('bsd,edf->bsef', t, _u(bmm0_weight)) + _u(bmm0_bias).squeeze(1)
    h = torch.nn.functional.gelu(h) if act_type == 'gelu' else torch.relu(h)
    o = torch.einsum('bsef,efd->bsed', h, _u(bmm1_weight)) + _u(bmm1_bias).squeeze(1)
    return Tensor((o * g.unsqueeze(-1)).sum(2))
