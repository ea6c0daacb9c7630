"""fused_multi_transformer: context phase against a plain composition of the reference's
pseudo code (incubate/nn/functional/fused_transformer.py:910-940), and generation — a
prompt through the context phase with KV caches, then token-by-token decode steps with
``time_step`` — against the context phase over the whole sequence with a causal mask.
GPU: the HIP decode-attention kernel against the fp32 reference, including the split-K
path over long caches, masks, and every supported head dim."""
import math

import numpy as np
import pytest
import torch

import paddle_ray_amd as paddle
from paddle_ray_amd.incubate.nn import FusedMultiTransformer
from paddle_ray_amd.incubate.nn import functional as IF


def _plain(x, m, mask, pre_ln):
    """Reference pseudo code, layer by layer, fp32 torch."""
    E, H = m.embed_dim, m.num_heads
    D = E // H
    ln = lambda t, w, b: torch.nn.functional.layer_norm(t, (E,), w, b, m._epsilon)  # noqa
    h = x
    for i in range(len(m.qkv_weights)):
        P = lambda n: getattr(m, n)[i]._t.detach().float()  # noqa
        res = h
        y = ln(h, P('ln_scales'), P('ln_biases')) if pre_ln else h
        qkv = torch.einsum('bse,thde->bsthd', y, P('qkv_weights')) + P('qkv_biases')
        q, k, v = qkv.unbind(2)
        s = torch.einsum('bqhd,bkhd->bhqk', q, k) / math.sqrt(D)
        if mask is not None:
            s = s + mask
        o = torch.einsum('bhqk,bkhd->bqhd', torch.softmax(s, -1), v).reshape(*x.shape[:2], E)
        o = o @ P('linear_weights') + P('linear_biases')
        h = res + o if pre_ln else ln(res + o, P('ln_scales'), P('ln_biases'))
        res = h
        y = ln(h, P('ffn_ln_scales'), P('ffn_ln_biases')) if pre_ln else h
        f = torch.nn.functional.gelu(y @ P('ffn1_weights') + P('ffn1_biases'))
        f = f @ P('ffn2_weights') + P('ffn2_biases')
        h = res + f if pre_ln else ln(res + f, P('ffn_ln_scales'), P('ffn_ln_biases'))
    return h


def _model(pre_ln, E=32, H=4, F=64, L=2, seed=0):
    paddle.seed(seed)
    m = FusedMultiTransformer(E, H, F, normalize_before=pre_ln, num_layers=L)
    rs = np.random.RandomState(seed)
    for p in m.parameters():  # non-trivial LN params and biases
        p.set_value((rs.randn(*p.shape) * (0.3 if len(p.shape) > 1 else 0.2)).astype('float32')
                    + (1.0 if 'scale' in p.name else 0.0))
    m.eval()
    return m


def _causal(S, B):
    return torch.triu(torch.full((S, S), float('-inf')), 1).expand(B, 1, S, S)


@pytest.mark.parametrize('pre_ln', [True, False])
def test_context_phase_matches_pseudo_code(pre_ln):
    m = _model(pre_ln)
    x = torch.randn(2, 7, 32)
    mask = _causal(7, 2)
    got = m(paddle.Tensor(x), attn_mask=paddle.Tensor(mask))
    np.testing.assert_allclose(got.numpy(), _plain(x, m, mask, pre_ln).numpy(), rtol=2e-4,
                               atol=2e-4)
    got = m(paddle.Tensor(x))  # unmasked
    np.testing.assert_allclose(got.numpy(), _plain(x, m, None, pre_ln).numpy(), rtol=2e-4,
                               atol=2e-4)


def _close(a, b, tol):
    """max error relative to the tensor's scale (bf16 rounds ~2^-8 of each value's magnitude;
    element-wise rtol is meaningless for entries near zero)."""
    a, b = a.float(), b.float()
    err = float((a - b).abs().max()) / max(float(b.abs().max()), 1e-6)
    assert err < tol, err


def _generate_vs_full(m, B, S0, steps, device='cpu', dtype=torch.float32, tol=2e-5):
    E, H = m.embed_dim, m.num_heads
    D = E // H
    L = len(m.qkv_weights)
    x = torch.randn(B, S0 + steps, E).to(device=device, dtype=dtype)
    full = m(paddle.Tensor(x), attn_mask=paddle.Tensor(_causal(S0 + steps, B).to(device, dtype)))._t
    caches = [paddle.Tensor(torch.zeros(2, B, H, S0 + steps + 3, D, device=device, dtype=dtype))
              for _ in range(L)]
    out, caches = m(paddle.Tensor(x[:, :S0]), attn_mask=paddle.Tensor(_causal(S0, B).to(device, dtype)),
                    caches=caches)
    _close(out._t, full[:, :S0], tol)
    for t in range(S0, S0 + steps):
        mask = torch.zeros(B, 1, 1, t + 1, device=device)
        out, caches = m(paddle.Tensor(x[:, t:t + 1]), attn_mask=paddle.Tensor(mask), caches=caches,
                        time_step=paddle.to_tensor(np.array([t], 'int32')))
        _close(out._t[:, 0], full[:, t], tol)
    return caches


@pytest.mark.parametrize('pre_ln', [True, False])
def test_generation_with_cache_matches_full_causal(pre_ln):
    m = _model(pre_ln)
    caches = _generate_vs_full(m, 2, 5, 4)
    assert float(caches[0]._t[:, :, :, 9:].abs().sum()) == 0.0  # untouched tail


def test_decode_padding_mask_and_rotary():
    m = _model(True)
    B, S, E, H = 2, 6, 32, 4
    D = E // H
    x = torch.randn(B, S, E)
    pos = torch.arange(S, dtype=torch.float32)
    inv = 1.0 / (10000 ** (torch.arange(0, D // 2, dtype=torch.float32) / (D // 2)))
    ang = pos[:, None] * inv[None, :]
    cos = torch.cat([ang.cos(), ang.cos()], -1).expand(B, S, D)
    sin = torch.cat([ang.sin(), ang.sin()], -1).expand(B, S, D)
    rot = torch.stack([cos, sin])[:, :, None]                 # [2, B, 1, S, D]
    full = m(paddle.Tensor(x), attn_mask=paddle.Tensor(_causal(S, B)),
             rotary_embs=paddle.Tensor(rot), rotary_emb_dims=1)._t
    caches = [paddle.Tensor(torch.zeros(2, B, H, S, D)) for _ in range(2)]
    m(paddle.Tensor(x[:, :S - 1]), attn_mask=paddle.Tensor(_causal(S - 1, B)), caches=caches,
      rotary_embs=paddle.Tensor(rot[:, :, :, :S - 1].contiguous()), rotary_emb_dims=1)
    # decode the last token with the padding mask hiding position 0 for batch 1
    mask = torch.zeros(B, 1, 1, S)
    out, _ = m(paddle.Tensor(x[:, S - 1:]), attn_mask=paddle.Tensor(mask), caches=caches,
               rotary_embs=paddle.Tensor(rot[:, :, :, S - 1:].contiguous()), rotary_emb_dims=1,
               time_step=S - 1)
    torch.testing.assert_close(out._t[:, 0], full[:, S - 1], rtol=2e-4, atol=2e-4)
    mask[1, ..., 0] = float('-inf')
    out2, _ = m(paddle.Tensor(x[:, S - 1:]), attn_mask=paddle.Tensor(mask), caches=caches,
                rotary_embs=paddle.Tensor(rot[:, :, :, S - 1:].contiguous()), rotary_emb_dims=1,
                time_step=S - 1)
    torch.testing.assert_close(out2._t[0], out._t[0])
    assert not torch.allclose(out2._t[1], out._t[1])


def test_fused_bias_dropout_residual_layer_norm_uses_adl():
    x, r = torch.randn(3, 5, 16), torch.randn(3, 5, 16)
    b, w, lb = torch.randn(16), torch.rand(16) + 0.5, torch.randn(16)
    got = IF.fused_bias_dropout_residual_layer_norm(
        paddle.Tensor(x), paddle.Tensor(r), paddle.Tensor(b), paddle.Tensor(w), paddle.Tensor(lb),
        dropout_rate=0.0)
    ref = torch.nn.functional.layer_norm(r + x + b, (16,), w, lb, 1e-5)
    torch.testing.assert_close(got._t, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize('D', [64, 128, 256])
@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float32])
def test_mmha_decode_hip_kernel_gpu(D, dtype):
    from paddle_ray_amd.ops import fused as K
    from paddle_ray_amd.ops import registry as R
    g = torch.Generator().manual_seed(D)
    for B, H, L, t, use_mask in ((1, 8, 4100, 4095, True), (3, 4, 64, 0, False),
                                 (2, 16, 700, 513, True), (4, 2, 40, 37, False)):
        qkv = torch.randn(B, 3, H, D, generator=g).to(dtype).cuda()
        cache = torch.randn(2, B, H, L, D, generator=g).to(dtype).cuda()
        mask = None
        if use_mask:
            mask = torch.zeros(B, t + 1 + 3)
            mask[:, ::7] = float('-inf')
            mask[:, t] = 0.0
            mask = mask.cuda()
        c_ref = cache.clone()
        ref = R.get_kernel('mmha_decode', 'ref')(qkv, c_ref, t, mask)
        out = K.mmha_decode(qkv, cache, t, mask)
        tol = 2e-2 if dtype == torch.bfloat16 else 2e-5
        torch.testing.assert_close(out.float(), ref.float(), rtol=tol, atol=tol)
        torch.testing.assert_close(cache, c_ref)  # the token's K/V appended at t, nothing else
    assert K._native.lib() is not None


@pytest.mark.gpu
def test_generation_on_gpu_bf16():
    paddle.set_device('gpu')
    m = _model(True, E=256, H=2, F=512, L=2)       # head_dim 128
    m.to(dtype='bfloat16')
    _generate_vs_full(m, 2, 9, 6, device='cuda', dtype=torch.bfloat16, tol=2e-2)


def _decoder_vs_full(dev, dtype, tol, E=32, H=4, L=2):
    from paddle_ray_amd.incubate.nn import FusedMultiTransformerDecoder
    m = _model(True, E=E, H=H, F=2 * E, L=L)
    if dtype != torch.float32:
        m.to(dtype='bfloat16')
    B, S0, steps = 2, 5, 4
    x = torch.randn(B, S0 + steps, E).to(device=dev, dtype=dtype)
    full = m(paddle.Tensor(x), attn_mask=paddle.Tensor(_causal(S0 + steps, B).to(dev, dtype)))._t
    dec = FusedMultiTransformerDecoder(m, B, 16)
    out = dec.prefill(paddle.Tensor(x[:, :S0]))
    _close(out._t, full[:, :S0], tol)
    for t in range(S0, S0 + steps):
        o = dec.step(paddle.Tensor(x[:, t:t + 1]))
        _close(o._t[:, 0], full[:, t], tol)
    assert int(dec.t.item()) == S0 + steps
    return dec


def test_decoder_runner_cpu():
    dec = _decoder_vs_full('cpu', torch.float32, 2e-5)
    assert dec._graph is None


@pytest.mark.gpu
def test_decoder_runner_hip_graph_gpu():
    paddle.set_device('gpu')
    dec = _decoder_vs_full('cuda', torch.bfloat16, 2e-2, E=256, H=2)
    assert dec._graph is not None   # steps after the first replayed the captured graph
