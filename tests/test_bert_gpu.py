"""BERT encoder layer on the device: the fused path (packed-QKV flash attention with the key
padding mask, GEMM+bias+GELU epilogue MLP, add+dropout+LayerNorm kernels) against an fp32 copy of
the same layer on the unfused torch composition, forward and backward."""
import pytest
import torch

import paddle_ray_amd as paddle
from paddle_ray_amd.models.bert import BertLayer, bert_config


@pytest.mark.gpu
def test_bert_layer_fused_matches_unfused():
    paddle.set_device('gpu')
    paddle.seed(3)
    cfg = bert_config('bert-base-uncased', hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    paddle.set_default_dtype('bfloat16')
    layer = BertLayer(cfg)
    paddle.set_default_dtype('float32')
    B, S = 2, 256
    x = torch.randn(B, S, cfg.hidden_size, device='cuda', dtype=torch.bfloat16)
    mask = torch.zeros(B, 1, 1, S, device='cuda', dtype=torch.bfloat16)
    mask[1, ..., 200:] = -1e4
    g = torch.randn(B, S, cfg.hidden_size, device='cuda', dtype=torch.bfloat16)
    import copy
    ref = copy.deepcopy(layer)
    ref.to(dtype='float32')   # fp32 reference: the unfused torch composition in fp32
    ref.fused = False
    layer.fused = True
    xi = paddle.Tensor(x.clone().requires_grad_(True))
    y = layer(xi, paddle.Tensor(mask))
    y._t.backward(g)
    xr = paddle.Tensor(x.float().clone().requires_grad_(True))
    yr = ref(xr, paddle.Tensor(mask.float()))
    yr._t.backward(g.float())

    def grads(m):
        return [p.grad._t.float() if hasattr(p.grad, '_t') else p.grad.float()
                for p in (m.fc1.weight, m.fc1.bias, m.attn.qkv_proj.weight)]

    def rel(a, b):
        return ((a.float() - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()
    assert rel(y._t, yr._t) < 3e-2
    assert rel(xi._t.grad, xr._t.grad) < 5e-2
    for a, b in zip(grads(layer), grads(ref)):
        assert rel(a, b) < 5e-2
