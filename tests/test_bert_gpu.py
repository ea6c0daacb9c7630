"""BERT encoder layer on the device: the fused path (packed-QKV flash attention with the key
padding mask, GEMM+bias+GELU epilogue MLP, add+dropout+LayerNorm kernels) against the unfused
torch composition of the same layer, forward and backward."""
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
    outs = []
    for fused in (True, False):
        layer.fused = fused
        xi = paddle.Tensor(x.clone().requires_grad_(True))
        y = layer(xi, paddle.Tensor(mask))
        y._t.backward(g)
        grads = [p.grad._t.float().clone() if hasattr(p.grad, '_t') else p.grad.float().clone()
                 for p in (layer.fc1.weight, layer.fc1.bias, layer.attn.qkv_proj.weight)]
        outs.append((y._t.float(), xi._t.grad.float(), grads))
        for p in layer.parameters():
            p.clear_gradient()
    (y1, dx1, g1), (y2, dx2, g2) = outs

    def rel(a, b):
        return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()
    assert rel(y1, y2) < 3e-2
    assert rel(dx1, dx2) < 5e-2
    for a, b in zip(g1, g2):
        assert rel(a, b) < 5e-2
