"""Convolution + BatchNorm with the statistics taken in the implicit-GEMM epilogue
(ops.fused.conv_bn_act_nhwc; parity: fluid/operators/fused/cudnn_norm_conv.cu.h,
resnet_unit_op.cu) against an fp32 PyTorch reference of conv2d + batch_norm (+ add) + relu:
outputs, running statistics and gradients, for every tile configuration (Cout 64 / 128 / 256)."""
import pytest
import torch
import torch.nn.functional as TF

from paddle_ray_amd.ops import fused as K

pytestmark = pytest.mark.gpu


def _ref(x, w, s, b, rm, rv, stride, pad, z, relu, mom, eps):
    c = TF.conv2d(x.permute(0, 3, 1, 2), w, None, stride, pad)
    y = TF.batch_norm(c, rm, rv, s, b, True, 1 - mom, eps)
    if z is not None:
        y = y + z.permute(0, 3, 1, 2)
    if relu:
        y = torch.relu(y)
    return y.permute(0, 2, 3, 1)


@pytest.mark.parametrize('cin,cout,hw,stride,k', [(64, 64, 16, 1, 3), (128, 128, 14, 2, 3),
                                                  (64, 256, 9, 1, 3), (256, 512, 7, 1, 3)])
@pytest.mark.parametrize('res', [False, True])
def test_conv_bn_stats_matches_reference(cin, cout, hw, stride, k, res):
    torch.manual_seed(0)
    dev = 'cuda'
    pad = k // 2
    x = (torch.randn(4, hw, hw, cin, device=dev) + 0.5).bfloat16().requires_grad_()
    w = (torch.randn(cout, cin, k, k, device=dev) * (2.0 / (k * k * cin)) ** 0.5).bfloat16().requires_grad_()
    s = (torch.rand(cout, device=dev) + 0.5).requires_grad_()
    b = (torch.randn(cout, device=dev) * 0.1).requires_grad_()
    rm = torch.randn(cout, device=dev) * 0.1
    rv = torch.rand(cout, device=dev) + 0.5
    ho = (hw + 2 * pad - k) // stride + 1
    z = torch.randn(4, ho, ho, cout, device=dev).bfloat16() if res else None
    assert K.conv_bn_stats_ok(x, w, stride, pad, rm, True)
    rm1, rv1 = rm.clone(), rv.clone()
    y = K.conv_bn_act_nhwc(x, w, stride, pad, s, b, rm1, rv1, True, 0.9, 1e-5, z, True)
    xf, wf = x.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    sf, bf = s.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    rm2, rv2 = rm.clone(), rv.clone()
    ref = _ref(xf, wf, sf, bf, rm2, rv2, stride, pad, z.float() if res else None, True, 0.9, 1e-5)
    torch.cuda.synchronize()
    assert (y.float() - ref).abs().max().item() < 0.06
    torch.testing.assert_close(rm1, rm2, rtol=1e-2, atol=2e-3)
    torch.testing.assert_close(rv1, rv2, rtol=2e-2, atol=2e-3)
    # gradients: the fusion changes only how the forward statistics are taken, so they must
    # match the unfused in-tree path (conv_kxk_nhwc + batch_norm_act) on the same bf16 data
    g = torch.randn_like(ref).bfloat16()
    y.backward(g)
    x2, w2 = x.detach().clone().requires_grad_(), w.detach().clone().requires_grad_()
    s2, b2 = s.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    y2 = K.batch_norm_act(K.conv_kxk_nhwc(x2, w2, None, stride, pad), z, s2, b2, rm.clone(), rv.clone(),
                          True, 0.9, 1e-5, True)
    y2.backward(g)
    assert (y.float() - y2.float()).abs().max().item() < 0.04
    for got, want in ((x.grad, x2.grad), (w.grad, w2.grad), (s.grad, s2.grad), (b.grad, b2.grad)):
        err = (got.float() - want.float()).abs().max().item() / (want.float().abs().max().item() + 1e-6)
        assert err < 0.03, err
    # and loosely against fp32 autograd (bf16 rounding of y, dy and the conv operands)
    ref.backward(g.float())
    for got, want in ((s.grad, sf.grad), (b.grad, bf.grad)):
        err = (got.float() - want).abs().max().item() / (want.abs().max().item() + 1e-6)
        assert err < 0.1, err


def test_stats_shift_large_offset_matches_unfused():
    """A large common offset (conv outputs ~ 38 +- 1) and a running mean far from the batch
    mean: the epilogue's shifted sums give the same normalisation as the unfused statistics
    pass over the same bf16 conv output."""
    torch.manual_seed(1)
    x = (torch.randn(8, 8, 8, 64, device='cuda') * 0.05 + 3.0).bfloat16()
    w = (torch.randn(64, 64, 3, 3, device='cuda') * 0.05).bfloat16()
    w[:, :, 1, 1] += 0.2
    rm = torch.full((64,), 30.0, device='cuda')
    rv = torch.ones(64, device='cuda')
    rm1, rv1, rm2, rv2 = rm.clone(), rv.clone(), rm.clone(), rv.clone()
    y = K.conv_bn_act_nhwc(x, w, 1, 1, None, None, rm1, rv1, True, 0.9, 1e-5, None, False)
    y2 = K.batch_norm_act(K.conv_kxk_nhwc(x, w, None, 1, 1), None, None, None, rm2, rv2, True, 0.9,
                          1e-5, False)
    assert (y.float() - y2.float()).abs().max().item() < 0.04
    torch.testing.assert_close(rm1, rm2, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(rv1, rv2, rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize('cin,cout,hw,stride', [(64, 256, 14, 1), (256, 64, 14, 1), (128, 512, 14, 2),
                                                (512, 128, 9, 1)])
@pytest.mark.parametrize('res', [False, True])
def test_conv1x1_bn_stats_matches_reference(cin, cout, hw, stride, res):
    """1x1 convolutions (ResNet bottleneck conv1 / conv3 / strided downsample) with the BN
    statistics from the implicit-GEMM epilogue: outputs, running stats and gradients against
    fp32 conv2d + batch_norm and against the unfused in-tree path (conv1x1_nhwc + batch_norm_act)."""
    torch.manual_seed(2)
    dev = 'cuda'
    x = (torch.randn(4, hw, hw, cin, device=dev) + 0.3).bfloat16().requires_grad_()
    w = (torch.randn(cout, cin, 1, 1, device=dev) * (2.0 / cin) ** 0.5).bfloat16().requires_grad_()
    s = (torch.rand(cout, device=dev) + 0.5).requires_grad_()
    b = (torch.randn(cout, device=dev) * 0.1).requires_grad_()
    rm = torch.randn(cout, device=dev) * 0.1
    rv = torch.rand(cout, device=dev) + 0.5
    ho = (hw - 1) // stride + 1
    z = torch.randn(4, ho, ho, cout, device=dev).bfloat16() if res else None
    assert K.conv1x1_bn_stats_ok(x, w, stride, 0, rm, True)
    rm1, rv1 = rm.clone(), rv.clone()
    y = K.conv_bn_act_nhwc(x, w, stride, 0, s, b, rm1, rv1, True, 0.9, 1e-5, z, True)
    xf, wf = x.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    sf, bf = s.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    rm2, rv2 = rm.clone(), rv.clone()
    ref = _ref(xf, wf, sf, bf, rm2, rv2, stride, 0, z.float() if res else None, True, 0.9, 1e-5)
    torch.cuda.synchronize()
    assert (y.float() - ref).abs().max().item() < 0.06
    torch.testing.assert_close(rm1, rm2, rtol=1e-2, atol=2e-3)
    torch.testing.assert_close(rv1, rv2, rtol=2e-2, atol=2e-3)
    g = torch.randn_like(ref).bfloat16()
    y.backward(g)
    x2, w2 = x.detach().clone().requires_grad_(), w.detach().clone().requires_grad_()
    s2, b2 = s.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    y2 = K.batch_norm_act(K.conv1x1_nhwc(x2, w2, None, (stride, stride)), z, s2, b2, rm.clone(), rv.clone(),
                          True, 0.9, 1e-5, True)
    y2.backward(g)
    assert (y.float() - y2.float()).abs().max().item() < 0.04
    for got, want in ((x.grad, x2.grad), (w.grad, w2.grad), (s.grad, s2.grad), (b.grad, b2.grad)):
        err = (got.float() - want.float()).abs().max().item() / (want.float().abs().max().item() + 1e-6)
        assert err < 0.03, err
