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
    g = torch.randn_like(ref)
    y.backward(g.bfloat16())
    ref.backward(g)
    for got, want, tol in ((x.grad, xf.grad, 0.08), (w.grad, wf.grad, 0.08), (s.grad, sf.grad, 0.05),
                           (b.grad, bf.grad, 0.05)):
        err = (got.float() - want).abs().max().item() / (want.abs().max().item() + 1e-6)
        assert err < tol, err


def test_stats_shift_handles_large_mean():
    """Running mean far from the batch mean and a large common offset: the shifted sums keep
    the variance (no E[y^2] - E[y]^2 cancellation)."""
    torch.manual_seed(1)
    x = (torch.randn(8, 8, 8, 64, device='cuda') * 0.05 + 3.0).bfloat16()
    w = (torch.randn(64, 64, 3, 3, device='cuda') * 0.05).bfloat16()
    w[:, :, 1, 1] += 0.2
    rm = torch.full((64,), 30.0, device='cuda')
    rv = torch.ones(64, device='cuda')
    y = K.conv_bn_act_nhwc(x, w, 1, 1, None, None, rm.clone(), rv.clone(), True, 0.9, 1e-5, None, False)
    c = TF.conv2d(x.float().permute(0, 3, 1, 2), w.float(), None, 1, 1)
    ref = TF.batch_norm(c, None, None, None, None, True, 0.1, 1e-5).permute(0, 2, 3, 1)
    assert (y.float() - ref).abs().max().item() < 0.08
