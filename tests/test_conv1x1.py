"""1x1 channels-last convolution through the in-tree split-K MFMA GEMMs (dgrad, wgrad) and
hipBLASLt (forward) against the fp32 PyTorch conv2d reference, values and gradients."""
import pytest
import torch

def _check(stride, n, h, cin, cout, dev):
    from paddle_ray_amd.ops import fused as K
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(n, h, h, cin, device=dev, dtype=torch.bfloat16, generator=g).requires_grad_()
    w = (torch.randn(cout, cin, 1, 1, device=dev, dtype=torch.bfloat16, generator=g) * cin ** -0.5
         ).requires_grad_()
    b = torch.randn(cout, device=dev, dtype=torch.bfloat16, generator=g).requires_grad_()
    y = K.conv1x1_nhwc(x, w, b, (stride, stride))
    dy = torch.randn_like(y)
    y.backward(dy)
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = torch.nn.functional.conv2d(xr.permute(0, 3, 1, 2), wr, br, stride).permute(0, 2, 3, 1)
    yr.backward(dy.float())

    def rel(a, r):
        return float((a.float() - r).abs().max() / r.abs().max().clamp_min(1e-6))
    assert rel(y, yr) < 2e-2
    assert rel(x.grad, xr.grad) < 2e-2
    assert rel(w.grad, wr.grad) < 2e-2
    assert rel(b.grad, br.grad) < 2e-2


@pytest.mark.gpu
@pytest.mark.parametrize('stride', [1, 2])
@pytest.mark.parametrize('n,h,cin,cout', [(8, 28, 256, 64), (4, 14, 512, 1024), (32, 56, 64, 256)])
def test_conv1x1_nhwc_matches_conv2d_gpu(stride, n, h, cin, cout):
    _check(stride, n, h, cin, cout, 'cuda')


@pytest.mark.parametrize('stride', [1, 2])
def test_conv1x1_nhwc_cpu(stride):
    _check(stride, 2, 8, 64, 128, 'cpu')
