"""Implicit-GEMM KxK convolution (ops/fused.py ConvKxKFn over gemm_lds.hip ConvDmaA) against
a plain PyTorch fp32 conv2d of the same op."""
import pytest
import torch

from paddle_ray_amd.ops import fused as K

CASES = [
    # n, h, w, cin, cout, k, stride, pad
    (2, 14, 14, 64, 64, 3, 1, 1),
    (2, 15, 13, 64, 128, 3, 2, 1),
    (3, 9, 11, 128, 96, 3, 1, 1),
    (1, 12, 12, 64, 64, 5, 1, 2),
    (2, 10, 10, 128, 64, 3, 1, 0),
    (4, 7, 7, 512, 512, 3, 1, 1),
]


def test_conv_kxk_supported_cpu():
    x = torch.zeros(1, 8, 8, 64, dtype=torch.bfloat16)
    w = torch.zeros(64, 64, 3, 3, dtype=torch.bfloat16)
    assert not K.conv_kxk_supported(x, w, 1, 1)  # host tensors never reach the kernel


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_conv_kxk_fwd_bwd(case, dtype):
    n, h, w_, cin, cout, k, s, p = case
    torch.manual_seed(0)
    x = torch.randn(n, h, w_, cin, device='cuda', dtype=dtype)
    w = (torch.randn(cout, cin, k, k, device='cuda') / (cin * k * k) ** 0.5).to(dtype)
    b = torch.randn(cout, device='cuda', dtype=dtype)
    assert K.conv_kxk_supported(x, w, s, p)
    xr, wr, br = (t.float().requires_grad_() for t in (x, w, b))
    xh, wh, bh = (t.clone().requires_grad_() for t in (x, w, b))
    y = K.conv_kxk_nhwc(xh, wh, bh, s, p)
    yr = torch.nn.functional.conv2d(xr.permute(0, 3, 1, 2), wr, br, s, p).permute(0, 2, 3, 1)
    assert y.shape == yr.shape
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=3e-2)
    dy = torch.randn_like(yr)
    yr.backward(dy)
    y.backward(dy.to(dtype))
    for got, ref in ((xh.grad, xr.grad), (wh.grad, wr.grad), (bh.grad, br.grad)):
        err = (got.float() - ref).abs().max().item()
        scale = ref.abs().max().item() + 1e-6
        assert err <= 2e-2 * scale + 2e-2, (err, scale)
    # second pass: the weight gradient is accumulated in place into the existing w.grad
    K.conv_kxk_nhwc(xh, wh, bh, s, p).backward(dy.to(dtype))
    err = (wh.grad.float() - 2 * wr.grad).abs().max().item()
    assert err <= 4e-2 * wr.grad.abs().max().item() + 4e-2, err


@pytest.mark.gpu
def test_flip_t_filter():
    torch.manual_seed(0)
    w = torch.randn(96, 64, 3, 3, device='cuda', dtype=torch.bfloat16)
    ref = w.flip(2, 3).permute(1, 2, 3, 0).reshape(64, 9 * 96)
    assert torch.equal(K._flip_t(w), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("case", [(2, 8, 8, 64, 64, 3, 1, 1), (4, 16, 16, 64, 128, 3, 2, 1),
                                  (2, 16, 16, 128, 256, 3, 1, 1), (16, 4, 4, 256, 64, 3, 1, 0),
                                  (1, 16, 8, 64, 72, 5, 1, 2),
                                  # narrow 128-row tiles with split-K over the pixels
                                  (8, 32, 32, 64, 64, 3, 1, 1), (8, 32, 32, 128, 128, 3, 1, 1),
                                  (4, 16, 16, 128, 96, 3, 2, 1)])
def test_conv_wgrad_lds(case):
    n, h, w_, cin, cout, k, s, p = case
    torch.manual_seed(0)
    x = torch.randn(n, h, w_, cin, device='cuda', dtype=torch.bfloat16)
    ho, wo = (h + 2 * p - k) // s + 1, (w_ + 2 * p - k) // s + 1
    dy = torch.randn(n, ho, wo, cout, device='cuda', dtype=torch.bfloat16)
    if (n * ho * wo) % 64:
        pytest.skip("pixel count not a multiple of 64 (MIOpen path)")
    got = K._conv_wgrad_lds(dy, x, k, k, s, p).permute(0, 3, 1, 2).float()
    wr = torch.zeros(cout, cin, k, k, device='cuda', requires_grad=True)
    torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), wr, None, s, p).backward(
        dy.float().permute(0, 3, 1, 2))
    err = (got - wr.grad).abs().max().item()
    assert err <= 1e-2 * wr.grad.abs().max().item() + 1e-2, err


STEM_CASES = [
    # n, h, w, cin, cout, k, pad
    (2, 224, 224, 3, 64, 7, 3),     # ResNet stem
    (3, 30, 26, 3, 64, 7, 3),
    (2, 20, 18, 4, 32, 7, 3),
    (1, 18, 14, 3, 16, 7, 3),       # 63 output pixels: weight gradient falls back
]


def test_stem_supported_cpu():
    x = torch.zeros(1, 224, 224, 3, dtype=torch.bfloat16)
    w = torch.zeros(64, 3, 7, 7, dtype=torch.bfloat16)
    assert not K.stem_conv_supported(x, w, 2, 3)   # host tensors never reach the kernel
    idx = K._stem_index(w)                         # every filter tap appears exactly once
    v = idx[idx >= 0]
    assert v.numel() == w.numel() and v.unique().numel() == w.numel()


@pytest.mark.gpu
@pytest.mark.parametrize("case", STEM_CASES)
def test_stem_conv_s2d(case):
    """Stride-2 narrow-input conv through space-to-depth + the pixel-pitch implicit GEMM: forward,
    BN partial statistics and the weight gradient vs fp32 PyTorch."""
    n, h, w_, cin, cout, k, p = case
    torch.manual_seed(1)
    x = torch.randn(n, h, w_, cin, device='cuda', dtype=torch.bfloat16)
    w = (torch.randn(cout, cin, k, k, device='cuda') / (cin * k * k) ** 0.5).to(torch.bfloat16)
    assert K.stem_conv_supported(x, w, 2, p)
    shift = torch.randn(cout, device='cuda') * 0.1
    wh = w.clone().requires_grad_()
    y, part = K.StemConvFn.apply(x, wh, p, shift)
    wr = w.float().requires_grad_()
    yr = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), wr, None, 2, p).permute(0, 2, 3, 1)
    assert y.shape == yr.shape
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=3e-2)
    d = y.float().reshape(-1, cout) - shift
    torch.testing.assert_close(part[0].sum(0), d.sum(0), atol=0.5, rtol=1e-2)
    torch.testing.assert_close(part[1].sum(0), (d * d).sum(0), atol=0.5, rtol=1e-2)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g.float())
    torch.testing.assert_close(wh.grad.float(), wr.grad, atol=5e-2 * wr.grad.abs().max().item(), rtol=3e-2)


def test_strided_dgrad_phase_index_cpu():
    """The four stride-2 phase sub-filters use the 9 taps 1 + 2 + 2 + 4 times in total, and each
    phase's taps are the ones with (phase + 1 - k) even."""
    w = torch.zeros(64, 8, 3, 3)
    idx, table = K._s2_phase_index(w)
    assert [t[2] * t[3] for t in table] == [1, 2, 2, 4]
    assert idx.numel() == 9 * 64 * 8
    assert idx.unique().numel() == 9 * 64 * 8        # every (co, ci, ky, kx) exactly once


S2_CASES = [(2, 8, 8, 64, 64), (2, 14, 10, 128, 128), (1, 6, 6, 256, 256), (3, 12, 12, 64, 128)]


@pytest.mark.gpu
@pytest.mark.parametrize("case", S2_CASES)
def test_strided_dgrad_phases(case, monkeypatch):
    """3x3 / stride 2 / pad 1 input gradient through the four sub-pixel phase convs vs fp32."""
    monkeypatch.setattr(K, '_STRIDED_DGRAD', True)
    n, h, w_, cin, cout = case
    torch.manual_seed(2)
    x = torch.randn(n, h, w_, cin, device='cuda', dtype=torch.bfloat16)
    w = (torch.randn(cout, cin, 3, 3, device='cuda') / (9 * cin) ** 0.5).to(torch.bfloat16)
    ho, wo = h // 2, w_ // 2
    dy = torch.randn(n, ho, wo, cout, device='cuda', dtype=torch.bfloat16)
    assert K.strided_dgrad_ok(x, dy, w, 2, 1)
    got = K._conv_dgrad_s2(dy, w, x.shape)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_()
    torch.nn.functional.conv2d(xr, w.float(), None, 2, 1).backward(dy.float().permute(0, 3, 1, 2))
    want = xr.grad.permute(0, 2, 3, 1)
    err = (got.float() - want).abs().max().item()
    assert err <= 2e-2 * want.abs().max().item() + 1e-2, err
