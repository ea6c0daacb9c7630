"""Channels-last max pool HIP kernels (ops/csrc/pool.hip) against PyTorch fp32 max_pool2d."""
import pytest
import torch

from paddle_ray_amd.ops import fused as K


@pytest.mark.gpu
@pytest.mark.parametrize("shape,k,s,p", [((2, 17, 15, 64), 3, 2, 1), ((3, 8, 8, 16), 2, 2, 0),
                                         ((1, 9, 10, 24), 3, 1, 1), ((2, 12, 12, 8), 5, 3, 2)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_max_pool_nhwc(shape, k, s, p, dtype):
    torch.manual_seed(0)
    x = torch.randn(*shape, device='cuda').to(dtype)
    xh = x.clone().requires_grad_()
    y = K.max_pool2d_nhwc(xh, (k, k), (s, s), (p, p))
    xr = x.float().permute(0, 3, 1, 2).requires_grad_()
    yr = torch.nn.functional.max_pool2d(xr, k, s, p)
    torch.testing.assert_close(y.float(), yr.permute(0, 2, 3, 1), rtol=0, atol=0)
    dy = torch.randn_like(yr)
    yr.backward(dy)
    y.backward(dy.permute(0, 2, 3, 1).to(dtype))
    tol = 0 if dtype == torch.float32 else 3e-2
    torch.testing.assert_close(xh.grad.float(), xr.grad.permute(0, 2, 3, 1), rtol=tol, atol=tol)
