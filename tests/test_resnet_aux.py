"""ResNet auxiliaries. GradJoin (ops.fused): a residual block input's gradient summed from its consumers in place.
Host check of the join order cases: strided contributions arriving before any full-size buffer
are deferred and added into their sampled positions of the final one."""
import itertools

import pytest
import torch

from paddle_ray_amd.ops import fused as K


@pytest.mark.parametrize('order', list(itertools.permutations(['gemm', 'strided', 'tensor'])))
def test_grad_join_any_order(order):
    torch.manual_seed(0)
    n, h, w, c, co = 2, 4, 6, 8, 5
    xshape = (n, h, w, c)
    dy2 = torch.randn(n * h * w, co)
    w2 = torch.randn(co, c)
    dxs = torch.randn(n, h // 2, w // 2, c)
    g = torch.randn(xshape)
    want = (dy2 @ w2).view(xshape).clone()
    want[:, ::2, ::2, :] += dxs
    want += g
    j = K.GradJoin(torch.empty(xshape))
    j.n = 3
    outs = []
    for o in order:
        if o == 'gemm':
            outs.append(j.add_gemm(dy2, w2, xshape))
        elif o == 'strided':
            outs.append(j.add_strided(dxs, xshape, 2, 2))
        else:
            outs.append(j.add_tensor(g.clone(), owned=True))
    assert all(r is None for r in outs[:-1])
    torch.testing.assert_close(outs[-1], want, rtol=1e-5, atol=1e-5)


def test_grad_join_only_strided():
    xshape = (1, 4, 4, 3)
    a, b = torch.randn(1, 2, 2, 3), torch.randn(1, 2, 2, 3)
    j = K.GradJoin(torch.empty(xshape))
    j.n = 2
    assert j.add_strided(a, xshape, 2, 2) is None
    out = j.add_strided(b, xshape, 2, 2)
    want = torch.zeros(xshape)
    want[:, ::2, ::2, :] = a + b
    torch.testing.assert_close(out, want)


@pytest.mark.gpu
def test_global_avg_pool_nhwc_backward():
    """Global average pool (NHWC) forward + the broadcast-write backward kernel vs fp32 autograd."""
    import paddle_ray_amd.nn.functional as F
    from paddle_ray_amd.framework.core import _u
    torch.manual_seed(0)
    x = torch.randn(3, 7, 5, 24, device='cuda').bfloat16().requires_grad_()
    y = _u(F.adaptive_avg_pool2d(x, (1, 1), data_format='NHWC'))
    assert y.shape == (3, 1, 1, 24)
    g = torch.randn_like(y)
    y.backward(g)
    xf = x.detach().float().requires_grad_()
    yf = xf.mean((1, 2), keepdim=True)
    yf.backward(g.float())
    torch.testing.assert_close(y.float(), yf, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(x.grad.float(), xf.grad, atol=1e-3, rtol=1e-2)
