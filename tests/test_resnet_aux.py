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


def test_wgrad_pair_defers_and_hooks_fire_after_cpu():
    """WgradPair on the host (no grouped kernel there): the output projection's weight gradient
    is deferred to the QKV Linear's backward, and its post-accumulate hook fires only after the
    deferred accumulation (the QKV Linear holds that weight as a dependency)."""
    torch.manual_seed(0)
    h, t = 16, 12
    x = torch.randn(t, h, requires_grad=True)
    wq = (torch.randn(h, 3 * h) * 0.1).requires_grad_()
    wo = (torch.randn(h, h) * 0.1).requires_grad_()
    for p in (wq, wo):
        p.grad = torch.zeros_like(p)
    seen = []
    wo.register_post_accumulate_grad_hook(lambda p: seen.append(p.grad.clone()))
    pair = K.WgradPair()
    qkv = K.linear(x, wq, None, pair=pair, w_dep=wo)
    a = qkv[:, :h] * qkv[:, h:2 * h] + qkv[:, 2 * h:]
    y = K.linear(a, wo, pair=pair)
    g = torch.randn_like(y)
    y.backward(g)
    assert pair.job is None and len(seen) == 1
    xr, wqr, wor = (v.detach().clone().requires_grad_() for v in (x, wq, wo))
    qr = xr @ wqr
    ((qr[:, :h] * qr[:, h:2 * h] + qr[:, 2 * h:]) @ wor).backward(g)
    torch.testing.assert_close(seen[0], wor.grad, rtol=1e-5, atol=1e-5)   # final value at hook time
    torch.testing.assert_close(wo.grad, wor.grad, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(wq.grad, wqr.grad, rtol=1e-5, atol=1e-5)
