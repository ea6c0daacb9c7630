"""incubate.autograd functional API against torch.autograd.functional (reference:
python/paddle/incubate/autograd/functional.py vjp / jvp / Jacobian / Hessian, primapi.py
forward_grad / grad)."""
import numpy as np
import pytest
import torch

import paddle_ray_amd as paddle
from paddle_ray_amd.incubate import autograd as IA


def _f(x, y):
    return paddle.tanh(x) * y.sum() + paddle.matmul(x, x)


def _t(a):
    return paddle.to_tensor(a)


def test_vjp_jvp_match_torch():
    rs = np.random.RandomState(0)
    x, y = rs.randn(3, 3).astype('float64'), rs.randn(2).astype('float64')
    f_t = lambda a, b: torch.tanh(a) * b.sum() + a @ a  # noqa: E731
    v = rs.randn(3, 3)
    ys, g = IA.vjp(_f, [_t(x), _t(y)], _t(v))
    _, ref = torch.autograd.functional.vjp(f_t, (torch.tensor(x), torch.tensor(y)), torch.tensor(v))
    np.testing.assert_allclose(g[0].numpy(), ref[0].numpy(), rtol=1e-10)
    np.testing.assert_allclose(g[1].numpy(), ref[1].numpy(), rtol=1e-10)
    u = [rs.randn(3, 3), rs.randn(2)]
    _, jv = IA.jvp(_f, [_t(x), _t(y)], [_t(u[0]), _t(u[1])])
    _, jref = torch.autograd.functional.jvp(f_t, (torch.tensor(x), torch.tensor(y)),
                                            (torch.tensor(u[0]), torch.tensor(u[1])))
    np.testing.assert_allclose(jv.numpy(), jref.numpy(), rtol=1e-10)
    # single input, default v = ones
    _, g1 = IA.vjp(paddle.sin, _t(x))
    np.testing.assert_allclose(g1.numpy(), np.cos(x), rtol=1e-12)
    with pytest.raises(ValueError):
        IA.jvp(_f, [_t(x), _t(y)], [_t(u[0])])


def test_jacobian_lazy_rows_and_indexing():
    rs = np.random.RandomState(1)
    x, y = rs.randn(3, 3), rs.randn(2)
    J = IA.Jacobian(_f, [_t(x), _t(y)])
    assert J.shape == [9, 11]
    f_t = lambda a, b: (torch.tanh(a) * b.sum() + a @ a).reshape(-1)  # noqa: E731
    ja, jb = torch.autograd.functional.jacobian(f_t, (torch.tensor(x), torch.tensor(y)))
    ref = torch.cat([ja.reshape(9, 9), jb.reshape(9, 2)], 1).numpy()
    np.testing.assert_allclose(J[4].numpy(), ref[4], rtol=1e-10)
    assert len(J._j._cache) == 1                      # only the requested row was evaluated
    np.testing.assert_allclose(J[2:5, 3].numpy(), ref[2:5, 3], rtol=1e-10)
    np.testing.assert_allclose(J[:].numpy(), ref, rtol=1e-10)
    np.testing.assert_allclose(J[..., -1].numpy(), ref[:, -1], rtol=1e-10)
    with pytest.raises(IndexError):
        J[9]


def test_batched_jacobian_and_hessian():
    rs = np.random.RandomState(2)
    xb = rs.randn(4, 3)
    fb = lambda x: paddle.concat([paddle.sin(x), (x * x).sum(axis=1, keepdim=True)], axis=1)  # noqa: E731
    J = IA.Jacobian(fb, _t(xb), is_batched=True)
    assert J.shape == [4, 4, 3]
    for b in range(4):
        ref = torch.autograd.functional.jacobian(
            lambda x: torch.cat([torch.sin(x), (x * x).sum(0, keepdim=True)]), torch.tensor(xb[b])).numpy()
        np.testing.assert_allclose(J[b].numpy(), ref, rtol=1e-10)
        np.testing.assert_allclose(J[b, 3, :].numpy(), ref[3], rtol=1e-10)
    np.testing.assert_allclose(J[:, 1, 1].numpy(), np.cos(xb[:, 1]), rtol=1e-12)
    np.testing.assert_allclose(J[:, 1, 2].numpy(), np.zeros(4))
    # Hessian of a scalar function
    x = rs.randn(3)
    fs = lambda x: (paddle.sin(x) * x).sum() + (x * x).sum() ** 2  # noqa: E731
    H = IA.Hessian(fs, _t(x))
    assert H.shape == [3, 3]
    ref = torch.autograd.functional.hessian(lambda t: (torch.sin(t) * t).sum() + (t * t).sum() ** 2,
                                            torch.tensor(x)).numpy()
    np.testing.assert_allclose(H[:].numpy(), ref, rtol=1e-9)
    # batched Hessian: per-sample [B, 1] outputs
    Hb = IA.Hessian(lambda x: (x ** 3).sum(axis=1, keepdim=True), _t(xb), is_batched=True)
    assert Hb.shape == [4, 3, 3]
    np.testing.assert_allclose(Hb[1].numpy(), np.diag(6 * xb[1]), rtol=1e-10)
    with pytest.raises(RuntimeError):
        IA.Hessian(lambda x: x * 2, _t(x))[:]


def test_forward_grad_grad_and_prim_switch():
    rs = np.random.RandomState(3)
    x = paddle.to_tensor(rs.randn(5), stop_gradient=False)
    y = paddle.exp(x) * 3
    t = rs.randn(5)
    fg = IA.forward_grad(y, x, paddle.to_tensor(t))
    np.testing.assert_allclose(fg.numpy(), 3 * np.exp(x.numpy()) * t, rtol=1e-12)
    g = IA.grad(y, x)
    np.testing.assert_allclose(g.numpy(), 3 * np.exp(x.numpy()), rtol=1e-12)
    assert not IA.prim_enabled()
    IA.enable_prim()
    assert IA.prim_enabled()
    IA.disable_prim()
    assert not IA.prim_enabled()
