"""paddle.sparse.nn and paddle.distribution.transform (parity:
test/legacy_test/test_sparse_conv_op.py, test_sparse_pooling_op.py, test_sparse_norm_op.py,
test_sparse_softmax_op.py, test_distribution_transform.py)."""
import numpy as np
import torch
import torch.nn.functional as TF

import paddle_ray_amd as paddle
from paddle_ray_amd import distribution as D
from paddle_ray_amd.sparse import nn as SN


def _voxels(seed=0, C=4):
    g = torch.Generator().manual_seed(seed)
    idx = torch.tensor([[0, 0, 0, 1], [1, 2, 2, 0], [1, 1, 3, 2], [1, 3, 2, 4]])
    return paddle.Tensor(torch.sparse_coo_tensor(idx, torch.randn(4, C, generator=g),
                                                 (2, 4, 5, 6, C)).coalesce())


def test_subm_conv_matches_dense_at_active_sites():
    paddle.seed(0)
    x = _voxels()
    conv = SN.SubmConv3D(4, 8, 3)
    y = conv(x)._t
    dense = x._t.to_dense().permute(0, 4, 1, 2, 3)
    ref = TF.conv3d(dense, conv.weight._t.permute(4, 3, 0, 1, 2), conv.bias._t, 1, 1)
    ref = ref.permute(0, 2, 3, 4, 1)
    idx = x._t.indices()
    torch.testing.assert_close(y.indices(), idx)
    torch.testing.assert_close(y.values(), ref[tuple(idx)], atol=1e-5, rtol=1e-5)


def test_conv3d_output_pattern_and_pool():
    x = _voxels()
    y = SN.Conv3D(4, 6, 3, padding=1)(x)._t
    occ = torch.zeros(2, 4, 5, 6)
    occ[tuple(x._t.indices())] = 1
    dil = TF.conv3d(occ[:, None], torch.ones(1, 1, 3, 3, 3), padding=1)[:, 0] > 0
    assert y._nnz() == int(dil.sum())
    p = SN.MaxPool3D(2)(x)._t
    assert p.shape == (2, 2, 2, 3, 4) and p._nnz() == 4
    # each pooled value is its (only) active input's value
    np.testing.assert_allclose(np.sort(p.values().numpy().ravel()),
                               np.sort(x._t.values().numpy().ravel()), atol=1e-6)


def test_sparse_activations_and_norm():
    x = _voxels()
    v = x._t.values()
    torch.testing.assert_close(SN.ReLU()(x)._t.values(), torch.relu(v))
    torch.testing.assert_close(SN.ReLU6()(x)._t.values(), v.clamp(0, 6))
    torch.testing.assert_close(SN.LeakyReLU(0.2)(x)._t.values(), TF.leaky_relu(v, 0.2))
    bn = SN.BatchNorm(4)
    bn.train()
    out = bn(x)._t.values()
    torch.testing.assert_close(out.mean(0), torch.zeros(4), atol=1e-5, rtol=0)
    dense = torch.tensor([[0.0, 1.0, 2.0], [3.0, 0.0, 0.0]])
    sm = SN.Softmax()(paddle.Tensor(dense.to_sparse_csr()))._t.to_dense()
    np.testing.assert_allclose(sm[0, 1:].numpy(), torch.softmax(torch.tensor([1.0, 2.0]), 0),
                               atol=1e-6)
    assert float(sm[1, 0]) == 1.0


def test_sparse_attention():
    torch.manual_seed(0)
    q, k, v = (torch.randn(1, 2, 4, 8) for _ in range(3))
    mask = torch.tril(torch.ones(2, 4, 4))
    out = SN.functional.attention(paddle.Tensor(q), paddle.Tensor(k), paddle.Tensor(v),
                                  paddle.Tensor(mask.to_sparse_csr()))._t
    ref = TF.scaled_dot_product_attention(q, k, v, is_causal=True)
    torch.testing.assert_close(out, ref, atol=1e-5, rtol=1e-5)


def test_distribution_transforms():
    x = paddle.to_tensor([0.5, 1.5])
    aff = D.AffineTransform(paddle.to_tensor(1.0), paddle.to_tensor(2.0))
    np.testing.assert_allclose(aff.forward(x).numpy(), [2.0, 4.0])
    np.testing.assert_allclose(aff.inverse(aff.forward(x)).numpy(), x.numpy())
    np.testing.assert_allclose(aff.forward_log_det_jacobian(x).numpy(), np.log(2.0) * np.ones(2),
                               rtol=1e-6)
    ch = D.ChainTransform([D.ExpTransform(), aff])
    np.testing.assert_allclose(ch.forward(x).numpy(), 1 + 2 * np.exp([0.5, 1.5]), rtol=1e-6)
    for t in (D.SigmoidTransform(), D.TanhTransform(), D.PowerTransform(paddle.to_tensor(2.0))):
        np.testing.assert_allclose(t.inverse(t.forward(x)).numpy(), x.numpy(), rtol=1e-5)
    neg, pos = D.AbsTransform().inverse(paddle.to_tensor([2.0]))
    assert float(neg) == -2.0 and float(pos) == 2.0
    sb = D.StickBreakingTransform().forward(paddle.to_tensor([0.1, 0.2]))
    assert sb.shape == [3] and abs(float(sb.sum()) - 1) < 1e-6
    assert D.ReshapeTransform((2, 3), (3, 2)).forward_shape([4, 2, 3]) == [4, 3, 2]
    lognormal = D.TransformedDistribution(D.Normal(0.0, 1.0), [D.ExpTransform()])
    np.testing.assert_allclose(float(lognormal.log_prob(paddle.to_tensor(1.0))),
                               -0.5 * np.log(2 * np.pi), rtol=1e-6)

    class MyNormal(D.Normal):
        pass

    @D.register_kl(MyNormal, MyNormal)
    def _kl(p, q):
        return paddle.to_tensor(42.0)
    assert float(D.kl_divergence(MyNormal(0.0, 1.0), MyNormal(1.0, 1.0))) == 42.0
    assert abs(float(D.kl_divergence(D.Normal(0.0, 1.0), D.Normal(1.0, 1.0))) - 0.5) < 1e-6


def test_sparse_conv_rulebook_large_grid_and_grads():
    """Rulebook convolution on a 1 x 256^3 grid with 64 active sites (a dense grid would be 16M
    sites x C): output pattern, values against a dense conv3d of the small neighbourhood, and
    gradients through gather/GEMM/scatter."""
    import torch
    import paddle_ray_amd.sparse as sp
    rs = np.random.RandomState(0)
    pts = np.unique(rs.randint(0, 256, (64, 3)), axis=0)
    idx = torch.tensor(np.concatenate([np.zeros((len(pts), 1), np.int64), pts], 1).T)
    vals = torch.randn(len(pts), 4, dtype=torch.float64, requires_grad=True)
    x = paddle.Tensor(torch.sparse_coo_tensor(idx, vals, (1, 256, 256, 256, 4)).coalesce())
    w = torch.randn(3, 3, 3, 4, 5, dtype=torch.float64, requires_grad=True)
    y = sp.nn.functional.subm_conv3d(x, paddle.Tensor(w), padding=1)
    yt = y._t
    assert yt._nnz() == len(pts) and torch.equal(yt.indices(), x._t.indices())
    # reference for one site: sum over its active neighbours
    ci = x._t.indices().t()
    site = ci[0]
    ref = torch.zeros(5, dtype=torch.float64)
    for j, c in enumerate(ci):
        d = (c[1:] - site[1:] + 1)
        if bool(((d >= 0) & (d <= 2)).all()):
            ref = ref + x._t.values()[j] @ w[d[0], d[1], d[2]]
    np.testing.assert_allclose(yt.values()[0].detach().numpy(), ref.detach().numpy(), rtol=1e-10)
    yt.values().sum().backward()
    assert vals.grad is not None and w.grad is not None and float(w.grad.abs().sum()) > 0
    z = sp.nn.functional.conv3d(x, paddle.Tensor(w.detach()), stride=2)
    assert z._t.shape[1:4] == (127, 127, 127) and z._t._nnz() <= 27 * len(pts)


def test_sparse_reshape_keeps_sparsity():
    import torch
    import paddle_ray_amd.sparse as sp
    d = torch.zeros(4, 6)
    d[1, 2], d[3, 5], d[0, 0] = 1.0, 2.0, 3.0
    x = paddle.Tensor(d.to_sparse())
    y = sp.reshape(x, [3, 8])
    assert y.is_sparse_coo() and y.nnz() == 3
    np.testing.assert_allclose(y.to_dense().numpy(), d.reshape(3, 8).numpy())
    y2 = sp.reshape(x, [2, -1, 3])
    np.testing.assert_allclose(y2.to_dense().numpy(), d.reshape(2, 4, 3).numpy())
    c = sp.reshape(paddle.Tensor(d.to_sparse_csr()), [8, 3])
    assert c.is_sparse_csr()
    np.testing.assert_allclose(c.to_dense().numpy(), d.reshape(8, 3).numpy())
