"""paddle.* tensor API vs NumPy (reference test strategy: OpTest compares against NumPy)."""
import numpy as np
import pytest

import paddle_ray_amd as paddle


def A(x):
    return np.asarray(x.numpy() if isinstance(x, paddle.Tensor) else x)


def test_to_tensor_and_meta():
    x = paddle.to_tensor([[1, 2], [3, 4]])
    assert x.dtype == paddle.int64
    assert x.shape == [2, 2]
    assert x.ndim == 2 and x.size == 4
    y = paddle.to_tensor([1.5, 2.5])
    assert y.dtype == paddle.float32
    assert y.stop_gradient
    z = paddle.to_tensor(np.ones((2, 3), np.float64))
    assert z.dtype == paddle.float64
    assert 'Tensor(shape=[2, 2]' in repr(x)
    assert x.place.is_cpu_place() or x.place.is_gpu_place()


def test_creation():
    assert A(paddle.zeros([2, 3])).sum() == 0
    assert A(paddle.ones([2, 3], 'int32')).dtype == np.int32
    np.testing.assert_allclose(A(paddle.full([2], 7.0)), [7, 7])
    np.testing.assert_allclose(A(paddle.arange(0, 5, 2)), [0, 2, 4])
    np.testing.assert_allclose(A(paddle.linspace(0, 1, 5)), np.linspace(0, 1, 5), rtol=1e-6)
    np.testing.assert_allclose(A(paddle.eye(3)), np.eye(3))
    x = paddle.to_tensor(np.arange(9.).reshape(3, 3).astype('float32'))
    np.testing.assert_allclose(A(paddle.tril(x)), np.tril(A(x)))
    np.testing.assert_allclose(A(paddle.triu(x, 1)), np.triu(A(x), 1))
    np.testing.assert_allclose(A(paddle.zeros_like(x)), np.zeros((3, 3)))
    np.testing.assert_allclose(A(paddle.full_like(x, 2)), np.full((3, 3), 2))
    gx, gy = paddle.meshgrid(paddle.arange(3), paddle.arange(2))
    assert gx.shape == [3, 2]
    np.testing.assert_allclose(A(paddle.diag(paddle.to_tensor([1., 2.]))), np.diag([1., 2.]))


def test_math_elementwise():
    a = np.random.rand(3, 4).astype('float32') + 0.5
    b = np.random.rand(3, 4).astype('float32') + 0.5
    x, y = paddle.to_tensor(a), paddle.to_tensor(b)
    np.testing.assert_allclose(A(x + y), a + b, rtol=1e-6)
    np.testing.assert_allclose(A(x - y), a - b, rtol=1e-6)
    np.testing.assert_allclose(A(x * y), a * b, rtol=1e-6)
    np.testing.assert_allclose(A(x / y), a / b, rtol=1e-6)
    np.testing.assert_allclose(A(x ** 2), a ** 2, rtol=1e-6)
    np.testing.assert_allclose(A(2 - x), 2 - a, rtol=1e-6)
    np.testing.assert_allclose(A(paddle.add(x, y)), a + b, rtol=1e-6)
    np.testing.assert_allclose(A(paddle.multiply(x, y)), a * b, rtol=1e-6)
    np.testing.assert_allclose(A(paddle.maximum(x, y)), np.maximum(a, b))
    np.testing.assert_allclose(A(paddle.exp(x)), np.exp(a), rtol=1e-5)
    np.testing.assert_allclose(A(paddle.log(x)), np.log(a), rtol=1e-5)
    np.testing.assert_allclose(A(paddle.sqrt(x)), np.sqrt(a), rtol=1e-5)
    np.testing.assert_allclose(A(paddle.tanh(x)), np.tanh(a), rtol=1e-5)
    np.testing.assert_allclose(A(paddle.clip(x, 0.7, 1.0)), np.clip(a, 0.7, 1.0))
    np.testing.assert_allclose(A(paddle.scale(x, 2.0, 1.0)), a * 2 + 1, rtol=1e-6)
    i = paddle.to_tensor([7, -7])
    np.testing.assert_array_equal(A(paddle.floor_divide(i, paddle.to_tensor([2, 2]))), [3, -4])
    np.testing.assert_array_equal(A(paddle.remainder(i, paddle.to_tensor([3, 3]))), [1, 2])


def test_reductions():
    a = np.random.rand(2, 3, 4).astype('float32')
    x = paddle.to_tensor(a)
    np.testing.assert_allclose(A(paddle.sum(x)), a.sum(), rtol=1e-5)
    np.testing.assert_allclose(A(paddle.sum(x, axis=1)), a.sum(1), rtol=1e-5)
    np.testing.assert_allclose(A(paddle.sum(x, axis=[0, 2], keepdim=True)),
                               a.sum((0, 2), keepdims=True), rtol=1e-5)
    np.testing.assert_allclose(A(paddle.mean(x, axis=-1)), a.mean(-1), rtol=1e-5)
    np.testing.assert_allclose(A(paddle.max(x, axis=1)), a.max(1))
    np.testing.assert_allclose(A(paddle.min(x)), a.min())
    np.testing.assert_allclose(A(paddle.prod(x, axis=0)), a.prod(0), rtol=1e-5)
    np.testing.assert_allclose(A(paddle.var(x, axis=1)), a.var(1, ddof=1), rtol=1e-4)
    np.testing.assert_allclose(A(paddle.std(x)), a.std(ddof=1), rtol=1e-4)
    np.testing.assert_allclose(A(paddle.logsumexp(x, axis=2)),
                               np.log(np.exp(a).sum(2)), rtol=1e-5)
    np.testing.assert_allclose(A(paddle.cumsum(x, axis=1)), a.cumsum(1), rtol=1e-5)
    np.testing.assert_array_equal(A(paddle.argmax(x, axis=2)), a.argmax(2))
    assert paddle.sum(paddle.to_tensor([1, 2], 'int32')).dtype == paddle.int64
    b = paddle.to_tensor([[True, False], [True, True]])
    assert not bool(paddle.all(b)) and bool(paddle.any(b))
    np.testing.assert_allclose(A(paddle.median(paddle.to_tensor([3., 1., 2., 4.]))), 2.5)


def test_manipulation():
    a = np.arange(24).reshape(2, 3, 4).astype('float32')
    x = paddle.to_tensor(a)
    assert paddle.reshape(x, [4, -1]).shape == [4, 6]
    assert paddle.reshape(x, [0, 12]).shape == [2, 12]
    np.testing.assert_allclose(A(paddle.transpose(x, [2, 0, 1])), a.transpose(2, 0, 1))
    np.testing.assert_allclose(A(paddle.concat([x, x], axis=1)), np.concatenate([a, a], 1))
    np.testing.assert_allclose(A(paddle.stack([x, x])), np.stack([a, a]))
    parts = paddle.split(x, [1, -1], axis=2)
    assert parts[0].shape == [2, 3, 1] and parts[1].shape == [2, 3, 3]
    assert len(paddle.chunk(x, 2, axis=2)) == 2
    assert paddle.unsqueeze(x, [0, 4]).shape == [1, 2, 3, 4, 1]
    assert paddle.squeeze(paddle.zeros([1, 3, 1]), axis=0).shape == [3, 1]
    assert paddle.flatten(x, 1).shape == [2, 12]
    np.testing.assert_allclose(A(paddle.expand(paddle.to_tensor([1., 2.]), [3, 2])),
                               np.tile([1., 2.], (3, 1)))
    np.testing.assert_allclose(A(paddle.tile(paddle.to_tensor([1., 2.]), [2])), [1, 2, 1, 2])
    idx = paddle.to_tensor([2, 0])
    np.testing.assert_allclose(A(paddle.gather(x, idx, axis=1)), a[:, [2, 0]])
    np.testing.assert_allclose(A(paddle.index_select(x, idx, axis=2)), a[:, :, [2, 0]])
    nd = paddle.to_tensor([[0, 1], [1, 2]])
    np.testing.assert_allclose(A(paddle.gather_nd(x, nd)), a[[0, 1], [1, 2]])
    np.testing.assert_allclose(A(paddle.flip(x, [0])), a[::-1])
    np.testing.assert_allclose(A(paddle.roll(x, 1, 2)), np.roll(a, 1, 2))
    np.testing.assert_allclose(A(paddle.slice(x, [1], [1], [3])), a[:, 1:3])
    np.testing.assert_allclose(A(paddle.strided_slice(x, [2], [0], [4], [2])), a[:, :, 0:4:2])
    s = paddle.scatter(paddle.zeros([3, 2]), paddle.to_tensor([1]), paddle.ones([1, 2]))
    np.testing.assert_allclose(A(s), [[0, 0], [1, 1], [0, 0]])
    t = paddle.take_along_axis(x, paddle.to_tensor(np.zeros((2, 3, 1), 'int64')), 2)
    np.testing.assert_allclose(A(t), a[:, :, :1])
    u = paddle.unique(paddle.to_tensor([3, 1, 3, 2]))
    np.testing.assert_array_equal(A(u), [1, 2, 3])
    w = paddle.where(x > 10, x, paddle.zeros_like(x))
    np.testing.assert_allclose(A(w), np.where(a > 10, a, 0))
    v, i = paddle.topk(paddle.to_tensor([1., 5., 3.]), 2)
    np.testing.assert_allclose(A(v), [5, 3])
    np.testing.assert_array_equal(A(paddle.sort(paddle.to_tensor([3, 1, 2]))), [1, 2, 3])


def test_indexing_and_setitem():
    x = paddle.to_tensor(np.arange(12.).reshape(3, 4).astype('float32'))
    np.testing.assert_allclose(A(x[1]), [4, 5, 6, 7])
    np.testing.assert_allclose(A(x[:, 1:3]), np.arange(12.).reshape(3, 4)[:, 1:3])
    np.testing.assert_allclose(A(x[x > 9]), [10, 11])
    x[0, 0] = 100.
    assert float(x[0, 0]) == 100.
    x[paddle.to_tensor([1, 2])] = 0.
    assert float(paddle.sum(x[1:])) == 0.


def test_linalg():
    a = np.random.rand(3, 3).astype('float32') + np.eye(3, dtype='float32') * 3
    b = np.random.rand(3, 2).astype('float32')
    x, y = paddle.to_tensor(a), paddle.to_tensor(b)
    np.testing.assert_allclose(A(paddle.matmul(x, y)), a @ b, rtol=1e-5)
    np.testing.assert_allclose(A(paddle.matmul(x, x, transpose_y=True)), a @ a.T, rtol=1e-5)
    np.testing.assert_allclose(A(x @ y), a @ b, rtol=1e-5)
    np.testing.assert_allclose(A(paddle.linalg.inv(x)), np.linalg.inv(a), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(A(paddle.linalg.det(x)), np.linalg.det(a), rtol=1e-4)
    np.testing.assert_allclose(A(paddle.linalg.norm(y)), np.linalg.norm(b), rtol=1e-5)
    np.testing.assert_allclose(A(paddle.linalg.solve(x, y)), np.linalg.solve(a, b), rtol=1e-4)
    np.testing.assert_allclose(A(paddle.einsum('ij,jk->ik', x, y)), a @ b, rtol=1e-5)
    np.testing.assert_allclose(A(paddle.bmm(paddle.to_tensor(a[None]), paddle.to_tensor(b[None]))),
                               (a @ b)[None], rtol=1e-5)
    np.testing.assert_allclose(A(paddle.dot(paddle.to_tensor([1., 2.]), paddle.to_tensor([3., 4.]))),
                               11.)


def test_random_and_seed():
    paddle.seed(42)
    a = paddle.rand([4])
    paddle.seed(42)
    b = paddle.rand([4])
    np.testing.assert_allclose(A(a), A(b))
    assert paddle.randint(0, 10, [100]).numpy().max() < 10
    assert paddle.randn([2, 3]).shape == [2, 3]
    assert sorted(A(paddle.randperm(5)).tolist()) == [0, 1, 2, 3, 4]
    st = paddle.get_rng_state()
    c = paddle.rand([3])
    paddle.set_rng_state(st)
    np.testing.assert_allclose(A(paddle.rand([3])), A(c))


def test_logic():
    x = paddle.to_tensor([1., 2., 3.])
    y = paddle.to_tensor([1., 0., 3.])
    np.testing.assert_array_equal(A(x == y), [True, False, True])
    np.testing.assert_array_equal(A(paddle.equal(x, y)), [True, False, True])
    assert bool(paddle.allclose(x, x))
    assert bool(paddle.equal_all(x, x))
    np.testing.assert_array_equal(A(paddle.logical_and(x > 1, y > 1)), [False, False, True])
    assert bool(paddle.isnan(paddle.to_tensor([float('nan')]))[0])


def test_cast_and_methods():
    x = paddle.to_tensor([1.7, -2.2])
    assert x.astype('int32').dtype == paddle.int32
    assert paddle.cast(x, 'float64').dtype == paddle.float64
    assert x.numpy().tolist() == pytest.approx([1.7, -2.2])
    assert x.abs().tolist() == pytest.approx([1.7, 2.2])
    assert x.sum().item() == pytest.approx(-0.5)
    assert x.reshape([2, 1]).shape == [2, 1]
    assert x.unsqueeze(0).shape == [1, 2]
    b = x.astype('bfloat16')
    assert b.dtype == paddle.bfloat16
    assert b.numpy().dtype == np.float32


def test_fft_and_misc():
    a = np.random.rand(8).astype('float32')
    np.testing.assert_allclose(A(paddle.fft.rfft(paddle.to_tensor(a))), np.fft.rfft(a), rtol=1e-4,
                               atol=1e-5)
    assert paddle.iinfo(paddle.int32).max == 2 ** 31 - 1
    assert paddle.finfo(paddle.float32).eps > 0
    assert paddle.get_default_dtype() == paddle.float32
