"""LoD sequence ops against the worked examples in the reference's docstrings
(python/paddle/static/nn/sequence_lod.py) and a plain per-sequence loop."""
import numpy as np
import pytest
import torch

import paddle_ray_amd as paddle
from paddle_ray_amd.static import nn as snn
from paddle_ray_amd.static import create_lod_tensor


def _lod_t(data, lod):
    t = paddle.to_tensor(np.asarray(data, dtype='float32'))
    t.set_lod(lod)
    return t


def test_lod_api():
    t = _lod_t(np.zeros((5, 2)), [[0, 2, 5]])
    assert t.lod() == [[0, 2, 5]]
    assert t.recursive_sequence_lengths() == [[2, 3]]
    t.set_recursive_sequence_lengths([[1, 4]])
    assert t.lod() == [[0, 1, 5]] and t.has_valid_recursive_sequence_lengths()
    with pytest.raises(ValueError):
        t.set_lod([[0, 2, 4]])
    c = create_lod_tensor(np.arange(6).reshape(6, 1), [[2, 4]])
    assert c.lod() == [[0, 2, 6]]


@pytest.mark.parametrize("pool,expect", [
    ('average', [2., 4., 3., 0.]), ('sum', [4., 12., 6., 0.]),
    ('sqrt', [4 / 2 ** .5, 12 / 3 ** .5, 6 / 2 ** .5, 0.]), ('max', [3., 6., 5., 0.]),
    ('last', [3., 6., 1., 0.]), ('first', [1., 2., 5., 0.])])
def test_sequence_pool_reference_example(pool, expect):
    x = _lod_t([[1.], [3.], [2.], [4.], [6.], [5.], [1.]], [[0, 2, 5, 7, 7]])
    out = snn.sequence_pool(x, pool)
    np.testing.assert_allclose(out.numpy().reshape(-1), expect, rtol=1e-5)


def test_sequence_pool_grad():
    x = _lod_t(np.random.RandomState(0).randn(7, 3), [[0, 2, 5, 7]])
    x.stop_gradient = False
    snn.sequence_pool(x, 'max').sum().backward()
    g = x.grad.numpy()
    xs = x.numpy()
    for a, b in [(0, 2), (2, 5), (5, 7)]:
        am = xs[a:b].argmax(0)
        ref = np.zeros((b - a, 3))
        ref[am, np.arange(3)] = 1
        np.testing.assert_allclose(g[a:b], ref)


def test_sequence_softmax_matches_loop():
    v = np.random.RandomState(1).randn(6).astype('float32')
    x = _lod_t(v.reshape(6, 1), [[0, 1, 4, 6]])
    out = snn.sequence_softmax(x).numpy().reshape(-1)
    for a, b in [(0, 1), (1, 4), (4, 6)]:
        e = np.exp(v[a:b] - v[a:b].max())
        np.testing.assert_allclose(out[a:b], e / e.sum(), rtol=1e-5)


def test_sequence_concat_reference_example():
    x1 = _lod_t([[1], [2], [3], [4], [5]], [[0, 3, 5]])
    x2 = _lod_t([[6], [7], [8], [9]], [[0, 2, 4]])
    out = snn.sequence_concat([x1, x2])
    assert out.numpy().reshape(-1).tolist() == [1, 2, 3, 6, 7, 4, 5, 8, 9]
    assert out.lod() == [[0, 5, 9]]


def test_sequence_slice_reference_example():
    x = _lod_t(np.arange(10).reshape(5, 2), [[0, 3, 5]])
    out = snn.sequence_slice(x, paddle.to_tensor([[0], [1]]), paddle.to_tensor([[2], [1]]))
    assert out.numpy().tolist() == [[0, 1], [2, 3], [8, 9]]
    assert out.recursive_sequence_lengths() == [[2, 1]]


def test_sequence_expand_reference_examples():
    x = _lod_t([[1], [2], [3], [4]], [[0, 2, 4]])
    y = _lod_t(np.zeros((8, 1)), [[0, 2, 4], [0, 3, 6, 7, 8]])
    out = snn.sequence_expand(x, y, ref_level=0)
    assert out.numpy().reshape(-1).tolist() == [1, 2, 1, 2, 3, 4, 3, 4]
    assert out.lod() == [[0, 2, 4, 6, 8]]
    x2 = paddle.to_tensor(np.array([[1.], [2.], [3.]], dtype='float32'))
    y2 = _lod_t(np.zeros((5, 1)), [[0, 2, 2, 5]])
    out2 = snn.sequence_expand(x2, y2, ref_level=-1)
    assert out2.numpy().reshape(-1).tolist() == [1, 1, 3, 3, 3]


def test_sequence_expand_as_reference_example():
    x = paddle.to_tensor(np.array([[1.], [2.], [3.], [4.]], dtype='float32'))
    y = _lod_t(np.zeros((8, 1)), [[0, 3, 6, 7, 8]])
    out = snn.sequence_expand_as(x, y)
    assert out.numpy().reshape(-1).tolist() == [1, 1, 1, 2, 2, 2, 3, 4]
    assert out.lod() == [[0, 3, 6, 7, 8]]


def test_sequence_pad_unpad_roundtrip():
    x = _lod_t(np.arange(10).reshape(5, 2), [[0, 2, 5]])
    out, length = snn.sequence_pad(x, paddle.to_tensor(np.array([-1., -2.], dtype='float32')))
    assert length.numpy().tolist() == [2, 3]
    assert out.numpy().tolist() == [[[0, 1], [2, 3], [-1, -2]], [[4, 5], [6, 7], [8, 9]]]
    out4, _ = snn.sequence_pad(x, paddle.to_tensor(np.array([0.], dtype='float32')), maxlen=4)
    assert out4.shape == [2, 4, 2]
    back = snn.sequence_unpad(out4, length)
    np.testing.assert_array_equal(back.numpy(), x.numpy())
    assert back.lod() == [[0, 2, 5]]
    # reference sequence_unpad example
    xp = paddle.to_tensor(np.arange(1, 16, dtype='float32').reshape(3, 5))
    u = snn.sequence_unpad(xp, paddle.to_tensor(np.array([2, 3, 4])))
    assert u.numpy().tolist() == [1, 2, 6, 7, 8, 11, 12, 13, 14]
    assert u.lod() == [[0, 2, 5, 9]]


def test_sequence_reshape_reference_example():
    x = _lod_t(np.arange(1, 13).reshape(6, 2), [[0, 2, 6]])
    out = snn.sequence_reshape(x, 4)
    assert out.lod() == [[0, 1, 3]]
    assert out.numpy().tolist() == [[1, 2, 3, 4], [5, 6, 7, 8], [9, 10, 11, 12]]


def test_sequence_scatter_reference_example():
    inp = paddle.to_tensor(np.ones((3, 6), dtype='float32'))
    idx = paddle.to_tensor(np.array([[0], [1], [2], [5], [4], [3], [2], [1], [3], [2], [5], [4]]))
    idx.set_lod([[0, 3, 8, 12]])
    upd = _lod_t([[.3], [.3], [.4], [.1], [.2], [.3], [.4], [0.], [.2], [.3], [.1], [.4]],
                 [[0, 3, 8, 12]])
    out = snn.sequence_scatter(inp, idx, upd).numpy()
    np.testing.assert_allclose(out, [[1.3, 1.3, 1.4, 1.0, 1.0, 1.0],
                                     [1.0, 1.0, 1.4, 1.3, 1.2, 1.1],
                                     [1.0, 1.0, 1.3, 1.2, 1.4, 1.1]], rtol=1e-6)


def test_sequence_enumerate_reference_example():
    x = paddle.to_tensor(np.array([[1], [2], [3], [4], [5]]))
    x.set_lod([[0, 3, 5]])
    out = snn.sequence_enumerate(x, 2)
    assert out.numpy().tolist() == [[1, 2], [2, 3], [3, 0], [4, 5], [5, 0]]
    assert out.lod() == [[0, 3, 5]]


def test_sequence_reverse_reference_example():
    x = _lod_t(np.arange(1, 21).reshape(5, 4), [[0, 2, 5]])
    out = snn.sequence_reverse(x).numpy()
    assert out[:, 0].tolist() == [5, 1, 17, 13, 9]


def test_sequence_first_last_step():
    x = _lod_t([[1.], [3.], [2.], [4.], [6.]], [[0, 2, 5]])
    assert snn.sequence_first_step(x).numpy().reshape(-1).tolist() == [1, 2]
    assert snn.sequence_last_step(x).numpy().reshape(-1).tolist() == [3, 6]


def test_sequence_conv_context_projection():
    torch.manual_seed(0)
    x = _lod_t([[1, 1], [2, 2], [3, 3], [4, 4]], [[0, 3, 4]])
    out = snn.sequence_conv(x, num_filters=3, filter_size=3, bias_attr=False)
    assert out.shape == [4, 3] and out.lod() == [[0, 3, 4]]
    # reference example: padded projection rows
    from paddle_ray_amd.static.sequence_lod import _context_project
    proj = _context_project(torch.tensor([[1., 1], [2, 2], [3, 3], [4, 4]]), [0, 3, 4], 3, -1)
    assert proj.tolist() == [[0, 0, 1, 1, 2, 2], [1, 1, 2, 2, 3, 3], [2, 2, 3, 3, 0, 0],
                             [0, 0, 4, 4, 0, 0]]
    # out = proj @ W
    w = snn._layers[-1].weight.numpy()
    np.testing.assert_allclose(out.numpy(), proj.numpy() @ w, rtol=1e-5, atol=1e-6)


def test_sparse_attention_reference_example():
    F = paddle.nn.functional
    q = paddle.to_tensor(np.array([[[[0, 1], [2, 3], [0, 1], [2, 3]]]], dtype='float32'))
    off = paddle.to_tensor(np.array([[[0, 2, 4, 6, 8]]], dtype='int32'))
    cols = paddle.to_tensor(np.array([[[0, 1, 0, 1, 2, 3, 2, 3]]], dtype='int32'))
    kpm = paddle.to_tensor(np.array([[1, 1, 1, 0]], dtype='float32'))
    am = paddle.to_tensor(np.array([[1, 0, 1, 1], [1, 1, 1, 1], [1, 1, 1, 1], [1, 1, 1, 1]],
                                   dtype='float32'))
    np.testing.assert_allclose(F.sparse_attention(q, q, q, off, cols, kpm, am).numpy()[0, 0],
                               [[0, 1], [1.9983027, 2.9983027], [0, 1], [0, 1]], rtol=1e-5)
    np.testing.assert_allclose(F.sparse_attention(q, q, q, off, cols).numpy()[0, 0],
                               [[1.60885942, 2.60885954], [1.9983027, 2.9983027],
                                [1.60885942, 2.60885954], [1.9983027, 2.9983027]], rtol=1e-5)


def test_static_auc_and_ctr_bundle():
    from sklearn.metrics import roc_auc_score
    from paddle_ray_amd.static.graph import auc, ctr_metric_bundle
    rs = np.random.RandomState(0)
    p1 = rs.rand(64)
    y = (rs.rand(64) < p1).astype('int64')
    pred = paddle.to_tensor(np.stack([1 - p1, p1], 1).astype('float32'))
    a, ba, stats = auc(pred, paddle.to_tensor(y.reshape(-1, 1)), num_thresholds=100000)
    np.testing.assert_allclose(float(a.numpy()[0]), roc_auc_score(y, p1), atol=1e-3)
    assert len(stats) == 4 and int(stats[2].numpy().sum()) == int(y.sum())
    s = ctr_metric_bundle(paddle.to_tensor(np.array([[0.2], [0.9]], dtype='float32')),
                          paddle.to_tensor(np.array([[0], [1]], dtype='int64')))
    np.testing.assert_allclose([float(t.numpy()[0]) for t in s],
                               [0.04 + 0.01, 0.2 + 0.1, 1.1, 1 / (1 + np.exp(-0.2)) +
                                1 / (1 + np.exp(-0.9)), 1, 2], rtol=1e-5)


def test_static_auc_accumulates_in_program():
    from sklearn.metrics import roc_auc_score
    paddle.enable_static()
    try:
        main, startup = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, startup):
            pred = paddle.static.data('pred', [-1, 2], 'float32')
            lab = paddle.static.data('lab', [-1, 1], 'int64')
            a, ba, _ = paddle.static.auc(pred, lab, num_thresholds=100000, slide_steps=1)
        exe = paddle.static.Executor()
        rs = np.random.RandomState(1)
        ps, ys = [], []
        for _ in range(3):
            p1 = rs.rand(50).astype('float32')
            y = (rs.rand(50) < p1).astype('int64')
            ps.append(p1)
            ys.append(y)
            out = exe.run(main, feed={'pred': np.stack([1 - p1, p1], 1), 'lab': y.reshape(-1, 1)},
                          fetch_list=[a, ba])
        np.testing.assert_allclose(float(np.asarray(out[0]).reshape(-1)[0]),
                                   roc_auc_score(np.concatenate(ys), np.concatenate(ps)), atol=1e-3)
        np.testing.assert_allclose(float(np.asarray(out[1]).reshape(-1)[0]),
                                   roc_auc_score(ys[-1], ps[-1]), atol=1e-3)
    finally:
        paddle.disable_static()
