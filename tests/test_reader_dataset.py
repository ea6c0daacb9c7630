"""paddle.reader decorators and legacy paddle.dataset readers (parity:
test/legacy_test/test_reader_decorator (decorator_test.py), test_multiprocess_reader_exception,
dataset/tests/*)."""
import gzip
import struct
import warnings

import numpy as np
import pytest

import paddle_ray_amd as paddle
from paddle_ray_amd import reader as R


def _r(n):
    return lambda: iter(range(n))


def test_basic_decorators():
    assert list(R.firstn(_r(10), 3)()) == [0, 1, 2]
    assert list(R.chain(_r(2), _r(3))()) == [0, 1, 0, 1, 2]
    assert list(R.map_readers(lambda a, b: a * b, _r(4), _r(4))()) == [0, 1, 4, 9]
    assert sorted(R.shuffle(_r(10), 4)()) == list(range(10))
    c = R.cache(_r(3))
    assert list(c()) == list(c()) == [0, 1, 2]
    assert list(R.buffered(_r(100), 7)()) == list(range(100))
    pairs = lambda: iter([(i, i + 1) for i in range(3)])  # noqa: E731
    assert list(R.compose(pairs, _r(3))()) == [(0, 1, 0), (1, 2, 1), (2, 3, 2)]
    with pytest.raises(R.ComposeNotAligned):
        list(R.compose(_r(2), _r(3))())
    assert list(R.compose(_r(2), _r(3), check_alignment=False)()) == [(0, 0), (1, 1)]
    assert paddle.batch(_r(5), 2)().__next__() == [0, 1]


def test_xmap_and_multiprocess():
    out = list(R.xmap_readers(lambda x: x * 2, _r(50), 4, 8, order=True)())
    assert out == [2 * i for i in range(50)]
    assert sorted(R.xmap_readers(lambda x: x + 1, _r(30), 3, 4)()) == list(range(1, 31))
    mp = R.multiprocess_reader([_r(5), lambda: iter(range(10, 13))], queue_size=4)
    assert sorted(mp()) == [0, 1, 2, 3, 4, 10, 11, 12]


def test_buffered_propagates_errors():
    def bad():
        yield 1
        raise RuntimeError("boom")
    with pytest.raises(RuntimeError):
        list(R.buffered(bad, 2)())


def test_dataset_mnist_reader(tmp_path):
    rs = np.random.RandomState(0)
    imgs = rs.randint(0, 256, (4, 28, 28)).astype(np.uint8)
    labs = np.array([1, 2, 3, 4], np.uint8)
    for name, arr in [('i.gz', imgs), ('l.gz', labs)]:
        with gzip.open(tmp_path / name, 'wb') as f:
            f.write(struct.pack('>I', 0x0800 | arr.ndim) +
                    struct.pack('>' + 'I' * arr.ndim, *arr.shape) + arr.tobytes())
    rd = paddle.dataset.mnist.reader_creator(str(tmp_path / 'i.gz'), str(tmp_path / 'l.gz'))
    samples = list(rd())
    assert len(samples) == 4 and samples[2][1] == 3
    np.testing.assert_allclose(samples[0][0], imgs[0].reshape(-1) / 255.0 * 2 - 1, atol=1e-6)


def test_dataset_cifar_synthetic_and_uci(tmp_path):
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        x, y = next(paddle.dataset.cifar.test10()())
    assert x.shape == (3072,) and 0 <= x.min() and x.max() <= 1 and isinstance(y, int)
    rows = np.random.RandomState(1).rand(20, 14)
    p = tmp_path / 'housing.data'
    p.write_text('\n'.join(' '.join(f'{v:.4f}' for v in r) for r in rows))
    tr = list(paddle.dataset.uci_housing.train(str(p))())
    te = list(paddle.dataset.uci_housing.test(str(p))())
    assert len(tr) + len(te) == 20 and tr[0][0].shape == (13,)


def test_dataset_common_split(tmp_path):
    import pickle
    from paddle_ray_amd.dataset import common
    common.split(_r(10), 4, suffix=str(tmp_path / 'part-%05d.pickle'))
    r0 = common.cluster_files_reader(str(tmp_path / 'part-*.pickle'), 2, 0)
    r1 = common.cluster_files_reader(str(tmp_path / 'part-*.pickle'), 2, 1)
    assert sorted(list(r0()) + list(r1())) == list(range(10))
    with pytest.raises(RuntimeError):
        common.download('http://x/y.tgz', 'nothing_here', None)
    assert pickle  # files above were written by this test (safe to load)


def test_dataset_image_helpers():
    from paddle_ray_amd.dataset import image as I
    im = (np.random.RandomState(0).rand(40, 50, 3) * 255).astype(np.uint8)
    out = I.simple_transform(im, 32, 24, is_train=False, mean=[1.0, 2.0, 3.0])
    assert out.shape == (3, 24, 24) and out.dtype == np.float32
    assert I.random_crop(im, 10).shape == (10, 10, 3)


def test_cost_model():
    cm = paddle.cost_model.CostModel()
    s, m = cm.build_program()
    try:
        r = cm.profile_measure(s, m, device='cpu')
    finally:
        paddle.disable_static()
    # the backward is per-op grad OpDescs now: each appears with its own measured time
    assert r['time'] > 0 and any(k.endswith('_grad') for k in r['op_time']) and len(r['ops']) >= 3
    data = cm.static_cost_data()  # measured on MI355X by scripts/op_benchmark.py
    assert any(d['op'] == 'flash_attention' for d in data)
    fwd = cm.get_static_op_time('matmul', forward=True, dtype='bfloat16')
    bwd = cm.get_static_op_time('matmul', forward=False, dtype='bfloat16')
    assert fwd['op_time'] > 0 and bwd['op_time'] > 0 and 'bfloat16' in fwd['config']
    with pytest.raises(ValueError):
        cm.get_static_op_time(None)
