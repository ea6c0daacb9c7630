"""vision.datasets file formats (parity: test/legacy_test/test_datasets.py,
test_dataset_cifar.py, test_dataset_voc.py, test_image_folder ...): fixtures in the
reference's on-disk formats are generated here (no network)."""
import gzip
import io
import os
import pickle
import struct
import tarfile

import numpy as np
import pytest
from PIL import Image

import paddle_ray_amd as paddle
from paddle_ray_amd.vision import datasets as D
from paddle_ray_amd.vision import transforms as T


def _idx(path, arr):
    hdr = struct.pack('>I', 0x0800 | arr.ndim) + struct.pack('>' + 'I' * arr.ndim, *arr.shape)
    with gzip.open(path, 'wb') as f:
        f.write(hdr + arr.astype(np.uint8).tobytes())


def test_mnist_idx(tmp_path):
    rs = np.random.RandomState(0)
    imgs = rs.randint(0, 256, (5, 28, 28))
    labs = np.array([3, 1, 4, 1, 5])
    _idx(tmp_path / 'i.gz', imgs)
    _idx(tmp_path / 'l.gz', labs)
    ds = D.MNIST(str(tmp_path / 'i.gz'), str(tmp_path / 'l.gz'), mode='test', backend='cv2')
    assert len(ds) == 5
    img, lab = ds[2]
    np.testing.assert_array_equal(img, imgs[2].astype(np.float32))
    assert lab.tolist() == [4] and lab.dtype == np.int64
    ds2 = D.FashionMNIST(str(tmp_path / 'i.gz'), str(tmp_path / 'l.gz'), backend='pil',
                         transform=T.ToTensor())
    assert ds2[0][0].shape == [1, 28, 28]


def test_cifar_tar(tmp_path):
    rs = np.random.RandomState(1)
    path = tmp_path / 'cifar-10-python.tar.gz'
    with tarfile.open(path, 'w:gz') as tf:
        for name, n in [('data_batch_1', 4), ('data_batch_2', 3), ('test_batch', 2)]:
            batch = {b'data': rs.randint(0, 256, (n, 3072)).astype(np.uint8),
                     b'labels': list(range(n))}
            raw = pickle.dumps(batch)
            ti = tarfile.TarInfo('cifar-10-batches-py/' + name)
            ti.size = len(raw)
            tf.addfile(ti, io.BytesIO(raw))
    tr = D.Cifar10(str(path), mode='train', backend='cv2')
    te = D.Cifar10(str(path), mode='test', backend='cv2')
    assert len(tr) == 7 and len(te) == 2
    img, lab = tr[5]
    assert img.shape == (32, 32, 3) and int(lab) == 1


def test_cifar_refuses_code_pickles(tmp_path):
    path = tmp_path / 'bad.tar.gz'

    class Evil:
        def __reduce__(self):
            return (os.getcwd, ())
    with tarfile.open(path, 'w:gz') as tf:
        raw = pickle.dumps({b'data': Evil(), b'labels': [0]})
        ti = tarfile.TarInfo('cifar-10-batches-py/data_batch_1')
        ti.size = len(raw)
        tf.addfile(ti, io.BytesIO(raw))
    with pytest.raises(pickle.UnpicklingError):
        D.Cifar10(str(path), mode='train')


def _jpg(arr):
    b = io.BytesIO()
    Image.fromarray(arr).save(b, format='JPEG')
    return b.getvalue()


def _add(tf, name, data):
    ti = tarfile.TarInfo(name)
    ti.size = len(data)
    tf.addfile(ti, io.BytesIO(data))


def test_flowers(tmp_path):
    import scipy.io as scio
    rs = np.random.RandomState(2)
    with tarfile.open(tmp_path / '102flowers.tgz', 'w:gz') as tf:
        for i in range(1, 5):
            _add(tf, 'jpg/image_%05d.jpg' % i, _jpg(rs.randint(0, 255, (8, 10, 3), np.uint8)))
    scio.savemat(tmp_path / 'imagelabels.mat', {'labels': np.array([[7, 8, 9, 10]])})
    scio.savemat(tmp_path / 'setid.mat', {'tstid': np.array([[1, 3]]), 'trnid': np.array([[2]]),
                                          'valid': np.array([[4]])})
    ds = D.Flowers(str(tmp_path / '102flowers.tgz'), str(tmp_path / 'imagelabels.mat'),
                   str(tmp_path / 'setid.mat'), mode='train', backend='cv2')
    assert len(ds) == 2
    img, lab = ds[1]
    assert img.shape == (8, 10, 3) and lab.tolist() == [9]
    with pytest.raises(FileNotFoundError):
        D.Flowers(str(tmp_path / 'missing.tgz'), mode='test')


def test_voc2012(tmp_path):
    rs = np.random.RandomState(3)
    root = 'VOCdevkit/VOC2012/'
    with tarfile.open(tmp_path / 'voc.tar', 'w') as tf:
        _add(tf, root + 'ImageSets/Segmentation/trainval.txt', b'a\nb\n')
        for n in 'ab':
            _add(tf, root + f'JPEGImages/{n}.jpg', _jpg(rs.randint(0, 255, (6, 7, 3), np.uint8)))
            b = io.BytesIO()
            Image.fromarray(rs.randint(0, 20, (6, 7), np.uint8), mode='L').save(b, format='PNG')
            _add(tf, root + f'SegmentationClass/{n}.png', b.getvalue())
    ds = D.VOC2012(str(tmp_path / 'voc.tar'), mode='train', backend='cv2')
    img, lab = ds[1]
    assert len(ds) == 2 and img.shape == (6, 7, 3) and lab.shape == (6, 7)


def test_dataset_and_image_folder(tmp_path):
    rs = np.random.RandomState(4)
    for c, n in [('cat', 2), ('dog', 3)]:
        os.makedirs(tmp_path / c)
        for i in range(n):
            Image.fromarray(rs.randint(0, 255, (5, 5, 3), np.uint8)).save(tmp_path / c / f'{i}.png')
    (tmp_path / 'cat' / 'notes.txt').write_text('x')
    ds = D.DatasetFolder(str(tmp_path))
    assert ds.classes == ['cat', 'dog'] and len(ds) == 5 and ds.targets == [0, 0, 1, 1, 1]
    s, t = ds[4]
    assert t == 1 and s.size == (5, 5)
    paddle.vision.set_image_backend('cv2')
    try:
        assert D.DatasetFolder(str(tmp_path))[0][0].shape == (5, 5, 3)
    finally:
        paddle.vision.set_image_backend('pil')
    imf = D.ImageFolder(str(tmp_path), transform=T.ToTensor())
    assert len(imf) == 5 and imf[0][0].shape == [3, 5, 5]
    img = paddle.vision.image_load(str(tmp_path / 'cat' / '0.png'), backend='cv2')
    assert img.shape == (5, 5, 3)
