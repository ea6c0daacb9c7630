"""Legacy CIFAR readers (parity: python/paddle/dataset/cifar.py): (3072 float32 in [0, 1]
CHW-flattened, int label)."""
import numpy as np

from ._readers import from_dataset

__all__ = []


def _conv(s):
    img, lab = s
    a = np.asarray(img, np.float32)
    if a.ndim == 3 and a.shape[-1] == 3:
        a = a.transpose(2, 0, 1)
    a = a.reshape(-1)
    if a.max() > 1.0:
        a = a / 255.0
    return a.astype(np.float32), int(np.asarray(lab).reshape(-1)[0])


def _reader(cls, mode, data_file=None, cycle=False):
    from ..vision import datasets as D
    return from_dataset(lambda: getattr(D, cls)(data_file, mode=mode, backend='cv2'), _conv,
                        cycle)


def reader_creator(filename, sub_name, cycle=False):
    cls = 'Cifar100' if '100' in filename else 'Cifar10'
    return _reader(cls, 'test' if 'test' in sub_name else 'train', filename, cycle)


def train10(cycle=False):
    return _reader('Cifar10', 'train', cycle=cycle)


def test10(cycle=False):
    return _reader('Cifar10', 'test', cycle=cycle)


def train100():
    return _reader('Cifar100', 'train')


def test100():
    return _reader('Cifar100', 'test')


def fetch():
    pass
