"""Legacy MNIST readers (parity: python/paddle/dataset/mnist.py): (784 float32 in [-1, 1],
int label)."""
import numpy as np

from ._readers import from_dataset

__all__ = []


def _conv(s):
    img, lab = s
    a = np.asarray(img, np.float32).reshape(-1)
    if a.max() > 1.0:
        a = a / 255.0
    return a * 2.0 - 1.0, int(np.asarray(lab).reshape(-1)[0])


def _make(mode, image_path=None, label_path=None):
    from ..vision.datasets import MNIST
    return lambda: MNIST(image_path, label_path, mode=mode, backend='cv2')


def reader_creator(image_filename, label_filename, buffer_size=100):
    return from_dataset(_make('train', image_filename, label_filename), _conv)


def train():
    return from_dataset(_make('train'), _conv)


def test():
    return from_dataset(_make('test'), _conv)


def fetch():
    pass
