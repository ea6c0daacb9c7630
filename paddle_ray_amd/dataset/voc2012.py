"""Legacy VOC2012 segmentation readers (parity: python/paddle/dataset/voc2012.py)."""
from ._readers import from_dataset

__all__ = []


def _reader(mode, data_file):
    from ..vision.datasets import VOC2012
    return from_dataset(lambda: VOC2012(data_file, mode=mode, backend='cv2'))


def train(data_file=None):
    return _reader('train', data_file)


def test(data_file=None):
    return _reader('test', data_file)


def val(data_file=None):
    return _reader('valid', data_file)
