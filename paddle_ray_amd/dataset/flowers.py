"""Legacy Flowers readers (parity: python/paddle/dataset/flowers.py): (CHW float32 image,
int label) with the reference's train/test mapping."""
import numpy as np

from . import image as I
from ._readers import from_dataset

__all__ = []


def default_mapper(is_train, sample):
    img, label = sample
    img = I.simple_transform(np.asarray(img), 256, 224, is_train,
                             mean=[103.94, 116.78, 123.68])
    return img.flatten().astype('float32'), label


def _reader(mode, mapper, data_file, label_file, setid_file, cycle):
    from ..vision.datasets import Flowers
    mapper = mapper or (lambda s: default_mapper(mode == 'train', s))
    return from_dataset(lambda: Flowers(data_file, label_file, setid_file, mode=mode,
                                        backend='cv2'),
                        lambda s: mapper((np.asarray(s[0], np.uint8), int(s[1][0]))), cycle)


def train(mapper=None, buffered_size=1024, use_xmap=True, cycle=False, data_file=None,
          label_file=None, setid_file=None):
    return _reader('train', mapper, data_file, label_file, setid_file, cycle)


def test(mapper=None, buffered_size=1024, use_xmap=True, cycle=False, data_file=None,
         label_file=None, setid_file=None):
    return _reader('test', mapper, data_file, label_file, setid_file, cycle)


def valid(mapper=None, buffered_size=1024, use_xmap=True, data_file=None, label_file=None,
          setid_file=None):
    return _reader('valid', mapper, data_file, label_file, setid_file, False)
