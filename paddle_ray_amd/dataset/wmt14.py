"""Legacy WMT14 readers (parity: python/paddle/dataset/wmt14.py)."""
from .text import _ds, _tuple, from_dataset

__all__ = []


def train(dict_size, data_file=None):
    return from_dataset(lambda: _ds('WMT14', data_file, mode='train', dict_size=dict_size),
                        _tuple)


def test(dict_size, data_file=None):
    return from_dataset(lambda: _ds('WMT14', data_file, mode='test', dict_size=dict_size),
                        _tuple)


def get_dict(dict_size, reverse=True, data_file=None):
    return _ds('WMT14', data_file, mode='train', dict_size=dict_size).get_dict(reverse)
