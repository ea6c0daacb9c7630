"""Legacy MovieLens readers (parity: python/paddle/dataset/movielens.py)."""
from .text import _ds, _tuple, from_dataset

__all__ = []


def train(data_file=None):
    return from_dataset(lambda: _ds('Movielens', data_file, mode='train'), _tuple)


def test(data_file=None):
    return from_dataset(lambda: _ds('Movielens', data_file, mode='test'), _tuple)
