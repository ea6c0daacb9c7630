"""Legacy IMDB readers (parity: python/paddle/dataset/imdb.py): (word ids, label)."""
from .text import _ds, _tuple, from_dataset

__all__ = []


def word_dict(data_file=None, cutoff=150):
    return _ds('Imdb', data_file, mode='train', cutoff=cutoff).word_idx


def train(word_idx=None, data_file=None):
    return from_dataset(lambda: _ds('Imdb', data_file, mode='train'),
                        lambda s: (s[0].tolist(), int(s[1][0])))


def test(word_idx=None, data_file=None):
    return from_dataset(lambda: _ds('Imdb', data_file, mode='test'),
                        lambda s: (s[0].tolist(), int(s[1][0])))
