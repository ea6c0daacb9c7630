"""Legacy CoNLL-05 SRL readers (parity: python/paddle/dataset/conll05.py)."""
from .text import _ds, _tuple, from_dataset

__all__ = []


def get_dict(data_file=None, **kw):
    return _ds('Conll05st', data_file, **kw).get_dict()


def get_embedding(data_file=None, **kw):
    return _ds('Conll05st', data_file, **kw).get_embedding()


def test(data_file=None, **kw):
    return from_dataset(lambda: _ds('Conll05st', data_file, **kw), _tuple)
