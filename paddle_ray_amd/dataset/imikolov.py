"""Legacy PTB readers (parity: python/paddle/dataset/imikolov.py)."""
from .text import _ds, _tuple, from_dataset

__all__ = []


class DataType:
    NGRAM = 1
    SEQ = 2


def build_dict(min_word_freq=50, data_file=None):
    return _ds('Imikolov', data_file, mode='train', min_word_freq=min_word_freq).word_idx


def _reader(mode, n, data_type, data_file):
    dt = 'NGRAM' if data_type in (DataType.NGRAM, 'NGRAM') else 'SEQ'
    return from_dataset(lambda: _ds('Imikolov', data_file, data_type=dt, window_size=n,
                                    mode=mode), _tuple)


def train(word_idx=None, n=5, data_type=DataType.NGRAM, data_file=None):
    return _reader('train', n, data_type, data_file)


def test(word_idx=None, n=5, data_type=DataType.NGRAM, data_file=None):
    return _reader('test', n, data_type, data_file)
