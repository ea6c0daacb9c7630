"""Legacy WMT16 readers (parity: python/paddle/dataset/wmt16.py)."""
from .text import _ds, _tuple, from_dataset

__all__ = []


def _reader(mode, src_dict_size, trg_dict_size, src_lang, data_file):
    return from_dataset(lambda: _ds('WMT16', data_file, mode=mode, src_dict_size=src_dict_size,
                                    trg_dict_size=trg_dict_size, lang=src_lang), _tuple)


def train(src_dict_size, trg_dict_size, src_lang='en', data_file=None):
    return _reader('train', src_dict_size, trg_dict_size, src_lang, data_file)


def test(src_dict_size, trg_dict_size, src_lang='en', data_file=None):
    return _reader('test', src_dict_size, trg_dict_size, src_lang, data_file)


def validation(src_dict_size, trg_dict_size, src_lang='en', data_file=None):
    return _reader('val', src_dict_size, trg_dict_size, src_lang, data_file)


def get_dict(lang, dict_size, reverse=False, data_file=None):
    ds = _ds('WMT16', data_file, mode='train', src_dict_size=dict_size, trg_dict_size=dict_size,
             lang=lang)
    src, trg = ds.get_dict(reverse)
    return src
