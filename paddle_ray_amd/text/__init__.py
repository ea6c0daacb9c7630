"""paddle.text (parity: python/paddle/text/): Viterbi decoding and the classic NLP datasets."""
from .viterbi_decode import viterbi_decode, ViterbiDecoder  # noqa: F401
from . import datasets  # noqa: F401
from .datasets import (Conll05st, Imdb, Imikolov, Movielens, UCIHousing, WMT14,  # noqa: F401
                       WMT16)

__all__ = ['Conll05st', 'Imdb', 'Imikolov', 'Movielens', 'UCIHousing', 'WMT14', 'WMT16',
           'ViterbiDecoder', 'viterbi_decode']
