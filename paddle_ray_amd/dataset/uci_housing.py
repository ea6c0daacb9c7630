"""Legacy UCI housing readers (parity: python/paddle/dataset/uci_housing.py)."""
from ._readers import from_dataset

__all__ = []
feature_names = ['CRIM', 'ZN', 'INDUS', 'CHAS', 'NOX', 'RM', 'AGE', 'DIS', 'RAD', 'TAX',
                 'PTRATIO', 'B', 'LSTAT']


def _make(mode, data_file=None):
    from ..text.datasets import UCIHousing
    return lambda: UCIHousing(data_file, mode=mode)


def train(data_file=None):
    return from_dataset(_make('train', data_file))


def test(data_file=None):
    return from_dataset(_make('test', data_file))


def fetch():
    pass
