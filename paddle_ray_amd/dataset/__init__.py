"""paddle.dataset: legacy reader-creator datasets (parity: python/paddle/dataset/
__init__.py)."""
from . import (common, image, mnist, cifar, uci_housing, imdb, imikolov, movielens,  # noqa
               conll05, wmt14, wmt16, flowers, voc2012)

__all__ = []
