"""Legacy text readers (parity: python/paddle/dataset/{imdb,imikolov,movielens,conll05,
wmt14,wmt16}.py) over paddle_ray_amd.text.datasets (local archives only)."""
from ._readers import from_dataset


def _ds(name, *a, **k):
    from ..text import datasets as T
    return getattr(T, name)(*a, **k)


def _tuple(s):
    return tuple(x.tolist() if hasattr(x, 'tolist') else x for x in s)
