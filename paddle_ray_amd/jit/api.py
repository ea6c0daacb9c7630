"""paddle.jit (parity: python/paddle/jit/api.py)."""
import functools
import os

from ..framework.io import save as _save, load as _load

_enabled = [True]


def enable_to_static(flag):
    _enabled[0] = bool(flag)


def set_code_level(level=100, also_to_stdout=False):
    pass


def set_verbosity(level=0, also_to_stdout=False):
    pass


def not_to_static(fn):
    fn._not_to_static = True
    return fn


def ignore_module(modules):
    pass


def to_static(function=None, input_spec=None, build_strategy=None, backend=None, **kwargs):
    def deco(fn):
        return fn
    return deco(function) if function is not None else deco


class TranslatedLayer:
    pass


def save(layer, path, input_spec=None, **configs):
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    _save(layer.state_dict(), path + '.pdparams')


def load(path, **configs):
    return _load(path + '.pdparams')
